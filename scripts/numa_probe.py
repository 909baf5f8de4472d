"""Where the GPU, the CPUs this process may use and its pinned memory sit (NUMA)."""
import glob
import os

import torch

print("affinity cpus", len(os.sched_getaffinity(0)), sorted(os.sched_getaffinity(0))[:8], "...")
props = torch.cuda.get_device_properties(0)
print("gpu", props.name, getattr(props, "pci_bus_id", None), getattr(props, "pci_device_id", None))
for d in glob.glob("/sys/bus/pci/devices/*"):
    try:
        cls = open(d + "/class").read().strip()
        if cls.startswith("0x0380") or cls.startswith("0x0300"):
            print(d.rsplit("/", 1)[-1], cls, "numa", open(d + "/numa_node").read().strip())
    except OSError:
        pass
for n in sorted(glob.glob("/sys/devices/system/node/node*/cpulist")):
    print(n.split("/")[-2], open(n).read().strip())
