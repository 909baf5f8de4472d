"""NUMA placement of a GPU's host-side pipeline.

A raw batch crosses PCIe from pinned host memory; when that memory (or the threads writing it) sit
on the other socket, every DMA also crosses the socket interconnect.  ``bind_to_gpu_node`` pins
the calling process to the CPUs of the GPU's NUMA node before anything is allocated, so first-touch
places pinned pools, bus segments and producer buffers next to the GPU's PCIe root."""
from __future__ import annotations

import glob
import os


def gpu_numa_node(pci_bus: int, pci_device: int = 0) -> int | None:
    """NUMA node of the PCI function at bus ``pci_bus`` (any domain), or None."""
    for d in glob.glob(f"/sys/bus/pci/devices/*:{pci_bus:02x}:{pci_device:02x}.0"):
        try:
            node = int(open(os.path.join(d, "numa_node")).read().strip())
        except (OSError, ValueError):
            continue
        if node >= 0:
            return node
    return None


def node_cpus(node: int) -> set[int]:
    out = set()
    try:
        spec = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
    except OSError:
        return out
    for part in spec.split(","):
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        elif part:
            out.add(int(part))
    return out


def bind_to_gpu_node(device_index: int = 0) -> int | None:
    """Restrict this process to the CPUs of GPU ``device_index``'s NUMA node (intersected with the
    CPUs it may use).  Returns the node, or None when it cannot be determined or would leave no CPU.
    Call before the process initialises the GPU or allocates its pinned buffers."""
    import torch
    props = torch.cuda.get_device_properties(device_index)
    node = gpu_numa_node(int(getattr(props, "pci_bus_id", -1)), int(getattr(props, "pci_device_id", 0) or 0))
    if node is None:
        return None
    cpus = node_cpus(node) & os.sched_getaffinity(0)
    if not cpus:
        return None
    os.sched_setaffinity(0, cpus)
    return node
