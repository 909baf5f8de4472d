"""Multi-GPU data parallelism of the inbound pipeline: device-key sharding + RCCL re-keying.

Reference parallelism: Kafka key partitioning (records of one device token on one
partition, ``murmur2(key) % partitions``) + consumer groups; the Hazelcast near cache replicates the
registry to every consumer.  MI355X form:

* **ownership** -- each rank owns the devices whose 128-bit token fingerprint satisfies
  ``(fp_hi >> 32) % world == rank`` (``sw_owner`` in ``csrc/include/swtypes.h``).  The owner holds the
  device's state, dedup window and event-store rows, so every stateful stage is shard-local -- no
  cross-GPU atomics.  The registry (fingerprint -> device, active assignment, context) is
  replicated on every rank, as the reference's near cache replicates it to every consumer: the
  rank that decoded a record sends it to the owner only when its device is registered and assigned,
  and rejects every other record itself -- it holds the payload bytes the slow path routes.
* **re-keying** -- every rank decodes the payloads it received, partitions the decoded records into
  per-owner slabs (``k_part_count``/``k_part_write``), and one ``all_to_all_single`` of the slab
  counts plus one of the slabs moves each record to its owner over xGMI (the GPU analogue of
  producing to the key's partition).  Records cross xGMI in a lossless 64-byte packed form
  (``SwWireRec``: fields no event type uses together share words), 20% fewer bytes than the
  80-byte decoded record; their strings (alternate id, metadata, alert message) travel beside them
  in per-destination byte slabs (``EngineConfig.str_bytes`` per slot).  Control records
  (registration, acks, streams) and records of unknown devices stay on the receiving rank, whose
  host owns their raw bytes.
* **slab sizing** -- fixed-size slabs keep the exchange free of host synchronisation: capacity per
  destination = ``shuffle_slack * rec_cap / world + 1024`` (``EngineConfig.shuf_cap``, slack 1.1).
  A uniform key hash puts ~rec_cap/world records per destination (sigma ~ sqrt of that, so 1.1x
  is > 30 sigma at 1M records/step).  Skewed keys cannot lose records: whatever does not fit a slab
  is *spilled* in deterministic order and sent first by the next step's exchange (``carry``);
  only records beyond ``carry_cap`` are dropped, counted in ``shuffle_overflow``.  Slack is kept
  small because xGMI is point-to-point: at N=2 every slab byte crosses one link.
* **pipelined exchange** -- ``GpuInboundEngine.round_async`` software-pipelines the step across
  two streams: the compute stream runs decode+partition of batch k and then unpack+process of
  batch k-1, while the all-to-all of batch k runs on a communication stream, overlapped with the
  process phase of batch k-1 (double-buffered send slabs; one receive buffer, released by unpack).
  A step then costs max(H2D, compute, exchange) instead of compute + exchange.
"""
from __future__ import annotations

import os

import numpy as np


def owner_of(fp_hi: np.ndarray, world: int) -> np.ndarray:
    """Owner rank of each device fingerprint (same function as the GPU kernels)."""
    return ((np.asarray(fp_hi, np.uint64) >> np.uint64(32)) % np.uint64(world)).astype(np.int64)


def shard_mask(fp_hi: np.ndarray, world: int, rank: int) -> np.ndarray:
    return owner_of(fp_hi, world) == rank


def env_rank() -> tuple[int, int, int]:
    """(rank, local_rank, world) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def _cpulist(text: str) -> set[int]:
    cpus: set[int] = set()
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    return cpus


def gpu_numa_node(index: int) -> int:
    """NUMA node of GPU ``index``'s PCIe function (-1 if unknown / single node)."""
    import torch
    p = torch.cuda.get_device_properties(index)
    path = f"/sys/bus/pci/devices/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0/numa_node"
    try:
        with open(path) as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return -1


def bind_numa(index: int) -> int:
    """Pin this rank's host threads to the CPUs of its GPU's NUMA node (``SW_NUMA_BIND=0`` disables).

    The pipeline streams ~56 GB/s of payload bytes per GPU from pinned host memory; keeping the
    host side (pinned staging, launch thread, RCCL proxies) on the GPU's socket avoids crossing the
    inter-socket fabric with 8 ranks at once.  Returns the node (-1 when nothing was changed)."""
    if os.environ.get("SW_NUMA_BIND", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return -1
    node = gpu_numa_node(index)
    if node < 0:
        return -1
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            cpus = _cpulist(f.read()) & os.sched_getaffinity(0)
        if cpus:
            os.sched_setaffinity(0, cpus)
            return node
    except OSError:
        pass
    return -1


def init_distributed(use_gpu: bool = True):
    """One process per GPU: bind the local device (and its NUMA node's CPUs), create the RCCL (or
    gloo) process group.  Returns (rank, local device index, world, device).

    Rehearsal knobs (not for production runs): ``SW_SHARED_DEVICE=1`` puts every rank on GPU 0 and
    ``SW_DIST_BACKEND=gloo`` exchanges through gloo (RCCL refuses two ranks on one GPU), so the
    N>1 engine path -- partition, pipelined exchange on the comm stream, spill carry, cross-rank
    stats -- runs on a one-GPU box with real kernels."""
    import torch
    import torch.distributed as dist
    rank, local, world = env_rank()
    device = None
    if use_gpu:
        if os.environ.get("SW_SHARED_DEVICE", "0") == "1":
            local = 0
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
        if world > 1:
            bind_numa(local)
    if world > 1 and not dist.is_initialized():
        backend = os.environ.get("SW_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
        dist.init_process_group(backend, device_id=device if backend == "nccl" else None)
    return rank, local, world, device


def exchange_slabs(send_cnt, recv_cnt, send, recv, group=None, extra=()):
    """The re-key collective: counts, then the fixed-size slabs (all stream-ordered, no host sync).
    ``extra``: more (send, recv) pairs split evenly over the ranks the same way -- the string
    exchange's byte counts, refs and byte slabs."""
    import torch.distributed as dist
    dist.all_to_all_single(recv_cnt, send_cnt, group=group)
    dist.all_to_all_single(recv, send, group=group)
    for s, r in extra:
        dist.all_to_all_single(r, s, group=group)


def exchange_bytes_per_rank(rec_cap: int, world: int, slack: float = 1.1, rec_bytes: int = 64, pad: int = 1024) -> int:
    """Bytes one rank sends per step (its slab for every destination, self included)."""
    cap = int(slack * rec_cap / max(1, world)) + pad
    return world * cap * rec_bytes
