"""GPU inbound-pipeline engine shard (MI355X / gfx950).

Owns every hot table of one tenant shard in HBM and drives the kernels of
``csrc/hip/swgpu.hip`` through ``libswgpu.so``:

    H2D(raw batch)  ->  decode  ->  [owner partition -> RCCL all_to_all_single -> unpack]
                    ->  validate + dedup + persist/enrich + state + rules + presence
                    ->  D2H(outbound records)

``step_async`` only enqueues work on the current HIP stream (no host sync, so a
step can be captured into a hipGraph); :class:`PipelinedRunner` overlaps the
H2D copy of batch k+1 and the D2H copy of batch k-1 with the compute of batch k
on three streams.
"""
from __future__ import annotations

import ctypes
import os
import time

import numpy as np
import torch

from .._native import gpu_gil as gpu_lib
from ..models.columnar import EVENT_REC, N_STATS, OUT_REC, NAME_REF, OUT_REC_SIZE, ST_RECHECK, STR_REF, WIRE_REC
from ..ops.engine_abi import SwEngineArgs
from .config import EngineConfig
from .bus_io import host_view
from .engine_base import EngineBase, StepResult

_ALIGN = 64


def _ptr(t: torch.Tensor) -> int:
    return t.data_ptr()


class HostBuffer:
    """Mapped pinned host memory (hipHostMalloc Mapped): kernels store outbound rows into it directly."""

    def __init__(self, lib, nbytes: int):
        self.lib = lib
        self.nbytes = int(nbytes)
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        rc = lib.sw_host_alloc(self.nbytes, ctypes.byref(h), ctypes.byref(d))
        if rc:
            raise RuntimeError(f"hipHostMalloc failed ({rc})")
        self.host, self.dev = h.value, d.value
        self._arr = np.ctypeslib.as_array((ctypes.c_uint8 * self.nbytes).from_address(self.host))

    def view(self, dtype, n: int) -> np.ndarray:
        return self._arr[:n * np.dtype(dtype).itemsize].view(dtype)

    def __del__(self):
        try:
            if self.host:
                self.lib.sw_host_free(ctypes.c_void_p(self.host))
                self.host = None
        except Exception:
            pass


class _Submitted:
    """One batch in :meth:`GpuInboundEngine.submit_framed`'s pipeline."""
    __slots__ = ("slot", "batch", "token", "small", "rows", "sig", "ev", "bmeta", "bbuf", "bsig", "bev", "now",
                 "mapped")

    def __init__(self, slot, batch, token):
        self.slot, self.batch, self.token = slot, batch, token
        self.small = self.rows = self.sig = self.ev = None
        self.bmeta = self.bbuf = self.bsig = self.bev = None
        self.now = 0
        self.mapped = False             # step snapshot + rejects written into the slot's mapped host memory


def _host_addr(buf) -> int:
    """Address of a host buffer (bytes-like, numpy array or memoryview; read-only views included)."""
    if isinstance(buf, np.ndarray):
        return buf.ctypes.data
    return np.frombuffer(buf, np.uint8).ctypes.data


def _chk(rc: int):
    if rc:
        raise RuntimeError(f"HIP stream call failed ({rc})")


class _FramedSlots:
    """Slot state of :meth:`GpuInboundEngine.submit_framed`: device raw / varint-length / offset
    buffers per slot (grown on demand), the H2D copy stream and its events, and the batches still in
    flight (oldest first)."""
    SLOTS = 3

    def __init__(self, e: "GpuInboundEngine"):
        from collections import deque
        if e.n_out_bufs < self.SLOTS:
            raise ValueError(f"overlapped framed steps need {self.SLOTS} outbound buffers")
        self.e = e
        self.h2d = torch.cuda.Stream(e.device)
        self.d2h = torch.cuda.Stream(e.device)      # rows when the SDMA engine is unavailable
        self.ev_h2d = [torch.cuda.Event() for _ in range(self.SLOTS)]
        self.ev_comp = [torch.cuda.Event() for _ in range(self.SLOTS)]
        for ev in self.ev_h2d + self.ev_comp:      # created now (torch creates them on first record):
            ev.record(self.h2d)                    # the submit path passes their raw handles natively
        self.h2d.synchronize()
        self.bufs = [None] * self.SLOTS
        self.inflight = deque()
        self.k = 0
        self.no_sdma = False

    def buffers(self, b: int, nb: int, nl: int):
        e = self.e
        cur = self.bufs[b]
        if cur is None or cur[0].numel() < nb or cur[1].numel() < nl:
            self.ev_comp[b].synchronize()           # the old slot buffers may still be read
            # grow geometrically: coalesced steps vary in size, and a reallocation per new maximum
            # (device memory + a sync) would land in the middle of a burst
            grow = 2 * cur[0].numel() if cur is not None else 0
            cur = self.bufs[b] = (
                torch.empty(max(nb, grow, int(getattr(e, "_stg_hint", 0))), dtype=torch.uint8, device=e.device),
                torch.empty(max(nl, 5 * e.cfg.max_msgs + 64), dtype=torch.uint8, device=e.device),
                torch.empty(e.cfg.max_msgs + 1, dtype=torch.int32, device=e.device))
        return cur


class GpuInboundEngine(EngineBase):
    def __init__(self, cfg: EngineConfig, device: str | torch.device = "cuda", group=None):
        super().__init__(cfg)
        self.lib = gpu_lib()
        self.device = torch.device(device)
        self.group = group
        d = self.device
        c = cfg
        i32, i64, u8 = torch.int32, torch.int64, torch.uint8

        def z(n, dt):
            return torch.zeros(int(n), dtype=dt, device=d)

        def full(n, v, dt):
            return torch.full((int(n),), v, dtype=dt, device=d)

        tile = 1024
        ntiles = (c.rec_cap + tile - 1) // tile
        mtiles = (c.max_msgs + tile - 1) // tile
        ptiles = (c.carry_cap + c.rec_cap + tile - 1) // tile     # partition input: carry + records
        # single-pass scans keep u64 look-back state (2 + tiles words) in it, zeroed by each scan
        scan_tmp = 2 * (max(ptiles * 2 * max(1, c.world), mtiles, 2 * ntiles) + 64)
        self.t = t = {}
        # decode
        t["msg_cnt"] = z(c.max_msgs + 1, i32)
        t["msg_evoff"] = z(c.max_msgs + 1, i32)
        t["scan_tmp"] = z(scan_tmp, i32)
        t["recs"] = z(c.rec_cap * EVENT_REC.itemsize, u8)
        t["spans"] = z(c.rec_cap * STR_REF.itemsize, u8)          # string refs beside each record
        t["seen_key"] = z(c.name_slots, i64)
        t["new_names"] = z(c.names_cap * NAME_REF.itemsize, u8)
        t["vlen_tmp"] = z(2 * ((5 * c.max_msgs + tile - 1) // tile) + 64, i32)   # varint framing scan
        t["scalars"] = z(64, i32)  # n_recs, n_new_names, overflow, n_work, n_ok, n_rej, n_gen, n_out, n_rule
        # shuffle
        if c.world > 1:
            # send slabs are double-buffered (the pipelined exchange of batch k reads one while batch
            # k+1 is partitioned into the other); carry/spill alternate roles every partition
            self.send_bufs = [z(c.world * c.shuf_cap * WIRE_REC.itemsize, u8) for _ in range(2)]
            self.send_cnts = [z(c.world, i32) for _ in range(2)]
            t["recv"] = z(c.world * c.shuf_cap * WIRE_REC.itemsize, u8)
            t["recv_cnt"] = z(c.world, i32)
            t["part_tmp"] = z(2 * c.world * ptiles + 64, i32)
            t["work"] = z(c.rec_cap * EVENT_REC.itemsize, u8)
            self.carry_bufs = [z(c.carry_cap * EVENT_REC.itemsize, u8) for _ in range(2)]
            t["n_carry"] = z(2, i32)
            t["part_owner"] = z(c.carry_cap + c.rec_cap + 64, u8)      # re-key destination per input
            t["part_bytes"] = z(2 * c.world * ptiles + 64, i64)          # string bytes per tile, scanned
            t["part_meta"] = z(256, i64)                                # cut / bytes per destination
            if c.str_cap:
                # string exchange: byte slabs + refs beside the record slabs (double-buffered the same
                # way), gathered into work_str by the unpack (see SwEngineArgs)
                sr = STR_REF.itemsize
                self.send_strs = [z(c.world * c.str_cap, u8) for _ in range(2)]
                self.send_str_cnts = [z(c.world, i32) for _ in range(2)]
                self.send_spans = [z(c.world * c.shuf_cap * sr, u8) for _ in range(2)]
                t["recv_str"] = z(c.world * c.str_cap, u8)
                t["recv_str_cnt"] = z(c.world, i32)
                t["recv_spans"] = z(c.world * c.shuf_cap * sr, u8)
                t["work_str"] = z(c.world * c.str_cap + 64, u8)
                t["work_spans"] = z(c.rec_cap * sr, u8)
                # lossless re-key: spilled records keep their strings in the carry's heap (parity
                # like the carry records); exchange bytes of every partition input
                self.carry_spans = [z(c.carry_cap * sr, u8) for _ in range(2)]
                self.carry_strs = [z(c.carry_str_cap + 64, u8) for _ in range(2)]
                t["n_carry_str"] = z(2, i32)
                t["part_len"] = z(c.carry_cap + c.rec_cap + 64, i32)
        t["str_drops"] = z(2, i32)
        # validated
        t["status"] = z(c.rec_cap, u8)
        t["ev_dev"] = z(c.rec_cap, i32)
        t["ev_asg"] = z(c.rec_cap, i32)
        t["ok_idx"] = z(c.rec_cap, i32)
        if c.cluster:
            # persist clustering by assignment: radix-sort ping-pong buffers + histograms
            t["cl_keys"] = z(2 * c.rec_cap, i32)
            t["cl_vals"] = z(2 * c.rec_cap, i32)
            t["cl_hist"] = z(int(self.lib.sw_radix_tmp_words(c.rec_cap)), i32)
        t["rej_idx"] = z(c.rec_cap, i32)
        t["cmp_tmp"] = z(4 * ntiles + 64, i32)
        # registry (packed SwRegSlot: lo, hi, dev, asg, pad) + assignment context (device, customer, area, asset)
        t["reg"] = z(c.reg_slots * 4, i64)
        t["asg_ctx"] = full(c.max_assignments * 4, -1, i32)
        t["asg_active"] = z(c.max_assignments, u8)
        # dedup window
        # two generations (see k_dedup_rotate) of packed 16-byte slots {alternate-id hash, first sequence}
        t["dd_tab"] = z(4 * c.dedup_slots, i64).view(2 * c.dedup_slots, 2)
        t["dd_tab"][:, 1] = -1
        # store-backed dedup filter: generational fingerprint tables of the persisted alternate ids
        # (pipeline/dedup_filter.py; [buckets][gens][16] u32, meta words)
        self._ff_on = c.dedup_filter_ids > 0
        t["dd_ff"] = z(max(16, c.ff_buckets * c.dedup_filter_gens * 16) if self._ff_on else 16, torch.int32)
        from .dedup_filter import meta_words
        t["dd_ff_meta"] = torch.from_numpy(meta_words(c.dedup_filter_gens, max(1, c.dedup_filter_ids))).to(d)
        t["dd_meta"] = torch.from_numpy(self._armed_dedup_meta(np.zeros(4, np.int64), c)).to(d)
        t["seq_base"] = z(1, i64)
        # names intern
        t["nm_key"] = z(c.name_slots, i64)
        t["nm_id"] = full(c.name_slots, -1, i32)
        t["nm_first"] = full(c.name_slots, 0x7FFFFFFF, i32)
        t["nm_counter"] = z(1, i32)
        # device state (packed SwAsgState per assignment, SwMsSlot map)
        t["st"] = z(c.max_assignments * 4, i64)
        t["ms"] = z(c.state_slots * 4, i64)
        # event store (SoA ring)
        sc = c.store_cap
        t["cursor"] = z(2, i64)  # [store_cursor, step_cursor0]
        self.store = {
            "etype": z(sc, u8), "level": z(sc, u8), "date": z(sc, i64), "recv": z(sc, i64), "dev": z(sc, i32),
            "asg": z(sc, i32), "cust": z(sc, i32), "area": z(sc, i32), "asset": z(sc, i32), "name": z(sc, i64),
            "v0": z(sc, torch.float64), "v1": z(sc, torch.float64), "v2": z(sc, torch.float64), "alt": z(sc, i64),
            "aux": z(sc, i64), "batch": z(sc, i32),
        }
        # outbound ring: mapped pinned host memory the kernels store into (zero-copy), double-buffered
        out_cap = c.rec_cap + c.gen_cap
        self.out_cap = out_cap
        self.n_out_bufs = int(c.extra.get("out_buffers", 3))
        self.out_host = [HostBuffer(self.lib, out_cap * OUT_REC_SIZE) for _ in range(self.n_out_bufs)]
        # device-side staging for the outbound push (see PipelinedRunner); OUTBOUND_MODE=direct stores to host
        self.out_dev = [z(out_cap * OUT_REC_SIZE, u8) for _ in range(self.n_out_bufs)]
        # rules
        t["gen"] = z(c.gen_cap * EVENT_REC.itemsize, u8)
        t["gen_dev"] = z(c.gen_cap, i32)
        t["gen_asg"] = z(c.gen_cap, i32)
        t["ev_slot"] = z(2 * max(c.rec_cap, c.gen_cap), torch.int64)   # (slot, date) state pass-2 items
        t["zmask"] = z(c.rec_cap, i64)
        t["ztile"] = z(2 * ntiles + 64, i32)
        t["stats"] = z(N_STATS, i64)
        t["sp"] = z(8, i64)                      # SwStepParams (per-step values read by the process phase)
        self._set_zone_tensors()
        self.args = a = SwEngineArgs()
        sc_ptr = _ptr(t["scalars"])
        S = lambda k: sc_ptr + 4 * k  # noqa: E731
        a.rank, a.world = c.rank, c.world
        a.msg_cnt, a.msg_evoff = _ptr(t["msg_cnt"]), _ptr(t["msg_evoff"])
        a.scan_tmp, a.scan_tmp_len = _ptr(t["scan_tmp"]), scan_tmp
        a.recs, a.rec_cap, a.n_recs = _ptr(t["recs"]), c.rec_cap, S(0)
        a.spans = _ptr(t["spans"])
        a.seen_key, a.seen_mask = _ptr(t["seen_key"]), c.name_slots - 1
        a.new_names, a.n_new_names, a.names_cap = _ptr(t["new_names"]), S(1), c.names_cap
        a.overflow = S(2)
        if c.world > 1:
            a.recv, a.shuf_cap, a.recv_cnt = _ptr(t["recv"]), c.shuf_cap, _ptr(t["recv_cnt"])
            if c.str_cap:
                a.recv_str, a.recv_str_cnt, a.recv_spans = _ptr(t["recv_str"]), _ptr(t["recv_str_cnt"]), _ptr(t["recv_spans"])
                a.work_str, a.work_spans, a.str_cap = _ptr(t["work_str"]), _ptr(t["work_spans"]), c.str_cap
            a.part_tmp, a.part_tmp_len = _ptr(t["part_tmp"]), t["part_tmp"].numel() // 2
            a.work = _ptr(t["work"])
            a.carry_cap = c.carry_cap
            a.part_owner = _ptr(t["part_owner"])
            a.part_bytes, a.part_meta = _ptr(t["part_bytes"]), _ptr(t["part_meta"])
            if c.str_cap:
                a.part_len, a.carry_str_cap = _ptr(t["part_len"]), c.carry_str_cap
        else:
            a.work = a.recs
        a.str_drops = _ptr(t["str_drops"])
        a.n_work = S(3)
        a.status, a.ev_dev, a.ev_asg = _ptr(t["status"]), _ptr(t["ev_dev"]), _ptr(t["ev_asg"])
        a.ok_idx, a.n_ok, a.rej_idx, a.n_rej = _ptr(t["ok_idx"]), S(4), _ptr(t["rej_idx"]), S(5)
        a.cmp_tmp = _ptr(t["cmp_tmp"])
        if c.cluster:
            a.cl_keys, a.cl_vals, a.cl_hist, a.cl_bits = _ptr(t["cl_keys"]), _ptr(t["cl_vals"]), _ptr(t["cl_hist"]), c.cl_bits
        a.reg, a.reg_mask = _ptr(t["reg"]), c.reg_slots - 1
        a.asg_ctx, a.asg_active, a.n_asg = _ptr(t["asg_ctx"]), _ptr(t["asg_active"]), c.max_assignments
        a.dd_key, a.dd_seq, a.dd_mask, a.seq_base = _ptr(t["dd_tab"]), 0, c.dedup_slots - 1, _ptr(t["seq_base"])
        a.dd_ff = _ptr(t["dd_ff"]) if self._ff_on else 0
        a.dd_ff_bmask = c.ff_buckets - 1 if self._ff_on else 0
        a.dd_ff_gens = c.dedup_filter_gens if self._ff_on else 0
        a.dd_ff_meta = _ptr(t["dd_ff_meta"])
        a.dd_meta = _ptr(t["dd_meta"])
        a.nm_key, a.nm_id, a.nm_first = _ptr(t["nm_key"]), _ptr(t["nm_id"]), _ptr(t["nm_first"])
        a.nm_mask, a.nm_counter = c.name_slots - 1, _ptr(t["nm_counter"])
        a.st, a.ms, a.ms_mask = _ptr(t["st"]), _ptr(t["ms"]), c.state_slots - 1
        a.ev_slot = _ptr(t["ev_slot"])
        a.store_cap = sc
        a.store_cursor = _ptr(t["cursor"])
        a.step_cursor0 = _ptr(t["cursor"]) + 8
        st = self.store
        (a.s_etype, a.s_level, a.s_date, a.s_recv, a.s_dev, a.s_asg, a.s_cust, a.s_area, a.s_asset, a.s_name,
         a.s_v0, a.s_v1, a.s_v2, a.s_alt, a.s_aux, a.s_batch) = [
            _ptr(st[k]) for k in ("etype", "level", "date", "recv", "dev", "asg", "cust", "area", "asset", "name",
                                  "v0", "v1", "v2", "alt", "aux", "batch")]
        a.out, a.n_out = self.out_host[0].dev, S(7)
        a.gen, a.gen_dev, a.gen_asg, a.n_gen, a.gen_cap = _ptr(t["gen"]), _ptr(t["gen_dev"]), _ptr(t["gen_asg"]), S(6), c.gen_cap
        a.zmask, a.ztile = _ptr(t["zmask"]), _ptr(t["ztile"])
        a.presence_missing_ms = 0
        a.presence_name_hash = self.presence_hash
        a.stats = _ptr(t["stats"])
        a.sp = _ptr(t["sp"])
        self._rule_scratch = S(8)
        # hipGraph of the process phase: captured on first use, replayed each step, re-captured
        # whenever a by-value argument of its kernels changes (zone rules)
        import os
        self.use_graph = os.environ.get("SW_GRAPH", "1") != "0"
        self._graph = None
        self._cap_stream = torch.cuda.Stream(self.device) if self.use_graph else None
        self._out_sel = 0
        # multi-rank exchange state: parity of the send slabs / carry buffer the next partition uses
        self._send_par = 0
        self._carry_par = 0
        self._last_send_par = 0
        # pipelined exchange (round_async): the batch whose exchange is in flight, and its events
        self._pend = None
        self._comm = torch.cuda.Stream(self.device) if c.world > 1 else None
        self._ev_part = torch.cuda.Event()
        self._ev_unp = torch.cuda.Event()
        self._ev_x = torch.cuda.Event()
        self._graph_nu = None                  # process graph without unpack (pipelined rounds)
        self._apply_zone_ptrs()

    # ------------------------------------------------------------------ control-plane hooks
    def _h2d(self, dst: torch.Tensor, src: np.ndarray):
        dst.copy_(torch.from_numpy(np.ascontiguousarray(src)).view(dst.dtype).reshape(dst.shape), non_blocking=False)

    def _upload_slots(self, slots: np.ndarray):
        slots = np.unique(np.asarray(slots, np.int64))
        slots = slots[slots >= 0]
        if not len(slots):
            return
        rows = self.packed_registry(slots).view(np.int64).reshape(-1, 4)
        reg = self.t["reg"].view(-1, 4)
        if len(slots) > self.cfg.reg_slots // 4:
            full = self.packed_registry(np.arange(self.cfg.reg_slots)).view(np.int64)
            self.t["reg"].copy_(torch.from_numpy(full))
            return
        reg.index_copy_(0, torch.from_numpy(slots).to(self.device), torch.from_numpy(np.ascontiguousarray(rows)).to(self.device))
        self._control_done()

    def _control_done(self):
        """Complete a control-plane table write before the update returns.  Registry and assignment
        changes come from the model-update consumer thread, whose current stream is not the one
        steps are enqueued on (another thread's, or a pipeline stream): left in flight, the scatter
        raced the next step's lookup, which then saw the device as unregistered (a tenant test's
        first batch persisted nothing).  Control-plane writes are rare; one stream sync each."""
        torch.cuda.current_stream(self.device).synchronize()

    def _dirty_registry(self, slots: np.ndarray):
        self._upload_slots(slots)

    def _dirty_assignments(self, idx):
        idx = np.unique(np.asarray(idx, np.int64))
        ctx = np.stack([self.asg_device[idx], self.asg_customer[idx], self.asg_area[idx], self.asg_asset[idx]], 1)
        it = torch.from_numpy(idx).to(self.device)
        self.t["asg_ctx"].view(-1, 4).index_copy_(0, it, torch.from_numpy(np.ascontiguousarray(ctx, np.int32)).to(self.device))
        self.t["asg_active"].index_copy_(0, it, torch.from_numpy(np.ascontiguousarray(self.asg_active[idx])).to(self.device))
        self._control_done()

    def _dirty_devices(self, idx):
        idx = np.asarray(idx, np.int64)
        self._upload_slots(self.dev_slot[idx])

    def _set_zone_tensors(self):
        vtx, off, bbox, tests, hashes = self.zone_arrays()
        d = self.device
        self.t["zone_vtx"] = torch.from_numpy(vtx).to(d)
        self.t["zone_off"] = torch.from_numpy(off).to(d)
        self.t["zone_bbox"] = torch.from_numpy(bbox).to(d)
        self.t["tests"] = torch.from_numpy(tests.view(np.uint8).copy() if len(tests) else np.zeros(16, np.uint8)).to(d)
        self.t["test_hash"] = torch.from_numpy(hashes.view(np.int64).copy() if len(hashes) else np.zeros(1, np.int64)).to(d)
        self._n_zones, self._n_tests = len(off) - 1, len(tests)
        self._n_zone_vtx = int(off[-1]) if len(off) else 0

    def _apply_zone_ptrs(self):
        a = self.args
        a.zone_vtx, a.zone_off, a.zone_bbox = _ptr(self.t["zone_vtx"]), _ptr(self.t["zone_off"]), _ptr(self.t["zone_bbox"])
        a.n_zones, a.tests, a.n_tests = self._n_zones, _ptr(self.t["tests"]), self._n_tests
        a.n_zone_vtx = self._n_zone_vtx
        a.test_name_hash = _ptr(self.t["test_hash"])

    def _zones_changed(self):
        if hasattr(self, "args"):
            self._set_zone_tensors()
            self._apply_zone_ptrs()
            self._drop_graph()

    def _drop_graph(self):
        for attr in ("_graph", "_graph_nu"):
            if getattr(self, attr, None) is not None:
                self._sync_streams()
                self.lib.sw_graph_destroy(ctypes.c_void_p(getattr(self, attr)))
                setattr(self, attr, None)

    # ------------------------------------------------------------------ data plane
    def step_async(self, raw_dev: torch.Tensor, off_dev: torch.Tensor, n_msgs: int, now_ms: int,
                   presence: bool = False, out_sel: int | None = None, out_to_device: bool = False):
        """Enqueue one micro-batch on the current stream.  raw_dev needs >= 16 B of tail padding."""
        sel = self.prepare(raw_dev, off_dev, n_msgs, now_ms, presence, out_sel, out_to_device)
        self.phase_decode()
        if self.world > 1:
            self.phase_exchange()
        self.phase_process()
        return sel

    def prepare(self, raw_dev, off_dev, n_msgs, now_ms, presence=False, out_sel=None, out_to_device=False):
        self._set_batch(raw_dev, off_dev, n_msgs, now_ms)
        return self._set_step_params(now_ms, presence, out_sel, out_to_device)

    def _set_batch(self, raw_dev, off_dev, n_msgs, now_ms):
        """By-value decode arguments of the next decode phase."""
        if n_msgs > self.cfg.max_msgs:
            raise ValueError(f"batch of {n_msgs} payloads exceeds EngineConfig.max_msgs={self.cfg.max_msgs}")
        a = self.args
        a.raw, a.msg_off, a.n_msgs, a.now_ms = _ptr(raw_dev), _ptr(off_dev), int(n_msgs), int(now_ms)
        self._raw_bytes = int(raw_dev.numel())      # bound of the batch's strings (block encoder)

    def _set_step_params(self, now_ms, presence=False, out_sel=None, out_to_device=False):
        """Stream-ordered SwStepParams of the next process phase (receive time, batch, presence, rows)."""
        a = self.args
        a.batch_seq = self.batch_seq
        self._step_now = int(now_ms)           # receive time of the batch this process phase runs
        a.presence_missing_ms = self.cfg.presence_missing_ms if presence else 0
        sel = self._out_sel if out_sel is None else out_sel
        self._last_sel = sel
        a.out = _ptr(self.out_dev[sel]) if out_to_device else self.out_host[sel].dev
        # rows kept on the device may be encoded into a durable block: the persist kernel writes each
        # row's encoder aux beside it
        aux = _ptr(self._aux_buffer(sel)) if out_to_device else 0
        # strings: the raw batch on one rank; the exchanged string slabs (work_str) on several
        raw_bytes = getattr(self, "_raw_bytes", 0) if self.world == 1 else self.world * self.cfg.str_cap
        rc = self.lib.sw_set_step_params(ctypes.c_void_p(a.sp), int(now_ms), a.batch_seq, a.presence_missing_ms,
                                         ctypes.c_void_p(a.out), ctypes.c_void_p(aux), int(raw_bytes), self._stream())
        if rc:
            raise RuntimeError(f"sw_set_step_params failed ({rc})")
        return sel

    # The three phases of a step (split so a multi-rank step can be driven without torch.distributed,
    # e.g. the loopback test that runs W engine shards on one GPU).
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _sync_streams(self):
        """Wait for this engine's work only: the caller's current stream plus the engine's own
        streams.  Never a device-wide synchronize -- several engines (tenants, replicas) can share a
        GPU, and a device sync both waits on their work and breaks a hipGraph capture another
        engine has in progress ("operation not permitted when stream is capturing")."""
        torch.cuda.current_stream(self.device).synchronize()
        for s in (getattr(self, "_comm", None), getattr(self, "_cap_stream", None)):
            if s is not None:
                s.synchronize()
        fp = self.__dict__.get("_fp")
        if fp is not None:
            fp.h2d.synchronize()
            fp.d2h.synchronize()

    def frame_varint(self, lens_dev: torch.Tensor, nbytes: int, n_msgs: int, off_dev: torch.Tensor, raw_bytes: int):
        """Rebuild u32 payload offsets from the varint length stream on the current stream."""
        if n_msgs > self.cfg.max_msgs or nbytes > lens_dev.numel() or off_dev.numel() < n_msgs + 1:
            raise ValueError("varint framing buffers too small for this batch")
        rc = self.lib.sw_frame_varint(ctypes.c_void_p(_ptr(lens_dev)), int(nbytes), int(n_msgs),
                                      ctypes.c_void_p(_ptr(off_dev)), int(raw_bytes),
                                      ctypes.c_void_p(_ptr(self.t["vlen_tmp"])), self.t["vlen_tmp"].numel(),
                                      self._stream())
        if rc:
            raise RuntimeError(f"sw_frame_varint failed ({rc})")

    def phase_decode(self):
        ap = ctypes.byref(self.args)
        rc = self.lib.sw_phase_decode(ap, self._stream())
        if rc:
            raise RuntimeError(f"sw_phase_decode failed ({rc})")
        if self.world > 1:
            a = self.args
            sp, cp = self._send_par, self._carry_par
            a.send, a.send_cnt = _ptr(self.send_bufs[sp]), _ptr(self.send_cnts[sp])
            if self.cfg.str_cap:
                a.send_str, a.send_str_cnt = _ptr(self.send_strs[sp]), _ptr(self.send_str_cnts[sp])
                a.send_spans = _ptr(self.send_spans[sp])
            a.carry, a.n_carry = _ptr(self.carry_bufs[cp]), _ptr(self.t["n_carry"]) + 4 * cp
            a.spill, a.n_spill = _ptr(self.carry_bufs[1 - cp]), _ptr(self.t["n_carry"]) + 4 * (1 - cp)
            if self.cfg.str_cap:
                a.carry_spans, a.carry_str = _ptr(self.carry_spans[cp]), _ptr(self.carry_strs[cp])
                a.spill_spans, a.spill_str = _ptr(self.carry_spans[1 - cp]), _ptr(self.carry_strs[1 - cp])
                a.n_spill_str = _ptr(self.t["n_carry_str"]) + 4 * (1 - cp)
            rc = self.lib.sw_phase_partition(ap, self._stream())
            if rc:
                raise RuntimeError(f"sw_phase_partition failed ({rc})")
            self._last_send_par = sp
            self._send_par, self._carry_par = 1 - sp, 1 - cp

    def phase_exchange(self):
        """RCCL all-to-all re-keying of the per-owner slabs (the Kafka key-partitioning analogue)."""
        from ..parallel.sharding import exchange_slabs
        p = self._last_send_par
        extra = ()
        if self.cfg.str_cap:
            extra = ((self.send_str_cnts[p], self.t["recv_str_cnt"]), (self.send_spans[p], self.t["recv_spans"]),
                     (self.send_strs[p], self.t["recv_str"]))
        exchange_slabs(self.send_cnts[p], self.t["recv_cnt"], self.send_bufs[p], self.t["recv"], self.group, extra)

    def phase_unpack(self):
        rc = self.lib.sw_phase_unpack(ctypes.byref(self.args), self._stream())
        if rc:
            raise RuntimeError(f"sw_phase_unpack failed ({rc})")

    def _capture(self, with_unpack: bool):
        ex = ctypes.c_void_p()
        rc = self.lib.sw_graph_capture_process(ctypes.byref(self.args), ctypes.c_void_p(self._rule_scratch),
                                               int(with_unpack), ctypes.c_void_p(self._cap_stream.cuda_stream),
                                               ctypes.byref(ex))
        if rc:
            import warnings
            warnings.warn(f"hipGraph capture of the process phase failed ({rc}); using direct launches")
            self.use_graph = False
            return None
        return ex.value

    def phase_process(self, with_unpack: bool | None = None):
        """Process phase of the batch in ``work`` (unpacked from the receive slabs first when world > 1,
        unless the caller already ran :meth:`phase_unpack`)."""
        unpack = self.world > 1 if with_unpack is None else with_unpack
        ap = ctypes.byref(self.args)
        if self.use_graph:
            attr = "_graph" if unpack or self.world == 1 else "_graph_nu"
            if getattr(self, attr) is None:
                setattr(self, attr, self._capture(unpack))
            g = getattr(self, attr)
            if g is not None:
                rc = self.lib.sw_graph_launch(ctypes.c_void_p(g), self._stream())
                if rc:
                    raise RuntimeError(f"sw_graph_launch failed ({rc})")
                self.batch_seq += 1
                return
        if unpack:
            self.phase_unpack()
        rc = self.lib.sw_phase_process(ap, ctypes.c_void_p(self._rule_scratch), self._stream())
        if rc:
            raise RuntimeError(f"sw_phase_process failed ({rc})")
        self.batch_seq += 1

    # ------------------------------------------------------------------ pipelined exchange (world > 1)
    def round_async(self, raw_dev=None, off_dev=None, n_msgs: int = 0, now_ms: int = 0, presence: bool = False,
                    out_sel: int | None = None, out_to_device: bool = False, exchange: bool = True):
        """One round of the software-pipelined multi-rank step (see ``parallel/sharding.py``).

        On the current (compute) stream: decode + partition of the new batch (if ``raw_dev`` is given),
        then unpack + process of the previous batch, whose all-to-all ran on the communication stream
        meanwhile.  Then the all-to-all of the new batch is enqueued on the communication stream; it
        overlaps this round's process phase.  ``out_sel`` names the outbound buffer of the rows this
        round produces.  Returns True when a batch was processed (False on the first round).
        ``exchange=False`` leaves the exchange to the caller (loopback tests), who then calls
        :meth:`exchange_done` on the stream that performed it.
        """
        if self.world == 1:
            raise RuntimeError("round_async is the multi-rank pipeline; use step_async for world == 1")
        cur = torch.cuda.current_stream(self.device)
        new = None
        if raw_dev is not None:
            self._set_batch(raw_dev, off_dev, n_msgs, now_ms)
            self.phase_decode()
            self._ev_part.record(cur)
            new = (int(now_ms), bool(presence))
        processed = False
        if self._pend is not None:
            p_now, p_presence = self._pend
            cur.wait_event(self._ev_x)
            self._set_step_params(p_now, p_presence, out_sel, out_to_device)
            self.phase_unpack()
            self._ev_unp.record(cur)
            self.phase_process(with_unpack=False)
            processed = True
        self._pend = new
        if new is not None and exchange:
            comm = self._comm
            comm.wait_event(self._ev_part)
            if processed:
                comm.wait_event(self._ev_unp)      # the single receive buffer is free once unpacked
            with torch.cuda.stream(comm):
                self.phase_exchange()
                self._ev_x.record(comm)
        return processed

    def exchange_done(self, stream=None):
        """Mark the pending batch's exchange complete at this point of ``stream`` (manual exchange)."""
        self._ev_x.record(stream or torch.cuda.current_stream(self.device))

    @property
    def exchange_pending(self) -> bool:
        return self._pend is not None

    def send_slab(self, q: int) -> torch.Tensor:
        """Destination-q slab (packed WIRE_REC) of the most recent partition."""
        n = self.cfg.shuf_cap * WIRE_REC.itemsize
        return self.send_bufs[self._last_send_par][q * n:(q + 1) * n]

    def send_count(self, q: int) -> torch.Tensor:
        return self.send_cnts[self._last_send_par][q]

    def recv_slab(self, q: int) -> torch.Tensor:
        n = self.cfg.shuf_cap * WIRE_REC.itemsize
        return self.t["recv"][q * n:(q + 1) * n]

    def loopback_strings(self, peers: list):
        """Loopback exchange of the string slabs (tests that run every rank's engine in one process):
        what the all-to-all in :meth:`phase_exchange` moves for them, copied from each peer's last
        partition into this engine's receive buffers (``peers[r]`` = rank r's engine)."""
        c = self.cfg
        if not c.str_cap:
            return
        sr = c.shuf_cap * STR_REF.itemsize
        q = self.rank
        for r, e in enumerate(peers):
            p = e._last_send_par
            self.t["recv_str_cnt"][r] = e.send_str_cnts[p][q]
            self.t["recv_spans"][r * sr:(r + 1) * sr].copy_(e.send_spans[p][q * sr:(q + 1) * sr])
            self.t["recv_str"][r * c.str_cap:(r + 1) * c.str_cap].copy_(
                e.send_strs[p][q * c.str_cap:(q + 1) * c.str_cap])

    def string_drops(self) -> dict:
        """Records sent without their strings because those alone exceed a whole slab (the only
        case: a record deferred by a full slab keeps its strings in the carry heap)."""
        v = self.t["str_drops"].cpu().numpy()
        return {"oversize": int(v[0])}

    def scalars(self) -> dict:
        v = self.t["scalars"][:9].cpu().numpy()
        return dict(n_recs=int(v[0]), n_new_names=int(v[1]), overflow=int(v[2]), n_work=int(v[3]), n_ok=int(v[4]),
                    n_rej=int(v[5]), n_gen=int(v[6]), n_out=int(v[7]), n_rule=int(v[8]))

    def step(self, raw: np.ndarray, offs: np.ndarray, now_ms: int, presence: bool | None = None) -> StepResult:
        """Synchronous convenience step (tests, control-plane use): H2D, run, D2H, learn names."""
        n_msgs = len(offs) - 1
        with self._lock:            # serialised against hot-store queries (cursor + shared scratch)
            self._no_framed_pending()
            raw_dev, off_dev = self._stage(raw, offs)
            do_presence = self.presence_due(now_ms) if presence is None else presence
            # rows land in HBM and come back in one DMA: reading them out of the mapped host buffer
            # is CPU-uncached (~2.6 GB/s measured, 0.8 ms per 64K rows; profiles/r1_tenant_step)
            sel = self.step_async(raw_dev, off_dev, n_msgs, now_ms, presence=do_presence, out_to_device=True)
            self._sync_streams()
            return self._with_block(self.collect(sel, raw, from_device=True), sel, now_ms)

    def decode_only(self, raw: np.ndarray, offs: np.ndarray, now_ms: int, spans: bool = False):
        """Run only the decode phase (``k_decode_count`` / ``k_decode_emit``) of a
        host batch and return the decoded ``EVENT_REC`` records in batch order.  A test hook: it
        checks the device decoder against an independent decoder (``tests/decode_oracle.py``)
        without validation rewriting the records.  Names it sees count as seen by later steps.
        ``spans``: also return the records' string refs (STR_REF)."""
        n_msgs = len(offs) - 1
        with self._lock:
            self._no_framed_pending()
            raw_dev, off_dev = self._stage(raw, offs)
            self._set_batch(raw_dev, off_dev, n_msgs, now_ms)
            rc = self.lib.sw_phase_decode(ctypes.byref(self.args), self._stream())
            if rc:
                raise RuntimeError(f"sw_phase_decode failed ({rc})")
            self._sync_streams()
            n = min(int(self.t["scalars"][0].item()), self.cfg.rec_cap)
            recs = self.t["recs"][:n * EVENT_REC.itemsize].cpu().numpy().view(EVENT_REC).copy()
            if not spans:
                return recs
            return recs, self.t["spans"][:n * STR_REF.itemsize].cpu().numpy().view(STR_REF).copy()

    def step_framed(self, batch, now_ms: int, presence: bool | None = None) -> StepResult:
        """Synchronous step of a raw-payload record read from the bus: the payload (with its padding)
        and the varint lengths are DMA'd straight from the record -- in place when the record is a
        pinned zero-copy record of the topic, no host staging copy -- and the offsets are rebuilt on
        the GPU (``sw_frame_varint``)."""
        if batch.lens is None:
            return EngineBase.step_framed(self, batch, now_ms, presence)
        import warnings
        n, nb, nl = batch.n_msgs, len(batch.payload), len(batch.lens)
        if n > self.cfg.max_msgs:
            raise ValueError(f"batch of {n} payloads exceeds EngineConfig.max_msgs={self.cfg.max_msgs}")
        if nb < batch.payload_bytes + _ALIGN:
            raise ValueError("raw batch payload lacks its tail padding")
        with self._lock:
            self._no_framed_pending()
            st = getattr(self, "_stg_framed", None)
            if st is None or st[0].numel() < nb or st[1].numel() < nl:
                st = self._stg_framed = (
                    torch.empty(max(nb, int(getattr(self, "_stg_hint", 0))), dtype=torch.uint8, device=self.device),
                    torch.empty(max(nl, 5 * self.cfg.max_msgs + 64), dtype=torch.uint8, device=self.device),
                    torch.empty(self.cfg.max_msgs + 1, dtype=torch.int32, device=self.device))
            dev_r, dev_l, dev_o = st
            with warnings.catch_warnings():       # read-only topic views: torch only reads them here
                warnings.simplefilter("ignore", UserWarning)
                pt = torch.frombuffer(batch.payload, dtype=torch.uint8) if nb else None
                lt = torch.frombuffer(batch.lens, dtype=torch.uint8) if nl else None
            if pt is not None:
                dev_r[:nb].copy_(pt, non_blocking=True)
            if lt is not None:
                dev_l[:nl].copy_(lt, non_blocking=True)
            self.frame_varint(dev_l, nl, n, dev_o, batch.payload_bytes)
            do_presence = self.presence_due(now_ms) if presence is None else presence
            sel = self.step_async(dev_r[:nb], dev_o[:n + 1], n, now_ms, presence=do_presence, out_to_device=True)
            self._sync_streams()
            return self._with_block(self.collect(sel, np.asarray(batch.payload), from_device=True), sel, now_ms)

    # durable blocks of service tenants (``storage: durable``): every step's block is encoded on the
    # MI355X and returned with its result (``StepResult.block``), sealed with ``block_boot``
    encode_blocks = False
    block_boot = 0

    def _with_block(self, res: StepResult, sel: int, now_ms: int) -> StepResult:
        if self.encode_blocks:
            res.block = self.encode_block(now_ms, res, slot=sel, boot=self.block_boot)
        return res

    def _no_framed_pending(self):
        fp = self.__dict__.get("_fp")
        if fp is not None and fp.inflight:
            raise RuntimeError("a submitted framed batch is pending: drain_framed() before a synchronous step")

    def _stage(self, raw: np.ndarray, offs: np.ndarray):
        """H2D of a host batch through persistent pinned staging (a pageable ``.to(device)`` ran at
        ~6 GB/s plus a fresh padded copy per batch).  Only for the synchronous :meth:`step`: the
        staging buffers are reused by the next call."""
        nb, no = len(raw) + _ALIGN, len(offs)
        st = getattr(self, "_stg", None)
        if st is None or st[0].numel() < nb or st[1].numel() < no:
            cap_b = max(nb, int(getattr(self, "_stg_hint", 0)))
            pin_r = torch.empty(cap_b, dtype=torch.uint8).pin_memory()
            pin_o = torch.empty(max(no, self.cfg.max_msgs + 1), dtype=torch.int32).pin_memory()
            st = self._stg = (pin_r, pin_o, torch.empty(cap_b, dtype=torch.uint8, device=self.device),
                              torch.empty(pin_o.numel(), dtype=torch.int32, device=self.device))
        pin_r, pin_o, dev_r, dev_o = st
        pr = pin_r.numpy()
        pr[:len(raw)] = raw
        pr[len(raw):nb] = 0
        pin_o.numpy()[:no] = np.asarray(offs, np.uint32).view(np.int32)
        dev_r[:nb].copy_(pin_r[:nb], non_blocking=True)
        dev_o[:no].copy_(pin_o[:no], non_blocking=True)
        return dev_r[:nb], dev_o[:no]

    ROW_HEADROOM = 1 << 16      # bytes kept free in front of the rows: a columnar batch header is
                                # written there, making header + rows one contiguous payload

    def _pinned_out(self, nbytes: int, kind: str = "rows"):
        """A pinned host buffer (torch tensor + its full numpy view) with ``ROW_HEADROOM`` bytes in
        front of the rows, that no earlier StepResult still references: a live ``result.out`` view
        pins its base array, so results are returned without a copy and without fresh pageable pages
        per step.  Returns (tensor, array, pooled); a result whose buffer is not pooled must not be
        retained (``StepResult.frame_base`` is left unset)."""
        import sys
        need = nbytes + self.ROW_HEADROOM
        sfx = "" if kind == "rows" else "_" + kind
        pool = self.__dict__.setdefault("_pin_pool" + sfx, [])
        spill = self.__dict__.setdefault("_pin_spill" + sfx, [])
        st = self.__dict__.setdefault("pin_stats" + sfx, {"reused": 0, "new_pooled": 0, "spill": 0,
                                                          "new_unpooled": 0})
        for pin, arr in pool:
            if arr.nbytes >= need and sys.getrefcount(arr) <= 3:   # pool tuple, loop variable, the call
                st["reused"] += 1
                return pin, arr, True
        # sized to this step's rows plus slack (steps of one tenant are about the same size), not to
        # the engine's full output capacity: pinning a buffer costs time in proportion to its size
        if kind == "rows":
            full = self.out_cap * OUT_REC_SIZE + self.ROW_HEADROOM
        else:
            from ..persistence.segments import max_block_bytes
            full = max_block_bytes(self.out_cap) + self.ROW_HEADROOM
        size = max(need, min(full, -(-(need + need // 4) // (1 << 20)) * (1 << 20)))
        # never smaller than the largest pooled buffer: steps of a tenant that coalesces records vary
        # in size, and pinning a fresh buffer for each new maximum costs milliseconds per step
        if pool:
            size = max(size, min(full, max(a.nbytes for _, a in pool)))
        # results held by an overlapped tenant: in flight + store queue + storing, and -- with zero-copy
        # columnar payloads -- the batches the store and the enriched-batch topic retain
        if len(pool) < (self.PIN_POOL if kind == "rows" else self.PIN_POOL_BLOCKS):
            pin = torch.empty(size, dtype=torch.uint8).pin_memory()
            pool.append((pin, pin.numpy()))
            st["new_pooled"] += 1
            return pin, pool[-1][1], True
        # every pooled buffer is retained downstream: hand out a spill buffer that must not be
        # retained (the caller copies its rows), so a full pool costs a copy, not a pinned
        # allocation per step
        for pin, arr in spill:
            if arr.nbytes >= need and sys.getrefcount(arr) <= 3:
                st["spill"] += 1
                return pin, arr, False
        pin = torch.empty(size, dtype=torch.uint8).pin_memory()
        if len(spill) < self.PIN_SPILL:
            spill.append((pin, pin.numpy()))
            st["spill"] += 1
            return pin, spill[-1][1], False
        st["new_unpooled"] += 1
        return pin, pin.numpy(), False

    PIN_POOL = 24
    PIN_POOL_BLOCKS = 64        # durable blocks: also held by the enriched-batch topic's retention window
    PIN_SPILL = 6

    def collect(self, sel: int, raw_host: np.ndarray | None, from_device: bool = False) -> StepResult:
        part = self._collect_small(raw_host)
        n_out = part["n_persisted"]
        frame = None
        if from_device:
            nb = n_out * OUT_REC_SIZE
            h = self.ROW_HEADROOM
            pin, arr, pooled = self._pinned_out(nb)
            if nb:
                pin[h:h + nb].copy_(self.out_dev[sel][:nb])      # pinned target: a full-rate DMA
            out = arr[h:h + nb].view(OUT_REC)
            frame = (arr, h) if pooled else None
        else:
            out = self.out_host[sel].view(OUT_REC, n_out).copy()
        return StepResult(out=out, world=self.world, rank=self.rank, frame_base=frame, **part)

    def _collect_small(self, raw_host: np.ndarray | None) -> dict:
        """Everything of the last step but its rows: counts, learned names, first store sequence and
        rejected records.  Reads tables the next step overwrites, so it runs before that step is
        enqueued."""
        sc = self.scalars()
        nn = min(sc["n_new_names"], self.cfg.names_cap)
        new = {}
        if nn and raw_host is not None:
            refs = self.t["new_names"][:nn * NAME_REF.itemsize].cpu().numpy().view(NAME_REF)
            new = self.learn_names(refs, raw_host)
        first_seq = int(self.t["cursor"][1].item())
        n_rej = sc["n_rej"]
        if n_rej:
            work = self.t["work"] if self.world > 1 else self.t["recs"]
            rej_idx = self.t["rej_idx"][:n_rej].long()
            rows = work.view(-1, EVENT_REC.itemsize)[rej_idx].cpu().numpy().reshape(-1).view(EVENT_REC)
            rst = self.t["status"][rej_idx].cpu().numpy()
        else:
            rows, rst = np.zeros(0, EVENT_REC), np.zeros(0, np.uint8)
        recheck = None
        if n_rej and self.world > 1 and self.cfg.str_cap:
            rk = np.nonzero(rst == ST_RECHECK)[0]
            if len(rk):
                # the owner settles them by alternate id: their strings, gathered from work_str
                from .recheck import compact_strings
                ridx = rej_idx[torch.from_numpy(rk).to(rej_idx.device)]
                sp = self.t["work_spans"].view(-1, STR_REF.itemsize)[ridx].cpu().numpy().reshape(-1).view(STR_REF)
                ws = self.t["work_str"]
                recheck = compact_strings(rows[rk], sp, lambda pos: ws[torch.from_numpy(pos).to(ws.device)].cpu().numpy())
        return dict(n_msgs=int(self.args.n_msgs), n_events=sc["n_work"], n_persisted=sc["n_out"], rejects=rows,
                    reject_status=rst, new_names=new, first_seq=first_seq, recheck=recheck)

    def rechecks(self, res):
        """The step's rechecks with their strings (records, refs, heap), or None (see
        ``pipeline/recheck.py``)."""
        return res.recheck

    def inject_settled(self, recs, spans, heap):
        """Re-inject records whose store-backed dedup the host settled at the end of the re-key
        carry the next partition reads, strings appended to its heap (``F_SETTLED``: the filter
        skips them).  Call between rounds."""
        from ..models.columnar import F_SETTLED
        from .recheck import rebase_into
        if self.world == 1 or not self.cfg.str_cap:
            raise RuntimeError("settled records re-enter through the re-key carry (several ranks, strings on)")
        self._sync_streams()
        cp = self._carry_par
        n, nb, k = int(self.t["n_carry"][cp].item()), int(self.t["n_carry_str"][cp].item()), len(recs)
        heap = np.asarray(heap, np.uint8)
        if n + k > self.cfg.carry_cap or nb + len(heap) > self.cfg.carry_str_cap:
            raise RuntimeError("re-key carry full: settle after a drain round")
        r, sp = rebase_into(recs, spans, nb, F_SETTLED)
        ri, si = EVENT_REC.itemsize, STR_REF.itemsize
        self.carry_bufs[cp][n * ri:(n + k) * ri].copy_(torch.from_numpy(np.ascontiguousarray(r).view(np.uint8)))
        self.carry_spans[cp][n * si:(n + k) * si].copy_(torch.from_numpy(np.ascontiguousarray(sp).view(np.uint8)))
        if len(heap):
            self.carry_strs[cp][nb:nb + len(heap)].copy_(torch.from_numpy(heap))
        self.t["n_carry"][cp] = n + k
        self.t["n_carry_str"][cp] = nb + len(heap)
        self.__dict__.pop("_carry_seen", None)
        self._sync_streams()

    # ------------------------------------------------------------------ overlapped framed steps
    def submit_framed(self, batch, now_ms: int, token=None, presence: bool | None = None) -> list:
        """Overlapped form of :meth:`step_framed` for service tenants (see ``EngineBase``).  Three
        slots of raw / offsets / outbound buffers rotate; submitting batch k

        1. enqueues the H2D of k's payload and lengths straight from the record on a copy stream
           (it runs while batch k-1 computes),
        2. returns batch k-2, whose rows the SDMA engine has been copying meanwhile,
        3. waits for batch k-1's compute and reads its counts, learned names and rejects (tables
           the next step overwrites),
        4. enqueues batch k's step and starts the SDMA copy of k-1's rows (no CUs: a HIP runtime
           D2H here runs as a blit kernel beside the step's kernels).

        The host never waits on a copy it just started, so PCIe stays busy in both directions."""
        if batch.lens is None or self.world > 1:
            return EngineBase.submit_framed(self, batch, now_ms, token, presence)
        import warnings
        parts = getattr(batch, "parts", None)          # coalesced records: DMA'd back to back
        n, nl = batch.n_msgs, len(batch.lens)
        nb = batch.payload_bytes + _ALIGN if parts is not None else len(batch.payload)
        if n > self.cfg.max_msgs:
            raise ValueError(f"batch of {n} payloads exceeds EngineConfig.max_msgs={self.cfg.max_msgs}")
        if nb < batch.payload_bytes + _ALIGN:
            raise ValueError("raw batch payload lacks its tail padding")
        tr = self.framed_trace
        t0 = time.perf_counter() if tr is not None else 0.0
        with self._lock:
            if getattr(self, "_lagged", None) is not None:      # a host-lagged batch (no lens) first
                done = EngineBase.drain_framed(self)
            else:
                done = []
            fp = self.__dict__.get("_fp")
            if fp is None:
                fp = self._fp = _FramedSlots(self)
            b = fp.k % _FramedSlots.SLOTS
            dev_r, dev_l, dev_o = fp.buffers(b, nb, nl)
            segs = []                                      # (device offset, host address, bytes)
            if parts is None:
                if nb:
                    segs.append((0, _host_addr(batch.payload), nb))
                lsegs = [(_host_addr(batch.lens), len(batch.lens))] if nl else []
            else:
                for part, st in zip(parts, batch.starts):
                    if part.payload_bytes:
                        segs.append((int(st), _host_addr(part.payload), part.payload_bytes))
                lsegs = [(_host_addr(part.lens), len(part.lens)) for part in parts if len(part.lens)]
            # the H2D of the zero-copy record straight from its pinned bytes, on the copy stream,
            # enqueued natively with the GIL held (see sw_memcpy_h2d_async)
            L, hs = self.lib, ctypes.c_void_p(fp.h2d.cuda_stream)
            _chk(L.sw_stream_wait_event(hs, ctypes.c_void_p(fp.ev_comp[b].cuda_event)))  # step k-3 read slot b last
            rd, ld = _ptr(dev_r), _ptr(dev_l)
            for st, src, m in segs:
                _chk(L.sw_memcpy_h2d_async(ctypes.c_void_p(rd + st), ctypes.c_void_p(src), int(m), hs))
            if parts is not None:                          # the records' zero padding, after the last part
                _chk(L.sw_memset_async(ctypes.c_void_p(rd + batch.payload_bytes), 0, _ALIGN, hs))
            lo = 0
            for src, m in lsegs:
                _chk(L.sw_memcpy_h2d_async(ctypes.c_void_p(ld + lo), ctypes.c_void_p(src), int(m), hs))
                lo += m
            _chk(L.sw_event_record(ctypes.c_void_p(fp.ev_h2d[b].cuda_event), hs))
            t0 = self._ft("h2d_enqueue", t0)
            while len(fp.inflight) > 1 or (fp.inflight and fp.inflight[0].rows is not None):
                done.append(self._framed_finish(fp.inflight.popleft()))      # batch k-2
            t0 = self._ft("finish_k2", t0)
            prev = fp.inflight[0] if fp.inflight else None
            if prev is not None:                                             # batch k-1
                fp.ev_comp[prev.slot].synchronize()
                t0 = self._ft("wait_k1", t0)
                prev.small = self._collect_done(fp, prev)
                t0 = self._ft("collect_k1", t0)
                self._block_meta(prev)              # before batch k is queued: no wait on it
                t0 = self._ft("block_meta_k1", t0)
            cur = torch.cuda.current_stream(self.device)
            _chk(self.lib.sw_stream_wait_event(ctypes.c_void_p(cur.cuda_stream),
                                               ctypes.c_void_p(fp.ev_h2d[b].cuda_event)))
            self.frame_varint(dev_l, nl, n, dev_o, batch.payload_bytes)
            do_presence = self.presence_due(now_ms) if presence is None else presence
            self.step_async(dev_r[:nb], dev_o[:n + 1], n, now_ms, presence=do_presence, out_sel=b,
                            out_to_device=True)
            sub = _Submitted(b, batch, token)
            if self.encode_blocks:
                sub.bmeta, sub.now = self.encode_block_async(b), now_ms
            if self.world == 1:
                self._snapshot_async(fp, b, sub)
            _chk(self.lib.sw_event_record(ctypes.c_void_p(fp.ev_comp[b].cuda_event), ctypes.c_void_p(cur.cuda_stream)))
            t0 = self._ft("step_enqueue", t0)
            if prev is not None:
                self._framed_rows_start(prev)
            t0 = self._ft("copies_start_k1", t0)
            fp.inflight.append(sub)
            fp.k += 1
            return done

    # SW_FRAMED_TRACE=1: host wall-clock per phase of submit_framed (seconds, summed)
    framed_trace = {} if os.environ.get("SW_FRAMED_TRACE") == "1" else None

    def _ft(self, name: str, t0: float) -> float:
        tr = self.framed_trace
        if tr is None:
            return t0
        t1 = time.perf_counter()
        tr[name] = tr.get(name, 0.0) + (t1 - t0)
        return t1

    def drain_framed(self) -> list:
        with self._lock:
            done = EngineBase.drain_framed(self) if getattr(self, "_lagged", None) is not None else []
            fp = self.__dict__.get("_fp")
            while fp is not None and fp.inflight:
                s = fp.inflight.popleft()
                if s.small is None:
                    fp.ev_comp[s.slot].synchronize()
                    s.small = self._collect_done(fp, s)
                    self._block_meta(s)
                    self._framed_rows_start(s)
                done.append(self._framed_finish(s))
            return done

    @property
    def framed_pending(self) -> int:
        fp = self.__dict__.get("_fp")
        return EngineBase.framed_pending.fget(self) + (len(fp.inflight) if fp is not None else 0)

    # rejects per step read from the mapped snapshot; a step with more goes through _collect_small
    MAPPED_REJECTS = 1 << 18

    def _snapshot_async(self, fp, b: int, sub: "_Submitted"):
        """Behind step ``sub`` on the current stream: its scalars and encoder meta
        (``k_step_snapshot``) and its rejected records with their statuses (``k_reject_pack``) into
        slot ``b``'s mapped host memory, so completing the step reads host memory only -- no
        synchronising device reads (each one gives the GIL up and waits to win it back from the
        tenant's other threads)."""
        bufs = fp.__dict__.setdefault("snap", {})
        cap = min(self.cfg.rec_cap, self.MAPPED_REJECTS)
        m = bufs.get(b)
        if m is None:
            m = bufs[b] = (HostBuffer(self.lib, 256), HostBuffer(self.lib, cap * EVENT_REC.itemsize),
                           HostBuffer(self.lib, cap))
        snap, rej, st = m
        st_ = self._stream()
        sc = ctypes.c_void_p(_ptr(self.t["scalars"]))
        meta = ctypes.c_void_p(sub.bmeta.data_ptr() if sub.bmeta is not None else 0)
        rc = self.lib.sw_step_snapshot(sc, meta, None, None, 1, ctypes.c_void_p(snap.dev), st_)
        if rc:
            raise RuntimeError(f"sw_step_snapshot failed ({rc})")
        rc = self.lib.sw_reject_pack(ctypes.c_void_p(_ptr(self.t["recs"])), ctypes.c_void_p(_ptr(self.t["rej_idx"])),
                                     ctypes.c_void_p(_ptr(self.t["status"])), sc, cap, ctypes.c_void_p(rej.dev),
                                     ctypes.c_void_p(st.dev), st_)
        if rc:
            raise RuntimeError(f"sw_reject_pack failed ({rc})")
        sub.mapped = True

    def _collect_done(self, fp, s: "_Submitted") -> dict:
        """:meth:`_collect_small` of a completed framed step, from its mapped snapshot when it has one
        (no device reads) -- unless the step learned names or rejected more than the snapshot holds."""
        if not s.mapped:
            return self._collect_small(host_view(s.batch))
        snap, rej, st = fp.snap[s.slot]
        v = snap.view(np.uint32, 32)
        n_rej = int(v[5])
        cap = min(self.cfg.rec_cap, self.MAPPED_REJECTS)
        if int(v[1]) or n_rej > cap or s.bmeta is None:
            return self._collect_small(host_view(s.batch))
        nb, err, first = (int(x) for x in snap.view(np.uint64, 11)[8:11])
        if err or nb <= 0 or nb > self._seg_buffers(s.slot)[3]:
            raise RuntimeError(f"durable block encoder failed (bytes={nb}, errors={err})")
        s.bmeta = (nb, first)
        rows = rej.view(EVENT_REC, n_rej).copy() if n_rej else np.zeros(0, EVENT_REC)
        rst = st.view(np.uint8, n_rej).copy() if n_rej else np.zeros(0, np.uint8)
        return dict(n_msgs=int(self.args.n_msgs), n_events=int(v[3]), n_persisted=int(v[7]), rejects=rows,
                    reject_status=rst, new_names={}, first_seq=first, recheck=None)

    def _framed_rows_start(self, s: "_Submitted"):
        """Start copying the rows (and the durable block) of completed step ``s`` to pinned host
        buffers."""
        if s.bmeta is not None:
            self._framed_block_start(s)
        nb = s.small["n_persisted"] * OUT_REC_SIZE
        s.rows = self._pinned_out(nb)
        if not nb:
            return
        fp = self._fp
        h = ctypes.c_uint64()
        rc = 1 if fp.no_sdma else self.lib.sw_sdma_copy(ctypes.c_void_p(s.rows[0].data_ptr() + self.ROW_HEADROOM),
                                                         ctypes.c_void_p(_ptr(self.out_dev[s.slot])), nb, 0,
                                                         ctypes.byref(h))
        if rc == 0:
            s.sig = h.value
            return
        fp.no_sdma = True                       # no copy engine on this node: HIP runtime copy
        with torch.cuda.stream(fp.d2h):
            hr = self.ROW_HEADROOM
            s.rows[0][hr:hr + nb].copy_(self.out_dev[s.slot][:nb], non_blocking=True)
            s.ev = torch.cuda.Event()
            s.ev.record(fp.d2h)

    def _block_meta(self, s: "_Submitted"):
        """Encoder result of completed step ``s`` (read while nothing newer is queued)."""
        if s.bmeta is None or isinstance(s.bmeta, tuple):
            return
        nb, err, first = (int(x) for x in s.bmeta.cpu().numpy())
        if err or nb <= 0 or nb > self._seg_buffers(s.slot)[3]:
            raise RuntimeError(f"durable block encoder failed (bytes={nb}, errors={err})")
        s.bmeta = (nb, first)

    def _framed_block_start(self, s: "_Submitted"):
        self._block_meta(s)
        nb = s.bmeta[0]
        s.bbuf = self._pinned_out(nb, kind="blocks")
        dst = s.bbuf[0].data_ptr() + self.ROW_HEADROOM
        fp = self._fp
        h = ctypes.c_uint64()
        rc = 1 if fp.no_sdma else self.lib.sw_sdma_copy(ctypes.c_void_p(dst), ctypes.c_void_p(_ptr(self.block_device(s.slot))),
                                                         nb, 0, ctypes.byref(h))
        if rc == 0:
            s.bsig = h.value
            return
        fp.no_sdma = True
        with torch.cuda.stream(fp.d2h):
            hr = self.ROW_HEADROOM
            s.bbuf[0][hr:hr + nb].copy_(self.block_device(s.slot)[:nb], non_blocking=True)
            s.bev = torch.cuda.Event()
            s.bev.record(fp.d2h)

    def _framed_block_finish(self, s: "_Submitted", res: StepResult):
        from ..persistence.segments import seal
        if s.bsig is not None:
            rc = self.lib.sw_sdma_wait(s.bsig)
            s.bsig = None
            if rc:
                raise RuntimeError(f"sw_sdma_wait failed ({rc})")
        elif s.bev is not None:
            s.bev.synchronize()
        nb, first = s.bmeta
        hr = self.ROW_HEADROOM
        pin, arr, pooled = s.bbuf
        blk = arr[hr:hr + nb]
        seal(blk, first, s.now, self.block_boot, self.rank, self.world)
        if pooled:
            res.block, res.block_frame = blk, (arr, hr)
        else:
            res.block = blk.copy()          # spill buffer: reused by the next step
        s.bbuf = s.bmeta = None

    def _framed_finish(self, s: "_Submitted"):
        if s.sig is not None:
            rc = self.lib.sw_sdma_wait(s.sig)
            s.sig = None
            if rc:
                raise RuntimeError(f"sw_sdma_wait failed ({rc})")
        elif s.ev is not None:
            s.ev.synchronize()
        nb = s.small["n_persisted"] * OUT_REC_SIZE
        hr = self.ROW_HEADROOM
        pin, arr, pooled = s.rows
        res = StepResult(out=arr[hr:hr + nb].view(OUT_REC), world=self.world, rank=self.rank,
                         frame_base=(arr, hr) if pooled else None, **s.small)
        s.rows = None
        if s.bmeta is not None:
            self._framed_block_finish(s, res)
        return s.token, res

    # ------------------------------------------------------------------ durable blocks
    # heap budget of a step's durable block: strings (alternate id, alert message, metadata) per row
    # on average -- each row's strings are bounded by its payload, 256 B covers realistic device
    # payloads with room; a step beyond it fails loudly in the encoder (never a truncated block)
    BLOCK_STRING_BYTES_PER_ROW = 256

    def _seg_buffers(self, slot: int):
        """(HBM block buffer, encoder state, max pages, capacity) of outbound slot ``slot``: each slot
        keeps its block until the copy engine has moved it to the host."""
        segs = self.__dict__.setdefault("_segs", {})
        s = segs.get(slot)
        if s is None:
            from ..persistence.segments import PAGE_ROWS, SEG_ALIGN, max_block_bytes
            cap = max_block_bytes(self.out_cap, self.BLOCK_STRING_BYTES_PER_ROW * self.out_cap)
            if self.cfg.block_index:               # + the index trailer (swindex.h)
                cap = -(-(cap + int(self.lib.sw_seg_index_max_bytes(self.out_cap))) // SEG_ALIGN) * SEG_ALIGN
            pages = -(-self.out_cap // PAGE_ROWS)
            s = segs[slot] = (torch.empty(cap, dtype=torch.uint8, device=self.device),
                              torch.zeros(pages + 8, dtype=torch.int64, device=self.device), pages, cap)
        return s

    SEG_AUX_SIZE = 32             # sizeof(SwSegAux), csrc/include/swseg.h

    def _aux_buffer(self, slot: int) -> torch.Tensor:
        """Encoder aux rows (SwSegAux) of outbound slot ``slot``, beside ``out_dev[slot]``."""
        bufs = self.__dict__.setdefault("_aux_dev", {})
        b = bufs.get(slot)
        if b is None:
            b = bufs[slot] = torch.zeros(self.out_cap * self.SEG_AUX_SIZE, dtype=torch.uint8, device=self.device)
        return b

    def encode_block_async(self, slot: int, snapshot: tuple | None = None) -> torch.Tensor:
        """Enqueue ``k_seg_encode`` of the step just processed on the current stream: its rows (in
        ``out_dev[slot]``), their encoder aux (written beside them by the persist kernel) and, on a
        single rank, their strings from the raw batch the step decoded (still in HBM); on several
        ranks from the string slabs the re-key exchange brought with the records (``work_str``; none
        with ``str_bytes`` = 0).  Returns the device view (block bytes, encoder errors, first store
        sequence) the host reads once the step is done.  ``snapshot`` = (scalars, reject counters,
        carry counts, mapped host snapshot) device pointers: the encoder's last workgroup also writes
        the end-of-step snapshot (``k_step_snapshot``'s job, no extra dispatch)."""
        dev, state, pages, cap = self._seg_buffers(slot)
        a = self.args
        src = a.raw if self.world == 1 else (a.work_str or 0)
        P = ctypes.c_void_p
        if snapshot is not None:
            rc = self.lib.sw_seg_encode_snap(P(_ptr(self.out_dev[slot])), P(_ptr(self._aux_buffer(slot))), P(src),
                                             P(_ptr(self.t["cursor"])), P(_ptr(dev)), cap, P(_ptr(state)), pages,
                                             *(P(x) for x in snapshot), self._stream())
            if rc:
                raise RuntimeError(f"sw_seg_encode_snap failed ({rc})")
        else:
            rc = self.lib.sw_seg_encode(P(_ptr(self.out_dev[slot])), P(_ptr(self._aux_buffer(slot))), P(src),
                                        P(_ptr(self.t["cursor"])), P(_ptr(dev)), cap, P(_ptr(state)), pages,
                                        self._stream())
            if rc:
                raise RuntimeError(f"sw_seg_encode failed ({rc})")
        if self.cfg.block_index:
            # the block's index trailer, built right behind the encoder on the same stream; its last
            # workgroup publishes the final block bytes (state, and the host snapshot when given)
            nk = self.ctx_key_spaces()
            rc = self.lib.sw_seg_index(P(_ptr(self.out_dev[slot])), P(_ptr(self._aux_buffer(slot))), P(src),
                                       P(_ptr(self.t["cursor"])), P(_ptr(self.store["alt"])), self.cfg.store_cap,
                                       P(_ptr(self.t["asg_ctx"])), self.cfg.max_assignments, P(nk.ctypes.data),
                                       P(_ptr(dev)), cap, P(_ptr(state)), pages,
                                       P(snapshot[3] if snapshot is not None else 0),
                                       P(_ptr(self._index_scratch(nk))), self.out_cap,
                                       P(_ptr(self.ix_stamps) if self.ix_stamps is not None else 0), self._stream())
            if rc:
                raise RuntimeError(f"sw_seg_index failed ({rc})")
        return state[pages + 1:pages + 4]

    ix_stamps = None                # profiling: s_memrealtime stamps of the index build (see ix_probe)

    def _index_scratch(self, nk: np.ndarray) -> torch.Tensor:
        """Scratch of the block index build (one per engine: the builds run in stream order), sized for
        the context key spaces; zeroed when (re)allocated -- the build keeps it re-armed."""
        need = int(self.lib.sw_seg_index_scratch_words(self.out_cap, int(np.maximum(nk, 0).sum())))
        t = self.__dict__.get("_ix_scratch")
        if t is None or t.numel() < need:
            if t is not None:
                self._sync_streams()            # the previous build may still read the old buffer
            t = self._ix_scratch = torch.zeros(need, dtype=torch.int32, device=self.device)
        return t

    REJECT_BYTES = 8 << 20          # compact copies of rejected payloads per step (beyond: host reads the record)

    def reject_refs_async(self, slot: int, raw_dev: torch.Tensor, off_dev: torch.Tensor, n_msgs: int):
        """Snapshot this step's routable rejects (duplicates dropped) for outbound slot ``slot``
        (``k_reject_refs``, current stream): device counters ``[refs, bytes]`` and, written straight
        into mapped pinned host memory, the refs ``(start, end, status | src_rank << 8, copy offset)``
        and the compact copies of their payloads.  ``raw_dev`` / ``off_dev`` / ``n_msgs``: the batch
        whose local events this step processed.  Returns (counters, host buffer); the refs start at
        byte 0 of the host buffer, the copies at ``16 * rec_cap``."""
        refs = self.__dict__.setdefault("_rej_refs", {})
        bufs = refs.get(slot)
        cap = self.cfg.rec_cap
        if bufs is None:
            bufs = refs[slot] = (torch.zeros(8, dtype=torch.int32, device=self.device),     # see k_reject_refs
                                 HostBuffer(self.lib, 16 * cap + self.REJECT_BYTES))
        cnt, hb = bufs
        rc = self.lib.sw_reject_refs(ctypes.byref(self.args), ctypes.c_void_p(_ptr(raw_dev)),
                                     ctypes.c_void_p(_ptr(off_dev)), int(n_msgs), ctypes.c_void_p(_ptr(cnt)),
                                     ctypes.c_void_p(hb.dev), cap, ctypes.c_void_p(hb.dev + 16 * cap),
                                     self.REJECT_BYTES, self._stream())
        if rc:
            raise RuntimeError(f"sw_reject_refs failed ({rc})")
        return bufs

    def reject_snapshot(self, slot: int, n_refs: int, n_bytes: int):
        """(refs u32 [n, 4], compact payload bytes) of slot ``slot``'s snapshot (host views, valid
        until the slot's next snapshot)."""
        cnt, hb = self._rej_refs[slot]
        cap = self.cfg.rec_cap
        n_refs = min(int(n_refs), cap)
        refs = hb.view(np.uint32, 4 * n_refs).reshape(-1, 4)
        nb = min(int(n_bytes), self.REJECT_BYTES)
        comp = hb._arr[16 * cap:16 * cap + max(1, nb)]
        return refs, comp

    def block_device(self, slot: int) -> torch.Tensor:
        return self._seg_buffers(slot)[0]

    def encode_block(self, now_ms: int, res=None, slot: int | None = None, boot: int = 0) -> np.ndarray:
        """Synchronous durable block of the last step (after :meth:`step`): encoded on the MI355X,
        copied back, sealed.  The bytes equal ``persistence.segments.encode_block`` of the step's rows."""
        from ..persistence.segments import seal
        slot = self._last_sel if slot is None else slot
        with self._lock:
            meta = self.encode_block_async(slot)
            self._sync_streams()
            nb, err, first = (int(x) for x in meta.cpu().numpy())
            if err or nb <= 0 or nb > self._seg_buffers(slot)[3]:
                raise RuntimeError(f"block encoder failed (bytes={nb}, errors={err})")
            blk = self.block_device(slot)[:nb].cpu().numpy().copy()
        seal(blk, first, now_ms, boot, self.rank, self.world)
        return blk

    def carry_count(self) -> int:
        """Re-key carry: from the pipelined runner's last snapshot, else read (a sync)."""
        if self.world == 1:
            return 0
        v = self.__dict__.get("_carry_seen")
        return v if v is not None else int(self.t["n_carry"].max().item())

    # ------------------------------------------------------------------ queries
    def stats_dict(self) -> dict:  # type: ignore[override]
        return EngineBase.stats_dict(self.t["stats"].cpu().numpy().view(np.uint64))

    @property
    def cursor(self) -> int:
        return int(self.t["cursor"][0].item())

    def intern_table(self) -> dict:
        keys = self.t["nm_key"].cpu().numpy().view(np.uint64)
        ids = self.t["nm_id"].cpu().numpy()
        sel = (keys != 0) & (ids >= 0)
        return {int(k): int(i) for k, i in zip(keys[sel], ids[sel])}

    def device_state(self, asg: int) -> dict:
        """Last-known state of one assignment.  ``k_state_lookup`` probes the merged-state map for
        the assignment's (name id, kind) keys -- 2 x names read-only probes, not a pass over the
        ``state_slots`` x 32 B table (GBs at bench sizing) -- and only the hits (and their
        name-table entries) cross PCIe."""
        from ..models.columnar import ASG_STATE
        with self._lock:
            stream = torch.cuda.current_stream(self.device)
            n_ids = int(self.t["nm_counter"].item())
            if getattr(self, "_sl_rows", None) is None or self._sl_rows.shape[0] < 2 * max(n_ids, 1):
                self._sl_rows = torch.zeros((2 * max(n_ids, 64), 4), dtype=torch.int64, device=self.device)
                self._sl_n = torch.zeros(1, dtype=torch.int32, device=self.device)
            rc = self.lib.sw_state_lookup(ctypes.c_void_p(_ptr(self.t["ms"])), self.cfg.state_slots - 1, int(asg),
                                          n_ids, ctypes.c_void_p(_ptr(self._sl_rows)), ctypes.c_void_p(_ptr(self._sl_n)),
                                          ctypes.c_void_p(stream.cuda_stream))
            if rc:
                raise RuntimeError(f"sw_state_lookup failed ({rc})")
            rows = self._sl_rows[:int(self._sl_n.item())].cpu().numpy().view(np.uint64)
            st = self.t["st"].view(-1, 4)[asg].cpu().numpy().view(ASG_STATE)[0]
            nids = np.unique(((rows[:, 0] - np.uint64(1)) & np.uint64(0xFFFFFFFF)) >> np.uint64(1)).astype(np.int64)
            inv = {}
            if len(nids):
                sel = torch.nonzero(torch.isin(self.t["nm_id"].long(), torch.from_numpy(nids).to(self.device))).flatten()
                ks = self.t["nm_key"][sel].cpu().numpy().view(np.uint64)
                ids = self.t["nm_id"][sel].cpu().numpy()
                inv = {int(i): int(k) for k, i in zip(ks, ids) if k != 0}
        mx, al = {}, {}
        for key, date, eid1, _ in rows:
            k = int(key) - 1
            nid, kind = (k & 0xFFFFFFFF) >> 1, k & 1
            h = inv.get(nid)
            name = self.names.get(h, str(h))
            (al if kind else mx)[name] = (int(eid1) - 1, int(date))
        le = int(st["loc_eid1"])
        return {
            "assignment": asg,
            "last_interaction": int(st["last"]),
            "presence_missing": int(st["missing"]),
            "last_location": (le - 1, int(st["loc_date"])) if le else None,
            "measurements": mx,
            "alerts": al,
        }

    def query_store(self, event_type, asg_idx, start=None, end=None, page_number=1, page_size=100):
        """Hot-store query on the MI355X: one k_store_filter pass over the HBM ring (assignment set
        as a bitmap), then the match set is ordered on the device and only the page comes back.
        Holds the engine lock: the cursor read, the filter into the shared match buffer and the
        gather are one unit against concurrent queries and steps."""
        with self._lock:
            return self._query_store(event_type, asg_idx, start, end, page_number, page_size)

    def _query_store(self, event_type, asg_idx, start, end, page_number, page_size):
        cur = self.cursor
        n = min(cur, self.cfg.store_cap)
        nbits = self.cfg.max_assignments
        words = np.zeros((nbits + 31) // 32, np.uint32)
        a = np.asarray(list(asg_idx), np.int64)
        a = a[(a >= 0) & (a < nbits)]
        np.bitwise_or.at(words, a >> 5, (np.uint32(1) << (a & 31).astype(np.uint32)))
        bits = torch.from_numpy(words.view(np.int32)).to(self.device)
        if getattr(self, "_q_rows", None) is None or self._q_rows.numel() < max(n, 1):
            self._q_rows = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
            self._q_n = torch.zeros(1, dtype=torch.int32, device=self.device)
        i64 = np.iinfo(np.int64)
        st = self.store
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        rc = self.lib.sw_store_filter(ctypes.c_void_p(_ptr(st["etype"])), ctypes.c_void_p(_ptr(st["asg"])),
                                      ctypes.c_void_p(_ptr(st["date"])), n, int(event_type),
                                      ctypes.c_void_p(_ptr(bits)), nbits, i64.min if start is None else int(start),
                                      i64.max if end is None else int(end), ctypes.c_void_p(_ptr(self._q_rows)),
                                      self._q_rows.numel(), ctypes.c_void_p(_ptr(self._q_n)), stream)
        if rc:
            raise RuntimeError(f"sw_store_filter failed ({rc})")
        total = int(self._q_n.item())
        rows = self._q_rows[:total].long()
        seq = self._row_seq(rows, cur)
        # newest first, ties by latest id: stable sort by seq desc, then stable by date desc
        o1 = torch.sort(seq, descending=True, stable=True).indices
        dates = st["date"][rows[o1]]
        o2 = torch.sort(dates, descending=True, stable=True).indices
        lo, hi = self._window(page_number, page_size, total)
        sel = o1[o2[lo:hi]]
        page = rows[sel]
        cols = {k: v[page].cpu().numpy() for k, v in st.items()}
        for k in ("name", "alt", "aux"):
            cols[k] = cols[k].view(np.uint64)
        return total, cols, seq[sel].cpu().numpy() * self.world + self.rank

    def store_rows(self):
        cur = self.cursor
        cap = self.cfg.store_cap
        n = min(cur, cap)
        idx = torch.arange(n, device=self.device)
        if cur > cap:
            idx = (idx + cur % cap) % cap
        cols = {k: v[idx].cpu().numpy() for k, v in self.store.items()}
        for k in ("name", "alt", "aux"):
            cols[k] = cols[k].view(np.uint64)
        return cols, (np.arange(cur - n, cur) * self.world + self.rank)

    # ------------------------------------------------------------------ checkpoint / resume
    kind = "gpu"
    _CKPT_TABLES = ("reg", "asg_ctx", "asg_active", "dd_tab", "dd_meta", "seq_base", "nm_key", "nm_id", "nm_first",
                    "nm_counter", "seen_key", "st", "ms", "stats", "cursor")

    # store-backed filter primitives (EngineBase.filter_seed / filter_state); host-driven, between steps
    def _ff_meta_get(self) -> np.ndarray:
        self._sync_streams()
        return self.t["dd_ff_meta"].cpu().numpy().copy()

    def _ff_meta_set(self, m):
        self._sync_streams()
        self.t["dd_ff_meta"].copy_(torch.from_numpy(np.ascontiguousarray(np.asarray(m, np.int64))))
        torch.cuda.current_stream(self.device).synchronize()

    def _ff_add(self, hashes, g: int):
        h = np.ascontiguousarray(np.asarray(hashes, np.uint64))
        if not self._ff_on or not len(h):
            return
        c = self.cfg
        dev = torch.from_numpy(h.view(np.int64)).to(self.device)
        torch.cuda.current_stream(self.device).synchronize()
        rc = self.lib.sw_ff_add(ctypes.c_void_p(_ptr(self.t["dd_ff"])), c.ff_buckets - 1, c.dedup_filter_gens, int(g),
                                ctypes.c_void_p(_ptr(self.t["dd_ff_meta"])), ctypes.c_void_p(_ptr(dev)), len(h),
                                self._stream())
        if rc:
            raise RuntimeError(f"sw_ff_add failed ({rc})")
        self._sync_streams()

    def _ff_clear(self, g: int):
        c = self.cfg
        rc = self.lib.sw_ff_clear(ctypes.c_void_p(_ptr(self.t["dd_ff"])), c.ff_buckets - 1, c.dedup_filter_gens,
                                  int(g), self._stream())
        if rc:
            raise RuntimeError(f"sw_ff_clear failed ({rc})")
        self._sync_streams()

    def _ckpt_tables(self):
        return self._CKPT_TABLES + (("dd_ff_meta",) if self._ff_on else ())

    def _ff_export(self) -> dict:
        """The filter's non-empty 64-byte buckets (the sparse form every engine checkpoints)."""
        v = self.t["dd_ff"].view(-1, 16)
        idx = torch.nonzero(v.ne(0).any(dim=1)).flatten()
        return {"dd_ff_idx": idx.cpu().numpy().astype(np.int64), "dd_ff_rows": v[idx].cpu().numpy().view(np.uint32)}

    def _ff_import(self, idx, rows):
        v = self.t["dd_ff"].view(-1, 16)
        v.zero_()
        if len(idx):
            i = torch.from_numpy(np.ascontiguousarray(idx, np.int64)).to(self.device)
            v[i] = torch.from_numpy(np.ascontiguousarray(rows, np.uint32).reshape(-1, 16).view(np.int32)).to(self.device)

    def checkpoint_state(self, include_store: bool = False) -> dict:
        if self._pend is not None:
            raise RuntimeError("checkpoint with a pipelined exchange in flight: drain the round first")
        self._sync_streams()
        st = {k: self.t[k].cpu().numpy() for k in self._ckpt_tables()}
        if self._ff_on:
            st.update(self._ff_export())
        if self.world > 1:
            cp = self._carry_par
            n = int(self.t["n_carry"][cp].item())
            st["carry"] = self.carry_bufs[cp][:n * EVENT_REC.itemsize].cpu().numpy()
            if self.cfg.str_cap:
                nb = int(self.t["n_carry_str"][cp].item())
                st["carry_spans"] = self.carry_spans[cp][:n * STR_REF.itemsize].cpu().numpy()
                st["carry_str"] = self.carry_strs[cp][:nb].cpu().numpy()
        if include_store:
            st.update({f"store.{k}": v.cpu().numpy() for k, v in self.store.items()})
        return st

    def restore_state(self, a: dict, include_store: bool):
        self._sync_streams()
        for k in self._ckpt_tables():
            if k == "dd_tab" and k not in a and "dd_key" in a:
                # an older checkpoint's split key / sequence tables: {key, win = sequence's low 32
                # bits, lmin = none}
                self.t["dd_tab"][:, 0].copy_(torch.from_numpy(a["dd_key"]))
                sq = np.asarray(a["dd_seq"], np.int64)
                self.t["dd_tab"][:, 1].copy_(torch.from_numpy((sq & 0xFFFFFFFF) | np.int64(-1 << 32)))
                continue
            if k not in a:
                continue
            src = torch.from_numpy(a[k])
            if k == "stats" and src.numel() != self.t[k].numel():     # a checkpoint with fewer counters
                self.t[k].zero_()
                self.t[k][:src.numel()].copy_(src)
                continue
            self.t[k].copy_(src)       # in place: captured graphs keep their pointers
        if self._ff_on and "dd_ff_idx" in a:
            self._ff_import(a["dd_ff_idx"], a["dd_ff_rows"])
        if "dd_tab" not in a and "dd_meta" in a:
            # older checkpoints decided the rotation at the start of a step; now the end of the
            # previous step does (k_step_end): apply that decision to the restored window
            m0 = a["dd_meta"].astype(np.int64).copy()
            m = self._armed_dedup_meta(m0.copy(), self.cfg)
            if m[0] != m0[0]:                  # flipped here: the new live table starts empty
                slots = self.cfg.dedup_slots
                self.t["dd_tab"][int(m[0]) * slots:(int(m[0]) + 1) * slots, 0] = 0
                self.t["dd_tab"][int(m[0]) * slots:(int(m[0]) + 1) * slots, 1] = -1
            self.t["dd_meta"].copy_(torch.from_numpy(m))
        if self.world > 1 and "carry" in a:
            cp = self._carry_par
            c = torch.from_numpy(a["carry"])
            self.carry_bufs[cp][:c.numel()].copy_(c)
            self.t["n_carry"].zero_()
            self.t["n_carry"][cp] = c.numel() // EVENT_REC.itemsize
            if self.cfg.str_cap:
                # the carry's strings (an older checkpoint has none: its records go without them)
                sp = torch.from_numpy(a.get("carry_spans", np.zeros(c.numel() // EVENT_REC.itemsize, STR_REF)
                                            .view(np.uint8)))
                hp = torch.from_numpy(a.get("carry_str", np.zeros(0, np.uint8)))
                self.carry_spans[cp][:sp.numel()].copy_(sp)
                self.carry_strs[cp][:hp.numel()].copy_(hp)
                self.t["n_carry_str"].zero_()
                self.t["n_carry_str"][cp] = hp.numel()
        if include_store:
            for k, v in self.store.items():
                v.copy_(torch.from_numpy(a[f"store.{k}"]))
        self._sync_streams()

    @staticmethod
    def _armed_dedup_meta(m: np.ndarray, cfg) -> np.ndarray:
        """dd_meta = [generation, ids in the live table, rotation state, ids that met a claimed key]
        as k_step_end leaves it: a rotation the next step needs (the live table could pass half
        load) already flipped (state 2: k_lookup counts it) -- what the first step after an
        allocation, a reset or an old checkpoint needs.  The caller clears the new live table when
        it is not empty."""
        m[3] = 0
        if m[1] + cfg.rec_cap > cfg.dedup_slots // 2:
            m[0], m[1], m[2] = m[0] ^ 1, 0, 2
        else:
            m[2] = 0
        return m

    def reset_dedup(self):
        self.dedup_valid_from = self.cursor           # the window holds no id of the rows before
        self.t["dd_tab"][:, 0] = 0
        self.t["dd_tab"][:, 1] = -1
        self.t["dd_meta"].copy_(torch.from_numpy(self._armed_dedup_meta(np.zeros(4, np.int64), self.cfg)))


class PipelinedRunner:
    """Multi-buffered pipeline: H2D(k+1) || compute(k) || outbound D2H(k-1).

    * copy stream: SDMA H2D of the raw payload batch and its offsets (``nbuf`` device buffers, so the
      H2D of later batches runs ahead of compute -- the step is then bound by max(H2D, compute))
    * compute stream: the fused step; enriched rows land in an HBM staging ring
    * outbound, by ``mode``:
      - ``"hsa"`` (default): once step k's row count is known (the host syncs on step k while k+1
        runs) an explicit copy-engine transfer (``hsa_amd_memory_async_copy``) moves exactly those
        rows to pinned host memory -- no CUs used (measured on MI355X: the HIP runtime serves
        ``hipMemcpyAsync`` D2H with a blit *kernel* that occupies CUs for the whole PCIe transfer
        and slows the pipeline's kernels); delivered one step later
      - ``"sdma"``: same schedule through ``hipMemcpyAsync`` on a third stream
      - ``"push"``: ``k_push_out`` stores rows into mapped host memory from a side stream
      - ``"direct"``: the persist kernel stores rows straight into mapped host memory
    * world > 1: each submit is one :meth:`GpuInboundEngine.round_async` (decode batch k, process
      batch k-1, all-to-all of batch k on a communication stream overlapped with that process
      phase); rows of a round belong to the previous batch and :meth:`flush` runs the last round.
      ``SW_PIPELINE_EXCHANGE=0`` falls back to the serial decode -> exchange -> process step.
    """

    def __init__(self, engine: GpuInboundEngine, max_raw_bytes: int, deliver_outbound: bool = True,
                 on_outbound=None, mode: str | None = None, push_blocks: int = 128, nbuf: int = 3,
                 out_target=None, block_sink=None, on_rejects=None):
        """``out_target(n_bytes) -> (host address, token)`` (copy-engine modes): where each step's rows
        land, e.g. a pinned buffer a bus topic then publishes in place; ``on_outbound(token, n_rows)``
        is called once they are there.  Without it rows land in the engine's outbound ring and
        ``on_outbound(rows)`` gets a view of them.

        ``block_sink`` (``persistence.segments.DurableBlockSink``): every step's persisted events are
        also encoded on the GPU into a durable block (``k_seg_encode``, right after the step on the
        compute stream); the copy engine moves the compressed block to the sink's pinned buffer and
        the sink seals it, queues it to the durable store and publishes it.  ``submit(tag=...)``
        labels a batch; ``block_sink.committable()`` returns the labels whose blocks are durable."""
        import os
        self.e = engine
        self.out_target = out_target
        dev = engine.device
        self.mode = mode or os.environ.get("SW_OUTBOUND_MODE", "hsa")
        if out_target is not None and self.mode not in ("hsa", "sdma"):
            raise ValueError("out_target needs a copy-engine outbound mode (hsa or sdma)")
        self.h2d = torch.cuda.Stream(dev)
        self.comp = torch.cuda.current_stream(dev)
        self.push = torch.cuda.Stream(dev)
        self.push_blocks = int(os.environ.get("SW_PUSH_BLOCKS", push_blocks))
        self.sdma_engine = int(os.environ.get("SW_SDMA_ENGINE", 0))
        nb = self.nbuf = max(2, min(int(os.environ.get("SW_PIPELINE_BUFFERS", nbuf)), engine.n_out_bufs))
        self.raw = [torch.empty(max_raw_bytes + _ALIGN, dtype=torch.uint8, device=dev) for _ in range(nb)]
        self.off = [torch.empty(engine.cfg.max_msgs + 1, dtype=torch.int32, device=dev) for _ in range(nb)]
        self.lens = [torch.empty(5 * engine.cfg.max_msgs + 64, dtype=torch.uint8, device=dev) for _ in range(nb)]
        self.nout = [torch.zeros(4, dtype=torch.int32, device=dev) for _ in range(nb)]
        self.ev_h2d = [torch.cuda.Event() for _ in range(nb)]
        self.ev_comp = [torch.cuda.Event() for _ in range(nb)]
        self.ev_push = [torch.cuda.Event() for _ in range(nb)]
        self.deliver = deliver_outbound
        self.on_outbound = on_outbound
        self.k = 0
        self.delivered = 0
        # steps enqueued but not yet drained.  Draining step k-depth (not k-1) when submitting k
        # leaves the host a whole extra step of slack: the H2D of the next batch is enqueued while
        # the copy stream is still busy, so the PCIe-bound copy stream never idles on host jitter.
        # The multi-GPU exchange keeps depth 1 (its stall decisions read the carry of the last round).
        from collections import deque
        self.pending = deque()
        self.copying = None          # sdma mode: (buffer, n_out) whose D2H copy is in flight
        self.rounds = engine.world > 1 and os.environ.get("SW_PIPELINE_EXCHANGE", "1") != "0"
        self.produced = [False] * nb  # rounds mode: did the round in slot b process a batch
        self.depth = 1 if self.rounds else max(1, min(int(os.environ.get("SW_PIPELINE_DEPTH", 2)), nb - 1))
        self.block_sink = block_sink
        if block_sink is not None:
            if self.mode != "hsa":
                raise ValueError("durable blocks need the copy-engine outbound mode (hsa)")
            self.btag = [None] * nb       # caller tag of the batch whose block slot b holds
            self.bnow = [0] * nb
            self._prev_tag = None
        self.bcopying = None              # (slot, signal, buffer, bytes, first_seq, now, tag)
        # SW_RUNNER_TRACE=1: host wall-clock per phase (bench attribution)
        self.trace = {} if os.environ.get("SW_RUNNER_TRACE") == "1" else None
        if self.trace is not None:      # device-side H2D and step time per slot (CUDA events)
            self.tev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(nb)]
            self.tev_on = [False] * nb
        # on_rejects(tag, refs u32 [n, 4], compact payload bytes): the slow path of each step
        # (see reject_refs_async; refs whose copy offset is ~0 need the raw record named by tag)
        self.on_rejects = on_rejects
        self.rtag = [None] * nb
        # per-slot end-of-step snapshot in mapped host memory (k_step_snapshot): scalars, encoder
        # meta, reject counters -- read after the step's event, no copy calls
        self.snap = [HostBuffer(engine.lib, 256) for _ in range(nb)]
        self.cpar = [0] * nb              # live carry parity when slot b's snapshot was taken
        # the slow path runs off the submit thread: the GPU writes the snapshot into mapped host
        # memory, routing runs on one worker thread in batch order; rejects_floor() tells callers the
        # oldest batch whose rejects are not routed yet (its input offset must not be committed)
        if on_rejects is not None:
            from collections import deque
            from concurrent.futures import ThreadPoolExecutor
            self.rej_pool = ThreadPoolExecutor(1, thread_name_prefix="reject-router")
            self.rej_job = [None] * nb
            self.rej_inflight = deque()           # (tag, future)
        self._prev_batch = None           # rounds mode: (slot, n_msgs, tag) of the batch in flight
        self.rejects_seen = 0

    def submit(self, raw_host: torch.Tensor | None, off_host: torch.Tensor | None, n_msgs: int,
               now_ms: int | None = None, presence: bool = False, lens_host: torch.Tensor | None = None,
               raw_bytes: int | None = None, tag=None):
        """Enqueue one batch (``raw_host=None``: a drain round of the pipelined exchange, no new batch).

        The batch is framed either by u32 offsets (``off_host``) or by a varint length stream
        (``lens_host``, see ``pipeline/framing.py``; ``raw_bytes`` = payload bytes without padding),
        which crosses PCIe in ~1 B per payload and is turned into offsets on the GPU."""
        k = self.k
        b = k % self.nbuf
        t_sub = time.perf_counter()
        now_ms = int(time.time() * 1000) if now_ms is None else now_ms
        if raw_host is not None:
            nbytes = int(raw_host.numel())
            with torch.cuda.stream(self.h2d):
                if k >= self.nbuf:
                    self.h2d.wait_event(self.ev_comp[b])  # compute k-nbuf was the last reader of buffer b
                if self.trace is not None:
                    self.tev[b][0].record(self.h2d)
                self.raw[b][:nbytes].copy_(raw_host, non_blocking=True)
                if lens_host is not None:
                    self.lens[b][:lens_host.numel()].copy_(lens_host, non_blocking=True)
                else:
                    self.off[b][:n_msgs + 1].copy_(off_host[:n_msgs + 1], non_blocking=True)
                self.ev_h2d[b].record(self.h2d)
                if self.trace is not None:
                    self.tev[b][1].record(self.h2d)
        t_sub = self._t("sub_h2d", t_sub)
        if self.mode == "hsa" and ((self.copying is not None and self.copying[0] == b) or
                                   (self.bcopying is not None and self.bcopying[0] == b)):
            self._finish_copy()                           # SDMA copy k-2 still reads staging ring b
        t_sub = self._t("sub_copy_wait", t_sub)
        if raw_host is not None:
            self.comp.wait_event(self.ev_h2d[b])
            if lens_host is not None:
                self.e.frame_varint(self.lens[b], lens_host.numel(), n_msgs, self.off[b],
                                    nbytes if raw_bytes is None else raw_bytes)
        if k >= self.nbuf and self.mode in ("push", "sdma"):
            self.comp.wait_event(self.ev_push[b])         # push k-2 was the last reader of staging ring b
        to_dev = self.mode in ("push", "sdma", "hsa")
        if self.rounds:
            src = (self.raw[b], self.off[b]) if raw_host is not None else (None, None)
            self.produced[b] = self.e.round_async(src[0], src[1], n_msgs, now_ms, presence=presence, out_sel=b,
                                                  out_to_device=to_dev)
        else:
            self.e.step_async(self.raw[b], self.off[b], n_msgs, now_ms, presence=presence, out_sel=b,
                              out_to_device=to_dev)
            self.produced[b] = True
        t_sub = self._t("sub_step", t_sub)
        if self.mode == "push":
            if not self.produced[b]:
                self.nout[b].zero_()
            else:
                self.nout[b].copy_(self.e.t["scalars"][7:11])    # n_out on the device (stream-ordered)
        rej_cnt = seg_meta = None
        if self.on_rejects is not None:
            self.rtag[b] = None
            # in rounds mode the round processes the batch submitted by the previous call
            cur = (b, n_msgs, tag) if raw_host is not None else None
            done = self._prev_batch if self.rounds else cur
            if self.rounds:
                self._prev_batch = cur
            if self.produced[b] and done is not None:
                if self.rej_job[b] is not None:
                    self.rej_job[b].result()           # the router is done with slot b's host buffer
                t_sub = self._t("sub_router_wait", t_sub)
                rej_cnt, _ = self.e.reject_refs_async(b, self.raw[done[0]], self.off[done[0]], done[1])
                self.rtag[b] = done[2]
        nc = self.e.t.get("n_carry")
        self.cpar[b] = getattr(self.e, "_carry_par", 0)
        snapped = False
        if self.block_sink is not None:
            done_tag = self._prev_tag if self.rounds else tag
            self._prev_tag = tag
            if self.produced[b]:
                # the encoder's last workgroup writes the step snapshot too (one dispatch fewer)
                seg_meta = self.e.encode_block_async(b, snapshot=(
                    self.e.t["scalars"].data_ptr(), 0 if rej_cnt is None else rej_cnt.data_ptr(),
                    0 if nc is None else nc.data_ptr(), self.snap[b].dev))
                snapped = True
                self.btag[b], self.bnow[b] = done_tag, self.e._step_now
        if not snapped:
            rc = self.e.lib.sw_step_snapshot(ctypes.c_void_p(self.e.t["scalars"].data_ptr()),
                                             ctypes.c_void_p(0 if seg_meta is None else seg_meta.data_ptr()),
                                             ctypes.c_void_p(0 if rej_cnt is None else rej_cnt.data_ptr()),
                                             ctypes.c_void_p(0 if nc is None else nc.data_ptr()),
                                             int(self.produced[b]), ctypes.c_void_p(self.snap[b].dev),
                                             ctypes.c_void_p(self.comp.cuda_stream))
            if rc:
                raise RuntimeError(f"sw_step_snapshot failed ({rc})")
        self.ev_comp[b].record(self.comp)
        if self.trace is not None:
            self.tev[b][2].record(self.comp)
            self.tev_on[b] = raw_host is not None
        if self.mode == "push" and self.deliver:
            with torch.cuda.stream(self.push):
                self.push.wait_event(self.ev_comp[b])
                rc = self.e.lib.sw_push_out(ctypes.c_void_p(_ptr(self.e.out_dev[b])),
                                            ctypes.c_void_p(self.e.out_host[b].dev),
                                            ctypes.c_void_p(_ptr(self.nout[b])), self.e.out_cap, self.push_blocks,
                                            ctypes.c_void_p(self.push.cuda_stream))
                if rc:
                    raise RuntimeError(f"sw_push_out failed ({rc})")
                self.ev_push[b].record(self.push)
        self._t("enqueue", t_sub)
        self.pending.append(b)
        while len(self.pending) > self.depth:
            self._drain()
        self.k += 1

    def _rejects_async(self, pb: int, n_rej: int, n_bytes: int):
        """Route slot pb's reject snapshot (already in mapped host memory) on the worker thread, in
        batch order; the slot is not overwritten before the job is done (see submit)."""
        if n_rej > self.e.cfg.rec_cap:
            raise RuntimeError(f"reject snapshot overflow ({n_rej} refs > rec_cap)")
        refs, comp = self.e.reject_snapshot(pb, n_rej, n_bytes)
        tag = self.rtag[pb]
        self.rejects_seen += n_rej
        fut = self.rej_job[pb] = self.rej_pool.submit(self.on_rejects, tag, refs, comp)
        self.rej_inflight.append((tag, fut))

    def rejects_floor(self):
        """Tag of the oldest batch whose rejects are still being routed (None when all are done);
        routing failures surface here."""
        q = getattr(self, "rej_inflight", None)
        while q and q[0][1].done():
            q.popleft()[1].result()
        return q[0][0] if q else None

    def _deliver(self, b: int, n_out: int, token=None):
        if self.deliver and self.on_outbound is not None and n_out:
            if self.out_target is not None:
                self.on_outbound(token, n_out)
            else:
                self.on_outbound(self.e.out_host[b].view(OUT_REC, n_out))
        self.delivered += n_out

    def _dest(self, b: int, n_out: int):
        """(host address, token) the rows of staging slot ``b`` are copied to."""
        if self.out_target is None:
            return self.e.out_host[b].host, None
        return self.out_target(n_out * OUT_REC.itemsize)

    def _finish_copy(self):
        self._finish_block()
        self._finish_rows()

    def _finish_block(self):
        if self.bcopying is not None:
            _, sig, buf, nb, first, now, tag = self.bcopying
            self.bcopying = None
            t0 = time.perf_counter()
            rc = self.e.lib.sw_sdma_wait(sig)
            if rc:
                raise RuntimeError(f"sw_sdma_wait failed ({rc})")
            t0 = self._t("block_copy_wait", t0)
            self.block_sink.publish(buf, nb, first, now, tag)
            self._t("block_publish", t0)

    def _finish_rows(self):
        if self.copying is not None:
            cb, cn, sig, tok = self.copying
            if sig is not None:
                rc = self.e.lib.sw_sdma_wait(sig)
                if rc:
                    raise RuntimeError(f"sw_sdma_wait failed ({rc})")
            else:
                self.ev_push[cb].synchronize()
            self._deliver(cb, cn, tok)
            self.copying = None

    def _t(self, name, t0):
        if self.trace is not None:
            t1 = time.perf_counter()
            self.trace[name] = self.trace.get(name, 0.0) + (t1 - t0)
            return t1
        return t0

    def _drain(self):
        if not self.pending:
            return
        pb = self.pending.popleft()
        t0 = time.perf_counter()
        self.ev_comp[pb].synchronize()
        t0 = self._t("wait_step", t0)
        if self.trace is not None and self.tev_on[pb]:
            ev = self.tev[pb]
            ev[2].synchronize()                 # recorded just after ev_comp: may complete a moment later
            self.trace["gpu_h2d"] = self.trace.get("gpu_h2d", 0.0) + ev[0].elapsed_time(ev[1]) / 1000
            self.trace["gpu_h2d_to_step_end"] = self.trace.get("gpu_h2d_to_step_end", 0.0) + \
                ev[1].elapsed_time(ev[2]) / 1000
        if self.mode == "push" and self.deliver:
            self.ev_push[pb].synchronize()
        snap = self.snap[pb].view(np.uint32, 32)
        n_out = int(snap[7]) if self.produced[pb] else 0
        if self.e.world > 1:
            # re-key carry after this round: the parity its partition spilled into
            self.e._carry_seen = int(snap[22 + self.cpar[pb]])
        if self.on_rejects is not None and self.produced[pb] and self.rtag[pb] is not None:
            n_rej = int(snap[24])
            if n_rej:
                self._rejects_async(pb, n_rej, int(snap[25]))
                t0 = self._t("rejects_enqueue", t0)
        if self.mode not in ("sdma", "hsa"):
            self._deliver(pb, n_out)
            return
        self._finish_copy()
        t0 = self._t("finish_copy", t0)
        if self.block_sink is not None and self.produced[pb]:
            nb, err, first = (int(x) for x in self.snap[pb].view(np.uint64, 11)[8:11])
            if err or nb <= 0 or nb > self.e._seg_buffers(pb)[3]:
                raise RuntimeError(f"durable block encoder failed (bytes={nb}, errors={err})")
            dst, buf = self.block_sink.target(nb)
            h = ctypes.c_uint64()
            rc = self.e.lib.sw_sdma_copy(ctypes.c_void_p(dst), ctypes.c_void_p(_ptr(self.e.block_device(pb))), nb,
                                         self.sdma_engine, ctypes.byref(h))
            if rc:
                raise RuntimeError(f"sw_sdma_copy of the durable block failed ({rc})")
            self.bcopying = (pb, h.value, buf, nb, first, self.bnow[pb], self.btag[pb])
            t0 = self._t("block_copy_start", t0)
        dst, tok = self._dest(pb, n_out) if self.deliver and n_out else (None, None)
        if self.mode == "hsa":
            sig = None
            if self.deliver and n_out:
                h = ctypes.c_uint64()
                rc = self.e.lib.sw_sdma_copy(ctypes.c_void_p(dst),
                                             ctypes.c_void_p(_ptr(self.e.out_dev[pb])), n_out * OUT_REC.itemsize,
                                             self.sdma_engine, ctypes.byref(h))
                if rc == 0:
                    sig = h.value
                else:
                    # copy engine unavailable on this node: degrade to the HIP runtime path (loudly)
                    import warnings
                    warnings.warn(f"sw_sdma_copy failed ({rc}); falling back to hipMemcpyAsync outbound")
                    self.mode = "sdma"
            if self.mode == "hsa":
                self.copying = (pb, n_out, sig, tok)
                if sig is None:
                    self._finish_rows()
                return
        if self.deliver and n_out:
            rc = self.e.lib.sw_copy_d2h(ctypes.c_void_p(dst),
                                        ctypes.c_void_p(_ptr(self.e.out_dev[pb])), n_out * OUT_REC.itemsize,
                                        ctypes.c_void_p(self.push.cuda_stream))
            if rc:
                raise RuntimeError(f"sw_copy_d2h failed ({rc})")
        self.ev_push[pb].record(self.push)
        self.copying = (pb, n_out, None, tok)

    def flush(self):
        if self.rounds and self.e.exchange_pending:
            self.submit(None, None, 0)                    # last round: process the batch in flight
        while self.pending:
            self._drain()
        self._finish_copy()
        self.comp.synchronize()
        self.push.synchronize()
        for _, fut in list(getattr(self, "rej_inflight", ())):
            fut.result()                                  # every reject routed
        self.rejects_floor()

    def outbound(self, b: int) -> np.ndarray:
        n = int(self.snap[b].view(np.uint32, 32)[7]) if self.produced[b] else 0
        return self.e.out_host[b].view(OUT_REC, n)
