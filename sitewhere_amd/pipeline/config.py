"""Sizing of the inbound pipeline engine (HBM/host tables and batch capacities)."""
from __future__ import annotations

from dataclasses import dataclass, field

from ..utils import pow2_at_least


@dataclass
class EngineConfig:
    """Capacities of one engine shard (one tenant engine on one GPU / rank).

    Defaults are sized for MI355X (288 GB HBM3E): the event store alone holds
    2^27 events (~12 GB) so a shard keeps hours of hot events resident.
    """

    max_msgs: int = 1 << 20          # payloads per micro-batch
    rec_cap: int = 0                 # decoded events per micro-batch (0 = 2 * max_msgs)
    gen_cap: int = 1 << 16           # rule alerts + presence events per step
    max_devices: int = 1 << 20
    max_assignments: int = 1 << 20
    store_cap: int = 1 << 27         # HBM event-store ring capacity (events)
    dedup_slots: int = 1 << 22       # alternate-id window (slots; window = slots / 2)
    # store-backed dedup beyond the window: generational fingerprint tables of the persisted
    # alternate ids (csrc/include/swtypes.h SW_FF_*).  Each of ``dedup_filter_gens`` generations
    # takes ``dedup_filter_ids`` persisted ids (0 = off); the filter always holds the newest
    # (gens - 1) * ids ids -- the durable store's retention by rows is set from it
    # (``filter_retention_rows``).  HBM: gens * 2 * (ids + rec_cap) * 4 bytes (~8 B per id and
    # generation at load <= 1/2); false positives ~1e-8 of new ids.
    dedup_filter_ids: int = 0
    dedup_filter_gens: int = 4
    name_slots: int = 1 << 16        # distinct measurement names / alert types
    state_slots: int = 0             # (assignment, name) state map slots (0 = 16 * max_assignments)
    names_cap: int = 4096            # new-name reports per step
    shuffle_slack: float = 1.1       # per-destination slab = slack * rec_cap / world (+1024)
    shuffle_pad: int = 1024          # records added to every slab (small-batch headroom)
    carry_cap: int = 0               # records full slabs can defer to the next exchange (0 = 3 * rec_cap)
    carry_high: int = 0              # drivers stall new input while the carry exceeds this (0 = rec_cap)
    # world > 1: string bytes (alternate id + metadata + alert message) exchanged per record slot of
    # a re-key slab; the owner rank stores them losslessly (0 = strings stay on the decoding rank)
    str_bytes: int = 40
    # persist each step's events stable-sorted by assignment (the durable block is then clustered by
    # assignment: its page zone maps are the assignment index, csrc/include/swindex.h); every engine
    # (MI355X, native C++, Python oracle) uses the same order
    cluster: bool = True
    # durable blocks carry their index trailer (alternate ids, page zone maps, context-key heads),
    # built in the step that encodes them
    block_index: bool = True
    presence_missing_ms: int = 8 * 3600 * 1000   # DevicePresenceManager default (8h)
    presence_check_ms: int = 10 * 60 * 1000      # DevicePresenceManager default (10 min)
    rank: int = 0
    world: int = 1
    extra: dict = field(default_factory=dict)

    def __post_init__(self):
        if self.rec_cap <= 0:
            self.rec_cap = 2 * self.max_msgs
        if self.state_slots <= 0:
            self.state_slots = 16 * self.max_assignments
        self.reg_slots = pow2_at_least(2 * self.max_devices)
        # a generation must take a whole batch at <= 50% load (rotation happens before a step that
        # would pass that): smaller tables overflow on every step and probe to their limit
        self.dedup_slots = pow2_at_least(max(self.dedup_slots, 2 * self.rec_cap))
        self.name_slots = pow2_at_least(self.name_slots)
        self.state_slots = pow2_at_least(self.state_slots)
        # key bits of the clustering sort (assignment indices < max_assignments)
        self.cl_bits = max(1, (self.max_assignments - 1).bit_length()) if self.cluster else 0
        self.shuf_cap = int(self.shuffle_slack * self.rec_cap / max(1, self.world)) + self.shuffle_pad
        local = self.rec_cap
        # per-destination string slab, 16-byte multiple (the unpack gathers it 16 B at a time)
        self.str_cap = (self.shuf_cap * self.str_bytes + 15) // 16 * 16 if self.world > 1 and self.str_bytes > 0 else 0
        if self.world > 1:
            # a rank can receive a full slab from every rank: the work batch after the exchange
            # must hold world * shuf_cap records (skewed keys), or the surplus would be cut
            self.rec_cap = max(self.rec_cap, self.world * self.shuf_cap)
        # Lossless re-keying: spilled records carry over (up to carry_cap) and drivers feed an empty
        # round instead of a new batch while the carry is above carry_high (should_stall), so with
        # two rounds in flight the carry stays below carry_high + 2 * local <= carry_cap
        if self.carry_high <= 0:
            self.carry_high = local
        if self.carry_cap <= 0:
            self.carry_cap = self.carry_high + 2 * local
        # the carry keeps its records' strings: a heap of carry_cap records at twice the slab's
        # per-record budget (spilled records beyond it are dropped and counted, like those beyond
        # carry_cap); u32 offsets
        self.carry_str_cap = min((self.carry_cap * max(2 * self.str_bytes, 64) + 15) // 16 * 16, 0xFFFFFFF0) \
            if self.world > 1 and self.str_bytes > 0 else 0
        if self.dedup_filter_ids > 0:
            if not 2 <= self.dedup_filter_gens <= 8:
                raise ValueError("dedup_filter_gens must be 2..8")
            # the window's retired generation is probed only for ids the filter holds (k_dedup_claim):
            # the filter's newest (gens - 1) generations must hold at least the window's ids
            self.dedup_filter_ids = max(self.dedup_filter_ids, self.dedup_slots)
            # load <= 1/2 even for the step that crosses the generation's ids (it still adds to it)
            self.ff_buckets = pow2_at_least(max(64, (2 * (self.dedup_filter_ids + self.rec_cap) + 15) // 16))
        else:
            self.dedup_filter_ids = 0
            self.ff_buckets = 0

    # a durable store bounded to N rows holds at most 1.25 N (the file being written, at most N / 4
    # rows, is never deleted: DurableEventStore.limit_retention_rows)
    STORE_ROWS_OVERSHOOT = 1.25

    def filter_retention_rows(self, slack_rows: int = 0) -> int:
        """The row limit of the durable store under which the filter holds every retained id (0: no
        filter, no bound).  The filter holds at least the newest (gens - 1) * dedup_filter_ids ids; a
        store that keeps at most that many rows (newest first) keeps no id older than them.  The
        store can overshoot its limit by the file being written; ``slack_rows``: rows of the blocks
        in flight (written between two retention checks)."""
        if not self.dedup_filter_ids:
            return 0
        held = (self.dedup_filter_gens - 1) * self.dedup_filter_ids - int(slack_rows)
        return max(self.rec_cap, int(held / self.STORE_ROWS_OVERSHOOT))

    def filter_bytes(self) -> int:
        return self.ff_buckets * self.dedup_filter_gens * 64 if self.dedup_filter_ids else 0

    @classmethod
    def small(cls, **kw):
        """Test-sized configuration (fits easily on CPU)."""
        base = dict(max_msgs=4096, gen_cap=4096, max_devices=4096, max_assignments=4096, store_cap=1 << 16,
                    dedup_slots=1 << 14, name_slots=1 << 10, names_cap=1024)
        base.update(kw)
        return cls(**base)
