// Argument block for the GPU inbound-pipeline engine (csrc/hip/swgpu.hip).
//
// Every field is 8 bytes (pointer or int64) so the ctypes mirror in
// sitewhere_amd/ops/engine_abi.py has no padding ambiguity.  The Python side
// allocates every buffer as a torch tensor (so the caching allocator owns HBM)
// and passes raw pointers; the library never allocates.
#pragma once
#include <stdint.h>
#include "swtypes.h"

typedef struct SwNameRef {
  uint64_t hash;
  uint32_t off;
  uint16_t len;
  uint8_t src_rank;
  uint8_t pad;
} SwNameRef;

// Registry slot (32 B, one cache-line quarter): exact 128-bit token fingerprint -> device and
// its *active* assignment (-1 when unassigned or released), so validation is one probe.
typedef struct __attribute__((aligned(16))) SwRegSlot {
  uint64_t lo;
  uint64_t hi;
  int32_t dev;
  int32_t asg;
  uint64_t pad;
} SwRegSlot;

// Assignment context gathered by enrichment (one 16-B load).
typedef struct __attribute__((aligned(16))) SwAsgCtx {
  int32_t device;
  int32_t customer;
  int32_t area;
  int32_t asset;
} SwAsgCtx;

// Device state per assignment (reference IDeviceState), 32 B.
typedef struct __attribute__((aligned(16))) SwAsgState {
  uint64_t last;       // last interaction (ms)
  uint64_t missing;    // presence missing date (0 = present)
  uint64_t loc_date;   // date of the latest location
  uint64_t loc_eid1;   // event id + 1 of that location (0 = none)
} SwAsgState;

// (assignment, name, kind) -> latest measurement / alert, 32 B.
typedef struct __attribute__((aligned(16))) SwMsSlot {
  uint64_t key;        // (asg << 32 | name_id << 1 | kind) + 1, 0 = empty
  uint64_t date;
  uint64_t eid1;
  uint64_t pad;
} SwMsSlot;

// Per-step values read by the process-phase kernels from device memory (written in-stream by
// sw_set_step_params before each step), so the process phase can be captured once as a hipGraph and
// replayed: graph nodes keep their by-value SwEngineArgs, these change every step.
typedef struct SwStepParams {
  int64_t now_ms;
  int64_t batch_seq;
  int64_t presence_missing_ms;  // <= 0: no presence scan this step
  SwOutRec* out;                // outbound rows of this step
  void* aux;                    // SwSegAux per row of this step (durable-block encoder input; null: none)
  int64_t raw_bytes;            // bound of the batch's strings (0: rows carry no strings, e.g. world > 1)
} SwStepParams;

typedef struct SwEngineArgs {
  // ---------------------------------------------------------------- batch input
  const uint8_t* raw;          // raw wire bytes of the batch (device)
  const uint32_t* msg_off;     // n_msgs + 1 offsets into raw (device)
  int64_t n_msgs;
  int64_t now_ms;              // receive time of the batch
  int64_t rank;
  int64_t world;
  int64_t batch_seq;           // step counter of this rank (raw-log addressing)
  // ---------------------------------------------------------------- decode
  uint32_t* msg_cnt;           // [msg_cap]
  uint32_t* msg_evoff;         // [msg_cap] decode: scanned per-workgroup record sums
  uint32_t* scan_tmp;          // [scan_tmp_len] block sums
  int64_t scan_tmp_len;
  SwEventRec* recs;            // [rec_cap] decoded records (pre-shuffle)
  int64_t rec_cap;
  uint32_t* n_recs;            // device scalar
  // new-name capture on the source rank (strings live in this rank's raw batch)
  uint64_t* seen_key;
  int64_t seen_mask;
  SwNameRef* new_names;        // [names_cap]
  uint32_t* n_new_names;
  int64_t names_cap;
  // ---------------------------------------------------------------- shuffle (world > 1)
  SwWireRec* send;             // [world * shuf_cap] packed exchange records
  SwWireRec* recv;             // [world * shuf_cap]
  int64_t shuf_cap;
  uint32_t* send_cnt;          // [world]
  uint32_t* recv_cnt;          // [world]
  uint32_t* part_tmp;          // [world * n_tiles]
  int64_t part_tmp_len;
  uint32_t* overflow;          // device scalar: records dropped by the bounded shuffle
  // ---------------------------------------------------------------- validated batch
  SwEventRec* work;            // records after shuffle (== recs when world == 1)
  uint32_t* n_work;            // device scalar
  uint8_t* status;             // [rec_cap]
  int32_t* ev_dev;             // [rec_cap]
  int32_t* ev_asg;             // [rec_cap]
  uint32_t* ok_idx;            // [rec_cap]
  uint32_t* n_ok;
  uint32_t* rej_idx;           // [rec_cap]
  uint32_t* n_rej;
  uint32_t* cmp_tmp;           // [scan_tmp_len]
  // ---------------------------------------------------------------- registry (host-built, read-only here)
  const SwRegSlot* reg;
  int64_t reg_mask;
  const SwAsgCtx* asg_ctx;
  const uint8_t* asg_active;
  int64_t n_asg;
  // ---------------------------------------------------------------- dedup window
  uint64_t* dd_key;            // packed 16-byte slots {key, first sequence}, two generations of dd_mask + 1
  int64_t* dd_seq;             // unused by the MI355X engine (host engines keep split tables)
  int64_t dd_mask;
  int64_t* seq_base;           // device scalar: events seen so far on this rank
  // ---------------------------------------------------------------- names intern (state-map keys)
  uint64_t* nm_key;
  int32_t* nm_id;
  int32_t* nm_first;
  int64_t nm_mask;
  int32_t* nm_counter;
  // ---------------------------------------------------------------- device state (per assignment)
  SwAsgState* st;
  SwMsSlot* ms;
  int64_t ms_mask;
  // ---------------------------------------------------------------- event store (HBM ring, SoA)
  int64_t store_cap;
  int64_t* store_cursor;       // device scalar: events persisted so far on this rank
  int64_t* step_cursor0;       // device scalar: cursor at step start
  uint8_t* s_etype;
  uint8_t* s_level;
  int64_t* s_date;
  int64_t* s_recv;
  int32_t* s_dev;
  int32_t* s_asg;
  int32_t* s_cust;
  int32_t* s_area;
  int32_t* s_asset;
  uint64_t* s_name;
  double* s_v0;
  double* s_v1;
  double* s_v2;
  uint64_t* s_alt;
  uint64_t* s_aux;             // src_rank << 48 | len << 32 | batch-relative offset
  int32_t* s_batch;            // batch_seq of the source rank when decoded
  // ---------------------------------------------------------------- outbound (D2H to connectors)
  SwOutRec* out;               // [rec_cap + gen_cap]
  uint32_t* n_out;
  // ---------------------------------------------------------------- rules (zone tests)
  const double* zone_vtx;      // [2 * n_vertices] (lat, lon) pairs
  const int32_t* zone_off;     // [n_zones + 1]
  const double* zone_bbox;     // [4 * n_zones] min_lat, min_lon, max_lat, max_lon
  int64_t n_zones;
  const SwZoneTest* tests;
  int64_t n_tests;
  const uint64_t* test_name_hash; // alert type hash per test
  uint64_t* zmask;             // [rec_cap] fired-test bitmask per persisted row
  uint32_t* ztile;             // [2 * ntiles] tile counts + scanned offsets
  // generated events (rule alerts, presence state changes)
  SwEventRec* gen;
  int32_t* gen_dev;
  int32_t* gen_asg;
  uint32_t* n_gen;
  int64_t gen_cap;
  // ---------------------------------------------------------------- presence
  int64_t presence_missing_ms; // <= 0 disables the scan this step
  uint64_t presence_name_hash; // hash of "presence"
  // ---------------------------------------------------------------- stats
  uint64_t* stats;             // [SW_N_STATS] cumulative counters (see SW_STAT_*)
  // ---------------------------------------------------------------- per-step params (device)
  SwStepParams* sp;
  // ---------------------------------------------------------------- shuffle spill (world > 1)
  // Records that did not fit their destination slab are not dropped: they are written (in
  // deterministic destination/position order) to `spill` and sent first by the next partition,
  // which reads them back as `carry`.  Only records beyond carry_cap are dropped (counted).
  const SwEventRec* carry;
  const uint32_t* n_carry;
  SwEventRec* spill;
  uint32_t* n_spill;
  int64_t carry_cap;
  // ---------------------------------------------------------------- rules, host-side sizes
  int64_t n_zone_vtx;          // zone_off[n_zones]: sizes k_zone_mask's dynamic LDS vertex table
  // ---------------------------------------------------------------- state merge scratch
  int64_t* ev_slot;            // [2 * max(rec_cap, gen_cap)] state pass-2 items: (ms slot | -2 - asg | -1, date)
  // ---------------------------------------------------------------- dedup generations
  int64_t* dd_meta;            // [generation, ids in the current table, rotate flag, pad]; dd_key / dd_seq
                               // hold two tables of dd_mask + 1 slots (current = dd_meta[0])
  // ---------------------------------------------------------------- string refs
  SwStrRef* spans;             // [rec_cap] per decoded record (decode writes, the block encoder reads)
  // ---------------------------------------------------------------- store-backed dedup filter
  // generational fingerprint tables (swtypes.h, SW_FF_*): [buckets][gens][SW_FF_SLOTS] u32
  uint32_t* dd_ff;             // null: off
  int64_t dd_ff_bmask;         // buckets per generation - 1
  int64_t dd_ff_gens;
  int64_t* dd_ff_meta;         // [SW_FF_META + gens]
  // ---------------------------------------------------------------- string exchange (world > 1)
  // A record's strings (alternate id, metadata, alert message) live in the raw batch of the rank
  // that decoded it.  The partition copies them into per-destination byte slabs beside the record
  // slabs (string refs rewritten to slab offsets), the all-to-all moves them with the records, and
  // the unpack gathers them into work_str ([world][str_cap], the encoder's string source) with the
  // refs rebased (+ source rank * str_cap).  Null send_str: strings stay on the decoding rank.
  uint8_t* send_str;           // [world][str_cap] (this partition's parity)
  uint32_t* send_str_cnt;      // [world] bytes used per destination (k_part_cut)
  SwStrRef* send_spans;        // [world][shuf_cap] string refs beside the send slabs
  const uint8_t* recv_str;     // [world][str_cap]
  const uint32_t* recv_str_cnt;
  const SwStrRef* recv_spans;  // [world][shuf_cap]
  uint8_t* work_str;           // [world][str_cap] gathered by k_unpack
  SwStrRef* work_spans;        // [rec_cap] refs of the work batch (rebased into work_str)
  int64_t str_cap;             // bytes per destination slab
  uint32_t* str_drops;         // [2] records sent without strings (larger than a slab) / unused
  // ---------------------------------------------------------------- re-key owner (world > 1)
  uint8_t* part_owner;         // [carry_cap + rec_cap] destination of each partition input (k_part_count)
  // ---------------------------------------------------------------- persist clustering
  // Each step's validated events persist stable-sorted by assignment index (the block's clustered
  // order: an assignment's rows of a step share one or two pages, see swindex.h).  Radix-sort
  // buffers: keys / values [2][rec_cap] ping-pong, histograms [sw_radix_tmp_words(rec_cap)].
  uint32_t* cl_keys;
  uint32_t* cl_vals;
  uint32_t* cl_hist;
  int64_t cl_bits;             // assignment index bits (0: persist in arrival order)
  // ---------------------------------------------------------------- lossless re-key (world > 1)
  // Per destination the slab takes the longest prefix of its records (input order) that fits both
  // shuf_cap records and str_cap string bytes (k_part_cut); the rest spill into the next carry WITH
  // their strings, copied into the spill heap (which the next partition reads back as carry_str).
  uint32_t* part_len;          // [carry_cap + rec_cap] exchange bytes per input (bit 31: sent without strings)
  uint64_t* part_bytes;        // [2][world][ntiles] string bytes per tile and destination, then their prefix
  uint64_t* part_meta;         // [256] per destination: cut, cut bytes, total bytes; kept spill counters
  const SwStrRef* carry_spans; // [carry_cap] refs of the carry's records into carry_str
  const uint8_t* carry_str;    // the carry's string heap
  SwStrRef* spill_spans;       // [carry_cap] refs of the spilled records into spill_str
  uint8_t* spill_str;          // [carry_str_cap]
  uint32_t* n_spill_str;       // bytes of spill_str in use (k_part_counts)
  int64_t carry_str_cap;
} SwEngineArgs;

#define SW_N_STATS 24

enum {
  SW_STAT_MSGS = 0,
  SW_STAT_EVENTS = 1,
  SW_STAT_PERSISTED = 2,
  SW_STAT_UNREGISTERED = 3,
  SW_STAT_UNASSIGNED = 4,
  SW_STAT_DUPLICATE = 5,
  SW_STAT_DECODE_ERROR = 6,
  SW_STAT_CONTROL = 7,
  SW_STAT_RULE_ALERTS = 8,
  SW_STAT_PRESENCE = 9,
  SW_STAT_SHUFFLE_OVERFLOW = 10,
  SW_STAT_NEW_NAMES = 11,
  SW_STAT_STATE_OVERFLOW = 12,
  SW_STAT_SHUFFLE_DEFERRED = 13,   // records spilled to the next step's exchange
  SW_STAT_DEDUP_OVERFLOW = 14,     // alternate ids the window could not place (probe bound hit)
  SW_STAT_DEDUP_ROTATIONS = 15,    // dedup generations retired
  SW_STAT_DEDUP_RECHECKS = 16,     // ids handed to the host: new to the window, maybe in the store
  SW_STAT_N = 16,
};
