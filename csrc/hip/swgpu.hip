// SiteWhere-AMD GPU data plane: the inbound event pipeline as CDNA4 kernels.
//
// One step processes a micro-batch of raw device payloads end to end:
//   decode (protobuf wire protocol) -> [multi-GPU: owner partition + RCCL all-to-all]
//   -> registry lookup / assignment validation -> alternate-id dedup
//   -> persist into the HBM event store with enrichment -> device-state merge
//   -> zone-test rules (point-in-polygon) -> presence scan -> outbound records.
//
// Reference behaviour (per stage):
//   decode      service-event-sources/.../decoder/protobuf/ProtobufDeviceEventDecoder.java:79-281
//   dedup       service-event-sources/.../deduplicator/AlternateIdDeduplicator.java
//   validate    service-inbound-processing/.../InboundPayloadProcessingLogic.java:119-218
//   persist     service-event-management/.../KafkaEventPersistenceTriggers.java:72-97
//   enrich      service-inbound-processing/.../OutboundPayloadEnrichmentLogic.java:54-92
//   state       service-device-state/.../DeviceStateProcessingLogic.java:116-200
//   rules       service-rule-processing/.../ZoneTestRuleProcessor.java:47-62
//   presence    service-device-state/.../DevicePresenceManager.java:110-200
//
// Conventions: 256-thread blocks (4 wave64), grid-stride loops capped at
// 2048 blocks (8 per CU on 256 CUs), counts that are only known on the device
// are read from device scalars so the host never synchronises inside a step
// (the whole step is hipGraph-capturable).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdint.h>
#include "swtypes.h"
#include "swdecode.h"
#include "swengine.h"
#include "swseg.h"

#define BLK 256
#define WAVES (BLK / 64)
#define TILE_ITEMS 4
#define TILE (BLK * TILE_ITEMS)
#define MAX_GRID 2048
#define STAGE_BYTES (32 * 1024)
#define MAX_PROBE 4096  // open-addressing probe bound (tables are sized for load <= 0.5)

typedef unsigned long long ull;

// Workgroup id as the kernels see it.  The dispatcher deals workgroups round-robin over the 8 XCDs
// (each with its own L2); with SW_XCD_REMAP the ids are permuted (bijectively, any grid size) so the
// workgroups that share an XCD own one contiguous range of tiles / grid-stride slots.  Every kernel
// uses BID for all its block-id arithmetic, so either numbering is correct; it is a speed choice,
// measured in profiles/r1_xcd.
#ifndef SW_XCD_REMAP
#define SW_XCD_REMAP 0
#endif
__device__ __forceinline__ uint32_t sw_block_id() {
#if SW_XCD_REMAP
  const uint32_t nwg = gridDim.x, orig = blockIdx.x, x = orig % 8u, q = nwg / 8u, r = nwg % 8u;
  return (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + orig / 8u;
#else
  return blockIdx.x;
#endif
}
#define BID sw_block_id()

static inline int grid_for(int64_t n) {
  int64_t g = (n + BLK - 1) / BLK;
  if (g < 1) g = 1;
  if (g > MAX_GRID) g = MAX_GRID;
  return (int)g;
}

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ ull lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// Block-wide exclusive scan of one value per thread; returns the prefix and the block total.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* total, uint32_t* lds) {
  const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t t = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += t;
  }
  if (lane == 63) lds[wid] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int w = 0; w < WAVES; ++w) { uint32_t t = lds[w]; lds[w] = acc; acc += t; }
    lds[WAVES] = acc;
  }
  __syncthreads();
  uint32_t res = inc - v + lds[wid];
  *total = lds[WAVES];
  __syncthreads();
  return res;
}

// Sum of v[0 .. k), returned to every thread of the block: the prologue reduce of the per-tile sums
// the PREVIOUS kernel wrote, in place of a separate single-workgroup scan dispatch between the two
// (a few thousand L2-resident u32s: ~1-2 us of loads per block against ~5-8 us per extra dispatch,
// and no flags, fences or counters -- the kernel boundary is the only synchronisation).
__device__ __forceinline__ uint32_t block_sum_prefix(const uint32_t* v, int64_t k, uint32_t* lds) {
  uint32_t s = 0;
  for (int64_t i = threadIdx.x; i < k; i += BLK) s += v[i];
  uint32_t tot;
  block_excl_scan(s, &tot, lds);
  return tot;
}

// ============================================================================ scan
// Exclusive scan of u32[n] -> out, total -> *total.  n <= TILE * (BLK * 64).
__global__ void k_scan_tiles(const uint32_t* __restrict__ in, int64_t n, uint32_t* __restrict__ tsum) {
  __shared__ uint32_t lds[WAVES + 1];
  const int64_t base = (int64_t)BID * TILE;
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < TILE_ITEMS; ++k) {
    int64_t i = base + (int64_t)k * BLK + threadIdx.x;
    if (i < n) s += in[i];
  }
  uint32_t tot;
  block_excl_scan(s, &tot, lds);
  if (threadIdx.x == 0) tsum[BID] = tot;
}

__global__ void k_scan_apply(const uint32_t* __restrict__ in, int64_t n, const uint32_t* __restrict__ tsum,
                             uint32_t* __restrict__ out) {
  __shared__ uint32_t lds[WAVES + 1];
  const int64_t base = (int64_t)BID * TILE;
  uint32_t run = tsum[BID];
#pragma unroll
  for (int k = 0; k < TILE_ITEMS; ++k) {
    int64_t i = base + (int64_t)k * BLK + threadIdx.x;
    uint32_t v = i < n ? in[i] : 0;
    uint32_t tot;
    uint32_t pre = block_excl_scan(v, &tot, lds);
    if (i < n) out[i] = run + pre;
    run += tot;
  }
}

// Single-pass exclusive scan (decoupled look-back): one dispatch instead of tiles + sums + apply.
// Workgroups take tiles in ticket order, publish their tile aggregate, then walk back over their
// predecessors' 64-bit state words (flag in the top bits) until an inclusive prefix.  The
// workgroup that finishes last zeroes the state (ticket, done counter, tile words), so the next
// launch -- including a hipGraph replay with the same arguments -- starts clean: no memset node.
// state = u64[2 + nt]: [0] ticket, [1] done, [2..] tile words.
#define SLB_AGG (1ull << 62)
#define SLB_INC (2ull << 62)
#define SLB_VAL ((1ull << 62) - 1)
#define SLB_SPIN_LIMIT (1u << 26)

__device__ __forceinline__ ull slb_load(const ull* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void slb_store(ull* p, ull v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_scan_lb(const uint32_t* __restrict__ in, int64_t n, uint32_t* __restrict__ out,
                          uint32_t* __restrict__ total, ull* __restrict__ state, int64_t nt) {
  __shared__ uint32_t lds[WAVES + 1];
  __shared__ uint32_t s_tile;
  __shared__ ull s_excl;
  if (threadIdx.x == 0) s_tile = (uint32_t)atomicAdd(&state[0], 1ull);
  __syncthreads();
  const int64_t tile = s_tile;
  const int64_t base = tile * TILE + (int64_t)threadIdx.x * TILE_ITEMS;
  uint32_t v[TILE_ITEMS];
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < TILE_ITEMS; ++k) {
    const int64_t i = base + k;
    v[k] = i < n ? in[i] : 0u;
    sum += v[k];
  }
  uint32_t agg;
  const uint32_t pre = block_excl_scan(sum, &agg, lds);
  if (threadIdx.x == 0) {
    ull excl = 0;
    ull* tw = state + 2;
    if (tile == 0) {
      slb_store(&tw[0], SLB_INC | agg);
    } else {
      slb_store(&tw[tile], SLB_AGG | agg);
      for (int64_t p = tile - 1; p >= 0;) {
        ull w = slb_load(&tw[p]);
        uint32_t spins = 0;
        while ((w >> 62) == 0 && ++spins < SLB_SPIN_LIMIT) {
          __builtin_amdgcn_s_sleep(1);
          w = slb_load(&tw[p]);
        }
        excl += w & SLB_VAL;
        if ((w >> 62) == 2) break;
        --p;
      }
      slb_store(&tw[tile], SLB_INC | (excl + agg));
    }
    s_excl = excl;
    if (tile == nt - 1 && total) *total = (uint32_t)(excl + agg);
  }
  __syncthreads();
  uint32_t run = (uint32_t)s_excl + pre;
#pragma unroll
  for (int k = 0; k < TILE_ITEMS; ++k) {
    const int64_t i = base + k;
    if (i < n) out[i] = run;
    run += v[k];
  }
  __syncthreads();
  // the last workgroup to finish resets the state for the next launch (nobody reads it any more)
  if (threadIdx.x == 0) s_tile = (uint32_t)(atomicAdd(&state[1], 1ull) == (ull)(nt - 1));
  __syncthreads();
  if (s_tile) {
    for (int64_t i = threadIdx.x; i < nt + 2; i += BLK) state[i] = 0;
  }
}

// One-workgroup exclusive scan for short arrays (tile counters: a few thousand entries): each thread
// scans a contiguous run.  Cheaper than any multi-workgroup scheme at this size -- the look-back
// below pays cross-XCD flag latency even for 2 tiles (10-15 us measured against ~5 us here).
__global__ void k_scan_block(const uint32_t* __restrict__ in, int64_t n, uint32_t* __restrict__ out,
                             uint32_t* __restrict__ total) {
  __shared__ uint32_t lds[WAVES + 1];
  const int64_t per = (n + BLK - 1) / BLK;
  const int64_t b = (int64_t)threadIdx.x * per;
  uint32_t s = 0;
  for (int64_t i = 0; i < per; ++i) if (b + i < n) s += in[b + i];
  uint32_t tot;
  uint32_t pre = block_excl_scan(s, &tot, lds);
  for (int64_t i = 0; i < per; ++i) {
    if (b + i < n) { const uint32_t t = in[b + i]; out[b + i] = pre; pre += t; }
  }
  if (threadIdx.x == 0 && total) *total = tot;
}
#define SCAN_BLOCK_MAX (BLK * 64)

static int launch_scan(const uint32_t* in, int64_t n, uint32_t* out, uint32_t* total, uint32_t* tmp,
                       int64_t tmp_len, hipStream_t s) {
  if (n <= SCAN_BLOCK_MAX) {
    k_scan_block<<<1, BLK, 0, s>>>(in, n, out, total);
    return 0;
  }
  int64_t nt = (n + TILE - 1) / TILE;
  if (nt < 1) nt = 1;
  if (2 * (nt + 2) > tmp_len || ((uintptr_t)tmp & 7)) return -2;     // tmp holds u64[2 + nt]
  k_scan_lb<<<(unsigned)nt, BLK, 0, s>>>(in, n, out, total, reinterpret_cast<ull*>(tmp), nt);
  return 0;
}

// ============================================================================ framing
// The raw batch travels as payload bytes + a LEB128 varint length per payload (1 byte for payloads
// under 128 B) instead of u32 offsets: 3+ fewer PCIe bytes per message on an H2D-bound pipeline
// (Kafka record batches frame records the same way).  Offsets are rebuilt here with a two-component
// (message index, byte offset) scan over the length stream.
__device__ __forceinline__ bool vlen_end(const uint8_t* __restrict__ L, int64_t i) { return (L[i] & 0x80u) == 0; }

// Value of the varint whose last (most significant) byte is L[i].
__device__ __forceinline__ uint32_t vlen_value(const uint8_t* __restrict__ L, int64_t i) {
  uint32_t v = L[i] & 0x7fu;
  for (int k = 0; k < 4 && i - 1 - k >= 0 && (L[i - 1 - k] & 0x80u); ++k) v = (v << 7) | (L[i - 1 - k] & 0x7fu);
  return v;
}

__global__ void k_vlen_tiles(const uint8_t* __restrict__ L, int64_t nbytes, uint32_t* __restrict__ tcnt,
                             uint32_t* __restrict__ tlen) {
  __shared__ uint32_t lds[WAVES + 1];
  const int64_t base = (int64_t)BID * TILE;
  uint32_t c = 0, v = 0;
#pragma unroll
  for (int k = 0; k < TILE_ITEMS; ++k) {
    const int64_t i = base + (int64_t)k * BLK + threadIdx.x;
    if (i < nbytes && vlen_end(L, i)) { ++c; v += vlen_value(L, i); }
  }
  uint32_t tc, tv;
  block_excl_scan(c, &tc, lds);
  block_excl_scan(v, &tv, lds);
  if (threadIdx.x == 0) { tcnt[BID] = tc; tlen[BID] = tv; }
}

// Offsets from the tile sums of k_vlen_tiles, reduced in this kernel's prologue (no scan dispatch);
// the last tile also writes the terminal offset msg_off[n_msgs] = the byte total, clamped to the batch.
__global__ void k_vlen_apply(const uint8_t* __restrict__ L, int64_t nbytes, const uint32_t* __restrict__ tcnt,
                             const uint32_t* __restrict__ tlen, uint32_t* __restrict__ msg_off, int64_t n_msgs,
                             uint32_t raw_bytes) {
  __shared__ uint32_t lds[WAVES + 1];
  const int64_t base = (int64_t)BID * TILE;
  uint32_t run_c = block_sum_prefix(tcnt, BID, lds), run_v = block_sum_prefix(tlen, BID, lds);
  if (BID == gridDim.x - 1 && threadIdx.x == 0) {
    const uint32_t tl = run_v + tlen[BID];
    msg_off[n_msgs] = tl < raw_bytes ? tl : raw_bytes;
  }
#pragma unroll
  for (int k = 0; k < TILE_ITEMS; ++k) {
    const int64_t i = base + (int64_t)k * BLK + threadIdx.x;
    const bool e = i < nbytes && vlen_end(L, i);
    const uint32_t v = e ? vlen_value(L, i) : 0u;
    uint32_t tc, tv;
    const uint32_t pc = block_excl_scan(e ? 1u : 0u, &tc, lds);
    const uint32_t pv = block_excl_scan(v, &tv, lds);
    if (e && run_c + pc < n_msgs) {
      const uint32_t off = run_v + pv;
      msg_off[run_c + pc] = off < raw_bytes ? off : raw_bytes;   // never past the batch
    }
    run_c += tc;
    run_v += tv;
  }
}

// ============================================================================ decode
// Stage the block's 256 consecutive payloads into LDS with 16-B loads, then parse each
// payload from LDS (one lane per payload).  The parse is instantiated separately for the
// LDS and the global source so the compiler emits ds_read (not flat) loads on the fast path.
// Oversized windows (mean payload > 128 B) parse straight from global memory.
__device__ __forceinline__ bool stage_window(const uint8_t* __restrict__ raw, const uint32_t* __restrict__ off,
                                             int64_t n_msgs, uint8_t* lds, uint32_t* base_abs) {
  const int64_t m0 = (int64_t)BID * BLK;
  int64_t m1 = m0 + BLK;
  if (m1 > n_msgs) m1 = n_msgs;
  const uint32_t s = off[m0], e = off[m1];
  const uint32_t a0 = s & ~15u;
  const uint32_t span = e - a0;
  if (span > STAGE_BYTES) return false;
  const uint32_t nvec = (span + 15) >> 4;
  const uint4* src = reinterpret_cast<const uint4*>(raw + a0);
  uint4* dst = reinterpret_cast<uint4*>(lds);
  for (uint32_t v = threadIdx.x; v < nvec; v += BLK) dst[v] = src[v];
  __syncthreads();
  *base_abs = a0;
  return true;
}

// k_decode_count's per-message count carries the count pass's decode verdict in its top bit
// (a payload never expands to 2^31 records)
#define CNT_ERR 0x80000000u
#define CNT_OVR 0x40000000u   // oversize event (SW_DEC_OVERSIZE): one host-routed record

__global__ __launch_bounds__(BLK) void k_decode_count(const uint8_t* __restrict__ raw, const uint32_t* __restrict__ off,
                                                      int64_t n_msgs, uint32_t* __restrict__ cnt,
                                                      uint32_t* __restrict__ tsum, SwEngineArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[STAGE_BYTES];
  if (BID == 0 && threadIdx.x == 0) {     // the decode phase's resets (k_decode_emit counts names after)
    *a.n_new_names = 0;
    *a.overflow = 0;
    ((ull*)a.stats)[SW_STAT_MSGS] += (ull)a.n_msgs;
  }
  uint32_t base = 0;
  const bool staged = stage_window(raw, off, n_msgs, lds, &base);
  __shared__ uint32_t red[WAVES + 1];
  const int64_t m = (int64_t)BID * BLK + threadIdx.x;
  uint32_t c = 0;
  if (m < n_msgs) {
    uint32_t verdict = SW_DEC_UNKNOWN;
    c = staged ? sw_decode_payload(lds, off[m] - base, off[m + 1] - base, base, 0, 0, nullptr, 0, &verdict)
               : sw_decode_payload(raw, off[m], off[m + 1], 0, 0, 0, nullptr, 0, &verdict);
    cnt[m] = c | (verdict == SW_DEC_ERROR ? CNT_ERR : 0u) | (verdict == SW_DEC_OVERSIZE ? CNT_OVR : 0u);  // reused by emit
  }
  // per-block record total: k_decode_emit reduces the block sums before it in its prologue and
  // rebuilds the in-block prefix itself -- reduce-then-scan with no look-back chain across the 4K
  // blocks of a 1M batch (the single-pass scan serialised on cross-XCD flag polls, ~350 us per
  // step: profiles/r3_fold) and no scan dispatch between the two
  uint32_t tot;
  block_excl_scan(c, &tot, red);
  if (threadIdx.x == 0) tsum[BID] = tot;
}

// First sighting of a name/type hash on this rank: report (hash, offset, len) so the host can read
// the string from its raw batch (strings never travel with the fixed-width records).
__device__ __forceinline__ void note_name(const SwEventRec& r, ull* __restrict__ key, int64_t mask,
                                          SwNameRef* __restrict__ list, uint32_t* __restrict__ n_list, int64_t cap) {
  if (r.name_hash == 0 || r.etype >= 16) return;
  const ull h = r.name_hash;
  int64_t slot = (int64_t)(h & (ull)mask);
  for (int64_t p = 0; p <= mask && p < MAX_PROBE; ++p) {
    ull old = key[slot];
    if (old == h) return;
    if (old == 0) {
      old = atomicCAS(&key[slot], 0ull, h);
      if (old == 0) {
        const uint32_t k = atomicAdd(n_list, 1u);
        if (k < cap) {
          SwNameRef ref;
          ref.hash = h; ref.off = r.aux_off; ref.len = r.aux_len; ref.src_rank = r.src_rank; ref.pad = r.etype;
          list[k] = ref;
        } else {
          atomicExch(&key[slot], 0ull);  // list full: forget, retry in a later batch
        }
        return;
      }
      if (old == h) return;
    }
    slot = (slot + 1) & mask;
  }
}

__global__ __launch_bounds__(BLK) void k_decode_emit(SwEngineArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[STAGE_BYTES];
  uint32_t base = 0;
  const bool staged = stage_window(a.raw, a.msg_off, a.n_msgs, lds, &base);
  __shared__ uint32_t red[WAVES + 1];
  const int64_t m = (int64_t)BID * BLK + threadIdx.x;
  uint32_t tot;
  const uint32_t cv = m < a.n_msgs ? a.msg_cnt[m] : 0u;
  const uint32_t pre = block_excl_scan(cv & ~(CNT_ERR | CNT_OVR), &tot, red);
  const uint32_t blk_off = block_sum_prefix(a.msg_evoff, BID, red);   // msg_evoff: the block sums
  if (BID == 0) {                           // the batch's record count (clamped by the consumers)
    const uint32_t all = block_sum_prefix(a.msg_evoff, gridDim.x, red);
    if (threadIdx.x == 0) *a.n_recs = all;
  }
  if (m >= a.n_msgs) return;
  uint32_t verdict = (cv & CNT_ERR) ? SW_DEC_ERROR : (cv & CNT_OVR) ? SW_DEC_OVERSIZE : SW_DEC_VALID;
  const int64_t o = (int64_t)blk_off + pre;
  if (o >= a.rec_cap) return;
  const uint32_t room = (uint32_t)((a.rec_cap - o) < 0xffffffffll ? (a.rec_cap - o) : 0xffffffffll);
  SwEventRec* out = a.recs + o;
  uint32_t n;
  SwStrRef* sp = a.spans ? a.spans + o : nullptr;
  if (staged)
    n = sw_decode_payload(lds, a.msg_off[m] - base, a.msg_off[m + 1] - base, base, a.now_ms, (uint8_t)a.rank, out, room,
                          &verdict, sp);
  else
    n = sw_decode_payload(a.raw, a.msg_off[m], a.msg_off[m + 1], 0, a.now_ms, (uint8_t)a.rank, out, room, &verdict, sp);
  // fused new-name capture (one probe of a small L2-resident table per named record)
  for (uint32_t k = 0; k < n && k < room; ++k)
    note_name(out[k], (ull*)a.seen_key, a.seen_mask, a.new_names, a.n_new_names, a.names_cap);
}

// End of the decode phase: clamp the record count, account the names first seen in this batch.
__global__ void k_decode_end(SwEngineArgs a) {
  if (threadIdx.x == 0 && BID == 0) {
    if (*a.n_recs > a.rec_cap) *a.n_recs = (uint32_t)a.rec_cap;
    ((ull*)a.stats)[SW_STAT_NEW_NAMES] += *a.n_new_names;
  }
}

// ============================================================================ shuffle (owner partition)
// Stable multi-way partition of records by owner rank into [world][shuf_cap] slabs.
// Destination of a record in the re-key.  The registry is replicated on every rank (the
// reference's near cache does the same for its consumers), so the rank that decoded a record knows
// whether its device is registered and assigned: such records go to the device's owner; every other
// record (unknown or unassigned device, control, decode error) stays on the decoding rank, whose raw
// batch holds the payload bytes the slow path routes (unregistered-device events, registrations).
__device__ __forceinline__ uint32_t part_dest(const SwEngineArgs& a, const SwEventRec& r, uint32_t world,
                                              uint32_t rank) {
  if (r.etype >= 16) return rank;
  int64_t slot = (int64_t)(r.fp_lo & (ull)a.reg_mask);
  for (int64_t p = 0; p <= a.reg_mask && p < MAX_PROBE; ++p) {
    const ulonglong2 k = *reinterpret_cast<const ulonglong2*>(&a.reg[slot].lo);
    if (k.x == r.fp_lo && k.y == r.fp_hi) return a.reg[slot].asg >= 0 ? sw_owner(r.fp_hi, world) : rank;
    if (k.x == 0 && k.y == 0) break;
    slot = (slot + 1) & a.reg_mask;
  }
  return rank;
}

// Partition input = this step's carry (records deferred by the previous partition, sent first)
// followed by the freshly decoded records.
__device__ __forceinline__ const SwEventRec& part_in(const SwEventRec* __restrict__ carry, uint32_t nc,
                                                     const SwEventRec* __restrict__ recs, int64_t i) {
  return i < (int64_t)nc ? carry[i] : recs[i - nc];
}

// Exchange bytes of partition input i: alternate id + metadata + alert message (control records
// keep their raw-batch offsets and send none).  Carried records' refs point into the carry heap.
__device__ __forceinline__ uint32_t part_str_len(const SwEngineArgs& a, const SwEventRec& r, uint32_t nc, int64_t i) {
  if (r.etype >= 16) return 0u;
  const SwStrRef s = i < (int64_t)nc ? a.carry_spans[i] : a.spans[i - nc];
  const uint32_t al = (s.has & SW_SR_ALT) ? s.alt_len : 0u;
  const uint32_t ml = (s.has & SW_SR_META) ? s.meta_len : 0u;
  const uint32_t gl = r.etype == SW_EV_ALERT ? r.aux2_len : 0u;
  return al + ml + gl;
}

#define PART_STRIP 0x80000000u   // part_len flag: sent without its strings (they exceed a whole slab)
// part_meta layout (u64 words)
#define PM_CUT 0                 // [64] records the slab takes per destination
#define PM_CUT_BYTES 64          // [64] their string bytes
#define PM_BYTES 128             // [64] string bytes of all the destination's records
#define PM_KEPT 192              // spilled records kept in the next carry
#define PM_KEPT_BYTES 193        // their string bytes (the next carry heap's size)

// Block-wide exclusive scan of one u64 per thread (string byte prefixes can pass 2^32).
__device__ __forceinline__ ull block_excl_scan64(ull v, ull* total, ull* lds) {
  const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
  ull inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const ull t = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += t;
  }
  if (lane == 63) lds[wid] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    ull acc = 0;
    for (int w = 0; w < WAVES; ++w) { const ull t = lds[w]; lds[w] = acc; acc += t; }
    lds[WAVES] = acc;
  }
  __syncthreads();
  const ull res = inc - v + lds[wid];
  *total = lds[WAVES];
  __syncthreads();
  return res;
}

// Per tile: records and string bytes per destination ([world][ntiles] each), the destination of
// every input (part_owner) and its exchange bytes (part_len; a record whose strings alone exceed a
// whole slab goes without them, counted in str_drops[0]).
__global__ void k_part_count(const SwEventRec* __restrict__ carry, const uint32_t* __restrict__ nc_ptr,
                             const SwEventRec* __restrict__ recs, const uint32_t* __restrict__ n_ptr,
                             int world, int rank, uint32_t* __restrict__ tcount /*[world][ntiles]*/, int64_t ntiles,
                             SwEngineArgs a) {
  __shared__ uint32_t cnt[64];
  __shared__ ull byt[64];
  if (threadIdx.x < 64) { cnt[threadIdx.x] = 0; byt[threadIdx.x] = 0; }
  if (BID == 0 && threadIdx.x < 2) a.part_meta[PM_KEPT + threadIdx.x] = 0;   // k_part_write counts into them
  __syncthreads();
  const bool strings = a.send_str != nullptr;
  const uint32_t nc = *nc_ptr;
  const int64_t n = (int64_t)nc + *n_ptr;
  const int64_t base = (int64_t)BID * TILE;
  for (int k = 0; k < TILE_ITEMS; ++k) {
    int64_t i = base + (int64_t)k * BLK + threadIdx.x;
    if (i < n) {
      const SwEventRec& r = part_in(carry, nc, recs, i);
      const uint32_t o = part_dest(a, r, (uint32_t)world, (uint32_t)rank);
      a.part_owner[i] = (uint8_t)o;           // k_part_cut / k_part_write read it back
      atomicAdd(&cnt[o], 1u);
      if (strings) {
        uint32_t L = part_str_len(a, r, nc, i);
        if ((int64_t)L > a.str_cap) {
          atomicAdd(&a.str_drops[0], 1u);
          L = PART_STRIP;
        } else if (L) {
          atomicAdd(&byt[o], (ull)L);
        }
        a.part_len[i] = L;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < world) {
    tcount[(int64_t)threadIdx.x * ntiles + BID] = cnt[threadIdx.x];
    a.part_bytes[(int64_t)threadIdx.x * ntiles + BID] = byt[threadIdx.x];
  }
}

// Records per destination from the scanned [world][ntiles] matrix.
__device__ __forceinline__ uint32_t part_total(const uint32_t* __restrict__ toff, const uint32_t* __restrict__ tcount,
                                               int64_t ntiles, int q) {
  const int64_t last = (int64_t)q * ntiles + ntiles - 1;
  return toff[last] + tcount[last] - toff[(int64_t)q * ntiles];
}

// One workgroup per destination q: the byte prefix of q's string slab per tile (u64 exclusive scan
// of its row of part_bytes), then the cut -- the prefix of q's records, in input order, that the
// slab takes: at most shuf_cap records whose strings fit str_cap bytes (CpuInboundEngine.partition).
// The cut falls in the first tile where either bound is crossed; that tile is walked record by
// record.  Writes the send counts (records, string bytes) and part_meta.
__global__ __launch_bounds__(BLK) void k_part_cut(const uint32_t* __restrict__ toff, const uint32_t* __restrict__ tcount,
                                                  int64_t ntiles, const uint32_t* __restrict__ nc_ptr,
                                                  const uint32_t* __restrict__ n_ptr, SwEngineArgs a) {
  __shared__ ull red[WAVES + 1];
  __shared__ int tstar;
  __shared__ uint32_t fit_c;
  __shared__ ull fit_b;
  const int q = (int)blockIdx.x;
  const ull* tb = (const ull*)a.part_bytes + (int64_t)q * ntiles;
  ull* bo = (ull*)a.part_bytes + (int64_t)a.world * ntiles + (int64_t)q * ntiles;
  ull acc = 0;
  for (int64_t c0 = 0; c0 < ntiles; c0 += BLK) {
    const int64_t t = c0 + threadIdx.x;
    const ull v = t < ntiles ? tb[t] : 0ull;
    ull tot;
    const ull ex = block_excl_scan64(v, &tot, red);
    if (t < ntiles) bo[t] = acc + ex;
    acc += tot;
  }
  const bool strings = a.send_str != nullptr;
  const ull blim = strings ? (ull)a.str_cap : ~0ull;
  const int64_t row = (int64_t)q * ntiles;
  const uint32_t c0q = toff[row];
  if (threadIdx.x == 0) { tstar = (int)ntiles; fit_c = 0; fit_b = 0; }
  __syncthreads();
  for (int64_t t = threadIdx.x; t < ntiles; t += BLK) {
    const ull cofs = toff[row + t] - c0q;
    if (cofs + tcount[row + t] > (ull)a.shuf_cap || bo[t] + tb[t] > blim) atomicMin(&tstar, (int)t);
  }
  __syncthreads();
  const int64_t ts = tstar;
  ull cut, bcut;
  if (ts >= ntiles) {
    cut = part_total(toff, tcount, ntiles, q);
    bcut = acc;
  } else {
    const uint32_t nc = *nc_ptr;
    const int64_t n = (int64_t)nc + *n_ptr;
    ull rc = toff[row + ts] - c0q, rb = bo[ts];
    const int64_t base = ts * TILE;
    for (int k = 0; k < TILE_ITEMS; ++k) {
      const int64_t i = base + (int64_t)k * BLK + threadIdx.x;
      const bool mine = i < n && a.part_owner[i] == (uint8_t)q;
      const ull L = mine && strings ? (ull)(a.part_len[i] & ~PART_STRIP) : 0ull;
      ull totc, totb;
      const ull exc = block_excl_scan64(mine ? 1ull : 0ull, &totc, red);
      const ull exb = block_excl_scan64(L, &totb, red);
      if (mine && rc + exc + 1 <= (ull)a.shuf_cap && rb + exb + L <= blim) {
        atomicAdd(&fit_c, 1u);
        atomicAdd(&fit_b, L);
      }
      rc += totc;
      rb += totb;
    }
    __syncthreads();
    cut = (ull)(toff[row + ts] - c0q) + fit_c;
    bcut = bo[ts] + fit_b;
  }
  if (threadIdx.x == 0) {
    a.part_meta[PM_CUT + q] = cut;
    a.part_meta[PM_CUT_BYTES + q] = bcut;
    a.part_meta[PM_BYTES + q] = acc;
    a.send_cnt[q] = (uint32_t)cut;
    if (strings) a.send_str_cnt[q] = (uint32_t)bcut;
  }
}

// A record's strings (alternate id, metadata, alert message, back to back) copied from `src` (this
// rank's raw batch, or the carry heap for a carried record) to dst[at..); returns its refs
// rewritten to those offsets and rebases the alert message in r.  `strip`: the record goes without
// its strings (they exceed a whole slab).
__device__ __forceinline__ SwStrRef part_strings(SwEventRec& r, const SwStrRef* s, const uint8_t* __restrict__ src,
                                                 bool strip, uint8_t* __restrict__ dst, ull at) {
  SwStrRef z;
  z.alt_off = 0; z.meta_off = 0; z.alt_len = 0; z.meta_len = 0; z.k = 0; z.has = 0; z.pad = 0;
  if (r.etype >= 16) return z;
  const SwStrRef sr = *s;
  const bool alert = r.etype == SW_EV_ALERT;
  const uint8_t has = strip ? (uint8_t)(sr.has & SW_SR_MULTI) : sr.has;
  const uint32_t al = (has & SW_SR_ALT) ? sr.alt_len : 0u;
  const uint32_t ml = (has & SW_SR_META) ? sr.meta_len : 0u;
  const uint32_t gl = alert && !strip ? r.aux2_len : 0u;
  z.k = sr.k;
  if (al + ml + gl == 0) {
    z.has = has & SW_SR_MULTI;
    if (alert) { r.aux2_off = 0; r.aux2_len = 0; }
    return z;
  }
  uint8_t* d = dst + at;
  for (uint32_t b = 0; b < al; ++b) d[b] = src[sr.alt_off + b];
  for (uint32_t b = 0; b < ml; ++b) d[al + b] = src[sr.meta_off + b];
  for (uint32_t b = 0; b < gl; ++b) d[al + ml + b] = src[r.aux2_off + b];
  z.has = has;
  z.alt_off = (uint32_t)at;
  z.meta_off = (uint32_t)(at + al);
  z.alt_len = (uint16_t)al;
  z.meta_len = (uint16_t)ml;
  if (alert) { r.aux2_off = (uint32_t)(at + al + ml); r.aux2_len = (uint16_t)gl; }
  return z;
}

// Stable scatter: a record's position among its destination's records (and its strings' byte
// position) decides its place -- in the slab below the cut, else in the spill (the next carry,
// destination-major) with its strings in the spill heap.  Spilled records beyond carry_cap or the
// spill heap (a prefix of the spill order, like the oracle's) are dropped and counted.
__global__ __launch_bounds__(BLK) void k_part_write(const SwEventRec* __restrict__ carry, const uint32_t* __restrict__ nc_ptr,
                             const SwEventRec* __restrict__ recs, const uint32_t* __restrict__ n_ptr, int world,
                             int rank, const uint32_t* __restrict__ toff /*scanned [world][ntiles]*/,
                             const uint32_t* __restrict__ tcount, int64_t ntiles, SwWireRec* __restrict__ send,
                             int64_t shuf_cap, SwEventRec* __restrict__ spill, int64_t carry_cap, SwEngineArgs a) {
  __shared__ uint32_t run[64];
  __shared__ ull rbyt[64];
  __shared__ uint32_t cutq[64];
  __shared__ ull bcutq[64];
  __shared__ uint32_t spill_base[64];
  __shared__ ull spill_bbase[64];
  __shared__ uint32_t wcnt[WAVES][64];
  __shared__ ull wbyt[WAVES][64];
  __shared__ uint32_t kept_c;
  __shared__ ull kept_b;
  const uint32_t nc = *nc_ptr;
  const int64_t n = (int64_t)nc + *n_ptr;
  const int64_t base = (int64_t)BID * TILE;
  const uint32_t wid = threadIdx.x >> 6, lane = lane_id();
  const bool strings = a.send_str != nullptr;
  const ull* bo = (const ull*)a.part_bytes + (int64_t)world * ntiles;
  if (threadIdx.x < world) {
    const int64_t row = (int64_t)threadIdx.x * ntiles;
    run[threadIdx.x] = toff[row + BID] - toff[row];
    rbyt[threadIdx.x] = bo[row + BID];
    cutq[threadIdx.x] = (uint32_t)a.part_meta[PM_CUT + threadIdx.x];
    bcutq[threadIdx.x] = a.part_meta[PM_CUT_BYTES + threadIdx.x];
  }
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    ull bacc = 0;
    for (int q = 0; q < world; ++q) {
      spill_base[q] = acc;
      spill_bbase[q] = bacc;
      acc += part_total(toff, tcount, ntiles, q) - (uint32_t)a.part_meta[PM_CUT + q];
      bacc += a.part_meta[PM_BYTES + q] - a.part_meta[PM_CUT_BYTES + q];
    }
    kept_c = 0;
    kept_b = 0;
  }
  __syncthreads();
  for (int k = 0; k < TILE_ITEMS; ++k) {
    const int64_t i = base + (int64_t)k * BLK + threadIdx.x;
    const bool valid = i < n;
    const uint32_t o = valid ? a.part_owner[i] : 0u;
    const uint32_t L = valid && strings ? a.part_len[i] : 0u;
    const ull Lb = L & ~PART_STRIP;
    if (lane < (uint32_t)world) { wcnt[wid][lane] = 0; wbyt[wid][lane] = 0; }
    // rank and byte prefix among the wave's records of the same destination, one pass per
    // destination present in the wave
    uint32_t my_rank = 0;
    ull my_b = 0;
    ull rem = __ballot(valid);
    while (rem) {
      const uint32_t q = __shfl(o, (int)__ffsll((long long)rem) - 1, 64);
      const bool mine = valid && o == q;
      const ull m = __ballot(mine);
      ull inc = mine ? Lb : 0ull;
      if (strings) {
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const ull t = __shfl_up(inc, d, 64);
          if (lane >= (uint32_t)d) inc += t;
        }
      }
      if (mine) { my_rank = __popcll(m & lanemask_lt()); my_b = inc - Lb; }
      if (lane == 63) { wcnt[wid][q] = __popcll(m); wbyt[wid][q] = inc; }
      rem &= ~m;
    }
    __syncthreads();
    if (valid) {
      uint32_t pre = run[o];
      ull bpre = rbyt[o];
      for (uint32_t w = 0; w < wid; ++w) { pre += wcnt[w][o]; bpre += wbyt[w][o]; }
      pre += my_rank;
      bpre += my_b;
      SwEventRec r = part_in(carry, nc, recs, i);
      const bool fresh = i >= (int64_t)nc;
      const SwStrRef* sr = strings ? (fresh ? a.spans + (i - nc) : a.carry_spans + i) : nullptr;
      const uint8_t* src = fresh ? a.raw : a.carry_str;
      if (pre < cutq[o]) {
        const int64_t at = (int64_t)o * shuf_cap + pre;
        if (strings)
          a.send_spans[at] = part_strings(r, sr, src, (L & PART_STRIP) != 0, a.send_str + (int64_t)o * a.str_cap, bpre);
        send[at] = sw_wire_pack(r);
      } else {
        const int64_t j = (int64_t)spill_base[o] + (pre - cutq[o]);
        const ull sb = spill_bbase[o] + (bpre - bcutq[o]);
        if (j < carry_cap && (!strings || sb + Lb <= (ull)a.carry_str_cap)) {
          if (strings) a.spill_spans[j] = part_strings(r, sr, src, (L & PART_STRIP) != 0, a.spill_str, sb);
          spill[j] = r;
          atomicAdd(&kept_c, 1u);
          if (Lb) atomicAdd(&kept_b, Lb);
        }
      }
    }
    __syncthreads();
    if (threadIdx.x < world) {
      uint32_t t = 0;
      ull tb = 0;
      for (int w = 0; w < WAVES; ++w) { t += wcnt[w][threadIdx.x]; tb += wbyt[w][threadIdx.x]; }
      run[threadIdx.x] += t;
      rbyt[threadIdx.x] += tb;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && kept_c) {
    atomicAdd((ull*)&a.part_meta[PM_KEPT], (ull)kept_c);
    atomicAdd((ull*)&a.part_meta[PM_KEPT_BYTES], kept_b);
  }
}

__global__ void k_part_counts(const uint32_t* __restrict__ toff, const uint32_t* __restrict__ tcount, int64_t ntiles,
                              int world, SwEngineArgs a) {
  if (threadIdx.x == 0 && BID == 0) {
    ull over = 0;
    for (int o = 0; o < world; ++o) over += part_total(toff, tcount, ntiles, o) - a.part_meta[PM_CUT + o];
    const ull kept = a.part_meta[PM_KEPT];
    *a.n_spill = (uint32_t)kept;
    if (a.n_spill_str) *a.n_spill_str = (uint32_t)a.part_meta[PM_KEPT_BYTES];
    *a.overflow = (uint32_t)(over - kept);
    ((ull*)a.stats)[SW_STAT_SHUFFLE_DEFERRED] += kept;
    ((ull*)a.stats)[SW_STAT_SHUFFLE_OVERFLOW] += over - kept;
  }
}

// Concatenate the received [world][shuf_cap] slabs into one dense batch (rank order).  With the
// string exchange on, each record's refs come along rebased into work_str (+ source rank *
// str_cap), and the received byte slabs are gathered into work_str -- the receive buffers are
// reused by the next exchange while this step's block may still be encoding.
__global__ void k_unpack(const SwWireRec* __restrict__ recv, const uint32_t* __restrict__ recv_cnt, int world,
                         int64_t shuf_cap, SwEventRec* __restrict__ work, uint32_t* __restrict__ n_work, int64_t cap,
                         SwEngineArgs a) {
  __shared__ uint32_t pre[65];
  if (threadIdx.x == 0) {
    pre[0] = 0;
    for (int q = 0; q < world; ++q) pre[q + 1] = pre[q] + (recv_cnt[q] < shuf_cap ? recv_cnt[q] : (uint32_t)shuf_cap);
  }
  __syncthreads();
  const uint32_t total = pre[world] < cap ? pre[world] : (uint32_t)cap;
  if (BID == 0 && threadIdx.x == 0) *n_work = total;
  const bool strings = a.work_str != nullptr;
  for (int64_t i = (int64_t)BID * BLK + threadIdx.x; i < total; i += (int64_t)gridDim.x * BLK) {
    int q = 0;
    while (q + 1 < world && i >= pre[q + 1]) ++q;
    SwEventRec r = sw_wire_unpack(recv[(int64_t)q * shuf_cap + (i - pre[q])], (uint8_t)q);
    if (strings) {
      SwStrRef sr = a.recv_spans[(int64_t)q * shuf_cap + (i - pre[q])];
      const uint32_t base = (uint32_t)((int64_t)q * a.str_cap);
      sr.alt_off += base;
      sr.meta_off += base;
      if (r.etype == SW_EV_ALERT) r.aux2_off += base;
      a.work_spans[i] = sr;
    }
    work[i] = r;
  }
  if (strings) {                             // the used part of every received byte slab, 16 B at a time
    for (int q = 0; q < world; ++q) {
      const uint32_t used = a.recv_str_cnt[q] < a.str_cap ? a.recv_str_cnt[q] : (uint32_t)a.str_cap;
      const uint4* src = reinterpret_cast<const uint4*>(a.recv_str + (int64_t)q * a.str_cap);
      uint4* dst = reinterpret_cast<uint4*>(a.work_str + (int64_t)q * a.str_cap);
      for (int64_t v = (int64_t)BID * BLK + threadIdx.x; v < (used + 15) / 16; v += (int64_t)gridDim.x * BLK)
        dst[v] = src[v];
    }
  }
}

// ============================================================================ validate
// Intern a name hash; the thread that claims a new slot gives it the next dense id (the ids are
// rank-local state-map keys, read by later kernels of the step -- no table-wide assign pass).
__device__ __forceinline__ void intern_insert(ull* __restrict__ key, int32_t* __restrict__ ids,
                                              int32_t* __restrict__ counter, int64_t mask, ull h) {
  int64_t slot = (int64_t)(h & (ull)mask);
  for (int64_t p = 0; p <= mask && p < MAX_PROBE; ++p) {
    ull old = key[slot];
    if (old == h) return;
    if (old == 0) {
      old = atomicCAS(&key[slot], 0ull, h);
      if (old == 0) {
        ids[slot] = atomicAdd(counter, 1);
        return;
      }
      if (old == h) return;
    }
    slot = (slot + 1) & mask;
  }
}

// Alternate-id dedup window (reference AlternateIdDeduplicator.java:41-56), generational: two
// open-addressing tables, `cur` (ids first seen in the current generation) and `prev` (the
// generation before).  An event whose id is in `prev` is a duplicate; otherwise it is inserted into
// `cur`, where the first occurrence (lowest global sequence) wins and every later one -- in this
// batch or any later batch of the generation -- is a duplicate.  When a step leaves `cur` past half
// its slots less one batch, the generations rotate for the next step: k_persist decides, k_state_p2
// clears the retiring table, k_step_end flips (dd_meta = [generation, ids in cur, rotation state,
// ids that met a claimed key]).  The window therefore covers the last slots/2 - rec_cap to
// slots - rec_cap distinct ids, probes stay short (load <= 0.5), and a probe that still hits
// MAX_PROBE is counted (SW_STAT_DEDUP_OVERFLOW) rather than silently ignored.
//
// Tables of packed 16-byte slots {key, win: u32, lmin: u32} (two generations of dd_mask + 1 slots):
//   key  -- the alternate-id hash, claimed by CAS;
//   win  -- low 32 bits of the sequence of the id that claimed the slot (plain store by the CAS
//           winner: the slot's other fields are disjoint bytes);
//   lmin -- lowest in-batch index of the ids that found the key already claimed in THIS batch
//           (atomicMin; rare: only repeats inside one batch).
// First occurrence = the slot was claimed in this batch and min(win - sb, lmin) is the id's index:
// the same lowest-sequence rule as the host engines, with ONE memory-side atomic per new id (each
// device-scope atomic is its own 64-byte request on the MI355X; the CAS + atomicMin form paid two).
// win - sb needs the window (< 2^31 ids) to stay far below 2^32 sequences, which rotation ensures.
// A step where no id met an already-claimed key (dd_meta[3] == 0: fresh ids, the common case) needs
// no verdict pass: every claimer is its key's first occurrence, and its store-backed filter probe
// (SW_ST_RECHECK) is done at the claim.  Otherwise k_cmp_count settles every id from its slot.
__device__ __forceinline__ bool dd_find(const ull* __restrict__ tab, int64_t mask, ull h) {
  int64_t slot = (int64_t)(h & (ull)mask);
  for (int64_t p = 0; p <= mask && p < MAX_PROBE; ++p) {
    const ull k = tab[2 * slot];
    if (k == h) return true;
    if (k == 0) return false;
    slot = (slot + 1) & mask;
  }
  return false;
}

// Store-backed filter (generational fingerprint tables, swtypes.h SW_FF_*).  Does a live generation
// hold the id's fingerprint?  It may have been persisted before (beyond the window).  The G buckets
// of a home position are adjacent: one probe round reads G * 64 contiguous bytes (16-byte loads),
// and a generation's chain goes on to the next position only while its bucket is full.
__device__ __forceinline__ bool ff_has(const uint32_t* __restrict__ t, int64_t bmask, int gens, ull h) {
  const ull m = sw_ff_mix(h);
  const uint32_t fp = sw_ff_fp(m);
  int64_t b = (int64_t)sw_ff_bucket(m, bmask);
  uint32_t open = (1u << gens) - 1u;
  for (int p = 0; p < SW_FF_MAX_PROBE && open; ++p) {
    const uint4* __restrict__ q = reinterpret_cast<const uint4*>(t + b * gens * SW_FF_SLOTS);
    for (int g = 0; g < gens; ++g) {
      if (!((open >> g) & 1u)) continue;
      bool empty = false;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint4 v = q[g * 4 + k];
        if (v.x == fp || v.y == fp || v.z == fp || v.w == fp) return true;
        empty |= !v.x || !v.y || !v.z || !v.w;
      }
      if (empty) open &= ~(1u << g);
    }
    b = (b + 1) & bmask;
  }
  return false;
}

// Add the id's fingerprint to generation g: one CAS into the first free slot of its chain (a slot
// another thread took first holds a different id, or the same one: then it is in).  False: the
// probe bound was hit (dropped, counted by the caller).
__device__ __forceinline__ bool ff_add(uint32_t* __restrict__ t, int64_t bmask, int gens, int g, ull h) {
  const ull m = sw_ff_mix(h);
  const uint32_t fp = sw_ff_fp(m);
  int64_t b = (int64_t)sw_ff_bucket(m, bmask);
  for (int p = 0; p < SW_FF_MAX_PROBE; ++p) {
    uint32_t* s = t + (b * gens + g) * SW_FF_SLOTS;
    uint32_t v[SW_FF_SLOTS];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 x = reinterpret_cast<const uint4*>(s)[k];
      v[4 * k] = x.x; v[4 * k + 1] = x.y; v[4 * k + 2] = x.z; v[4 * k + 3] = x.w;
    }
#pragma unroll
    for (int k = 0; k < SW_FF_SLOTS; ++k)
      if (v[k] == fp) return true;
#pragma unroll
    for (int k = 0; k < SW_FF_SLOTS; ++k) {
      if (v[k]) continue;
      const uint32_t old = atomicCAS(&s[k], 0u, fp);
      if (old == 0u || old == fp) return true;
    }
    b = (b + 1) & bmask;
  }
  return false;
}

// Clear generation g (grid-stride over the buckets; 64 bytes per bucket).
__device__ __forceinline__ void ff_clear_gen(uint32_t* __restrict__ t, int64_t bmask, int gens, int g) {
  const int64_t nb = bmask + 1;
  const int64_t n = nb * 4;
  for (int64_t i = (int64_t)BID * BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK)
    reinterpret_cast<uint4*>(t + ((i >> 2) * gens + g) * SW_FF_SLOTS)[i & 3] = make_uint4(0u, 0u, 0u, 0u);
}

struct DedupCounts {
  uint32_t fresh, over, lose;
};

// Claim the id's slot in `cur` (k_dedup_claim, after k_lookup validated the record).  Returns
// the id's provisional status: DUPLICATE (held by `prev`), RECHECK (first claim of an id the
// filter sees, maybe stored before; see filter_sees) or OK.
// Everything a claim needs, read once per thread (not per id: loads through the by-value engine
// arguments cannot be hoisted past the claim's stores).
struct DedupClaim {
  ull* __restrict__ ct;                      // live generation
  const ull* __restrict__ pt;                // retired generation
  int64_t mask;
  ull sb;                                    // the step's first sequence
  const uint32_t* __restrict__ ff;           // store-backed filter (null: off)
  int64_t fbmask;
  int fgens;
  int rank;                                  // filter_rank (-1: every record)
};

// Does the store-backed filter see this record?  Every record this rank owns when the strings came
// along with the re-key (work_str: the host settles a recheck by its alternate id), else only those
// decoded here (the host path re-reads their payload).  A record the host already settled skips it.
__device__ __forceinline__ int filter_rank(const SwEngineArgs& a) { return a.work_str ? -1 : (int)a.rank; }
__device__ __forceinline__ bool filter_sees(const SwEventRec& r, int rank) {
  return !(r.flags & SW_F_SETTLED) && (rank < 0 || r.src_rank == (uint8_t)rank);
}

__device__ __forceinline__ DedupClaim dedup_claim_args(const SwEngineArgs& a) {
  DedupClaim d;
  const int64_t slots = a.dd_mask + 1, g = a.dd_meta[0];
  d.ct = (ull*)a.dd_key + 2 * g * slots;
  d.pt = (const ull*)a.dd_key + 2 * (1 - g) * slots;
  d.mask = a.dd_mask;
  d.sb = (ull)*a.seq_base;
  d.ff = a.dd_ff;
  d.fbmask = a.dd_ff_bmask;
  d.fgens = (int)a.dd_ff_gens;
  d.rank = filter_rank(a);
  return d;
}

// `maybe_stored`: the filter holds the id's bits and sees this record (a first claim is a recheck).
// `check_prev`: the id may be in the retired generation.  Every id a generation holds was persisted
// (or was a recheck, itself a filter hit), and every persisted id is in the store-backed filter, so
// an id the filter does not hold cannot be there: with the filter on, its probe (needed for the
// recheck anyway) stands in for the retired-generation probe of every fresh id.
__device__ __forceinline__ uint8_t dedup_claim(const DedupClaim& dc, ull h, int64_t i, bool maybe_stored,
                                               bool check_prev, DedupCounts& c) {
  const int64_t mask = dc.mask;
  ull* __restrict__ ct = dc.ct;
  if (check_prev && dd_find(dc.pt, mask, h)) return SW_ST_DUPLICATE;
  const ull sb = dc.sb;
  int64_t slot = (int64_t)(h & (ull)mask);
  for (int64_t p = 0; p <= mask && p < MAX_PROBE; ++p) {
    const ull old = atomicCAS(&ct[2 * slot], 0ull, h);
    if (old == 0) {
      ++c.fresh;
      reinterpret_cast<uint32_t*>(&ct[2 * slot + 1])[0] = (uint32_t)(sb + (ull)i);
      return maybe_stored ? (uint8_t)SW_ST_RECHECK : (uint8_t)SW_ST_OK;
    }
    if (old == h) {
      atomicMin(reinterpret_cast<uint32_t*>(&ct[2 * slot + 1]) + 1, (uint32_t)i);
      ++c.lose;
      return SW_ST_OK;
    }
    slot = (slot + 1) & mask;
  }
  ++c.over;                                  // not placed: kept (counted)
  return SW_ST_OK;
}

// One probe of the packed registry resolves device AND active assignment; names of every
// decodable event are interned here too (fused: one pass over the records).
__global__ void k_lookup(SwEngineArgs a) {
  // world == 1: the work batch is the decoded batch, clamped (every block derives the same count;
  // block 0 stores it for the kernels after this one)
  const uint32_t n = a.world == 1 ? (*a.n_recs < (uint32_t)a.rec_cap ? *a.n_recs : (uint32_t)a.rec_cap) : *a.n_work;
  if (BID == 0 && threadIdx.x == 0) {      // start of the process phase (was its own dispatch)
    if (a.world == 1) {
      *a.n_recs = n;
      *a.n_work = n;
      ((ull*)a.stats)[SW_STAT_NEW_NAMES] += *a.n_new_names;
    }
    *a.step_cursor0 = *a.store_cursor;
    *a.n_gen = 0;
    *a.n_out = 0;
    if (a.dd_meta[2] == 2) {               // the generations rotated at the end of the last step
      ((ull*)a.stats)[SW_STAT_DEDUP_ROTATIONS] += 1;
      a.dd_meta[2] = 0;
    }
  }
  const SwEventRec* __restrict__ recs = a.work;
  for (int64_t i = (int64_t)BID * BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK) {
    const ull lo = recs[i].fp_lo, hi = recs[i].fp_hi;
    const uint8_t et = recs[i].etype;
    const ull nh = recs[i].name_hash;
    uint8_t st;
    int32_t dev = -1, asg = -1;
    if (et == SW_EV_DECODE_ERROR) st = SW_ST_DECODE_ERROR;
    else {
      int64_t slot = (int64_t)(lo & (ull)a.reg_mask);
      for (int64_t p = 0; p <= a.reg_mask && p < MAX_PROBE; ++p) {
        const ulonglong2 k = *reinterpret_cast<const ulonglong2*>(&a.reg[slot].lo);
        if (k.x == lo && k.y == hi) {
          const int2 v = *reinterpret_cast<const int2*>(&a.reg[slot].dev);
          dev = v.x; asg = v.y;
          break;
        }
        if (k.x == 0 && k.y == 0) break;
        slot = (slot + 1) & a.reg_mask;
      }
      if (et >= 16) { st = SW_ST_CONTROL; asg = -1; }
      else if (dev < 0) st = SW_ST_UNREGISTERED;
      else st = asg >= 0 ? SW_ST_OK : SW_ST_UNASSIGNED;
      if (st == SW_ST_OK && nh) intern_insert((ull*)a.nm_key, a.nm_id, a.nm_counter, a.nm_mask, nh);
    }
    a.status[i] = st;
    a.ev_dev[i] = dev;
    a.ev_asg[i] = asg;
    // the claim's input, dense: the id to claim (0: none -- not valid, no id, or settled) and
    // whether the store-backed filter sees the record (ev_slot is free until k_persist)
    const SwEventRec& r = recs[i];
    const bool claim = st == SW_ST_OK && r.alt_hash && !(r.flags & SW_F_SETTLED);
    ull* ck = reinterpret_cast<ull*>(a.ev_slot);
    ck[i] = claim ? r.alt_hash : 0ull;
    reinterpret_cast<uint8_t*>(ck + a.rec_cap)[i] = (uint8_t)filter_sees(r, filter_rank(a));
  }
}

// The store-backed filter's verdict for every id to claim, before the claim: 16 lanes per id, lane q
// loading 16-byte word q (and q + 16 with more than 4 generations) of the id's home span -- the G
// adjacent 64-byte buckets -- so one load instruction covers four ids' spans in full lines (one thread
// per id issued 16 scattered loads per id and ran ~220 us per 1M ids, profiles/r6_kernels).  A
// generation whose bucket is full without the fingerprint goes on to the next span.  Sets bit 1 of
// the id's claim flag (ev_slot + rec_cap) when a generation may hold it.
__global__ __launch_bounds__(BLK) void k_ff_probe(SwEngineArgs a) {
  const uint32_t n = *a.n_work;
  const ull* __restrict__ ck = reinterpret_cast<const ull*>(a.ev_slot);
  uint8_t* __restrict__ cf = reinterpret_cast<uint8_t*>(reinterpret_cast<ull*>(a.ev_slot) + a.rec_cap);
  const uint32_t* __restrict__ t = a.dd_ff;
  const int gens = (int)a.dd_ff_gens;
  const int64_t bmask = a.dd_ff_bmask;
  const uint32_t lane = threadIdx.x & 63u, sub = lane & 15u, grp = lane >> 4;
  const int64_t g0 = ((int64_t)BID * BLK + threadIdx.x) >> 4;
  const int64_t gstride = ((int64_t)gridDim.x * BLK) >> 4;
  const int words = gens * 4;                     // 16-byte words of a span
  for (int64_t base = g0 - grp; base < (int64_t)n; base += gstride) {
    // the wave's four groups take ids base + 0..3 (group-uniform: every lane of a group agrees)
    const int64_t i = base + grp;
    const ull h = i < (int64_t)n ? ck[i] : 0ull;
    const ull m = sw_ff_mix(h);
    const uint32_t fp = sw_ff_fp(m);
    int64_t b = (int64_t)sw_ff_bucket(m, bmask);
    uint32_t open = h ? (1u << gens) - 1u : 0u;
    bool held = false;
    for (int p = 0; p < SW_FF_MAX_PROBE; ++p) {
      bool hit = false;
      uint32_t empty_g = 0;
      const uint4* __restrict__ q = reinterpret_cast<const uint4*>(t + b * gens * SW_FF_SLOTS);
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int w = (int)sub + 16 * r;
        const int gg = w >> 2;
        if (w < words && ((open >> gg) & 1u)) {
          const uint4 v = q[w];
          hit |= v.x == fp || v.y == fp || v.z == fp || v.w == fp;
          if (!v.x || !v.y || !v.z || !v.w) empty_g |= 1u << gg;
        }
      }
      // the group's answer: any lane's hit; a generation is closed once any of its words has a hole
      const ull hb = __ballot(hit);
      uint32_t e = empty_g;
#pragma unroll
      for (int o = 8; o >= 1; o >>= 1) e |= __shfl_xor(e, o, 16);
      if ((hb >> (16 * grp)) & 0xffffull) { held = true; open = 0; }
      open &= ~e;
      const bool more = open != 0;
      if (!__any(more)) break;
      b = (b + 1) & bmask;
    }
    if (held && sub == 0) cf[i] |= 2u;
  }
}

// The dedup claims of the step's validated records.  A kernel of its own: fused into k_lookup the
// three dependent round trips per id (registry probe, `prev` probe, CAS) ran 255 us per 1M ids
// against 48 + 143 us as two kernels (profiles/r4_fused_claim).
__global__ void k_dedup_claim(SwEngineArgs a) {
  __shared__ uint32_t blk_new, blk_over, blk_lose;
  if (threadIdx.x == 0) { blk_new = 0; blk_over = 0; blk_lose = 0; }
  __syncthreads();
  DedupCounts dc = {0u, 0u, 0u};
  const DedupClaim d = dedup_claim_args(a);
  const uint32_t n = *a.n_work;
  uint8_t* __restrict__ status = a.status;
  // k_lookup's dense claim list: the id (0: nothing to claim; a settled recheck skips the window,
  // its id was claimed when it came back as a recheck) and the filter's view of the record
  const ull* __restrict__ ck = reinterpret_cast<const ull*>(a.ev_slot);
  const uint8_t* __restrict__ cf = reinterpret_cast<const uint8_t*>(ck + a.rec_cap);
  for (int64_t i = (int64_t)BID * BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK) {
    const ull ah = ck[i];
    if (!ah) continue;
    const bool held = d.ff && (cf[i] & 2u);                 // k_ff_probe's verdict
    const uint8_t st = dedup_claim(d, ah, i, held && (cf[i] & 1u), !d.ff || held, dc);
    if (st != SW_ST_OK) status[i] = st;
  }
  // dedup counters aggregated per workgroup: one global atomic per block, not one per id (1M
  // same-address atomics per step serialised the kernel, profiles/r3_dedup)
  if (dc.fresh) atomicAdd(&blk_new, dc.fresh);
  if (dc.over) atomicAdd(&blk_over, dc.over);
  if (dc.lose) atomicAdd(&blk_lose, dc.lose);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (blk_new) atomicAdd((unsigned long long*)&a.dd_meta[1], (ull)blk_new);
    if (blk_over) atomicAdd((ull*)&a.stats[SW_STAT_DEDUP_OVERFLOW], (ull)blk_over);
    if (blk_lose) atomicAdd((unsigned long long*)&a.dd_meta[3], (ull)blk_lose);
  }
}

// Second half of the dedup (fused into the compaction count, k_cmp_count): the id's verdict from
// its slot's {key, win, lmin}, one 16-byte load; a first sighting the store-backed filter may hold
// becomes SW_ST_RECHECK.
struct DedupView {
  const ulonglong2* ct;       // live generation (null: no alternate-id dedup this step)
  int64_t mask;
  uint32_t sb, n;
  const uint32_t* ff;
  int64_t fbmask;
  int fgens;
};

__device__ __forceinline__ uint8_t dedup_verdict(const DedupView& d, ull h, uint32_t i, bool local) {
  int64_t slot = (int64_t)(h & (ull)d.mask);
  for (int64_t p = 0; p <= d.mask && p < MAX_PROBE; ++p) {
    const ulonglong2 kq = d.ct[slot];
    if (kq.x == h) {
      const uint32_t wrel = (uint32_t)kq.y - d.sb;
      const uint32_t lmin = (uint32_t)(kq.y >> 32);
      const bool first = wrel < d.n && (wrel < lmin ? wrel : lmin) == i;
      if (!first) return SW_ST_DUPLICATE;
      return (local && d.ff && ff_has(d.ff, d.fbmask, d.fgens, h)) ? SW_ST_RECHECK : SW_ST_OK;   // first sight
    }
    if (kq.x == 0) break;                // not placed (probe overflow, counted): kept
    slot = (slot + 1) & d.mask;
  }
  return SW_ST_OK;
}

// ============================================================================ compaction
// Stable split of [0, n) into ok (status == OK) and rejected lists.  The count pass also settles the
// dedup verdict of every id k_lookup's claim left OK / RECHECK (dedup_verdict): no separate check dispatch.
__global__ void k_cmp_count(uint8_t* __restrict__ status, const uint32_t* __restrict__ n_ptr,
                            uint32_t* __restrict__ tcnt /*[2][ntiles]*/, int64_t ntiles, ull* __restrict__ stats,
                            const SwEventRec* __restrict__ recs, const ull* __restrict__ dd_tab, int64_t dd_mask,
                            const int64_t* __restrict__ seq_base, const int64_t* __restrict__ dd_meta,
                            const uint32_t* __restrict__ ff, int64_t fbmask, int fgens, int rank) {
  __shared__ uint32_t c[2];
  __shared__ uint32_t rs[8];          // rejects by status (the reject counters of the step)
  if (threadIdx.x < 2) c[threadIdx.x] = 0;
  if (threadIdx.x < 8) rs[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t n = *n_ptr;
  DedupView dv;
  // no id met a claimed key this step: the claim's statuses are final (see dedup_claim)
  dv.ct = (dd_tab && dd_meta[3]) ? reinterpret_cast<const ulonglong2*>(dd_tab) + dd_meta[0] * (dd_mask + 1) : nullptr;
  dv.mask = dd_mask;
  dv.sb = (uint32_t)*seq_base;
  dv.n = n;
  dv.ff = ff;
  dv.fbmask = fbmask;
  dv.fgens = fgens;
  const int64_t base = (int64_t)BID * TILE;
  uint32_t ok = 0, all = 0;
#pragma unroll
  for (int k = 0; k < TILE_ITEMS; ++k) {
    const int64_t i = base + (int64_t)k * BLK + threadIdx.x;
    const bool v = i < n;
    uint8_t st = v ? status[i] : (uint8_t)SW_ST_OK;
    if (v && (st == SW_ST_OK || st == SW_ST_RECHECK) && dv.ct) {
      const ull h = recs[i].alt_hash;
      if (h && !(recs[i].flags & SW_F_SETTLED)) {
        const uint8_t vst = dedup_verdict(dv, h, (uint32_t)i, filter_sees(recs[i], rank));
        if (vst != st) status[i] = vst;
        st = vst;
      }
    }
    ok += __popcll(__ballot(v && st == SW_ST_OK));
    all += __popcll(__ballot(v));
    if (st != SW_ST_OK) atomicAdd(&rs[st & 7], 1u);       // rare: ~1% of events
  }
  if (lane_id() == 0) { atomicAdd(&c[0], ok); atomicAdd(&c[1], all - ok); }
  __syncthreads();
  if (threadIdx.x == 0) { tcnt[BID] = c[0]; tcnt[ntiles + BID] = c[1]; }
  if (threadIdx.x < 8 && rs[threadIdx.x]) {
    const int slot = threadIdx.x == SW_ST_UNREGISTERED ? SW_STAT_UNREGISTERED
                   : threadIdx.x == SW_ST_UNASSIGNED ? SW_STAT_UNASSIGNED
                   : threadIdx.x == SW_ST_DUPLICATE ? SW_STAT_DUPLICATE
                   : threadIdx.x == SW_ST_DECODE_ERROR ? SW_STAT_DECODE_ERROR
                   : threadIdx.x == SW_ST_CONTROL ? SW_STAT_CONTROL
                   : threadIdx.x == SW_ST_RECHECK ? SW_STAT_DEDUP_RECHECKS : -1;
    if (slot >= 0) atomicAdd(&stats[slot], (ull)rs[threadIdx.x]);
  }
}

// Tile offsets from k_cmp_count's tile counts, reduced in the prologue (no scan dispatch).
__global__ void k_cmp_write(const uint8_t* __restrict__ status, const uint32_t* __restrict__ n_ptr,
                            const uint32_t* __restrict__ tcnt, int64_t ntiles,
                            uint32_t* __restrict__ ok_idx, uint32_t* __restrict__ rej_idx,
                            uint32_t* __restrict__ n_ok, uint32_t* __restrict__ n_rej) {
  __shared__ uint32_t lds[WAVES + 1];
  const uint32_t n = *n_ptr;
  const int64_t base = (int64_t)BID * TILE;
  uint32_t run_ok = block_sum_prefix(tcnt, BID, lds);
  uint32_t run_rj = block_sum_prefix(tcnt + ntiles, BID, lds);
  if (BID == gridDim.x - 1 && threadIdx.x == 0) {
    *n_ok = run_ok + tcnt[BID];
    *n_rej = run_rj + tcnt[ntiles + BID];
  }
  for (int k = 0; k < TILE_ITEMS; ++k) {
    const int64_t i = base + (int64_t)k * BLK + threadIdx.x;
    const bool valid = i < n;
    const bool ok = valid && status[i] == SW_ST_OK;
    const bool rj = valid && !ok;
    uint32_t tot_ok, tot_rj;
    uint32_t p_ok = block_excl_scan(ok ? 1u : 0u, &tot_ok, lds);
    uint32_t p_rj = block_excl_scan(rj ? 1u : 0u, &tot_rj, lds);
    if (ok) ok_idx[run_ok + p_ok] = (uint32_t)i;
    if (rj) rej_idx[run_rj + p_rj] = (uint32_t)i;
    run_ok += tot_ok;
    run_rj += tot_rj;
  }
}

// ============================================================================ names intern
template <typename K>
__device__ __forceinline__ int64_t nm_probe(const K* __restrict__ key, int64_t mask, ull h) {
  int64_t slot = (int64_t)(h & (ull)mask);
  for (int64_t p = 0; p <= mask && p < MAX_PROBE; ++p) {
    const ull k = key[slot];
    if (k == h) return slot;
    if (k == 0) return -1;
    slot = (slot + 1) & mask;
  }
  return -1;
}

__global__ void k_intern_insert_list(const SwEventRec* __restrict__ recs, const uint32_t* __restrict__ n_ptr,
                                     ull* __restrict__ key, int32_t* __restrict__ ids, int32_t* __restrict__ counter,
                                     int64_t mask, uint32_t cap) {
  const uint32_t n = *n_ptr < cap ? *n_ptr : cap;
  for (int64_t j = (int64_t)BID * BLK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLK)
    if (recs[j].name_hash) intern_insert(key, ids, counter, mask, recs[j].name_hash);
}

// ============================================================================ device state map
__device__ __forceinline__ int64_t ms_slot(SwMsSlot* __restrict__ ms, int64_t mask, ull k) {
  int64_t slot = (int64_t)(sw_mix64(k) & (ull)mask);
  for (int64_t p = 0; p <= mask && p < MAX_PROBE; ++p) {
    ull* kp = (ull*)&ms[slot].key;
    ull old = *kp;
    if (old == k) return slot;
    if (old == 0) {
      old = atomicCAS(kp, 0ull, k);
      if (old == 0 || old == k) return slot;
    }
    slot = (slot + 1) & mask;
  }
  return -1;
}

// ============================================================================ persist + enrich + state pass 1
// One pass over the validated events: write the HBM ring row and the outbound row, and run pass 1
// of the device-state merge (max event date per assignment location / per (assignment, name)
// slot).  The (assignment, name) slot found or claimed here is kept in ev_slot[j] for pass 2, so
// the name probe and the state-map probe run once per event instead of once per pass.
// Tried and measured in round 5 (profiles/r5_kernels): plain stores for the state words of rows alone
// in their assignment's run (clustered order), and the filter adds as their own pass on a parallel
// graph branch -- neither made the phase faster, so the merges stay atomic and the adds in line.
__global__ void k_persist(SwEngineArgs a, const SwEventRec* __restrict__ R, const uint32_t* __restrict__ idx,
                          const int32_t* __restrict__ devs, const int32_t* __restrict__ asgs,
                          const uint32_t* __restrict__ n_ptr, uint32_t cap, const SwStrRef* __restrict__ spans,
                          const uint32_t* __restrict__ after) {
  const uint32_t n = *n_ptr < cap ? *n_ptr : cap;     // generated events: n_gen may pass gen_cap
  const int64_t cur = *a.store_cursor + (after ? (int64_t)*after : 0);   // rows start past `after` rows
  if (idx && BID == 0 && threadIdx.x == 0) {
    // every claim of the step is counted: rotate the dedup generations for the next step when it
    // could push the live table past half load (k_state_p2 clears, k_step_end flips)
    if (a.dd_meta[1] + a.rec_cap > (a.dd_mask + 1) / 2) a.dd_meta[2] = 1;
  }
  uint32_t ff_ids = 0;
  const int64_t c0 = *a.step_cursor0;
  const int64_t now = a.sp->now_ms;
  SwSegAux* const aux = reinterpret_cast<SwSegAux*>(a.sp->aux);
  const int64_t raw_bytes = a.sp->raw_bytes;
  for (int64_t j = (int64_t)BID * BLK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLK) {
    const uint32_t i = idx ? idx[j] : (uint32_t)j;
    const SwEventRec r = R[i];
    const int32_t dev = devs[i], asg = asgs[i];
    const int64_t seq = cur + j;
    const int64_t row = seq % a.store_cap;
    a.s_etype[row] = r.etype;
    a.s_level[row] = r.level;
    a.s_date[row] = r.event_date;
    a.s_recv[row] = now;
    a.s_dev[row] = dev;
    a.s_asg[row] = asg;
    const int4 ctx = *reinterpret_cast<const int4*>(&a.asg_ctx[asg]);
    a.s_cust[row] = ctx.y;
    a.s_area[row] = ctx.z;
    a.s_asset[row] = ctx.w;
    a.s_name[row] = r.name_hash;
    a.s_v0[row] = r.v0;
    a.s_v1[row] = r.v1;
    a.s_v2[row] = r.v2;
    a.s_alt[row] = r.alt_hash;
    a.s_aux[row] = ((ull)r.src_rank << 48) | ((ull)r.aux_len << 32) | (ull)r.aux_off;
    a.s_batch[row] = (int32_t)a.sp->batch_seq;
    SwOutRec o;
    o.event_date = r.event_date;
    o.v0 = r.v0;
    o.v1 = r.v1;
    o.assignment = asg;
    const int64_t ns = r.name_hash ? nm_probe(a.nm_key, a.nm_mask, r.name_hash) : -1;
    const int32_t nid = ns >= 0 ? a.nm_id[ns] : -1;
    o.name_id = (nid >= 0 && nid < 0xffff) ? (uint16_t)nid : (uint16_t)0xffff;
    o.etype = r.etype;
    o.level = r.level;
    a.sp->out[seq - c0] = o;
    if (a.dd_ff && r.alt_hash) ++ff_ids;     // added to the live generation by k_ff_add_rows
    if (aux) {                   // the durable-block encoder's input, beside the row (coalesced)
      SwStrRef sr;
      if (spans) {
        sr = spans[i];
      } else {
        sr.alt_off = 0; sr.meta_off = 0; sr.alt_len = 0; sr.meta_len = 0; sr.k = 0; sr.has = 0; sr.pad = 0;
      }
      aux[seq - c0] = seg_make_aux(r, sr, raw_bytes);
    }
    // ---- state pass 1
    int64_t slot = -1;
    if (r.etype == SW_EV_MEASUREMENT || r.etype == SW_EV_LOCATION || r.etype == SW_EV_ALERT) {
      // Read the 32 B state once; issue an atomic only where it can change something.  Every
      // writer of `last` in this kernel stores the same step time, so a checked plain store gives
      // max(last, now) without an atomic per event.
      SwAsgState* st = &a.st[asg];
      const ulonglong2 lm = *reinterpret_cast<const ulonglong2*>(&st->last);   // last, missing
      if (lm.x < (ull)now) st->last = (ull)now;
      if (lm.y) st->missing = 0;  // presence detected again
      const ull d = (ull)r.event_date;
      if (r.etype == SW_EV_LOCATION) {
        if (d > st->loc_date) atomicMax((ull*)&st->loc_date, d);
      } else if (nid >= 0) {
        // +1 keeps key 0 reserved as empty
        const ull k = ((((ull)(uint32_t)asg) << 32) | ((ull)(uint32_t)nid << 1) | (r.etype == SW_EV_ALERT ? 1ull : 0ull)) + 1ull;
        slot = ms_slot(a.ms, a.ms_mask, k);
        if (slot >= 0) {
          if (d > a.ms[slot].date) atomicMax((ull*)&a.ms[slot].date, d);
        } else {
          atomicAdd((ull*)&a.stats[SW_STAT_STATE_OVERFLOW], 1ull);
        }
      }
    }
    // pass-2 work item, coalesced: (ms slot | -2 - assignment for a location | -1, event date)
    if (r.etype == SW_EV_LOCATION) slot = -2 - (int64_t)asg;
    reinterpret_cast<longlong2*>(a.ev_slot)[j] = make_longlong2(slot, (int64_t)r.event_date);
  }
  if (a.dd_ff) {
    // ids the live generation took (its rotation rule: k_state_p2, k_step_end), one atomic per wave
    const ull w = __ballot(ff_ids != 0);
    if (w) {
      for (int o = 32; o > 0; o >>= 1) ff_ids += __shfl_xor(ff_ids, o);
      if (lane_id() == 0) atomicAdd((ull*)&a.dd_ff_meta[6], (ull)ff_ids);
    }
  }
}

// ============================================================================ device state
// Pass 2: among events carrying the max date, the highest event id wins (ids are monotonic).
// Reads only k_persist's coalesced (slot, date) work items -- no event records, no probes.
__global__ void k_state_p2(SwEngineArgs a, const uint32_t* __restrict__ n_ptr, uint32_t cap,
                           const uint32_t* __restrict__ after) {
  const uint32_t n = *n_ptr < cap ? *n_ptr : cap;
  const int64_t cur = *a.store_cursor + (after ? (int64_t)*after : 0);
  if (!after && a.dd_meta[2] == 1) {
    // dedup rotation decided by k_persist: clear the retiring generation (no reader is left this
    // step: `prev` was probed by the claims in k_lookup); it becomes `cur` when k_step_end flips
    const int64_t slots = a.dd_mask + 1;
    ulonglong2* t = reinterpret_cast<ulonglong2*>(a.dd_key) + (1 - a.dd_meta[0]) * slots;
    for (int64_t i = (int64_t)BID * BLK + threadIdx.x; i < slots; i += (int64_t)gridDim.x * BLK)
      t[i] = make_ulonglong2(0ull, ~0ull);
  }
  // the filter's live generation has taken its ids (k_persist counted them): clear the oldest, which
  // k_step_end makes the live one (the step's generated events carry no alternate id)
  if (!after && a.dd_ff && a.dd_ff_meta[6] >= a.dd_ff_meta[2])
    ff_clear_gen(a.dd_ff, a.dd_ff_bmask, (int)a.dd_ff_gens, (int)((a.dd_ff_meta[0] + 1) % a.dd_ff_gens));
  const longlong2* __restrict__ work = reinterpret_cast<const longlong2*>(a.ev_slot);
  for (int64_t j = (int64_t)BID * BLK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLK) {
    const longlong2 w = work[j];
    if (w.x == -1) continue;
    const ull eid1 = (ull)((cur + j) * a.world + a.rank) + 1ull;  // stored +1, 0 = none
    const ull d = (ull)w.y;
    if (w.x <= -2) {                         // location: assignment -2 - w.x
      SwAsgState* st = &a.st[-2 - w.x];
      const ulonglong2 le = *reinterpret_cast<const ulonglong2*>(&st->loc_date);   // loc_date, loc_eid1
      if (le.x == d && le.y < eid1) atomicMax((ull*)&st->loc_eid1, eid1);
    } else {
      const ulonglong2 de = *reinterpret_cast<const ulonglong2*>(&a.ms[w.x].date);  // date, eid1
      if (de.x == d && de.y < eid1) atomicMax((ull*)&a.ms[w.x].eid1, eid1);
    }
  }
}

// ============================================================================ zone-test rules
#define ZONE_LDS_VTX 2048  // 32 KiB of (lat, lon) doubles
#define ZONE_LDS_TESTS 64

__device__ __forceinline__ bool pip(const double* __restrict__ v, int n, double x, double y) {
  // even-odd crossing number; v = [lat0, lon0, lat1, lon1, ...], x = lat, y = lon.
  // Division-free form of  x < (xj - xi) * (y - yi) / (yj - yi) + xi  (sign of (yj - yi) folded in).
  bool inside = false;
  double xj = v[2 * (n - 1)], yj = v[2 * (n - 1) + 1];
  for (int i = 0; i < n; ++i) {
    const double xi = v[2 * i], yi = v[2 * i + 1];
    if ((yi > y) != (yj > y)) {
      const double lhs = (x - xi) * (yj - yi);
      const double rhs = (xj - xi) * (y - yi);
      if ((yj > yi) ? (lhs < rhs) : (lhs > rhs)) inside = !inside;
    }
    xj = xi; yj = yi;
  }
  return inside;
}

// Same predicate with the division (reference form, for the standalone batch kernel parity).
__device__ __forceinline__ bool pip_div(const double* __restrict__ v, int n, double x, double y) {
  bool inside = false;
  for (int i = 0, j = n - 1; i < n; j = i++) {
    const double xi = v[2 * i], yi = v[2 * i + 1], xj = v[2 * j], yj = v[2 * j + 1];
    if (((yi > y) != (yj > y)) && (x < (xj - xi) * (y - yi) / (yj - yi) + xi)) inside = !inside;
  }
  return inside;
}

struct ZoneLds {
  double bb[4 * ZONE_LDS_TESTS];
  int4 t[ZONE_LDS_TESTS];
  int2 zo[ZONE_LDS_TESTS];
};
// The vertex table lives in dynamic LDS sized to the zones actually configured (16 B per vertex;
// none when it exceeds ZONE_LDS_VTX and the PIP reads global memory): a static 32 KiB table held
// k_zone_mask to 2 workgroups per CU.
extern __shared__ double zone_vtx_lds[];

__host__ __device__ __forceinline__ bool zone_vtx_in_lds(const SwEngineArgs& a) {
  return a.n_zone_vtx <= ZONE_LDS_VTX;
}

__device__ __forceinline__ int zone_lds_load(const SwEngineArgs& a, ZoneLds& L, const double** V) {
  const int nt = a.n_tests < ZONE_LDS_TESTS ? (int)a.n_tests : ZONE_LDS_TESTS;
  const int64_t nv = a.n_zone_vtx;
  const bool in_lds = zone_vtx_in_lds(a);
  for (int64_t t = threadIdx.x; in_lds && t < 2 * nv; t += BLK) zone_vtx_lds[t] = a.zone_vtx[t];
  *V = in_lds ? zone_vtx_lds : a.zone_vtx;
  for (int t = threadIdx.x; t < nt; t += BLK) {
    const SwZoneTest zt = a.tests[t];
    L.t[t] = make_int4(zt.zone, zt.condition, zt.alert_name_id, zt.level);
    L.zo[t] = make_int2(a.zone_off[zt.zone], a.zone_off[zt.zone + 1]);
    for (int q = 0; q < 4; ++q) L.bb[4 * t + q] = a.zone_bbox[4 * zt.zone + q];
  }
  __syncthreads();
  return nt;
}

// Pass 1: per persisted row, the bitmask of zone tests that fire (row-major, test-ascending order is
// the alert order, identical to the CPU oracle); per-tile alert counts.
//
// Block-cooperative so the expensive FP64 point-in-polygon work runs on dense lanes: a thread per
// row would leave ~3/4 of every wave idle (only ~25 % of rows are locations) and run each PIP for
// the whole wave whenever one lane's point falls in a zone's bbox.  Instead the block
//   1. compacts its tile's location rows into LDS (block scan),
//   2. expands (location, test) pairs in rounds, keeping the bbox hits as a dense candidate list,
//   3. runs one candidate PIP per lane and ORs "inside" bits into the row's LDS mask,
//   4. fires = inside ^ outside-condition mask (location rows only), writes zmask + the tile count.
#define ZM_ROUND (BLK * 8)
struct ZoneMaskLds {
  double x[TILE], y[TILE];
  ull inside[TILE];
  uint16_t loc_j[TILE];
  uint32_t cand[ZM_ROUND];
  uint32_t ncand, count;
  uint32_t scan[WAVES + 1];
};

__global__ __launch_bounds__(BLK) void k_zone_mask(SwEngineArgs a, ull* __restrict__ zmask, uint32_t* __restrict__ ztile) {
  __shared__ ZoneLds L;
  __shared__ ZoneMaskLds M;
  const double* V;
  const int nt = zone_lds_load(a, L, &V);
  ull outside_mask = 0;
  for (int t = 0; t < nt; ++t) outside_mask |= (L.t[t].y != 0) ? (1ull << t) : 0ull;
  const int64_t c0 = *a.step_cursor0;
  const uint32_t n = *a.n_ok;              // this step's persisted device events, from c0
  const int64_t base = (int64_t)BID * TILE;
  if (base >= n) {                       // tile past this step's rows
    if (threadIdx.x == 0) ztile[BID] = 0;
    return;
  }
  // 1. compact location rows (stable) into LDS
  bool isloc[TILE_ITEMS];
  uint32_t myloc = 0;
#pragma unroll
  for (int k = 0; k < TILE_ITEMS; ++k) {
    const int64_t j = base + (int64_t)k * BLK + threadIdx.x;
    isloc[k] = false;
    if (j < n) {
      const int64_t row = (c0 + j) % a.store_cap;
      isloc[k] = a.s_etype[row] == SW_EV_LOCATION;
    }
    myloc += isloc[k];
  }
  uint32_t nloc;
  uint32_t pos = block_excl_scan(myloc, &nloc, M.scan);
#pragma unroll
  for (int k = 0; k < TILE_ITEMS; ++k) {
    if (isloc[k]) {
      const int64_t j = base + (int64_t)k * BLK + threadIdx.x;
      const int64_t row = (c0 + j) % a.store_cap;
      M.x[pos] = a.s_v0[row];
      M.y[pos] = a.s_v1[row];
      M.loc_j[pos] = (uint16_t)(k * BLK + threadIdx.x);
      M.inside[pos] = 0;
      ++pos;
    }
  }
  if (threadIdx.x == 0) M.count = 0;
  __syncthreads();
  // 2 + 3. rounds of (location, test) bbox expansion -> dense PIP candidates
  const uint32_t npairs = nloc * (uint32_t)nt;
  for (uint32_t r0 = 0; r0 < npairs; r0 += ZM_ROUND) {
    if (threadIdx.x == 0) M.ncand = 0;
    __syncthreads();
    for (uint32_t p = r0 + threadIdx.x; p < r0 + ZM_ROUND && p < npairs; p += BLK) {
      const uint32_t li = p / (uint32_t)nt, t = p - li * (uint32_t)nt;
      const double* bb = L.bb + 4 * t;
      const double x = M.x[li], y = M.y[li];
      if (x >= bb[0] && y >= bb[1] && x <= bb[2] && y <= bb[3]) M.cand[atomicAdd(&M.ncand, 1u)] = p;
    }
    __syncthreads();
    const uint32_t nc = M.ncand;
    for (uint32_t c = threadIdx.x; c < nc; c += BLK) {
      const uint32_t p = M.cand[c];
      const uint32_t li = p / (uint32_t)nt, t = p - li * (uint32_t)nt;
      if (pip(V + 2 * L.zo[t].x, L.zo[t].y - L.zo[t].x, M.x[li], M.y[li])) atomicOr(&M.inside[li], 1ull << t);
    }
    __syncthreads();
  }
  // 4. fired masks for every row of the tile (0 for non-locations), tile alert count
  for (uint32_t i = threadIdx.x; i < nloc; i += BLK) {
    const ull fired = M.inside[i] ^ outside_mask;
    M.inside[i] = fired;
    if (fired) atomicAdd(&M.count, (uint32_t)__popcll(fired));
  }
  __syncthreads();
  // scatter: default 0, then the location rows' masks
#pragma unroll
  for (int k = 0; k < TILE_ITEMS; ++k) {
    const int64_t j = base + (int64_t)k * BLK + threadIdx.x;
    if (j < n && !isloc[k]) zmask[j] = 0ull;
  }
  for (uint32_t i = threadIdx.x; i < nloc; i += BLK) zmask[base + M.loc_j[i]] = M.inside[i];
  if (threadIdx.x == 0) ztile[BID] = M.count;
}

// Pass 2: write the alerts at their scanned offsets (stable, no global atomics).
// Tile offsets from k_zone_mask's tile counts, reduced in the prologue (no scan dispatch); the last
// tile stores the step's rule alerts as n_gen and, clamped, n_rule -- before k_presence appends to
// n_gen.
__global__ __launch_bounds__(BLK) void k_zone_emit(SwEngineArgs a, const ull* __restrict__ zmask,
                                                   const uint32_t* __restrict__ ztile, uint32_t* __restrict__ n_rule) {
  __shared__ uint32_t lds[WAVES + 1];
  __shared__ int4 lt[ZONE_LDS_TESTS];
  uint32_t run = block_sum_prefix(ztile, BID, lds);
  if (BID == gridDim.x - 1 && threadIdx.x == 0) {
    const uint32_t all = run + ztile[BID];
    *a.n_gen = all;
    *n_rule = all < a.gen_cap ? all : (uint32_t)a.gen_cap;
  }
  const int nt = a.n_tests < ZONE_LDS_TESTS ? (int)a.n_tests : ZONE_LDS_TESTS;
  for (int t = threadIdx.x; t < nt; t += BLK) {
    const SwZoneTest zt = a.tests[t];
    lt[t] = make_int4(zt.zone, zt.condition, zt.alert_name_id, zt.level);
  }
  __syncthreads();
  const int64_t c0 = *a.step_cursor0;
  const uint32_t n = *a.n_ok;              // this step's persisted device events, from c0
  const int64_t base = (int64_t)BID * TILE;
  for (int k = 0; k < TILE_ITEMS; ++k) {
    const int64_t j = base + (int64_t)k * BLK + threadIdx.x;
    ull fired = j < n ? zmask[j] : 0ull;
    const uint32_t cnt = __popcll(fired);
    uint32_t tot;
    uint32_t g = run + block_excl_scan(cnt, &tot, lds);
    if (fired) {
      const int64_t row = (c0 + j) % a.store_cap;
      const int32_t odev = a.s_dev[row], oasg = a.s_asg[row];
      while (fired) {
        const int t = __ffsll(fired) - 1;
        fired &= fired - 1;
        if (g < a.gen_cap) {
          SwEventRec r;
          r.fp_lo = 0; r.fp_hi = 0;
          r.event_date = a.sp->now_ms;  // reference: alert.setEventDate(new Date())
          r.name_hash = a.test_name_hash[t];
          r.v0 = 0; r.v1 = 0; r.v2 = 0; r.alt_hash = 0;
          r.aux_off = (uint32_t)t; r.aux2_off = 0; r.aux_len = 0; r.aux2_len = 0;
          r.etype = SW_EV_ALERT; r.flags = 0; r.src_rank = (uint8_t)a.rank; r.level = (uint8_t)lt[t].w;
          a.gen[g] = r;
          a.gen_dev[g] = odev;
          a.gen_asg[g] = oasg;
        }
        ++g;
      }
    }
    run += tot;
  }
}

// ============================================================================ presence
__global__ void k_presence(SwEngineArgs a) {
  const SwStepParams P = *a.sp;
  if (P.presence_missing_ms <= 0) return;
  const ull limit = (ull)(P.now_ms - P.presence_missing_ms);
  for (int64_t s = (int64_t)BID * BLK + threadIdx.x; s < a.n_asg; s += (int64_t)gridDim.x * BLK) {
    SwAsgState* st = &a.st[s];
    const ull last = st->last;
    const bool miss = last != 0 && last < limit && st->missing == 0 && a.asg_active[s];
    if (!miss) continue;
    st->missing = (ull)P.now_ms;  // send-once strategy
    const uint32_t g = atomicAdd(a.n_gen, 1u);
    if (g < a.gen_cap) {
      SwEventRec r;
      r.fp_lo = 0; r.fp_hi = 0; r.event_date = P.now_ms; r.name_hash = a.presence_name_hash;
      r.v0 = 0; r.v1 = 0; r.v2 = 0; r.alt_hash = 0;
      r.aux_off = 0; r.aux2_off = 0; r.aux_len = 0; r.aux2_len = 0;
      r.etype = SW_EV_STATE_CHANGE; r.flags = 0; r.src_rank = (uint8_t)a.rank; r.level = 0;
      a.gen[g] = r;
      a.gen_dev[g] = a.asg_ctx[s].device;
      a.gen_asg[g] = (int32_t)s;
    }
  }
}

// ============================================================================ step bookkeeping
// Decode-side and process-side resets are separate kernels: with the pipelined exchange the
// decode of batch k runs before the process phase of batch k-1 on the same stream.
__global__ void k_decode_begin(SwEngineArgs a) {
  if (threadIdx.x == 0 && BID == 0) {
    *a.n_new_names = 0;
    *a.overflow = 0;
    ((ull*)a.stats)[SW_STAT_MSGS] += (ull)a.n_msgs;   // by-value batch size
  }
}

__global__ void k_gen_clamp(SwEngineArgs a, uint32_t* gen_rules) {
  if (threadIdx.x == 0 && BID == 0) {
    if (*a.n_gen > a.gen_cap) *a.n_gen = (uint32_t)a.gen_cap;
    if (gen_rules) *gen_rules = *a.n_gen;
  }
}

__global__ void k_step_end(SwEngineArgs a, const uint32_t* n_rule_alerts) {
  if (threadIdx.x == 0 && BID == 0) {
    if (*a.n_gen > a.gen_cap) *a.n_gen = (uint32_t)a.gen_cap;   // presence appends past the cap were dropped
    *a.store_cursor += (int64_t)*a.n_ok + *a.n_gen;   // device events, then the generated ones
    *a.n_out = (uint32_t)(*a.store_cursor - *a.step_cursor0);
    *a.seq_base += *a.n_work;
    ull* st = (ull*)a.stats;
    st[SW_STAT_EVENTS] += *a.n_work;
    st[SW_STAT_PERSISTED] += *a.n_out;
    st[SW_STAT_RULE_ALERTS] += *n_rule_alerts;
    st[SW_STAT_PRESENCE] += *a.n_gen - *n_rule_alerts;
    // dedup rotation decided and cleared this step: flip the generations (the next step's
    // k_lookup counts it)
    int64_t* meta = a.dd_meta;
    if (meta[2] == 1) {
      meta[0] ^= 1;
      meta[1] = 0;
      meta[2] = 2;
    }
    meta[3] = 0;
    if (a.dd_ff && a.dd_ff_meta[6] >= a.dd_ff_meta[2]) {
      int64_t* fm = a.dd_ff_meta;
      fm[0] = (fm[0] + 1) % a.dd_ff_gens;
      fm[SW_FF_META + fm[0]] = *a.store_cursor;
      fm[6] = 0;
      fm[4] += 1;
    }
  }
}

// ============================================================================ C ABI
// ============================================================================ hot-store query
// Event-management reads over the HBM event ring (DeviceEventManagement.list*ForIndex,
// EventManagementImpl.java): rows of one event type whose assignment is in a bitmap and whose
// event date lies in [lo, hi].  One pass over the ring: the 1-byte type column is read for every
// row, assignment and date only where the type matches.  Matches are compacted per wave (ballot +
// one atomic per wave that has any) into out_rows -- unordered; the host orders the (usually small)
// match set by (date desc, event id desc).  *n_match receives the total even past cap.
__global__ __launch_bounds__(BLK) void k_store_filter(const uint8_t* __restrict__ etype, const int32_t* __restrict__ asg,
                                                      const int64_t* __restrict__ date, int64_t n_rows, int32_t et,
                                                      const uint32_t* __restrict__ bits, int64_t n_asg, int64_t lo,
                                                      int64_t hi, uint32_t* __restrict__ out_rows, int64_t cap,
                                                      uint32_t* __restrict__ n_match) {
  const int64_t stride = (int64_t)gridDim.x * BLK;
  // every lane of a wave iterates the same number of times (ballot needs the whole wave)
  const int64_t iters = (n_rows + stride - 1) / stride;
  int64_t r = (int64_t)BID * BLK + threadIdx.x;
  for (int64_t it = 0; it < iters; ++it, r += stride) {
    bool hit = false;
    if (r < n_rows && etype[r] == (uint8_t)et) {
      const int32_t a = asg[r];
      if (a >= 0 && a < n_asg && ((bits[a >> 5] >> (a & 31)) & 1u)) {
        const int64_t d = date[r];
        hit = d >= lo && d <= hi;
      }
    }
    const ull mask = __ballot(hit);
    if (!mask) continue;
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(n_match, (uint32_t)__popcll(mask));
    base = __shfl(base, 0, 64);
    if (hit) {
      const uint64_t pos = (uint64_t)base + (uint64_t)__popcll(mask & lanemask_lt());
      if ((int64_t)pos < cap) out_rows[pos] = (uint32_t)r;
    }
  }
}

// ============================================================================ reject refs
// Snapshot of a step's rejected events for the host slow path, taken on the compute stream right
// after the process phase (the next step overwrites the reject list).  Duplicates are dropped here
// (dedup discards them).  Every other reject of a locally received payload gets a ref
//   (payload start in the batch, payload end, status | src_rank << 8, offset of its copy)
// and the payload bytes are copied into a compact buffer, so only those bytes cross PCIe and the
// host parses them sequentially (csrc/native/swroute.cpp), never the scattered raw batch.
// out = u32[8] device counters: out[0] = refs (may exceed cap), out[1] = bytes used (may exceed
// bytes_cap: such refs carry copy offset ~0 and the host reads the raw record instead); out[4..6]
// are the kernel's own accumulators and done count, which the last workgroup publishes to out[0..1]
// and zeroes for the next launch (no memset before each snapshot; the allocation starts zeroed).  `refs`
// (u32[4 * cap]) and `bytes` are usually mapped pinned host memory: written straight over PCIe, no
// copy call.  Refs are in any order; events decoded on another rank keep start = end = 0.
//
// Several ranks with strings exchanged (wstr != null): a recheck is settled by its owner by
// alternate id (pipeline/recheck.py), whatever rank decoded it, so instead of its payload the copy
// holds a recheck package -- the 80-byte record, its SwStrRef and its strings (alternate id,
// metadata, alert message) back to back, string offsets relative to the strings' start (the layout
// of recheck.compact_strings) -- and the ref is (0, package bytes, status | src_rank << 8 |
// SW_REF_PACKED, offset of the package).
#define SW_REF_PACKED 0x10000u
__global__ void k_reject_refs(const SwEventRec* __restrict__ work, const uint32_t* __restrict__ rej_idx,
                              const uint32_t* __restrict__ n_rej_ptr, const uint8_t* __restrict__ status,
                              const uint8_t* __restrict__ raw, const uint32_t* __restrict__ msg_off, int64_t n_msgs,
                              int rank, uint32_t* __restrict__ out, uint32_t* __restrict__ refs, int64_t cap,
                              uint8_t* __restrict__ bytes, int64_t bytes_cap, const SwStrRef* __restrict__ wsp,
                              const uint8_t* __restrict__ wstr) {
  __shared__ uint32_t last;
  const uint32_t n = *n_rej_ptr;
  uint32_t* acc = out + 4;
  for (int64_t j = (int64_t)BID * BLK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLK) {
    const uint32_t i = rej_idx[j];
    const uint8_t st = status[i];
    if (st == SW_ST_DUPLICATE) continue;
    const SwEventRec& r = work[i];
    uint32_t s = 0, e = 0, copy = 0xffffffffu, packed = 0u;
    if (st == SW_ST_RECHECK && wstr != nullptr) {
      const SwStrRef sp = wsp[i];
      const uint32_t al = (sp.has & SW_SR_ALT) ? sp.alt_len : 0u;
      const uint32_t ml = (sp.has & SW_SR_META) ? sp.meta_len : 0u;
      const uint32_t gl = r.etype == SW_EV_ALERT ? r.aux2_len : 0u;
      const uint32_t sl = al + ml + gl;
      const uint32_t len = (uint32_t)(sizeof(SwEventRec) + sizeof(SwStrRef)) + sl;
      const uint32_t at = atomicAdd(acc + 1, len);
      packed = SW_REF_PACKED;
      e = len;
      if ((int64_t)at + len <= bytes_cap) {
        SwEventRec c = r;
        if (r.etype == SW_EV_ALERT) c.aux2_off = gl ? al + ml : 0u;
        SwStrRef o = sp;
        o.alt_off = 0u;
        o.meta_off = sl ? al : 0u;
        o.alt_len = (uint16_t)al;
        o.meta_len = (uint16_t)ml;
        if (!sl) o.has = sp.has & SW_SR_MULTI;
        const uint8_t* cb = reinterpret_cast<const uint8_t*>(&c);
        const uint8_t* ob = reinterpret_cast<const uint8_t*>(&o);
        uint8_t* d = bytes + at;
        for (uint32_t b = 0; b < sizeof(SwEventRec); ++b) d[b] = cb[b];
        d += sizeof(SwEventRec);
        for (uint32_t b = 0; b < sizeof(SwStrRef); ++b) d[b] = ob[b];
        d += sizeof(SwStrRef);
        for (uint32_t b = 0; b < al; ++b) d[b] = wstr[sp.alt_off + b];
        for (uint32_t b = 0; b < ml; ++b) d[al + b] = wstr[sp.meta_off + b];
        for (uint32_t b = 0; b < gl; ++b) d[al + ml + b] = wstr[r.aux2_off + b];
        copy = at;
      }
    } else if (r.src_rank == (uint8_t)rank && n_msgs > 0) {
      int64_t lo = 0, hi = n_msgs;              // msg_off[lo] <= off < msg_off[hi]
      const uint32_t off = r.aux_off;
      while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (msg_off[mid] <= off) lo = mid; else hi = mid;
      }
      s = msg_off[lo];
      e = msg_off[lo + 1];
      const uint32_t len = e > s ? e - s : 0u;
      const uint32_t at = atomicAdd(acc + 1, len);
      if ((int64_t)at + len <= bytes_cap) {
        for (uint32_t b = 0; b < len; ++b) bytes[at + b] = raw[s + b];
        copy = at;
      }
    }
    const uint32_t k = atomicAdd(acc, 1u);
    if (k < cap) {
      refs[4 * k] = s;
      refs[4 * k + 1] = e;
      refs[4 * k + 2] = (uint32_t)st | ((uint32_t)r.src_rank << 8) | packed;
      refs[4 * k + 3] = copy;
    }
  }
  // last workgroup out: publish the counters (device-scope atomics, visible without a release fence)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(acc + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (last && threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    out[0] = __hip_atomic_load(acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    out[1] = __hip_atomic_load(acc + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int w = 0; w < 3; ++w) __hip_atomic_store(acc + w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

extern "C" {

int sw_reject_refs(const SwEngineArgs* ap, const uint8_t* raw, const uint32_t* msg_off, int64_t n_msgs, uint32_t* out,
                   uint32_t* refs, int64_t cap, uint8_t* bytes, int64_t bytes_cap, hipStream_t s) {
  const SwEngineArgs a = *ap;
  // rejects are a small share of a step: a small grid keeps the last-workgroup count (one atomic
  // per workgroup on one word) off the critical path
  const int g = grid_for(a.rec_cap) < 256 ? grid_for(a.rec_cap) : 256;
  k_reject_refs<<<g, BLK, 0, s>>>(a.work, a.rej_idx, a.n_rej, a.status, raw, msg_off, n_msgs,
                                  (int)a.rank, out, refs, cap, bytes, bytes_cap,
                                  a.world > 1 ? a.work_spans : nullptr, a.world > 1 ? a.work_str : nullptr);
  return (int)hipGetLastError();
}

// End-of-step snapshot into mapped host memory (one launch instead of one copy per value): the
// step's u32 scalars (n_out at [7], n_rej at [5]) -> host[0..15]; the durable-block encoder's
// (bytes, errors, first sequence) u64s -> host[16..21]; the reject-ref counters -> host[24..25].
__global__ void k_step_snapshot(const uint32_t* __restrict__ scalars, const uint32_t* __restrict__ seg_meta,
                                const uint32_t* __restrict__ rej_cnt, const uint32_t* __restrict__ n_carry,
                                int produced, uint32_t* __restrict__ host) {
  const uint32_t t = threadIdx.x;
  if (t < 16) host[t] = produced ? scalars[t] : 0u;
  else if (t < 22) host[t] = (produced && seg_meta) ? seg_meta[t - 16] : 0u;
  else if (t == 22 || t == 23) host[t] = n_carry ? n_carry[t - 22] : 0u;     // re-key carry (both parities)
  else if (t == 24 || t == 25) host[t] = (produced && rej_cnt) ? rej_cnt[t - 24] : 0u;
}

// The step's rejected records (SwEventRec, 80 B) and their statuses, gathered by rej_idx straight
// into mapped host memory, bounded by the step's own reject count (scalars[5], read on the device) and
// `cap`: the host reads them after the step's event, with no copy call and no synchronising read of
// the count first (GpuInboundEngine.submit_framed).
__global__ __launch_bounds__(256) void k_reject_pack(const uint4* __restrict__ recs, const int32_t* __restrict__ rej_idx,
                                                      const uint8_t* __restrict__ status,
                                                      const uint32_t* __restrict__ scalars, uint32_t cap,
                                                      uint4* __restrict__ out, uint8_t* __restrict__ out_st) {
  const uint32_t n = scalars[5] < cap ? scalars[5] : cap;
  const uint32_t words = 5;                     // sizeof(SwEventRec) / 16
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < n * words; w += gridDim.x * blockDim.x) {
    const uint32_t i = w / words, q = w - i * words;
    const int32_t r = rej_idx[i];
    out[w] = recs[(int64_t)r * words + q];
    if (q == 0) out_st[i] = status[r];
  }
}

int sw_reject_pack(const void* recs, const int32_t* rej_idx, const uint8_t* status, const uint32_t* scalars,
                   int64_t cap, void* out, uint8_t* out_st, hipStream_t s) {
  static_assert(sizeof(SwEventRec) == 80, "k_reject_pack copies 5 x 16 B per record");
  if (cap <= 0 || cap > 0xffffffffll / 5) return -1;
  k_reject_pack<<<512, 256, 0, s>>>(reinterpret_cast<const uint4*>(recs), rej_idx, status, scalars, (uint32_t)cap,
                                    reinterpret_cast<uint4*>(out), out_st);
  return (int)hipGetLastError();
}

// Stream / event / copy enqueues for the tenant's submit path, bound without releasing the GIL
// (sitewhere_amd/_native.py _GilBound): torch's equivalents give the interpreter lock up on every
// call and wait to win it back from the tenant's other threads (~0.2 ms each at the instance's
// switch interval, ~1 ms per step over the H2D's five calls -- profiles/r6_soak).
int sw_stream_wait_event(hipStream_t s, hipEvent_t e) { return (int)hipStreamWaitEvent(s, e, 0); }
int sw_event_record(hipEvent_t e, hipStream_t s) { return (int)hipEventRecord(e, s); }
int sw_memcpy_h2d_async(void* dst, const void* src, int64_t n, hipStream_t s) {
  return n > 0 ? (int)hipMemcpyAsync(dst, src, (size_t)n, hipMemcpyHostToDevice, s) : 0;
}
int sw_memset_async(void* dst, int32_t v, int64_t n, hipStream_t s) {
  return n > 0 ? (int)hipMemsetAsync(dst, v, (size_t)n, s) : 0;
}

int sw_step_snapshot(const uint32_t* scalars, const uint32_t* seg_meta, const uint32_t* rej_cnt,
                     const uint32_t* n_carry, int32_t produced, uint32_t* host, hipStream_t s) {
  k_step_snapshot<<<1, 64, 0, s>>>(scalars, seg_meta, rej_cnt, n_carry, produced, host);
  return (int)hipGetLastError();
}

// Framing: varint length stream -> msg_off[n_msgs + 1].  tmp needs 2 * ceil(nbytes / 1024) u32.
int sw_frame_varint(const uint8_t* lens, int64_t nbytes, int64_t n_msgs, uint32_t* msg_off, uint32_t raw_bytes,
                    uint32_t* tmp, int64_t tmp_len, hipStream_t s) {
  int64_t nt = (nbytes + TILE - 1) / TILE;
  if (nt < 1) nt = 1;
  if (2 * nt > tmp_len) return -2;
  if (nbytes <= 0 || n_msgs <= 0) return (int)hipMemsetAsync(msg_off, 0, sizeof(uint32_t) * (n_msgs + 1), s);
  uint32_t* tcnt = tmp;
  uint32_t* tlen = tmp + nt;
  k_vlen_tiles<<<(unsigned)nt, BLK, 0, s>>>(lens, nbytes, tcnt, tlen);
  k_vlen_apply<<<(unsigned)nt, BLK, 0, s>>>(lens, nbytes, tcnt, tlen, msg_off, n_msgs, raw_bytes);
  return (int)hipGetLastError();
}

// Phase A: decode the raw batch into records (+ new-name capture).  msg counts are host-known.
int sw_phase_decode(const SwEngineArgs* ap, hipStream_t s) {
  const SwEngineArgs a = *ap;
  if (a.n_msgs <= 0) {
    k_decode_begin<<<1, 64, 0, s>>>(a);
    (void)hipMemsetAsync(a.n_recs, 0, sizeof(uint32_t), s);
    return (int)hipGetLastError();
  }
  const unsigned nb = (unsigned)((a.n_msgs + BLK - 1) / BLK);
  k_decode_count<<<nb, BLK, 0, s>>>(a.raw, a.msg_off, a.n_msgs, a.msg_cnt, a.msg_evoff, a);   // + phase resets
  k_decode_emit<<<nb, BLK, 0, s>>>(a);
  if (a.world > 1) k_decode_end<<<1, 64, 0, s>>>(a);     // world == 1: k_lookup does it
  return (int)hipGetLastError();
}

// Phase B (world > 1): stable partition of records into per-owner send slabs.
int sw_phase_partition(const SwEngineArgs* ap, hipStream_t s) {
  const SwEngineArgs a = *ap;
  const int64_t ntiles = (a.carry_cap + a.rec_cap + TILE - 1) / TILE;
  if (a.world > 64 || ntiles * a.world > a.part_tmp_len || !a.carry || !a.n_carry || !a.spill || !a.n_spill ||
      a.carry == a.spill || !a.part_owner || !a.part_bytes || !a.part_meta || ntiles >= 0x7fffffff)
    return -3;
  if (a.send_str && (!a.part_len || !a.carry_spans || !a.carry_str || !a.spill_spans || !a.spill_str ||
                     a.carry_str == a.spill_str || a.carry_str_cap <= 0 || a.carry_str_cap > 0xffffffffll ||
                     a.str_cap > 0x7fffffffll))
    return -4;
  k_part_count<<<(unsigned)ntiles, BLK, 0, s>>>(a.carry, a.n_carry, a.recs, a.n_recs, (int)a.world, (int)a.rank,
                                                a.part_tmp, ntiles, a);
  // scan the flat [world][ntiles] count matrix in place
  int rc = launch_scan(a.part_tmp, ntiles * a.world, a.part_tmp + ntiles * a.world, nullptr, a.scan_tmp,
                       a.scan_tmp_len, s);
  if (rc) return rc;
  const uint32_t* toff = a.part_tmp + ntiles * a.world;
  k_part_cut<<<(unsigned)a.world, BLK, 0, s>>>(toff, a.part_tmp, ntiles, a.n_carry, a.n_recs, a);
  k_part_write<<<(unsigned)ntiles, BLK, 0, s>>>(a.carry, a.n_carry, a.recs, a.n_recs, (int)a.world, (int)a.rank, toff,
                                                a.part_tmp, ntiles, a.send, a.shuf_cap, a.spill, a.carry_cap, a);
  k_part_counts<<<1, 64, 0, s>>>(toff, a.part_tmp, ntiles, (int)a.world, a);
  return (int)hipGetLastError();
}

// Phase C (world > 1): concatenate received slabs into the work batch.
int sw_phase_unpack(const SwEngineArgs* ap, hipStream_t s) {
  const SwEngineArgs a = *ap;
  if (a.work_str && (a.str_cap & 15)) return -5;      // 16-byte slab copies
  k_unpack<<<grid_for(a.rec_cap), BLK, 0, s>>>(a.recv, a.recv_cnt, (int)a.world, a.shuf_cap, a.work, a.n_work,
                                               a.rec_cap, a);
  return (int)hipGetLastError();
}

// (assignment, ok index) pairs of the validated events, for the clustering sort
__global__ void k_cl_prep(const uint32_t* __restrict__ ok_idx, const uint32_t* __restrict__ n_ok,
                          const int32_t* __restrict__ ev_asg, uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const uint32_t n = *n_ok;
  for (int64_t j = (int64_t)BID * BLK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLK) {
    const uint32_t i = ok_idx[j];
    keys[j] = (uint32_t)ev_asg[i];
    vals[j] = i;
  }
}

int sw_radix_sort_u32(uint32_t* keys, uint32_t* vals, const uint32_t* n_ptr, int64_t cap, int bits, uint32_t* hist,
                      uint32_t* vals_final, hipStream_t s);

__global__ __launch_bounds__(BLK) void k_ff_add_rows(SwEngineArgs a, const SwEventRec* __restrict__ R,
                                                     const uint32_t* __restrict__ idx,
                                                     const uint32_t* __restrict__ n_ptr, uint32_t cap);

// Phase D: validate, dedup, persist, enrich, state, rules, presence.
int sw_phase_process(const SwEngineArgs* ap, uint32_t* scratch4, hipStream_t s) {
  const SwEngineArgs a = *ap;
  const int g = grid_for(a.rec_cap);
  const int64_t ntiles = (a.rec_cap + TILE - 1) / TILE;
  if (2 * ntiles > a.scan_tmp_len) return -4;
  if (a.dd_ff && (a.dd_ff_gens < 2 || a.dd_ff_gens > SW_FF_MAX_GENS || !a.dd_ff_meta || a.dd_ff_bmask < 0))
    return -6;
  k_lookup<<<g, BLK, 0, s>>>(a);         // + the phase's resets (block 0)
  if (a.dd_ff) k_ff_probe<<<g, BLK, 0, s>>>(a);
  k_dedup_claim<<<g, BLK, 0, s>>>(a);
  // stable split ok / rejected, with the dedup verdicts
  k_cmp_count<<<(unsigned)ntiles, BLK, 0, s>>>(a.status, a.n_work, a.cmp_tmp, ntiles, (ull*)a.stats, a.work,
                                               (const ull*)a.dd_key, a.dd_mask, a.seq_base, a.dd_meta,
                                               a.dd_ff, a.dd_ff_bmask, (int)a.dd_ff_gens, a.work_str ? -1 : (int)a.rank);
  k_cmp_write<<<(unsigned)ntiles, BLK, 0, s>>>(a.status, a.n_work, a.cmp_tmp, ntiles, a.ok_idx, a.rej_idx, a.n_ok,
                                               a.n_rej);
  int rc = 0;
  if (a.cl_bits > 0) {
    // persist order: stable by assignment (the durable block's clustering, swindex.h)
    k_cl_prep<<<g, BLK, 0, s>>>(a.ok_idx, a.n_ok, a.ev_asg, a.cl_keys, a.cl_vals);
    rc = sw_radix_sort_u32(a.cl_keys, a.cl_vals, a.n_ok, a.rec_cap, (int)a.cl_bits, a.cl_hist, a.ok_idx, s);
    if (rc < 0) return rc;
  }
  // persist + enrich + state for the validated events
  // string refs of the work batch: the decoder's (one rank) or the exchange's (rebased into work_str)
  const SwStrRef* wsp = a.world > 1 ? a.work_spans : a.spans;
  k_persist<<<g, BLK, 0, s>>>(a, a.work, a.ok_idx, a.ev_dev, a.ev_asg, a.n_ok, (uint32_t)a.rec_cap, wsp, nullptr);
  if (a.dd_ff) k_ff_add_rows<<<g, BLK, 0, s>>>(a, a.work, a.ok_idx, a.n_ok, (uint32_t)a.rec_cap);
  k_state_p2<<<g, BLK, 0, s>>>(a, a.n_ok, (uint32_t)a.rec_cap, nullptr);
  // rules on this step's persisted locations, then presence scan; generated events persist too
  uint32_t* n_rule = scratch4;
  if (a.n_tests > 0) {
    const int64_t otiles = (a.rec_cap + TILE - 1) / TILE;
    ull* zmask = (ull*)a.zmask;
    uint32_t* ztile = a.ztile;
    const size_t vtx_bytes = zone_vtx_in_lds(a) ? (size_t)a.n_zone_vtx * 2 * sizeof(double) : 0;
    k_zone_mask<<<(unsigned)otiles, BLK, vtx_bytes, s>>>(a, zmask, ztile);
    k_zone_emit<<<(unsigned)otiles, BLK, 0, s>>>(a, zmask, ztile, n_rule);
  } else {
    k_gen_clamp<<<1, 64, 0, s>>>(a, n_rule);        // no zone tests: n_rule = n_gen = 0
  }
  k_presence<<<grid_for(a.n_asg), BLK, 0, s>>>(a);   // exits at once when presence is off this step
  // consumers of the generated events clamp n_gen to gen_cap themselves; k_step_end stores it
  const int gg = grid_for(a.gen_cap);
  const uint32_t gcap = (uint32_t)a.gen_cap;
  k_intern_insert_list<<<gg, BLK, 0, s>>>(a.gen, a.n_gen, (ull*)a.nm_key, a.nm_id, a.nm_counter, a.nm_mask, gcap);
  // generated events persist after the step's device events (store cursor + n_ok)
  k_persist<<<gg, BLK, 0, s>>>(a, a.gen, nullptr, a.gen_dev, a.gen_asg, a.n_gen, gcap, nullptr, a.n_ok);
  if (a.dd_ff) k_ff_add_rows<<<gg, BLK, 0, s>>>(a, a.gen, nullptr, a.n_gen, gcap);
  k_state_p2<<<gg, BLK, 0, s>>>(a, a.n_gen, gcap, a.n_ok);
  k_step_end<<<1, 64, 0, s>>>(a, n_rule);
  return (int)hipGetLastError();
}

__global__ void k_set_step_params(SwStepParams* sp, int64_t now_ms, int64_t batch_seq, int64_t presence_ms,
                                  SwOutRec* out, void* aux, int64_t raw_bytes) {
  if (threadIdx.x == 0 && BID == 0) {
    sp->now_ms = now_ms; sp->batch_seq = batch_seq; sp->presence_missing_ms = presence_ms; sp->out = out;
    sp->aux = aux; sp->raw_bytes = raw_bytes;
  }
}

// Add ids to generation g of the store-backed dedup filter (warm start from the event store's
// blocks, newest first; see EngineBase.filter_seed).
// The persisted rows' ids into the live generation of the store-backed filter, right behind
// k_persist: 4 lanes per id, lane q loading 16-byte word q of the id's 64-byte bucket (one full-line
// load per id instead of four 16-byte loads by one thread), a hit anywhere ends the id, else the lowest
// lane holding a free slot claims it with one CAS (another id winning the slot: the group looks
// again); a full bucket sends the id on to the next.  The bucket rule of ff_add.
__global__ __launch_bounds__(BLK) void k_ff_add_rows(SwEngineArgs a, const SwEventRec* __restrict__ R,
                                                     const uint32_t* __restrict__ idx,
                                                     const uint32_t* __restrict__ n_ptr, uint32_t cap) {
  if (!a.dd_ff) return;
  const uint32_t n = *n_ptr < cap ? *n_ptr : cap;
  uint32_t* __restrict__ t = a.dd_ff;
  const int gens = (int)a.dd_ff_gens, g = (int)a.dd_ff_meta[0];
  const int64_t bmask = a.dd_ff_bmask;
  const uint32_t lane = threadIdx.x & 63u, sub = lane & 3u, grp = lane >> 2;   // 16 ids per wave
  const ull gmask = 0xfull << (4u * grp);
  const int64_t g0 = ((int64_t)BID * BLK + threadIdx.x) >> 2;
  const int64_t gstride = ((int64_t)gridDim.x * BLK) >> 2;
  uint32_t dropped = 0;
  for (int64_t base = g0 - grp; base < (int64_t)n; base += gstride) {
    const int64_t j = base + grp;
    ull h = 0ull;
    if (j < (int64_t)n) h = R[idx ? idx[j] : (uint32_t)j].alt_hash;
    const ull m = sw_ff_mix(h);
    const uint32_t fp = sw_ff_fp(m);
    int64_t b = (int64_t)sw_ff_bucket(m, bmask);
    bool pending = h != 0ull;
    for (int p = 0; p < 2 * SW_FF_MAX_PROBE && __any(pending); ++p) {
      uint32_t* sl = t + (b * gens + g) * SW_FF_SLOTS;
      uint4 v = make_uint4(1u, 1u, 1u, 1u);
      if (pending) v = reinterpret_cast<const uint4*>(sl)[sub];
      const bool hit = pending && (v.x == fp || v.y == fp || v.z == fp || v.w == fp);
      if (__ballot(hit) & gmask) pending = false;
      const bool zero = pending && (!v.x || !v.y || !v.z || !v.w);
      const ull zb = __ballot(zero) & gmask;
      bool ok = false;
      if (pending && zb && lane == (uint32_t)(__ffsll((long long)zb) - 1)) {
        const int k = !v.x ? 0 : !v.y ? 1 : !v.z ? 2 : 3;
        const uint32_t old = atomicCAS(&sl[4u * sub + (uint32_t)k], 0u, fp);
        ok = old == 0u || old == fp;
      }
      if (__ballot(ok) & gmask) pending = false;
      else if (pending && !zb) b = (b + 1) & bmask;   // full without the id: the chain goes on
    }
    if (pending && sub == 0u) ++dropped;
  }
  if (dropped) atomicAdd((ull*)&a.dd_ff_meta[5], (ull)dropped);
}

__global__ void k_ff_add(uint32_t* t, int64_t bmask, int gens, int g, int64_t* meta, const ull* __restrict__ h,
                         int64_t n) {
  uint32_t dropped = 0;
  for (int64_t i = (int64_t)BID * BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK)
    if (h[i] && !ff_add(t, bmask, gens, g, h[i])) ++dropped;
  if (dropped) atomicAdd((ull*)&meta[5], (ull)dropped);
}

__global__ void k_ff_clear(uint32_t* t, int64_t bmask, int gens, int g) { ff_clear_gen(t, bmask, gens, g); }

int sw_ff_add(void* tab, int64_t bmask, int64_t gens, int64_t gen, void* meta, const void* hashes, int64_t n,
              hipStream_t s) {
  if (n <= 0) return 0;
  if (gens < 2 || gens > SW_FF_MAX_GENS || gen < 0 || gen >= gens) return -2;
  const int64_t g = (n + BLK - 1) / BLK;
  k_ff_add<<<(unsigned)(g < 4096 ? g : 4096), BLK, 0, s>>>((uint32_t*)tab, bmask, (int)gens, (int)gen,
                                                          (int64_t*)meta, (const ull*)hashes, n);
  return (int)hipGetLastError();
}

// Clear generation g (host-driven rotation while seeding; in the step it is k_state_p2's).
int sw_ff_clear(void* tab, int64_t bmask, int64_t gens, int64_t g, hipStream_t s) {
  if (gens < 2 || gens > SW_FF_MAX_GENS || g < 0 || g >= gens) return -2;
  const int64_t nb = (bmask + 1) * 4;
  const int64_t gr = (nb + BLK - 1) / BLK;
  k_ff_clear<<<(unsigned)(gr < 8192 ? gr : 8192), BLK, 0, s>>>((uint32_t*)tab, bmask, (int)gens, (int)g);
  return (int)hipGetLastError();
}

// Stream-ordered write of this step's params (before the decode / process phases of the step).
// aux: SwSegAux per row for the durable-block encoder (null: not encoding); raw_bytes: the bound of
// the batch's strings (0 when rows carry none).
int sw_set_step_params(SwStepParams* sp, int64_t now_ms, int64_t batch_seq, int64_t presence_ms, void* out,
                       void* aux, int64_t raw_bytes, hipStream_t s) {
  k_set_step_params<<<1, 64, 0, s>>>(sp, now_ms, batch_seq, presence_ms, (SwOutRec*)out, aux, raw_bytes);
  return (int)hipGetLastError();
}

// hipGraph of the process phase (unpack when world > 1, then ~30 kernels + scans): captured once per
// engine configuration, replayed every step -- one launch instead of ~35 from the host.
int sw_graph_capture_process(const SwEngineArgs* ap, uint32_t* scratch4, int32_t with_unpack, hipStream_t s,
                             void** exec_out) {
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) return 5000 + (int)e;
  int rc = 0;
  if (with_unpack) rc = sw_phase_unpack(ap, s);
  if (!rc) rc = sw_phase_process(ap, scratch4, s);
  e = hipStreamEndCapture(s, &g);
  if (rc) { if (g) (void)hipGraphDestroy(g); return rc; }
  if (e != hipSuccess) return 6000 + (int)e;
  hipGraphExec_t x = nullptr;
  e = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) return 7000 + (int)e;
  *exec_out = (void*)x;
  return 0;
}

int sw_graph_launch(void* exec, hipStream_t s) { return (int)hipGraphLaunch((hipGraphExec_t)exec, s); }

int sw_graph_destroy(void* exec) { return exec ? (int)hipGraphExecDestroy((hipGraphExec_t)exec) : 0; }

// Registry patch: scatter host-built packed slots (bulk load and incremental upserts).
__global__ void k_reg_patch(SwRegSlot* reg, const int64_t* slots, const SwRegSlot* vals, int64_t n) {
  for (int64_t i = (int64_t)BID * BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK) reg[slots[i]] = vals[i];
}

int sw_registry_patch(SwRegSlot* reg, const int64_t* slots, const SwRegSlot* vals, int64_t n, hipStream_t s) {
  if (n <= 0) return 0;
  k_reg_patch<<<grid_for(n), BLK, 0, s>>>(reg, slots, vals, n);
  return (int)hipGetLastError();
}

// Per-assignment device-state lookup: one thread per candidate (name id, kind) probes the state map
// read-only for its (assignment, name, kind) key.  Name ids are dense (claim-time counter), so the
// candidates are 2 x names -- a few thousand probes instead of a pass over all state_slots (GBs at
// bench sizing).  Hits are appended to `out` (at most 2 x n_ids rows).
__global__ void k_state_lookup(const SwMsSlot* __restrict__ ms, int64_t mask, int32_t asg, int32_t n_ids,
                               SwMsSlot* __restrict__ out, uint32_t* __restrict__ n_out) {
  for (int64_t i = (int64_t)BID * BLK + threadIdx.x; i < 2 * (int64_t)n_ids; i += (int64_t)gridDim.x * BLK) {
    const ull k = ((((ull)(uint32_t)asg) << 32) | ((ull)(uint32_t)(i >> 1) << 1) | (ull)(i & 1)) + 1ull;
    int64_t slot = (int64_t)(sw_mix64(k) & (ull)mask);
    for (int64_t p = 0; p <= mask && p < MAX_PROBE; ++p) {
      const ull kk = ms[slot].key;
      if (kk == k) { out[atomicAdd(n_out, 1u)] = ms[slot]; break; }
      if (kk == 0) break;
      slot = (slot + 1) & mask;
    }
  }
}

// Standalone batched point-in-polygon (used by the rule service for ad-hoc zone queries).
__global__ void k_pip_batch(const double* pts, int64_t n_pts, const double* vtx, const int32_t* off, int64_t n_zones,
                            uint8_t* out) {
  for (int64_t i = (int64_t)BID * BLK + threadIdx.x; i < n_pts * n_zones; i += (int64_t)gridDim.x * BLK) {
    const int64_t p = i / n_zones, z = i % n_zones;
    out[i] = pip(vtx + 2 * off[z], off[z + 1] - off[z], pts[2 * p], pts[2 * p + 1]) ? 1 : 0;
  }
}

int sw_store_filter(const uint8_t* etype, const int32_t* asg, const int64_t* date, int64_t n_rows, int32_t et,
                    const uint32_t* bits, int64_t n_asg, int64_t lo, int64_t hi, uint32_t* out_rows, int64_t cap,
                    uint32_t* n_match, hipStream_t s) {
  hipError_t e = hipMemsetAsync(n_match, 0, sizeof(uint32_t), s);
  if (e != hipSuccess) return (int)e;
  if (n_rows > 0)
    k_store_filter<<<grid_for(n_rows), BLK, 0, s>>>(etype, asg, date, n_rows, et, bits, n_asg, lo, hi, out_rows, cap,
                                                    n_match);
  return (int)hipGetLastError();
}

int sw_state_lookup(const SwMsSlot* ms, int64_t mask, int32_t asg, int32_t n_ids, SwMsSlot* out, uint32_t* n_out,
                    hipStream_t s) {
  hipError_t e = hipMemsetAsync(n_out, 0, sizeof(uint32_t), s);
  if (e != hipSuccess) return (int)e;
  if (n_ids > 0) k_state_lookup<<<grid_for(2 * (int64_t)n_ids), BLK, 0, s>>>(ms, mask, asg, n_ids, out, n_out);
  return (int)hipGetLastError();
}

int sw_pip_batch(const double* pts, int64_t n_pts, const double* vtx, const int32_t* off, int64_t n_zones,
                 uint8_t* out, hipStream_t s) {
  k_pip_batch<<<grid_for(n_pts * n_zones), BLK, 0, s>>>(pts, n_pts, vtx, off, n_zones, out);
  return (int)hipGetLastError();
}

// Standalone exclusive scan (tests / host utilities).
int sw_scan_u32(const uint32_t* in, int64_t n, uint32_t* out, uint32_t* total, uint32_t* tmp, int64_t tmp_len,
                hipStream_t s) {
  int rc = launch_scan(in, n, out, total, tmp, tmp_len, s);
  if (rc) return rc;
  return (int)hipGetLastError();
}

// Outbound push: copy this step's enriched rows (count read on the device, no host sync) from
// HBM into the mapped host ring.  Runs on its own stream, overlapping the next step's compute;
// a few blocks with 16-B stores saturate the PCIe write direction while H2D uses SDMA.
__global__ void k_push_out(const uint4* __restrict__ src, uint4* __restrict__ dst, const uint32_t* __restrict__ n_ptr,
                           int64_t cap) {
  const int64_t n = (int64_t)(*n_ptr < cap ? *n_ptr : cap) * (int64_t)(sizeof(SwOutRec) / 16);
  for (int64_t i = (int64_t)BID * BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK) dst[i] = src[i];
}

int sw_push_out(const void* src, void* dst_dev, const uint32_t* n_ptr, int64_t cap, int32_t blocks, hipStream_t s) {
  k_push_out<<<blocks > 0 ? blocks : 256, BLK, 0, s>>>((const uint4*)src, (uint4*)dst_dev, n_ptr, cap);
  return (int)hipGetLastError();
}

// Mapped pinned host memory the kernels can store into directly (zero-copy outbound ring).
int sw_host_alloc(int64_t bytes, void** host, void** dev) {
  hipError_t e = hipHostMalloc(host, (size_t)bytes, hipHostMallocMapped | hipHostMallocPortable);
  if (e != hipSuccess) return (int)e;
  e = hipHostGetDevicePointer(dev, *host, 0);
  return (int)e;
}

int sw_host_free(void* host) { return (int)hipHostFree(host); }

// Stream-ordered SDMA copy device -> pinned host (outbound rows of a finished step, overlapped with
// the next step's kernels and H2D on a third stream; PCIe is full duplex).
int sw_copy_d2h(void* dst_host, const void* src_dev, int64_t bytes, hipStream_t s) {
  return (int)hipMemcpyAsync(dst_host, src_dev, (size_t)bytes, hipMemcpyDeviceToHost, s);
}

// ---------------------------------------------------------------------------------------------
// Explicit SDMA copies through the HSA runtime.  hipMemcpyAsync D2H into pinned memory is served by
// a blit *kernel* on this ROCm (it occupies CUs for the whole PCIe-bound transfer and slows the
// pipeline's kernels); hsa_amd_memory_async_copy_on_engine puts the transfer on a copy engine that
// uses no CUs.  The caller orders the copy after the producing step by host sync (the runner has
// already waited for the step), so no dependency signal is needed.
static hsa_agent_t g_cpu_agent = {0};
static hsa_status_t sw_find_cpu(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    g_cpu_agent = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

// engine: 0 = runtime's choice (hsa_amd_memory_async_copy), k>0 = SDMA engine bit (1 << (k-1)).
int sw_sdma_copy(void* dst_host, const void* src_dev, int64_t bytes, int32_t engine, uint64_t* signal_out) {
  if (g_cpu_agent.handle == 0) {
    hsa_status_t st = hsa_iterate_agents(sw_find_cpu, nullptr);
    if (st != HSA_STATUS_SUCCESS && st != HSA_STATUS_INFO_BREAK) return 1000 + (int)st;
    if (g_cpu_agent.handle == 0) return 999;
  }
  hsa_amd_pointer_info_t info;
  info.size = sizeof(info);
  hsa_status_t st = hsa_amd_pointer_info(src_dev, &info, nullptr, nullptr, nullptr);
  if (st != HSA_STATUS_SUCCESS) return 2000 + (int)st;
  hsa_agent_t gpu_agent = info.agentOwner;
  hsa_signal_t sig;
  st = hsa_signal_create(1, 0, nullptr, &sig);
  if (st != HSA_STATUS_SUCCESS) return 3000 + (int)st;
  if (engine > 0) {
    st = hsa_amd_memory_async_copy_on_engine(dst_host, g_cpu_agent, src_dev, gpu_agent, (size_t)bytes, 0, nullptr,
                                             sig, (hsa_amd_sdma_engine_id_t)(1u << (engine - 1)), true);
  } else {
    st = hsa_amd_memory_async_copy(dst_host, g_cpu_agent, src_dev, gpu_agent, (size_t)bytes, 0, nullptr, sig);
  }
  if (st != HSA_STATUS_SUCCESS) {
    hsa_signal_destroy(sig);
    return 4000 + (int)st;
  }
  *signal_out = sig.handle;
  return 0;
}

// Host -> device on a copy engine (probe / H2D experiments): the mirror of sw_sdma_copy.
int sw_sdma_h2d(void* dst_dev, const void* src_host, int64_t bytes, int32_t engine, uint64_t* signal_out) {
  if (g_cpu_agent.handle == 0) {
    hsa_status_t st = hsa_iterate_agents(sw_find_cpu, nullptr);
    if (st != HSA_STATUS_SUCCESS && st != HSA_STATUS_INFO_BREAK) return 1000 + (int)st;
    if (g_cpu_agent.handle == 0) return 999;
  }
  hsa_amd_pointer_info_t info;
  info.size = sizeof(info);
  hsa_status_t st = hsa_amd_pointer_info(dst_dev, &info, nullptr, nullptr, nullptr);
  if (st != HSA_STATUS_SUCCESS) return 2000 + (int)st;
  hsa_agent_t gpu_agent = info.agentOwner;
  hsa_signal_t sig;
  st = hsa_signal_create(1, 0, nullptr, &sig);
  if (st != HSA_STATUS_SUCCESS) return 3000 + (int)st;
  if (engine > 0) {
    st = hsa_amd_memory_async_copy_on_engine(dst_dev, gpu_agent, src_host, g_cpu_agent, (size_t)bytes, 0, nullptr,
                                             sig, (hsa_amd_sdma_engine_id_t)(1u << (engine - 1)), true);
  } else {
    st = hsa_amd_memory_async_copy(dst_dev, gpu_agent, src_host, g_cpu_agent, (size_t)bytes, 0, nullptr, sig);
  }
  if (st != HSA_STATUS_SUCCESS) {
    hsa_signal_destroy(sig);
    return 4000 + (int)st;
  }
  *signal_out = sig.handle;
  return 0;
}

int sw_sdma_wait(uint64_t handle) {
  hsa_signal_t sig;
  sig.handle = handle;
  while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED) >= 1) {
  }
  return (int)hsa_signal_destroy(sig);
}

int sw_abi_sizes(int64_t* out) {
  out[0] = sizeof(SwEventRec);
  out[1] = sizeof(SwOutRec);
  out[2] = sizeof(SwEngineArgs);
  out[3] = sizeof(SwNameRef);
  out[4] = sizeof(SwZoneTest);
  out[5] = sizeof(SwRegSlot);
  out[6] = sizeof(SwAsgState);
  out[7] = sizeof(SwMsSlot);
  out[8] = sizeof(SwWireRec);
  out[9] = sizeof(SwStrRef);
  return 0;
}

}  // extern "C"
