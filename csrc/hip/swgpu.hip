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
#include <stdint.h>
#include "swtypes.h"
#include "swdecode.h"
#include "swengine.h"

#define BLK 256
#define WAVES (BLK / 64)
#define TILE_ITEMS 4
#define TILE (BLK * TILE_ITEMS)
#define MAX_GRID 2048
#define STAGE_BYTES (32 * 1024)

typedef unsigned long long ull;

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

// ============================================================================ scan
// Exclusive scan of u32[n] -> out, total -> *total.  n <= TILE * (BLK * 64).
__global__ void k_scan_tiles(const uint32_t* __restrict__ in, int64_t n, uint32_t* __restrict__ tsum) {
  __shared__ uint32_t lds[WAVES + 1];
  const int64_t base = (int64_t)blockIdx.x * TILE;
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < TILE_ITEMS; ++k) {
    int64_t i = base + (int64_t)k * BLK + threadIdx.x;
    if (i < n) s += in[i];
  }
  uint32_t tot;
  block_excl_scan(s, &tot, lds);
  if (threadIdx.x == 0) tsum[blockIdx.x] = tot;
}

__global__ void k_scan_sums(uint32_t* __restrict__ tsum, int64_t nt, uint32_t* __restrict__ total) {
  __shared__ uint32_t lds[WAVES + 1];
  const int64_t per = (nt + BLK - 1) / BLK;
  const int64_t b = (int64_t)threadIdx.x * per;
  uint32_t s = 0;
  for (int64_t i = 0; i < per; ++i) if (b + i < nt) s += tsum[b + i];
  uint32_t tot;
  uint32_t pre = block_excl_scan(s, &tot, lds);
  for (int64_t i = 0; i < per; ++i) {
    if (b + i < nt) { uint32_t t = tsum[b + i]; tsum[b + i] = pre; pre += t; }
  }
  if (threadIdx.x == 0 && total) *total = tot;
}

__global__ void k_scan_apply(const uint32_t* __restrict__ in, int64_t n, const uint32_t* __restrict__ tsum,
                             uint32_t* __restrict__ out) {
  __shared__ uint32_t lds[WAVES + 1];
  const int64_t base = (int64_t)blockIdx.x * TILE;
  uint32_t run = tsum[blockIdx.x];
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

static int launch_scan(const uint32_t* in, int64_t n, uint32_t* out, uint32_t* total, uint32_t* tmp,
                       int64_t tmp_len, hipStream_t s) {
  int64_t nt = (n + TILE - 1) / TILE;
  if (nt < 1) nt = 1;
  if (nt > tmp_len) return -2;
  k_scan_tiles<<<(unsigned)nt, BLK, 0, s>>>(in, n, tmp);
  k_scan_sums<<<1, BLK, 0, s>>>(tmp, nt, total);
  k_scan_apply<<<(unsigned)nt, BLK, 0, s>>>(in, n, tmp, out);
  return 0;
}

// ============================================================================ decode
// Stage the block's 256 consecutive payloads into LDS with 16-B loads, then parse
// each payload from LDS (one lane per payload).  Oversized windows parse from global.
struct StageWin {
  const uint8_t* buf;   // base pointer parsed from
  uint32_t base_abs;    // absolute raw offset of buf[0]
};

__device__ __forceinline__ StageWin stage_window(const uint8_t* __restrict__ raw, const uint32_t* __restrict__ off,
                                                 int64_t n_msgs, uint8_t* lds) {
  const int64_t m0 = (int64_t)blockIdx.x * BLK;
  int64_t m1 = m0 + BLK;
  if (m1 > n_msgs) m1 = n_msgs;
  const uint32_t s = off[m0], e = off[m1];
  const uint32_t a0 = s & ~15u;
  const uint32_t span = e - a0;
  StageWin w;
  if (span <= STAGE_BYTES) {
    const uint32_t nvec = (span + 15) >> 4;
    const uint4* src = reinterpret_cast<const uint4*>(raw + a0);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (uint32_t v = threadIdx.x; v < nvec; v += BLK) dst[v] = src[v];
    __syncthreads();
    w.buf = lds;
    w.base_abs = a0;
  } else {
    w.buf = raw;
    w.base_abs = 0;
  }
  return w;
}

__global__ __launch_bounds__(BLK) void k_decode_count(const uint8_t* __restrict__ raw, const uint32_t* __restrict__ off,
                                                      int64_t n_msgs, uint32_t* __restrict__ cnt) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[STAGE_BYTES];
  StageWin w = stage_window(raw, off, n_msgs, lds);
  const int64_t m = (int64_t)blockIdx.x * BLK + threadIdx.x;
  if (m >= n_msgs) return;
  const uint32_t s = off[m] - w.base_abs, e = off[m + 1] - w.base_abs;
  cnt[m] = sw_decode_payload(w.buf, s, e, w.base_abs, 0, 0, nullptr, 0);
}

__global__ __launch_bounds__(BLK) void k_decode_emit(const uint8_t* __restrict__ raw, const uint32_t* __restrict__ off,
                                                     int64_t n_msgs, const uint32_t* __restrict__ evoff,
                                                     const uint32_t* __restrict__ n_total, SwEventRec* __restrict__ recs,
                                                     int64_t cap, int64_t now_ms, int rank) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[STAGE_BYTES];
  StageWin w = stage_window(raw, off, n_msgs, lds);
  const int64_t m = (int64_t)blockIdx.x * BLK + threadIdx.x;
  if (m >= n_msgs) return;
  const uint32_t s = off[m] - w.base_abs, e = off[m + 1] - w.base_abs;
  const int64_t o = evoff[m];
  if (o >= cap) return;
  const uint32_t room = (uint32_t)((cap - o) < 0xffffffffll ? (cap - o) : 0xffffffffll);
  sw_decode_payload(w.buf, s, e, w.base_abs, now_ms, (uint8_t)rank, recs + o, room);
}

__global__ void k_clamp_count(uint32_t* n, int64_t cap, ull* stats) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    if (*n > cap) *n = (uint32_t)cap;
  }
}

// New-name capture: the first time this rank's decoder sees a name/type hash, report
// (hash, offset, len) so the host can read the string from its raw batch.
__global__ void k_names_seen(const SwEventRec* __restrict__ recs, const uint32_t* __restrict__ n_ptr,
                             ull* __restrict__ key, int64_t mask, SwNameRef* __restrict__ list,
                             uint32_t* __restrict__ n_list, int64_t cap) {
  const uint32_t n = *n_ptr;
  for (int64_t i = (int64_t)blockIdx.x * BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK) {
    const SwEventRec& r = recs[i];
    if (r.name_hash == 0 || r.etype >= 16) continue;
    ull h = r.name_hash;
    int64_t slot = (int64_t)(h & (ull)mask);
    for (int64_t p = 0; p <= mask; ++p) {
      ull old = key[slot];
      if (old == h) break;
      if (old == 0) {
        old = atomicCAS(&key[slot], 0ull, h);
        if (old == 0) {
          uint32_t k = atomicAdd(n_list, 1u);
          if (k < cap) {
            SwNameRef ref;
            ref.hash = h; ref.off = r.aux_off; ref.len = r.aux_len; ref.src_rank = r.src_rank; ref.pad = r.etype;
            list[k] = ref;
          } else {
            atomicExch(&key[slot], 0ull);  // list full: forget, retry in a later batch
          }
          break;
        }
        if (old == h) break;
      }
      slot = (slot + 1) & mask;
    }
  }
}

// ============================================================================ shuffle (owner partition)
// Stable multi-way partition of records by owner rank into [world][shuf_cap] slabs.
__device__ __forceinline__ uint32_t owner_of(const SwEventRec& r, uint32_t world) {
  // Control/error records stay on the rank that received them (the host there owns the raw bytes).
  return r.etype >= 16 ? 0xffffffffu : sw_owner(r.fp_hi, world);
}

__global__ void k_part_count(const SwEventRec* __restrict__ recs, const uint32_t* __restrict__ n_ptr, int64_t cap,
                             int world, int rank, uint32_t* __restrict__ tcount /*[world][ntiles]*/, int64_t ntiles) {
  __shared__ uint32_t cnt[64];
  if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t n = *n_ptr;
  const int64_t base = (int64_t)blockIdx.x * TILE;
  for (int k = 0; k < TILE_ITEMS; ++k) {
    int64_t i = base + (int64_t)k * BLK + threadIdx.x;
    if (i < n) {
      uint32_t o = owner_of(recs[i], world);
      if (o == 0xffffffffu) o = rank;
      atomicAdd(&cnt[o], 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x < world) tcount[(int64_t)threadIdx.x * ntiles + blockIdx.x] = cnt[threadIdx.x];
}

__global__ void k_part_write(const SwEventRec* __restrict__ recs, const uint32_t* __restrict__ n_ptr, int world, int rank,
                             const uint32_t* __restrict__ toff /*scanned [world][ntiles]*/, int64_t ntiles,
                             SwEventRec* __restrict__ send, int64_t shuf_cap, uint32_t* __restrict__ overflow) {
  __shared__ uint32_t run[64];
  __shared__ uint32_t wcnt[WAVES][64];
  const uint32_t n = *n_ptr;
  const int64_t base = (int64_t)blockIdx.x * TILE;
  const uint32_t wid = threadIdx.x >> 6;
  if (threadIdx.x < world) {
    run[threadIdx.x] = toff[(int64_t)threadIdx.x * ntiles + blockIdx.x] - toff[(int64_t)threadIdx.x * ntiles];
  }
  __syncthreads();
  for (int k = 0; k < TILE_ITEMS; ++k) {
    const int64_t i = base + (int64_t)k * BLK + threadIdx.x;
    const bool valid = i < n;
    uint32_t o = 0;
    if (valid) { o = owner_of(recs[i], world); if (o == 0xffffffffu) o = rank; }
    uint32_t my_rank = 0;
    for (int q = 0; q < world; ++q) {
      ull m = __ballot(valid && o == (uint32_t)q);
      if (valid && o == (uint32_t)q) my_rank = __popcll(m & lanemask_lt());
      if (lane_id() == 0) wcnt[wid][q] = __popcll(m);
    }
    __syncthreads();
    if (valid) {
      uint32_t pre = run[o];
      for (uint32_t w = 0; w < wid; ++w) pre += wcnt[w][o];
      pre += my_rank;
      if (pre < shuf_cap) send[(int64_t)o * shuf_cap + pre] = recs[i];
      else atomicAdd(overflow, 1u);
    }
    __syncthreads();
    if (threadIdx.x < world) {
      uint32_t t = 0;
      for (int w = 0; w < WAVES; ++w) t += wcnt[w][threadIdx.x];
      run[threadIdx.x] += t;
    }
    __syncthreads();
  }
}

__global__ void k_part_counts(const uint32_t* __restrict__ toff, const uint32_t* __restrict__ tcount, int64_t ntiles,
                              int world, int64_t shuf_cap, uint32_t* __restrict__ send_cnt) {
  int o = threadIdx.x;
  if (o < world) {
    int64_t last = (int64_t)o * ntiles + ntiles - 1;
    uint32_t tot = toff[last] + tcount[last] - toff[(int64_t)o * ntiles];
    send_cnt[o] = tot < shuf_cap ? tot : (uint32_t)shuf_cap;
  }
}

// Concatenate the received [world][shuf_cap] slabs into one dense batch (rank order).
__global__ void k_unpack(const SwEventRec* __restrict__ recv, const uint32_t* __restrict__ recv_cnt, int world,
                         int64_t shuf_cap, SwEventRec* __restrict__ work, uint32_t* __restrict__ n_work, int64_t cap) {
  __shared__ uint32_t pre[65];
  if (threadIdx.x == 0) {
    pre[0] = 0;
    for (int q = 0; q < world; ++q) pre[q + 1] = pre[q] + (recv_cnt[q] < shuf_cap ? recv_cnt[q] : (uint32_t)shuf_cap);
  }
  __syncthreads();
  const uint32_t total = pre[world] < cap ? pre[world] : (uint32_t)cap;
  if (blockIdx.x == 0 && threadIdx.x == 0) *n_work = total;
  for (int64_t i = (int64_t)blockIdx.x * BLK + threadIdx.x; i < total; i += (int64_t)gridDim.x * BLK) {
    int q = 0;
    while (q + 1 < world && i >= pre[q + 1]) ++q;
    work[i] = recv[(int64_t)q * shuf_cap + (i - pre[q])];
  }
}

// ============================================================================ validate
__global__ void k_lookup(const SwEventRec* __restrict__ recs, const uint32_t* __restrict__ n_ptr,
                         const ull* __restrict__ reg_lo, const ull* __restrict__ reg_hi, const int32_t* __restrict__ reg_val,
                         int64_t reg_mask, const int32_t* __restrict__ dev_asg, const uint8_t* __restrict__ asg_active,
                         uint8_t* __restrict__ status, int32_t* __restrict__ ev_dev, int32_t* __restrict__ ev_asg) {
  const uint32_t n = *n_ptr;
  for (int64_t i = (int64_t)blockIdx.x * BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK) {
    const ull lo = recs[i].fp_lo, hi = recs[i].fp_hi;
    const uint8_t et = recs[i].etype;
    uint8_t st;
    int32_t dev = -1, asg = -1;
    if (et == SW_EV_DECODE_ERROR) st = SW_ST_DECODE_ERROR;
    else {
      int64_t slot = (int64_t)(lo & (ull)reg_mask);
      for (int64_t p = 0; p <= reg_mask; ++p) {
        const ull k = reg_lo[slot];
        if (k == lo && reg_hi[slot] == hi) { dev = reg_val[slot]; break; }
        if (k == 0 && reg_hi[slot] == 0) break;
        slot = (slot + 1) & reg_mask;
      }
      if (et >= 16) st = SW_ST_CONTROL;
      else if (dev < 0) st = SW_ST_UNREGISTERED;
      else {
        asg = dev_asg[dev];
        st = (asg >= 0 && asg_active[asg]) ? SW_ST_OK : SW_ST_UNASSIGNED;
      }
    }
    status[i] = st;
    ev_dev[i] = dev;
    ev_asg[i] = asg;
  }
}

// Alternate-id dedup window: first occurrence (lowest global sequence) wins; anything
// seen in an earlier batch is a duplicate.  Only events that would be persisted insert.
__global__ void k_dedup_insert(const SwEventRec* __restrict__ recs, const uint32_t* __restrict__ n_ptr,
                               const uint8_t* __restrict__ status, ull* __restrict__ key, ull* __restrict__ seq,
                               int64_t mask, const int64_t* __restrict__ seq_base) {
  const uint32_t n = *n_ptr;
  const ull sb = (ull)*seq_base;
  for (int64_t i = (int64_t)blockIdx.x * BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK) {
    const ull h = recs[i].alt_hash;
    if (h == 0 || status[i] != SW_ST_OK) continue;
    int64_t slot = (int64_t)(h & (ull)mask);
    for (int64_t p = 0; p <= mask; ++p) {
      ull old = atomicCAS(&key[slot], 0ull, h);
      if (old == 0 || old == h) { atomicMin(&seq[slot], sb + (ull)i); break; }
      slot = (slot + 1) & mask;
    }
  }
}

__global__ void k_dedup_check(const SwEventRec* __restrict__ recs, const uint32_t* __restrict__ n_ptr,
                              uint8_t* __restrict__ status, const ull* __restrict__ key, const ull* __restrict__ seq,
                              int64_t mask, const int64_t* __restrict__ seq_base) {
  const uint32_t n = *n_ptr;
  const ull sb = (ull)*seq_base;
  for (int64_t i = (int64_t)blockIdx.x * BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK) {
    const ull h = recs[i].alt_hash;
    if (h == 0 || status[i] != SW_ST_OK) continue;
    int64_t slot = (int64_t)(h & (ull)mask);
    for (int64_t p = 0; p <= mask; ++p) {
      const ull k = key[slot];
      if (k == h) { if (seq[slot] != sb + (ull)i) status[i] = SW_ST_DUPLICATE; break; }
      if (k == 0) break;
      slot = (slot + 1) & mask;
    }
  }
}

// ============================================================================ compaction
// Stable split of [0, n) into ok (status == OK) and rejected lists.
__global__ void k_cmp_count(const uint8_t* __restrict__ status, const uint32_t* __restrict__ n_ptr,
                            uint32_t* __restrict__ tcnt /*[2][ntiles]*/, int64_t ntiles) {
  __shared__ uint32_t lds[WAVES + 1];
  const uint32_t n = *n_ptr;
  const int64_t base = (int64_t)blockIdx.x * TILE;
  uint32_t ok = 0, rj = 0;
  for (int k = 0; k < TILE_ITEMS; ++k) {
    int64_t i = base + (int64_t)k * BLK + threadIdx.x;
    if (i < n) { if (status[i] == SW_ST_OK) ++ok; else ++rj; }
  }
  uint32_t t_ok, t_rj;
  block_excl_scan(ok, &t_ok, lds);
  block_excl_scan(rj, &t_rj, lds);
  if (threadIdx.x == 0) { tcnt[blockIdx.x] = t_ok; tcnt[ntiles + blockIdx.x] = t_rj; }
}

__global__ void k_cmp_write(const uint8_t* __restrict__ status, const uint32_t* __restrict__ n_ptr,
                            const uint32_t* __restrict__ toff, const uint32_t* __restrict__ tcnt, int64_t ntiles,
                            uint32_t* __restrict__ ok_idx, uint32_t* __restrict__ rej_idx,
                            uint32_t* __restrict__ n_ok, uint32_t* __restrict__ n_rej) {
  __shared__ uint32_t lds[WAVES + 1];
  const uint32_t n = *n_ptr;
  const int64_t base = (int64_t)blockIdx.x * TILE;
  const uint32_t rej_base = toff[ntiles];  // rejected region starts after all ok counts in the flat scan
  uint32_t run_ok = toff[blockIdx.x];
  uint32_t run_rj = toff[ntiles + blockIdx.x] - rej_base;
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
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    const int64_t last = ntiles - 1;
    *n_ok = toff[last] + tcnt[last];
    *n_rej = toff[ntiles + last] + tcnt[ntiles + last] - rej_base;
  }
}

// ============================================================================ names intern
template <typename K>
__device__ __forceinline__ int64_t nm_probe(const K* __restrict__ key, int64_t mask, ull h) {
  int64_t slot = (int64_t)(h & (ull)mask);
  for (int64_t p = 0; p <= mask; ++p) {
    const ull k = key[slot];
    if (k == h) return slot;
    if (k == 0) return -1;
    slot = (slot + 1) & mask;
  }
  return -1;
}

__global__ void k_intern_insert(const SwEventRec* __restrict__ recs, const uint32_t* __restrict__ idx,
                                const uint32_t* __restrict__ n_ptr, ull* __restrict__ key, int32_t* __restrict__ first,
                                int64_t mask) {
  const uint32_t n = *n_ptr;
  for (int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLK) {
    const uint32_t i = idx ? idx[j] : (uint32_t)j;
    const ull h = recs[i].name_hash;
    if (h == 0) continue;
    int64_t slot = (int64_t)(h & (ull)mask);
    for (int64_t p = 0; p <= mask; ++p) {
      ull old = key[slot];
      if (old == 0) old = atomicCAS(&key[slot], 0ull, h);
      if (old == 0) { atomicMin(&first[slot], (int32_t)j); break; }
      if (old == h) break;
      slot = (slot + 1) & mask;
    }
  }
}

__global__ void k_intern_assign(const SwEventRec* __restrict__ recs, const uint32_t* __restrict__ idx,
                                const uint32_t* __restrict__ n_ptr, const ull* __restrict__ key,
                                int32_t* __restrict__ ids, int32_t* __restrict__ first, int64_t mask,
                                int32_t* __restrict__ counter) {
  const uint32_t n = *n_ptr;
  for (int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLK) {
    const uint32_t i = idx ? idx[j] : (uint32_t)j;
    const ull h = recs[i].name_hash;
    if (h == 0) continue;
    const int64_t slot = nm_probe(key, mask, h);
    if (slot >= 0 && ids[slot] < 0 && first[slot] == (int32_t)j) {
      ids[slot] = atomicAdd(counter, 1);
      first[slot] = 0x7fffffff;
    }
  }
}

// ============================================================================ persist + enrich
__global__ void k_persist(SwEngineArgs a, const SwEventRec* __restrict__ R, const uint32_t* __restrict__ idx,
                          const int32_t* __restrict__ devs, const int32_t* __restrict__ asgs,
                          const uint32_t* __restrict__ n_ptr) {
  const uint32_t n = *n_ptr;
  const int64_t cur = *a.store_cursor;
  const int64_t c0 = *a.step_cursor0;
  for (int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLK) {
    const uint32_t i = idx ? idx[j] : (uint32_t)j;
    const SwEventRec r = R[i];
    const int32_t dev = devs[i], asg = asgs[i];
    const int64_t seq = cur + j;
    const int64_t row = seq % a.store_cap;
    const int64_t eid = seq * a.world + a.rank;
    a.s_etype[row] = r.etype;
    a.s_level[row] = r.level;
    a.s_date[row] = r.event_date;
    a.s_recv[row] = a.now_ms;
    a.s_dev[row] = dev;
    a.s_asg[row] = asg;
    a.s_cust[row] = a.asg_customer[asg];
    a.s_area[row] = a.asg_area[asg];
    a.s_asset[row] = a.asg_asset[asg];
    a.s_name[row] = r.name_hash;
    a.s_v0[row] = r.v0;
    a.s_v1[row] = r.v1;
    a.s_v2[row] = r.v2;
    a.s_alt[row] = r.alt_hash;
    a.s_aux[row] = ((ull)r.src_rank << 48) | ((ull)r.aux_len << 32) | (ull)r.aux_off;
    a.s_batch[row] = (int32_t)a.batch_seq;
    SwOutRec o;
    o.event_id = eid;
    o.event_date = r.event_date;
    o.v0 = r.v0;
    o.v1 = r.v1;
    o.assignment = asg;
    o.device = dev;
    const int64_t ns = r.name_hash ? nm_probe(a.nm_key, a.nm_mask, r.name_hash) : -1;
    o.name_id = ns >= 0 ? a.nm_id[ns] : -1;
    o.etype = r.etype;
    o.level = r.level;
    o.status = 0;
    a.out[seq - c0] = o;
  }
}

// ============================================================================ device state
__device__ __forceinline__ int64_t ms_slot(uint64_t* __restrict__ key_, int64_t mask, ull k) {
  ull* key = (ull*)key_;
  int64_t slot = (int64_t)(sw_mix64(k) & (ull)mask);
  for (int64_t p = 0; p <= mask; ++p) {
    ull old = key[slot];
    if (old == k) return slot;
    if (old == 0) {
      old = atomicCAS(&key[slot], 0ull, k);
      if (old == 0 || old == k) return slot;
    }
    slot = (slot + 1) & mask;
  }
  return -1;
}

__device__ __forceinline__ ull state_key(const SwEngineArgs& a, const SwEventRec& r, int32_t asg) {
  const int64_t ns = nm_probe(a.nm_key, a.nm_mask, r.name_hash);
  if (ns < 0) return 0;
  const int32_t id = a.nm_id[ns];
  if (id < 0) return 0;
  // +1 keeps key 0 reserved as empty
  return (((ull)(uint32_t)asg) << 32 | ((ull)(uint32_t)id << 1) | (r.etype == SW_EV_ALERT ? 1ull : 0ull)) + 1ull;
}

// Pass 1: max event date per (assignment) location and per (assignment, name) measurement/alert.
__global__ void k_state_p1(SwEngineArgs a, const SwEventRec* __restrict__ R, const uint32_t* __restrict__ idx,
                           const int32_t* __restrict__ asgs, const uint32_t* __restrict__ n_ptr) {
  const uint32_t n = *n_ptr;
  for (int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLK) {
    const uint32_t i = idx ? idx[j] : (uint32_t)j;
    const SwEventRec r = R[i];
    const int32_t asg = asgs[i];
    if (r.etype != SW_EV_MEASUREMENT && r.etype != SW_EV_LOCATION && r.etype != SW_EV_ALERT) continue;
    atomicMax((ull*)&a.st_last[asg], (ull)a.now_ms);
    if (a.st_missing[asg]) a.st_missing[asg] = 0;  // presence detected again
    const ull d = (ull)r.event_date;
    if (r.etype == SW_EV_LOCATION) {
      atomicMax((ull*)&a.st_loc_date[asg], d);
    } else if (r.name_hash) {
      const ull k = state_key(a, r, asg);
      if (!k) continue;
      const int64_t s = ms_slot(a.ms_key, a.ms_mask, k);
      if (s >= 0) atomicMax((ull*)&a.ms_date[s], d);
    }
  }
}

// Pass 2: among events carrying the max date, the highest event id wins (ids are monotonic).
__global__ void k_state_p2(SwEngineArgs a, const SwEventRec* __restrict__ R, const uint32_t* __restrict__ idx,
                           const int32_t* __restrict__ asgs, const uint32_t* __restrict__ n_ptr) {
  const uint32_t n = *n_ptr;
  const int64_t cur = *a.store_cursor;
  for (int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLK) {
    const uint32_t i = idx ? idx[j] : (uint32_t)j;
    const SwEventRec r = R[i];
    const int32_t asg = asgs[i];
    const ull eid1 = (ull)((cur + j) * a.world + a.rank) + 1ull;  // stored +1, 0 = none
    const ull d = (ull)r.event_date;
    if (r.etype == SW_EV_LOCATION) {
      if (a.st_loc_date[asg] == d) atomicMax((ull*)&a.st_loc_eid[asg], eid1);
    } else if ((r.etype == SW_EV_MEASUREMENT || r.etype == SW_EV_ALERT) && r.name_hash) {
      const ull k = state_key(a, r, asg);
      if (!k) continue;
      const int64_t s = ms_slot(a.ms_key, a.ms_mask, k);
      if (s >= 0 && a.ms_date[s] == d) atomicMax((ull*)&a.ms_eid[s], eid1);
    }
  }
}

__global__ void k_advance(int64_t* __restrict__ cursor, const uint32_t* __restrict__ n_ptr) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *cursor += *n_ptr;
}

// ============================================================================ zone-test rules
#define ZONE_LDS_VTX 3072  // 48 KiB of (lat, lon) doubles

__device__ __forceinline__ bool pip(const double* __restrict__ v, int n, double x, double y) {
  // even-odd crossing number; v = [lat0, lon0, lat1, lon1, ...], x = lat, y = lon
  bool inside = false;
  for (int i = 0, j = n - 1; i < n; j = i++) {
    const double xi = v[2 * i], yi = v[2 * i + 1], xj = v[2 * j], yj = v[2 * j + 1];
    if (((yi > y) != (yj > y)) && (x < (xj - xi) * (y - yi) / (yj - yi) + xi)) inside = !inside;
  }
  return inside;
}

__global__ __launch_bounds__(BLK) void k_zones(SwEngineArgs a) {
  __shared__ double lv[2 * ZONE_LDS_VTX];
  const int64_t nv = a.n_zones ? a.zone_off[a.n_zones] : 0;
  const bool in_lds = nv <= ZONE_LDS_VTX;
  if (in_lds) {
    for (int64_t t = threadIdx.x; t < 2 * nv; t += BLK) lv[t] = a.zone_vtx[t];
    __syncthreads();
  }
  const double* V = in_lds ? lv : a.zone_vtx;
  const int64_t c0 = *a.step_cursor0;
  const uint32_t n = (uint32_t)(*a.store_cursor - c0);  // events persisted so far this step
  for (int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLK) {
    const SwOutRec o = a.out[j];
    if (o.etype != SW_EV_LOCATION) continue;
    const double x = o.v0, y = o.v1;
    for (int t = 0; t < a.n_tests; ++t) {
      const SwZoneTest zt = a.tests[t];
      const int z = zt.zone;
      const double* bb = a.zone_bbox + 4 * z;
      bool inside = x >= bb[0] && y >= bb[1] && x <= bb[2] && y <= bb[3];
      if (inside) {
        const int v0 = a.zone_off[z], v1 = a.zone_off[z + 1];
        inside = pip(V + 2 * v0, v1 - v0, x, y);
      }
      if ((zt.condition == 0) == inside) {
        const uint32_t g = atomicAdd(a.n_gen, 1u);
        if (g < a.gen_cap) {
          SwEventRec r;
          r.fp_lo = 0; r.fp_hi = 0;
          r.event_date = a.now_ms;  // reference: alert.setEventDate(new Date())
          r.name_hash = a.test_name_hash[t];
          r.v0 = 0; r.v1 = 0; r.v2 = 0; r.alt_hash = 0;
          r.aux_off = (uint32_t)t; r.aux2_off = 0; r.aux_len = 0; r.aux2_len = 0;
          r.etype = SW_EV_ALERT; r.flags = 0; r.src_rank = (uint8_t)a.rank; r.level = (uint8_t)zt.level;
          a.gen[g] = r;
          a.gen_dev[g] = o.device;
          a.gen_asg[g] = o.assignment;
        }
      }
    }
  }
}

// ============================================================================ presence
__global__ void k_presence(SwEngineArgs a) {
  const ull limit = (ull)(a.now_ms - a.presence_missing_ms);
  for (int64_t s = (int64_t)blockIdx.x * BLK + threadIdx.x; s < a.n_asg; s += (int64_t)gridDim.x * BLK) {
    const ull last = a.st_last[s];
    const bool miss = a.asg_active[s] && last != 0 && last < limit && a.st_missing[s] == 0;
    if (!miss) continue;
    a.st_missing[s] = (ull)a.now_ms;  // send-once strategy
    const uint32_t g = atomicAdd(a.n_gen, 1u);
    if (g < a.gen_cap) {
      SwEventRec r;
      r.fp_lo = 0; r.fp_hi = 0; r.event_date = a.now_ms; r.name_hash = a.presence_name_hash;
      r.v0 = 0; r.v1 = 0; r.v2 = 0; r.alt_hash = 0;
      r.aux_off = 0; r.aux2_off = 0; r.aux_len = 0; r.aux2_len = 0;
      r.etype = SW_EV_STATE_CHANGE; r.flags = 0; r.src_rank = (uint8_t)a.rank; r.level = 0;
      a.gen[g] = r;
      a.gen_dev[g] = a.asg_device[s];
      a.gen_asg[g] = (int32_t)s;
    }
  }
}

// ============================================================================ step bookkeeping
__global__ void k_step_begin(SwEngineArgs a) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    *a.step_cursor0 = *a.store_cursor;
    *a.n_gen = 0;
    *a.n_new_names = 0;
    *a.n_out = 0;
    *a.overflow = 0;
  }
}

__global__ void k_gen_clamp(SwEngineArgs a, uint32_t* gen_rules) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    if (*a.n_gen > a.gen_cap) *a.n_gen = (uint32_t)a.gen_cap;
    if (gen_rules) *gen_rules = *a.n_gen;
  }
}

__global__ void k_step_end(SwEngineArgs a, const uint32_t* n_rule_alerts) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    *a.n_out = (uint32_t)(*a.store_cursor - *a.step_cursor0);
    *a.seq_base += *a.n_work;
    ull* st = (ull*)a.stats;
    st[SW_STAT_MSGS] += (ull)a.n_msgs;
    st[SW_STAT_EVENTS] += *a.n_work;
    st[SW_STAT_PERSISTED] += *a.n_out;
    st[SW_STAT_RULE_ALERTS] += *n_rule_alerts;
    st[SW_STAT_PRESENCE] += *a.n_gen - *n_rule_alerts;
    st[SW_STAT_SHUFFLE_OVERFLOW] += *a.overflow;
    st[SW_STAT_NEW_NAMES] += *a.n_new_names;
  }
}

__global__ void k_reject_stats(SwEngineArgs a) {
  __shared__ uint32_t c[8];
  if (threadIdx.x < 8) c[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t n = *a.n_rej;
  for (int64_t j = (int64_t)blockIdx.x * BLK + threadIdx.x; j < n; j += (int64_t)gridDim.x * BLK) {
    atomicAdd(&c[a.status[a.rej_idx[j]] & 7], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd((ull*)&a.stats[SW_STAT_UNREGISTERED], (ull)c[SW_ST_UNREGISTERED]);
    atomicAdd((ull*)&a.stats[SW_STAT_UNASSIGNED], (ull)c[SW_ST_UNASSIGNED]);
    atomicAdd((ull*)&a.stats[SW_STAT_DUPLICATE], (ull)c[SW_ST_DUPLICATE]);
    atomicAdd((ull*)&a.stats[SW_STAT_DECODE_ERROR], (ull)c[SW_ST_DECODE_ERROR]);
    atomicAdd((ull*)&a.stats[SW_STAT_CONTROL], (ull)c[SW_ST_CONTROL]);
  }
}

// ============================================================================ C ABI
extern "C" {

// Phase A: decode the raw batch into records (+ new-name capture).  msg counts are host-known.
int sw_phase_decode(const SwEngineArgs* ap, hipStream_t s) {
  const SwEngineArgs a = *ap;
  k_step_begin<<<1, 64, 0, s>>>(a);
  if (a.n_msgs <= 0) {
    (void)hipMemsetAsync(a.n_recs, 0, sizeof(uint32_t), s);
    return (int)hipGetLastError();
  }
  const unsigned nb = (unsigned)((a.n_msgs + BLK - 1) / BLK);
  k_decode_count<<<nb, BLK, 0, s>>>(a.raw, a.msg_off, a.n_msgs, a.msg_cnt);
  int rc = launch_scan(a.msg_cnt, a.n_msgs, a.msg_evoff, a.n_recs, a.scan_tmp, a.scan_tmp_len, s);
  if (rc) return rc;
  k_decode_emit<<<nb, BLK, 0, s>>>(a.raw, a.msg_off, a.n_msgs, a.msg_evoff, a.n_recs, a.recs, a.rec_cap, a.now_ms,
                                   (int)a.rank);
  k_clamp_count<<<1, 64, 0, s>>>(a.n_recs, a.rec_cap, (ull*)a.stats);
  k_names_seen<<<grid_for(a.rec_cap), BLK, 0, s>>>(a.recs, a.n_recs, (ull*)a.seen_key, a.seen_mask, a.new_names,
                                                    a.n_new_names, a.names_cap);
  return (int)hipGetLastError();
}

// Phase B (world > 1): stable partition of records into per-owner send slabs.
int sw_phase_partition(const SwEngineArgs* ap, hipStream_t s) {
  const SwEngineArgs a = *ap;
  const int64_t ntiles = (a.rec_cap + TILE - 1) / TILE;
  if (a.world > 64 || ntiles * a.world > a.part_tmp_len) return -3;
  k_part_count<<<(unsigned)ntiles, BLK, 0, s>>>(a.recs, a.n_recs, a.rec_cap, (int)a.world, (int)a.rank, a.part_tmp,
                                                ntiles);
  // scan the flat [world][ntiles] count matrix in place
  int rc = launch_scan(a.part_tmp, ntiles * a.world, a.part_tmp + ntiles * a.world, nullptr, a.scan_tmp,
                       a.scan_tmp_len, s);
  if (rc) return rc;
  const uint32_t* toff = a.part_tmp + ntiles * a.world;
  k_part_write<<<(unsigned)ntiles, BLK, 0, s>>>(a.recs, a.n_recs, (int)a.world, (int)a.rank, toff, ntiles, a.send,
                                                a.shuf_cap, a.overflow);
  k_part_counts<<<1, 64, 0, s>>>(toff, a.part_tmp, ntiles, (int)a.world, a.shuf_cap, a.send_cnt);
  return (int)hipGetLastError();
}

// Phase C (world > 1): concatenate received slabs into the work batch.
int sw_phase_unpack(const SwEngineArgs* ap, hipStream_t s) {
  const SwEngineArgs a = *ap;
  k_unpack<<<grid_for(a.rec_cap), BLK, 0, s>>>(a.recv, a.recv_cnt, (int)a.world, a.shuf_cap, a.work, a.n_work,
                                               a.rec_cap);
  return (int)hipGetLastError();
}

// Phase D: validate, dedup, persist, enrich, state, rules, presence.
int sw_phase_process(const SwEngineArgs* ap, uint32_t* scratch4, hipStream_t s) {
  const SwEngineArgs a = *ap;
  const int g = grid_for(a.rec_cap);
  const int64_t ntiles = (a.rec_cap + TILE - 1) / TILE;
  if (2 * ntiles > a.scan_tmp_len) return -4;
  if (a.world == 1) (void)hipMemcpyAsync(a.n_work, a.n_recs, sizeof(uint32_t), hipMemcpyDeviceToDevice, s);
  k_lookup<<<g, BLK, 0, s>>>(a.work, a.n_work, (const ull*)a.reg_lo, (const ull*)a.reg_hi, a.reg_val, a.reg_mask,
                             a.dev_asg, a.asg_active, a.status, a.ev_dev, a.ev_asg);
  k_dedup_insert<<<g, BLK, 0, s>>>(a.work, a.n_work, a.status, (ull*)a.dd_key, (ull*)a.dd_seq, a.dd_mask, a.seq_base);
  k_dedup_check<<<g, BLK, 0, s>>>(a.work, a.n_work, a.status, (const ull*)a.dd_key, (const ull*)a.dd_seq, a.dd_mask,
                                  a.seq_base);
  // stable split ok / rejected
  k_cmp_count<<<(unsigned)ntiles, BLK, 0, s>>>(a.status, a.n_work, a.cmp_tmp, ntiles);
  uint32_t* cmp_off = a.cmp_tmp + 2 * ntiles;
  int rc = launch_scan(a.cmp_tmp, 2 * ntiles, cmp_off, nullptr, a.scan_tmp, a.scan_tmp_len, s);
  if (rc) return rc;
  k_cmp_write<<<(unsigned)ntiles, BLK, 0, s>>>(a.status, a.n_work, cmp_off, a.cmp_tmp, ntiles, a.ok_idx, a.rej_idx,
                                               a.n_ok, a.n_rej);
  k_reject_stats<<<g, BLK, 0, s>>>(a);
  // names intern for state keys
  k_intern_insert<<<g, BLK, 0, s>>>(a.work, a.ok_idx, a.n_ok, (ull*)a.nm_key, a.nm_first, a.nm_mask);
  k_intern_assign<<<g, BLK, 0, s>>>(a.work, a.ok_idx, a.n_ok, (const ull*)a.nm_key, a.nm_id, a.nm_first, a.nm_mask,
                                    a.nm_counter);
  // persist + enrich + state for the validated events
  k_persist<<<g, BLK, 0, s>>>(a, a.work, a.ok_idx, a.ev_dev, a.ev_asg, a.n_ok);
  k_state_p1<<<g, BLK, 0, s>>>(a, a.work, a.ok_idx, a.ev_asg, a.n_ok);
  k_state_p2<<<g, BLK, 0, s>>>(a, a.work, a.ok_idx, a.ev_asg, a.n_ok);
  k_advance<<<1, 64, 0, s>>>(a.store_cursor, a.n_ok);
  // rules on this step's persisted locations, then presence scan; generated events persist too
  uint32_t* n_rule = scratch4;
  if (a.n_tests > 0) k_zones<<<g, BLK, 0, s>>>(a);
  k_gen_clamp<<<1, 64, 0, s>>>(a, n_rule);
  if (a.presence_missing_ms > 0) k_presence<<<grid_for(a.n_asg), BLK, 0, s>>>(a);
  k_gen_clamp<<<1, 64, 0, s>>>(a, nullptr);
  const int gg = grid_for(a.gen_cap);
  k_intern_insert<<<gg, BLK, 0, s>>>(a.gen, nullptr, a.n_gen, (ull*)a.nm_key, a.nm_first, a.nm_mask);
  k_intern_assign<<<gg, BLK, 0, s>>>(a.gen, nullptr, a.n_gen, (const ull*)a.nm_key, a.nm_id, a.nm_first, a.nm_mask,
                                     a.nm_counter);
  k_persist<<<gg, BLK, 0, s>>>(a, a.gen, nullptr, a.gen_dev, a.gen_asg, a.n_gen);
  k_state_p1<<<gg, BLK, 0, s>>>(a, a.gen, nullptr, a.gen_asg, a.n_gen);
  k_state_p2<<<gg, BLK, 0, s>>>(a, a.gen, nullptr, a.gen_asg, a.n_gen);
  k_advance<<<1, 64, 0, s>>>(a.store_cursor, a.n_gen);
  k_step_end<<<1, 64, 0, s>>>(a, n_rule);
  return (int)hipGetLastError();
}

// Registry patch: scatter host-built table slots (bulk load and incremental upserts).
__global__ void k_reg_patch(ull* lo, ull* hi, int32_t* val, const int64_t* slots, const ull* plo, const ull* phi,
                            const int32_t* pval, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * BLK + threadIdx.x; i < n; i += (int64_t)gridDim.x * BLK) {
    const int64_t s = slots[i];
    lo[s] = plo[i]; hi[s] = phi[i]; val[s] = pval[i];
  }
}

int sw_registry_patch(uint64_t* lo, uint64_t* hi, int32_t* val, const int64_t* slots, const uint64_t* plo,
                      const uint64_t* phi, const int32_t* pval, int64_t n, hipStream_t s) {
  if (n <= 0) return 0;
  k_reg_patch<<<grid_for(n), BLK, 0, s>>>((ull*)lo, (ull*)hi, val, slots, (const ull*)plo, (const ull*)phi, pval, n);
  return (int)hipGetLastError();
}

// Standalone batched point-in-polygon (used by the rule service for ad-hoc zone queries).
__global__ void k_pip_batch(const double* pts, int64_t n_pts, const double* vtx, const int32_t* off, int64_t n_zones,
                            uint8_t* out) {
  for (int64_t i = (int64_t)blockIdx.x * BLK + threadIdx.x; i < n_pts * n_zones; i += (int64_t)gridDim.x * BLK) {
    const int64_t p = i / n_zones, z = i % n_zones;
    out[i] = pip(vtx + 2 * off[z], off[z + 1] - off[z], pts[2 * p], pts[2 * p + 1]);
  }
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

int sw_abi_sizes(int64_t* out) {
  out[0] = sizeof(SwEventRec);
  out[1] = sizeof(SwOutRec);
  out[2] = sizeof(SwEngineArgs);
  out[3] = sizeof(SwNameRef);
  out[4] = sizeof(SwZoneTest);
  return 0;
}

}  // extern "C"
