// Read-side indexes of a durable event block, built on the MI355X in the step that encodes the block
// (format: csrc/include/swindex.h; C++ reference: csrc/native/swindex.cpp swseg_index_append, bit for
// bit).  Also the stable LSD radix sort the engine uses to persist each step clustered by assignment.
//
// Reference: MongoDeviceEventManagement.java:129-141 -- the indexes Mongo maintains on every insert
// (alternateId; assignment / customer / area / asset + eventType + eventDate).  Here they are built
// for a whole step at once, in HBM, and cost ~4 B per event on disk; the host threads that indexed
// finished blocks after the fact (~59M events/s on 16 cores) are gone.
//
// Radix sort (sw_radix_sort_u32): per 8-bit pass a count, an offsets and a scatter dispatch -- no
// look-back chains and no same-address atomics (both serialise on this chip: a decoupled look-back
// over 257 tiles that all start together walks ~16 tiles per round trip; one hot counter takes every
// workgroup's atomic in turn).  Items are ranked stably in 16 rounds of 256 (each wave matches its 64
// digits by ballots, wave counts prefixed in LDS), staged in LDS in digit order and written out as
// runs of consecutive addresses.  Wave64 throughout: ballots are 64-bit.
//
// Trailer build (sw_seg_index, after k_seg_encode on the same stream):
//   k_ix_prep     per row: alternate-id sort key (top 15 hash bits; rows without an id sort last);
//                 per workgroup a histogram of the context keys of its rows (LDS), written out whole
//   radix sort    (sort key, row), 16 bits: two passes
//   k_ix_scan     one workgroup per dimension: key totals and each workgroup's offset in a key's
//                 bucket (column prefix over the workgroup histograms), bucket starts, present-key
//                 ranks, head and chunk offsets; the last workgroup out lays the trailer out
//   k_ix_scatter  (row, date) into the key buckets at the reserved offsets (no global atomics)
//   k_ix_write    page zone maps, the alternate-id directory and its packed entries, and one wave per
//                 1024-row chunk of a key: count, date range and lane-local top-16 lists merged by 16
//                 rounds of wave argmax; a key of several chunks is finished by its last chunk, which
//                 merges the chunks' partial top-16s
//   k_ix_finish   checksum of the whole trailer (xor of mixed words: order free); the last workgroup
//                 publishes the block's bytes to the encoder state and the host snapshot
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "swindex.h"
#include "swseg.h"
#include "swtypes.h"

typedef unsigned long long ull;

#define RS_BLK 256
#define RS_ITEMS 16
#define RS_TILE (RS_BLK * RS_ITEMS)
#define RS_WAVES (RS_BLK / 64)

__device__ __forceinline__ uint32_t ix_lane() { return threadIdx.x & 63; }

// Block-wide exclusive scan of one u32 per thread (256 threads); *total = the sum.
__device__ __forceinline__ uint32_t rs_block_scan(uint32_t v, uint32_t* red, uint32_t* total) {
  const uint32_t lane = ix_lane(), wid = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += o;
  }
  if (lane == 63) red[wid] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < RS_WAVES; ++w) {
    const uint32_t x = red[w];
    pre += (uint32_t)w < wid ? x : 0u;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return inc - v + pre;
}

// ============================================================================ radix sort
// Per pass, three dispatches and no cross-workgroup waiting: k_rs_count (each tile's digit counts,
// tile-major), k_rs_offsets (one workgroup per digit: the tiles' exclusive prefix and the digit's
// total), k_rs_scatter (digit starts from the totals' prefix + the tile's offset; stable ranks; LDS
// staging in digit order; runs of consecutive output addresses).  State: hist / off [tiles][256],
// tot [256] -- fully rewritten by every pass, nothing to re-arm.
struct RsState {
  uint32_t* hist;
  uint32_t* off;
  uint32_t* tot;
};

__device__ __host__ __forceinline__ int64_t rs_tiles(int64_t cap) {
  const int64_t t = (cap + RS_TILE - 1) / RS_TILE;
  return t < 1 ? 1 : t;
}
__device__ __host__ __forceinline__ RsState rs_state(uint32_t* st, int64_t cap) {
  RsState r;
  const int64_t tiles = rs_tiles(cap);
  r.hist = st;
  r.off = st + tiles * 256;
  r.tot = r.off + tiles * 256;
  return r;
}

__global__ __launch_bounds__(RS_BLK) void k_rs_count(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ n_ptr,
                                                     int shift, uint32_t mask, uint32_t* st_words, int64_t cap) {
  __shared__ uint32_t h[256];
  const RsState st = rs_state(st_words, cap);
  const uint32_t n = *n_ptr;
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
  if (base >= (int64_t)n) return;
  h[threadIdx.x] = 0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < RS_ITEMS; ++k) {
    const int64_t i = base + (int64_t)k * RS_BLK + threadIdx.x;
    if (i < (int64_t)n) atomicAdd(&h[(keys[i] >> shift) & mask], 1u);
  }
  __syncthreads();
  st.hist[(int64_t)blockIdx.x * 256 + threadIdx.x] = h[threadIdx.x];
}

// one workgroup per digit: exclusive prefix of the digit's tile counts, and its total
__global__ __launch_bounds__(RS_BLK) void k_rs_offsets(const uint32_t* __restrict__ n_ptr, uint32_t* st_words, int64_t cap) {
  __shared__ uint32_t red[RS_WAVES];
  const RsState st = rs_state(st_words, cap);
  const uint32_t n = *n_ptr;
  const int64_t ntiles = ((int64_t)n + RS_TILE - 1) / RS_TILE;
  const uint32_t d = blockIdx.x;
  uint32_t run = 0;
  for (int64_t t0 = 0; t0 < ntiles; t0 += RS_BLK) {
    const int64_t t = t0 + threadIdx.x;
    const uint32_t v = t < ntiles ? st.hist[t * 256 + d] : 0u;
    uint32_t tot;
    const uint32_t pre = rs_block_scan(v, red, &tot);
    if (t < ntiles) st.off[t * 256 + d] = run + pre;
    run += tot;
  }
  if (threadIdx.x == 0) st.tot[d] = run;
}

struct RsLds {
  uint32_t sk[RS_TILE];
  uint32_t sv[RS_TILE];
  uint32_t wc[RS_WAVES][256];
  uint32_t ls[256];         // where a digit's run starts in the staged tile
  uint32_t run[256];        // ranked so far per digit
  uint32_t gb[256];         // where the tile's run of a digit starts in the output
  uint32_t red[RS_WAVES];
};

__global__ __launch_bounds__(RS_BLK) void k_rs_scatter(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                       uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                       const uint32_t* __restrict__ n_ptr, int shift, int dbits,
                                                       uint32_t* st_words, int64_t cap) {
  __shared__ RsLds L;
  const RsState st = rs_state(st_words, cap);
  const uint32_t n = *n_ptr;
  const int64_t tile = blockIdx.x;
  const int64_t base = tile * RS_TILE;
  if (base >= (int64_t)n) return;
  const uint32_t t = threadIdx.x, lane = ix_lane(), wid = t >> 6;
  const uint32_t mask = (1u << dbits) - 1u;
  uint32_t K[RS_ITEMS], V[RS_ITEMS];
#pragma unroll
  for (int k = 0; k < RS_ITEMS; ++k) {
    const int64_t i = base + (int64_t)k * RS_BLK + t;
    const bool ok = i < (int64_t)n;
    K[k] = ok ? kin[i] : 0u;
    V[k] = ok ? vin[i] : 0u;
  }
  uint32_t gtot, ctot;
  const uint32_t gpre = rs_block_scan(t <= mask ? st.tot[t] : 0u, L.red, &gtot);
  const uint32_t c = t <= mask ? st.hist[tile * 256 + t] : 0u;
  L.ls[t] = rs_block_scan(c, L.red, &ctot);
  L.gb[t] = gpre + (t <= mask ? st.off[tile * 256 + t] : 0u);
  L.run[t] = 0;
#pragma unroll
  for (int w = 0; w < RS_WAVES; ++w) L.wc[w][t] = 0;
  __syncthreads();
  // ---- stable ranks: striped rounds, ballot match per wave; staged in LDS in digit order
  const ull lt = (1ull << lane) - 1ull;
#pragma unroll            // K / V stay in registers (a rolled loop would index them dynamically)
  for (int k = 0; k < RS_ITEMS; ++k) {
    const int64_t i = base + (int64_t)k * RS_BLK + t;
    const bool valid = i < (int64_t)n;
    const uint32_t d = (K[k] >> shift) & mask;
    ull peers = __ballot(valid);
    for (int b = 0; b < dbits; ++b) {
      const bool bit = (d >> b) & 1u;
      const ull m = __ballot(valid && bit);
      peers &= bit ? m : ~m;
    }
    const uint32_t rank = (uint32_t)__popcll(peers & lt);
    if (valid && rank == 0) L.wc[wid][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pos = L.ls[d] + L.run[d] + rank;
      for (uint32_t w = 0; w < wid; ++w) pos += L.wc[w][d];
      L.sk[pos] = K[k];
      L.sv[pos] = V[k];
    }
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (int w = 0; w < RS_WAVES; ++w) { add += L.wc[w][t]; L.wc[w][t] = 0; }
    L.run[t] += add;
    __syncthreads();
  }
  // ---- write out: a digit's items are consecutive in LDS and in the output
  const uint32_t m = (uint32_t)(((int64_t)n - base) < RS_TILE ? (int64_t)n - base : RS_TILE);
  for (uint32_t i = t; i < m; i += RS_BLK) {
    const uint32_t key = L.sk[i];
    const uint32_t d = (key >> shift) & mask;
    const uint32_t pos = L.gb[d] + (i - L.ls[d]);
    kout[pos] = key;
    vout[pos] = L.sv[i];
  }
}

extern "C" {

int64_t sw_radix_tmp_words(int64_t cap) { return 2 * 256 * rs_tiles(cap) + 256 + 8; }

// Stable LSD radix sort of *n_ptr (<= cap) u32 (key, value) pairs by the low `bits` (<= 32) bits of
// the key.  keys / vals: [2][cap] ping-pong buffers, input in buffer 0.  vals_final (optional): where
// the last pass writes the values instead of the ping-pong buffer.  state: sw_radix_tmp_words(cap)
// words (no initialisation needed).  Returns the buffer (0 / 1) holding the sorted keys (and values,
// without vals_final): passes = ceil(bits / 8).
int sw_radix_sort_u32(uint32_t* keys, uint32_t* vals, const uint32_t* n_ptr, int64_t cap, int bits, uint32_t* state,
                      uint32_t* vals_final, hipStream_t s) {
  if (bits <= 0) return 0;
  if (bits > 32) bits = 32;
  const unsigned grid = (unsigned)rs_tiles(cap);
  int cur = 0;
  const int passes = (bits + 7) / 8;
  for (int p = 0; p < passes; ++p) {
    const int db = bits - 8 * p < 8 ? bits - 8 * p : 8;
    const uint32_t mask = (1u << db) - 1u;
    const bool last = p == passes - 1;
    uint32_t* vo = (last && vals_final) ? vals_final : vals + (int64_t)(1 - cur) * cap;
    k_rs_count<<<grid, RS_BLK, 0, s>>>(keys + (int64_t)cur * cap, n_ptr, 8 * p, mask, state, cap);
    k_rs_offsets<<<1u << db, RS_BLK, 0, s>>>(n_ptr, state, cap);
    k_rs_scatter<<<grid, RS_BLK, 0, s>>>(keys + (int64_t)cur * cap, vals + (int64_t)cur * cap,
                                         keys + (int64_t)(1 - cur) * cap, vo, n_ptr, 8 * p, db, state, cap);
    cur = 1 - cur;
  }
  const int rc = (int)hipGetLastError();
  return rc ? -rc : cur;
}

}  // extern "C"

// ============================================================================ index trailer
// Device scratch of the trailer build (zeroed at allocation, re-armed by k_ix_finish).
struct SwIxScratch {
  SwIxHdr h;                 // layout of this step's trailer (k_ix_scan's last workgroup)
  uint64_t tstart;           // trailer offset in the block
  uint64_t cs;               // checksum accumulator
  uint32_t n_alt;
  uint32_t n_chunks[SIX_DIMS];
  uint32_t scans_done;
  uint32_t finish_done;
  uint32_t err;
  uint32_t n_sort;           // rows this step (the radix sort's count)
  uint32_t unsorted;         // some row breaks SIX_F_CLUSTERED (k_ix_prep)
};

#define IX_CHUNK 1024          // bucket rows per wave in the heads pass
#define IX_PREP_BLK 1024
#define IX_LDS_KEYS 16384      // context keys a workgroup counts in LDS (64 KiB)

struct SwIxArgs {
  const SwOutRec* rows;      // this step's rows (persisted order)
  const SwSegAux* aux;       // their encoder aux (SEG_FLAGS)
  const uint8_t* raw;        // non-null when the block carries strings (else no alternate ids)
  const int64_t* cursor;     // [store_cursor, step_cursor0]: rows = cursor[0] - cursor[1]
  const uint64_t* s_alt;     // HBM event ring: alternate-id hash per store row
  int64_t store_cap;
  const int4* asg_ctx;       // (device, customer, area, asset) per assignment
  int64_t n_asg;
  uint8_t* out;              // the block
  int64_t out_cap;
  uint64_t* seg_state;       // the encoder's state: [max_pages + 1] bytes, [+2] errors
  int64_t max_pages;
  uint32_t* snap_host;       // mapped end-of-step snapshot (bytes at [16..17]) or null
  int32_t nk[SIX_DIMS];      // key space per dimension ((max context id + 1) << 3), -1: not indexed
  int32_t nk_off[SIX_DIMS];  // each dimension's offset in a workgroup histogram row
  int32_t nk_total;          // histogram row length
  int32_t lds_all;           // every dimension's keys fit the LDS counters together
  int32_t groups;            // workgroups of k_ix_prep / k_ix_scatter
  uint32_t* skeys;           // [2][cap] alternate-id sort keys
  uint32_t* svals;           // [2][cap] rows
  uint32_t* rstate;          // radix sort state
  uint32_t* whist;           // [groups][nk_total] per-workgroup key counts, then its bucket offsets
  uint32_t* ccnt;            // [3][SIX_KEYS] rows per key
  uint32_t* coff;            // [3][SIX_KEYS] bucket start
  uint32_t* ckeys;           // [3][SIX_KEYS] present keys in order
  uint4* krec;               // [3][SIX_KEYS][2] by present rank: key, rows, bucket start, first head,
                             // first partial slot, first chunk (IxKeyRec)
  uint32_t* cmap;            // [3][mcap] chunk -> present rank of its key
  int64_t mcap;
  uint32_t* cdone;           // [3][SIX_KEYS] by present rank: chunks finished (re-armed by the merger)
  uint32_t* brow;            // [3][cap] bucket rows
  int64_t* bdate;            // [3][cap] bucket dates
  int64_t* part;             // [3][pcap][2 + 2 * SIX_HEADS] chunk partials: min, max, (date, row) x 16
  int64_t pcap;
  SwIxScratch* sc;
  int64_t cap;               // rows capacity
  uint64_t* stamps;          // profiling (null: off): per heads chunk [start, loaded, selected, done]
};

#define IX_PART_WORDS (2 + 2 * SIX_HEADS)

// what a chunk needs of its key, in one 32-byte load
struct IxKeyRec {
  uint32_t key, cnt, off, hoff, pch, chunk0, pad0, pad1;
};

__device__ __forceinline__ int64_t ix_rows(const SwIxArgs& a) {
  const int64_t n = a.cursor[0] - a.cursor[1];
  return n < 0 ? 0 : (n > a.cap ? a.cap : n);
}
__device__ __forceinline__ int32_t ix_ctx(const SwIxArgs& a, int32_t asg, int d) {
  if (asg < 0 || asg >= a.n_asg) return -1;
  const int4 c = a.asg_ctx[asg];
  return d == 0 ? c.y : d == 1 ? c.z : c.w;
}
__device__ __forceinline__ bool ix_encoder_failed(const SwIxArgs& a) {
  return a.seg_state[a.max_pages + 2] != 0;
}
__device__ __forceinline__ void ix_range(const SwIxArgs& a, int64_t n, int64_t* r0, int64_t* r1) {
  const int64_t per = ((n + a.groups - 1) / a.groups + 63) & ~63ll;
  *r0 = (int64_t)blockIdx.x * per;
  *r1 = *r0 + per < n ? *r0 + per : n;
}
// the key of row o in dimension d (-1: none)
__device__ __forceinline__ int32_t ix_key(const SwIxArgs& a, const SwOutRec& o, int d) {
  if (a.nk[d] <= 0) return -1;
  const int32_t c = ix_ctx(a, o.assignment, d);
  if (c < 0) return -1;
  const int32_t k = (c << 3) | (int32_t)(o.etype & 7u);
  return k < a.nk[d] ? k : -1;
}
// dimensions counted in pass p of a workgroup sweep (all at once when they fit the LDS together)
__device__ __forceinline__ bool ix_in_pass(const SwIxArgs& a, int d, int p) { return a.lds_all ? true : d == p; }
__device__ __forceinline__ bool ix_lds_dim(const SwIxArgs& a, int d) { return a.lds_all || a.nk[d] <= IX_LDS_KEYS; }

// ---- per row: alternate-id sort key; per workgroup: its rows' context key histogram
__global__ __launch_bounds__(IX_PREP_BLK) void k_ix_prep(SwIxArgs a) {
  __shared__ uint32_t lc[IX_LDS_KEYS];
  __shared__ uint32_t lalt;
  const int64_t n = ix_rows(a);
  if (blockIdx.x == 0 && threadIdx.x == 0) a.sc->n_sort = (uint32_t)n;
  int64_t r0, r1;
  ix_range(a, n, &r0, &r1);
  uint32_t* hrow = a.whist + (int64_t)blockIdx.x * a.nk_total;
  if (threadIdx.x == 0) lalt = 0;
  const int64_t c0 = a.cursor[1];
  uint32_t nalt = 0;
  for (int64_t j = r0 + threadIdx.x; j < r1; j += IX_PREP_BLK) {
    const bool has = a.raw && (a.aux[j].flags & SEGF_HAS_ALT);
    uint32_t key = 1u << SIX_ALT_SORT_BITS;
    if (has) {
      key = six_sort_key(a.s_alt[(c0 + j) % a.store_cap]);
      ++nalt;
    }
    a.skeys[j] = key;
    a.svals[j] = (uint32_t)j;
  }
  for (int off = 32; off >= 1; off >>= 1) nalt += __shfl_xor(nalt, off, 64);
  // SIX_F_CLUSTERED: persisted rows first, their assignments non-decreasing (row j against j - 1)
  bool bad = false;
  for (int64_t j = r0 + threadIdx.x; j < r1; j += IX_PREP_BLK) {
    if (j == 0) continue;
    const bool g0 = a.aux && (a.aux[j - 1].flags & SEGF_GEN), g1 = a.aux && (a.aux[j].flags & SEGF_GEN);
    bad |= (g0 && !g1) || (!g0 && !g1 && a.rows[j].assignment < a.rows[j - 1].assignment);
  }
  if (__ballot(bad) && ix_lane() == 0) atomicOr(&a.sc->unsorted, 1u);
  __syncthreads();
  if (ix_lane() == 0 && nalt) atomicAdd(&lalt, nalt);
  // context keys, one sweep per LDS pass
  const int npass = a.lds_all ? 1 : SIX_DIMS;
  for (int p = 0; p < npass; ++p) {
    bool any = false;
    for (int d = 0; d < SIX_DIMS; ++d) any |= ix_in_pass(a, d, p) && a.nk[d] > 0;
    if (!any) continue;
    const bool lds = a.lds_all || ix_lds_dim(a, p);
    const int32_t span = a.lds_all ? a.nk_total : (a.nk[p] > 0 ? a.nk[p] : 0);
    const int32_t obase = a.lds_all ? 0 : a.nk_off[p];
    for (int32_t i = threadIdx.x; i < span; i += IX_PREP_BLK) {
      if (lds) lc[i] = 0;
      else hrow[obase + i] = 0;
    }
    __syncthreads();
    if (!lds) __threadfence_block();
    for (int64_t j = r0 + threadIdx.x; j < r1; j += IX_PREP_BLK) {
      const SwOutRec o = a.rows[j];
#pragma unroll
      for (int d = 0; d < SIX_DIMS; ++d) {
        if (!ix_in_pass(a, d, p)) continue;
        const int32_t k = ix_key(a, o, d);
        if (k < 0) continue;
        const int32_t at = (a.lds_all ? a.nk_off[d] : 0) + k;
        if (lds) atomicAdd(&lc[at], 1u);
        else atomicAdd(&hrow[obase + at], 1u);
      }
    }
    __syncthreads();
    if (lds)
      for (int32_t i = threadIdx.x; i < span; i += IX_PREP_BLK) hrow[obase + i] = lc[i];
    __syncthreads();
  }
  // every wave's count is in lalt before thread 0 reads it: the passes above synchronise only when
  // some context dimension is indexed (a tenant without customers / areas / assets has none)
  __syncthreads();
  if (threadIdx.x == 0 && lalt) atomicAdd(&a.sc->n_alt, lalt);
}

// ---- per key (every dimension, one thread each): its total over the workgroup histograms and each
// workgroup's offset in the key's bucket (the column prefix, written in place)
__global__ __launch_bounds__(256) void k_ix_colscan(SwIxArgs a) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= a.nk_total) return;
  int d = 0;
  while (d + 1 < SIX_DIMS && k >= a.nk_off[d + 1]) ++d;
  if (a.nk[d] <= 0 || k - a.nk_off[d] >= a.nk[d]) return;
  uint32_t acc = 0;
  const int64_t stride = a.nk_total;
  int w = 0;
  for (; w + 8 <= a.groups; w += 8) {
    uint32_t v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = a.whist[(int64_t)(w + i) * stride + k];
#pragma unroll
    for (int i = 0; i < 8; ++i) { a.whist[(int64_t)(w + i) * stride + k] = acc; acc += v[i]; }
  }
  for (; w < a.groups; ++w) {
    const uint32_t v = a.whist[(int64_t)w * stride + k];
    a.whist[(int64_t)w * stride + k] = acc;
    acc += v;
  }
  a.ccnt[(int64_t)d * SIX_KEYS + (k - a.nk_off[d])] = acc;
}

// ---- one workgroup per dimension: bucket starts, present-key ranks, head / chunk / partial offsets;
// the last one lays the trailer out
#define IX_SCAN_BLK 1024
#define IX_NQ 5
__global__ __launch_bounds__(IX_SCAN_BLK) void k_ix_scan(SwIxArgs a) {
  __shared__ uint32_t wsum[IX_NQ][IX_SCAN_BLK / 64];
  __shared__ uint32_t last;
  const int d = blockIdx.x;
  const bool indexed = a.nk[d] >= 0;
  const uint32_t nk = indexed ? (uint32_t)a.nk[d] : 0u;
  uint32_t* cnt = a.ccnt + (int64_t)d * SIX_KEYS;
  // scans over the keys (totals from k_ix_colscan): rows, present keys, heads, chunks, partial slots
  const uint32_t per = (nk + IX_SCAN_BLK - 1) / IX_SCAN_BLK;
  const uint32_t k0 = threadIdx.x * per, k1 = k0 + per < nk ? k0 + per : nk;
  uint32_t v[IX_NQ] = {0, 0, 0, 0, 0};
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t c = cnt[k];
    const uint32_t nch = (c + IX_CHUNK - 1) / IX_CHUNK;
    v[0] += c;
    v[1] += c ? 1u : 0u;
    v[2] += c < SIX_HEADS ? c : SIX_HEADS;
    v[3] += nch;
    v[4] += nch > 1 ? nch : 0u;
  }
  const uint32_t lane = ix_lane(), wid = threadIdx.x >> 6;
  uint32_t inc[IX_NQ];
#pragma unroll
  for (int q = 0; q < IX_NQ; ++q) {
    inc[q] = v[q];
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = __shfl_up(inc[q], o, 64);
      if (lane >= (uint32_t)o) inc[q] += x;
    }
    if (lane == 63) wsum[q][wid] = inc[q];
  }
  __syncthreads();
  if (threadIdx.x < IX_NQ) {
    uint32_t acc = 0;
    for (int w = 0; w < IX_SCAN_BLK / 64; ++w) { const uint32_t x = wsum[threadIdx.x][w]; wsum[threadIdx.x][w] = acc; acc += x; }
    if (threadIdx.x == 1) a.sc->h.n_keys[d] = indexed ? acc : SIX_NOT_INDEXED;
    if (threadIdx.x == 2) a.sc->h.n_heads[d] = indexed ? acc : 0u;
    if (threadIdx.x == 3) a.sc->n_chunks[d] = indexed ? acc : 0u;
  }
  __syncthreads();
  uint32_t pr = inc[0] - v[0] + wsum[0][wid], pk = inc[1] - v[1] + wsum[1][wid], ph = inc[2] - v[2] + wsum[2][wid];
  uint32_t pc = inc[3] - v[3] + wsum[3][wid], pp = inc[4] - v[4] + wsum[4][wid];
  const int64_t db = (int64_t)d * SIX_KEYS;
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t c = cnt[k];
    const uint32_t nch = (c + IX_CHUNK - 1) / IX_CHUNK;
    a.coff[db + k] = pr;
    if (c) {
      a.ckeys[db + pk] = k;
      IxKeyRec r;
      r.key = k; r.cnt = c; r.off = pr; r.hoff = ph; r.pch = pp; r.chunk0 = pc; r.pad0 = 0; r.pad1 = 0;
      *reinterpret_cast<IxKeyRec*>(a.krec + 2 * (db + pk)) = r;
      uint32_t* cm = a.cmap + (int64_t)d * a.mcap;
      for (uint32_t x = 0; x < nch && pc + x < a.mcap; ++x) cm[pc + x] = pk;
    }
    pr += c;
    pk += c ? 1u : 0u;
    ph += c < SIX_HEADS ? c : SIX_HEADS;
    pc += nch;
    pp += nch > 1 ? nch : 0u;
  }
  if ((pp > a.pcap || pc > a.mcap) && threadIdx.x == IX_SCAN_BLK - 1) atomicOr(&a.sc->err, 2u);
  // ---- last workgroup out: the layout
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(&a.sc->scans_done, 1u) == (uint32_t)gridDim.x - 1;
  __syncthreads();
  if (!last || threadIdx.x != 0) return;
  __threadfence();
  SwIxScratch* sc = a.sc;
  const int64_t n = ix_rows(a);
  const int64_t np = (n + SEG_PAGE_ROWS - 1) / SEG_PAGE_ROWS;
  SwIxHdr h;
  for (int i = 0; i < (int)(sizeof(SwIxHdr) / 4); ++i) reinterpret_cast<uint32_t*>(&h)[i] = 0;
  h.magic = SIX_MAGIC;
  h.version = SIX_VERSION;
  h.n_dims = SIX_DIMS;
  h.n_rows = (uint32_t)n;
  h.n_pages = (uint32_t)np;
  h.n_alt = atomicAdd(&sc->n_alt, 0u);
  h.alt_bits = six_alt_bits(h.n_alt);
  h.alt_pbits = six_page_bits((uint32_t)np);
  h.flags = __hip_atomic_load(&sc->unsorted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? 0u : SIX_F_CLUSTERED;
  for (int q = 0; q < SIX_DIMS; ++q) {
    h.n_keys[q] = __hip_atomic_load(&sc->h.n_keys[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    h.n_heads[q] = __hip_atomic_load(&sc->h.n_heads[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const uint32_t tb = six_layout(&h);
  const uint32_t* pt = reinterpret_cast<const uint32_t*>(a.out + 64);
  const uint64_t tstart = pt[np];
  sc->h = h;
  sc->tstart = tstart;
  if (ix_encoder_failed(a) || (tstart & 7) || (int64_t)(tstart + tb) > a.out_cap) {
    sc->err |= 1;
    return;
  }
  if (sc->err) return;
  // header words (checksum 0 for now) and the head-row sections' padding word
  uint8_t* t = a.out + tstart;
  const uint64_t* hw = reinterpret_cast<const uint64_t*>(&h);
  for (uint32_t i = 0; i < SIX_HDR_BYTES / 8; ++i) reinterpret_cast<uint64_t*>(t)[i] = hw[i];
  for (int q = 0; q < SIX_DIMS; ++q)
    if (h.n_heads[q] & 1u) *reinterpret_cast<uint32_t*>(t + h.off_heads[q] + 4u * h.n_heads[q]) = 0u;
  SwSegBlockHdr* bh = reinterpret_cast<SwSegBlockHdr*>(a.out);
  bh->flags = SEG_FLAG_INDEX;
  bh->bytes = tstart + tb;
}

// ---- (row, date) into the key buckets: the workgroup's reserved run of each key (k_ix_scan), then a
// local rank (LDS counter; order inside a bucket is free: every per-key output is order-independent)
__global__ __launch_bounds__(IX_PREP_BLK) void k_ix_scatter(SwIxArgs a) {
  __shared__ uint32_t lc[IX_LDS_KEYS];
  if (a.sc->err) return;
  const int64_t n = ix_rows(a);
  int64_t r0, r1;
  ix_range(a, n, &r0, &r1);
  uint32_t* hrow = a.whist + (int64_t)blockIdx.x * a.nk_total;
  const int npass = a.lds_all ? 1 : SIX_DIMS;
  for (int p = 0; p < npass; ++p) {
    bool any = false;
    for (int d = 0; d < SIX_DIMS; ++d) any |= ix_in_pass(a, d, p) && a.nk[d] > 0;
    if (!any) continue;
    const bool lds = a.lds_all || ix_lds_dim(a, p);
    const int32_t span = a.lds_all ? a.nk_total : (a.nk[p] > 0 ? a.nk[p] : 0);
    const int32_t obase = a.lds_all ? 0 : a.nk_off[p];
    // the workgroup's next position in every key's bucket, in LDS (one LDS atomic per row and key)
    if (lds)
      for (int32_t i = threadIdx.x; i < span; i += IX_PREP_BLK) {
        int d = 0;
        const int32_t at = obase + i;
        while (d + 1 < SIX_DIMS && at >= a.nk_off[d + 1]) ++d;
        const int32_t k = at - a.nk_off[d];
        lc[i] = k < (a.nk[d] > 0 ? a.nk[d] : 0) ? a.coff[(int64_t)d * SIX_KEYS + k] + hrow[at] : 0u;
      }
    __syncthreads();
    for (int64_t j = r0 + threadIdx.x; j < r1; j += IX_PREP_BLK) {
      const SwOutRec o = a.rows[j];
#pragma unroll
      for (int d = 0; d < SIX_DIMS; ++d) {
        if (!ix_in_pass(a, d, p)) continue;
        const int32_t k = ix_key(a, o, d);
        if (k < 0) continue;
        const int32_t at = a.nk_off[d] + k;
        const uint32_t pos = lds ? atomicAdd(&lc[at - obase], 1u)
                                 : a.coff[(int64_t)d * SIX_KEYS + k] + atomicAdd(&hrow[at], 1u);
        a.brow[(int64_t)d * a.cap + pos] = (uint32_t)j;
        a.bdate[(int64_t)d * a.cap + pos] = o.event_date;
      }
    }
    __syncthreads();
  }
}

// ---- page zone maps, alternate-id directory + entries
#define IX_WRITE_WGS 1024
#define IX_WBLK 256
__device__ __forceinline__ void ix_write_pages(const SwIxArgs& a, const SwIxHdr& h, uint8_t* t, int64_t gtid, int64_t gthreads) {
  const uint32_t* pt = reinterpret_cast<const uint32_t*>(a.out + 64);
  for (int64_t p = gtid; p < h.n_pages; p += gthreads) {
    const SwSegPageHdr* ph = reinterpret_cast<const SwSegPageHdr*>(a.out + pt[p]);
    SwIxPage z;
    z.asg_min = (int32_t)seg_unord(ph->cols[SEG_ASG].base);
    z.asg_max = ph->asg_max;
    z.date_min = seg_unord(ph->cols[SEG_DATE].base);
    z.date_max = ph->date_max;
    z.off = pt[p];
    z.bytes = pt[p + 1] - pt[p];
    *reinterpret_cast<SwIxPage*>(t + h.off_pages + p * sizeof(SwIxPage)) = z;
  }
  // directory: dir[b] = entries whose bucket is < b (lower bound in the sorted keys, buffer 0)
  const uint32_t* sk = a.skeys;
  const uint32_t nb = 1u << h.alt_bits, sh = SIX_ALT_SORT_BITS - h.alt_bits;
  const uint32_t dwords = (nb + 2u) / 2u;  // (nb + 1) u32 entries, padded to u64 words
  for (int64_t w = gtid; w < dwords; w += gthreads) {
    uint32_t e[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const uint32_t b = 2u * (uint32_t)w + q;
      if (b > nb) { e[q] = 0; continue; }
      if (b == nb) { e[q] = h.n_alt; continue; }
      const uint32_t target = b << sh;
      uint32_t lo = 0, hi = h.n_alt;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sk[mid] < target) lo = mid + 1; else hi = mid;
      }
      e[q] = lo;
    }
    *reinterpret_cast<ull*>(t + h.off_alt_dir + 8 * w) = (ull)e[0] | ((ull)e[1] << 32);
  }
  // entries, one u64 word per thread (entries straddle words)
  const uint32_t nw = six_alt_words(h.n_alt);
  const int64_t c0 = a.cursor[1];
  for (int64_t w = gtid; w < nw; w += gthreads) {
    const uint64_t b0 = (uint64_t)w * 64, b1 = b0 + 64;
    const uint32_t i0 = (uint32_t)(b0 / SIX_ALT_EBITS);
    uint32_t i1 = (uint32_t)((b1 + SIX_ALT_EBITS - 1) / SIX_ALT_EBITS);
    if (i1 > h.n_alt) i1 = h.n_alt;
    ull word = 0;
    for (uint32_t i = i0; i < i1; ++i) {
      const uint32_t row = a.svals[i];
      const uint64_t hv = a.s_alt[(c0 + row) % a.store_cap];
      const ull v = six_entry(hv, h.alt_bits, h.alt_pbits, row / SEG_PAGE_ROWS);
      const int64_t bp = (int64_t)i * SIX_ALT_EBITS - (int64_t)b0;     // entry start relative to the word
      if (bp >= 0) word |= v << bp;
      else word |= v >> (-bp);
    }
    *reinterpret_cast<ull*>(t + h.off_alt + 8 * w) = word;
  }
}

// ---- heads.  A wave takes up to 1024 (date, row) items, 16 per lane: each lane sorts its 16 in
// registers (bitonic network, newest first), then 16 rounds each take the wave's newest remaining
// item -- a DPP max over the lanes' heads (VALU lane moves; no LDS round trip, no ds_bpermute
// chain), the winning lane shifts its list.  A key of several chunks leaves one partial top-16 per
// chunk; k_ix_merge folds them (the kernel boundary publishes the partials: no device-scope fence,
// which on this chip writes back the XCD's whole L2).
#define IX_SLOTS 16

template <int CTRL, int RM = 0xf, int BM = 0xf>
__device__ __forceinline__ uint32_t ix_dpp(uint32_t v, uint32_t old) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, RM, BM, false);
}
// wave-wide max of an unsigned 64-bit value, broadcast (row_shr 1/2/4/8, row_bcast 15/31, lane 63)
__device__ __forceinline__ ull ix_wave_max64(ull v) {
#define IX_M64(C, R) { const ull o = ((ull)ix_dpp<C, R>((uint32_t)(v >> 32), 0u) << 32) | ix_dpp<C, R>((uint32_t)v, 0u); \
                       v = o > v ? o : v; }
  IX_M64(0x111, 0xf) IX_M64(0x112, 0xf) IX_M64(0x114, 0xf) IX_M64(0x118, 0xf) IX_M64(0x142, 0xa) IX_M64(0x143, 0xc)
#undef IX_M64
  return ((ull)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63) << 32) |
         (ull)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
}
__device__ __forceinline__ uint32_t ix_wave_max32(uint32_t v) {
#define IX_M32(C, R) { const uint32_t o = ix_dpp<C, R>(v, 0u); v = o > v ? o : v; }
  IX_M32(0x111, 0xf) IX_M32(0x112, 0xf) IX_M32(0x114, 0xf) IX_M32(0x118, 0xf) IX_M32(0x142, 0xa) IX_M32(0x143, 0xc)
#undef IX_M32
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ ull ix_ord(int64_t d) { return (ull)d ^ 0x8000000000000000ull; }

// the lane's items sorted newest first: K = ordered date, R = row (compare-exchange network)
__device__ __forceinline__ void ix_sort16(ull (&K)[IX_SLOTS], uint32_t (&R)[IX_SLOTS]) {
#pragma unroll
  for (int k = 2; k <= IX_SLOTS; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int i = 0; i < IX_SLOTS; ++i) {
        const int l = i ^ j;
        if (l > i) {
          // descending within blocks whose (i & k) == 0, ascending otherwise: a bitonic sort to
          // one descending run
          const bool desc = (i & k) == 0;
          const bool gt = K[l] > K[i] || (K[l] == K[i] && R[l] > R[i]);      // l newer than i
          const bool sw = desc ? gt : !gt;
          const ull tk = sw ? K[l] : K[i];
          const uint32_t tr = sw ? R[l] : R[i];
          K[l] = sw ? K[i] : K[l];
          R[l] = sw ? R[i] : R[l];
          K[i] = tk;
          R[i] = tr;
        }
      }
    }
  }
}

// k rounds of wave argmax over the lanes' sorted lists (n = the lane's valid items); lane r < k ends
// with the r-th newest in (od, orow)
__device__ __forceinline__ void ix_take(ull (&K)[IX_SLOTS], uint32_t (&R)[IX_SLOTS], int n, uint32_t k, int64_t& od,
                                        uint32_t& orow) {
  const uint32_t lane = ix_lane();
  od = INT64_MIN;
  orow = 0;
  for (uint32_t r = 0; r < k; ++r) {
    const bool have = n > 0;
    // newest date over the lanes that still hold items, then the highest row among its holders
    // (lanes without items offer 0 and can never win the row round: exact for every date)
    const ull hk = have ? K[0] : 0ull;
    const ull mk = ix_wave_max64(hk);
    const uint32_t cr = (have && hk == mk) ? R[0] + 1u : 0u;
    const uint32_t mr = ix_wave_max32(cr);
    if (lane == r) { od = (int64_t)(mk ^ 0x8000000000000000ull); orow = mr - 1u; }
    if (have && hk == mk && cr == mr) {                 // rows are unique: one lane wins
#pragma unroll
      for (int s = 0; s + 1 < IX_SLOTS; ++s) { K[s] = K[s + 1]; R[s] = R[s + 1]; }
      --n;
    }
  }
}

__device__ __forceinline__ void wave_minmax(int64_t& mn, int64_t& mx) {
  const ull a = ix_wave_max64(ix_ord(mx));
  const ull b = ix_wave_max64(~ix_ord(mn));
  mx = (int64_t)(a ^ 0x8000000000000000ull);
  mn = (int64_t)((~b) ^ 0x8000000000000000ull);
}

// the key's summary and heads (lane r < nh carries head r)
__device__ void ix_write_final(const SwIxArgs& a, const SwIxHdr& h, uint8_t* t, int d, uint32_t q, uint32_t k,
                               uint32_t cnt, uint32_t hoff, int64_t mn, int64_t mx, int64_t cd, uint32_t cr) {
  const uint32_t nh = cnt < SIX_HEADS ? cnt : SIX_HEADS;
  const uint32_t lane = ix_lane();
  if (lane < nh) {
    reinterpret_cast<uint32_t*>(t + h.off_heads[d])[hoff + lane] = cr;
    reinterpret_cast<int64_t*>(t + h.off_hdates[d])[hoff + lane] = cd;
  }
  if (lane == 0) {
    SwIxKey e;
    e.key = k;
    e.count = cnt;
    e.date_min = mn;
    e.date_max = mx;
    e.head_off = hoff;
    e.n_heads = nh;
    *reinterpret_cast<SwIxKey*>(t + h.off_keys[d] + (uint64_t)q * sizeof(SwIxKey)) = e;
  }
}

// load up to 1024 (date, row) items, 16 per lane (item i = base + lane + 64 s): sorted, counted
template <typename F>
__device__ __forceinline__ int ix_load16(uint32_t nitems, F item, ull (&K)[IX_SLOTS], uint32_t (&R)[IX_SLOTS],
                                         int64_t& mn, int64_t& mx) {
  const uint32_t lane = ix_lane();
  int n = 0;
#pragma unroll
  for (int s = 0; s < IX_SLOTS; ++s) {
    const uint32_t i = lane + 64u * s;
    int64_t dt = INT64_MIN;
    uint32_t row = 0;
    if (i < nitems) {
      item(i, dt, row);
      mn = dt < mn ? dt : mn;
      mx = dt > mx ? dt : mx;
      ++n;
    }
    K[s] = i < nitems ? ix_ord(dt) : 0ull;
    R[s] = row;
  }
  ix_sort16(K, R);
  return n;
}

// one chunk (up to IX_CHUNK bucket rows) of present key q of dimension d
__device__ void ix_chunk(const SwIxArgs& a, const SwIxHdr& h, uint8_t* t, int d, uint32_t q, const IxKeyRec& kr,
                         uint32_t c) {
  const uint32_t k = kr.key, cnt = kr.cnt;
  const uint32_t nch = (cnt + IX_CHUNK - 1) / IX_CHUNK;
  const uint32_t lo = kr.off + c * IX_CHUNK;
  const uint32_t rows_c = cnt - c * IX_CHUNK < IX_CHUNK ? cnt - c * IX_CHUNK : IX_CHUNK;
  const uint32_t* br = a.brow + (int64_t)d * a.cap + lo;
  const int64_t* bd = a.bdate + (int64_t)d * a.cap + lo;
  uint64_t* stp = a.stamps ? a.stamps + 4 * ((int64_t)d * a.mcap + kr.chunk0 + c) : nullptr;
  ull K[IX_SLOTS];
  uint32_t R[IX_SLOTS];
  int64_t mn = INT64_MAX, mx = INT64_MIN;
  const int n = ix_load16(rows_c, [&](uint32_t i, int64_t& dt, uint32_t& row) { dt = bd[i]; row = br[i]; }, K, R, mn, mx);
  wave_minmax(mn, mx);
  if (stp && ix_lane() == 0) stp[1] = __builtin_amdgcn_s_memrealtime();
  int64_t cd;
  uint32_t cr;
  ix_take(K, R, n, rows_c < SIX_HEADS ? rows_c : SIX_HEADS, cd, cr);
  if (stp && ix_lane() == 0) stp[2] = __builtin_amdgcn_s_memrealtime();
  if (nch == 1) {
    ix_write_final(a, h, t, d, q, k, cnt, kr.hoff, mn, mx, cd, cr);
    return;
  }
  // a partial of a multi-chunk key (k_ix_merge folds them): min, max, its top-16
  int64_t* P = a.part + ((int64_t)d * a.pcap + kr.pch + c) * IX_PART_WORDS;
  const uint32_t lane = ix_lane();
  if (lane < SIX_HEADS) { P[2 + 2 * lane] = cd; P[3 + 2 * lane] = (int64_t)cr; }
  if (lane == 0) { P[0] = mn; P[1] = mx; }
}

// fold a multi-chunk key's partials: 64 partials (1024 candidates) per round, in place, until one
// is left (keys of more than 64K rows need more than one round)
__device__ void ix_merge_key(const SwIxArgs& a, const SwIxHdr& h, uint8_t* t, int d, uint32_t q, const IxKeyRec& kr) {
  const uint32_t cnt = kr.cnt;
  uint32_t np = (cnt + IX_CHUNK - 1) / IX_CHUNK;          // partials left
  int64_t* P0 = a.part + ((int64_t)d * a.pcap + kr.pch) * IX_PART_WORDS;
  // heads held by partial j: a short last chunk holds fewer
  uint32_t last_heads = cnt - (np - 1) * IX_CHUNK < SIX_HEADS ? cnt - (np - 1) * IX_CHUNK : SIX_HEADS;
  int64_t cd = INT64_MIN, mn = INT64_MAX, mx = INT64_MIN;
  uint32_t cr = 0;
  while (true) {
    const uint32_t groups = (np + 63) / 64;
    for (uint32_t gi = 0; gi < groups; ++gi) {
      const uint32_t j0 = gi * 64, j1 = j0 + 64 < np ? j0 + 64 : np;
      const uint32_t items = (j1 - j0) * SIX_HEADS;
      ull K[IX_SLOTS];
      uint32_t R[IX_SLOTS];
      int64_t gmn = INT64_MAX, gmx = INT64_MIN;
      int n = 0;
      const uint32_t lane = ix_lane();
#pragma unroll
      for (int s = 0; s < IX_SLOTS; ++s) {
        const uint32_t i = lane + 64u * s;
        const uint32_t j = j0 + i / SIX_HEADS, sl = i % SIX_HEADS;
        const bool ok = i < items && (j + 1 < np || sl < last_heads);
        const int64_t* p = P0 + (int64_t)j * IX_PART_WORDS;
        K[s] = ok ? ix_ord(p[2 + 2 * sl]) : 0ull;
        R[s] = ok ? (uint32_t)p[3 + 2 * sl] : 0u;
        n += ok ? 1 : 0;
        if (i < items && sl == 0) { gmn = p[0] < gmn ? p[0] : gmn; gmx = p[1] > gmx ? p[1] : gmx; }
      }
      ix_sort16(K, R);
      wave_minmax(gmn, gmx);
      const uint32_t tot = (j1 - j0) * SIX_HEADS - (j1 == np ? SIX_HEADS - last_heads : 0u);
      ix_take(K, R, n, tot < SIX_HEADS ? tot : SIX_HEADS, cd, cr);
      mn = gmn;
      mx = gmx;
      if (groups > 1) {                                   // the group's fold becomes partial gi
        int64_t* P = P0 + (int64_t)gi * IX_PART_WORDS;
        if (lane < SIX_HEADS) { P[2 + 2 * lane] = cd; P[3 + 2 * lane] = (int64_t)cr; }
        if (lane == 0) { P[0] = gmn; P[1] = gmx; }
      }
    }
    if (groups == 1) break;
    last_heads = SIX_HEADS;
    np = groups;
  }
  ix_write_final(a, h, t, d, q, kr.key, cnt, kr.hoff, mn, mx, cd, cr);
}

__global__ __launch_bounds__(IX_WBLK) void k_ix_write(SwIxArgs a) {
  if (a.sc->err) return;
  const SwIxHdr h = a.sc->h;
  uint8_t* t = a.out + a.sc->tstart;
  ix_write_pages(a, h, t, (int64_t)blockIdx.x * IX_WBLK + threadIdx.x, (int64_t)gridDim.x * IX_WBLK);
}

__global__ __launch_bounds__(IX_WBLK) void k_ix_heads(SwIxArgs a) {
  if (a.sc->err) return;
  const SwIxHdr& h = a.sc->h;             // fields indexed by dimension: read in place (a private copy
                                          // indexed at run time would live in scratch memory)
  uint8_t* t = a.out + a.sc->tstart;
  // one wave per chunk of every indexed dimension's keys
  // (scalars per dimension, not arrays: a run-time index into a private array spills to scratch)
  const uint32_t nk0 = h.n_keys[0] == SIX_NOT_INDEXED ? 0u : h.n_keys[0];
  const uint32_t nk1 = h.n_keys[1] == SIX_NOT_INDEXED ? 0u : h.n_keys[1];
  const uint32_t nk2 = h.n_keys[2] == SIX_NOT_INDEXED ? 0u : h.n_keys[2];
  const uint32_t nc0 = nk0 ? a.sc->n_chunks[0] : 0u, nc1 = nk1 ? a.sc->n_chunks[1] : 0u;
  const uint32_t nc2 = nk2 ? a.sc->n_chunks[2] : 0u;
  const uint32_t total = nc0 + nc1 + nc2;
  const uint32_t wave = blockIdx.x * (IX_WBLK / 64) + (threadIdx.x >> 6), nwaves = gridDim.x * (IX_WBLK / 64);
  for (uint32_t g = wave; g < total; g += nwaves) {
    const int d = g < nc0 ? 0 : g < nc0 + nc1 ? 1 : 2;
    const uint32_t gc = d == 0 ? g : d == 1 ? g - nc0 : g - nc0 - nc1;
    const uint64_t t0 = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint32_t q = a.cmap[(int64_t)d * a.mcap + gc];
    const IxKeyRec kr = *reinterpret_cast<const IxKeyRec*>(a.krec + 2 * ((int64_t)d * SIX_KEYS + q));
    ix_chunk(a, h, t, d, q, kr, gc - kr.chunk0);
    if (a.stamps && ix_lane() == 0) {
      uint64_t* stp = a.stamps + 4 * ((int64_t)d * a.mcap + gc);
      stp[0] = t0;
      stp[3] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

// ---- one wave per present key of several chunks: fold its chunks' partials
__global__ __launch_bounds__(IX_WBLK) void k_ix_merge(SwIxArgs a) {
  if (a.sc->err) return;
  const SwIxHdr& h = a.sc->h;
  uint8_t* t = a.out + a.sc->tstart;
  const uint32_t nk0 = h.n_keys[0] == SIX_NOT_INDEXED ? 0u : h.n_keys[0];
  const uint32_t nk1 = h.n_keys[1] == SIX_NOT_INDEXED ? 0u : h.n_keys[1];
  const uint32_t nk2 = h.n_keys[2] == SIX_NOT_INDEXED ? 0u : h.n_keys[2];
  const uint32_t total = nk0 + nk1 + nk2;
  const uint32_t wave = blockIdx.x * (IX_WBLK / 64) + (threadIdx.x >> 6), nwaves = gridDim.x * (IX_WBLK / 64);
  for (uint32_t g = wave; g < total; g += nwaves) {
    const int d = g < nk0 ? 0 : g < nk0 + nk1 ? 1 : 2;
    const uint32_t q = d == 0 ? g : d == 1 ? g - nk0 : g - nk0 - nk1;
    const IxKeyRec kr = *reinterpret_cast<const IxKeyRec*>(a.krec + 2 * ((int64_t)d * SIX_KEYS + q));
    if (kr.cnt > IX_CHUNK) ix_merge_key(a, h, t, d, q, kr);
  }
}

// ---- checksum of the whole trailer; the last workgroup publishes and re-arms
__global__ __launch_bounds__(IX_WBLK) void k_ix_finish(SwIxArgs a) {
  __shared__ ull red[IX_WBLK / 64];
  __shared__ uint32_t last;
  SwIxScratch* sc = a.sc;
  const bool ok = !sc->err;
  ull cs = 0;
  if (ok) {
    const uint8_t* t = a.out + sc->tstart;
    const uint64_t words = sc->h.bytes / 8;
    for (uint64_t i = (uint64_t)blockIdx.x * IX_WBLK + threadIdx.x; i < words; i += (uint64_t)gridDim.x * IX_WBLK)
      if (i != SIX_CHECKSUM_WORD) cs ^= seg_mix_word(reinterpret_cast<const ull*>(t)[i], i);
  }
  for (int off = 32; off >= 1; off >>= 1) cs ^= __shfl_xor(cs, off, 64);
  if (ix_lane() == 0) red[threadIdx.x >> 6] = cs;
  __syncthreads();
  if (threadIdx.x == 0) {
    ull x = 0;
    for (int w = 0; w < IX_WBLK / 64; ++w) x ^= red[w];
    if (x) atomicXor(reinterpret_cast<ull*>(&sc->cs), x);
    __threadfence();
    last = atomicAdd(&sc->finish_done, 1u) == (uint32_t)gridDim.x - 1;
  }
  __syncthreads();
  if (!last || threadIdx.x != 0) return;
  __threadfence();
  const ull total_cs = atomicXor(reinterpret_cast<ull*>(&sc->cs), 0ull);
  const uint64_t bytes = sc->tstart + sc->h.bytes;
  if (ok) {
    reinterpret_cast<ull*>(a.out + sc->tstart)[SIX_CHECKSUM_WORD] = total_cs;
    a.seg_state[a.max_pages + 1] = bytes;
    if (a.snap_host) { a.snap_host[16] = (uint32_t)bytes; a.snap_host[17] = (uint32_t)(bytes >> 32); }
  } else if (!ix_encoder_failed(a)) {
    // the trailer could not be built: a loud encoder error, never a block without its index
    a.seg_state[a.max_pages + 2] += 1;
    a.seg_state[a.max_pages + 1] = ~0ull;
    if (a.snap_host) { a.snap_host[16] = ~0u; a.snap_host[17] = ~0u; a.snap_host[18] += 1; }
  }
  sc->cs = 0;
  sc->n_alt = 0;
  sc->unsorted = 0;
  sc->scans_done = 0;
  sc->finish_done = 0;
  sc->err = 0;
}

static int64_t ix_mcap(int64_t cap) { return cap / IX_CHUNK + SIX_KEYS + 1; }

extern "C" {

// Scratch words (u32) of a trailer build for `cap` rows and `groups` x `nk_total` workgroup
// histograms (see SwIxArgs; the host sizes it from the context key spaces).
static int64_t ix_pcap(int64_t cap) { return 2 * (cap / IX_CHUNK) + 2; }

int64_t sw_seg_index_groups(int64_t cap) {
  const int64_t g = (cap + 4095) / 4096;
  return g < 1 ? 1 : (g > 256 ? 256 : g);
}


int64_t sw_seg_index_scratch_words(int64_t cap, int64_t nk_total) {
  const int64_t g = sw_seg_index_groups(cap);
  return 4 * cap + sw_radix_tmp_words(cap) + g * (nk_total > 0 ? nk_total : 1) + 4ll * SIX_DIMS * SIX_KEYS +
         SIX_DIMS * ix_mcap(cap) + 4 + 8ll * SIX_DIMS * SIX_KEYS +
         SIX_DIMS * cap + 2 * SIX_DIMS * cap + 2 * SIX_DIMS * ix_pcap(cap) * IX_PART_WORDS +
         (int64_t)((sizeof(SwIxScratch) + 15) / 4) + 16;
}

int64_t sw_seg_index_max_bytes(int64_t rows) { return (int64_t)six_max_bytes((uint64_t)rows); }

// stamps buffer words of sw_seg_index (4 per heads chunk, every dimension)
int64_t sw_seg_index_stamp_words(int64_t cap) { return 4ll * SIX_DIMS * ix_mcap(cap); }

// Build the index trailer of the block k_seg_encode just wrote (same stream, same arguments) and
// append it to the block.  nk[d]: key space of dimension d ((max context id + 1) << 3 over the
// engine's assignment table, 0: no context; -1: not indexed -- ids reach SIX_CTX_MAX).  scratch:
// u32[sw_seg_index_scratch_words(cap, sum of the non-negative nk)], zeroed at allocation.
int sw_seg_index(const void* rows, const void* aux, const uint8_t* raw, const int64_t* cursor, const uint64_t* s_alt,
                 int64_t store_cap, const void* asg_ctx, int64_t n_asg, const int32_t* nk, uint8_t* out,
                 int64_t out_cap, uint64_t* seg_state, int64_t max_pages, uint32_t* snap_host, uint32_t* scratch,
                 int64_t cap, uint64_t* stamps, hipStream_t s) {
  SwIxArgs a;
  a.stamps = stamps;
  a.rows = (const SwOutRec*)rows;
  a.aux = (const SwSegAux*)aux;
  a.raw = raw;
  a.cursor = cursor;
  a.s_alt = s_alt;
  a.store_cap = store_cap;
  a.asg_ctx = (const int4*)asg_ctx;
  a.n_asg = n_asg;
  a.out = out;
  a.out_cap = out_cap;
  a.seg_state = seg_state;
  a.max_pages = max_pages;
  a.snap_host = snap_host;
  int32_t tot = 0;
  for (int d = 0; d < SIX_DIMS; ++d) {
    a.nk[d] = nk[d] > SIX_KEYS ? -1 : nk[d];
    a.nk_off[d] = tot;
    tot += a.nk[d] > 0 ? a.nk[d] : 0;
  }
  a.nk_total = tot > 0 ? tot : 1;
  a.lds_all = tot <= IX_LDS_KEYS ? 1 : 0;
  a.groups = (int32_t)sw_seg_index_groups(cap);
  uint32_t* p = scratch;
  a.skeys = p; p += 2 * cap;
  a.svals = p; p += 2 * cap;
  a.rstate = p; p += sw_radix_tmp_words(cap);
  a.whist = p; p += (int64_t)a.groups * a.nk_total;
  a.ccnt = p; p += (int64_t)SIX_DIMS * SIX_KEYS;
  a.coff = p; p += (int64_t)SIX_DIMS * SIX_KEYS;
  a.ckeys = p; p += (int64_t)SIX_DIMS * SIX_KEYS;
  a.cdone = p; p += (int64_t)SIX_DIMS * SIX_KEYS;
  a.mcap = ix_mcap(cap);
  a.cmap = p; p += SIX_DIMS * a.mcap;
  p += (4 - ((uintptr_t)p & 15) / 4) & 3;          // 16-byte alignment
  a.krec = reinterpret_cast<uint4*>(p); p += 8ll * SIX_DIMS * SIX_KEYS;
  a.brow = p; p += SIX_DIMS * cap;
  p += ((uintptr_t)p & 7) ? 1 : 0;
  a.bdate = reinterpret_cast<int64_t*>(p); p += 2 * SIX_DIMS * cap;
  a.pcap = ix_pcap(cap);
  a.part = reinterpret_cast<int64_t*>(p); p += 2 * SIX_DIMS * a.pcap * IX_PART_WORDS;
  p += ((uintptr_t)p & 7) ? 1 : 0;
  a.sc = reinterpret_cast<SwIxScratch*>(p);
  a.cap = cap;
  k_ix_prep<<<(unsigned)a.groups, IX_PREP_BLK, 0, s>>>(a);
  // (sort key, row) by the 16-bit key (15 hash bits + the no-id flag): two passes, result in buffer 0
  const int rc = sw_radix_sort_u32(a.skeys, a.svals, &a.sc->n_sort, cap, SIX_ALT_SORT_BITS + 1, a.rstate, nullptr, s);
  if (rc < 0) return -rc;
  k_ix_colscan<<<(unsigned)((a.nk_total + 255) / 256), 256, 0, s>>>(a);
  k_ix_scan<<<SIX_DIMS, IX_SCAN_BLK, 0, s>>>(a);
  k_ix_scatter<<<(unsigned)a.groups, IX_PREP_BLK, 0, s>>>(a);
  k_ix_write<<<IX_WRITE_WGS, IX_WBLK, 0, s>>>(a);
  k_ix_heads<<<IX_WRITE_WGS, IX_WBLK, 0, s>>>(a);
  k_ix_merge<<<64, IX_WBLK, 0, s>>>(a);
  k_ix_finish<<<256, IX_WBLK, 0, s>>>(a);
  return (int)hipGetLastError();
}

}  // extern "C"
