// Read-side indexes of a durable event block, built on the MI355X in the step that encodes the block
// (format: csrc/include/swindex.h; C++ reference: csrc/native/swindex.cpp swseg_index_append, bit for
// bit).  Also the stable LSD radix sort the engine uses to persist each step clustered by assignment.
//
// Reference: MongoDeviceEventManagement.java:129-141 -- the indexes Mongo maintains on every insert
// (alternateId; assignment / customer / area / asset + eventType + eventDate).  Here they are built
// for a whole step at once, in HBM, and cost ~4 B per event on disk; the host threads that indexed
// finished blocks after the fact (~59M events/s on 16 cores) are gone.
//
// Radix sort (sw_radix_sort_u32): per 8-bit digit pass two dispatches -- per-tile digit histograms
// (LDS atomics), then a scatter whose prologue sums the earlier tiles' histograms for its digit base
// (tile-major histograms: coalesced, L2-resident; no scan dispatch) and whose ranks are stable: items
// go through the tile in 16 rounds of 256, each wave ranks its 64 by a ballot match on the digit
// bits, the waves' counts are prefixed in LDS.  Wave64 throughout: ballots are 64-bit.
//
// Trailer build (sw_seg_index, after k_seg_encode on the same stream, 9 dispatches):
//   k_ix_prep     per row: alternate-id sort key (top 15 hash bits; rows without an id sort last),
//                 context-key counts per dimension (LDS-aggregated for small key spaces), max context id
//   radix sort    (sort key, row), 16 bits: two passes
//   k_ix_scan     one workgroup per dimension: bucket offsets, present-key ranks, head offsets; the
//                 last one out lays the trailer out (header, block header bytes / flags)
//   k_ix_scatter  rows into per-key buckets (per-workgroup reservations, LDS ranks)
//   k_ix_write    page zone maps (from the page headers), the alternate-id directory and its packed
//                 entries, and -- one wave per present key -- count, date range and the 16 newest rows
//                 (lane-local top-16 lists merged by 16 rounds of wave argmax)
//   k_ix_finish   checksum of the whole trailer (xor of mixed words: order free); the last workgroup
//                 publishes the block's bytes to the encoder state and the host snapshot and re-arms
//                 the scratch for the next step
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

// ============================================================================ radix sort
__global__ __launch_bounds__(RS_BLK) void k_rs_hist(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ n_ptr,
                                                    int shift, uint32_t mask, uint32_t* __restrict__ hist) {
  __shared__ uint32_t c[256];
  const uint32_t n = *n_ptr;
  const int64_t base = (int64_t)blockIdx.x * RS_TILE;
  if (base >= (int64_t)n) return;
  c[threadIdx.x] = 0;
  __syncthreads();
#pragma unroll 4
  for (int k = 0; k < RS_ITEMS; ++k) {
    const int64_t i = base + (int64_t)k * RS_BLK + threadIdx.x;
    if (i < (int64_t)n) atomicAdd(&c[(keys[i] >> shift) & mask], 1u);
  }
  __syncthreads();
  hist[(int64_t)blockIdx.x * 256 + threadIdx.x] = c[threadIdx.x];
}

__global__ __launch_bounds__(RS_BLK) void k_rs_scatter(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                       uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                       const uint32_t* __restrict__ n_ptr, int shift, int dbits,
                                                       const uint32_t* __restrict__ hist) {
  __shared__ uint32_t dbase[256];
  __shared__ uint32_t wc[RS_WAVES][256];
  __shared__ uint32_t red[RS_WAVES + 1];
  const uint32_t n = *n_ptr;
  const int64_t tile = blockIdx.x;
  const int64_t base = tile * RS_TILE;
  if (base >= (int64_t)n) return;
  const int64_t ntiles = ((int64_t)n + RS_TILE - 1) / RS_TILE;
  const uint32_t mask = (1u << dbits) - 1u;
  const uint32_t t = threadIdx.x, lane = ix_lane(), wid = t >> 6;
  // ---- digit t: earlier tiles' count and the total (tile-major histograms, coalesced)
  uint32_t pre = 0, tot = 0;
  for (int64_t q = 0; q < ntiles; ++q) {
    const uint32_t v = hist[q * 256 + t];
    pre += q < tile ? v : 0u;
    tot += v;
  }
  // exclusive scan of the totals over the digits
  uint32_t inc = tot;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += o;
  }
  if (lane == 63) red[wid] = inc;
  __syncthreads();
  if (t == 0) {
    uint32_t acc = 0;
    for (int w = 0; w < RS_WAVES; ++w) { const uint32_t x = red[w]; red[w] = acc; acc += x; }
  }
  __syncthreads();
  dbase[t] = inc - tot + red[wid] + pre;
#pragma unroll
  for (int w = 0; w < RS_WAVES; ++w) wc[w][t] = 0;
  // ---- the tile's items, all loads in flight before the ranking rounds
  uint32_t K[RS_ITEMS], V[RS_ITEMS];
#pragma unroll
  for (int k = 0; k < RS_ITEMS; ++k) {
    const int64_t i = base + (int64_t)k * RS_BLK + t;
    K[k] = i < (int64_t)n ? kin[i] : 0u;
    V[k] = i < (int64_t)n ? vin[i] : 0u;
  }
  __syncthreads();
  const ull lt = (1ull << lane) - 1ull;
#pragma unroll 1
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
    if (valid && rank == 0) wc[wid][d] = (uint32_t)__popcll(peers);   // the group's lowest lane
    __syncthreads();
    if (valid) {
      uint32_t pos = dbase[d] + rank;
      for (uint32_t w = 0; w < wid; ++w) pos += wc[w][d];
      kout[pos] = K[k];
      vout[pos] = V[k];
    }
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (int w = 0; w < RS_WAVES; ++w) { add += wc[w][t]; wc[w][t] = 0; }
    dbase[t] += add;
    __syncthreads();
  }
}

extern "C" {

int64_t sw_radix_tmp_words(int64_t cap) { return 256 * ((cap + RS_TILE - 1) / RS_TILE) + 256; }

// Stable LSD radix sort of *n_ptr (<= cap) u32 (key, value) pairs by the low `bits` bits of the key.
// keys / vals: [2][cap] ping-pong buffers, input in buffer 0.  vals_final (optional): where the last
// pass writes the values instead of the ping-pong buffer.  Returns the buffer (0 / 1) holding the
// sorted keys (and values, without vals_final): passes = ceil(bits / 8), ~0 bits: no pass.
int sw_radix_sort_u32(uint32_t* keys, uint32_t* vals, const uint32_t* n_ptr, int64_t cap, int bits, uint32_t* hist,
                      uint32_t* vals_final, hipStream_t s) {
  const unsigned grid = (unsigned)((cap + RS_TILE - 1) / RS_TILE > 0 ? (cap + RS_TILE - 1) / RS_TILE : 1);
  int cur = 0;
  for (int shift = 0; shift < bits; shift += 8) {
    const int db = bits - shift < 8 ? bits - shift : 8;
    const uint32_t mask = (1u << db) - 1u;
    k_rs_hist<<<grid, RS_BLK, 0, s>>>(keys + (int64_t)cur * cap, n_ptr, shift, mask, hist);
    const bool last = shift + 8 >= bits;
    uint32_t* vo = (last && vals_final) ? vals_final : vals + (int64_t)(1 - cur) * cap;
    k_rs_scatter<<<grid, RS_BLK, 0, s>>>(keys + (int64_t)cur * cap, vals + (int64_t)cur * cap,
                                         keys + (int64_t)(1 - cur) * cap, vo, n_ptr, shift, db, hist);
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
  int32_t maxc[SIX_DIMS];    // max context id per dimension (-1: none)
  uint32_t scans_done;
  uint32_t finish_done;
  uint32_t err;
  uint32_t n_sort;           // rows this step (the radix sort's count)
};

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
  uint32_t* skeys;           // [2][cap] alternate-id sort keys
  uint32_t* svals;           // [2][cap] rows
  uint32_t* shist;           // radix histograms
  uint32_t* ccnt;            // [3][SIX_KEYS] rows per key
  uint32_t* coff;            // [3][SIX_KEYS] bucket start (scan), then the scatter's cursor
  uint32_t* cidx;            // [3][SIX_KEYS] rank among present keys
  uint32_t* chof;            // [3][SIX_KEYS] first head (entries)
  uint32_t* ckeys;           // [3][SIX_KEYS] present keys in order
  uint32_t* cbuck;           // [3][cap] rows by key bucket
  SwIxScratch* sc;
  int64_t cap;               // rows capacity
};

#define IX_BLK 256
#define IX_LDS_KEYS 4096     // keys per dimension counted in LDS (larger keys: global atomics)

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

// ---- per row: alternate-id sort key; context key counts
__global__ __launch_bounds__(IX_BLK) void k_ix_prep(SwIxArgs a) {
  __shared__ uint32_t lc[SIX_DIMS][IX_LDS_KEYS];
  __shared__ int32_t lmax[SIX_DIMS];
  __shared__ uint32_t lalt;
  const int64_t n = ix_rows(a);
  if (blockIdx.x == 0 && threadIdx.x == 0) a.sc->n_sort = (uint32_t)n;
  const int64_t per = ((n + gridDim.x - 1) / gridDim.x + 255) & ~255ll;
  const int64_t r0 = (int64_t)blockIdx.x * per, r1 = r0 + per < n ? r0 + per : n;
  if (r0 >= n) return;
  for (int i = threadIdx.x; i < SIX_DIMS * IX_LDS_KEYS; i += IX_BLK) (&lc[0][0])[i] = 0;
  if (threadIdx.x < SIX_DIMS) lmax[threadIdx.x] = -1;
  if (threadIdx.x == 0) lalt = 0;
  __syncthreads();
  const int64_t c0 = a.cursor[1];
  uint32_t nalt = 0;
  int32_t mx[SIX_DIMS] = {-1, -1, -1};
  for (int64_t j = r0 + threadIdx.x; j < r1; j += IX_BLK) {
    const SwOutRec o = a.rows[j];
    const bool has = a.raw && (a.aux[j].flags & SEGF_HAS_ALT);
    uint32_t key = 1u << SIX_ALT_SORT_BITS;
    if (has) {
      key = six_sort_key(a.s_alt[(c0 + j) % a.store_cap]);
      ++nalt;
    }
    a.skeys[j] = key;
    a.svals[j] = (uint32_t)j;
#pragma unroll
    for (int d = 0; d < SIX_DIMS; ++d) {
      const int32_t c = ix_ctx(a, o.assignment, d);
      if (c < 0) continue;
      mx[d] = c > mx[d] ? c : mx[d];
      if (c >= SIX_CTX_MAX) continue;
      const uint32_t k = ((uint32_t)c << 3) | (uint32_t)(o.etype & 7u);
      if (k < IX_LDS_KEYS) atomicAdd(&lc[d][k], 1u);
      else atomicAdd(&a.ccnt[(int64_t)d * SIX_KEYS + k], 1u);
    }
  }
  for (int off = 32; off >= 1; off >>= 1) nalt += __shfl_xor(nalt, off, 64);
  if (ix_lane() == 0 && nalt) atomicAdd(&lalt, nalt);
#pragma unroll
  for (int d = 0; d < SIX_DIMS; ++d) if (mx[d] >= 0) atomicMax(&lmax[d], mx[d]);
  __syncthreads();
  for (int i = threadIdx.x; i < SIX_DIMS * IX_LDS_KEYS; i += IX_BLK) {
    const uint32_t v = (&lc[0][0])[i];
    if (v) atomicAdd(&a.ccnt[(int64_t)(i / IX_LDS_KEYS) * SIX_KEYS + (i % IX_LDS_KEYS)], v);
  }
  if (threadIdx.x < SIX_DIMS && lmax[threadIdx.x] >= 0) atomicMax(&a.sc->maxc[threadIdx.x], lmax[threadIdx.x]);
  if (threadIdx.x == 0 && lalt) atomicAdd(&a.sc->n_alt, lalt);
}

// ---- one workgroup per dimension: offsets of the key buckets, ranks of the present keys, head
// offsets; the last workgroup out lays the trailer out
#define IX_SCAN_BLK 1024
__global__ __launch_bounds__(IX_SCAN_BLK) void k_ix_scan(SwIxArgs a) {
  __shared__ uint32_t wsum[3][IX_SCAN_BLK / 64];
  __shared__ uint32_t last;
  const int d = blockIdx.x;
  const int32_t mc = a.sc->maxc[d];
  const bool indexed = mc < SIX_CTX_MAX;
  const uint32_t nk = indexed ? ((uint32_t)(mc + 1) << 3) : 0u;     // key space in use
  const uint32_t per = (nk + IX_SCAN_BLK - 1) / IX_SCAN_BLK;
  const uint32_t k0 = threadIdx.x * per, k1 = k0 + per < nk ? k0 + per : nk;
  const uint32_t* cnt = a.ccnt + (int64_t)d * SIX_KEYS;
  uint32_t s_rows = 0, s_keys = 0, s_heads = 0;
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t c = cnt[k];
    s_rows += c;
    s_keys += c ? 1u : 0u;
    s_heads += c < SIX_HEADS ? c : SIX_HEADS;
  }
  // block exclusive scan of the three sums
  const uint32_t lane = ix_lane(), wid = threadIdx.x >> 6;
  uint32_t v[3] = {s_rows, s_keys, s_heads}, inc[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    inc[q] = v[q];
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t x = __shfl_up(inc[q], o, 64);
      if (lane >= (uint32_t)o) inc[q] += x;
    }
    if (lane == 63) wsum[q][wid] = inc[q];
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    uint32_t acc = 0;
    for (int w = 0; w < IX_SCAN_BLK / 64; ++w) { const uint32_t x = wsum[threadIdx.x][w]; wsum[threadIdx.x][w] = acc; acc += x; }
    if (threadIdx.x == 1) a.sc->h.n_keys[d] = indexed ? acc : SIX_NOT_INDEXED;
    if (threadIdx.x == 2) a.sc->h.n_heads[d] = indexed ? acc : 0u;
  }
  __syncthreads();
  uint32_t pr = inc[0] - v[0] + wsum[0][wid], pk = inc[1] - v[1] + wsum[1][wid], ph = inc[2] - v[2] + wsum[2][wid];
  uint32_t* off = a.coff + (int64_t)d * SIX_KEYS;
  uint32_t* idx = a.cidx + (int64_t)d * SIX_KEYS;
  uint32_t* hof = a.chof + (int64_t)d * SIX_KEYS;
  uint32_t* kl = a.ckeys + (int64_t)d * SIX_KEYS;
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t c = cnt[k];
    off[k] = pr;
    idx[k] = pk;
    hof[k] = ph;
    if (c) kl[pk] = k;
    pr += c;
    pk += c ? 1u : 0u;
    ph += c < SIX_HEADS ? c : SIX_HEADS;
  }
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
    sc->err = 1;
    return;
  }
  // header words (checksum 0 for now) and the heads sections' padding word
  uint8_t* t = a.out + tstart;
  const uint64_t* hw = reinterpret_cast<const uint64_t*>(&h);
  for (uint32_t i = 0; i < SIX_HDR_BYTES / 8; ++i) reinterpret_cast<uint64_t*>(t)[i] = hw[i];
  for (int q = 0; q < SIX_DIMS; ++q)
    if (h.n_heads[q] & 1u) *reinterpret_cast<uint32_t*>(t + h.off_heads[q] + 4u * h.n_heads[q]) = 0u;
  SwSegBlockHdr* bh = reinterpret_cast<SwSegBlockHdr*>(a.out);
  bh->flags = SEG_FLAG_INDEX;
  bh->bytes = tstart + tb;
}

// ---- rows into their key buckets (order inside a bucket is free: every per-key output is
// order-independent)
__global__ __launch_bounds__(IX_BLK) void k_ix_scatter(SwIxArgs a) {
  __shared__ uint32_t lc[IX_LDS_KEYS];
  __shared__ uint32_t lb[IX_LDS_KEYS];
  const int64_t n = ix_rows(a);
  const int64_t per = ((n + gridDim.x - 1) / gridDim.x + 255) & ~255ll;
  const int64_t r0 = (int64_t)blockIdx.x * per, r1 = r0 + per < n ? r0 + per : n;
  if (r0 >= n || a.sc->err) return;
  for (int d = 0; d < SIX_DIMS; ++d) {
    if (a.sc->maxc[d] >= SIX_CTX_MAX) continue;            // block-uniform
    uint32_t* cur = a.coff + (int64_t)d * SIX_KEYS;
    uint32_t* buck = a.cbuck + (int64_t)d * a.cap;
    for (int i = threadIdx.x; i < IX_LDS_KEYS; i += IX_BLK) lc[i] = 0;
    __syncthreads();
    for (int64_t j = r0 + threadIdx.x; j < r1; j += IX_BLK) {
      const SwOutRec o = a.rows[j];
      const int32_t c = ix_ctx(a, o.assignment, d);
      if (c < 0) continue;
      const uint32_t k = ((uint32_t)c << 3) | (uint32_t)(o.etype & 7u);
      if (k < IX_LDS_KEYS) atomicAdd(&lc[k], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < IX_LDS_KEYS; i += IX_BLK) {
      const uint32_t v = lc[i];
      lb[i] = v ? atomicAdd(&cur[i], v) : 0u;
      lc[i] = 0;
    }
    __syncthreads();
    for (int64_t j = r0 + threadIdx.x; j < r1; j += IX_BLK) {
      const SwOutRec o = a.rows[j];
      const int32_t c = ix_ctx(a, o.assignment, d);
      if (c < 0) continue;
      const uint32_t k = ((uint32_t)c << 3) | (uint32_t)(o.etype & 7u);
      const uint32_t pos = k < IX_LDS_KEYS ? lb[k] + atomicAdd(&lc[k], 1u) : atomicAdd(&cur[k], 1u);
      buck[pos] = (uint32_t)j;
    }
    __syncthreads();
  }
}

// ---- page zone maps, alternate-id directory + entries, per-key summaries and heads
#define IX_WRITE_WGS 1024
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
  // directory: dir[b] = entries whose bucket is < b (lower bound in the sorted keys)
  const uint32_t* sk = a.skeys;           // sorted (buffer 0 after two passes)
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

// wave-wide (date desc, row desc) maximum of (d, r); returns the winner, broadcast
__device__ __forceinline__ void ix_wave_best(int64_t& d, uint32_t& r) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int64_t od = __shfl_xor(d, off, 64);
    const uint32_t orow = __shfl_xor(r, off, 64);
    if (six_newer(od, orow, d, r)) { d = od; r = orow; }
  }
}

__device__ void ix_write_key(const SwIxArgs& a, const SwIxHdr& h, uint8_t* t, int d, uint32_t q) {
  const uint32_t lane = ix_lane();
  const uint32_t k = a.ckeys[(int64_t)d * SIX_KEYS + q];
  const uint32_t cnt = a.ccnt[(int64_t)d * SIX_KEYS + k];
  const uint32_t bo = a.coff[(int64_t)d * SIX_KEYS + k] - cnt;   // the scatter advanced the cursor by cnt
  const uint32_t* buck = a.cbuck + (int64_t)d * a.cap + bo;
  // lane-local top-16 (sorted, newest first), running min / max
  int64_t LD[SIX_HEADS];
  uint32_t LR[SIX_HEADS];
  int nl = 0;
  int64_t dmin = INT64_MAX, dmax = INT64_MIN;
#pragma unroll
  for (int i = 0; i < SIX_HEADS; ++i) { LD[i] = INT64_MIN; LR[i] = 0; }
  for (uint32_t i = lane; i < cnt; i += 64) {
    const uint32_t row = buck[i];
    const int64_t dt = a.rows[row].event_date;
    dmin = dt < dmin ? dt : dmin;
    dmax = dt > dmax ? dt : dmax;
    if (nl == SIX_HEADS && !six_newer(dt, row, LD[SIX_HEADS - 1], LR[SIX_HEADS - 1])) continue;
    // insert (unrolled shift: registers only)
    int64_t cd = dt;
    uint32_t cr = row;
#pragma unroll
    for (int s = 0; s < SIX_HEADS; ++s) {
      const bool take = s >= nl || six_newer(cd, cr, LD[s], LR[s]);
      if (take) {
        const int64_t td = LD[s];
        const uint32_t tr = LR[s];
        LD[s] = cd; LR[s] = cr;
        cd = td; cr = tr;
      }
    }
    nl = nl < SIX_HEADS ? nl + 1 : SIX_HEADS;
  }
  // wave min / max
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int64_t a1 = __shfl_xor(dmin, off, 64), a2 = __shfl_xor(dmax, off, 64);
    dmin = a1 < dmin ? a1 : dmin;
    dmax = a2 > dmax ? a2 : dmax;
  }
  // merge: 16 rounds of wave argmax over the lanes' list heads
  const uint32_t nh = cnt < SIX_HEADS ? cnt : SIX_HEADS;
  const uint32_t hoff = a.chof[(int64_t)d * SIX_KEYS + k];
  uint32_t* heads = reinterpret_cast<uint32_t*>(t + h.off_heads[d]) + hoff;
  int64_t* hdates = reinterpret_cast<int64_t*>(t + h.off_hdates[d]) + hoff;
  for (uint32_t r = 0; r < nh; ++r) {
    int64_t bd = nl > 0 ? LD[0] : INT64_MIN;
    uint32_t br = nl > 0 ? LR[0] : 0u;
    const bool have = nl > 0;
    // lanes without entries must never win: their (INT64_MIN, 0) loses to any real entry unless every
    // real entry is (INT64_MIN, 0) itself -- a row dated INT64_MIN with row 0 ties harmlessly
    int64_t wd = bd;
    uint32_t wr = br;
    ix_wave_best(wd, wr);
    if (lane == 0) { heads[r] = wr; hdates[r] = wd; }
    // the winner pops its head (rows are unique: exactly one lane holds (wd, wr))
    if (have && bd == wd && br == wr) {
#pragma unroll
      for (int s = 0; s + 1 < SIX_HEADS; ++s) { LD[s] = LD[s + 1]; LR[s] = LR[s + 1]; }
      LD[SIX_HEADS - 1] = INT64_MIN;
      LR[SIX_HEADS - 1] = 0;
      --nl;
    }
  }
  if (lane == 0) {
    SwIxKey e;
    e.key = k;
    e.count = cnt;
    e.date_min = dmin;
    e.date_max = dmax;
    e.head_off = hoff;
    e.n_heads = nh;
    *reinterpret_cast<SwIxKey*>(t + h.off_keys[d] + (uint64_t)q * sizeof(SwIxKey)) = e;
  }
}

__global__ __launch_bounds__(IX_BLK) void k_ix_write(SwIxArgs a) {
  if (a.sc->err) return;
  const SwIxHdr h = a.sc->h;
  uint8_t* t = a.out + a.sc->tstart;
  ix_write_pages(a, h, t, (int64_t)blockIdx.x * IX_BLK + threadIdx.x, (int64_t)gridDim.x * IX_BLK);
  // one wave per present key of every indexed dimension
  const uint32_t nk0 = h.n_keys[0] == SIX_NOT_INDEXED ? 0u : h.n_keys[0];
  const uint32_t nk1 = h.n_keys[1] == SIX_NOT_INDEXED ? 0u : h.n_keys[1];
  const uint32_t nk2 = h.n_keys[2] == SIX_NOT_INDEXED ? 0u : h.n_keys[2];
  const uint32_t total = nk0 + nk1 + nk2;
  const uint32_t wave = blockIdx.x * (IX_BLK / 64) + (threadIdx.x >> 6), nwaves = gridDim.x * (IX_BLK / 64);
  for (uint32_t g = wave; g < total; g += nwaves) {
    const int d = g < nk0 ? 0 : g < nk0 + nk1 ? 1 : 2;
    const uint32_t q = d == 0 ? g : d == 1 ? g - nk0 : g - nk0 - nk1;
    ix_write_key(a, h, t, d, q);
  }
}

// ---- checksum of the whole trailer; the last workgroup publishes and re-arms
__global__ __launch_bounds__(IX_BLK) void k_ix_finish(SwIxArgs a) {
  __shared__ ull red[IX_BLK / 64];
  __shared__ uint32_t last;
  SwIxScratch* sc = a.sc;
  const bool ok = !sc->err;
  ull cs = 0;
  if (ok) {
    const uint8_t* t = a.out + sc->tstart;
    const uint64_t words = sc->h.bytes / 8;
    for (uint64_t i = (uint64_t)blockIdx.x * IX_BLK + threadIdx.x; i < words; i += (uint64_t)gridDim.x * IX_BLK)
      if (i != SIX_CHECKSUM_WORD) cs ^= seg_mix_word(reinterpret_cast<const ull*>(t)[i], i);
  }
  for (int off = 32; off >= 1; off >>= 1) cs ^= __shfl_xor(cs, off, 64);
  if (ix_lane() == 0) red[threadIdx.x >> 6] = cs;
  __syncthreads();
  if (threadIdx.x == 0) {
    ull x = 0;
    for (int w = 0; w < IX_BLK / 64; ++w) x ^= red[w];
    if (x) atomicXor(reinterpret_cast<ull*>(&sc->cs), x);
    __threadfence();
    last = atomicAdd(&sc->finish_done, 1u) == (uint32_t)gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  if (threadIdx.x == 0) {
    const ull total_cs = atomicXor(reinterpret_cast<ull*>(&sc->cs), 0ull);
    const uint64_t bytes = sc->tstart + sc->h.bytes;
    if (ok) {
      reinterpret_cast<ull*>(a.out + sc->tstart)[SIX_CHECKSUM_WORD] = total_cs;
      a.seg_state[a.max_pages + 1] = bytes;
      if (a.snap_host) { a.snap_host[16] = (uint32_t)bytes; a.snap_host[17] = (uint32_t)(bytes >> 32); }
    } else if (!ix_encoder_failed(a)) {
      // the trailer did not fit: a loud encoder error, never a block without its index
      a.seg_state[a.max_pages + 2] += 1;
      a.seg_state[a.max_pages + 1] = ~0ull;
      if (a.snap_host) { a.snap_host[16] = ~0u; a.snap_host[17] = ~0u; a.snap_host[18] += 1; }
    }
    sc->cs = 0;
    sc->n_alt = 0;
    sc->scans_done = 0;
    sc->finish_done = 0;
    sc->err = 0;
  }
  // re-arm the key counts this step touched (k_ix_prep accumulates into zeros), then the maxima
  for (int q = 0; q < SIX_DIMS; ++q) {
    const int32_t mc = sc->maxc[q];
    const int64_t nk = mc < 0 ? 0 : ((int64_t)(mc < SIX_CTX_MAX ? mc : SIX_CTX_MAX - 1) + 1) << 3;
    for (int64_t k = threadIdx.x; k < nk; k += IX_BLK) a.ccnt[(int64_t)q * SIX_KEYS + k] = 0;
  }
  __syncthreads();
  if (threadIdx.x < SIX_DIMS) sc->maxc[threadIdx.x] = -1;
}

extern "C" {

// Scratch words (u32) of a trailer build for `cap` rows, laid out by sw_seg_index_layout's caller:
//   skeys [2 cap] | svals [2 cap] | shist [radix] | ccnt, coff, cidx, chof, ckeys [3 SIX_KEYS each]
//   | cbuck [3 cap] | SwIxScratch
int64_t sw_seg_index_scratch_words(int64_t cap) {
  return 4 * cap + (int64_t)sw_radix_tmp_words(cap) + 5ll * SIX_DIMS * SIX_KEYS + 3 * cap +
         (int64_t)((sizeof(SwIxScratch) + 15) / 4);
}

int64_t sw_seg_index_max_bytes(int64_t rows) { return (int64_t)six_max_bytes((uint64_t)rows); }

// Build the index trailer of the block k_seg_encode just wrote (same stream, same arguments) and
// append it to the block.  scratch: u32[sw_seg_index_scratch_words(cap)], zeroed once at allocation
// with its SwIxScratch maxc set to -1 (sw_seg_index_init).
int sw_seg_index(const void* rows, const void* aux, const uint8_t* raw, const int64_t* cursor, const uint64_t* s_alt,
                 int64_t store_cap, const void* asg_ctx, int64_t n_asg, uint8_t* out, int64_t out_cap,
                 uint64_t* seg_state, int64_t max_pages, uint32_t* snap_host, uint32_t* scratch, int64_t cap,
                 hipStream_t s) {
  SwIxArgs a;
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
  uint32_t* p = scratch;
  a.skeys = p; p += 2 * cap;
  a.svals = p; p += 2 * cap;
  a.shist = p; p += sw_radix_tmp_words(cap);
  a.ccnt = p; p += (int64_t)SIX_DIMS * SIX_KEYS;
  a.coff = p; p += (int64_t)SIX_DIMS * SIX_KEYS;
  a.cidx = p; p += (int64_t)SIX_DIMS * SIX_KEYS;
  a.chof = p; p += (int64_t)SIX_DIMS * SIX_KEYS;
  a.ckeys = p; p += (int64_t)SIX_DIMS * SIX_KEYS;
  a.cbuck = p; p += 3 * cap;
  a.sc = reinterpret_cast<SwIxScratch*>(p);
  a.cap = cap;
  const unsigned g = (unsigned)((cap + 4095) / 4096 > 0 ? ((cap + 4095) / 4096 < 1024 ? (cap + 4095) / 4096 : 1024) : 1);
  k_ix_prep<<<g, IX_BLK, 0, s>>>(a);
  // (sort key, row) by the 16-bit key (15 hash bits + the no-id flag): two passes, result in buffer 0
  const int rc = sw_radix_sort_u32(a.skeys, a.svals, &a.sc->n_sort, cap, SIX_ALT_SORT_BITS + 1, a.shist, nullptr, s);
  if (rc != 0) return rc < 0 ? -rc : -1;
  k_ix_scan<<<SIX_DIMS, IX_SCAN_BLK, 0, s>>>(a);
  k_ix_scatter<<<g, IX_BLK, 0, s>>>(a);
  k_ix_write<<<IX_WRITE_WGS, IX_BLK, 0, s>>>(a);
  k_ix_finish<<<256, IX_BLK, 0, s>>>(a);
  return (int)hipGetLastError();
}

// Arm a freshly zeroed scratch (the per-dimension maxima start at -1).
__global__ void k_ix_init(SwIxScratch* sc) {
  if (threadIdx.x < SIX_DIMS) sc->maxc[threadIdx.x] = -1;
}

int sw_seg_index_init(uint32_t* scratch, int64_t cap, hipStream_t s) {
  uint32_t* p = scratch + 4 * cap + sw_radix_tmp_words(cap) + 5ll * SIX_DIMS * SIX_KEYS + 3 * cap;
  k_ix_init<<<1, 64, 0, s>>>(reinterpret_cast<SwIxScratch*>(p));
  return (int)hipGetLastError();
}

}  // extern "C"
