// Durable-block encoder on the MI355X: one engine step's persisted rows -> one compressed columnar
// block (format: csrc/include/swseg.h), written into HBM so only the compressed bytes cross PCIe
// to the segment store.  Bit-identical to the CPU encoder (csrc/native/swseg.cpp, swseg_encode).
//
// One 256-thread workgroup (4 wave64) per 1024-row page, 4 consecutive rows per thread:
//   A. plan: per column, block scans give each row its index within the column (the column's
//      member rows, e.g. locations for latitude) and block reductions the frame-of-reference base,
//      bit width, decimal exponent and exception count -> the page's byte size;
//   B. single-pass decoupled look-back over the pages (ticketed workgroups, 64-bit state words:
//      flag | value in one agent-scope atomic, so no payload hand-off and no fence) -> the page's
//      offset in the block, without a separate scan launch;
//   C. write: member values are staged in LDS, then each thread assembles whole u64 words of the
//      bit-packed stream (no atomics, coalesced 8-byte stores) and folds them into the page
//      checksum; a block xor-reduction writes it.
// The grid is sized for the largest step (rows known on the device only); surplus tickets exit.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "swtypes.h"
#include "swseg.h"

#define SBLK 256
#define SWAVES (SBLK / 64)
#define ROWS_PER_THREAD 4

typedef unsigned long long ull;

struct SwSegArgs {
  const SwOutRec* rows;        // this step's rows (device)
  const double* ring_v2;       // event ring elevation column
  const uint64_t* ring_alt;    // event ring alternate-id hash column
  int64_t store_cap;
  const int64_t* cursor;       // [store_cursor, step_cursor0]: rows = cursor[0] - cursor[1]
  uint8_t* out;                // block (device)
  int64_t out_cap;
  uint64_t* state;             // [max_pages] look-back words, then ticket, bytes, errors (zeroed per call)
  int64_t max_pages;
};

#define LB_AGG (1ull << 62)
#define LB_INC (2ull << 62)
#define LB_VAL ((1ull << 62) - 1)
#define LB_SPIN_LIMIT (1u << 22)

__device__ __forceinline__ uint32_t lane64() { return threadIdx.x & 63; }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

__device__ __forceinline__ ull wave_min(ull v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) { const ull o = __shfl_xor(v, d, 64); v = o < v ? o : v; }
  return v;
}

__device__ __forceinline__ ull wave_max(ull v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) { const ull o = __shfl_xor(v, d, 64); v = o > v ? o : v; }
  return v;
}

__device__ __forceinline__ ull wave_xor(ull v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v ^= __shfl_xor(v, d, 64);
  return v;
}

struct SegRed {
  ull a[SWAVES], b[SWAVES];
  uint32_t s[SWAVES + 1];
};

// Exclusive block scan of one u32 per thread (returns the prefix; *total = block sum).
__device__ __forceinline__ uint32_t seg_scan(uint32_t v, uint32_t* total, SegRed& R) {
  const uint32_t lane = lane64(), wid = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += t;
  }
  if (lane == 63) R.s[wid] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int w = 0; w < SWAVES; ++w) { const uint32_t t = R.s[w]; R.s[w] = acc; acc += t; }
    R.s[SWAVES] = acc;
  }
  __syncthreads();
  const uint32_t res = inc - v + R.s[wid];
  *total = R.s[SWAVES];
  __syncthreads();
  return res;
}

// Block min and max of u64 values (threads without members pass ~0 / 0).
__device__ __forceinline__ void seg_minmax(ull lo, ull hi, ull* blo, ull* bhi, SegRed& R) {
  lo = wave_min(lo);
  hi = wave_max(hi);
  const uint32_t wid = threadIdx.x >> 6;
  if (lane64() == 0) { R.a[wid] = lo; R.b[wid] = hi; }
  __syncthreads();
  ull l = R.a[0], h = R.b[0];
#pragma unroll
  for (int w = 1; w < SWAVES; ++w) { l = R.a[w] < l ? R.a[w] : l; h = R.b[w] > h ? R.b[w] : h; }
  *blo = l;
  *bhi = h;
  __syncthreads();
}

struct SegRow {
  int64_t date;
  double v0, v1, v2;
  uint64_t alt;
  int32_t asg;
  uint16_t name;
  uint8_t et, level;
};

template <int C>
__device__ __forceinline__ uint64_t seg_int_value(const SegRow& r) {
  if (C == SEG_ETYPE) return seg_ord((int64_t)r.et);
  if (C == SEG_LEVEL) return seg_ord((int64_t)r.level);
  if (C == SEG_DATE) return seg_ord(r.date);
  if (C == SEG_ASG) return seg_ord((int64_t)r.asg);
  if (C == SEG_NAME) return seg_ord((int64_t)r.name);
  if (C == SEG_HASALT) return seg_ord(r.alt != 0 ? 1 : 0);
  return r.alt;   // SEG_ALT
}

template <int C>
__device__ __forceinline__ double seg_dbl_value(const SegRow& r) {
  return (C == SEG_MXV || C == SEG_LAT) ? r.v0 : (C == SEG_LON ? r.v1 : r.v2);
}

struct SegLds {
  ull vals[SEG_PAGE_ROWS];
  ull xraw[SEG_PAGE_ROWS];
  uint16_t xidx[SEG_PAGE_ROWS];
  SwSegPageHdr hdr;
  SegRed red;
  uint32_t page;
  uint32_t pad;
  ull page_base;
};

// Plan column C: count, base, bits, exponent, exceptions; per-thread member / exception prefixes.
template <int C>
__device__ __forceinline__ void seg_plan(const SegRow (&R)[ROWS_PER_THREAD], const bool (&valid)[ROWS_PER_THREAD],
                                         SegLds& L, uint32_t* pre, uint32_t* xpre) {
  uint32_t cnt = 0;
#pragma unroll
  for (int k = 0; k < ROWS_PER_THREAD; ++k) cnt += (valid[k] && seg_member(C, R[k].et, R[k].alt)) ? 1u : 0u;
  uint32_t count;
  *pre = seg_scan(cnt, &count, L.red);
  SwSegCol& cd = L.hdr.cols[C];
  if (!seg_is_double(C)) {
    ull lo = ~0ull, hi = 0;
#pragma unroll
    for (int k = 0; k < ROWS_PER_THREAD; ++k) {
      if (!(valid[k] && seg_member(C, R[k].et, R[k].alt))) continue;
      const ull u = seg_int_value<C>(R[k]);
      lo = u < lo ? u : lo;
      hi = u > hi ? u : hi;
    }
    ull blo, bhi;
    seg_minmax(lo, hi, &blo, &bhi, L.red);
    *xpre = 0;
    if (threadIdx.x == 0) {
      cd.base = count ? blo : 0;
      cd.bits = (uint8_t)(count ? seg_bitwidth(bhi - blo) : 0);
      cd.exp = -1;
      cd.count = (uint16_t)count;
      cd.n_exc = 0;
    }
  } else {
    // page exponent = the largest per-value exponent among decimal-exact values
    ull emax = 0;
#pragma unroll
    for (int k = 0; k < ROWS_PER_THREAD; ++k) {
      if (!(valid[k] && seg_member(C, R[k].et, R[k].alt))) continue;
      const int e = seg_dec_exp(seg_dbl_value<C>(R[k]));
      if (e != SEG_EXC_NONE && (ull)e > emax) emax = (ull)e;
    }
    ull dummy, be;
    seg_minmax(~0ull, emax, &dummy, &be, L.red);
    const int e = (int)be;
    ull lo = ~0ull, hi = 0;
    uint32_t nx = 0;
#pragma unroll
    for (int k = 0; k < ROWS_PER_THREAD; ++k) {
      if (!(valid[k] && seg_member(C, R[k].et, R[k].alt))) continue;
      int64_t q;
      if (seg_dec_at(seg_dbl_value<C>(R[k]), e, &q)) {
        const ull u = seg_ord(q);
        lo = u < lo ? u : lo;
        hi = u > hi ? u : hi;
      } else {
        ++nx;
      }
    }
    uint32_t n_exc;
    *xpre = seg_scan(nx, &n_exc, L.red);
    ull blo, bhi;
    seg_minmax(lo, hi, &blo, &bhi, L.red);
    if (threadIdx.x == 0) {
      const bool any = count > n_exc;
      cd.base = any ? blo : 0;
      cd.bits = (uint8_t)(any ? seg_bitwidth(bhi - blo) : 0);
      cd.exp = (int8_t)e;
      cd.count = (uint16_t)count;
      cd.n_exc = (uint16_t)n_exc;
    }
  }
}

// Stage column C's packed values in LDS, then write its words (+ exceptions); returns this thread's
// checksum contribution.
template <int C>
__device__ __forceinline__ ull seg_write(const SegRow (&R)[ROWS_PER_THREAD], const bool (&valid)[ROWS_PER_THREAD],
                                         SegLds& L, uint32_t pre, uint32_t xpre, uint8_t* page) {
  const SwSegCol cd = L.hdr.cols[C];
  uint32_t i = pre, x = xpre;
#pragma unroll
  for (int k = 0; k < ROWS_PER_THREAD; ++k) {
    if (!(valid[k] && seg_member(C, R[k].et, R[k].alt))) continue;
    if (!seg_is_double(C)) {
      L.vals[i] = seg_int_value<C>(R[k]) - cd.base;
    } else {
      const double v = seg_dbl_value<C>(R[k]);
      int64_t q;
      if (seg_dec_at(v, cd.exp, &q)) {
        L.vals[i] = seg_ord(q) - cd.base;
      } else {
        L.vals[i] = 0;
        L.xidx[x] = (uint16_t)i;
        L.xraw[x] = sw_f64_bits(v);
        ++x;
      }
    }
    ++i;
  }
  __syncthreads();
  ull cs = 0;
  const uint32_t bits = cd.bits, n = cd.count;
  const uint32_t nw = seg_col_words(n, (int)bits);
  for (uint32_t w = threadIdx.x; w < nw; w += SBLK) {
    ull word = 0;
    const ull bit0 = (ull)w * 64ull;
    for (uint32_t j = (uint32_t)(bit0 / bits); j < n; ++j) {
      const ull b = (ull)j * bits;
      if (b >= bit0 + 64) break;
      word |= b >= bit0 ? (L.vals[j] << (b - bit0)) : (L.vals[j] >> (bit0 - b));
    }
    const uint32_t off = cd.data_off + 8u * w;
    *reinterpret_cast<ull*>(page + off) = word;
    cs ^= seg_mix_word(word, off >> 3);
  }
  if (seg_is_double(C) && cd.n_exc) {
    const uint32_t ne = cd.n_exc;
    const uint32_t xo = cd.data_off + 8u * nw;
    const uint32_t nidx = (2u * ne + 7u) / 8u;
    for (uint32_t w = threadIdx.x; w < nidx; w += SBLK) {
      ull word = 0;
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j)
        if (4 * w + j < ne) word |= (ull)L.xidx[4 * w + j] << (16 * j);
      *reinterpret_cast<ull*>(page + xo + 8u * w) = word;
      cs ^= seg_mix_word(word, (xo >> 3) + w);
    }
    const uint32_t ro = xo + 8u * nidx;
    for (uint32_t j = threadIdx.x; j < ne; j += SBLK) {
      *reinterpret_cast<ull*>(page + ro + 8u * j) = L.xraw[j];
      cs ^= seg_mix_word(L.xraw[j], (ro >> 3) + j);
    }
  }
  __syncthreads();         // the next column reuses the staging arrays
  return cs;
}

__device__ __forceinline__ ull lb_load(uint64_t* p) {
  return __hip_atomic_load((ull*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void lb_store(uint64_t* p, ull v) {
  __hip_atomic_store((ull*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(SBLK) void k_seg_encode(SwSegArgs a) {
  __shared__ SegLds L;
  uint64_t* ticket = a.state + a.max_pages;
  uint64_t* bytes_out = ticket + 1;
  uint64_t* errors = ticket + 2;
  if (threadIdx.x == 0) L.page = (uint32_t)atomicAdd((ull*)ticket, 1ull);
  __syncthreads();
  const uint32_t page = L.page;
  const int64_t c1 = a.cursor[0], c0 = a.cursor[1];
  const int64_t n = c1 - c0;
  const int64_t np = (n + SEG_PAGE_ROWS - 1) / SEG_PAGE_ROWS;
  const uint32_t data_start = 64u + ((4u * (uint32_t)(np + 1) + 7u) & ~7u);
  if (np > a.max_pages || (int64_t)data_start > a.out_cap) {
    if (threadIdx.x == 0 && page == 0) { atomicAdd((ull*)errors, 1ull); atomicMax((ull*)bytes_out, ~0ull); }
    return;
  }
  uint32_t* page_off = reinterpret_cast<uint32_t*>(a.out + 64);
  if (page == 0 && threadIdx.x == 0) ticket[3] = (uint64_t)c0;     // first store sequence, for the host
  if (n <= 0) {
    if (page == 0 && threadIdx.x == 0) {
      SwSegBlockHdr* h = reinterpret_cast<SwSegBlockHdr*>(a.out);
      h->n_rows = 0; h->n_pages = 0; h->bytes = data_start;
      page_off[0] = data_start;
      page_off[1] = 0;
      atomicMax((ull*)bytes_out, (ull)data_start);
    }
    return;
  }
  if ((int64_t)page >= np) return;
  const int64_t r0 = (int64_t)page * SEG_PAGE_ROWS;
  const int m = (int)(n - r0 < SEG_PAGE_ROWS ? n - r0 : SEG_PAGE_ROWS);
  // ---- load 4 consecutive rows per thread
  SegRow R[ROWS_PER_THREAD];
  bool valid[ROWS_PER_THREAD];
#pragma unroll
  for (int k = 0; k < ROWS_PER_THREAD; ++k) {
    const int idx = ROWS_PER_THREAD * (int)threadIdx.x + k;
    valid[k] = idx < m;
    SegRow& r = R[k];
    if (valid[k]) {
      const int64_t j = r0 + idx;
      const uint4 q0 = *reinterpret_cast<const uint4*>(&a.rows[j]);
      const uint4 q1 = *(reinterpret_cast<const uint4*>(&a.rows[j]) + 1);
      r.date = (int64_t)(((ull)q0.y << 32) | q0.x);
      r.v0 = sw_bits_f64(((ull)q0.w << 32) | q0.z);
      r.v1 = sw_bits_f64(((ull)q1.y << 32) | q1.x);
      r.asg = (int32_t)q1.z;
      r.name = (uint16_t)(q1.w & 0xffffu);
      r.et = (uint8_t)((q1.w >> 16) & 0xffu);
      r.level = (uint8_t)(q1.w >> 24);
      const int64_t row = (c0 + j) % a.store_cap;
      r.v2 = a.ring_v2[row];
      r.alt = a.ring_alt[row];
    } else {
      r.date = 0; r.v0 = r.v1 = r.v2 = 0.0; r.alt = 0; r.asg = 0; r.name = 0; r.et = 0; r.level = 0;
    }
  }
  // ---- A. plan every column
  uint32_t pre[SEG_NCOL], xpre[SEG_NCOL];
  seg_plan<SEG_ETYPE>(R, valid, L, &pre[SEG_ETYPE], &xpre[SEG_ETYPE]);
  seg_plan<SEG_LEVEL>(R, valid, L, &pre[SEG_LEVEL], &xpre[SEG_LEVEL]);
  seg_plan<SEG_DATE>(R, valid, L, &pre[SEG_DATE], &xpre[SEG_DATE]);
  seg_plan<SEG_ASG>(R, valid, L, &pre[SEG_ASG], &xpre[SEG_ASG]);
  seg_plan<SEG_NAME>(R, valid, L, &pre[SEG_NAME], &xpre[SEG_NAME]);
  seg_plan<SEG_MXV>(R, valid, L, &pre[SEG_MXV], &xpre[SEG_MXV]);
  seg_plan<SEG_LAT>(R, valid, L, &pre[SEG_LAT], &xpre[SEG_LAT]);
  seg_plan<SEG_LON>(R, valid, L, &pre[SEG_LON], &xpre[SEG_LON]);
  seg_plan<SEG_ELEV>(R, valid, L, &pre[SEG_ELEV], &xpre[SEG_ELEV]);
  seg_plan<SEG_HASALT>(R, valid, L, &pre[SEG_HASALT], &xpre[SEG_HASALT]);
  seg_plan<SEG_ALT>(R, valid, L, &pre[SEG_ALT], &xpre[SEG_ALT]);
  // ---- B. page size, offsets; look-back for the page's place in the block
  if (threadIdx.x == 0) {
    uint32_t off = SEG_PAGE_HDR;
    for (int c = 0; c < SEG_NCOL; ++c) {
      SwSegCol& cd = L.hdr.cols[c];
      cd.data_off = off;
      cd.pad0 = 0;
      cd.pad1 = 0;
      off += seg_col_bytes(cd.count, cd.bits, cd.n_exc);
    }
    L.hdr.n_rows = (uint32_t)m;
    L.hdr.bytes = off;
    L.hdr.checksum = 0;
    const ull size = off;
    ull excl = 0;
    bool failed = false;
    if (page == 0) {
      lb_store(&a.state[0], LB_INC | size);
    } else {
      lb_store(&a.state[page], LB_AGG | size);
      for (int64_t p = (int64_t)page - 1; p >= 0;) {
        ull s = lb_load(&a.state[p]);
        uint32_t spins = 0;
        while ((s >> 62) == 0) {
          if (++spins > LB_SPIN_LIMIT) { failed = true; break; }
          __builtin_amdgcn_s_sleep(1);
          s = lb_load(&a.state[p]);
        }
        if (failed) break;
        excl += s & LB_VAL;
        if ((s >> 62) == 2) break;
        --p;
      }
      lb_store(&a.state[page], LB_INC | (excl + size));
    }
    const ull base = (ull)data_start + excl;
    if (failed || base + size > (ull)a.out_cap) {
      atomicAdd((ull*)errors, 1ull);
      atomicMax((ull*)bytes_out, ~0ull);
      L.page_base = ~0ull;
    } else {
      L.page_base = base;
      page_off[page] = (uint32_t)base;
      if ((int64_t)page == np - 1) {
        page_off[np] = (uint32_t)(base + size);
        SwSegBlockHdr* h = reinterpret_cast<SwSegBlockHdr*>(a.out);
        h->n_rows = (uint32_t)n;
        h->n_pages = (uint32_t)np;
        h->bytes = base + size;
        atomicMax((ull*)bytes_out, base + size);
      }
    }
  }
  __syncthreads();
  if (L.page_base == ~0ull) return;
  uint8_t* pg = a.out + L.page_base;
  // ---- C. write the columns
  ull cs = 0;
  cs ^= seg_write<SEG_ETYPE>(R, valid, L, pre[SEG_ETYPE], xpre[SEG_ETYPE], pg);
  cs ^= seg_write<SEG_LEVEL>(R, valid, L, pre[SEG_LEVEL], xpre[SEG_LEVEL], pg);
  cs ^= seg_write<SEG_DATE>(R, valid, L, pre[SEG_DATE], xpre[SEG_DATE], pg);
  cs ^= seg_write<SEG_ASG>(R, valid, L, pre[SEG_ASG], xpre[SEG_ASG], pg);
  cs ^= seg_write<SEG_NAME>(R, valid, L, pre[SEG_NAME], xpre[SEG_NAME], pg);
  cs ^= seg_write<SEG_MXV>(R, valid, L, pre[SEG_MXV], xpre[SEG_MXV], pg);
  cs ^= seg_write<SEG_LAT>(R, valid, L, pre[SEG_LAT], xpre[SEG_LAT], pg);
  cs ^= seg_write<SEG_LON>(R, valid, L, pre[SEG_LON], xpre[SEG_LON], pg);
  cs ^= seg_write<SEG_ELEV>(R, valid, L, pre[SEG_ELEV], xpre[SEG_ELEV], pg);
  cs ^= seg_write<SEG_HASALT>(R, valid, L, pre[SEG_HASALT], xpre[SEG_HASALT], pg);
  cs ^= seg_write<SEG_ALT>(R, valid, L, pre[SEG_ALT], xpre[SEG_ALT], pg);
  // page header words (word 1, the checksum, is written last and not summed)
  const ull* hw = reinterpret_cast<const ull*>(&L.hdr);
  for (uint32_t i = threadIdx.x; i < SEG_PAGE_HDR / 8; i += SBLK) {
    if (i == 1) continue;
    const ull w = hw[i];
    *reinterpret_cast<ull*>(pg + 8u * i) = w;
    cs ^= seg_mix_word(w, i);
  }
  cs = wave_xor(cs);
  if (lane64() == 0) L.red.a[threadIdx.x >> 6] = cs;
  __syncthreads();
  if (threadIdx.x == 0) {
    ull t = 0;
#pragma unroll
    for (int w = 0; w < SWAVES; ++w) t ^= L.red.a[w];
    *reinterpret_cast<ull*>(pg + 8) = t;
  }
}

extern "C" {

// Encode this step's rows into `out`.  state = u64[max_pages + 4], zeroed here (a memset node when
// captured); afterwards state[max_pages + 1] = block bytes (~0 on error), state[max_pages + 2] = errors,
// state[max_pages + 3] = the store sequence of the block's first row.
int sw_seg_encode(const void* rows, const double* ring_v2, const uint64_t* ring_alt, int64_t store_cap,
                  const int64_t* cursor, uint8_t* out, int64_t out_cap, uint64_t* state, int64_t max_pages,
                  hipStream_t s) {
  hipError_t e = hipMemsetAsync(state, 0, sizeof(uint64_t) * (size_t)(max_pages + 4), s);
  if (e != hipSuccess) return (int)e;
  SwSegArgs a;
  a.rows = (const SwOutRec*)rows;
  a.ring_v2 = ring_v2;
  a.ring_alt = ring_alt;
  a.store_cap = store_cap;
  a.cursor = cursor;
  a.out = out;
  a.out_cap = out_cap;
  a.state = state;
  a.max_pages = max_pages;
  const unsigned grid = (unsigned)(max_pages > 0 ? max_pages : 1);
  k_seg_encode<<<grid, SBLK, 0, s>>>(a);
  return (int)hipGetLastError();
}

}  // extern "C"
