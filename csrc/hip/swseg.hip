// Durable-block encoder on the MI355X: one engine step's persisted events -> one compressed columnar
// block (format: csrc/include/swseg.h), written into HBM so only the compressed bytes cross PCIe
// to the segment store.  Bit-identical to the CPU encoder (csrc/native/swseg.cpp, swseg_encode).
//
// Input per row j of the step, both written coalesced in persisted order by the persist kernel: the
// enriched row (rows[j], 32 B) and its encoder aux (aux[j], SwSegAux 32 B: elevation, SEG_FLAGS and
// the string refs into the raw batch, which is still resident in HBM).  No record is gathered here.
//
// One 512-thread workgroup (8 wave64) per 1024-row page, 2 consecutive rows per thread.  The plan
// is a few fused block-wide rounds instead of one scan / reduction per column:
//   R1  first row with an alternate id (its first 64 bytes staged in LDS); per double column the
//       decimal exponent (max of the rows' exponents, searched from a per-column hint)
//   R2  alternate ids read with aligned 8-byte loads (all the thread's rows' loads in flight at once): common
//       prefix with the first id (word xor + ctz), last non-hex byte and the value of the trailing hex
//       digits in one register pass; every integer column's min / max; quantised double min / max
//   R3  one multi-column scan: member indices of all 15 columns, exception indices, heap offsets
// then thread 0 lays the page out and wave 0 finds the page's offset in the block with a decoupled
// look-back that reads 64 predecessors per round (ballot for the nearest inclusive prefix).  The
// write stages two columns at a time in LDS (values ORed into their words, then coalesced 8-byte
// stores); the string heap is assembled in LDS by each row's owner (8-byte source loads) and written
// out word by word.  Every word is folded into the page checksum on the way out.  The grid is sized
// for the largest step; surplus tickets exit.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "swtypes.h"
#include "swseg.h"

// Workgroup geometry: SW_SEG_SBLK threads per page (RPT = 1024 / SBLK rows each); SW_SEG_MIN_WAVES
// asks the compiler for at least that many waves per SIMD (a VGPR budget).  Measured in
// profiles/r5_encode (1M rows with strings): 256 threads at 221 VGPRs (2 waves / SIMD) 181 us; 512
// threads held to 128 VGPRs (4 waves / SIMD, 18 spilled) 156 us -- twice the waves per page and per
// CU hide the page's dependent load rounds; 1024 threads 189 us (one page per CU).
#ifndef SW_SEG_SBLK
#define SW_SEG_SBLK 512
#endif
#ifndef SW_SEG_MIN_WAVES
#define SW_SEG_MIN_WAVES 4
#endif
#define SBLK SW_SEG_SBLK
#define SWAVES (SBLK / 64)
#define RPT (SEG_PAGE_ROWS / SBLK)
#define HEAP_LDS 26624     // heap bytes a page can stage in LDS (the column staging union); larger heaps
                           // are gathered straight from the raw batch

typedef unsigned long long ull;

struct SwSegArgs {
  const SwOutRec* rows;        // this step's rows (device), persisted order
  const SwSegAux* aux;         // their encoder aux (device), same order
  const uint8_t* raw;          // the batch the rows were decoded from (null: no row has strings)
  const int64_t* cursor;       // [store_cursor, step_cursor0]: rows = cursor[0] - cursor[1]
  uint8_t* out;                // block (device)
  int64_t out_cap;
  uint64_t* state;             // [max_pages + SEG_ST_WORDS]: look-back words, ticket, outputs, accumulators
  int64_t max_pages;
  uint64_t* stamps;            // profiling: [page * 16 + phase] s_memrealtime stamps (null: off)
  // end-of-step snapshot into mapped host memory, written by the last workgroup (what
  // k_step_snapshot does in its own dispatch; null host: none): the step's u32 scalars -> host[0..15],
  // this block's (bytes, errors, first sequence) -> host[16..21], the re-key carry counts ->
  // host[22..23], the reject-ref counters -> host[24..25]
  const uint32_t* snap_scalars;
  const uint32_t* snap_rej;
  const uint32_t* snap_carry;
  uint32_t* snap_host;
};

// phase stamps of a page (profiling builds of the caller only: a null pointer costs a branch)
#define SEG_STAMP(i) do { if (a.stamps && threadIdx.x == 0) a.stamps[(size_t)page * 16 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)

#define LB_AGG (1ull << 62)
#define LB_INC (2ull << 62)
#define LB_VAL ((1ull << 62) - 1)
#define LB_SPIN_LIMIT (1u << 22)

__device__ __forceinline__ uint32_t lane64() { return threadIdx.x & 63; }

__device__ __forceinline__ ull wmin(ull v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) { const ull o = __shfl_xor(v, d, 64); v = o < v ? o : v; }
  return v;
}
__device__ __forceinline__ ull wmax(ull v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) { const ull o = __shfl_xor(v, d, 64); v = o > v ? o : v; }
  return v;
}
__device__ __forceinline__ ull wxor(ull v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v ^= __shfl_xor(v, d, 64);
  return v;
}
__device__ __forceinline__ ull wsum(ull v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// Bytes [off, off + n) of the raw batch (n <= 64) as 8 words, w[k] = bytes 8k .. 8k+7, zero past n.
// Aligned 8-byte loads of only the words the span touches (never past its last word).
__device__ __forceinline__ void load_words8(const uint8_t* raw, uint32_t off, uint32_t n, ull (&w)[8]) {
  const ull* src = reinterpret_cast<const ull*>(raw + (off & ~7u));
  const uint32_t sh = (off & 7u) * 8u;
  const uint32_t nsrc = ((off & 7u) + n + 7u) >> 3;      // source words the span touches (<= 9)
  ull cur = nsrc > 0 ? src[0] : 0ull;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const ull nxt = (uint32_t)(k + 1) < nsrc ? src[k + 1] : 0ull;
    ull v = sh ? ((cur >> sh) | (nxt << (64u - sh))) : cur;
    const uint32_t b = 8u * (uint32_t)k;
    v = b >= n ? 0ull : (b + 8u > n ? (v & (~0ull >> (64u - 8u * (n - b)))) : v);
    w[k] = v;
    cur = nxt;
  }
}

// 0x80 in every byte of x that is not a lowercase hex digit ('0'-'9', 'a'-'f'): SWAR range tests
// (bytes with the high bit set are never hex; the adds cannot carry across bytes)
__device__ __forceinline__ ull nonhex_mask(ull x) {
  const ull H = 0x8080808080808080ull;
  const ull y = x & ~H;
  const ull ge30 = (y + 0x5050505050505050ull) & H, ge3a = (y + 0x4646464646464646ull) & H;
  const ull ge61 = (y + 0x1f1f1f1f1f1f1f1full) & H, ge67 = (y + 0x1919191919191919ull) & H;
  const ull hex = ((ge30 & ~ge3a) | (ge61 & ~ge67)) & ~(x & H);
  return ~hex & H;
}

// Last non-hex byte (+1, absolute) of an id chunk: bytes base .. base + n (n <= 64) in w.
__device__ __forceinline__ uint32_t last_nonhex(const ull (&w)[8], uint32_t n, uint32_t base, uint32_t last) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint32_t b0 = 8u * (uint32_t)q;
    if (b0 < n) {
      ull m = nonhex_mask(w[q]);
      const uint32_t nv = n - b0;
      if (nv < 8u) m &= (1ull << (8u * nv)) - 1ull;
      if (m) last = base + b0 + ((63u - (uint32_t)__builtin_clzll(m)) >> 3) + 1u;
    }
  }
  return last;
}

// raw bytes [off, off + n) -> LDS bytes dst[0 .. n) (aligned 8-byte source loads, two in flight)
__device__ __forceinline__ void copy_to_lds(const uint8_t* raw, uint32_t off, uint32_t n, uint8_t* dst) {
  const uint32_t end = off + n;
  for (uint32_t wa = off & ~7u; wa < end; wa += 16u) {
    const ull v0 = *reinterpret_cast<const ull*>(raw + wa);
    const ull v1 = wa + 8u < end ? *reinterpret_cast<const ull*>(raw + wa + 8u) : 0ull;
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const uint32_t p = wa + (uint32_t)b;
      if (p >= off && p < end) dst[p - off] = (uint8_t)((b < 8 ? v0 : v1) >> (8 * (b & 7)));
    }
  }
}

// ----------------------------------------------------------------------------- page row
struct SRow {
  int64_t date;
  double v0, v1, v2;
  int32_t asg;
  uint16_t name;
  uint8_t et, level;
  SegRowStr s;
  bool valid;
};

// integer value (order-preserving unsigned) of column c; altnum given by the caller
__device__ __forceinline__ ull sval(int c, const SRow& r, uint32_t pfx, ull altnum) {
  switch (c) {
    case SEG_ETYPE: return seg_ord((int64_t)r.et);
    case SEG_LEVEL: return seg_ord((int64_t)r.level);
    case SEG_DATE: return seg_ord(r.date);
    case SEG_ASG: return seg_ord((int64_t)r.asg);
    case SEG_NAME: return seg_ord((int64_t)r.name);
    case SEG_FLAGS: return seg_ord((int64_t)r.s.flags);
    case SEG_ALTK: return seg_ord((int64_t)r.s.altk);
    case SEG_ALTLEN: return seg_ord((int64_t)(r.s.alt_len - pfx));
    case SEG_ALTNUM: return altnum;
    case SEG_MSGLEN: return seg_ord((int64_t)r.s.msg_len);
    case SEG_METALEN: return seg_ord((int64_t)r.s.meta_len);
    default: return 0;
  }
}

__device__ __forceinline__ double sdbl(int c, const SRow& r) {
  return (c == SEG_MXV || c == SEG_LAT) ? r.v0 : (c == SEG_LON ? r.v1 : r.v2);
}

__device__ __forceinline__ int exp_hint(int c) { return c == SEG_MXV ? 2 : c == SEG_ELEV ? 1 : 6; }

__device__ __forceinline__ bool smem(int c, const SRow& r, int mode) {
  return r.valid && seg_member(c, r.et, r.s.flags, mode);
}

// block-scanned counters: 15 member counts, 4 exception counts (u16 prefixes); heap bytes (u32)
#define NCNT (SEG_NCOL + 4)
#define NDBL 4
#define NSLOT 48

// Columns are written two at a time; no pair holds two double columns (one exception stage).
__device__ __forceinline__ constexpr int seg_pair(int pr, int g) {
  return pr == 0 ? (g ? SEG_LEVEL : SEG_ETYPE) : pr == 1 ? (g ? SEG_ASG : SEG_DATE)
       : pr == 2 ? (g ? SEG_MXV : SEG_NAME) : pr == 3 ? (g ? SEG_FLAGS : SEG_LAT)
       : pr == 4 ? (g ? SEG_ALTK : SEG_LON) : pr == 5 ? (g ? SEG_ALTLEN : SEG_ELEV)
       : pr == 6 ? (g ? SEG_MSGLEN : SEG_ALTNUM) : (g ? -1 : SEG_METALEN);
}

struct SegLds {
  ull red[SWAVES][NSLOT];      // per-wave partial reductions
  ull res[NSLOT];              // block results
  uint32_t wtot[SWAVES][NCNT + 1];
  uint16_t pre[NCNT][SBLK];    // exclusive member / exception prefixes of each thread
  uint32_t hpre[SBLK];         // exclusive heap-byte prefix of each thread
  uint32_t tot[NCNT + 1];
  // staging (two columns, one exception list), or the staged string heap, or the heap gather tables
  union {
    struct {
      ull vals[2][SEG_PAGE_ROWS];
      ull xraw[SEG_PAGE_ROWS];
      uint16_t xidx[SEG_PAGE_ROWS];
    } st;
    uint8_t heap[HEAP_LDS];
    struct {
      uint32_t hoff[SEG_PAGE_ROWS + 1];    // row heap offsets (after the prefix)
      uint32_t src[SEG_PAGE_ROWS][3];      // alt remainder / msg / meta source offsets in raw
      uint16_t len[SEG_PAGE_ROWS][3];
    } hp;
  } u;
  SwSegPageHdr hdr;
  ull falt[8];                 // the page's first alternate id, bytes 0 .. 63 (the prefix source)
  int first_alt;
  uint32_t alt_off0, alt_len0;
  uint32_t page;
  ull page_base, page_size;
  int exps[NDBL];
};

__device__ __forceinline__ ull lb_load(uint64_t* p) {
  return __hip_atomic_load((ull*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t* p, ull v) {
  __hip_atomic_store((ull*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- wave reductions / scans on DPP (VALU lane moves, no LDS round trip per step).  Row prefix by
// row_shr 1, 2, 4, 8, then row_bcast15 (rows 1, 3) and row_bcast31 (rows 2, 3): lane 63 ends up with
// the whole wave.  Lanes without a source keep `old` (the operation's identity).
template <int CTRL, int RM = 0xf, int BM = 0xf>
__device__ __forceinline__ uint32_t dpp32(uint32_t v, uint32_t old) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, RM, BM, false);
}
template <int CTRL, int RM = 0xf, int BM = 0xf>
__device__ __forceinline__ ull dpp64(ull v, ull old) {
  return ((ull)dpp32<CTRL, RM, BM>((uint32_t)(v >> 32), (uint32_t)(old >> 32)) << 32) |
         (ull)dpp32<CTRL, RM, BM>((uint32_t)v, (uint32_t)old);
}
__device__ __forceinline__ ull readlane63(ull v) {
  return ((ull)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63) << 32) |
         (ull)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
}
template <bool MX>
__device__ __forceinline__ ull dpp_minmax(ull v) {
  const ull id = MX ? 0ull : ~0ull;
#define SEG_MM(x) { const ull o = (x); v = MX ? (o > v ? o : v) : (o < v ? o : v); }
  SEG_MM((dpp64<0x111>(v, id)));
  SEG_MM((dpp64<0x112>(v, id)));
  SEG_MM((dpp64<0x114>(v, id)));
  SEG_MM((dpp64<0x118>(v, id)));
  SEG_MM((dpp64<0x142, 0xa>(v, id)));
  SEG_MM((dpp64<0x143, 0xc>(v, id)));
#undef SEG_MM
  return readlane63(v);
}
// inclusive prefix sum over the wave (lane i: lanes 0..i)
__device__ __forceinline__ uint32_t dpp_scan(uint32_t v) {
  v += dpp32<0x111>(v, 0u);
  v += dpp32<0x112>(v, 0u);
  v += dpp32<0x114>(v, 0u);
  v += dpp32<0x118>(v, 0u);
  v += dpp32<0x142, 0xa>(v, 0u);
  v += dpp32<0x143, 0xc>(v, 0u);
  return v;
}

// Wave partial of one reduction slot (wave-uniform, stored once); block_finish combines the waves.
__device__ __forceinline__ void wave_put(SegLds& L, int slot, ull v, bool mx) {
  const ull r = mx ? dpp_minmax<true>(v) : dpp_minmax<false>(v);
  if (lane64() == 0) L.red[threadIdx.x >> 6][slot] = r;
}

// Slots [0, ns): bit i of maxmask = max, else min.  Two barriers; L.res valid for every thread after.
__device__ __forceinline__ void block_finish(SegLds& L, int ns, uint64_t maxmask) {
  __syncthreads();
  if ((int)threadIdx.x < ns) {
    const int i = threadIdx.x;
    const bool mx = (maxmask >> i) & 1;
    ull r = L.red[0][i];
#pragma unroll
    for (int w = 1; w < SWAVES; ++w) { const ull o = L.red[w][i]; r = mx ? (o > r ? o : r) : (o < r ? o : r); }
    L.res[i] = r;
  }
  __syncthreads();
}

// state = u64[max_pages + 8]: [0, max_pages) look-back words; then
//   +0 ticket, +1 block bytes (out), +2 errors (out), +3 first store sequence (out),
//   +4 bytes accumulator, +5 errors accumulator, +6 blocks done.
// The workgroup that finishes last publishes the accumulators to the outputs and zeroes every
// word the next launch relies on (look-back words, ticket, accumulators, done): no memset node
// before each encode.  The allocation starts zeroed.
#define SEG_ST_TICKET 0
#define SEG_ST_BYTES 1
#define SEG_ST_ERRORS 2
#define SEG_ST_FIRST 3
#define SEG_ST_BYTES_ACC 4
#define SEG_ST_ERRORS_ACC 5
#define SEG_ST_DONE 6
#define SEG_ST_WORDS 8

__device__ __forceinline__ void seg_encode_page(const SwSegArgs& a, SegLds& L) {
  uint64_t* ticket = a.state + a.max_pages;
  uint64_t* bytes_out = ticket + SEG_ST_BYTES_ACC;
  uint64_t* errors = ticket + SEG_ST_ERRORS_ACC;
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
  if (page == 0 && threadIdx.x == 0) ticket[SEG_ST_FIRST] = (uint64_t)c0;   // first store sequence, for the host
  if (n <= 0) {
    if (page == 0 && threadIdx.x == 0) {
      SwSegBlockHdr* h = reinterpret_cast<SwSegBlockHdr*>(a.out);
      h->n_rows = 0; h->n_pages = 0; h->bytes = data_start; h->flags = 0;
      page_off[0] = data_start;
      page_off[1] = 0;
      atomicMax((ull*)bytes_out, (ull)data_start);
    }
    return;
  }
  if ((int64_t)page >= np) return;
  const int64_t r0 = (int64_t)page * SEG_PAGE_ROWS;
  const int m = (int)(n - r0 < SEG_PAGE_ROWS ? n - r0 : SEG_PAGE_ROWS);
  SEG_STAMP(0);
  // ---- load RPT consecutive rows per thread: enriched row + encoder aux (both coalesced)
  SRow R[RPT];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const int idx = RPT * (int)threadIdx.x + k;
    SRow& r = R[k];
    r.valid = idx < m;
    if (r.valid) {
      const int64_t j = r0 + idx;
      const uint4 q0 = *reinterpret_cast<const uint4*>(&a.rows[j]);
      const uint4 q1 = *(reinterpret_cast<const uint4*>(&a.rows[j]) + 1);
      const SwSegAux x = a.aux[j];
      r.date = (int64_t)(((ull)q0.y << 32) | q0.x);
      r.v0 = sw_bits_f64(((ull)q0.w << 32) | q0.z);
      r.v1 = sw_bits_f64(((ull)q1.y << 32) | q1.x);
      r.asg = (int32_t)q1.z;
      r.name = (uint16_t)(q1.w & 0xffffu);
      r.et = (uint8_t)((q1.w >> 16) & 0xffu);
      r.level = (uint8_t)(q1.w >> 24);
      r.v2 = x.v2;
      r.s = seg_aux_strings(x);
      if (!a.raw) {                      // no batch: no strings (the CPU encoder without raw)
        r.s.flags &= ~(uint32_t)(SEGF_HAS_ALT | SEGF_HAS_META);
        r.s.alt_off = r.s.alt_len = r.s.meta_off = r.s.meta_len = r.s.msg_off = r.s.msg_len = r.s.altk = 0;
      }
    } else {
      r.date = 0; r.v0 = r.v1 = r.v2 = 0.0; r.asg = 0; r.name = 0; r.et = 0; r.level = 0;
      r.s.alt_off = r.s.alt_len = r.s.msg_off = r.s.msg_len = r.s.meta_off = r.s.meta_len = r.s.altk = r.s.flags = 0;
    }
  }

  SEG_STAMP(1);
  // ---- R1: first row with an alternate id; decimal exponent per double column
  {
    ull fa_local = ~0ull;
#pragma unroll
    for (int k = RPT - 1; k >= 0; --k)
      if (R[k].valid && (R[k].s.flags & SEGF_HAS_ALT)) fa_local = (ull)(RPT * threadIdx.x + k);
    wave_put(L, 0, fa_local, false);
#pragma unroll
    for (int d = 0; d < NDBL; ++d) {
      const int c = SEG_MXV + d;
      int e = 0;
#pragma unroll
      for (int k = 0; k < RPT; ++k) {
        if (!smem(c, R[k], SEG_ALT_RAW)) continue;
        const int ei = seg_dec_exp_from(sdbl(c, R[k]), exp_hint(c));
        if (ei != SEG_EXC_NONE && ei > e) e = ei;
      }
      wave_put(L, 1 + d, (ull)e, true);
    }
    block_finish(L, 1 + NDBL, 0x1eull);
    if (threadIdx.x == 0) {
      L.first_alt = L.res[0] == ~0ull ? -1 : (int)L.res[0];
#pragma unroll
      for (int d = 0; d < NDBL; ++d) L.exps[d] = (int)L.res[1 + d];
    }
    // the row's owner publishes the first alternate id's location
    const int fa = L.res[0] == ~0ull ? -1 : (int)L.res[0];
    if (fa >= 0 && fa / RPT == (int)threadIdx.x) {
      uint32_t o0 = 0, l0 = 0;
#pragma unroll
      for (int k = 0; k < RPT; ++k)
        if (RPT * (int)threadIdx.x + k == fa) { o0 = R[k].s.alt_off; l0 = R[k].s.alt_len; }
      L.alt_off0 = o0;
      L.alt_len0 = l0;
      ull fw[8];
      load_words8(a.raw, o0, l0 < SEG_ALT_PFX_MAX ? l0 : SEG_ALT_PFX_MAX, fw);
#pragma unroll
      for (int k = 0; k < 8; ++k) L.falt[k] = fw[k];
    }
    __syncthreads();
  }
  const int first_alt = L.first_alt;
  const uint32_t a_len0 = first_alt >= 0 ? L.alt_len0 : 0u;

  SEG_STAMP(2);
  // ---- R2: alternate-id prefix / hex test; integer min / max; quantised double min / max
  // slots: [0] min LCP, [1] max last-non-hex+1, [2] min alt len, [3] max alt len,
  //        [4 + 2c] / [5 + 2c] min / max of integer column c (ALTLEN follows from [2] / [3], ALTNUM
  //        needs the mode: R3), [34 + 2d] / [35 + 2d] min / max of the quantised double column d
  {
    const uint32_t plim = a_len0 < SEG_ALT_PFX_MAX ? a_len0 : SEG_ALT_PFX_MAX;
    ull lcp = ~0ull, lnh = 0, lmin = ~0ull, lmax = 0;
    // first 64 bytes of every row's id: all the thread's rows' loads issued before any is used
    ull W[RPT][8];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const SRow& r = R[k];
      const bool has = r.valid && (r.s.flags & SEGF_HAS_ALT);
      const uint32_t n = has ? (r.s.alt_len < 64u ? r.s.alt_len : 64u) : 0u;
      load_words8(a.raw, has ? r.s.alt_off : 0u, n, W[k]);
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      SRow& r = R[k];
      if (!(r.valid && (r.s.flags & SEGF_HAS_ALT))) continue;
      const uint32_t len = r.s.alt_len;
      // common prefix with the first id: first differing byte of the word xor
      uint32_t l = plim < len ? plim : len;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const ull x = W[k][q] ^ L.falt[q];
        if (x) {
          const uint32_t d = 8u * (uint32_t)q + ((uint32_t)__builtin_ctzll(x) >> 3);
          l = d < l ? d : l;
        }
      }
      uint32_t last = last_nonhex(W[k], len < 64u ? len : 64u, 0u, 0u);
      for (uint32_t base = 64; base < len; base += 64) {      // ids longer than 64 bytes (rare)
        ull w[8];
        const uint32_t n = len - base < 64u ? len - base : 64u;
        load_words8(a.raw, r.s.alt_off + base, n, w);
        last = last_nonhex(w, n, base, last);
      }
      lcp = (ull)l < lcp ? (ull)l : lcp;
      lnh = (ull)last > lnh ? (ull)last : lnh;
      lmin = (ull)len < lmin ? (ull)len : lmin;
      lmax = (ull)len > lmax ? (ull)len : lmax;
    }
    wave_put(L, 0, lcp, false);
    wave_put(L, 1, lnh, true);
    wave_put(L, 2, lmin, false);
    wave_put(L, 3, lmax, true);
#pragma unroll
    for (int c = 0; c < SEG_NCOL; ++c) {
      if (seg_is_double(c) || c == SEG_ALTLEN || c == SEG_ALTNUM) continue;
      ull lo = ~0ull, hi = 0;
#pragma unroll
      for (int k = 0; k < RPT; ++k) {
        if (!smem(c, R[k], SEG_ALT_RAW)) continue;
        const ull u = sval(c, R[k], 0, 0);
        lo = u < lo ? u : lo;
        hi = u > hi ? u : hi;
      }
      wave_put(L, 4 + 2 * c, lo, false);
      wave_put(L, 5 + 2 * c, hi, true);
    }
#pragma unroll
    for (int d = 0; d < NDBL; ++d) {
      const int c = SEG_MXV + d;
      const int e = L.exps[d];
      ull lo = ~0ull, hi = 0;
#pragma unroll
      for (int k = 0; k < RPT; ++k) {
        if (!smem(c, R[k], SEG_ALT_RAW)) continue;
        int64_t q;
        if (seg_dec_at(sdbl(c, R[k]), e, &q)) {
          const ull u = seg_ord(q);
          lo = u < lo ? u : lo;
          hi = u > hi ? u : hi;
        }
      }
      wave_put(L, 34 + 2 * d, lo, false);
      wave_put(L, 35 + 2 * d, hi, true);
    }
    // max slots: 1, 3, every odd slot from 5 (unused slots reduce garbage nobody reads)
    block_finish(L, 42, 0x2aaaaaaaaaaull);
  }
  // prefix and mode (every thread computes the same from L.res)
  uint32_t pfx = 0, mode = SEG_ALT_RAW, width = 0;
  if (first_alt >= 0) {
    pfx = (uint32_t)L.res[0];
    const uint32_t wmn = (uint32_t)L.res[2] - pfx, wmx = (uint32_t)L.res[3] - pfx;
    if ((uint32_t)L.res[1] <= pfx && wmn == wmx && wmn >= 1 && wmn <= 16) { mode = SEG_ALT_HEX; width = wmn; }
  }

  SEG_STAMP(3);
  // ---- R3: member / exception / heap scans (+ ALTNUM min / max in hex mode)
  ull altnum[RPT];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    // hex mode: each id's remainder (the last `width` <= 16 bytes) as a number
    altnum[k] = 0;
    if (mode == SEG_ALT_HEX && R[k].valid && (R[k].s.flags & SEGF_HAS_ALT)) {
      ull w[8];
      load_words8(a.raw, R[k].s.alt_off + pfx, width, w);
      ull v = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if ((uint32_t)i < width) {
          const uint32_t c = (uint32_t)((i < 8 ? w[0] : w[1]) >> (8 * (i & 7))) & 0xffu;
          v = (v << 4) | (ull)(c <= 57u ? c - 48u : c - 87u);
        }
      }
      altnum[k] = v;
    }
  }
  {
    const uint32_t lane = lane64(), wid = threadIdx.x >> 6;
    uint32_t hb = 0;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const SRow& r = R[k];
      if (!r.valid) continue;
      if (mode == SEG_ALT_RAW && (r.s.flags & SEGF_HAS_ALT)) hb += r.s.alt_len - pfx;
      hb += r.s.msg_len + r.s.meta_len;
    }
    uint32_t ex[NCNT + 1];
#pragma unroll
    for (int c = 0; c <= NCNT; ++c) {
      uint32_t x = 0;
      if (c < SEG_NCOL) {
#pragma unroll
        for (int k = 0; k < RPT; ++k) x += smem(c, R[k], (int)mode) ? 1u : 0u;
      } else if (c < NCNT) {
        const int d = c - SEG_NCOL;
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
          int64_t q;
          if (smem(SEG_MXV + d, R[k], (int)mode) && !seg_dec_at(sdbl(SEG_MXV + d, R[k]), L.exps[d], &q)) ++x;
        }
      } else {
        x = hb;
      }
      const uint32_t inc = dpp_scan(x);
      if (lane == 63) L.wtot[wid][c] = inc;
      ex[c] = inc - x;                 // exclusive within the wave
    }
    // ALTNUM min / max rides along (hex mode only)
    ull lo = ~0ull, hi = 0;
#pragma unroll
    for (int k = 0; k < RPT; ++k)
      if (smem(SEG_ALTNUM, R[k], (int)mode)) { lo = altnum[k] < lo ? altnum[k] : lo; hi = altnum[k] > hi ? altnum[k] : hi; }
    wave_put(L, 44, lo, false);
    wave_put(L, 45, hi, true);
    __syncthreads();
    if (threadIdx.x <= NCNT) {
      const int c = threadIdx.x;
      uint32_t acc = 0;
#pragma unroll
      for (int w = 0; w < SWAVES; ++w) { const uint32_t t = L.wtot[w][c]; L.wtot[w][c] = acc; acc += t; }
      L.tot[c] = acc;
    } else if (threadIdx.x == 64) {
      ull l2 = L.red[0][44], h2 = L.red[0][45];
#pragma unroll
      for (int w = 1; w < SWAVES; ++w) {
        l2 = L.red[w][44] < l2 ? L.red[w][44] : l2;
        h2 = L.red[w][45] > h2 ? L.red[w][45] : h2;
      }
      L.res[44] = l2;
      L.res[45] = h2;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NCNT; ++c) L.pre[c][threadIdx.x] = (uint16_t)(ex[c] + L.wtot[wid][c]);
    L.hpre[threadIdx.x] = ex[NCNT] + L.wtot[wid][NCNT];
  }

  SEG_STAMP(4);
  // ---- layout (thread 0) + look-back for the page's place in the block
  if (threadIdx.x == 0) {
    SwSegPageHdr& H = L.hdr;
    uint32_t off = SEG_PAGE_HDR;
    for (int c = 0; c < SEG_NCOL; ++c) {
      SwSegCol& cd = H.cols[c];
      const uint32_t count = L.tot[c];
      cd.count = (uint16_t)count;
      cd.pad0 = 0;
      cd.pad1 = 0;
      if (!seg_is_double(c)) {
        const int slo = c == SEG_ALTLEN ? 2 : c == SEG_ALTNUM ? 44 : 4 + 2 * c;
        const ull rlo = L.res[slo], rhi = L.res[slo + 1];
        const ull lo = c == SEG_ALTLEN ? seg_ord((int64_t)rlo - (int64_t)pfx) : rlo;
        const ull hi = c == SEG_ALTLEN ? seg_ord((int64_t)rhi - (int64_t)pfx) : rhi;
        cd.base = count ? lo : 0;
        cd.bits = (uint8_t)(count ? seg_bitwidth(hi - lo) : 0);
        cd.exp = -1;
        cd.n_exc = 0;
      } else {
        const int d = c - SEG_MXV;
        const uint32_t ne = L.tot[SEG_NCOL + d];
        const bool any = count > ne;
        cd.base = any ? L.res[34 + 2 * d] : 0;
        cd.bits = (uint8_t)(any ? seg_bitwidth(L.res[35 + 2 * d] - L.res[34 + 2 * d]) : 0);
        cd.exp = (int8_t)L.exps[d];
        cd.n_exc = (uint16_t)ne;
      }
      cd.data_off = off;
      off += seg_col_bytes(cd.count, cd.bits, cd.n_exc);
    }
    const uint32_t heap = pfx + L.tot[NCNT];
    H.n_rows = (uint32_t)m;
    H.heap_off = off;
    H.heap_bytes = heap;
    H.alt_pfx = (uint8_t)pfx;
    H.alt_mode = (uint8_t)mode;
    H.alt_width = (uint8_t)width;
    H.pad0 = 0;
    H.asg_max = (int32_t)seg_unord(L.res[5 + 2 * SEG_ASG]);
    H.date_max = seg_unord(L.res[5 + 2 * SEG_DATE]);
    H.bytes = off + ((heap + 7u) & ~7u);
    H.checksum = 0;
    L.page_size = H.bytes;
  }
  __syncthreads();
  SEG_STAMP(5);
  // column word staging starts zeroed (the pair writer ORs values in and re-zeroes what it wrote out)
  for (uint32_t w = threadIdx.x; w < 2u * SEG_PAGE_ROWS; w += SBLK) (&L.u.st.vals[0][0])[w] = 0;
  // ---- the page's offset in the block: decoupled look-back by wave 0, 64 predecessors per round
  if (threadIdx.x < 64) {
    const uint32_t lane = lane64();
    const ull size = L.page_size;
    ull excl = 0;
    bool failed = false;
    if (page == 0) {
      if (lane == 0) lb_store(&a.state[0], LB_INC | size);
    } else {
      if (lane == 0) lb_store(&a.state[page], LB_AGG | size);
      int64_t p = (int64_t)page - 1;
      while (true) {
        const int64_t q = p - (int64_t)lane;              // lane 0 = the nearest predecessor
        ull st = q >= 0 ? lb_load(&a.state[q]) : LB_INC;  // before page 0: an empty inclusive prefix
        uint32_t spins = 0;
        while (__any((st >> 62) == 0)) {                  // wait until the whole window is published
          if (++spins > LB_SPIN_LIMIT) { failed = true; break; }
          __builtin_amdgcn_s_sleep(1);
          if ((st >> 62) == 0) st = lb_load(&a.state[q]);
        }
        if (failed) break;
        const ull inc = __ballot((st >> 62) == 2);
        if (inc) {                                         // nearest inclusive prefix: stop there
          const int first = __ffsll((long long)inc) - 1;
          excl += wsum((int)lane <= first ? (st & LB_VAL) : 0ull);
          break;
        }
        excl += wsum(st & LB_VAL);
        p -= 64;
      }
      if (lane == 0 && !failed) lb_store(&a.state[page], LB_INC | (excl + size));
    }
    if (lane == 0) {
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
          h->flags = 0;                  // the index build (swindex.hip) sets SEG_FLAG_INDEX
          atomicMax((ull*)bytes_out, base + size);
        }
      }
    }
  }
  __syncthreads();
  SEG_STAMP(6);
  if (L.page_base == ~0ull) return;
  uint8_t* pg = a.out + L.page_base;
  ull cs = 0;

  SEG_STAMP(7);
  // ---- write the columns, two at a time through LDS.  One instantiation per pair: every column
  // index is a compile-time constant, so the rows' fields are selected statically (in registers)
  auto write_pair = [&](auto PR) {
    constexpr int pr = decltype(PR)::value;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int c = seg_pair(pr, g);
      if (c < 0) break;
      const SwSegCol& cd = L.hdr.cols[c];
      uint32_t i = L.pre[c][threadIdx.x];
      uint32_t x = seg_is_double(c) ? L.pre[SEG_NCOL + (c - SEG_MXV)][threadIdx.x] : 0u;
#pragma unroll
      for (int k = 0; k < RPT; ++k) {
        if (!smem(c, R[k], (int)mode)) continue;
        ull v = 0;
        if (!seg_is_double(c)) {
          v = sval(c, R[k], pfx, altnum[k]) - cd.base;
        } else {
          const double dv = sdbl(c, R[k]);
          int64_t q;
          if (seg_dec_at(dv, cd.exp, &q)) {
            v = seg_ord(q) - cd.base;
          } else {
            L.u.st.xidx[x] = (uint16_t)i;
            L.u.st.xraw[x] = sw_f64_bits(dv);
            ++x;
          }
        }
        // pack straight into the column's words (LDS 64-bit OR: values of neighbouring rows share words)
        if (v) {
          const uint32_t bp = i * (uint32_t)cd.bits, w = bp >> 6, sh = bp & 63u;
          atomicOr(&L.u.st.vals[g][w], v << sh);
          if (sh + cd.bits > 64u) atomicOr(&L.u.st.vals[g][w + 1], v >> (64u - sh));
        }
        ++i;
      }
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int c = seg_pair(pr, g);
      if (c < 0) break;
      const SwSegCol cd = L.hdr.cols[c];
      const uint32_t bits = cd.bits, cnt = cd.count;
      const uint32_t nw = seg_col_words(cnt, (int)bits);
      for (uint32_t w = threadIdx.x; w < nw; w += SBLK) {
        const ull word = L.u.st.vals[g][w];
        L.u.st.vals[g][w] = 0;             // zero again for the next pair (this thread's words only)
        const uint32_t off = cd.data_off + 8u * w;
        *reinterpret_cast<ull*>(pg + off) = word;
        cs ^= seg_mix_word(word, off >> 3);
      }
      if (seg_is_double(c) && cd.n_exc) {
        const uint32_t ne = cd.n_exc;
        const uint32_t xo = cd.data_off + 8u * nw;
        const uint32_t nidx = (2u * ne + 7u) / 8u;
        for (uint32_t w = threadIdx.x; w < nidx; w += SBLK) {
          ull word = 0;
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j)
            if (4 * w + j < ne) word |= (ull)L.u.st.xidx[4 * w + j] << (16 * j);
          *reinterpret_cast<ull*>(pg + xo + 8u * w) = word;
          cs ^= seg_mix_word(word, (xo >> 3) + w);
        }
        const uint32_t ro = xo + 8u * nidx;
        for (uint32_t j = threadIdx.x; j < ne; j += SBLK) {
          *reinterpret_cast<ull*>(pg + ro + 8u * j) = L.u.st.xraw[j];
          cs ^= seg_mix_word(L.u.st.xraw[j], (ro >> 3) + j);
        }
      }
    }
    __syncthreads();         // the next pair reuses the staging arrays
  };
  write_pair(std::integral_constant<int, 0>{});
  write_pair(std::integral_constant<int, 1>{});
  write_pair(std::integral_constant<int, 2>{});
  write_pair(std::integral_constant<int, 3>{});
  write_pair(std::integral_constant<int, 4>{});
  write_pair(std::integral_constant<int, 5>{});
  write_pair(std::integral_constant<int, 6>{});
  write_pair(std::integral_constant<int, 7>{});

  SEG_STAMP(8);
  // ---- string heap
  const uint32_t heap_bytes = L.hdr.heap_bytes;
  if (heap_bytes && heap_bytes <= HEAP_LDS) {
    // staged in LDS: each thread copies its rows' strings to its heap prefix; the page's first
    // alternate id supplies the common prefix; the tail is zero-padded to a word
    uint8_t* hp = L.u.heap;
    const uint32_t hend = (heap_bytes + 7u) & ~7u;
    if (threadIdx.x < pfx) hp[threadIdx.x] = (uint8_t)(L.falt[threadIdx.x >> 3] >> (8u * (threadIdx.x & 7u)));
    if (threadIdx.x < hend - heap_bytes) hp[heap_bytes + threadIdx.x] = 0;
    uint32_t h = pfx + L.hpre[threadIdx.x];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const SRow& r = R[k];
      if (!r.valid) continue;
      if (mode == SEG_ALT_RAW && (r.s.flags & SEGF_HAS_ALT)) {
        const uint32_t nb = r.s.alt_len - pfx;
        copy_to_lds(a.raw, r.s.alt_off + pfx, nb, hp + h);
        h += nb;
      }
      if (r.s.msg_len) {
        copy_to_lds(a.raw, r.s.msg_off, r.s.msg_len, hp + h);
        h += r.s.msg_len;
      }
      if (r.s.meta_len) {
        copy_to_lds(a.raw, r.s.meta_off, r.s.meta_len, hp + h);
        h += r.s.meta_len;
      }
    }
    __syncthreads();
    const uint32_t hbase = L.hdr.heap_off;
    const ull* h64 = reinterpret_cast<const ull*>(hp);
    for (uint32_t w = threadIdx.x; w < (hend >> 3); w += SBLK) {
      const ull word = h64[w];
      const uint32_t off = hbase + 8u * w;
      *reinterpret_cast<ull*>(pg + off) = word;
      cs ^= seg_mix_word(word, off >> 3);
    }
  } else if (heap_bytes) {
    // larger than LDS: row sources into LDS, then a word-parallel gather from the raw batch
    {
      uint32_t h = L.hpre[threadIdx.x];
#pragma unroll
      for (int k = 0; k < RPT; ++k) {
        const int idx = RPT * (int)threadIdx.x + k;
        const SRow& r = R[k];
        if (idx > m) break;
        if (idx < m) {
          L.u.hp.hoff[idx] = h;
          const uint32_t alen = (mode == SEG_ALT_RAW && (r.s.flags & SEGF_HAS_ALT)) ? r.s.alt_len - pfx : 0u;
          L.u.hp.src[idx][0] = r.s.alt_off + pfx;
          L.u.hp.src[idx][1] = r.s.msg_off;
          L.u.hp.src[idx][2] = r.s.meta_off;
          L.u.hp.len[idx][0] = (uint16_t)alen;
          L.u.hp.len[idx][1] = (uint16_t)r.s.msg_len;
          L.u.hp.len[idx][2] = (uint16_t)r.s.meta_len;
          h += alen + r.s.msg_len + r.s.meta_len;
        } else {
          L.u.hp.hoff[m] = h;           // sentinel: heap bytes after the prefix
        }
      }
      if (m == RPT * SBLK && threadIdx.x == SBLK - 1) L.u.hp.hoff[m] = h;
    }
    __syncthreads();
    const uint32_t hwords = (heap_bytes + 7u) >> 3;
    const uint32_t hbase = L.hdr.heap_off;
    for (uint32_t w = threadIdx.x; w < hwords; w += SBLK) {
      ull word = 0;
      const uint32_t b0 = 8u * w;
      // row of the first body byte of the word (binary search over the heap offsets)
      int row = 0;
      uint32_t rel = 0;
      if (b0 + 8u > pfx) {
        const uint32_t t = b0 > pfx ? b0 - pfx : 0u;
        int lo = 0, hi = m;                // hoff[lo] <= t < hoff[hi]
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (L.u.hp.hoff[mid] <= t) lo = mid; else hi = mid;
        }
        row = lo;
        rel = t - L.u.hp.hoff[row];
      }
#pragma unroll
      for (uint32_t i = 0; i < 8; ++i) {
        const uint32_t b = b0 + i;
        if (b >= heap_bytes) break;
        uint8_t byte;
        if (b < pfx) {
          byte = (uint8_t)(L.falt[b >> 3] >> (8u * (b & 7u)));
        } else {
          // advance to the row / segment holding this byte
          while (row < m && rel >= (uint32_t)L.u.hp.len[row][0] + L.u.hp.len[row][1] + L.u.hp.len[row][2]) {
            rel -= (uint32_t)L.u.hp.len[row][0] + L.u.hp.len[row][1] + L.u.hp.len[row][2];
            ++row;
          }
          uint32_t q = rel, seg = 0;
          while (seg < 2 && q >= L.u.hp.len[row][seg]) { q -= L.u.hp.len[row][seg]; ++seg; }
          byte = a.raw[L.u.hp.src[row][seg] + q];
          ++rel;
        }
        word |= (ull)byte << (8 * i);
      }
      const uint32_t off = hbase + 8u * w;
      *reinterpret_cast<ull*>(pg + off) = word;
      cs ^= seg_mix_word(word, off >> 3);
    }
  }

  SEG_STAMP(9);
  // ---- page header words (word 1, the checksum, is written last and not summed)
  const ull* hw = reinterpret_cast<const ull*>(&L.hdr);
  for (uint32_t i = threadIdx.x; i < SEG_PAGE_HDR / 8; i += SBLK) {
    if (i == 1) continue;
    const ull w = hw[i];
    *reinterpret_cast<ull*>(pg + 8u * i) = w;
    cs ^= seg_mix_word(w, i);
  }
  cs = wxor(cs);
  __syncthreads();
  if (lane64() == 0) L.red[threadIdx.x >> 6][0] = cs;
  __syncthreads();
  if (threadIdx.x == 0) {
    ull t = 0;
#pragma unroll
    for (int w = 0; w < SWAVES; ++w) t ^= L.red[w][0];
    *reinterpret_cast<ull*>(pg + 8) = t;
  }
  SEG_STAMP(10);
}

__global__ __launch_bounds__(SBLK, SW_SEG_MIN_WAVES) void k_seg_encode(SwSegArgs a) {
  __shared__ SegLds L;
  seg_encode_page(a, L);
  // ---- last workgroup out: publish the results, re-arm the state for the next launch.  Every
  // word the epilogue reads was written by a device-scope atomic (ticket, accumulators) or an
  // agent-scope store (look-back words), so no release fence is needed before the count.
  uint64_t* st = a.state + a.max_pages;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    L.page = (uint32_t)(__hip_atomic_fetch_add((ull*)&st[SEG_ST_DONE], 1ull, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT) == (ull)gridDim.x - 1);
  __syncthreads();
  if (!L.page) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (threadIdx.x == 0) {
    const ull bytes = lb_load(&st[SEG_ST_BYTES_ACC]), errors = lb_load(&st[SEG_ST_ERRORS_ACC]);
    st[SEG_ST_BYTES] = bytes;
    st[SEG_ST_ERRORS] = errors;
    if (a.snap_host) {
      const ull first = lb_load(&st[SEG_ST_FIRST]);
      a.snap_host[16] = (uint32_t)bytes; a.snap_host[17] = (uint32_t)(bytes >> 32);
      a.snap_host[18] = (uint32_t)errors; a.snap_host[19] = (uint32_t)(errors >> 32);
      a.snap_host[20] = (uint32_t)first; a.snap_host[21] = (uint32_t)(first >> 32);
    }
    lb_store(&st[SEG_ST_TICKET], 0);
    lb_store(&st[SEG_ST_BYTES_ACC], 0);
    lb_store(&st[SEG_ST_ERRORS_ACC], 0);
    lb_store(&st[SEG_ST_DONE], 0);
  }
  for (int64_t i = threadIdx.x; i < a.max_pages; i += SBLK) lb_store(&a.state[i], 0);
  if (a.snap_host) {
    const uint32_t t = threadIdx.x;
    if (t < 16) a.snap_host[t] = a.snap_scalars[t];
    else if (t == 22 || t == 23) a.snap_host[t] = a.snap_carry ? a.snap_carry[t - 22] : 0u;
    else if (t == 24 || t == 25) a.snap_host[t] = a.snap_rej ? a.snap_rej[t - 24] : 0u;
  }
}

extern "C" {

// Encode this step's rows into `out`.  state = u64[max_pages + 8], zeroed when allocated and re-armed
// by the kernel itself; afterwards state[max_pages + 1] = block bytes (~0 on error),
// state[max_pages + 2] = errors, state[max_pages + 3] = the store sequence of the block's first row.
int sw_seg_encode_stamped(const void* rows, const void* aux, const uint8_t* raw, const int64_t* cursor, uint8_t* out,
                          int64_t out_cap, uint64_t* state, int64_t max_pages, uint64_t* stamps, hipStream_t s);

static int seg_encode_launch(const SwSegArgs& a, hipStream_t s) {
  const unsigned grid = (unsigned)(a.max_pages > 0 ? a.max_pages : 1);
  k_seg_encode<<<grid, SBLK, 0, s>>>(a);
  return (int)hipGetLastError();
}

int sw_seg_encode(const void* rows, const void* aux, const uint8_t* raw, const int64_t* cursor, uint8_t* out,
                  int64_t out_cap, uint64_t* state, int64_t max_pages, hipStream_t s) {
  return sw_seg_encode_stamped(rows, aux, raw, cursor, out, out_cap, state, max_pages, nullptr, s);
}

// Encode + the end-of-step snapshot in the same dispatch (see SwSegArgs.snap_*): the engine's
// per-step path when it writes a durable block.
int sw_seg_encode_snap(const void* rows, const void* aux, const uint8_t* raw, const int64_t* cursor, uint8_t* out,
                       int64_t out_cap, uint64_t* state, int64_t max_pages, const uint32_t* scalars,
                       const uint32_t* rej_cnt, const uint32_t* n_carry, uint32_t* host, hipStream_t s) {
  SwSegArgs a;
  a.rows = (const SwOutRec*)rows;
  a.aux = (const SwSegAux*)aux;
  a.raw = raw;
  a.cursor = cursor;
  a.out = out;
  a.out_cap = out_cap;
  a.state = state;
  a.max_pages = max_pages;
  a.stamps = nullptr;
  a.snap_scalars = scalars;
  a.snap_rej = rej_cnt;
  a.snap_carry = n_carry;
  a.snap_host = host;
  return seg_encode_launch(a, s);
}

// Same, recording 16 phase stamps per page (s_memrealtime, 100 MHz) into stamps[max_pages * 16].
int sw_seg_encode_stamped(const void* rows, const void* aux, const uint8_t* raw, const int64_t* cursor, uint8_t* out,
                          int64_t out_cap, uint64_t* state, int64_t max_pages, uint64_t* stamps, hipStream_t s) {
  SwSegArgs a;
  a.rows = (const SwOutRec*)rows;
  a.aux = (const SwSegAux*)aux;
  a.raw = raw;
  a.cursor = cursor;
  a.out = out;
  a.out_cap = out_cap;
  a.state = state;
  a.max_pages = max_pages;
  a.stamps = stamps;
  a.snap_scalars = nullptr;
  a.snap_rej = nullptr;
  a.snap_carry = nullptr;
  a.snap_host = nullptr;
  return seg_encode_launch(a, s);
}

// Encoder aux of a step's rows from its records, for callers outside the engine (the engine's
// persist kernel writes the same records as it persists): row j < *n_ok <-> work[ok_idx[j]] with
// spans (null: no strings), row j >= *n_ok <-> gen[j - n_ok]; rows = cursor[0] - cursor[1].
__global__ void k_seg_aux(const SwEventRec* __restrict__ work, const uint32_t* __restrict__ ok_idx,
                          const uint32_t* __restrict__ n_ok, const SwEventRec* __restrict__ gen,
                          const SwStrRef* __restrict__ spans, int64_t raw_bytes, const int64_t* __restrict__ cursor,
                          SwSegAux* __restrict__ aux) {
  const int64_t n = cursor[0] - cursor[1];
  const uint32_t nok = *n_ok;
  SwStrRef none;
  none.alt_off = 0; none.meta_off = 0; none.alt_len = 0; none.meta_len = 0; none.k = 0; none.has = 0; none.pad = 0;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
    if (j < (int64_t)nok) {
      const uint32_t i = ok_idx[j];
      aux[j] = seg_make_aux(work[i], spans ? spans[i] : none, raw_bytes);
    } else {
      aux[j] = seg_make_aux(gen[j - nok], none, 0);
    }
  }
}

int sw_seg_aux(const void* work, const uint32_t* ok_idx, const uint32_t* n_ok, const void* gen, const void* spans,
               int64_t raw_bytes, const int64_t* cursor, void* aux, int64_t max_rows, hipStream_t s) {
  const int64_t blocks = (max_rows + 255) / 256;
  k_seg_aux<<<(unsigned)(blocks > 0 ? (blocks < 4096 ? blocks : 4096) : 1), 256, 0, s>>>(
      (const SwEventRec*)work, ok_idx, n_ok, (const SwEventRec*)gen, (const SwStrRef*)spans, raw_bytes, cursor,
      (SwSegAux*)aux);
  return (int)hipGetLastError();
}

}  // extern "C"
