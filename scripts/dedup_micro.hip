// Microbenchmark of the dedup claim (k_dedup_claim in csrc/hip/swgpu.hip) on synthetic ids: which of
// its memory operations the kernel time goes to.  Built on the CPU into
// sitewhere_amd/_lib/variants/libdedup_micro.so; driven by scripts/bench_dedup_micro.py.
//   mode 0  the engine's claim: status + id load, probe of the retired generation, CAS claim
//   mode 1  CAS claim only (no retired-generation probe)
//   mode 2  retired-generation probe only (no claim)
//   mode 3  probe and CAS issued together (the probe's result applied after the claim returns)
//   mode 4  mode 0 with two ids per thread in flight
//   mode 5  id + status loads only
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "swtypes.h"

typedef unsigned long long ull;
#define MBLK 256
#define MPROBE 4096

__device__ __forceinline__ bool m_find(const ull* __restrict__ tab, int64_t mask, ull h) {
  int64_t slot = (int64_t)(h & (ull)mask);
  for (int p = 0; p <= mask && p < MPROBE; ++p) {
    const ull k = tab[2 * slot];
    if (k == h) return true;
    if (k == 0) return false;
    slot = (slot + 1) & mask;
  }
  return false;
}

__device__ __forceinline__ uint8_t m_claim(ull* __restrict__ ct, int64_t mask, ull h, uint32_t seq) {
  int64_t slot = (int64_t)(h & (ull)mask);
  for (int p = 0; p <= mask && p < MPROBE; ++p) {
    const ull old = atomicCAS(&ct[2 * slot], 0ull, h);
    if (old == 0) {
      reinterpret_cast<uint32_t*>(&ct[2 * slot + 1])[0] = seq;
      return 0;
    }
    if (old == h) return 2;
    slot = (slot + 1) & mask;
  }
  return 3;
}

__global__ __launch_bounds__(MBLK) void k_claim_micro(const SwEventRec* __restrict__ recs, uint8_t* __restrict__ status,
                                                      int64_t n, ull* __restrict__ cur, const ull* __restrict__ prev,
                                                      int64_t mask, int mode, ull* __restrict__ sink) {
  ull acc = 0;
  const int64_t stride = (int64_t)gridDim.x * MBLK;
  if (mode == 4) {
    for (int64_t i = (int64_t)blockIdx.x * MBLK + threadIdx.x; i < n; i += 2 * stride) {
      const int64_t j = i + stride;
      const bool vj = j < n;
      const ull hi = status[i] == 0 ? recs[i].alt_hash : 0ull;
      const ull hj = vj && status[j] == 0 ? recs[j].alt_hash : 0ull;
      const bool di = hi && m_find(prev, mask, hi);
      const bool dj = hj && m_find(prev, mask, hj);
      if (hi && !di) status[i] = m_claim(cur, mask, hi, (uint32_t)i);
      else if (di) status[i] = 1;
      if (hj && !dj) status[j] = m_claim(cur, mask, hj, (uint32_t)j);
      else if (dj) status[j] = 1;
    }
    return;
  }
  for (int64_t i = (int64_t)blockIdx.x * MBLK + threadIdx.x; i < n; i += stride) {
    if (status[i] != 0) continue;
    const ull h = recs[i].alt_hash;
    if (!h) continue;
    if (mode == 5) { acc += h; continue; }
    if (mode == 2) { acc += m_find(prev, mask, h) ? 1 : 0; continue; }
    if (mode == 1) { status[i] = m_claim(cur, mask, h, (uint32_t)i); continue; }
    if (mode == 3) {
      const bool d = m_find(prev, mask, h);     // independent of the claim: both in flight
      const uint8_t st = m_claim(cur, mask, h, (uint32_t)i);
      status[i] = d ? (uint8_t)1 : st;
      continue;
    }
    if (m_find(prev, mask, h)) { status[i] = 1; continue; }
    status[i] = m_claim(cur, mask, h, (uint32_t)i);
  }
  if (acc == 0x12345) sink[0] = acc;             // keeps the loads
}

// persist-side scattered updates: one per id into `tab` (words, mask + 1 of them), word = mix(id)
//   mode 6  no-return atomicOr (the store-backed filter add)
//   mode 7  plain load + store of the same word (non-atomic read-modify-write)
//   mode 8  atomicMax on a 32-byte-slot table (the device-state date merge)
//   mode 9  checked plain store on the same (load, store if larger)
__global__ __launch_bounds__(MBLK) void k_update_micro(const SwEventRec* __restrict__ recs, int64_t n, ull* __restrict__ tab,
                                                       int64_t mask, int mode) {
  const int64_t stride = (int64_t)gridDim.x * MBLK;
  for (int64_t i = (int64_t)blockIdx.x * MBLK + threadIdx.x; i < n; i += stride) {
    const ull h = recs[i].alt_hash;
    const ull w = sw_mix64(h) & (ull)mask;
    const ull bit = 1ull << (h & 63);
    if (mode == 6) atomicOr(&tab[w], bit);
    else if (mode == 7) tab[w] = tab[w] | bit;
    else if (mode == 8) atomicMax(&tab[4 * (w >> 2)], h);
    else if (mode == 9) { ull* p = &tab[4 * (w >> 2)]; if (h > *p) *p = h; }
  }
}

extern "C" int dm_update(const void* recs, int64_t n, ull* tab, int64_t mask, int mode, int grid, hipStream_t s) {
  k_update_micro<<<grid, MBLK, 0, s>>>((const SwEventRec*)recs, n, tab, mask, mode);
  return (int)hipGetLastError();
}

extern "C" int dm_claim(const void* recs, uint8_t* status, int64_t n, ull* cur, const ull* prev, int64_t mask,
                        int mode, int grid, ull* sink, hipStream_t s) {
  k_claim_micro<<<grid, MBLK, 0, s>>>((const SwEventRec*)recs, status, n, cur, prev, mask, mode, sink);
  return (int)hipGetLastError();
}
