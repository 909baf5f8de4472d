// Block index trailers on the host (format: csrc/include/swindex.h): the C++ builder -- host engines'
// blocks, API-added blocks, and the reference the MI355X builder (csrc/hip/swindex.hip) is tested
// against bit for bit -- and the read side the durable event store queries through (alternate-id
// buckets, page zone maps, context-key heads over many blocks per call).
#include <stdint.h>
#include <string.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "swindex.h"
#include "swseg.h"

extern "C" {
int64_t swseg_decode(const uint8_t* b, int64_t p0, int64_t p1, uint8_t* etype, uint8_t* level, int64_t* date,
                     int32_t* asg, uint16_t* name, double* v0, double* v1, double* v2, uint8_t* flags,
                     uint8_t* str_heap, int64_t str_cap, int64_t* str_off);
int64_t swseg_string_bytes(const uint8_t* b, int64_t p0, int64_t p1);
void swseg_rechecksum(uint8_t* block);
}

namespace {

struct Trailer {
  std::vector<uint64_t> words;
  uint8_t* bytes() { return reinterpret_cast<uint8_t*>(words.data()); }
};

// head order (date desc, row desc) of a key's rows, the SIX_HEADS first kept
struct HeadCand {
  int64_t date;
  uint32_t row;
};

}  // namespace

extern "C" {

// Checksum of a trailer (its u64 words, the checksum word excluded).
uint64_t swseg_ix_checksum(const uint8_t* t, uint64_t bytes) {
  uint64_t cs = 0;
  for (uint64_t i = 0; i < bytes / 8; ++i) {
    if (i == SIX_CHECKSUM_WORD) continue;
    uint64_t w;
    memcpy(&w, t + 8 * i, 8);
    cs ^= seg_mix_word(w, i);
  }
  return cs;
}

// 0 = a well-formed trailer of a block of n_rows / n_pages within len bytes; > 0 otherwise.
int32_t swseg_ix_verify(const uint8_t* t, int64_t len, int64_t n_rows, int64_t n_pages) {
  if (len < (int64_t)SIX_HDR_BYTES) return 1;
  SwIxHdr h;
  memcpy(&h, t, sizeof(h));
  if (h.magic != SIX_MAGIC || h.version != SIX_VERSION || h.n_dims != SIX_DIMS) return 1;
  if ((int64_t)h.n_rows != n_rows || (int64_t)h.n_pages != n_pages) return 2;
  if ((int64_t)h.bytes > len || (h.bytes & 7) || h.alt_bits > SIX_ALT_SORT_BITS || h.n_alt > h.n_rows ||
      h.alt_pbits < 1 || h.alt_pbits > 20)
    return 3;
  SwIxHdr c = h;
  if (six_layout(&c) != h.bytes || c.off_pages != h.off_pages || c.off_alt_dir != h.off_alt_dir ||
      c.off_alt != h.off_alt)
    return 3;
  for (int d = 0; d < SIX_DIMS; ++d)
    if (c.off_keys[d] != h.off_keys[d] || c.off_heads[d] != h.off_heads[d] || c.off_hdates[d] != h.off_hdates[d])
      return 3;
  if (swseg_ix_checksum(t, h.bytes) != h.checksum) return 4;
  return 0;
}

// Build the index trailer of an encoded block (unsealed or sealed) and append it: the trailer goes at
// page_off[n_pages], the header gets SEG_FLAG_INDEX and its `bytes` covers the trailer (a sealed
// header is re-checksummed).  ctx = int32[n_ctx][4] (device, customer, area, asset) by assignment
// index -- the engine's assignment context table; rows whose assignment is outside it have no
// context; a null ctx leaves the context dimensions unindexed.  Returns the new block bytes, -(bytes needed) when cap is too small, or -1 on a malformed
// block.  A block that already has a trailer is rebuilt.
int64_t swseg_index_append(uint8_t* block, int64_t cap, const int32_t* ctx, int64_t n_ctx) {
  SwSegBlockHdr bh;
  memcpy(&bh, block, sizeof(bh));
  const int64_t n = bh.n_rows, np = bh.n_pages;
  const uint32_t* pt = reinterpret_cast<const uint32_t*>(block + 64);
  const uint64_t tstart = np ? pt[np] : 64 + ((4u * (uint32_t)(np + 1) + 7u) & ~7u);
  if (tstart & 7) return -1;
  std::vector<uint8_t> et(n), fl(n);
  std::vector<int64_t> date(n);
  std::vector<int32_t> asg(n);
  const int64_t scap = swseg_string_bytes(block, 0, np) + 64;
  std::vector<uint8_t> heap((size_t)scap);
  std::vector<int64_t> so(3 * n + 1);
  if (n && swseg_decode(block, 0, np, et.data(), nullptr, date.data(), asg.data(), nullptr, nullptr, nullptr, nullptr,
                        fl.data(), heap.data(), scap, so.data()) != n)
    return -1;
  SwIxHdr h;
  memset(&h, 0, sizeof(h));
  h.magic = SIX_MAGIC;
  h.version = SIX_VERSION;
  h.n_dims = SIX_DIMS;
  h.n_rows = (uint32_t)n;
  h.n_pages = (uint32_t)np;
  bool clustered = true;
  for (int64_t r = 1; r < n && clustered; ++r) {
    const bool g0 = fl[r - 1] & SEGF_GEN, g1 = fl[r] & SEGF_GEN;
    if ((g0 && !g1) || (!g0 && !g1 && asg[r] < asg[r - 1])) clustered = false;
  }
  h.flags = clustered ? SIX_F_CLUSTERED : 0u;
  // ---- alternate ids: (sort key, row) order
  std::vector<uint64_t> ah;
  std::vector<uint32_t> ar;
  for (int64_t r = 0; r < n; ++r) {
    if (!(fl[r] & SEGF_HAS_ALT)) continue;
    const int64_t a0 = so[3 * r], a1 = so[3 * r + 1];
    ah.push_back(sw_hash64(heap.data() + a0, (uint32_t)(a1 - a0)));
    ar.push_back((uint32_t)r);
  }
  std::vector<uint32_t> ord(ah.size());
  for (size_t i = 0; i < ord.size(); ++i) ord[i] = (uint32_t)i;
  std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return six_sort_key(ah[x]) < six_sort_key(ah[y]); });
  h.n_alt = (uint32_t)ah.size();
  h.alt_bits = six_alt_bits(h.n_alt);
  h.alt_pbits = six_page_bits((uint32_t)np);
  // ---- context dimensions
  std::vector<std::vector<SwIxKey>> keys(SIX_DIMS);
  std::vector<std::vector<uint32_t>> heads(SIX_DIMS);
  std::vector<std::vector<int64_t>> hdates(SIX_DIMS);
  for (int d = 0; d < SIX_DIMS; ++d) {
    std::vector<uint32_t> kr;        // key of every row (or ~0)
    kr.assign(n, ~0u);
    // indexed when the engine's context ids of this dimension (the whole table) stay below
    // SIX_CTX_MAX; no context table: the dimensions are not indexed
    bool indexed = ctx != nullptr;
    for (int64_t a = 0; indexed && a < n_ctx; ++a)
      if (ctx[4 * a + 1 + d] >= SIX_CTX_MAX) indexed = false;
    for (int64_t r = 0; indexed && r < n; ++r) {
      const int32_t a = asg[r];
      if (a < 0 || a >= n_ctx) continue;
      const int32_t c = ctx[4 * (int64_t)a + 1 + d];
      if (c < 0) continue;
      kr[r] = ((uint32_t)c << 3) | (uint32_t)(et[r] & 7u);
    }
    if (!indexed) {
      h.n_keys[d] = SIX_NOT_INDEXED;
      h.n_heads[d] = 0;
      continue;
    }
    std::vector<uint32_t> rows;
    for (int64_t r = 0; r < n; ++r)
      if (kr[r] != ~0u) rows.push_back((uint32_t)r);
    std::stable_sort(rows.begin(), rows.end(), [&](uint32_t x, uint32_t y) { return kr[x] < kr[y]; });
    size_t i = 0;
    while (i < rows.size()) {
      size_t j = i;
      const uint32_t k = kr[rows[i]];
      while (j < rows.size() && kr[rows[j]] == k) ++j;
      SwIxKey e;
      memset(&e, 0, sizeof(e));
      e.key = k;
      e.count = (uint32_t)(j - i);
      e.date_min = INT64_MAX;
      e.date_max = INT64_MIN;
      std::vector<HeadCand> hc;
      hc.reserve(j - i);
      for (size_t q = i; q < j; ++q) {
        const uint32_t r = rows[q];
        e.date_min = std::min(e.date_min, date[r]);
        e.date_max = std::max(e.date_max, date[r]);
        hc.push_back({date[r], r});
      }
      const size_t nh = std::min<size_t>(SIX_HEADS, hc.size());
      std::partial_sort(hc.begin(), hc.begin() + nh, hc.end(), [](const HeadCand& x, const HeadCand& y) {
        return six_newer(x.date, x.row, y.date, y.row);
      });
      e.head_off = (uint32_t)heads[d].size();
      e.n_heads = (uint32_t)nh;
      for (size_t q = 0; q < nh; ++q) {
        heads[d].push_back(hc[q].row);
        hdates[d].push_back(hc[q].date);
      }
      keys[d].push_back(e);
      i = j;
    }
    h.n_keys[d] = (uint32_t)keys[d].size();
    h.n_heads[d] = (uint32_t)heads[d].size();
  }
  const uint32_t tb = six_layout(&h);
  if ((int64_t)(tstart + tb) > cap) return -(int64_t)(tstart + tb);
  Trailer T;
  T.words.assign(tb / 8, 0ull);
  uint8_t* t = T.bytes();
  // pages: zone maps from the page headers
  for (int64_t p = 0; p < np; ++p) {
    SwSegPageHdr ph;
    memcpy(&ph, block + pt[p], sizeof(ph));
    SwIxPage z;
    z.asg_min = (int32_t)seg_unord(ph.cols[SEG_ASG].base);
    z.asg_max = ph.asg_max;
    z.date_min = seg_unord(ph.cols[SEG_DATE].base);
    z.date_max = ph.date_max;
    z.off = pt[p];
    z.bytes = pt[p + 1] - pt[p];
    memcpy(t + h.off_pages + p * sizeof(SwIxPage), &z, sizeof(z));
  }
  // alternate-id directory (prefix offsets per bucket) and packed entries
  {
    const uint32_t nb = 1u << h.alt_bits;
    std::vector<uint32_t> dir(nb + 1, 0);
    for (uint32_t i = 0; i < h.n_alt; ++i) ++dir[six_bucket(ah[ord[i]], h.alt_bits) + 1];
    for (uint32_t b = 0; b < nb; ++b) dir[b + 1] += dir[b];
    memcpy(t + h.off_alt_dir, dir.data(), 4 * (nb + 1));
    uint64_t* w = reinterpret_cast<uint64_t*>(t + h.off_alt);
    for (uint32_t i = 0; i < h.n_alt; ++i) {
      const uint32_t r = ar[ord[i]];
      const uint64_t v = six_entry(ah[ord[i]], h.alt_bits, h.alt_pbits, r / SEG_PAGE_ROWS);
      const uint64_t bp = (uint64_t)i * SIX_ALT_EBITS;
      const uint32_t wi = (uint32_t)(bp >> 6), sh = (uint32_t)(bp & 63);
      w[wi] |= v << sh;
      if (sh + SIX_ALT_EBITS > 64) w[wi + 1] |= v >> (64 - sh);
    }
  }
  for (int d = 0; d < SIX_DIMS; ++d) {
    if (h.n_keys[d] == SIX_NOT_INDEXED) continue;
    if (!keys[d].empty()) memcpy(t + h.off_keys[d], keys[d].data(), keys[d].size() * sizeof(SwIxKey));
    if (!heads[d].empty()) {
      memcpy(t + h.off_heads[d], heads[d].data(), 4 * heads[d].size());
      memcpy(t + h.off_hdates[d], hdates[d].data(), 8 * hdates[d].size());
    }
  }
  memcpy(t, &h, sizeof(h));
  h.checksum = swseg_ix_checksum(t, tb);
  memcpy(t, &h, sizeof(h));
  memcpy(block + tstart, t, tb);
  bh.flags |= SEG_FLAG_INDEX;
  bh.bytes = tstart + tb;
  memcpy(block, &bh, sizeof(bh));
  if (bh.magic == SEG_MAGIC) swseg_rechecksum(block);
  return (int64_t)(tstart + tb);
}

int64_t swseg_ix_max_bytes(int64_t n_rows) { return (int64_t)six_max_bytes((uint64_t)n_rows); }

// Offset of a block's trailer (0: none) from its header and page table.
int64_t swseg_ix_offset(const uint8_t* block) {
  SwSegBlockHdr bh;
  memcpy(&bh, block, sizeof(bh));
  if (!(bh.flags & SEG_FLAG_INDEX)) return 0;
  const uint32_t* pt = reinterpret_cast<const uint32_t*>(block + 64);
  return (int64_t)pt[bh.n_pages];
}

// ----------------------------------------------------------------------------- reads
// Alternate-id candidates over many blocks' trailers (t[i] null: skipped): for each block, from the
// last to the first, the pages holding an entry whose fingerprint matches `hash`.  Writes
// (block, page) pairs, newest block first, at most cap; returns the number found (may exceed cap).
int64_t swseg_ix_alt_pages(const uint8_t* const* t, int64_t n, uint64_t hash, int64_t* out_blk, int64_t* out_page,
                           int64_t cap) {
  int64_t k = 0;
  for (int64_t i = n - 1; i >= 0; --i) {
    const uint8_t* x = t[i];
    if (!x) continue;
    SwIxHdr h;
    memcpy(&h, x, sizeof(h));
    if (!h.n_alt) continue;
    const uint32_t b = six_bucket(hash, h.alt_bits);
    const uint32_t* dir = reinterpret_cast<const uint32_t*>(x + h.off_alt_dir);
    const uint32_t lo = dir[b], hi = dir[b + 1];
    const uint64_t want = six_entry(hash, h.alt_bits, h.alt_pbits, 0) >> h.alt_pbits;
    const uint8_t* words = x + h.off_alt;
    const uint64_t pmask = (1ull << h.alt_pbits) - 1ull;
    int64_t last_page = -1;
    for (uint32_t e = lo; e < hi && e < h.n_alt; ++e) {
      const uint64_t bp = (uint64_t)e * SIX_ALT_EBITS;
      uint64_t w0;
      memcpy(&w0, words + 8 * (bp >> 6), 8);
      const uint32_t sh = (uint32_t)(bp & 63);
      uint64_t v = w0 >> sh;
      if (sh + SIX_ALT_EBITS > 64) {
        uint64_t w1;
        memcpy(&w1, words + 8 * ((bp >> 6) + 1), 8);
        v |= w1 << (64 - sh);
      }
      v &= (1ull << SIX_ALT_EBITS) - 1ull;
      if ((v >> h.alt_pbits) != want) continue;
      const int64_t page = (int64_t)(v & pmask);
      if (page == last_page) continue;
      last_page = page;
      if (k < cap) { out_blk[k] = i; out_page[k] = page; }
      ++k;
    }
  }
  return k;
}

// Batch form for the store-backed dedup: for each of n_want hashes, whether any block may hold it
// (a fingerprint hit): the newest such block and page, -1 / -1 when none.
void swseg_ix_alt_find(const uint8_t* const* t, int64_t n, const uint64_t* want, int64_t n_want, int64_t* out_blk,
                       int64_t* out_page) {
  for (int64_t j = 0; j < n_want; ++j) {
    int64_t b = -1, p = -1;
    swseg_ix_alt_pages(t, n, want[j], &b, &p, 1);
    out_blk[j] = b;
    out_page[j] = p;
  }
}

// Pages of each block whose assignment zone map holds asg and whose date zone map meets [d_lo, d_hi]:
// (block, page) pairs in block order, at most cap; returns the number found.
int64_t swseg_ix_asg_pages(const uint8_t* const* t, int64_t n, int32_t asg, int64_t d_lo, int64_t d_hi,
                           int64_t* out_blk, int64_t* out_page, int64_t cap) {
  int64_t k = 0;
  for (int64_t i = 0; i < n; ++i) {
    const uint8_t* x = t[i];
    if (!x) continue;
    SwIxHdr h;
    memcpy(&h, x, sizeof(h));
    const SwIxPage* pg = reinterpret_cast<const SwIxPage*>(x + h.off_pages);
    for (uint32_t p = 0; p < h.n_pages; ++p) {
      if (asg < pg[p].asg_min || asg > pg[p].asg_max) continue;
      if (pg[p].date_max < d_lo || pg[p].date_min > d_hi) continue;
      if (k < cap) { out_blk[k] = i; out_page[k] = p; }
      ++k;
    }
  }
  return k;
}

// The pages of MANY assignments (sorted ascending, distinct) over the blocks of `t` whose mask byte is
// set (null mask: every block): each page once, (block, page) in block order.  Blocks are clustered
// by assignment, so an assignment's rows sit in one or two pages of a block; each page is tested with
// one binary search over the sorted assignments: O(pages * log assignments) per block, where the per
// assignment lookup above is O(pages) per assignment.  What routes a high-cardinality context
// dimension (one the trailers do not index: an asset per device, 10K customers) through its
// assignments in one call.  Returns the pages found (> cap: call again with that cap).
int64_t swseg_ix_asgs_pages(const uint8_t* const* t, int64_t n, const int32_t* asgs, int64_t n_asg,
                            const uint8_t* mask, int64_t d_lo, int64_t d_hi, int64_t* out_blk, int64_t* out_page,
                            int64_t cap, int64_t* out_lo, int64_t* out_hi, uint8_t* out_sorted) {
  int64_t k = 0;
  if (n_asg <= 0) return 0;
  for (int64_t i = 0; i < n; ++i) {
    const uint8_t* x = t[i];
    if (!x || (mask && !mask[i])) continue;
    SwIxHdr h;
    memcpy(&h, x, sizeof(h));
    const SwIxPage* pg = reinterpret_cast<const SwIxPage*>(x + h.off_pages);
    int64_t at = 0;                     // lower bound of the previous page's asg_min
    int32_t prev_min = INT32_MIN;
    for (uint32_t p = 0; p < h.n_pages; ++p) {
      const SwIxPage& q = pg[p];
      if (q.date_max < d_lo || q.date_min > d_hi) continue;
      // the first wanted assignment not below the page's range: walked forward while page ranges
      // ascend (the block's assignment-sorted pages), a binary search where they do not (its
      // generated rows; API-added blocks are not clustered)
      int64_t lo;
      if (q.asg_min >= prev_min) {
        lo = at;
        while (lo < n_asg && asgs[lo] < q.asg_min) ++lo;
      } else {
        lo = 0;
        int64_t hi = n_asg;
        while (lo < hi) {
          const int64_t mid = (lo + hi) >> 1;
          if (asgs[mid] < q.asg_min) lo = mid + 1; else hi = mid;
        }
      }
      at = lo;
      prev_min = q.asg_min;
      if (lo < n_asg && asgs[lo] <= q.asg_max) {     // one falls in [asg_min, asg_max]
        if (k < cap) {
          out_blk[k] = i;
          out_page[k] = p;
          if (out_lo) {                                  // the wanted assignments the page may hold
            int64_t e = lo + 1;
            while (e < n_asg && asgs[e] <= q.asg_max) ++e;
            out_lo[k] = lo;
            out_hi[k] = e;
          }
          if (out_sorted) out_sorted[k] = (h.flags & SIX_F_CLUSTERED) ? 1 : 0;
        }
        ++k;
      }
    }
  }
  return k;
}

void swseg_ix_ctx_find(const uint8_t* const* t, int64_t n, int32_t d, uint32_t key, int64_t* out);

// swseg_ix_ctx_find with the heads gathered: out[7 i ..] as there but o[4] = index of block i's
// first head in the flat outputs and o[6] = 0; the heads of every found block, block by block
// (newest first within a block), into head_blk / head_row / head_date (at most cap).  Returns the
// heads written in total (> cap: call again with that cap).
int64_t swseg_ix_ctx_heads(const uint8_t* const* t, int64_t n, int32_t d, uint32_t key, int64_t* out,
                           int64_t* head_blk, int64_t* head_row, int64_t* head_date, int64_t cap) {
  swseg_ix_ctx_find(t, n, d, key, out);
  int64_t k = 0;
  for (int64_t i = 0; i < n; ++i) {
    int64_t* o = out + 7 * i;
    if (o[0] != 1) { o[4] = k; o[6] = 0; continue; }
    const uint32_t* hr = reinterpret_cast<const uint32_t*>((uintptr_t)o[4]);
    const int64_t* hd = reinterpret_cast<const int64_t*>((uintptr_t)o[6]);
    const int64_t nh = o[5];
    for (int64_t j = 0; j < nh; ++j, ++k) {
      if (k < cap) {
        uint32_t r;
        int64_t dt;
        memcpy(&r, hr + j, 4);
        memcpy(&dt, hd + j, 8);
        head_blk[k] = i;
        head_row[k] = r;
        head_date[k] = dt;
      }
    }
    o[4] = k - nh;
    o[6] = 0;
  }
  return k;
}

// Geometry of pages pages[j] of blocks blk[j] from their trailers' page tables: offset in the block
// and bytes (out_bytes[j] = 0 where block blk[j] has no trailer, or the page is out of range).
// Returns how many could not be resolved.
int64_t swseg_ix_page_geom(const uint8_t* const* t, int64_t n_t, const int64_t* blk, const int64_t* pages, int64_t n,
                           uint32_t* out_off, uint32_t* out_bytes) {
  int64_t miss = 0;
  for (int64_t j = 0; j < n; ++j) {
    out_off[j] = 0;
    out_bytes[j] = 0;
    const int64_t b = blk[j];
    const uint8_t* x = b >= 0 && b < n_t ? t[b] : nullptr;
    if (!x) { ++miss; continue; }
    SwIxHdr h;
    memcpy(&h, x, sizeof(h));
    if (pages[j] < 0 || pages[j] >= (int64_t)h.n_pages) { ++miss; continue; }
    SwIxPage pg;
    memcpy(&pg, x + h.off_pages + sizeof(SwIxPage) * (size_t)pages[j], sizeof(pg));
    out_off[j] = pg.off;
    out_bytes[j] = pg.bytes;
  }
  return miss;
}

// Addresses of pages pages[j] of blocks bis[j] in the store's scan images (baddr[block]: image
// address, 0 = none; an image is u32 n_pages, u32, then u32 page offsets into the image): 0 where the
// block has no image or the page is out of range.  One pass for a listing's many pages.
void swseg_image_addrs(const uint64_t* baddr, const int64_t* bis, const int64_t* pages, int64_t n, uint64_t* out) {
  for (int64_t j = 0; j < n; ++j) {
    const uint64_t img = baddr[bis[j]];
    out[j] = 0;
    if (!img) continue;
    const uint8_t* p = reinterpret_cast<const uint8_t*>((uintptr_t)img);
    uint32_t npg, off;
    memcpy(&npg, p, 4);
    if (pages[j] < 0 || pages[j] >= (int64_t)npg) continue;
    memcpy(&off, p + 4 * (2 + pages[j]), 4);
    out[j] = img + off;
  }
}

// Context-key lookup over many blocks: for block i (trailer t[i]) and dimension d, the entry of
// `key`: out[7 i ..] = (status, count, date_min, date_max, head rows address, n_heads, head dates
// address) with status 1 = found, 0 = absent from the block, -1 = the dimension is not indexed there
// (or no trailer).
void swseg_ix_ctx_find(const uint8_t* const* t, int64_t n, int32_t d, uint32_t key, int64_t* out) {
  for (int64_t i = 0; i < n; ++i) {
    int64_t* o = out + 7 * i;
    o[0] = -1; o[1] = 0; o[2] = 0; o[3] = 0; o[4] = 0; o[5] = 0; o[6] = 0;
    const uint8_t* x = t[i];
    if (!x || d < 0 || d >= SIX_DIMS) continue;
    SwIxHdr h;
    memcpy(&h, x, sizeof(h));
    if (h.n_keys[d] == SIX_NOT_INDEXED) continue;
    const SwIxKey* ks = reinterpret_cast<const SwIxKey*>(x + h.off_keys[d]);
    const SwIxKey* e = std::lower_bound(ks, ks + h.n_keys[d], key,
                                        [](const SwIxKey& a, uint32_t k) { return a.key < k; });
    o[0] = 0;
    if (e == ks + h.n_keys[d] || e->key != key) continue;
    o[0] = 1;
    o[1] = e->count;
    o[2] = e->date_min;
    o[3] = e->date_max;
    o[4] = (int64_t)(uintptr_t)(x + h.off_heads[d] + 4ull * e->head_off);
    o[5] = e->n_heads;
    o[6] = (int64_t)(uintptr_t)(x + h.off_hdates[d] + 8ull * e->head_off);
  }
}


// Full 64-bit alternate-id hashes of a block's rows (the store-backed dedup filter's seed): writes
// up to cap hashes (rows with an id, in row order); returns how many, -1 on a malformed block.
int64_t swseg_alt_hashes(const uint8_t* block, uint64_t* out, int64_t cap) {
  SwSegBlockHdr bh;
  memcpy(&bh, block, sizeof(bh));
  const int64_t n = bh.n_rows, np = bh.n_pages;
  std::vector<uint8_t> fl(n);
  const int64_t scap = swseg_string_bytes(block, 0, np) + 64;
  std::vector<uint8_t> heap((size_t)scap);
  std::vector<int64_t> so(3 * n + 1);
  if (n && swseg_decode(block, 0, np, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                        fl.data(), heap.data(), scap, so.data()) != n)
    return -1;
  int64_t k = 0;
  for (int64_t r = 0; r < n; ++r) {
    if (!(fl[r] & SEGF_HAS_ALT)) continue;
    if (k < cap) out[k] = sw_hash64(heap.data() + so[3 * r], (uint32_t)(so[3 * r + 1] - so[3 * r]));
    ++k;
  }
  return k;
}

}  // extern "C"

namespace {

inline uint64_t ix_unpack(const uint8_t* words, uint32_t i, int bits) {
  if (bits == 0) return 0;
  const uint64_t b = (uint64_t)i * (uint64_t)bits;
  uint64_t w0;
  memcpy(&w0, words + 8 * (b >> 6), 8);
  const uint32_t s = (uint32_t)(b & 63);
  uint64_t v = w0 >> s;
  if (s + bits > 64) {
    uint64_t w1;
    memcpy(&w1, words + 8 * ((b >> 6) + 1), 8);
    v |= w1 << (64 - s);
  }
  return bits == 64 ? v : (v & ((1ull << bits) - 1));
}

struct ScanHit {
  int64_t task;
  int32_t row;
  int64_t date;
};

// All n codes of a bit-packed column (bits < 57) in order, one 64-bit word read per 64 bits: the
// sequential form of ix_unpack for a whole page column.
inline void ix_unpack_all(const uint8_t* words, uint32_t n, int bits, uint32_t* out) {
  if (bits == 0) {
    for (uint32_t r = 0; r < n; ++r) out[r] = 0;
    return;
  }
  const uint64_t mask = (1ull << bits) - 1;
  uint64_t cur;
  memcpy(&cur, words, 8);
  const uint8_t* next = words + 8;
  int avail = 64;
  for (uint32_t r = 0; r < n; ++r) {
    if (avail >= bits) {
      out[r] = (uint32_t)(cur & mask);
      cur = avail == bits ? 0 : cur >> bits;
      avail -= bits;
    } else {
      uint64_t nw;
      memcpy(&nw, next, 8);
      next += 8;
      out[r] = (uint32_t)((cur | (nw << avail)) & mask);
      const int used = bits - avail;
      cur = nw >> used;
      avail = 64 - used;
    }
  }
}

}  // namespace

extern "C" {

// Rows of the listed pages that pass a filter, reading with pread only each page's header and its
// leading columns (event type, level, date, assignment: the first four in the page).  Task i = page
// pg_index[i] of the block at file offset blk_off[i] in fds[i] (page offset / size in the block from
// the trailer's zone maps).  Filter: event type et (-1: any), date in [d_lo, d_hi], and assignment ==
// asg (asg >= 0), else ctx_tab[assignment] == ctx_id (ctx_tab: n_ctx ids by assignment index).
// Matches go out in task order, then row order: (task, row in block, date), at most cap; returns the
// number of matches (may exceed cap), -(1 + task) when a page cannot be read.
int64_t swseg_scan_pages(const int32_t* fds, const int64_t* blk_off, const uint32_t* pg_off, const uint32_t* pg_bytes,
                         const int32_t* pg_index, int64_t n_tasks, int32_t et, int32_t asg, const int32_t* ctx_tab,
                         int64_t n_ctx, int32_t ctx_id, int64_t d_lo, int64_t d_hi, int32_t threads,
                         int64_t* out_task, int32_t* out_row, int64_t* out_date, int64_t cap, const uint64_t* mem,
                         const int32_t* asg_list, const int64_t* task_lo, const int64_t* task_hi,
                         const uint8_t* sorted) {
  if (n_tasks <= 0) return 0;
  int T = threads > 0 ? threads : 1;
  if (T > 64) T = 64;
  if ((int64_t)T > (n_tasks + 3) / 4) T = (int)((n_tasks + 3) / 4);
  if (T < 1) T = 1;
  std::vector<std::vector<ScanHit>> hits(T);
  std::atomic<int64_t> bad{-1};
  auto work = [&](int w) {
    std::vector<uint8_t> buf;
    const int64_t b0 = n_tasks * w / T, b1 = n_tasks * (w + 1) / T;
    for (int64_t i = b0; i < b1; ++i) {
      // a page held in memory is read in place; from the file, one read of the page's first bytes
      // usually holds the header and the leading columns (etype, level, date, assignment), and a
      // second read fetches the rest when it does not
      const uint8_t* pg;
      uint64_t first = 0;
      if (mem && mem[i]) {
        if (pg_bytes[i] < sizeof(SwSegPageHdr)) { bad = i; return; }
        pg = reinterpret_cast<const uint8_t*>((uintptr_t)mem[i]);
      } else {
        first = std::min<uint64_t>(pg_bytes[i], 12288);
        if (first < sizeof(SwSegPageHdr)) { bad = i; return; }
        buf.resize(first + 8);
        if (pread(fds[i], buf.data(), first, blk_off[i] + pg_off[i]) != (ssize_t)first) { bad = i; return; }
        pg = buf.data();
      }
      SwSegPageHdr ph;
      memcpy(&ph, pg, sizeof(ph));
      const SwSegCol& ca = ph.cols[SEG_ASG];
      const uint64_t need = (uint64_t)ca.data_off + seg_col_bytes(ca.count, ca.bits, 0);
      if (need > pg_bytes[i] || ph.n_rows > SEG_PAGE_ROWS || ph.cols[SEG_ETYPE].count != ph.n_rows ||
          ph.cols[SEG_DATE].count != ph.n_rows || ca.count != ph.n_rows) { bad = i; return; }
      if (!(mem && mem[i]) && need > first) {
        buf.resize(need + 8);
        if (pread(fds[i], buf.data() + first, need - first, blk_off[i] + pg_off[i] + first) != (ssize_t)(need - first)) {
          bad = i;
          return;
        }
        pg = buf.data();
      }
      const SwSegCol& ce = ph.cols[SEG_ETYPE];
      const SwSegCol& cd = ph.cols[SEG_DATE];
      const int32_t row0 = pg_index[i] * SEG_PAGE_ROWS;
      // a page whose event types all differ from et (e.g. the block's generated alerts, persisted
      // after its assignment-sorted events, when listing measurements): its frame of reference says so
      if (et >= 0 && ce.bits < 32) {
        const int64_t t_lo = seg_unord(ce.base), t_hi = seg_unord(ce.base + ((1ull << ce.bits) - 1));
        if (et < t_lo || et > t_hi) continue;
      }
      if (asg_list) {
        // the wanted assignments this page may hold (sorted, asg_list[task_lo .. task_hi)): the
        // assignment column first -- one compare for the usual single candidate -- and the type
        // and date only for its rows (no per-row context table lookup)
        const int64_t l0 = task_lo[i], l1 = task_hi[i];
        const SwSegCol& cf = ph.cols[SEG_FLAGS];
        if (sorted && sorted[i] && ca.bits <= 32 && cf.bits < 32 &&
            seg_unord(cf.base + ((1ull << cf.bits) - 1)) < (int64_t)SEGF_GEN) {
          // a page of a clustered block without generated rows is sorted by assignment
          // (SIX_F_CLUSTERED): each wanted assignment's rows are one run, found by binary search
          auto code = [&](uint32_t r) { return ix_unpack(pg + ca.data_off, r, ca.bits); };
          for (int64_t q = l0; q < l1; ++q) {
            const uint64_t c = seg_ord(asg_list[q]) - ca.base;
            if (ca.bits ? (c >> ca.bits) != 0 : c != 0) continue;
            uint32_t lo = 0, hi = ph.n_rows;
            while (lo < hi) {
              const uint32_t mid = (lo + hi) >> 1;
              if (code(mid) < c) lo = mid + 1; else hi = mid;
            }
            for (uint32_t r = lo; r < ph.n_rows && code(r) == c; ++r) {
              if (et >= 0 && (int32_t)seg_unord(ce.base + ix_unpack(pg + ce.data_off, r, ce.bits)) != et) continue;
              const int64_t d = seg_unord(cd.base + ix_unpack(pg + cd.data_off, r, cd.bits));
              if (d < d_lo || d > d_hi) continue;
              hits[w].push_back({i, row0 + (int32_t)r, d});
            }
          }
          continue;
        }
        if (ca.bits <= 32) {
          // the whole assignment column unpacked sequentially, compared as codes (value - base)
          uint32_t codes[SEG_PAGE_ROWS];
          ix_unpack_all(pg + ca.data_off, ph.n_rows, ca.bits, codes);
          auto keep = [&](uint32_t r) {
            if (et >= 0 && (int32_t)seg_unord(ce.base + ix_unpack(pg + ce.data_off, r, ce.bits)) != et) return;
            const int64_t d = seg_unord(cd.base + ix_unpack(pg + cd.data_off, r, cd.bits));
            if (d < d_lo || d > d_hi) return;
            hits[w].push_back({i, row0 + (int32_t)r, d});
          };
          if (l1 - l0 == 1) {
            const uint64_t c = seg_ord(asg_list[l0]) - ca.base;
            if (ca.bits && c >> ca.bits) continue;           // not in this page's range
            if (!ca.bits && c) continue;
            const uint32_t cc = (uint32_t)c;
            for (uint32_t r = 0; r < ph.n_rows; ++r)
              if (codes[r] == cc) keep(r);
          } else if (l1 - l0 <= 16) {
            // a few candidates (a page straddling them): one compare pass per candidate, the
            // matching rows then kept in row order
            uint32_t mrow[SEG_PAGE_ROWS];
            uint32_t nm = 0;
            for (int64_t q = l0; q < l1; ++q) {
              const uint64_t c = seg_ord(asg_list[q]) - ca.base;
              if (ca.bits ? (c >> ca.bits) != 0 : c != 0) continue;
              const uint32_t cc = (uint32_t)c;
              for (uint32_t r = 0; r < ph.n_rows; ++r)
                if (codes[r] == cc && nm < SEG_PAGE_ROWS) mrow[nm++] = r;
            }
            std::sort(mrow, mrow + nm);
            for (uint32_t j = 0; j < nm; ++j) keep(mrow[j]);
          } else {
            for (uint32_t r = 0; r < ph.n_rows; ++r) {
              const uint64_t v = ca.base + codes[r];          // ordered value; asg_list is sorted
              int64_t lo = l0, hi = l1;
              while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (seg_ord(asg_list[mid]) < v) lo = mid + 1; else hi = mid;
              }
              if (lo < l1 && seg_ord(asg_list[lo]) == v) keep(r);
            }
          }
          continue;
        }
        for (uint32_t r = 0; r < ph.n_rows; ++r) {
          const int32_t a = (int32_t)seg_unord(ca.base + ix_unpack(pg + ca.data_off, r, ca.bits));
          if (l1 - l0 == 1) {
            if (a != asg_list[l0]) continue;
          } else {
            int64_t lo = l0, hi = l1;
            while (lo < hi) {
              const int64_t mid = (lo + hi) >> 1;
              if (asg_list[mid] < a) lo = mid + 1; else hi = mid;
            }
            if (lo >= l1 || asg_list[lo] != a) continue;
          }
          if (et >= 0 && (int32_t)seg_unord(ce.base + ix_unpack(pg + ce.data_off, r, ce.bits)) != et) continue;
          const int64_t d = seg_unord(cd.base + ix_unpack(pg + cd.data_off, r, cd.bits));
          if (d < d_lo || d > d_hi) continue;
          hits[w].push_back({i, row0 + (int32_t)r, d});
        }
        continue;
      }
      for (uint32_t r = 0; r < ph.n_rows; ++r) {
        if (et >= 0 && (int32_t)seg_unord(ce.base + ix_unpack(pg + ce.data_off, r, ce.bits)) != et) continue;
        const int32_t a = (int32_t)seg_unord(ca.base + ix_unpack(pg + ca.data_off, r, ca.bits));
        if (asg >= 0) {
          if (a != asg) continue;
        } else if (a < 0 || a >= n_ctx || ctx_tab[a] != ctx_id) {
          continue;
        }
        const int64_t d = seg_unord(cd.base + ix_unpack(pg + cd.data_off, r, cd.bits));
        if (d < d_lo || d > d_hi) continue;
        hits[w].push_back({i, row0 + (int32_t)r, d});
      }
    }
  };
  if (T == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int w = 0; w < T; ++w) th.emplace_back(work, w);
    for (auto& x : th) x.join();
  }
  if (bad.load() >= 0) return -(1 + bad.load());
  int64_t k = 0;
  for (int w = 0; w < T; ++w)
    for (const ScanHit& h : hits[w]) {
      if (k < cap) { out_task[k] = h.task; out_row[k] = h.row; out_date[k] = h.date; }
      ++k;
    }
  return k;
}

}  // extern "C"
