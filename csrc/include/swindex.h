// Block index trailer: the read-side indexes of one durable event block, built on the MI355X in the
// same engine step that encodes the block (csrc/hip/swindex.hip) and written to disk with it, in the
// same group commit.  The C++ builder in csrc/native/swindex.cpp (swseg_index_append) produces the
// same bytes from a decoded block (tests/test_gpu_index.py checks GPU == CPU bit for bit).
//
// Reference: MongoDeviceEventManagement.java:129-141 keeps five indexes on every insert -- unique
// sparse alternateId and (assignment | customer | area | asset, eventType, eventDate desc).  Here:
//
//  * assignment: the engine persists each step's events stable-sorted by assignment index (the
//    persist order of k_persist / the CPU engines), so a block is clustered by assignment and its
//    page zone maps (SwIxPage: assignment and date min / max, offset and size of every 1024-row
//    page) locate an assignment's rows in one or two pages, read as a few KB of leading columns.
//    No per-row bytes.
//  * customer / area / asset: per present key (context id << 3 | event type) its row count, date
//    range and its SIX_HEADS newest rows with their dates (date desc, row desc): a page-1 listing
//    merges the heads of every block instead of decoding blocks; a block is scanned only once the
//    merge passes its last head.
//    A dimension whose engine-wide context ids reach SIX_CTX_MAX is not indexed: such a context (an
//    asset per device, 10K customers) has few assignments, and its listing maps the id to them and
//    them to pages through every block's page zone maps in one native pass (swseg_ix_asgs_pages),
//    then scans only those pages (persistence/segments.py _ctx_via_assignments).
//  * alternate ids: (bucket = top SIX_ALT_SORT_BITS bits of the id's 64-bit hash, row) order, a
//    directory of the top alt_bits bits, and per id a SIX_ALT_EBITS-bit entry (hash fingerprint <<
//    pbits | page).  A lookup reads one bucket (~16-32 entries) per block and decodes the page of a
//    fingerprint hit, where the id string itself is compared (a hash match alone never decides).
//
// Trailer placement: a block with SEG_FLAG_INDEX has its trailer at page_off[n_pages] (the end of
// the pages, 8-aligned) and the block header's `bytes` covers it.  Layout (every section 8-aligned):
//   SwIxHdr | SwIxPage[n_pages] | u32 alt_dir[2^alt_bits + 1] | packed alt entries (u64 words)
//   | per dimension: SwIxKey[n_keys] | i64 head dates[n_heads] | u32 head rows[n_heads]
// Checksum: xor of seg_mix_word(word, index) over the trailer's u64 words, the checksum word
// (index 3) excluded.
#pragma once
#include <stdint.h>
#include "swtypes.h"
#include "swseg.h"

#define SEG_FLAG_INDEX 2
#define SIX_MAGIC 0x58495753u      // "SWIX"
#define SIX_VERSION 1
#define SIX_DIMS 3                 // customer, area, asset (SwAsgCtx fields 1..3)
#define SIX_HEADS 16               // newest rows kept per context key
#define SIX_CTX_MAX 8192           // a dimension is indexed when its context ids are < this
#define SIX_KEYS (SIX_CTX_MAX << 3)
#define SIX_ALT_SORT_BITS 15       // entries are ordered by (hash >> 49, row)
#define SIX_ALT_EBITS 26           // bits per alternate-id entry
#define SIX_NOT_INDEXED 0xffffffffu
#define SIX_CHECKSUM_WORD 3

typedef struct __attribute__((aligned(8))) SwIxHdr {
  uint32_t magic;
  uint16_t version;
  uint16_t n_dims;
  uint32_t n_rows;
  uint32_t n_pages;
  uint64_t bytes;                  // trailer bytes (multiple of 8)
  uint64_t checksum;
  uint32_t alt_bits;               // directory bits B
  uint32_t alt_pbits;              // page bits of an entry
  uint32_t n_alt;                  // entries (rows with an alternate id)
  uint32_t off_pages;              // section offsets, from the trailer start
  uint32_t off_alt_dir;
  uint32_t off_alt;
  uint32_t off_keys[SIX_DIMS];
  uint32_t n_keys[SIX_DIMS];       // SIX_NOT_INDEXED: the dimension is not indexed in this block
  uint32_t off_heads[SIX_DIMS];     // head rows (u32)
  uint32_t n_heads[SIX_DIMS];
  uint32_t off_hdates[SIX_DIMS];    // head dates (i64), same order
  uint32_t flags;                  // SIX_F_*
  uint32_t pad[2];
} SwIxHdr;

// SwIxHdr.flags: every engine-persisted row precedes every generated row (SEGF_GEN) and the persisted
// rows' assignments never decrease -- a page without generated rows is sorted by assignment, so a
// reader binary-searches its assignment column instead of reading every row
#define SIX_F_CLUSTERED 1u

typedef struct __attribute__((aligned(8))) SwIxPage {
  int32_t asg_min, asg_max;
  int64_t date_min, date_max;
  uint32_t off;                    // the page's offset in the block
  uint32_t bytes;                  // its size
} SwIxPage;

typedef struct __attribute__((aligned(8))) SwIxKey {
  uint32_t key;                    // context id << 3 | event type
  uint32_t count;                  // rows
  int64_t date_min, date_max;
  uint32_t head_off;               // first head, in entries from off_heads[d] / off_hdates[d]
  uint32_t n_heads;                // min(count, SIX_HEADS)
} SwIxKey;

#define SIX_HDR_BYTES ((uint32_t)sizeof(SwIxHdr))

SW_HD uint32_t six_rd8(uint32_t x) { return (x + 7u) & ~7u; }

// directory bits for n entries: ~16-32 entries per bucket, at most SIX_ALT_SORT_BITS
SW_HD uint32_t six_alt_bits(uint32_t n_alt) {
  if (!n_alt) return 0;
  const int w = 32 - __builtin_clz(n_alt);
  const int b = w - 5;
  return (uint32_t)(b < 0 ? 0 : (b > SIX_ALT_SORT_BITS ? SIX_ALT_SORT_BITS : b));
}
SW_HD uint32_t six_page_bits(uint32_t n_pages) {
  if (n_pages <= 2) return 1;
  return (uint32_t)(32 - __builtin_clz(n_pages - 1));
}
SW_HD uint32_t six_sort_key(uint64_t h) { return (uint32_t)(h >> (64 - SIX_ALT_SORT_BITS)); }
SW_HD uint32_t six_bucket(uint64_t h, uint32_t bits) { return bits ? (uint32_t)(h >> (64 - bits)) : 0u; }
// the entry of an id: fingerprint = the (EBITS - pbits) hash bits after the bucket bits
SW_HD uint64_t six_entry(uint64_t h, uint32_t bits, uint32_t pbits, uint32_t page) {
  const uint32_t fb = SIX_ALT_EBITS - pbits;
  const uint64_t fp = (h >> (64 - bits - fb)) & ((1ull << fb) - 1ull);
  return (fp << pbits) | (uint64_t)page;
}
SW_HD uint32_t six_alt_words(uint32_t n_alt) { return (uint32_t)(((uint64_t)n_alt * SIX_ALT_EBITS + 63) >> 6); }

// Section sizes -> offsets and total bytes.  n_keys[d] == SIX_NOT_INDEXED counts as 0 keys.
SW_HD uint32_t six_layout(SwIxHdr* h) {
  uint32_t off = SIX_HDR_BYTES;
  h->off_pages = off;
  off += six_rd8(h->n_pages * (uint32_t)sizeof(SwIxPage));
  h->off_alt_dir = off;
  off += six_rd8(4u * ((1u << h->alt_bits) + 1u));
  h->off_alt = off;
  off += 8u * six_alt_words(h->n_alt);
  for (int d = 0; d < SIX_DIMS; ++d) {
    const uint32_t nk = h->n_keys[d] == SIX_NOT_INDEXED ? 0u : h->n_keys[d];
    h->off_keys[d] = off;
    off += nk * (uint32_t)sizeof(SwIxKey);
    h->off_hdates[d] = off;
    off += 8u * h->n_heads[d];
    h->off_heads[d] = off;
    off += six_rd8(4u * h->n_heads[d]);
  }
  h->bytes = off;
  return off;
}

// Upper bound of a trailer for a block of n rows.
SW_HD uint64_t six_max_bytes(uint64_t n) {
  const uint64_t np = (n + SEG_PAGE_ROWS - 1) / SEG_PAGE_ROWS;
  const uint64_t keys = n < (uint64_t)SIX_KEYS ? n : (uint64_t)SIX_KEYS;
  return SIX_HDR_BYTES + np * sizeof(SwIxPage) + 8 + 4ull * ((1u << SIX_ALT_SORT_BITS) + 1u) + 8 +
         8ull * (((uint64_t)n * SIX_ALT_EBITS + 63) >> 6) +
         SIX_DIMS * (keys * sizeof(SwIxKey) + 12ull * n + 8);
}

// Does (d1, r1) come before (d2, r2) in head order (date desc, row desc)?
SW_HD bool six_newer(int64_t d1, uint32_t r1, int64_t d2, uint32_t r2) {
  return d1 > d2 || (d1 == d2 && r1 > r2);
}
