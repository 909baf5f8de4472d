// Durable columnar event segments (host side): block encoder / decoder / verifier and the
// segment store -- append-only segment files written by a group-commit writer thread.
//
// Format: csrc/include/swseg.h.  The MI355X engine encodes blocks on the GPU (swgpu.hip,
// k_seg_encode); swseg_encode here is the CPU encoder for host engines and the bit-exact reference
// the GPU encoder is tested against.
//
// Segment store (reference counterpart: the event store behind DeviceEventManagement --
// MongoDeviceEventManagement + DeviceEventBuffer.java:99-135, bulk writes every 250 ms / 200 docs):
//   * one directory per engine shard, files "<rank>-<first_seq:020>.sweg", rotated at rotate_bytes;
//   * every block starts at a 4 KiB boundary (O_DIRECT writes straight from the caller's pinned
//     buffer when it is aligned, a bounce copy otherwise);
//   * group commit: the writer drains everything queued, writes it, then one fdatasync; a block's
//     token is durable once that sync returned (the caller commits its input offsets only then);
//   * recovery on open: every block is verified (header + page checksums); the first bad or short
//     block ends its file, which is truncated there (torn tail after a crash);
//   * optional retention: oldest whole files are deleted beyond retention_bytes.
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <sys/mman.h>
#include <vector>

#include "swindex.h"
#include "swseg.h"

#define SEG_ALIGN 4096

namespace {

inline uint32_t rd8(uint32_t x) { return (x + 7u) & ~7u; }

// ----------------------------------------------------------------------------- encoder
// One row as the encoder sees it: the enriched outbound row, its record's elevation and strings.
struct Row {
  SwOutRec o;
  double v2;
  SegRowStr s;
};

struct ColPlan {
  uint64_t base = 0;
  uint32_t count = 0, n_exc = 0;
  int bits = 0, exp = -1;
};

struct PageEnc {
  ColPlan plan[SEG_NCOL];
  uint32_t heap_off = 0, heap_bytes = 0, bytes = 0;
  uint32_t pfx = 0, mode = SEG_ALT_RAW, width = 0;
  int64_t pfx_src = 0;        // raw offset of the prefix bytes (the page's first alternate id)
  int32_t asg_max = 0;
  int64_t date_max = 0;
};

// Exponent search start per double column (a hint only: the result is seg_dec_exp's exponent).
inline int exp_hint(int c) { return c == SEG_MXV ? 2 : c == SEG_ELEV ? 1 : 6; }

inline double dbl_value(int c, const Row& r) {
  return c == SEG_MXV || c == SEG_LAT ? r.o.v0 : c == SEG_LON ? r.o.v1 : r.v2;
}

// Order-preserving unsigned value of integer column c (ALTNUM is filled by the caller).
inline uint64_t int_value(int c, const Row& r, uint32_t pfx, uint64_t altnum) {
  switch (c) {
    case SEG_ETYPE: return seg_ord((int64_t)r.o.etype);
    case SEG_LEVEL: return seg_ord((int64_t)r.o.level);
    case SEG_DATE: return seg_ord(r.o.event_date);
    case SEG_ASG: return seg_ord((int64_t)r.o.assignment);
    case SEG_NAME: return seg_ord((int64_t)r.o.name_id);
    case SEG_FLAGS: return seg_ord((int64_t)r.s.flags);
    case SEG_ALTK: return seg_ord((int64_t)r.s.altk);
    case SEG_ALTLEN: return seg_ord((int64_t)(r.s.alt_len - pfx));
    case SEG_ALTNUM: return altnum;
    case SEG_MSGLEN: return seg_ord((int64_t)r.s.msg_len);
    case SEG_METALEN: return seg_ord((int64_t)r.s.meta_len);
    default: return 0;
  }
}

// hex value of an alternate id's remainder (hex-mode pages only)
inline uint64_t alt_hex(const uint8_t* raw, const Row& r, uint32_t pfx) {
  uint64_t v = 0;
  for (uint32_t i = pfx; i < r.s.alt_len; ++i) v = (v << 4) | seg_hex_value(raw[r.s.alt_off + i]);
  return v;
}

void plan_page(const Row* R, int m, const uint8_t* raw, PageEnc* pe, std::vector<uint64_t>& altnum) {
  // alternate ids: common prefix with the page's first one, then hex mode if every remainder is a
  // fixed-width lowercase hex number
  int first = -1;
  for (int k = 0; k < m; ++k)
    if (R[k].s.flags & SEGF_HAS_ALT) { first = k; break; }
  pe->pfx = 0;
  pe->mode = SEG_ALT_RAW;
  pe->width = 0;
  pe->pfx_src = 0;
  if (first >= 0) {
    const uint8_t* a0 = raw + R[first].s.alt_off;
    uint32_t p = std::min<uint32_t>(R[first].s.alt_len, SEG_ALT_PFX_MAX);
    uint32_t wmin = 0xffffffffu, wmax = 0;
    bool hex = true;
    for (int k = first; k < m; ++k) {
      if (!(R[k].s.flags & SEGF_HAS_ALT)) continue;
      const uint8_t* a = raw + R[k].s.alt_off;
      uint32_t l = 0;
      const uint32_t lim = std::min(p, R[k].s.alt_len);
      while (l < lim && a[l] == a0[l]) ++l;
      p = l;
    }
    for (int k = first; k < m; ++k) {
      if (!(R[k].s.flags & SEGF_HAS_ALT)) continue;
      const uint32_t w = R[k].s.alt_len - p;
      wmin = std::min(wmin, w);
      wmax = std::max(wmax, w);
      const uint8_t* a = raw + R[k].s.alt_off;
      for (uint32_t i = p; i < R[k].s.alt_len && hex; ++i) hex = seg_is_hex_digit(a[i]);
    }
    pe->pfx = p;
    pe->pfx_src = R[first].s.alt_off;
    if (hex && wmin == wmax && wmin >= 1 && wmin <= 16) {
      pe->mode = SEG_ALT_HEX;
      pe->width = wmin;
    }
  }
  altnum.assign((size_t)m, 0);
  if (pe->mode == SEG_ALT_HEX)
    for (int k = 0; k < m; ++k)
      if (R[k].s.flags & SEGF_HAS_ALT) altnum[k] = alt_hex(raw, R[k], pe->pfx);
  uint32_t off = SEG_PAGE_HDR;
  for (int c = 0; c < SEG_NCOL; ++c) {
    ColPlan& p = pe->plan[c];
    if (!seg_is_double(c)) {
      uint64_t lo = ~0ull, hi = 0;
      for (int k = 0; k < m; ++k) {
        const Row& r = R[k];
        if (!seg_member(c, r.o.etype, r.s.flags, (int)pe->mode)) continue;
        const uint64_t u = int_value(c, r, pe->pfx, altnum[k]);
        lo = std::min(lo, u);
        hi = std::max(hi, u);
        ++p.count;
      }
      p.base = p.count ? lo : 0;
      p.bits = p.count ? seg_bitwidth(hi - lo) : 0;
      p.exp = -1;
    } else {
      int e = 0;
      for (int k = 0; k < m; ++k) {
        const Row& r = R[k];
        if (!seg_member(c, r.o.etype, r.s.flags, (int)pe->mode)) continue;
        ++p.count;
        const int ei = seg_dec_exp_from(dbl_value(c, r), exp_hint(c));
        if (ei != SEG_EXC_NONE && ei > e) e = ei;
      }
      uint64_t lo = ~0ull, hi = 0;
      for (int k = 0; k < m; ++k) {
        const Row& r = R[k];
        if (!seg_member(c, r.o.etype, r.s.flags, (int)pe->mode)) continue;
        int64_t q;
        if (seg_dec_at(dbl_value(c, r), e, &q)) {
          lo = std::min(lo, seg_ord(q));
          hi = std::max(hi, seg_ord(q));
        } else {
          ++p.n_exc;
        }
      }
      const bool any = p.count > p.n_exc;
      p.base = any ? lo : 0;
      p.bits = any ? seg_bitwidth(hi - lo) : 0;
      p.exp = e;
    }
    off += seg_col_bytes(p.count, p.bits, p.n_exc);
  }
  uint32_t heap = pe->pfx;
  int32_t amax = INT32_MIN;
  int64_t dmax = INT64_MIN;
  for (int k = 0; k < m; ++k) {
    const Row& r = R[k];
    if (pe->mode == SEG_ALT_RAW && (r.s.flags & SEGF_HAS_ALT)) heap += r.s.alt_len - pe->pfx;
    heap += r.s.msg_len + r.s.meta_len;
    amax = std::max(amax, r.o.assignment);
    dmax = std::max(dmax, r.o.event_date);
  }
  pe->heap_off = off;
  pe->heap_bytes = heap;
  pe->bytes = off + rd8(heap);
  pe->asg_max = m ? amax : 0;
  pe->date_max = m ? dmax : 0;
}

struct WordSink {
  uint8_t* page;
  uint64_t cs = 0;
  void put(uint32_t byte_off, uint64_t w) {
    memcpy(page + byte_off, &w, 8);
    cs ^= seg_mix_word(w, byte_off >> 3);
  }
};

void write_page(const Row* R, int m, const uint8_t* raw, const PageEnc& pe, const std::vector<uint64_t>& altnum,
                uint8_t* page) {
  WordSink ws{page};
  std::vector<uint64_t> vals(SEG_PAGE_ROWS);
  std::vector<uint16_t> exc_idx(SEG_PAGE_ROWS);
  std::vector<uint64_t> exc_raw(SEG_PAGE_ROWS);
  SwSegPageHdr hdr;
  memset(&hdr, 0, sizeof(hdr));
  hdr.n_rows = (uint32_t)m;
  hdr.bytes = pe.bytes;
  hdr.heap_off = pe.heap_off;
  hdr.heap_bytes = pe.heap_bytes;
  hdr.alt_pfx = (uint8_t)pe.pfx;
  hdr.alt_mode = (uint8_t)pe.mode;
  hdr.alt_width = (uint8_t)pe.width;
  hdr.asg_max = pe.asg_max;
  hdr.date_max = pe.date_max;
  uint32_t off = SEG_PAGE_HDR;
  for (int c = 0; c < SEG_NCOL; ++c) {
    const ColPlan& p = pe.plan[c];
    SwSegCol& cd = hdr.cols[c];
    cd.base = p.base;
    cd.data_off = off;
    cd.count = (uint16_t)p.count;
    cd.n_exc = (uint16_t)p.n_exc;
    cd.bits = (uint8_t)p.bits;
    cd.exp = (int8_t)p.exp;
    uint32_t n = 0, ne = 0;
    for (int k = 0; k < m; ++k) {
      const Row& r = R[k];
      if (!seg_member(c, r.o.etype, r.s.flags, (int)pe.mode)) continue;
      if (!seg_is_double(c)) {
        vals[n++] = int_value(c, r, pe.pfx, altnum[k]) - p.base;
      } else {
        const double v = dbl_value(c, r);
        int64_t q;
        if (seg_dec_at(v, p.exp, &q)) {
          vals[n] = seg_ord(q) - p.base;
        } else {
          vals[n] = 0;
          exc_idx[ne] = (uint16_t)n;
          exc_raw[ne++] = sw_f64_bits(v);
        }
        ++n;
      }
    }
    const uint32_t nw = seg_col_words(n, p.bits);
    for (uint32_t w = 0; w < nw; ++w) {
      uint64_t word = 0;
      const uint64_t bit0 = (uint64_t)w * 64;
      uint32_t i = (uint32_t)(bit0 / (uint64_t)p.bits);
      for (; i < n; ++i) {
        const uint64_t b = (uint64_t)i * (uint64_t)p.bits;
        if (b >= bit0 + 64) break;
        if (b >= bit0) {
          word |= vals[i] << (b - bit0);
        } else {                        // value starts in the previous word
          word |= vals[i] >> (bit0 - b);
        }
      }
      ws.put(off + 8 * w, word);
    }
    off += 8 * nw;
    if (ne) {
      const uint32_t nidx = (2 * ne + 7) / 8;
      for (uint32_t w = 0; w < nidx; ++w) {
        uint64_t word = 0;
        for (uint32_t j = 0; j < 4; ++j)
          if (4 * w + j < ne) word |= (uint64_t)exc_idx[4 * w + j] << (16 * j);
        ws.put(off + 8 * w, word);
      }
      off += 8 * nidx;
      for (uint32_t j = 0; j < ne; ++j) ws.put(off + 8 * j, exc_raw[j]);
      off += 8 * ne;
    }
  }
  // string heap (zero padded to a word)
  std::vector<uint8_t> heap(rd8(pe.heap_bytes), 0);
  uint32_t h = 0;
  if (pe.pfx) memcpy(heap.data(), raw + pe.pfx_src, pe.pfx);
  h = pe.pfx;
  for (int k = 0; k < m; ++k) {
    const SegRowStr& s = R[k].s;
    if (pe.mode == SEG_ALT_RAW && (s.flags & SEGF_HAS_ALT)) {
      memcpy(heap.data() + h, raw + s.alt_off + pe.pfx, s.alt_len - pe.pfx);
      h += s.alt_len - pe.pfx;
    }
    if (s.msg_len) { memcpy(heap.data() + h, raw + s.msg_off, s.msg_len); h += s.msg_len; }
    if (s.meta_len) { memcpy(heap.data() + h, raw + s.meta_off, s.meta_len); h += s.meta_len; }
  }
  for (uint32_t w = 0; w < heap.size() / 8; ++w) {
    uint64_t word;
    memcpy(&word, heap.data() + 8 * w, 8);
    ws.put(pe.heap_off + 8 * w, word);
  }
  // header words (the checksum word, index 1, is excluded)
  uint64_t hw[sizeof(SwSegPageHdr) / 8];
  memcpy(hw, &hdr, sizeof(hdr));
  for (uint32_t i = 0; i < sizeof(SwSegPageHdr) / 8; ++i)
    if (i != 1) ws.cs ^= seg_mix_word(hw[i], i);
  hdr.checksum = ws.cs;
  memcpy(page, &hdr, sizeof(hdr));
}

uint64_t header_checksum(const uint8_t* block) {
  SwSegBlockHdr h;
  memcpy(&h, block, sizeof(h));
  h.checksum = 0;
  uint64_t w[8];
  memcpy(w, &h, 64);
  uint64_t cs = 0;
  for (int i = 0; i < 8; ++i) cs ^= seg_mix_word(w[i], i);
  const uint32_t pt = rd8(4u * (h.n_pages + 1));
  for (uint32_t i = 0; i < pt / 8; ++i) {
    uint64_t x;
    memcpy(&x, block + 64 + 8 * i, 8);
    cs ^= seg_mix_word(x, 8 + i);
  }
  return cs;
}

uint64_t unpack(const uint8_t* words, uint32_t i, int bits) {
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

inline uint64_t col_int(const uint8_t* pg, const SwSegCol& cd, uint32_t i) {
  return cd.base + unpack(pg + cd.data_off, i, cd.bits);
}

}  // namespace

extern "C" {

// Encode n rows (step order) into `out` (cap bytes).  rows[j] = the enriched row, recs[j] / spans[j]
// = its decoded record and string refs (may be null: rows without record carry no strings, no
// elevation, no flags), raw = the batch the records were decoded from (raw_bytes long; may be
// null when no row has strings).  Writes the block's n_rows / n_pages / bytes and the page table;
// swseg_seal fills the rest of the header.  Returns the block bytes, or -(bytes needed) when cap is
// too small.
int64_t swseg_encode(const SwOutRec* rows, const SwEventRec* recs, const SwStrRef* spans, const uint8_t* raw,
                     int64_t raw_bytes, int64_t n, uint8_t* out, int64_t cap) {
  const int64_t np = (n + SEG_PAGE_ROWS - 1) / SEG_PAGE_ROWS;
  std::vector<Row> R((size_t)n);
  SwEventRec zr;
  memset(&zr, 0, sizeof(zr));
  SwStrRef zs;
  memset(&zs, 0, sizeof(zs));
  for (int64_t j = 0; j < n; ++j) {
    R[j].o = rows[j];
    const SwEventRec& r = recs ? recs[j] : zr;
    R[j].v2 = recs ? r.v2 : 0.0;
    if (recs) {
      R[j].s = seg_row_strings(r, spans ? spans[j] : zs, raw ? raw_bytes : 0);
    } else {
      memset(&R[j].s, 0, sizeof(R[j].s));
    }
  }
  std::vector<PageEnc> pe((size_t)np);
  std::vector<std::vector<uint64_t>> altnum((size_t)np);
  const uint32_t start = 64 + rd8(4u * (uint32_t)(np + 1));
  uint64_t total = start;
  for (int64_t p = 0; p < np; ++p) {
    const int m = (int)std::min<int64_t>(SEG_PAGE_ROWS, n - p * SEG_PAGE_ROWS);
    plan_page(R.data() + p * SEG_PAGE_ROWS, m, raw, &pe[(size_t)p], altnum[(size_t)p]);
    total += pe[(size_t)p].bytes;
  }
  if ((int64_t)total > cap) return -(int64_t)total;
  memset(out, 0, start);
  uint32_t* pt = (uint32_t*)(out + 64);
  uint64_t off = start;
  for (int64_t p = 0; p < np; ++p) {
    pt[p] = (uint32_t)off;
    const int m = (int)std::min<int64_t>(SEG_PAGE_ROWS, n - p * SEG_PAGE_ROWS);
    write_page(R.data() + p * SEG_PAGE_ROWS, m, raw, pe[(size_t)p], altnum[(size_t)p], out + off);
    off += pe[(size_t)p].bytes;
  }
  pt[np] = (uint32_t)off;
  SwSegBlockHdr h;
  memset(&h, 0, sizeof(h));
  h.n_rows = (uint32_t)n;
  h.n_pages = (uint32_t)np;
  h.bytes = total;
  memcpy(out, &h, sizeof(h));
  return (int64_t)total;
}

// Fill the block header (identity of the batch) and its checksum.
void swseg_seal(uint8_t* block, int64_t first_seq, int64_t recv_ms, int64_t boot, int32_t rank, int32_t world) {
  SwSegBlockHdr h;
  memcpy(&h, block, sizeof(h));
  h.magic = SEG_MAGIC;
  h.version = SEG_VERSION;
  h.flags &= SEG_FLAG_INDEX;      // an index trailer built before sealing stays
  h.first_seq = first_seq;
  h.recv_ms = recv_ms;
  h.boot = boot;
  h.rank = rank;
  h.world = world;
  h.checksum = 0;
  memcpy(block, &h, sizeof(h));
  h.checksum = header_checksum(block);
  memcpy(block, &h, sizeof(h));
}

// Redo the header checksum of a sealed block (after its flags or bytes changed).
void swseg_rechecksum(uint8_t* block) {
  SwSegBlockHdr h;
  memcpy(&h, block, sizeof(h));
  h.checksum = 0;
  memcpy(block, &h, sizeof(h));
  h.checksum = header_checksum(block);
  memcpy(block, &h, sizeof(h));
}

// Set the header flags of a sealed block (SEG_FLAG_COMMIT) and redo its checksum (SEG_FLAG_INDEX,
// which says the block carries an index trailer, is kept).
void swseg_set_flags(uint8_t* block, int32_t flags) {
  SwSegBlockHdr h;
  memcpy(&h, block, sizeof(h));
  h.flags = (uint16_t)((flags & ~SEG_FLAG_INDEX) | (h.flags & SEG_FLAG_INDEX));
  h.checksum = 0;
  memcpy(block, &h, sizeof(h));
  h.checksum = header_checksum(block);
  memcpy(block, &h, sizeof(h));
}

// 0 = valid; 1 bad header, 2 bad page table, 3 bad page header, 4 page checksum, 5 short,
// 6 bad index trailer.
int32_t swseg_verify_pages(const uint8_t* b, int64_t len, int64_t p0, int64_t p1);
int32_t swseg_ix_verify(const uint8_t* t, int64_t len, int64_t n_rows, int64_t n_pages);

static int32_t verify_block(const uint8_t* b, int64_t len, int64_t p0, int64_t p1, bool trailer);

// One page of len bytes holding want_rows rows: its checksum and column / heap bounds (0 ok, 3 bad
// layout, 4 bad checksum).
static int32_t verify_page(const uint8_t* pg, uint32_t len, uint32_t want_rows) {
  if (len < SEG_PAGE_HDR) return 3;
  SwSegPageHdr ph;
  memcpy(&ph, pg, sizeof(ph));
  if (ph.bytes != len || (len & 7)) return 3;
  if (ph.n_rows != want_rows) return 3;
  uint64_t cs = 0;
  for (uint32_t i = 0; i < ph.bytes / 8; ++i) {
    if (i == 1) continue;
    uint64_t w;
    memcpy(&w, pg + 8 * i, 8);
    cs ^= seg_mix_word(w, i);
  }
  if (cs != ph.checksum) return 4;
  for (int c = 0; c < SEG_NCOL; ++c) {
    const SwSegCol& cd = ph.cols[c];
    if (cd.bits > 64 || cd.data_off + seg_col_bytes(cd.count, cd.bits, cd.n_exc) > ph.bytes) return 3;
  }
  if ((uint64_t)ph.heap_off + ph.heap_bytes > ph.bytes || ph.alt_mode > SEG_ALT_HEX || ph.alt_pfx > ph.heap_bytes ||
      ph.alt_width > 16)
    return 3;
  return 0;
}

// The whole block, its index trailer included.
int32_t swseg_verify(const uint8_t* b, int64_t len) { return verify_block(b, len, 0, INT64_MAX, true); }

// swseg_verify of the header, the page table and pages [p0, p1) only: a query that reads a few pages
// of a block checks what it read (the other pages' bytes, and the index trailer, need not be present).
int32_t swseg_verify_pages(const uint8_t* b, int64_t len, int64_t p0, int64_t p1) {
  return verify_block(b, len, p0, p1, false);
}

static int32_t verify_block(const uint8_t* b, int64_t len, int64_t p0, int64_t p1, bool trailer) {
  if (len < 64) return 5;
  SwSegBlockHdr h;
  memcpy(&h, b, sizeof(h));
  if (h.magic != SEG_MAGIC || h.version != SEG_VERSION) return 1;
  const uint64_t start = 64 + rd8(4u * (h.n_pages + 1));
  if ((int64_t)h.bytes > len || h.bytes < start) return 5;
  if ((uint64_t)h.n_pages != ((uint64_t)h.n_rows + SEG_PAGE_ROWS - 1) / SEG_PAGE_ROWS) return 1;
  if (header_checksum(b) != h.checksum) return 1;
  const uint32_t* pt = (const uint32_t*)(b + 64);
  if (h.n_pages && pt[0] != start) return 2;
  if (h.flags & SEG_FLAG_INDEX) {
    // the index trailer follows the pages; checked with the whole block (partial reads skip it)
    if (pt[h.n_pages] > h.bytes || (pt[h.n_pages] & 7) || h.bytes - pt[h.n_pages] < SIX_HDR_BYTES) return 2;
    if (trailer && swseg_ix_verify(b + pt[h.n_pages], (int64_t)(h.bytes - pt[h.n_pages]), h.n_rows, h.n_pages) != 0)
      return 6;
  } else if (pt[h.n_pages] != h.bytes) {
    return 2;
  }
  const uint32_t pend = pt[h.n_pages];
  for (uint32_t p = 0; p < h.n_pages; ++p)
    if (pt[p + 1] < pt[p] + SEG_PAGE_HDR || pt[p + 1] > pend || (pt[p] & 7)) return 2;
  if (p0 < 0) p0 = 0;
  if (p1 > (int64_t)h.n_pages) p1 = h.n_pages;
  for (uint32_t p = (uint32_t)p0; (int64_t)p < p1; ++p) {
    const uint32_t o = pt[p], e = pt[p + 1];
    if (e < o + SEG_PAGE_HDR || e > h.bytes || (o & 7)) return 2;
    const uint32_t want = p + 1 < h.n_pages ? SEG_PAGE_ROWS : h.n_rows - p * SEG_PAGE_ROWS;
    const int32_t rc = verify_page(b + o, e - o, want);
    if (rc) return rc;
  }
  return 0;
}

// Upper bound of the string bytes swseg_decode writes for pages [p0, p1).
int64_t swseg_string_bytes(const uint8_t* b, int64_t p0, int64_t p1) {
  SwSegBlockHdr h;
  memcpy(&h, b, sizeof(h));
  const uint32_t* pt = (const uint32_t*)(b + 64);
  if (p1 > (int64_t)h.n_pages) p1 = h.n_pages;
  int64_t total = 0;
  for (int64_t p = p0; p < p1; ++p) {
    SwSegPageHdr ph;
    memcpy(&ph, b + pt[p], sizeof(ph));
    total += ph.heap_bytes + (int64_t)ph.n_rows * (SEG_ALT_PFX_MAX + 16 + 8);
  }
  return total;
}

namespace {
struct PageScratch {
  std::vector<uint8_t> et = std::vector<uint8_t>(SEG_PAGE_ROWS);
  std::vector<uint32_t> fl = std::vector<uint32_t>(SEG_PAGE_ROWS);
  std::vector<double> dv = std::vector<double>(SEG_PAGE_ROWS);
  std::vector<uint64_t> ak = std::vector<uint64_t>(SEG_PAGE_ROWS), al = std::vector<uint64_t>(SEG_PAGE_ROWS),
                        an = std::vector<uint64_t>(SEG_PAGE_ROWS), ml = std::vector<uint64_t>(SEG_PAGE_ROWS),
                        dl = std::vector<uint64_t>(SEG_PAGE_ROWS);
};

// One (verified) page into rows r0.. of the outputs (any may be null); strings appended at *so.
// Returns the page's rows, -1 if str_cap is too small.
int64_t decode_page(const uint8_t* pg, int64_t r0, uint8_t* etype, uint8_t* level, int64_t* date, int32_t* asg,
                    uint16_t* name, double* v0, double* v1, double* v2, uint8_t* flags, uint8_t* str_heap,
                    int64_t str_cap, int64_t* so, int64_t* str_off, PageScratch& ws) {
  auto& et = ws.et; auto& fl = ws.fl; auto& dv = ws.dv;
  auto& ak = ws.ak; auto& al = ws.al; auto& an = ws.an; auto& ml = ws.ml; auto& dl = ws.dl;
  SwSegPageHdr ph;
  memcpy(&ph, pg, sizeof(ph));
  const uint32_t m = ph.n_rows;
  const int mode = ph.alt_mode;
  // etype and flags first: every other column's membership depends on them
  for (uint32_t k = 0; k < m; ++k) {
    et[k] = (uint8_t)seg_unord(col_int(pg, ph.cols[SEG_ETYPE], k));
    fl[k] = (uint32_t)seg_unord(col_int(pg, ph.cols[SEG_FLAGS], k));
  }
  if (etype) memcpy(etype + r0, et.data(), m);
  if (flags)
    for (uint32_t k = 0; k < m; ++k) flags[r0 + k] = (uint8_t)fl[k];
  for (int c = 0; c < SEG_NCOL; ++c) {
    if (c == SEG_ETYPE || c == SEG_FLAGS) continue;
    // columns nobody asked for are not unpacked (string lengths only feed the heap)
    const bool want = c == SEG_LEVEL ? level != nullptr : c == SEG_DATE ? date != nullptr
                    : c == SEG_ASG ? asg != nullptr : c == SEG_NAME ? name != nullptr
                    : (c == SEG_MXV || c == SEG_LAT) ? v0 != nullptr : c == SEG_LON ? v1 != nullptr
                    : c == SEG_ELEV ? v2 != nullptr : str_heap != nullptr;
    if (!want) continue;
    const SwSegCol& cd = ph.cols[c];
    const uint8_t* words = pg + cd.data_off;
    if (seg_is_double(c)) {
      const uint8_t* xi = words + 8 * seg_col_words(cd.count, cd.bits);
      const uint8_t* xr = xi + ((2u * cd.n_exc + 7u) & ~7u);
      for (uint32_t i = 0; i < cd.count; ++i)
        dv[i] = seg_dec_value(seg_unord(cd.base + unpack(words, i, cd.bits)), cd.exp);
      for (uint32_t j = 0; j < cd.n_exc; ++j) {
        uint16_t ix;
        uint64_t raw;
        memcpy(&ix, xi + 2 * j, 2);
        memcpy(&raw, xr + 8 * j, 8);
        if (ix < cd.count) dv[ix] = sw_bits_f64(raw);
      }
    }
    uint32_t i = 0;
    for (uint32_t k = 0; k < m; ++k) {
      const int64_t r = r0 + k;
      const bool mem = seg_member(c, et[k], fl[k], mode);
      const uint64_t u = mem && !seg_is_double(c) ? cd.base + unpack(words, i, cd.bits) : 0;
      switch (c) {
        case SEG_LEVEL:
          if (level) level[r] = mem ? (uint8_t)seg_unord(u) : 0;
          break;
        case SEG_DATE:
          if (date) date[r] = seg_unord(u);
          break;
        case SEG_ASG:
          if (asg) asg[r] = (int32_t)seg_unord(u);
          break;
        case SEG_NAME:
          if (name) name[r] = mem ? (uint16_t)seg_unord(u) : (uint16_t)0xffff;
          break;
        case SEG_MXV:                 // runs before SEG_LAT: zero v0 of every non-measurement
          if (v0) v0[r] = mem ? dv[i] : 0.0;
          break;
        case SEG_LAT:
          if (v0 && mem) v0[r] = dv[i];
          break;
        case SEG_LON:
          if (v1) v1[r] = mem ? dv[i] : 0.0;
          break;
        case SEG_ELEV:
          if (v2) v2[r] = mem ? dv[i] : 0.0;
          break;
        case SEG_ALTK: ak[k] = mem ? (uint64_t)seg_unord(u) : 0; break;
        case SEG_ALTLEN: al[k] = mem ? (uint64_t)seg_unord(u) : 0; break;
        case SEG_ALTNUM: an[k] = mem ? u : 0; break;
        case SEG_MSGLEN: ml[k] = mem ? (uint64_t)seg_unord(u) : 0; break;
        case SEG_METALEN: dl[k] = mem ? (uint64_t)seg_unord(u) : 0; break;
      }
      if (mem) ++i;
    }
  }
  if (str_heap) {
    const uint8_t* heap = pg + ph.heap_off;
    uint32_t ho = ph.alt_pfx;
    for (uint32_t k = 0; k < m; ++k) {
      const int64_t r = r0 + k;
      // alternate id
      if (fl[k] & SEGF_HAS_ALT) {
        const int64_t need = *so + ph.alt_pfx + (mode == SEG_ALT_HEX ? ph.alt_width : al[k]) + 8;
        if (need > str_cap) return -1;
        memcpy(str_heap + *so, heap, ph.alt_pfx);
        *so += ph.alt_pfx;
        if (mode == SEG_ALT_HEX) {
          for (int d = (int)ph.alt_width - 1; d >= 0; --d)
            str_heap[(*so)++] = "0123456789abcdef"[(an[k] >> (4 * d)) & 15];
        } else {
          memcpy(str_heap + *so, heap + ho, al[k]);
          *so += (int64_t)al[k];
          ho += (uint32_t)al[k];
        }
        if (ak[k]) {
          char sfx[8];
          const int n = snprintf(sfx, sizeof(sfx), ":%u", (unsigned)(ak[k] - 1));
          if (*so + n > str_cap) return -1;
          memcpy(str_heap + *so, sfx, (size_t)n);
          *so += n;
        }
      }
      if (str_off) str_off[3 * r + 1] = *so;
      if (*so + (int64_t)ml[k] + (int64_t)dl[k] > str_cap) return -1;
      memcpy(str_heap + *so, heap + ho, ml[k]);
      *so += (int64_t)ml[k];
      ho += (uint32_t)ml[k];
      if (str_off) str_off[3 * r + 2] = *so;
      memcpy(str_heap + *so, heap + ho, dl[k]);
      *so += (int64_t)dl[k];
      ho += (uint32_t)dl[k];
      if (str_off) str_off[3 * r + 3] = *so;
    }
  }
  return m;
}

// Rows rows[0..nw) (ascending, < the page's rows) of one (verified) page into slots 0..nw of the
// outputs, without decoding the rest: one pass over the leading rows counts each column's members
// (a row's value sits at its member index) and the string bytes before the row.  Strings as
// decode_page (str_off[3 w + 1..3], appended at *so).  Returns nw, -1 if str_cap is too small.
int64_t decode_rows(const uint8_t* pg, const int32_t* rows, int64_t nw, uint8_t* etype, uint8_t* level, int64_t* date,
                    int32_t* asg, uint16_t* name, double* v0, double* v1, double* v2, uint8_t* flags,
                    uint8_t* str_heap, int64_t str_cap, int64_t* so, int64_t* str_off) {
  SwSegPageHdr ph;
  memcpy(&ph, pg, sizeof(ph));
  const int mode = ph.alt_mode;
  const uint8_t* heap = pg + ph.heap_off;
  uint32_t cnt[SEG_NCOL] = {0};
  uint32_t ho = ph.alt_pfx;                         // heap bytes before row j's strings
  int64_t w = 0;
  auto member_value = [&](int c, uint32_t ix) -> uint64_t { return ph.cols[c].base + unpack(pg + ph.cols[c].data_off, ix, ph.cols[c].bits); };
  // exceptions are stored in ascending member order and rows are visited in ascending order: one
  // cursor per column walks each exception list once per call (not once per row)
  uint32_t xc[SEG_NCOL] = {0};
  auto dbl = [&](int c, uint32_t ix) -> double {
    const SwSegCol& cd = ph.cols[c];
    const uint8_t* words = pg + cd.data_off;
    const uint8_t* xi = words + 8 * seg_col_words(cd.count, cd.bits);
    const uint8_t* xr = xi + ((2u * cd.n_exc + 7u) & ~7u);
    uint32_t& j = xc[c];
    for (; j < cd.n_exc; ++j) {
      uint16_t x;
      memcpy(&x, xi + 2 * j, 2);
      if (x < ix) continue;
      if (x == ix) {
        uint64_t raw;
        memcpy(&raw, xr + 8 * j, 8);
        return sw_bits_f64(raw);
      }
      break;
    }
    return seg_dec_value(seg_unord(cd.base + unpack(words, ix, cd.bits)), cd.exp);
  };
  for (uint32_t j = 0; j < ph.n_rows && w < nw; ++j) {
    const uint8_t et = (uint8_t)seg_unord(col_int(pg, ph.cols[SEG_ETYPE], j));
    const uint32_t f = (uint32_t)seg_unord(col_int(pg, ph.cols[SEG_FLAGS], j));
    const bool has_alt = seg_member(SEG_ALTLEN, et, f, mode);
    const uint64_t al = has_alt ? (uint64_t)seg_unord(member_value(SEG_ALTLEN, cnt[SEG_ALTLEN])) : 0;
    const bool has_msg = seg_member(SEG_MSGLEN, et, f, mode);
    const uint64_t ml = has_msg ? (uint64_t)seg_unord(member_value(SEG_MSGLEN, cnt[SEG_MSGLEN])) : 0;
    const bool has_md = seg_member(SEG_METALEN, et, f, mode);
    const uint64_t dl = has_md ? (uint64_t)seg_unord(member_value(SEG_METALEN, cnt[SEG_METALEN])) : 0;
    const uint64_t a_raw = mode == SEG_ALT_HEX ? 0 : al;      // heap bytes of the id's remainder
    while (w < nw && (uint32_t)rows[w] == j) {
      if (etype) etype[w] = et;
      if (flags) flags[w] = (uint8_t)f;
      if (level) level[w] = seg_member(SEG_LEVEL, et, f, mode) ? (uint8_t)seg_unord(member_value(SEG_LEVEL, cnt[SEG_LEVEL])) : 0;
      if (date) date[w] = seg_unord(member_value(SEG_DATE, j));
      if (asg) asg[w] = (int32_t)seg_unord(member_value(SEG_ASG, j));
      if (name) name[w] = seg_member(SEG_NAME, et, f, mode) ? (uint16_t)seg_unord(member_value(SEG_NAME, cnt[SEG_NAME])) : (uint16_t)0xffff;
      if (v0) v0[w] = seg_member(SEG_MXV, et, f, mode) ? dbl(SEG_MXV, cnt[SEG_MXV])
                    : seg_member(SEG_LAT, et, f, mode) ? dbl(SEG_LAT, cnt[SEG_LAT]) : 0.0;
      if (v1) v1[w] = seg_member(SEG_LON, et, f, mode) ? dbl(SEG_LON, cnt[SEG_LON]) : 0.0;
      if (v2) v2[w] = seg_member(SEG_ELEV, et, f, mode) ? dbl(SEG_ELEV, cnt[SEG_ELEV]) : 0.0;
      if (str_heap) {
        if (has_alt) {
          const int64_t need = *so + ph.alt_pfx + (mode == SEG_ALT_HEX ? ph.alt_width : al) + 8;
          if (need > str_cap) return -1;
          memcpy(str_heap + *so, heap, ph.alt_pfx);
          *so += ph.alt_pfx;
          if (mode == SEG_ALT_HEX) {
            const uint64_t an = member_value(SEG_ALTNUM, cnt[SEG_ALTNUM]);
            for (int d = (int)ph.alt_width - 1; d >= 0; --d) str_heap[(*so)++] = "0123456789abcdef"[(an >> (4 * d)) & 15];
          } else {
            memcpy(str_heap + *so, heap + ho, al);
            *so += (int64_t)al;
          }
          const uint64_t ak = (uint64_t)seg_unord(member_value(SEG_ALTK, cnt[SEG_ALTK]));
          if (ak) {
            char sfx[8];
            const int n = snprintf(sfx, sizeof(sfx), ":%u", (unsigned)(ak - 1));
            if (*so + n > str_cap) return -1;
            memcpy(str_heap + *so, sfx, (size_t)n);
            *so += n;
          }
        }
        if (str_off) str_off[3 * w + 1] = *so;
        if (*so + (int64_t)ml + (int64_t)dl > str_cap) return -1;
        memcpy(str_heap + *so, heap + ho + a_raw, ml);
        *so += (int64_t)ml;
        if (str_off) str_off[3 * w + 2] = *so;
        memcpy(str_heap + *so, heap + ho + a_raw + ml, dl);
        *so += (int64_t)dl;
        if (str_off) str_off[3 * w + 3] = *so;
      }
      ++w;
    }
    // advance past row j: its members in every sparse column, its string bytes
    for (int c = 0; c < SEG_NCOL; ++c)
      if (c != SEG_ETYPE && c != SEG_FLAGS && c != SEG_DATE && c != SEG_ASG && seg_member(c, et, f, mode)) ++cnt[c];
    ho += (uint32_t)(a_raw + ml + dl);
  }
  return w == nw ? nw : -2;
}
}  // namespace

// Decode pages [p0, p1) of a (verified) block into per-row arrays (row 0 = the first row of page p0).
// Any output may be null.  name = 0xffff where the row has none; v0/v1/v2 = 0 where the type has no
// such value (flags tell whether an elevation was sent).  Strings (str_heap non-null, str_cap bytes,
// see swseg_string_bytes): per row its alternate id (full form, "<alt>:<k>" for measurement k of a
// multi-measurement payload), alert message and metadata span, back to back; str_off[3 r + 0..3]
// delimit them.  Returns the rows decoded, -1 if str_cap is too small.
int64_t swseg_decode(const uint8_t* b, int64_t p0, int64_t p1, uint8_t* etype, uint8_t* level, int64_t* date,
                     int32_t* asg, uint16_t* name, double* v0, double* v1, double* v2, uint8_t* flags,
                     uint8_t* str_heap, int64_t str_cap, int64_t* str_off) {
  SwSegBlockHdr h;
  memcpy(&h, b, sizeof(h));
  const uint32_t* pt = (const uint32_t*)(b + 64);
  if (p1 > (int64_t)h.n_pages) p1 = h.n_pages;
  PageScratch ws;
  int64_t r0 = 0, so = 0;
  if (str_off) str_off[0] = 0;
  for (int64_t p = p0; p < p1; ++p) {
    const int64_t m = decode_page(b + pt[p], r0, etype, level, date, asg, name, v0, v1, v2, flags, str_heap, str_cap,
                                  &so, str_off, ws);
    if (m < 0) return -1;
    r0 += m;
  }
  return r0;
}

// Point reads of single rows across blocks: request i is row row_in_page[i] of the page at file
// offset pg_pos[i] (pg_bytes[i] bytes, pg_rows[i] rows) of file fds[i].  Each distinct page (requests
// of one page adjacent) is pread and verified once, decoded on one of `threads` threads, and the
// requested rows copied out in request order (outputs as swseg_decode, one row per request; strings
// back to back in str_heap, str_off[3 i + 0..3]).  Returns n, -(1 + i) when request i's page cannot be
// read or fails its check, or -(1 << 40) - need when str_cap is below the `need` string bytes.
int64_t swseg_fetch_rows(const int32_t* fds, const int64_t* pg_pos, const uint32_t* pg_bytes, const uint32_t* pg_rows,
                         const int32_t* row_in_page, int64_t n, int32_t threads, uint8_t* etype, uint8_t* level,
                         int64_t* date, int32_t* asg, uint16_t* name, double* v0, double* v1, double* v2,
                         uint8_t* flags, uint8_t* str_heap, int64_t str_cap, int64_t* str_off,
                         const uint64_t* mem) {
  if (n <= 0) return 0;
  std::vector<int64_t> first;                       // first request of each distinct page
  for (int64_t i = 0; i < n; ++i)
    if (i == 0 || fds[i] != fds[i - 1] || pg_pos[i] != pg_pos[i - 1]) first.push_back(i);
  const int64_t np = (int64_t)first.size();
  first.push_back(n);
  // per distinct page: its requests sorted by row, decoded into slots at the group's start
  std::vector<int64_t> perm((size_t)n);
  std::vector<int32_t> srow((size_t)n);
  for (int64_t q = 0; q < np; ++q) {
    for (int64_t i = first[q]; i < first[q + 1]; ++i) perm[i] = i;
    std::stable_sort(perm.begin() + first[q], perm.begin() + first[q + 1],
                     [&](int64_t x, int64_t y) { return row_in_page[x] < row_in_page[y]; });
    for (int64_t i = first[q]; i < first[q + 1]; ++i) srow[i] = row_in_page[perm[i]];
  }
  std::vector<uint8_t> et(n), lv(n), fl(n);
  std::vector<int64_t> dt(n);
  std::vector<int32_t> as(n);
  std::vector<uint16_t> nm(n);
  std::vector<double> a0(n), a1(n), a2(n);
  std::vector<std::vector<uint8_t>> heaps((size_t)np);
  std::vector<int64_t> soff(3 * (size_t)n + 1, 0);   // per slot, relative to its page group's heap
  std::atomic<int64_t> bad{-1};
  int T = threads > 0 ? threads : 1;
  if (T > 32) T = 32;
  if ((int64_t)T > np) T = (int)np;
  auto work = [&](int w) {
    std::vector<uint8_t> buf;
    std::vector<int64_t> loc;
    for (int64_t q = np * w / T; q < np * (w + 1) / T; ++q) {
      const int64_t i = first[q], k = first[q + 1] - first[q];
      const uint32_t len = pg_bytes[i];
      if (len < SEG_PAGE_HDR || len > (64u << 20) || pg_rows[i] > SEG_PAGE_ROWS) { bad = i; return; }
      const uint8_t* pg = mem && mem[i] ? reinterpret_cast<const uint8_t*>((uintptr_t)mem[i]) : nullptr;
      if (!pg) {
        buf.resize(len);
        if (pread(fds[i], buf.data(), len, pg_pos[i]) != (ssize_t)len) { bad = i; return; }
        pg = buf.data();
      }
      if (verify_page(pg, len, pg_rows[i])) { bad = i; return; }
      for (int64_t j = i; j < i + k; ++j)
        if (srow[j] < 0 || (uint32_t)srow[j] >= pg_rows[i]) { bad = perm[j]; return; }
      SwSegPageHdr ph;
      memcpy(&ph, pg, sizeof(ph));
      heaps[(size_t)q].resize((size_t)ph.heap_bytes + (size_t)k * (SEG_ALT_PFX_MAX + 16 + 8) + 8);
      loc.assign(3 * (size_t)k + 1, 0);
      int64_t so = 0;
      if (decode_rows(pg, srow.data() + i, k, et.data() + i, lv.data() + i, dt.data() + i, as.data() + i,
                      nm.data() + i, a0.data() + i, a1.data() + i, a2.data() + i, fl.data() + i,
                      heaps[(size_t)q].data(), (int64_t)heaps[(size_t)q].size(), &so, loc.data()) != k) {
        bad = i;
        return;
      }
      for (int64_t j = 0; j < 3 * k; ++j) soff[3 * (size_t)i + 1 + j] = loc[1 + j];
    }
  };
  if (T <= 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int w = 0; w < T; ++w) th.emplace_back(work, w);
    for (auto& x : th) x.join();
  }
  if (bad.load() >= 0) return -(1 + bad.load());
  // slot j's strings: [start, end) of its group's heap, start = end of the slot before it in the group
  auto s_beg = [&](int64_t q, int64_t j) { return j == first[q] ? (int64_t)0 : soff[3 * (size_t)j]; };
  int64_t need = 0;
  for (int64_t q = 0; q < np; ++q)
    for (int64_t j = first[q]; j < first[q + 1]; ++j) need += soff[3 * (size_t)j + 3] - s_beg(q, j);
  if (str_heap && need > str_cap) return -(int64_t(1) << 40) - need;
  // out in request order: request perm[j] takes slot j
  int64_t so = 0;
  if (str_off) str_off[0] = 0;
  std::vector<int64_t> slot_of((size_t)n), grp((size_t)n);
  for (int64_t q = 0; q < np; ++q)
    for (int64_t j = first[q]; j < first[q + 1]; ++j) { slot_of[perm[j]] = j; grp[j] = q; }
  for (int64_t i = 0; i < n; ++i) {
    const int64_t j = slot_of[i], q = grp[j];
    if (etype) etype[i] = et[j];
    if (level) level[i] = lv[j];
    if (date) date[i] = dt[j];
    if (asg) asg[i] = as[j];
    if (name) name[i] = nm[j];
    if (v0) v0[i] = a0[j];
    if (v1) v1[i] = a1[j];
    if (v2) v2[i] = a2[j];
    if (flags) flags[i] = fl[j];
    if (str_heap) {
      int64_t s0 = s_beg(q, j);
      for (int k = 0; k < 3; ++k) {
        const int64_t s1 = soff[3 * (size_t)j + k + 1];
        memcpy(str_heap + so, heaps[(size_t)q].data() + s0, (size_t)(s1 - s0));
        so += s1 - s0;
        s0 = s1;
        if (str_off) str_off[3 * i + k + 1] = so;
      }
    }
  }
  return n;
}

// Rows whose alternate id hashes to hashes[i] in candidate page i (the pages a trailer's fingerprint
// search named): each page pread from fds[i] at pg_pos[i] (pg_bytes[i] bytes, pg_rows[i] rows),
// verified, its id column decoded, on `threads` threads.  Writes (page task, row in page) of every
// match, tasks in order and rows ascending; returns the matches (> cap: call again with that cap), or
// -(1 + i) when page i cannot be read or fails its check.
int64_t swseg_alt_page_rows(const int32_t* fds, const int64_t* pg_pos, const uint32_t* pg_bytes,
                            const uint32_t* pg_rows, const uint64_t* hashes, int64_t n, int32_t threads,
                            int64_t* out_task, int32_t* out_row, int64_t cap, const uint64_t* mem) {
  if (n <= 0) return 0;
  int T = threads > 0 ? threads : 1;
  if (T > 32) T = 32;
  if ((int64_t)T > n) T = (int)n;
  std::vector<std::vector<std::pair<int64_t, int32_t>>> hits(T);
  std::atomic<int64_t> bad{-1};
  auto work = [&](int w) {
    PageScratch ws;
    std::vector<uint8_t> buf, heap, fl(SEG_PAGE_ROWS);
    std::vector<int64_t> so(3 * SEG_PAGE_ROWS + 1);
    for (int64_t i = n * w / T; i < n * (w + 1) / T; ++i) {
      const uint32_t len = pg_bytes[i];
      if (len < SEG_PAGE_HDR || len > (64u << 20) || pg_rows[i] > SEG_PAGE_ROWS) { bad = i; return; }
      const uint8_t* pg = mem && mem[i] ? reinterpret_cast<const uint8_t*>((uintptr_t)mem[i]) : nullptr;
      if (!pg) {
        buf.resize(len);
        if (pread(fds[i], buf.data(), len, pg_pos[i]) != (ssize_t)len) { bad = i; return; }
        pg = buf.data();
      }
      if (verify_page(pg, len, pg_rows[i])) { bad = i; return; }
      SwSegPageHdr ph;
      memcpy(&ph, pg, sizeof(ph));
      heap.resize((size_t)ph.heap_bytes + (size_t)ph.n_rows * (SEG_ALT_PFX_MAX + 16 + 8) + 8);
      int64_t o = 0;
      so[0] = 0;
      if (decode_page(pg, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, fl.data(),
                      heap.data(), (int64_t)heap.size(), &o, so.data(), ws) != (int64_t)ph.n_rows) {
        bad = i;
        return;
      }
      for (uint32_t r = 0; r < ph.n_rows; ++r)
        if ((fl[r] & SEGF_HAS_ALT) &&
            sw_hash64(heap.data() + so[3 * r], (uint32_t)(so[3 * r + 1] - so[3 * r])) == hashes[i])
          hits[w].push_back({i, (int32_t)r});
    }
  };
  if (T <= 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int w = 0; w < T; ++w) th.emplace_back(work, w);
    for (auto& x : th) x.join();
  }
  if (bad.load() >= 0) return -(1 + bad.load());
  int64_t k = 0;
  for (int w = 0; w < T; ++w)
    for (const auto& h : hits[w]) {
      if (k < cap) { out_task[k] = h.first; out_row[k] = h.second; }
      ++k;
    }
  return k;
}

// Per-page summaries of a block (pages in order): first row, rows, assignment min / max, event date
// min / max -- the store's page index for indexed reads.  out = int64[6 * n_pages].
int64_t swseg_page_summary(const uint8_t* b, int64_t* out) {
  SwSegBlockHdr h;
  memcpy(&h, b, sizeof(h));
  const uint32_t* pt = (const uint32_t*)(b + 64);
  for (uint32_t p = 0; p < h.n_pages; ++p) {
    SwSegPageHdr ph;
    memcpy(&ph, b + pt[p], sizeof(ph));
    int64_t* o = out + 6 * p;
    o[0] = (int64_t)p * SEG_PAGE_ROWS;
    o[1] = ph.n_rows;
    o[2] = seg_unord(ph.cols[SEG_ASG].base);
    o[3] = ph.asg_max;
    o[4] = seg_unord(ph.cols[SEG_DATE].base);
    o[5] = ph.date_max;
  }
  return h.n_pages;
}

// ----------------------------------------------------------------------------- block indexes
// LSD radix sort of (key, value) pairs by key, 16-bit digits; stable (equal keys keep input order).
static void radix_sort_pairs(std::vector<uint64_t>& k, std::vector<uint32_t>& v, int key_bits) {
  const size_t n = k.size();
  std::vector<uint64_t> k2(n);
  std::vector<uint32_t> v2(n);
  std::vector<uint32_t> cnt(1u << 16);
  for (int shift = 0; shift < key_bits; shift += 16) {
    std::fill(cnt.begin(), cnt.end(), 0u);
    for (size_t i = 0; i < n; ++i) ++cnt[(k[i] >> shift) & 0xffff];
    uint32_t sum = 0;
    for (auto& c : cnt) { const uint32_t t = c; c = sum; sum += t; }
    for (size_t i = 0; i < n; ++i) {
      const uint32_t d = cnt[(k[i] >> shift) & 0xffff]++;
      k2[d] = k[i];
      v2[d] = v[i];
    }
    k.swap(k2);
    v.swap(v2);
  }
}

// The store's per-block indexes (persistence/segments.py BlockIndex), from a verified block:
//   postings, one per row, sorted by (key asc, event date desc, row desc):
//     post_key = assignment << 3 | event type, post_date = event date - min_date, post_row = row;
//     *date_wide = 1 when some date is outside [min_date, min_date + 2^32) ms (then post_date is
//     clamped and the caller must not order by it)
//   alternate ids, one per row that has one, sorted by hash: alt_hash = sw_hash64 of the full id
//     (the engine's dedup hash), alt_row = row.
// Returns the number of alternate ids, -1 on a malformed block.
int64_t swseg_index_block(const uint8_t* b, int64_t min_date, uint32_t* post_key, uint32_t* post_date,
                          uint32_t* post_row, uint64_t* alt_hash, uint32_t* alt_row, int32_t* date_wide) {
  SwSegBlockHdr h;
  memcpy(&h, b, sizeof(h));
  const int64_t n = h.n_rows;
  std::vector<uint8_t> et(n), fl(n);
  std::vector<int64_t> date(n);
  std::vector<int32_t> asg(n);
  const int64_t cap = swseg_string_bytes(b, 0, h.n_pages) + 64;
  std::vector<uint8_t> heap(cap);
  std::vector<int64_t> so(3 * n + 1);
  if (swseg_decode(b, 0, h.n_pages, et.data(), nullptr, date.data(), asg.data(), nullptr, nullptr, nullptr, nullptr,
                   fl.data(), heap.data(), cap, so.data()) != n)
    return -1;
  // postings: sort key (key << 32 | ~rel_date), rows fed newest first so equal keys keep row desc
  std::vector<uint64_t> k(n);
  std::vector<uint32_t> v(n);
  int32_t wide = 0;
  for (int64_t j = 0; j < n; ++j) {
    const int64_t r = n - 1 - j;
    int64_t rel = date[r] - min_date;
    if (rel < 0 || rel > 0xffffffffLL) { wide = 1; rel = rel < 0 ? 0 : 0xffffffffLL; }
    const uint64_t key = ((uint64_t)(uint32_t)asg[r] << 3) | (uint64_t)(et[r] & 7u);
    k[j] = (key << 32) | (uint64_t)(0xffffffffu - (uint32_t)rel);
    v[j] = (uint32_t)r;
  }
  radix_sort_pairs(k, v, 64);
  for (int64_t i = 0; i < n; ++i) {
    post_key[i] = (uint32_t)(k[i] >> 32);
    post_date[i] = 0xffffffffu - (uint32_t)k[i];
    post_row[i] = v[i];
  }
  *date_wide = wide;
  // alternate ids
  k.clear();
  v.clear();
  for (int64_t r = 0; r < n; ++r) {
    if (!(fl[r] & SEGF_HAS_ALT)) continue;
    const int64_t a0 = so[3 * r], a1 = so[3 * r + 1];
    k.push_back(sw_hash64(heap.data() + a0, (uint32_t)(a1 - a0)));
    v.push_back((uint32_t)r);
  }
  radix_sort_pairs(k, v, 64);
  for (size_t i = 0; i < k.size(); ++i) {
    alt_hash[i] = k[i];
    alt_row[i] = v[i];
  }
  return (int64_t)k.size();
}

// Point lookups over many blocks' indexes in one call (the store's per-query work is then a few
// binary searches per block in native code, not a Python loop).  For each of the n sorted arrays:
// [lo, hi) of `key`.  u32 variant (postings): with dates (u32, relative to base[i], descending within
// a key) the range is restricted to event dates in [d_lo, d_hi].
void swseg_multi_range_u64(const uint64_t* const* keys, const int64_t* lens, int64_t n, uint64_t key,
                           int64_t* lo_out, int64_t* hi_out) {
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t* a = keys[i];
    const uint64_t* l = std::lower_bound(a, a + lens[i], key);
    const uint64_t* h = std::upper_bound(l, a + lens[i], key);
    lo_out[i] = l - a;
    hi_out[i] = h - a;
  }
}

// Bulk form for the store-backed dedup: for each wanted key, the last array (highest i: blocks are
// in store order, so the newest block) that holds it and the key's last position there; -1 / -1 when
// no array does.  n_want x n binary searches, no Python per block.
void swseg_multi_find_u64(const uint64_t* const* keys, const int64_t* lens, int64_t n, const uint64_t* want,
                          int64_t n_want, int64_t* blk_out, int64_t* pos_out) {
  for (int64_t j = 0; j < n_want; ++j) {
    blk_out[j] = pos_out[j] = -1;
    const uint64_t w = want[j];
    for (int64_t i = n - 1; i >= 0; --i) {
      const uint64_t* a = keys[i];
      if (!a || lens[i] <= 0) continue;
      const uint64_t* h = std::upper_bound(a, a + lens[i], w);
      if (h != a && h[-1] == w) {
        blk_out[j] = i;
        pos_out[j] = (h - a) - 1;
        break;
      }
    }
  }
}

void swseg_multi_range_u32(const uint32_t* const* keys, const uint32_t* const* dates, const int64_t* lens,
                           const int64_t* base, int64_t n, uint32_t key, int64_t d_lo, int64_t d_hi,
                           int64_t* lo_out, int64_t* hi_out) {
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t* a = keys[i];
    int64_t lo = std::lower_bound(a, a + lens[i], key) - a;
    int64_t hi = std::upper_bound(a + lo, a + lens[i], key) - a;
    if (dates && lo < hi) {
      const uint32_t* d = dates[i];
      // dates descend within the key: first entry <= d_hi, first entry < d_lo
      const int64_t rhi = d_hi - base[i], rlo = d_lo - base[i];
      if (rhi < 0) { lo = hi; }
      else if (rhi < 0xffffffffLL) {
        const uint32_t x = (uint32_t)rhi;
        lo = std::partition_point(d + lo, d + hi, [x](uint32_t v) { return v > x; }) - d;
      }
      if (rlo > 0xffffffffLL) { hi = lo; }
      else if (rlo > 0) {
        const uint32_t x = (uint32_t)rlo;
        hi = std::partition_point(d + lo, d + hi, [x](uint32_t v) { return v >= x; }) - d;
      }
    }
    lo_out[i] = lo;
    hi_out[i] = hi < lo ? lo : hi;
  }
}

}  // extern "C"

// ----------------------------------------------------------------------------- segment store
struct SegFile {
  std::string path;
  int64_t first_seq;
  int64_t bytes;
  int32_t id;
  int64_t rows = 0;      // event rows of the file's blocks (retention by rows)
};

// Block index entry (kept in memory by the store, rebuilt by the recovery scan).
typedef struct SwSegIndexEnt {
  int64_t first_seq;
  int64_t recv_ms;
  int64_t offset;
  int64_t bytes;
  int32_t file;          // SegFile::id
  int32_t n_rows;
  int32_t rank;
  int32_t world;
  int64_t min_date;
  int64_t max_date;
  int64_t boot;
} SwSegIndexEnt;

static void block_dates(const uint8_t* b, int64_t* lo, int64_t* hi) {
  SwSegBlockHdr h;
  memcpy(&h, b, sizeof(h));
  const uint32_t* pt = (const uint32_t*)(b + 64);
  *lo = INT64_MAX;
  *hi = INT64_MIN;
  for (uint32_t p = 0; p < h.n_pages; ++p) {
    SwSegPageHdr ph;
    memcpy(&ph, b + pt[p], sizeof(ph));
    *lo = std::min(*lo, seg_unord(ph.cols[SEG_DATE].base));
    *hi = std::max(*hi, ph.date_max);
  }
}

static SwSegIndexEnt index_entry(const SwSegBlockHdr& hd, const uint8_t* b, int32_t file, int64_t off) {
  SwSegIndexEnt e;
  e.first_seq = hd.first_seq;
  e.recv_ms = hd.recv_ms;
  e.offset = off;
  e.bytes = (int64_t)hd.bytes;
  e.file = file;
  e.n_rows = (int32_t)hd.n_rows;
  e.rank = hd.rank;
  e.world = hd.world;
  e.boot = hd.boot;
  block_dates(b, &e.min_date, &e.max_date);
  return e;
}

struct SegItem {
  const uint8_t* ptr;
  int64_t len;          // block bytes (unpadded)
  int64_t token;
  std::vector<std::pair<uint64_t, int64_t>> src;   // commit record entries (flagged blocks)
};

static uint64_t commit_checksum(const uint8_t* rec, uint32_t n_src) {
  uint64_t cs = 0;
  const uint32_t words = (64 + 16 * n_src) / 8;
  for (uint32_t i = 0; i < words; ++i) {
    if (i == 7) continue;                 // the checksum word
    uint64_t w;
    memcpy(&w, rec + 8 * i, 8);
    cs ^= seg_mix_word(w, i);
  }
  return cs;
}

// 0 when rec (len bytes available) is a valid commit record
static int commit_valid(const uint8_t* rec, int64_t len) {
  if (len < 64) return 1;
  SwSegCommitHdr c;
  memcpy(&c, rec, sizeof(c));
  if (c.magic != SEG_COMMIT_MAGIC || c.version != SEG_VERSION || c.n_src > SEG_MAX_SRC) return 1;
  if (c.bytes != 64 + 16ull * c.n_src || (int64_t)c.bytes > len) return 1;
  return commit_checksum(rec, c.n_src) == c.checksum ? 0 : 1;
}

struct SegStore {
  std::string dir;
  int32_t rank = 0;
  int64_t rotate_bytes = 1ll << 30;
  int64_t retention_bytes = 0;
  // retention by rows (0: none): oldest whole files are deleted while the rows kept exceed it -- an
  // engine tenant's store-backed dedup filter remembers the newest N alternate ids, and a store that
  // keeps at most N rows keeps no id it has forgotten (EngineConfig.filter_retention_rows)
  int64_t retention_rows = 0;
  int64_t total_rows = 0;
  bool direct = true;
  std::mutex mu;
  std::condition_variable cv, cv_done;
  std::deque<SegItem> q;
  std::vector<SegFile> files;
  std::vector<SwSegIndexEnt> index;      // every retained block, in write order
  int32_t next_file_id = 0;
  int64_t next_number = 0;                // file name number of the next new file
  int fd = -1;
  int fd_direct = 0;
  int64_t cur_bytes = 0;
  std::atomic<int64_t> durable{-1};
  std::atomic<int64_t> bytes_written{0}, blocks_written{0}, syncs{0}, deleted_files{0}, deleted_bytes{0},
      deleted_rows{0};
  // where the writer's time goes (ns): block writes, fdatasync, waiting for the copier; the copier's own
  std::atomic<int64_t> write_ns{0}, sync_ns{0}, cwait_ns{0}, copy_ns{0};
  std::atomic<int32_t> error{0};
  bool stop = false;
  std::thread th;
  uint8_t* bounce = nullptr;
  int64_t bounce_cap = 0;
  int64_t total_bytes = 0;
  uint8_t* commit_buf = nullptr;          // one SEG_COMMIT_BYTES record, aligned for O_DIRECT
  std::map<uint64_t, int64_t> sources;    // durable input offsets (max per key)
  // What the store holds in memory for the read path, parallel to `index` (null: not held):
  //  * the scan image of each recent block (bk_*: every page's header and leading columns, about a
  //    third of the block), up to blk_cap bytes, newest kept -- the blocks were written with
  //    O_DIRECT, so without it every listing over fresh blocks goes to the device;
  //  * each block's index trailer (tr_*), up to trailer_cap bytes.
  // Copies are made while the block is written (copier threads, from the caller's buffer, which
  // stays valid until the block is durable) and, for trailers, on recovery.  A copy dropped by a cap
  // or by retention is reclaimed only once every read lease that could have seen it has ended
  // (swss_lease_begin / swss_lease_end: epochs), then recycled for the next block copy.
  std::vector<uint8_t*> tr_ptr;
  std::vector<int64_t> tr_len;
  std::vector<uint8_t> tr_own;                       // 1: the trailer is its own allocation
  std::vector<uint8_t*> bk_ptr;
  std::vector<int64_t> bk_cap;                       // allocation bytes of the block copy
  int64_t trailer_cap = 16ll << 30, trailer_bytes = 0;   // own trailer copies
  int64_t blk_cap = 0, blk_bytes = 0;                // block copies (0: none kept)
  int64_t epoch = 0;
  std::multiset<int64_t> leases;                     // start epochs of the active read leases
  struct Retired { int64_t epoch; uint8_t* p; int64_t cap; };
  std::vector<Retired> grave;
  std::vector<std::pair<uint8_t*, int64_t>> pool;    // reclaimed block buffers (ptr, cap) for reuse
  std::thread copier;
  std::mutex cmu;
  std::condition_variable ccv;
  const std::vector<SegItem>* cjob = nullptr;        // the batch to copy
  struct Copy { uint8_t* blk; int64_t bcap; uint8_t* tr; int64_t tlen; bool own; };
  std::vector<Copy> cout;                            // one per item
  bool cdone = true;
  bool cstop = false;
};

static int64_t round_up_mb(int64_t x) { return (x + (1ll << 20) - 1) >> 20 << 20; }

// A block's index trailer: (offset in the block, bytes); (0, 0) when it has none.
static std::pair<int64_t, int64_t> trailer_span(const uint8_t* b, int64_t len) {
  SwSegBlockHdr h;
  memcpy(&h, b, sizeof(h));
  if (!(h.flags & SEG_FLAG_INDEX) || (int64_t)h.bytes > len) return {0, 0};
  const uint32_t toff = ((const uint32_t*)(b + 64))[h.n_pages];
  if (toff >= h.bytes) return {0, 0};
  return {(int64_t)toff, (int64_t)h.bytes - toff};
}

// Scan image of a block: what the page scans read (each page's header and leading columns --
// etype, level, date, assignment), pages back to back.  Layout: u32 n_pages, u32 0, u32 offset of
// page p's prefix in the image (n_pages of them, padded to 8 bytes), then the prefixes (8-aligned).
// The copier's work for one block, on several threads: a step's block is ~20 MB, its scan image
// ~7 MB and trailer ~4.5 MB, mostly into freshly allocated memory, and one thread copying that
// (page faults included) took longer than the disk took to write the block -- the writer waits for
// the copier before it publishes a batch, so the copier paced ingest (bench: 335-446M events/s with
// scan images against 510-535M without, same box).  SW_SEG_COPY_THREADS overrides (default 4).
static int seg_copy_threads() {
  static const int t = [] {
    const char* e = getenv("SW_SEG_COPY_THREADS");
    const int v = e ? atoi(e) : 4;
    return v < 1 ? 1 : (v > 16 ? 16 : v);
  }();
  return t;
}

template <typename F>
static void parallel_for(int64_t n, int threads, F&& f) {
  if (threads <= 1 || n < 2) {
    f(0, n);
    return;
  }
  const int64_t t = std::min<int64_t>(threads, n);
  const int64_t chunk = (n + t - 1) / t;
  std::vector<std::thread> th;
  for (int64_t i = 1; i < t; ++i) {
    const int64_t a = i * chunk, b = std::min<int64_t>(n, a + chunk);
    if (a < b) th.emplace_back([&f, a, b] { f(a, b); });
  }
  f(0, std::min<int64_t>(n, chunk));
  for (auto& x : th) x.join();
}

// Memory for a multi-MB copy: 2 MiB aligned and advised for transparent huge pages, so the copy
// takes a few faults instead of one per 4 KiB page.  Freed with free().
static uint8_t* big_alloc(int64_t n, int64_t* cap_out = nullptr) {
  const int64_t H = 2ll << 20;
  const int64_t cap = (n + H - 1) / H * H;
  uint8_t* p = (uint8_t*)aligned_alloc((size_t)H, (size_t)cap);
  if (p) (void)madvise(p, (size_t)cap, MADV_HUGEPAGE);
  if (cap_out) *cap_out = cap;
  return p;
}

static uint8_t* own_copy_mt(const uint8_t* src, int64_t n, int threads) {
  uint8_t* c = n >= (2ll << 20) ? big_alloc(n) : (uint8_t*)aligned_alloc(64, (size_t)((n + 63) / 64 * 64));
  if (!c) return nullptr;
  const int64_t unit = 1 << 20;
  parallel_for((n + unit - 1) / unit, threads, [&](int64_t a, int64_t b) {
    const int64_t lo = a * unit, hi = std::min<int64_t>(n, b * unit);
    if (hi > lo) memcpy(c + lo, src + lo, (size_t)(hi - lo));
  });
  return c;
}

static int64_t page_prefix(const uint8_t* pg) {
  SwSegPageHdr ph;
  memcpy(&ph, pg, sizeof(ph));
  const SwSegCol& ca = ph.cols[SEG_ASG];
  const int64_t need = (int64_t)ca.data_off + (int64_t)seg_col_bytes(ca.count, ca.bits, 0);
  return std::min<int64_t>(std::max<int64_t>(need, sizeof(SwSegPageHdr)), ph.bytes);
}

static int64_t scan_image_bytes(const uint8_t* b, int64_t len) {
  SwSegBlockHdr h;
  memcpy(&h, b, sizeof(h));
  if ((int64_t)h.bytes > len || !h.n_pages) return 0;
  const uint32_t* pt = (const uint32_t*)(b + 64);
  int64_t n = 8 + rd8(4u * h.n_pages);
  for (uint32_t p = 0; p < h.n_pages; ++p) n += (page_prefix(b + pt[p]) + 7) & ~int64_t(7);
  return n;
}

static void scan_image_build(const uint8_t* b, uint8_t* dst, int threads = 1) {
  SwSegBlockHdr h;
  memcpy(&h, b, sizeof(h));
  const uint32_t* pt = (const uint32_t*)(b + 64);
  uint32_t* hdr = (uint32_t*)dst;
  hdr[0] = h.n_pages;
  hdr[1] = 0;
  std::vector<int64_t> len(h.n_pages);
  int64_t o = 8 + rd8(4u * h.n_pages);
  for (uint32_t p = 0; p < h.n_pages; ++p) {
    len[p] = page_prefix(b + pt[p]);
    hdr[2 + p] = (uint32_t)o;
    o += (len[p] + 7) & ~int64_t(7);
  }
  parallel_for((int64_t)h.n_pages, threads, [&](int64_t a, int64_t e) {
    for (int64_t p = a; p < e; ++p) memcpy(dst + hdr[2 + p], b + pt[p], (size_t)len[p]);
  });
}

static uint8_t* own_copy(const uint8_t* src, int64_t n) {
  uint8_t* c = (uint8_t*)aligned_alloc(64, (size_t)((n + 63) / 64 * 64));
  if (c) memcpy(c, src, (size_t)n);
  return c;
}


// Caller holds s->mu.  Retire a copy (reclaimed once no lease can still see it).
static void retire(SegStore* s, uint8_t* p, int64_t cap) {
  if (p) s->grave.push_back({s->epoch, p, cap});
}

// Caller holds s->mu: enforce the caps (oldest copies first), then reclaim retired copies no
// active lease started before.
static void mem_trim(SegStore* s) {
  bool any = false;
  for (size_t i = 0; i < s->bk_ptr.size() && s->blk_bytes > s->blk_cap; ++i) {
    if (!s->bk_ptr[i]) continue;
    if (s->tr_ptr[i] && !s->tr_own[i]) {            // the trailer outlives the block copy
      uint8_t* t = own_copy(s->tr_ptr[i], s->tr_len[i]);
      s->tr_ptr[i] = t;
      s->tr_own[i] = t != nullptr;
      if (!t) s->tr_len[i] = 0;
      s->trailer_bytes += t ? s->tr_len[i] : 0;
    }
    retire(s, s->bk_ptr[i], s->bk_cap[i]);
    s->blk_bytes -= s->bk_cap[i];
    s->bk_ptr[i] = nullptr;
    s->bk_cap[i] = 0;
    any = true;
  }
  for (size_t i = 0; i < s->tr_ptr.size() && s->trailer_bytes > s->trailer_cap; ++i) {
    if (!s->tr_ptr[i] || !s->tr_own[i]) continue;
    retire(s, s->tr_ptr[i], 0);
    s->trailer_bytes -= s->tr_len[i];
    s->tr_ptr[i] = nullptr;
    s->tr_len[i] = 0;
    s->tr_own[i] = 0;
    any = true;
  }
  if (any) ++s->epoch;
  const int64_t oldest = s->leases.empty() ? INT64_MAX : *s->leases.begin();
  size_t k = 0;
  for (auto& g : s->grave) {
    if (g.epoch < oldest) {
      if (g.cap > 0 && s->pool.size() < 8) s->pool.push_back({g.p, g.cap});
      else free(g.p);
    } else {
      s->grave[k++] = g;
    }
  }
  s->grave.resize(k);
}

// Copier: this batch's block copies (when blocks are kept) or trailer copies.
static void seg_copier(SegStore* s) {
  while (true) {
    const std::vector<SegItem>* job;
    int64_t keep;
    {
      std::unique_lock<std::mutex> lk(s->cmu);
      s->ccv.wait(lk, [&] { return s->cstop || s->cjob != nullptr; });
      if (!s->cjob) return;
      job = s->cjob;
    }
    {
      std::lock_guard<std::mutex> g(s->mu);
      keep = s->blk_cap;
    }
    const auto c0 = std::chrono::steady_clock::now();
    std::vector<SegStore::Copy> out;
    out.reserve(job->size());
    for (const SegItem& it : *job) {
      const auto ts = trailer_span(it.ptr, it.len);
      SegStore::Copy c{nullptr, 0, nullptr, 0, false};
      const int64_t isz = keep > 0 ? scan_image_bytes(it.ptr, it.len) : 0;
      if (isz > 0 && isz <= keep) {
        uint8_t* p = nullptr;
        int64_t cap = 0;
        {
          std::lock_guard<std::mutex> g(s->mu);
          for (size_t k = 0; k < s->pool.size(); ++k)
            if (s->pool[k].second >= isz) {
              p = s->pool[k].first;
              cap = s->pool[k].second;
              s->pool.erase(s->pool.begin() + (long)k);
              break;
            }
        }
        if (!p) {
          if (isz >= (2ll << 20)) {
            p = big_alloc(isz, &cap);
          } else {
            cap = round_up_mb(isz);
            p = (uint8_t*)aligned_alloc(4096, (size_t)cap);
          }
        }
        if (p) {
          scan_image_build(it.ptr, p, seg_copy_threads());
          c.blk = p;
          c.bcap = cap;
        }
      }
      if (ts.second) {
        c.tr = own_copy_mt(it.ptr + ts.first, ts.second, seg_copy_threads());
        c.tlen = c.tr ? ts.second : 0;
        c.own = c.tr != nullptr;
      }
      out.push_back(c);
    }
    s->copy_ns += (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - c0).count();
    {
      std::lock_guard<std::mutex> g(s->cmu);
      s->cout.swap(out);
      s->cjob = nullptr;
      s->cdone = true;
    }
    s->ccv.notify_all();
  }
}

// Files are numbered in write order ("<rank>-<number>.sweg"): sequences restart with a new engine
// incarnation, so they cannot name files.
static std::string seg_name(const std::string& dir, int32_t rank, int64_t number) {
  char b[64];
  snprintf(b, sizeof(b), "/%d-%012lld.sweg", rank, (long long)number);
  return dir + b;
}

static int64_t round_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

static bool seg_open_file(SegStore* s, int64_t first) {
  const std::string p = seg_name(s->dir, s->rank, s->next_number++);
  int flags = O_WRONLY | O_CREAT | O_EXCL | O_APPEND;
  int fd = -1;
  s->fd_direct = 0;
  if (s->direct) {
    fd = open(p.c_str(), flags | O_DIRECT, 0644);
    if (fd >= 0) s->fd_direct = 1;
  }
  if (fd < 0) fd = open(p.c_str(), flags, 0644);
  if (fd < 0) return false;
  s->fd = fd;
  s->cur_bytes = 0;
  // reserve the file's extents up front, size unchanged (recovery and readers only ever see written
  // bytes): appends then land in allocated space instead of running the block allocator inside
  // each group commit -- the cost that made the first durable run on a fresh disk the slowest
  // (profiles/r3_cold).  Best effort: a filesystem without fallocate just allocates as it goes.
  (void)fallocate(fd, FALLOC_FL_KEEP_SIZE, 0, (off_t)s->rotate_bytes + (1 << 20));
  {
    std::lock_guard<std::mutex> g(s->mu);
    s->files.push_back({p, first, 0, s->next_file_id++});
  }
  int dfd = open(s->dir.c_str(), O_RDONLY);
  if (dfd >= 0) {
    fsync(dfd);
    close(dfd);
  }
  return true;
}

static void seg_close_file(SegStore* s) {
  if (s->fd >= 0) {
    (void)ftruncate(s->fd, (off_t)s->cur_bytes);   // give back the reservation past the last block
    fdatasync(s->fd);
    close(s->fd);
    s->fd = -1;
  }
}

static void seg_retention(SegStore* s) {
  if (s->retention_bytes <= 0 && s->retention_rows <= 0) return;
  std::lock_guard<std::mutex> g(s->mu);
  while (s->files.size() > 1 && ((s->retention_bytes > 0 && s->total_bytes > s->retention_bytes) ||
                                 (s->retention_rows > 0 && s->total_rows > s->retention_rows))) {
    const SegFile f = s->files.front();
    if (unlink(f.path.c_str()) != 0) break;
    s->files.erase(s->files.begin());
    size_t k = 0;
    for (size_t i = 0; i < s->index.size(); ++i) {
      if (s->index[i].file == f.id) {
        if (s->tr_ptr[i] && s->tr_own[i]) {
          retire(s, s->tr_ptr[i], 0);
          s->trailer_bytes -= s->tr_len[i];
        }
        if (s->bk_ptr[i]) {
          retire(s, s->bk_ptr[i], s->bk_cap[i]);
          s->blk_bytes -= s->bk_cap[i];
        }
        continue;
      }
      s->index[k] = s->index[i];
      s->tr_ptr[k] = s->tr_ptr[i];
      s->tr_len[k] = s->tr_len[i];
      s->tr_own[k] = s->tr_own[i];
      s->bk_ptr[k] = s->bk_ptr[i];
      s->bk_cap[k] = s->bk_cap[i];
      ++k;
    }
    s->index.resize(k);
    s->tr_ptr.resize(k);
    s->tr_len.resize(k);
    s->tr_own.resize(k);
    s->bk_ptr.resize(k);
    s->bk_cap.resize(k);
    ++s->epoch;
    s->total_bytes -= f.bytes;
    s->total_rows -= f.rows;
    s->deleted_rows += f.rows;
    s->deleted_files += 1;
    s->deleted_bytes += f.bytes;
  }
}

// Writes go out in chunks of at most 4 MiB: on the MI355X box's segment disk, O_DIRECT writes of
// 4 MiB sustain 10.3 GB/s against 8.5 at 16 MiB and 6.9 at 64 MiB (scripts/disk_probe.py,
// profiles/r5_disk), and a step's block is ~20 MB.  SW_SEG_WRITE_CHUNK_MB overrides (0: whole).
static int64_t seg_write_chunk() {
  static const int64_t c = [] {
    const char* e = getenv("SW_SEG_WRITE_CHUNK_MB");
    const int64_t mb = e ? atoll(e) : 4;
    return mb > 0 ? mb << 20 : (int64_t)1 << 62;
  }();
  return c;
}

static bool seg_write_all(int fd, const uint8_t* p, int64_t n) {
  const int64_t chunk = seg_write_chunk();
  while (n > 0) {
    ssize_t w = write(fd, p, (size_t)(n < chunk ? n : chunk));
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= w;
  }
  return true;
}

static void seg_writer(SegStore* s) {
  std::vector<SegItem> batch;
  std::vector<std::pair<uint64_t, int64_t>> done_src;
  std::vector<SwSegIndexEnt> pend;       // the batch's blocks, indexed once durable
  while (true) {
    {
      std::unique_lock<std::mutex> lk(s->mu);
      s->cv.wait(lk, [&] { return s->stop || !s->q.empty(); });
      if (s->q.empty() && s->stop) return;
      batch.assign(s->q.begin(), s->q.end());
      s->q.clear();
    }
    int64_t last = -1;
    done_src.clear();
    {
      // the copier takes the batch's trailers while the blocks go to the disk
      std::lock_guard<std::mutex> g(s->cmu);
      s->cjob = &batch;
      s->cdone = false;
    }
    s->ccv.notify_all();
    pend.clear();
    const auto w0 = std::chrono::steady_clock::now();
    for (const SegItem& it : batch) {
      SwSegBlockHdr h;
      memcpy(&h, it.ptr, sizeof(h));
      const bool commit = (h.flags & SEG_FLAG_COMMIT) != 0;
      const int64_t padded = round_up(it.len, SEG_ALIGN);
      const int64_t extra = commit ? SEG_COMMIT_BYTES : 0;
      if (s->fd < 0 || s->cur_bytes + padded + extra > s->rotate_bytes) {
        seg_close_file(s);
        seg_retention(s);
        if (!seg_open_file(s, h.first_seq)) {
          s->error = errno ? errno : -1;
          break;
        }
      }
      const bool aligned = ((uintptr_t)it.ptr % SEG_ALIGN) == 0;
      bool ok;
      if (s->fd_direct && aligned) {
        // the caller padded the buffer to a 4 KiB multiple (swss_append contract)
        ok = seg_write_all(s->fd, it.ptr, padded);
      } else {
        if (s->bounce_cap < padded) {
          free(s->bounce);
          s->bounce = (uint8_t*)aligned_alloc(SEG_ALIGN, (size_t)padded);
          s->bounce_cap = s->bounce ? padded : 0;
        }
        if (!s->bounce) {
          s->error = ENOMEM;
          break;
        }
        memcpy(s->bounce, it.ptr, (size_t)it.len);
        memset(s->bounce + it.len, 0, (size_t)(padded - it.len));
        ok = seg_write_all(s->fd, s->bounce, padded);
      }
      if (ok && commit) {
        // the commit record right behind the block, before the group's fdatasync
        if (!s->commit_buf) s->commit_buf = (uint8_t*)aligned_alloc(SEG_ALIGN, SEG_COMMIT_BYTES);
        if (!s->commit_buf) {
          s->error = ENOMEM;
          break;
        }
        memset(s->commit_buf, 0, SEG_COMMIT_BYTES);
        SwSegCommitHdr c;
        memset(&c, 0, sizeof(c));
        c.magic = SEG_COMMIT_MAGIC;
        c.version = SEG_VERSION;
        c.n_src = (uint16_t)it.src.size();
        c.bytes = 64 + 16ull * c.n_src;
        c.token = it.token;
        memcpy(s->commit_buf, &c, sizeof(c));
        for (size_t k = 0; k < it.src.size(); ++k) {
          memcpy(s->commit_buf + 64 + 16 * k, &it.src[k].first, 8);
          memcpy(s->commit_buf + 64 + 16 * k + 8, &it.src[k].second, 8);
        }
        c.checksum = commit_checksum(s->commit_buf, c.n_src);
        memcpy(s->commit_buf, &c, sizeof(c));
        ok = seg_write_all(s->fd, s->commit_buf, SEG_COMMIT_BYTES);
        done_src.insert(done_src.end(), it.src.begin(), it.src.end());
      }
      if (!ok) {
        s->error = errno ? errno : -1;
        break;
      }
      pend.push_back(index_entry(h, it.ptr, s->files.back().id, s->cur_bytes));
      {
        std::lock_guard<std::mutex> g(s->mu);
        s->files.back().bytes += padded + extra;
        s->total_bytes += padded + extra;
        s->files.back().rows += h.n_rows;
        s->total_rows += h.n_rows;
      }
      s->cur_bytes += padded + extra;
      s->bytes_written += padded + extra;
      s->blocks_written += 1;
      last = it.token;
    }
    const auto w1 = std::chrono::steady_clock::now();
    const bool synced = !s->error && !(s->fd >= 0 && fdatasync(s->fd) != 0);
    if (!s->error && !synced) s->error = errno ? errno : -1;
    const auto w2 = std::chrono::steady_clock::now();
    std::vector<SegStore::Copy> copies;
    {
      std::unique_lock<std::mutex> lk(s->cmu);
      s->ccv.wait(lk, [&] { return s->cdone; });
      copies.swap(s->cout);
    }
    const auto w3 = std::chrono::steady_clock::now();
    auto ns = [](std::chrono::steady_clock::duration d) {
      return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(d).count();
    };
    s->write_ns += ns(w1 - w0);
    s->sync_ns += ns(w2 - w1);
    s->cwait_ns += ns(w3 - w2);
    auto drop = [](const SegStore::Copy& c) {
      free(c.blk);
      if (c.own) free(c.tr);
    };
    if (s->error) {
      for (auto& c : copies) drop(c);
      s->cv_done.notify_all();
      continue;                         // tokens stop advancing; the caller sees the error
    }
    s->syncs += 1;
    {
      std::lock_guard<std::mutex> g(s->mu);
      for (size_t i = 0; i < pend.size(); ++i) {
        s->index.push_back(pend[i]);
        const SegStore::Copy c = i < copies.size() ? copies[i] : SegStore::Copy{nullptr, 0, nullptr, 0, false};
        s->tr_ptr.push_back(c.tr);
        s->tr_len.push_back(c.tlen);
        s->tr_own.push_back(c.own ? 1 : 0);
        s->bk_ptr.push_back(c.blk);
        s->bk_cap.push_back(c.bcap);
        if (c.own) s->trailer_bytes += c.tlen;
        s->blk_bytes += c.bcap;
      }
      for (size_t i = pend.size(); i < copies.size(); ++i) drop(copies[i]);
      mem_trim(s);
    }
    if (last >= 0) {
      std::lock_guard<std::mutex> g(s->mu);
      for (const auto& kv : done_src) {
        auto f = s->sources.find(kv.first);
        if (f == s->sources.end() || f->second < kv.second) s->sources[kv.first] = kv.second;
      }
      if (last > s->durable) s->durable = last;
    }
    s->cv_done.notify_all();
    // retention after every group commit, not only when a file starts: with retention by rows the
    // store then holds at most the limit plus the file being written (its rotate size is kept small
    // against the limit, swss_set_retention)
    seg_retention(s);
  }
}

// Scan one segment file: verify every block (and the commit record of a flagged block), truncate a
// torn tail.  Calls emit(offset, header, block) and on_commit(record) for each commit record.
template <typename F, typename G>
static int64_t seg_scan_file(const std::string& path, bool truncate, F emit, G on_commit) {
  int fd = open(path.c_str(), truncate ? O_RDWR : O_RDONLY);
  if (fd < 0) return -1;
  struct stat st;
  fstat(fd, &st);
  const int64_t size = st.st_size;
  int64_t off = 0;
  std::vector<uint8_t> buf;
  while (off + 64 <= size) {
    SwSegBlockHdr h;
    if (pread(fd, &h, sizeof(h), off) != (ssize_t)sizeof(h)) break;
    if (h.magic != SEG_MAGIC || h.version != SEG_VERSION || h.bytes < 64 || off + (int64_t)h.bytes > size) break;
    buf.resize(h.bytes);
    if (pread(fd, buf.data(), h.bytes, off) != (ssize_t)h.bytes) break;
    if (swseg_verify(buf.data(), (int64_t)h.bytes) != 0) break;
    int64_t next = off + round_up((int64_t)h.bytes, SEG_ALIGN);
    if (h.flags & SEG_FLAG_COMMIT) {
      uint8_t rec[SEG_COMMIT_BYTES];
      if (next + SEG_COMMIT_BYTES > size ||
          pread(fd, rec, SEG_COMMIT_BYTES, next) != (ssize_t)SEG_COMMIT_BYTES ||
          commit_valid(rec, SEG_COMMIT_BYTES) != 0)
        break;                            // the block's offsets never made it: the block goes too
      emit(off, h, buf.data());
      on_commit(rec);
      next += SEG_COMMIT_BYTES;
    } else {
      emit(off, h, buf.data());
    }
    off = next;
  }
  if (off > size) off = size;
  if (truncate && off < size) {
    if (ftruncate(fd, off) == 0) fdatasync(fd);
  } else if (truncate) {
    // an intact file may still hold the writer's extent reservation past EOF (fallocate KEEP_SIZE,
    // released only by seg_close_file): a crash would otherwise leave it allocated and uncounted by
    // retention.  Growing by a byte and truncating back frees every block past the scanned end.
    if (ftruncate(fd, off + 1) == 0 && ftruncate(fd, off) == 0) fdatasync(fd);
  }
  close(fd);
  return off;
}

extern "C" {

void* swss_open(const char* dir, int32_t rank, int64_t rotate_bytes, int64_t retention_bytes, int32_t direct) {
  SegStore* s = new SegStore();
  s->dir = dir;
  s->rank = rank;
  if (rotate_bytes > 0) s->rotate_bytes = rotate_bytes;
  s->retention_bytes = retention_bytes;
  s->direct = direct != 0;
  mkdir(dir, 0755);
  // recovery: existing files of this rank, oldest first, torn tails truncated
  std::vector<SegFile> found;
  if (DIR* d = opendir(dir)) {
    while (dirent* e = readdir(d)) {
      int r;
      long long first;
      char tail[8];
      if (sscanf(e->d_name, "%d-%lld.%7s", &r, &first, tail) == 3 && r == rank && strcmp(tail, "sweg") == 0) {
        found.push_back({s->dir + "/" + e->d_name, (int64_t)first, 0, 0});
        s->next_number = std::max<int64_t>(s->next_number, (int64_t)first + 1);
      }
    }
    closedir(d);
  }
  std::sort(found.begin(), found.end(), [](const SegFile& a, const SegFile& b) { return a.first_seq < b.first_seq; });
  for (auto& f : found) {
    f.id = s->next_file_id;
    f.bytes = seg_scan_file(
        f.path, true,
        [&](int64_t off, const SwSegBlockHdr& hd, const uint8_t* b) {
          s->index.push_back(index_entry(hd, b, f.id, off));
          f.rows += hd.n_rows;
          const auto ts = trailer_span(b, (int64_t)hd.bytes);
          uint8_t* t = ts.second ? own_copy(b + ts.first, ts.second) : nullptr;
          s->tr_ptr.push_back(t);
          s->tr_len.push_back(t ? ts.second : 0);
          s->tr_own.push_back(t ? 1 : 0);
          s->bk_ptr.push_back(nullptr);
          s->bk_cap.push_back(0);
          s->trailer_bytes += t ? ts.second : 0;
          mem_trim(s);
        },
        [&](const uint8_t* rec) {
          SwSegCommitHdr c;
          memcpy(&c, rec, sizeof(c));
          for (uint32_t k = 0; k < c.n_src; ++k) {
            uint64_t key;
            int64_t o;
            memcpy(&key, rec + 64 + 16 * k, 8);
            memcpy(&o, rec + 64 + 16 * k + 8, 8);
            auto it = s->sources.find(key);
            if (it == s->sources.end() || it->second < o) s->sources[key] = o;
          }
        });
    if (f.bytes < 0) continue;
    ++s->next_file_id;
    s->files.push_back(f);
    s->total_bytes += f.bytes;
    s->total_rows += f.rows;
  }
  s->copier = std::thread(seg_copier, s);
  s->th = std::thread(seg_writer, s);
  return s;
}

// Queue a sealed block for writing.  `ptr` must stay valid and unchanged until swss_durable() >=
// token; when it is 4 KiB aligned it should be readable up to the next 4 KiB multiple of len
// (O_DIRECT writes the padding straight from it; the caller zeroes it).  Tokens must increase.
int32_t swss_append(void* h, const uint8_t* ptr, int64_t len, int64_t token) {
  SegStore* s = (SegStore*)h;
  if (s->error) return s->error;
  {
    std::lock_guard<std::mutex> g(s->mu);
    s->q.push_back({ptr, len, token, {}});
  }
  s->cv.notify_one();
  return 0;
}

// Append a block sealed with SEG_FLAG_COMMIT plus its commit record: the n_src input offsets
// (keys[i] -> offs[i]) become durable with the block, atomically across a crash.
int32_t swss_append_commit(void* h, const uint8_t* ptr, int64_t len, int64_t token, const uint64_t* keys,
                           const int64_t* offs, int32_t n_src) {
  SegStore* s = (SegStore*)h;
  if (s->error) return s->error;
  if (n_src < 0 || n_src > SEG_MAX_SRC || len < 64) return -EINVAL;
  SwSegBlockHdr hd;
  memcpy(&hd, ptr, sizeof(hd));
  if (!(hd.flags & SEG_FLAG_COMMIT)) return -EINVAL;
  SegItem it{ptr, len, token, {}};
  for (int32_t k = 0; k < n_src; ++k) it.src.emplace_back(keys[k], offs[k]);
  {
    std::lock_guard<std::mutex> g(s->mu);
    s->q.push_back(std::move(it));
  }
  s->cv.notify_one();
  return 0;
}

// Durable input offsets (max per key, from commit records); returns the count, fills <= cap.
int64_t swss_sources(void* h, uint64_t* keys, int64_t* offs, int64_t cap) {
  SegStore* s = (SegStore*)h;
  std::lock_guard<std::mutex> g(s->mu);
  int64_t i = 0;
  for (const auto& kv : s->sources) {
    if (i < cap) {
      keys[i] = kv.first;
      offs[i] = kv.second;
    }
    ++i;
  }
  return (int64_t)s->sources.size();
}

int64_t swss_durable(void* h) { return ((SegStore*)h)->durable.load(); }

int32_t swss_error(void* h) { return ((SegStore*)h)->error.load(); }

// Wait until `token` is durable (or an error / timeout).  Returns 0 when durable.
int32_t swss_wait(void* h, int64_t token, int64_t timeout_ms) {
  SegStore* s = (SegStore*)h;
  std::unique_lock<std::mutex> lk(s->mu);
  const auto until = std::chrono::system_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (s->durable.load() < token && !s->error) {
    if (s->cv_done.wait_until(lk, until) == std::cv_status::timeout) break;
  }
  if (s->error) return s->error;
  return s->durable.load() >= token ? 0 : -1;
}

// Counters: bytes written, blocks written, syncs, deleted files, deleted bytes, retained bytes, files.
void swss_stats(void* h, int64_t* out) {
  SegStore* s = (SegStore*)h;
  std::lock_guard<std::mutex> g(s->mu);
  out[0] = s->bytes_written;
  out[1] = s->blocks_written;
  out[2] = s->syncs;
  out[3] = s->deleted_files;
  out[4] = s->deleted_bytes;
  out[5] = s->total_bytes;
  out[6] = (int64_t)s->files.size();
  out[7] = s->fd_direct;
  out[8] = s->write_ns;
  out[9] = s->sync_ns;
  out[10] = s->cwait_ns;
  out[11] = s->copy_ns;
  out[12] = s->total_rows;
  out[13] = s->deleted_rows;
  out[14] = s->retention_rows;
  out[15] = s->retention_bytes;
}

// Retention limits (<= 0: unchanged; rows -1: none) and the size at which a new file starts (<= 0:
// unchanged; from the next file on).  Applied after the next group commit (whole files, oldest first).
void swss_set_retention(void* h, int64_t bytes, int64_t rows, int64_t rotate_bytes) {
  SegStore* s = (SegStore*)h;
  std::lock_guard<std::mutex> g(s->mu);
  if (bytes > 0) s->retention_bytes = bytes;
  if (rows > 0) s->retention_rows = rows;
  if (rows < 0) s->retention_rows = 0;
  if (rotate_bytes > 0) s->rotate_bytes = rotate_bytes;
}

void swss_close(void* h) {
  SegStore* s = (SegStore*)h;
  {
    std::lock_guard<std::mutex> g(s->mu);
    s->stop = true;
  }
  s->cv.notify_all();
  if (s->th.joinable()) s->th.join();
  {
    std::lock_guard<std::mutex> g(s->cmu);
    s->cstop = true;
  }
  s->ccv.notify_all();
  if (s->copier.joinable()) s->copier.join();
  seg_close_file(s);
  for (size_t i = 0; i < s->tr_ptr.size(); ++i)
    if (s->tr_own[i]) free(s->tr_ptr[i]);
  for (uint8_t* p : s->bk_ptr) free(p);
  for (auto& g : s->grave) free(g.p);
  for (auto& q : s->pool) free(q.first);
  free(s->bounce);
  free(s->commit_buf);
  delete s;
}

// Index of every retained block, in write order (durable or queued-and-written).  Returns the
// entry count; fills at most cap entries.
int64_t swss_index(void* h, SwSegIndexEnt* out, int64_t cap) {
  SegStore* s = (SegStore*)h;
  std::lock_guard<std::mutex> g(s->mu);
  const int64_t n = (int64_t)s->index.size();
  for (int64_t i = 0; i < n && i < cap; ++i) out[i] = s->index[(size_t)i];
  return n;
}

// swss_index plus, per entry, the in-memory copies the store holds: the index trailer's address
// and length, and the block copy's address (0 when not held).  Addresses stay valid while the
// caller holds a read lease taken before this call (swss_lease_begin).
int64_t swss_index_tr(void* h, SwSegIndexEnt* out, uint64_t* taddr, int64_t* tlen, uint64_t* baddr, int64_t cap) {
  SegStore* s = (SegStore*)h;
  std::lock_guard<std::mutex> g(s->mu);
  const int64_t n = (int64_t)s->index.size();
  for (int64_t i = 0; i < n && i < cap; ++i) {
    out[i] = s->index[(size_t)i];
    taddr[i] = (uint64_t)(uintptr_t)s->tr_ptr[(size_t)i];
    tlen[i] = s->tr_len[(size_t)i];
    if (baddr) baddr[i] = (uint64_t)(uintptr_t)s->bk_ptr[(size_t)i];
  }
  return n;
}

// Read leases: addresses from swss_index_tr stay valid from swss_lease_begin (returns the lease)
// to swss_lease_end(lease).
int64_t swss_lease_begin(void* h) {
  SegStore* s = (SegStore*)h;
  std::lock_guard<std::mutex> g(s->mu);
  s->leases.insert(s->epoch);
  return s->epoch;
}

void swss_lease_end(void* h, int64_t lease) {
  SegStore* s = (SegStore*)h;
  std::lock_guard<std::mutex> g(s->mu);
  auto it = s->leases.find(lease);
  if (it != s->leases.end()) s->leases.erase(it);
  mem_trim(s);
}

// Memory caps: bytes of own trailer copies and of block copies to hold (-1: leave as is).
// Returns the trailer bytes held; *blk_held (if non-null) the block-copy bytes.
int64_t swss_mem_caps(void* h, int64_t trailer_cap, int64_t blk_cap, int64_t* blk_held) {
  SegStore* s = (SegStore*)h;
  std::lock_guard<std::mutex> g(s->mu);
  if (trailer_cap >= 0) s->trailer_cap = trailer_cap;
  if (blk_cap >= 0) s->blk_cap = blk_cap;
  mem_trim(s);
  if (blk_held) *blk_held = s->blk_bytes;
  return s->trailer_bytes;
}

// Path of segment file `id` (SwSegIndexEnt::file) into buf; returns its length, -1 if deleted.
int32_t swss_file(void* h, int32_t id, char* buf, int32_t cap) {
  SegStore* s = (SegStore*)h;
  std::lock_guard<std::mutex> g(s->mu);
  for (const SegFile& f : s->files)
    if (f.id == id) return snprintf(buf, (size_t)cap, "%s", f.path.c_str());
  return -1;
}

// Summary of a block already in memory (min / max event date bounds) for index entries.
void swseg_dates(const uint8_t* b, int64_t* lo, int64_t* hi) { block_dates(b, lo, hi); }

}  // extern "C"

// ------------------------------------------------------------------------- connector selection
// An outbound connector's kept rows of one durable block, straight to their JSON documents: per page,
// each row's event type and assignment are read from the packed columns (no full decode) and tested
// against `etmask` (bit = event type) and `keep` (per assignment index; indexes >= n_keep take
// keep_default); the kept rows alone are decoded (decode_rows, strings included) and written by
// swjson_rows (csrc/native/swrowjson.cpp).  Pages run on `threads` workers, worker w writing its pages'
// documents / topics into slice w of `scratch` / `tscratch` (equal slices; reused caller memory, no
// allocation per call), then the slices are concatenated into out / tout (offsets out_off / tout_off,
// block order).  counts = {kept rows, block rows, missing entries}.  Returns the document bytes,
// -need when a buffer is too small (need = the scratch or output bytes to pass next time), -(1 << 40)
// - 1 - k when kept row k must take the caller's Python path (an API-added JSON row), -(1 << 41) on a
// page that fails to decode, or -(1 << 42) when kept rows' dictionary entries are missing
// (miss[0 .. counts[2]): an assignment index a >= 0 as a, a name id m as -1 - m; the caller resolves
// them and calls again).  The block must be verified by the caller.
extern "C" int64_t swjson_rows(const int64_t* rows, int64_t n, const uint8_t* etype, const uint8_t* level,
                               const int64_t* date, const int32_t* asg, const uint16_t* name, const double* v0,
                               const double* v1, const double* v2, const uint8_t* flags, const uint8_t* heap,
                               const int64_t* soff, int64_t boot, int64_t first_seq, int64_t world, int64_t rank,
                               int64_t recv_ms, int64_t row0, const uint8_t* a_heap, const int64_t* a_off,
                               const uint8_t* a_present, int64_t n_asg, const uint8_t* n_heap, const int64_t* n_off,
                               const uint8_t* n_present, int64_t n_names, const uint8_t* r_heap, const int64_t* r_off,
                               const uint8_t* r_present, const uint8_t* tpl, int64_t tpl_len, uint8_t* out,
                               int64_t cap, int64_t* out_off, uint8_t* tout, int64_t tcap, int64_t* tout_off,
                               const int64_t* block_rows);

extern "C" int64_t swjson_select_block(const uint8_t* b, int32_t etmask, const uint8_t* keep, int64_t n_keep,
                                       int32_t keep_default, const uint8_t* a_known, int64_t n_asg,
                                       const uint8_t* a_heap, const int64_t* a_off, const uint8_t* a_present,
                                       const uint8_t* n_heap, const int64_t* n_off, const uint8_t* n_present,
                                       int64_t n_names, const uint8_t* r_heap, const int64_t* r_off,
                                       const uint8_t* r_present, const uint8_t* tpl, int64_t tpl_len, int32_t threads,
                                       uint8_t* scratch, int64_t scap, uint8_t* tscratch, int64_t tscap, uint8_t* out,
                                       int64_t cap, int64_t* out_off, uint8_t* tout, int64_t tcap, int64_t* tout_off,
                                       int64_t* counts, int64_t* miss, int64_t miss_cap) {
  SwSegBlockHdr h;
  memcpy(&h, b, sizeof(h));
  const uint32_t* pt = (const uint32_t*)(b + 64);
  const int64_t np = h.n_pages;
  int T = threads > 0 ? threads : 1;
  if (T > 32) T = 32;
  if ((int64_t)T > np) T = (int)(np > 0 ? np : 1);
  const int64_t wcap = scap / T, wtcap = tpl ? tscap / T : 0;
  struct Worker {
    std::vector<int64_t> doff, toff;               // per kept row, relative to the worker's slice
    int64_t bytes = 0, tbytes = 0;                 // written (or needed, when past the slice)
    int64_t bad = -1;                              // kept row (worker-relative) for the Python path
    bool fail = false;
    std::vector<int64_t> miss;
  };
  std::vector<Worker> ws((size_t)T);
  auto work = [&](int w) {
    Worker& W = ws[(size_t)w];
    const int64_t p0 = np * w / T, p1 = np * (w + 1) / T;
    uint8_t* js = scratch + (int64_t)w * wcap;
    uint8_t* ts = tpl ? tscratch + (int64_t)w * wtcap : nullptr;
    std::vector<int32_t> sel;
    std::vector<int64_t> brow, idx, soff, jo, to;
    std::vector<uint8_t> et, lv, fl, heap;
    std::vector<int64_t> dt;
    std::vector<int32_t> as;
    std::vector<uint16_t> nm;
    std::vector<double> a0, a1, a2;
    W.doff.push_back(0);
    W.toff.push_back(0);
    for (int64_t p = p0; p < p1; ++p) {
      const uint8_t* pg = b + pt[p];
      SwSegPageHdr ph;
      memcpy(&ph, pg, sizeof(ph));
      sel.clear();
      for (uint32_t j = 0; j < ph.n_rows; ++j) {
        const uint32_t e = (uint32_t)seg_unord(col_int(pg, ph.cols[SEG_ETYPE], j));
        if (e > 31 || !((etmask >> e) & 1)) continue;
        const int64_t a = seg_unord(col_int(pg, ph.cols[SEG_ASG], j));
        if (a >= 0 && (a >= n_asg || !a_known[a])) {
          if (W.miss.empty() || W.miss.back() != a) W.miss.push_back(a);
          continue;
        }
        const bool k = (a >= 0 && a < n_keep) ? keep[a] != 0 : keep_default != 0;
        if (k) sel.push_back((int32_t)j);
      }
      const int64_t k = (int64_t)sel.size();
      if (!k || !W.miss.empty()) continue;
      if ((int64_t)et.size() < k) {
        et.resize(k); lv.resize(k); fl.resize(k); dt.resize(k); as.resize(k); nm.resize(k);
        a0.resize(k); a1.resize(k); a2.resize(k); brow.resize(k); idx.resize(k);
        jo.resize(k + 1); to.resize(k + 1); soff.resize(3 * (size_t)k + 1);
      }
      const size_t hb = (size_t)ph.heap_bytes + (size_t)k * (SEG_ALT_PFX_MAX + 16 + 8) + 8;
      if (heap.size() < hb) heap.resize(hb);
      soff[0] = 0;
      int64_t so = 0;
      if (decode_rows(pg, sel.data(), k, et.data(), lv.data(), dt.data(), as.data(), nm.data(), a0.data(), a1.data(),
                      a2.data(), fl.data(), heap.data(), (int64_t)heap.size(), &so, soff.data()) != k) {
        W.fail = true;
        return;
      }
      for (int64_t i = 0; i < k; ++i)
        if (nm[i] != 0xffff && ((int64_t)nm[i] >= n_names || !n_present[nm[i]])) W.miss.push_back(-1 - (int64_t)nm[i]);
      if (!W.miss.empty()) continue;
      for (int64_t i = 0; i < k; ++i) { brow[i] = p * SEG_PAGE_ROWS + sel[i]; idx[i] = i; }
      const int64_t jroom = W.bytes < wcap ? wcap - W.bytes : 0, troom = W.tbytes < wtcap ? wtcap - W.tbytes : 0;
      const int64_t r = swjson_rows(idx.data(), k, et.data(), lv.data(), dt.data(), as.data(), nm.data(), a0.data(),
                                    a1.data(), a2.data(), fl.data(), heap.data(), soff.data(), h.boot, h.first_seq,
                                    h.world, h.rank, h.recv_ms, 0, a_heap, a_off, a_present, n_asg, n_heap, n_off,
                                    n_present, n_names, r_heap, r_off, r_present, tpl, tpl_len,
                                    js + (W.bytes < wcap ? W.bytes : 0), jroom, jo.data(),
                                    ts ? ts + (W.tbytes < wtcap ? W.tbytes : 0) : nullptr, troom, to.data(), brow.data());
      if (r <= -1 && -r - 1 < k) {                 // a row for the Python path
        W.bad = (int64_t)W.doff.size() - 1 + (-r - 1);
        return;
      }
      // written, or (a slice too small) only measured: jo / to hold the sizes either way
      for (int64_t i = 0; i < k; ++i) {
        W.doff.push_back(W.bytes + jo[i + 1]);
        W.toff.push_back(W.tbytes + (tpl ? to[i + 1] : 0));
      }
      W.bytes += jo[k];
      W.tbytes += tpl ? to[k] : 0;
    }
  };
  if (T <= 1) work(0);
  else {
    std::vector<std::thread> th;
    for (int w = 0; w < T; ++w) th.emplace_back(work, w);
    for (auto& x : th) x.join();
  }
  counts[0] = counts[2] = 0;
  counts[1] = h.n_rows;
  for (const Worker& W : ws)
    if (W.fail) return -(int64_t(1) << 41);
  {
    std::vector<int64_t> ms;
    for (const Worker& W : ws) ms.insert(ms.end(), W.miss.begin(), W.miss.end());
    if (!ms.empty()) {
      std::sort(ms.begin(), ms.end());
      ms.erase(std::unique(ms.begin(), ms.end()), ms.end());
      const int64_t m = std::min<int64_t>((int64_t)ms.size(), miss_cap);
      for (int64_t i = 0; i < m; ++i) miss[i] = ms[(size_t)i];
      counts[2] = m;
      return -(int64_t(1) << 42);
    }
  }
  int64_t nk = 0, jb = 0, tb = 0, wmax = 0, twmax = 0;
  for (const Worker& W : ws) {
    if (W.bad >= 0) return -(int64_t(1) << 40) - 1 - (nk + W.bad);
    nk += (int64_t)W.doff.size() - 1;
    jb += W.bytes;
    tb += W.tbytes;
    wmax = std::max(wmax, W.bytes);
    twmax = std::max(twmax, W.tbytes);
  }
  counts[0] = nk;
  if (wmax > wcap || twmax > wtcap) {            // a worker's slice was too small: scratch for next time
    const int64_t need = std::max(wmax * T + 4096 * T, tpl ? twmax * T + 4096 * T : 0);
    return -std::max<int64_t>(need, 1);
  }
  if (jb > cap || (tout && tb > tcap)) return -std::max<int64_t>(jb, tb);
  int64_t w = 0, wj = 0, wt = 0;
  out_off[0] = 0;
  if (tout) tout_off[0] = 0;
  for (int x = 0; x < T; ++x) {
    const Worker& W = ws[(size_t)x];
    const int64_t k = (int64_t)W.doff.size() - 1;
    memcpy(out + wj, scratch + (int64_t)x * wcap, (size_t)W.bytes);
    if (tout && tpl) memcpy(tout + wt, tscratch + (int64_t)x * wtcap, (size_t)W.tbytes);
    for (int64_t i = 0; i < k; ++i) {
      out_off[w + i + 1] = wj + W.doff[(size_t)i + 1];
      if (tout) tout_off[w + i + 1] = wt + W.toff[(size_t)i + 1];
    }
    w += k;
    wj += W.bytes;
    wt += W.tbytes;
  }
  return wj;
}

// ------------------------------------------------------------------------- threshold rules
// Rows of a (verified) block whose measurement crosses a bound: event type Measurement, name id set
// in `name_mask` (n_mask bytes), value < lo (has_lo) or > hi (has_hi) -- services/rule_processing.py
// ThresholdRuleProcessor over the packed columns: only the event type, flags, name and value of the
// measurement rows are unpacked, nothing else of the block is decoded.  Pages on `threads` workers.
// Writes (row, assignment, value) in block order, at most cap; returns the number found (may exceed
// cap: call again with room for it), -1 on a page that does not decode.
extern "C" int64_t swseg_threshold_rows(const uint8_t* b, const uint8_t* name_mask, int64_t n_mask, double lo,
                                        double hi, int32_t has_lo, int32_t has_hi, int32_t threads, int64_t* out_rows,
                                        int32_t* out_asg, double* out_val, int64_t cap) {
  SwSegBlockHdr h;
  memcpy(&h, b, sizeof(h));
  const uint32_t* pt = (const uint32_t*)(b + 64);
  const int64_t np = h.n_pages;
  int T = threads > 0 ? threads : 1;
  if (T > 32) T = 32;
  if ((int64_t)T > np) T = (int)(np > 0 ? np : 1);
  struct Hit { int64_t row; int32_t asg; double v; };
  std::vector<std::vector<Hit>> hits((size_t)T);
  auto work = [&](int w) {
    std::vector<Hit>& out = hits[(size_t)w];
    for (int64_t p = np * w / T; p < np * (w + 1) / T; ++p) {
      const uint8_t* pg = b + pt[p];
      SwSegPageHdr ph;
      memcpy(&ph, pg, sizeof(ph));
      const int mode = ph.alt_mode;
      const SwSegCol& cv = ph.cols[SEG_MXV];
      const uint8_t* vw = pg + cv.data_off;
      const uint8_t* xi = vw + 8 * seg_col_words(cv.count, cv.bits);
      const uint8_t* xr = xi + ((2u * cv.n_exc + 7u) & ~7u);
      uint32_t xc = 0, cn = 0, cm = 0;
      for (uint32_t j = 0; j < ph.n_rows; ++j) {
        const uint8_t et = (uint8_t)seg_unord(col_int(pg, ph.cols[SEG_ETYPE], j));
        const uint32_t f = (uint32_t)seg_unord(col_int(pg, ph.cols[SEG_FLAGS], j));
        const bool hn = seg_member(SEG_NAME, et, f, mode), hv = seg_member(SEG_MXV, et, f, mode);
        if (et == 0 && hn && hv) {
          const int64_t nm = seg_unord(col_int(pg, ph.cols[SEG_NAME], cn));
          if (nm >= 0 && nm < n_mask && name_mask[nm]) {
            double v;
            for (; xc < cv.n_exc; ++xc) {
              uint16_t x;
              memcpy(&x, xi + 2 * xc, 2);
              if (x >= cm) break;
            }
            uint16_t x = 0xffff;
            if (xc < cv.n_exc) memcpy(&x, xi + 2 * xc, 2);
            if (xc < cv.n_exc && x == cm) {
              uint64_t raw;
              memcpy(&raw, xr + 8 * xc, 8);
              v = sw_bits_f64(raw);
            } else {
              v = seg_dec_value(seg_unord(cv.base + unpack(vw, cm, cv.bits)), cv.exp);
            }
            if ((has_lo && v < lo) || (has_hi && v > hi))
              out.push_back({p * SEG_PAGE_ROWS + j, (int32_t)seg_unord(col_int(pg, ph.cols[SEG_ASG], j)), v});
          }
        }
        cn += hn;
        cm += hv;
      }
    }
  };
  if (T <= 1) work(0);
  else {
    std::vector<std::thread> th;
    for (int w = 0; w < T; ++w) th.emplace_back(work, w);
    for (auto& x : th) x.join();
  }
  int64_t k = 0;
  for (const auto& v : hits)
    for (const Hit& x : v) {
      if (k < cap) { out_rows[k] = x.row; out_asg[k] = x.asg; out_val[k] = x.v; }
      ++k;
    }
  return k;
}
