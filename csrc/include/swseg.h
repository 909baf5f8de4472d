// Durable columnar event blocks: the on-disk (and enriched-topic) form of one engine step's
// persisted events.  Encoded on the MI355X right after the step (csrc/hip/swgpu.hip k_seg_encode),
// copied to the host already compressed, written to segment files by the native segment store
// (csrc/native/swseg.cpp) and decoded there for queries and recovery.  The C++ encoder in
// swseg.cpp produces the same bytes (tests/test_segments.py checks GPU == CPU bit for bit).
//
// Reference: the reference persists every event before it is enriched (DeviceEventBuffer.java:99-135
// bulk-writes Mongo documents; KafkaEventPersistenceTriggers.java:72-85 forwards what was stored).
// Here a step's events are one block: no per-event document, ids implicit in the row position.
//
// Block layout (little endian, every region 8-byte aligned):
//   SwSegBlockHdr (64 B)  |  u32 page_off[n_pages + 1] (offsets from the block start; padded to 8)
//   | pages...
// Page = up to SEG_PAGE_ROWS consecutive rows:
//   SwSegPageHdr (16 B + SEG_NCOL x 24 B column descriptors)  |  column data, in column order.
// Column data = ceil(count * bits / 64) u64 words of bit-packed values (value i at bit i * bits,
// LSB first, straddling into the next word), then for double columns the exceptions:
// u16 index[n_exc] (padded to 8 B) and the raw u64 bits of each exception value.
//
// Integer columns are frame-of-reference coded: x -> u = x ^ 2^63 (order-preserving unsigned),
// packed = u - min(u).  Double columns are decimal coded (the "ALP" idea: sensor values and GPS
// coordinates carry a few decimal digits): a page picks one exponent e, a value is stored as the
// integer q = rint(v * 10^e) when q / 10^e reproduces v bit for bit, otherwise as an exception
// (raw bits; its packed slot holds 0).  Page checksums (order-sensitive xor of mixed words) catch
// torn or corrupted writes on recovery.
#pragma once
#include <stdint.h>
#include "swtypes.h"

#define SEG_MAGIC 0x42455753u      // "SWEB"
#define SEG_VERSION 1
#define SEG_PAGE_ROWS 1024
#define SEG_MAXE 15
#define SEG_EXC_NONE 0xff

enum SwSegColumn {
  SEG_ETYPE = 0,   // all rows
  SEG_LEVEL,       // alerts
  SEG_DATE,        // all rows (event date, ms)
  SEG_ASG,         // all rows (assignment index; context via the block's dictionary deltas)
  SEG_NAME,        // rows that are not locations (interned measurement name / alert type id)
  SEG_MXV,         // measurements: value (decimal double)
  SEG_LAT,         // locations: latitude
  SEG_LON,         // locations: longitude
  SEG_ELEV,        // locations: elevation
  SEG_HASALT,      // all rows: 1 when the event carries an alternate id
  SEG_ALT,         // rows with an alternate id: its 64-bit hash
  SEG_NCOL
};

typedef struct __attribute__((aligned(8))) SwSegBlockHdr {
  uint32_t magic;
  uint16_t version;
  uint16_t flags;
  uint32_t n_rows;
  uint32_t n_pages;
  uint64_t bytes;        // block bytes without any tail padding
  int64_t first_seq;     // store sequence of row 0: event id = (first_seq + row) * world + rank
  int64_t recv_ms;       // receive time of the batch (every row)
  int64_t boot;          // engine incarnation: (boot, rank, sequence) identifies an event; ids and
                         // dictionary entries (assignment / name indices) are scoped by it
  int32_t rank;
  int32_t world;
  uint64_t checksum;     // header (checksum = 0) + page table
} SwSegBlockHdr;

// Commit record (exactly-once ingest): a block sealed with SEG_FLAG_COMMIT is followed, in the same
// group write, by one 4 KiB record naming the input offsets the block completes (key = 64-bit hash
// of the source, e.g. topic + partition; offset = next input offset).  Recovery drops a flagged
// block whose record is missing or torn, so a block is on disk exactly when its offsets are.
#define SEG_COMMIT_MAGIC 0x43455753u   // "SWEC"
#define SEG_FLAG_COMMIT 1
#define SEG_COMMIT_BYTES 4096
#define SEG_MAX_SRC 252

typedef struct __attribute__((aligned(8))) SwSegCommitHdr {
  uint32_t magic;
  uint16_t version;
  uint16_t n_src;
  uint64_t bytes;        // 64 + 16 * n_src
  int64_t token;
  uint64_t pad[4];
  uint64_t checksum;     // header (checksum = 0) + entries
} SwSegCommitHdr;        // then n_src x {uint64 key, int64 offset}

typedef struct __attribute__((aligned(8))) SwSegCol {
  uint64_t base;         // FOR base (min of the order-preserving unsigned values)
  uint32_t data_off;     // from the page start
  uint16_t count;        // values in the column (rows the column applies to)
  uint16_t n_exc;        // exceptions (double columns)
  uint8_t bits;          // packed width, 0..64
  int8_t exp;            // decimal exponent (double columns), -1 for integer columns
  uint16_t pad0;
  uint32_t pad1;
} SwSegCol;

typedef struct __attribute__((aligned(8))) SwSegPageHdr {
  uint32_t n_rows;
  uint32_t bytes;        // page bytes (multiple of 8)
  uint64_t checksum;     // every other u64 word of the page
  SwSegCol cols[SEG_NCOL];
} SwSegPageHdr;

#define SEG_PAGE_HDR ((uint32_t)sizeof(SwSegPageHdr))

SW_HD bool seg_is_double(int c) { return c >= SEG_MXV && c <= SEG_ELEV; }

// Does column c apply to a row of type `et` (alt: the row's alternate-id hash)?
SW_HD bool seg_member(int c, uint8_t et, uint64_t alt) {
  switch (c) {
    case SEG_LEVEL: return et == SW_EV_ALERT;
    case SEG_NAME: return et != SW_EV_LOCATION;
    case SEG_MXV: return et == SW_EV_MEASUREMENT;
    case SEG_LAT: case SEG_LON: case SEG_ELEV: return et == SW_EV_LOCATION;
    case SEG_ALT: return alt != 0;
    default: return true;
  }
}

SW_HD uint64_t seg_ord(int64_t x) { return (uint64_t)x ^ 0x8000000000000000ULL; }
SW_HD int64_t seg_unord(uint64_t u) { return (int64_t)(u ^ 0x8000000000000000ULL); }

SW_HD int seg_bitwidth(uint64_t range) {
  int b = 0;
  while (b < 64 && (range >> b) != 0) ++b;
  return b;
}

SW_HD uint32_t seg_col_words(uint32_t count, int bits) {
  return (uint32_t)(((uint64_t)count * (uint64_t)bits + 63) >> 6);
}

// bytes of a column's data region (packed words + exceptions)
SW_HD uint32_t seg_col_bytes(uint32_t count, int bits, uint32_t n_exc) {
  uint32_t b = 8u * seg_col_words(count, bits);
  if (n_exc) b += ((2u * n_exc + 7u) & ~7u) + 8u * n_exc;
  return b;
}

SW_HD double seg_p10(int e) {
  // exact powers of ten (all <= 1e15 are exactly representable)
  double p = 1.0;
  for (int i = 0; i < e; ++i) p *= 10.0;
  return p;
}

SW_HD bool seg_same_bits(double a, double b) { return sw_f64_bits(a) == sw_f64_bits(b); }

// Does q / 10^e reproduce v exactly at exponent e?  On success *q holds the integer.
SW_HD bool seg_dec_at(double v, int e, int64_t* q) {
  const double p = seg_p10(e);
  const double s = v * p;
  if (!(s > -4503599627370496.0 && s < 4503599627370496.0)) return false;   // |q| < 2^52 (NaN fails)
#if defined(__HIP_DEVICE_COMPILE__)
  const double r = rint(s);
#else
  const double r = __builtin_rint(s);
#endif
  const int64_t qi = (int64_t)r;
  if (!seg_same_bits((double)qi / p, v)) return false;
  *q = qi;
  return true;
}

// Smallest exponent at which v is decimal-exact, SEG_EXC_NONE if none.
SW_HD int seg_dec_exp(double v) {
  int64_t q;
  for (int e = 0; e <= SEG_MAXE; ++e)
    if (seg_dec_at(v, e, &q)) return e;
  return SEG_EXC_NONE;
}

SW_HD double seg_dec_value(int64_t q, int e) { return (double)q / seg_p10(e); }

// Checksum contribution of the u64 word at index i of a page (i counted from the page start).
SW_HD uint64_t seg_mix_word(uint64_t w, uint64_t i) { return sw_mix64(w + (i + 1) * 0x9E3779B97F4A7C15ULL); }
