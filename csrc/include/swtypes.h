// Shared record layouts and hash functions for the SiteWhere-AMD data plane.
//
// Compiled both by hipcc (device kernels, csrc/hip/*.hip) and by g++ (host
// runtime, csrc/native/*.cpp).  Every layout here is mirrored by a numpy
// dtype in sitewhere_amd/models/columnar.py; tests/test_columnar.py pins the
// offsets so the two never drift.
//
// Design notes (MI355X-first, see docs/ARCHITECTURE.md):
//  * Device tokens (reference: hardwareId / device token strings, e.g.
//    sitewhere-communication/src/main/proto/sitewhere.proto:14-60) are reduced
//    to a 128-bit fingerprint at decode time.  The registry, the shuffle and the
//    state tables only ever carry the fingerprint, so every hot record is fixed
//    width (80 B) and no variable-length token bytes cross xGMI.
//  * Records are 16-B aligned so a wave moves them with dwordx4 loads.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define SW_HD __host__ __device__ __forceinline__
#else
#define SW_HD static inline
#endif

// ---------------------------------------------------------------- event types
// Matches GDeviceEventType (sitewhere-grpc-event-management/.../device-event-model.proto).
enum SwEventType : uint8_t {
  SW_EV_MEASUREMENT = 0,
  SW_EV_LOCATION = 1,
  SW_EV_ALERT = 2,
  SW_EV_COMMAND_INVOCATION = 3,
  SW_EV_COMMAND_RESPONSE = 4,
  SW_EV_STATE_CHANGE = 5,
  // control messages (not persisted by the GPU path; routed to the host)
  SW_EV_REGISTRATION = 16,
  SW_EV_ACK = 17,
  SW_EV_STREAM_CREATE = 18,
  SW_EV_STREAM_DATA = 19,
  SW_EV_STREAM_DATA_REQUEST = 20,
  // an event whose alternate id, alert message or metadata span does not fit the engine's 16-bit
  // string lengths: handed to the host like a control message, which forwards the payload to the
  // per-event path (decoded-events topic) -- stored losslessly there instead of truncated here
  SW_EV_OVERSIZE = 21,
  SW_EV_DECODE_ERROR = 255,
};

// Processing status of an event after inbound validation
// (reference: InboundPayloadProcessingLogic.java:119-218).
enum SwStatus : uint8_t {
  SW_ST_OK = 0,
  SW_ST_UNREGISTERED = 1,   // no device with this token -> unregistered topic
  SW_ST_UNASSIGNED = 2,     // device has no active assignment -> unregistered topic
  SW_ST_DUPLICATE = 3,      // alternate id seen before (AlternateIdDeduplicator)
  SW_ST_DECODE_ERROR = 4,   // failed-decode topic
  SW_ST_CONTROL = 5,        // registration / ack / stream: host path
  SW_ST_RECHECK = 6,        // alternate id new to the dedup window but maybe stored before (the
                            // store-backed filter holds it): host path, checked against the store
};

// record flags
#define SW_F_HAS_UPDATE_STATE 0x1
#define SW_F_UPDATE_STATE 0x2
#define SW_F_HAS_DATE 0x4
#define SW_F_HAS_ELEVATION 0x8
#define SW_F_SYS_ALERT 0x10     // (API-added rows only) alert of source System with its own message
#define SW_F_JSON 0x20          // (API-added rows only) type-specific fields as JSON in the metadata span
#define SW_F_SETTLED 0x40       // store-backed dedup settled on the host (a recheck the store does not hold)

// Decoded event record, 80 bytes.  Output of the decoder, unit of the
// multi-GPU all-to-all, input of validation.
typedef struct __attribute__((aligned(16))) SwEventRec {
  uint64_t fp_lo;       // 0  device token fingerprint (low)
  uint64_t fp_hi;       // 8  device token fingerprint (high)
  int64_t event_date;   // 16 epoch ms
  uint64_t name_hash;   // 24 measurement name / alert type hash (0 if none)
  double v0;            // 32 measurement value | latitude
  double v1;            // 40 longitude
  double v2;            // 48 elevation
  uint64_t alt_hash;    // 56 alternate-id hash for dedup (0 = none)
  uint32_t aux_off;     // 64 offset of name/type string in source raw batch (control: msg start)
  uint32_t aux2_off;    // 68 offset of alert message string (control: msg end)
  uint16_t aux_len;     // 72
  uint16_t aux2_len;    // 74
  uint8_t etype;        // 76 SwEventType
  uint8_t flags;        // 77 SW_F_*
  uint8_t src_rank;     // 78 rank whose raw batch holds the aux bytes
  uint8_t level;        // 79 alert level (GAlertLevel)
} SwEventRec;

// Where the strings of a decoded event sit in its raw batch (written by the decoder beside each
// record, read by the durable-block encoder, csrc/include/swseg.h): the alternate id, the span of
// the body's metadata entries (first entry's tag to the last entry's end, wire bytes), and which
// measurement of a multi-measurement payload the record is.  The alert message is the record's
// aux2 string.  Offsets are absolute in the batch; lengths fit 16 bits (SW_EV_OVERSIZE otherwise).
// Reference fields: alternateId and metadata of every event (MongoDeviceEvent.java:64-82).
typedef struct __attribute__((aligned(16))) SwStrRef {
  uint32_t alt_off;
  uint32_t meta_off;
  uint16_t alt_len;
  uint16_t meta_len;
  uint16_t k;           // measurement index within its payload
  uint8_t has;          // SW_SR_* bits
  uint8_t pad;
} SwStrRef;
#define SW_SR_ALT 0x1     // the body carries an alternate id
#define SW_SR_META 0x2    // the body carries metadata entries
#define SW_SR_MULTI 0x4   // the payload has more than one measurement: alternate id "<alt>:<k>"

// Exchange form of a decoded record, 64 bytes: what crosses xGMI in the owner all-to-all.  The
// 80-byte record carries fields no event type uses together, so the exchange packs them
// losslessly (tests/test_multirank.py checks pack/unpack on every decoded type):
//   w0 = location ? elevation : name hash
//   w1 = measurement|location ? v0 : aux2_off | aux2_len << 32 | level << 48
//   w2 = v1 (longitude; 0 for the other types)
// src_rank is not sent: the receiving slab index is the source rank.
typedef struct __attribute__((aligned(16))) SwWireRec {
  uint64_t fp_lo;       // 0
  uint64_t fp_hi;       // 8
  int64_t event_date;   // 16
  uint64_t w0;          // 24
  uint64_t w1;          // 32
  uint64_t w2;          // 40
  uint64_t alt_hash;    // 48
  uint32_t aux_off;     // 56
  uint16_t aux_len;     // 60
  uint8_t etype;        // 62
  uint8_t flags;        // 63
} SwWireRec;

SW_HD uint64_t sw_f64_bits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
SW_HD double sw_bits_f64(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }

SW_HD SwWireRec sw_wire_pack(const SwEventRec& r) {
  SwWireRec w;
  const bool loc = r.etype == SW_EV_LOCATION;
  const bool val = r.etype == SW_EV_MEASUREMENT || loc;
  w.fp_lo = r.fp_lo; w.fp_hi = r.fp_hi; w.event_date = r.event_date;
  w.w0 = loc ? sw_f64_bits(r.v2) : r.name_hash;
  w.w1 = val ? sw_f64_bits(r.v0)
             : ((uint64_t)r.aux2_off | ((uint64_t)r.aux2_len << 32) | ((uint64_t)r.level << 48));
  w.w2 = sw_f64_bits(r.v1);
  w.alt_hash = r.alt_hash; w.aux_off = r.aux_off; w.aux_len = r.aux_len; w.etype = r.etype; w.flags = r.flags;
  return w;
}

SW_HD SwEventRec sw_wire_unpack(const SwWireRec& w, uint8_t src_rank) {
  SwEventRec r;
  const bool loc = w.etype == SW_EV_LOCATION;
  const bool val = w.etype == SW_EV_MEASUREMENT || loc;
  r.fp_lo = w.fp_lo; r.fp_hi = w.fp_hi; r.event_date = w.event_date;
  r.name_hash = loc ? 0 : w.w0;
  r.v2 = loc ? sw_bits_f64(w.w0) : 0.0;
  r.v0 = val ? sw_bits_f64(w.w1) : 0.0;
  r.v1 = sw_bits_f64(w.w2);
  r.aux2_off = val ? 0u : (uint32_t)w.w1;
  r.aux2_len = val ? (uint16_t)0 : (uint16_t)(w.w1 >> 32);
  r.level = val ? (uint8_t)0 : (uint8_t)(w.w1 >> 48);
  r.alt_hash = w.alt_hash; r.aux_off = w.aux_off; r.aux_len = w.aux_len; r.etype = w.etype; r.flags = w.flags;
  r.src_rank = src_rank;
  return r;
}

// Enriched, persisted event as delivered to outbound consumers, 32 bytes, written by the GPU
// straight into mapped pinned host memory (zero-copy outbound, no D2H copy stage).
// The event id is implicit: row j of a step is event (cursor0 + j) * world + rank; the device
// follows from the assignment on the host.  Reference: GEnrichedEventPayload.
typedef struct __attribute__((aligned(16))) SwOutRec {
  int64_t event_date;   // 0
  double v0;            // 8  value | latitude
  double v1;            // 16 longitude
  int32_t assignment;   // 24
  uint16_t name_id;     // 28 interned name / alert type id (0xffff none)
  uint8_t etype;        // 30
  uint8_t level;        // 31
} SwOutRec;

// Zone-test rule (reference: ZoneTestRuleProcessor.java:47-62).
typedef struct SwZoneTest {
  int32_t zone;         // index into zone polygon table
  int32_t condition;    // 0 = alert when INSIDE, 1 = alert when OUTSIDE
  int32_t alert_name_id;// interned alert type
  int32_t level;        // alert level
} SwZoneTest;

// ---------------------------------------------------------------- hashing
#define SW_FNV_OFFSET 0xcbf29ce484222325ULL
#define SW_FNV_PRIME 0x100000001b3ULL
#define SW_POLY_SEED 0x9e3779b97f4a7c15ULL
#define SW_POLY_MUL 0xff51afd7ed558ccdULL

SW_HD uint64_t sw_mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return x;
}

// Store-backed alternate-id filter: generational exact-fingerprint tables of the ids the engine
// persisted (the reference checks every alternate id against the store forever,
// AlternateIdDeduplicator.java:43-56; here only ids new to the HBM window that the filter holds go
// to the host as SW_ST_RECHECK, which checks them against the event store).
//   * G generations of >= ids_per_gen persisted ids each: once the live generation has taken
//     ids_per_gen ids (at the end of a step) the oldest is cleared and becomes the live one, so the
//     filter always holds the newest (G - 1) * ids_per_gen ids -- and the durable store's retention
//     keeps no more rows than that (retention by rows, persistence/segments.py; every retained id
//     is then among the newest ids), so every retained id stays checked and nothing else is.
//   * A generation is a linear-probed table of 16-slot buckets of 32-bit fingerprints (an id's
//     bucket from the low bits of mix(h), its fingerprint from the high 32 bits, 0 = empty).  The
//     G buckets of one home position are adjacent (bucket b of generation g at (b * G + g) * 16
//     slots), so a probe of every generation reads G * 64 contiguous bytes; an add is ONE CAS.
//   * False positives: an absent id matches a fingerprint of its bucket chain, ~(ids per bucket) /
//     2^32 per generation -- ~1e-8 at the sizing load (<= 1/2), where a one-word Bloom filter at 128
//     bits per id gave ~3e-6 and could only grow.
// Same functions in every engine (bit-exact).
#define SW_FF_SLOTS 16                 // fingerprints per bucket (64 bytes)
#define SW_FF_MAX_PROBE 64             // buckets probed per generation before an add is dropped
#define SW_FF_META 16                  // meta words before the per-generation row starts
#define SW_FF_MAX_GENS 8
// meta: [0] live generation, [1] unused, [2] ids per generation, [3] generations, [4] rotations,
// [5] adds dropped (probe bound), [6] ids the live generation took, [7..15] pad,
// [16 + g] store cursor when generation g became live
SW_HD uint64_t sw_ff_mix(uint64_t h) { return sw_mix64(h ^ 0x5bd1e9955bd1e995ULL); }
SW_HD uint64_t sw_ff_bucket(uint64_t m, int64_t bmask) { return m & (uint64_t)bmask; }
SW_HD uint32_t sw_ff_fp(uint64_t m) {
  const uint32_t f = (uint32_t)(m >> 32);
  return f ? f : 1u;
}

// 128-bit fingerprint of a byte string: FNV-1a-64 and an independent odd-multiplier
// polynomial hash, both finalised with splitmix64.  (0,0) is reserved as "empty".
SW_HD void sw_fingerprint(const uint8_t* p, uint32_t n, uint64_t* lo, uint64_t* hi) {
  uint64_t a = SW_FNV_OFFSET, b = SW_POLY_SEED ^ (uint64_t)n;
  for (uint32_t i = 0; i < n; ++i) {
    a = (a ^ p[i]) * SW_FNV_PRIME;
    b = (b + p[i] + 1) * SW_POLY_MUL;
  }
  a = sw_mix64(a);
  b = sw_mix64(b ^ (b >> 29));
  if (a == 0 && b == 0) a = 1;
  *lo = a;
  *hi = b;
}

// 64-bit string hash (names, alert types, alternate ids). 0 is reserved.
SW_HD uint64_t sw_hash64(const uint8_t* p, uint32_t n) {
  uint64_t a = SW_FNV_OFFSET;
  for (uint32_t i = 0; i < n; ++i) a = (a ^ p[i]) * SW_FNV_PRIME;
  a = sw_mix64(a ^ ((uint64_t)n << 56));
  return a ? a : 1;
}

// sw_hash64 of the string p[0..n) + ":" + decimal(k) without building it: the alternate id of
// measurement k of a multi-measurement payload (the per-event path names it "<alt>:<k>",
// services/event_sources.py), so both paths deduplicate and index the same ids.
SW_HD uint64_t sw_hash64_sfx(const uint8_t* p, uint32_t n, uint32_t k) {
  uint64_t a = SW_FNV_OFFSET;
  for (uint32_t i = 0; i < n; ++i) a = (a ^ p[i]) * SW_FNV_PRIME;
  a = (a ^ (uint8_t)':') * SW_FNV_PRIME;
  uint32_t div = 1, nd = 1;
  while (k / div >= 10u) { div *= 10u; ++nd; }
  for (; div; div /= 10u) a = (a ^ (uint8_t)('0' + (k / div) % 10u)) * SW_FNV_PRIME;
  a = sw_mix64(a ^ ((uint64_t)(n + 1u + nd) << 56));
  return a ? a : 1;
}

// Which rank owns a device (multi-GPU sharding of registry/state/store).
SW_HD uint32_t sw_owner(uint64_t fp_hi, uint32_t world) {
  return (uint32_t)((fp_hi >> 32) % (uint64_t)world);
}

// ------------------------------------------------------- protobuf wire helpers
// Wire protocol: reference sitewhere-communication/src/main/proto/sitewhere.proto.
// Each payload = varint-delimited SiteWhere.Header + varint-delimited body.
#define SW_CMD_SEND_REGISTRATION 1
#define SW_CMD_SEND_ACKNOWLEDGEMENT 2
#define SW_CMD_SEND_DEVICE_LOCATION 3
#define SW_CMD_SEND_DEVICE_ALERT 4
#define SW_CMD_SEND_DEVICE_MEASUREMENTS 5
#define SW_CMD_SEND_DEVICE_STREAM 6
#define SW_CMD_SEND_DEVICE_STREAM_DATA 7
#define SW_CMD_REQUEST_DEVICE_STREAM_DATA 8
// Extension field (not in the reference schema; ignored by reference parsers as an
// unknown field): string alternateId = 15 on DeviceLocation/DeviceAlert/DeviceMeasurements.
#define SW_FIELD_ALTERNATE_ID 15

// Read a varint in [*pos, end). Returns false on truncation/overlong.
SW_HD bool sw_read_varint(const uint8_t* buf, uint32_t* pos, uint32_t end, uint64_t* out) {
  uint64_t v = 0;
  uint32_t shift = 0, p = *pos;
  while (p < end && shift < 64) {
    uint8_t b = buf[p++];
    v |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) {
      *pos = p;
      *out = v;
      return true;
    }
    shift += 7;
  }
  return false;
}

SW_HD uint64_t sw_load_le64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

// Skip one field of the given wire type. Returns false on malformed input.
SW_HD bool sw_skip_field(const uint8_t* buf, uint32_t* pos, uint32_t end, uint32_t wt) {
  uint64_t tmp;
  switch (wt) {
    case 0: return sw_read_varint(buf, pos, end, &tmp);
    case 1: if (*pos + 8 > end) return false; *pos += 8; return true;
    case 2:
      if (!sw_read_varint(buf, pos, end, &tmp)) return false;
      if (tmp > (uint64_t)(end - *pos)) return false;
      *pos += (uint32_t)tmp;
      return true;
    case 5: if (*pos + 4 > end) return false; *pos += 4; return true;
    default: return false;
  }
}
