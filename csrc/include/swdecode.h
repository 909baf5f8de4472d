// Protobuf device-protocol decoder shared by the CPU runtime and the GPU kernel.
//
// Behavioural reference: service-event-sources/.../decoder/protobuf/ProtobufDeviceEventDecoder.java:79-281
//   * payload = delimited SiteWhere.Header, then delimited body message
//   * SEND_DEVICE_MEASUREMENTS expands to one event per Measurement entry
//   * a missing eventDate defaults to the receive time
//   * registration / acknowledgement / stream messages are control requests
// One source of truth: the same function body runs per-lane on gfx950 and per
// message on the host, so CPU/GPU parity is structural, not coincidental.
//
// `buf` points at the bytes of the payload window, positions are relative to it;
// `abs_base` is added to every recorded offset so records point into the raw batch.
#pragma once
#include "swtypes.h"

SW_HD void sw_fill_control(SwEventRec* r, uint8_t etype, uint32_t abs_start, uint32_t abs_end,
                           uint64_t lo, uint64_t hi, int64_t now_ms, uint8_t src_rank) {
  r->fp_lo = lo; r->fp_hi = hi; r->event_date = now_ms; r->name_hash = 0;
  r->v0 = 0; r->v1 = 0; r->v2 = 0; r->alt_hash = 0;
  r->aux_off = abs_start; r->aux2_off = abs_end; r->aux_len = 0; r->aux2_len = 0;
  r->etype = etype; r->flags = 0; r->src_rank = src_rank; r->level = 0;
}

// Read a field tag.  False on truncation and on tags protobuf refuses: field number 0 or a
// key past 32 bits.
SW_HD bool sw_read_tag(const uint8_t* buf, uint32_t* pos, uint32_t end, uint32_t* f, uint32_t* wt) {
  uint64_t key;
  if (!sw_read_varint(buf, pos, end, &key) || key > 0xffffffffull || (key >> 3) == 0) return false;
  *f = (uint32_t)(key >> 3);
  *wt = (uint32_t)(key & 7);
  return true;
}

// One embedded {required string 1; required <wt2> 2} message at the cursor (Model.Measurement with
// wt2 = fixed64, Model.Metadata with wt2 = length-delimited): well-formed and both required fields
// present, else protobuf-java's parseDelimitedFrom refuses the enclosing payload
// (ProtobufDeviceEventDecoder.java:79-95).  Advances the cursor past it.
SW_HD bool sw_check_pair(const uint8_t* buf, uint32_t* pos, uint32_t end, uint32_t wt2) {
  uint64_t len;
  if (!sw_read_varint(buf, pos, end, &len) || len > (uint64_t)(end - *pos)) return false;
  uint32_t p = *pos;
  const uint32_t e = p + (uint32_t)len;
  bool h1 = false, h2 = false;
  while (p < e) {
    uint32_t f, wt;
    if (!sw_read_tag(buf, &p, e, &f, &wt) || !sw_skip_field(buf, &p, e, wt)) return false;
    h1 |= f == 1 && wt == 2;
    h2 |= f == 2 && wt == wt2;
  }
  *pos = e;
  return h1 && h2;
}

// Decode one payload [start, end).  If `out` is null only counts records.
//
// Validity follows protobuf-java on the reference schema (proto2, `required` fields): a payload
// is a decode error when it is malformed, when the header has no known command, or when an event
// body misses a required field (hardwareId; latitude/longitude; alertType/alertMessage; the
// measurementId/measurementValue and Metadata name/value of every embedded entry).  Control bodies
// only need their hardwareId here: the host decodes those payloads in full.  Deprecated groups
// (wire types 3/4, unused by the schema) are refused.  Independent oracle: tests/decode_oracle.py.
// Returns the number of records produced (never more than max_out when out != null;
// a message whose expansion does not fit is reported as one decode error).
//
// `verdict` (optional) carries the validity between the two passes of the GPU decode: the count
// pass (out == null) stores SW_DEC_VALID or SW_DEC_ERROR there; an emit pass given that verdict
// writes a known error's record without parsing it again and skips re-validating the embedded
// entries of a known-valid payload (the same bytes were checked by the count pass).
#define SW_DEC_UNKNOWN 0u
#define SW_DEC_VALID 1u
#define SW_DEC_ERROR 2u
SW_HD uint32_t sw_decode_payload(const uint8_t* buf, uint32_t start, uint32_t end, uint32_t abs_base,
                                 int64_t now_ms, uint8_t src_rank, SwEventRec* out, uint32_t max_out,
                                 uint32_t* verdict = nullptr) {
  const uint32_t known = verdict ? *verdict : SW_DEC_UNKNOWN;
  if (out && known == SW_DEC_ERROR) {
    if (max_out) sw_fill_control(out, SW_EV_DECODE_ERROR, abs_base + start, abs_base + end, 0, 0, now_ms, src_rank);
    return 1;
  }
  const bool trusted = out && known == SW_DEC_VALID;
  uint32_t pos = start;
  uint64_t hlen = 0, blen = 0, v = 0;
  uint64_t cmd = 0;
  bool ok = sw_read_varint(buf, &pos, end, &hlen) && hlen <= (uint64_t)(end - pos);
  if (ok) {
    uint32_t hend = pos + (uint32_t)hlen;
    while (ok && pos < hend) {
      uint32_t f, wt;
      ok = sw_read_tag(buf, &pos, hend, &f, &wt);
      if (!ok) break;
      if (f == 1 && wt == 0) {
        ok = sw_read_varint(buf, &pos, hend, &v);
        if (v >= 1 && v <= 8) cmd = v;  // an unknown enum value is an unknown field (proto2)
      } else {
        ok = sw_skip_field(buf, &pos, hend, wt);
      }
    }
    ok = ok && sw_read_varint(buf, &pos, end, &blen) && blen <= (uint64_t)(end - pos);
  }
  if (!ok || cmd < 1 || cmd > 8) {
    if (out && max_out) sw_fill_control(out, SW_EV_DECODE_ERROR, abs_base + start, abs_base + end, 0, 0, now_ms, src_rank);
    if (!out && verdict) *verdict = SW_DEC_ERROR;
    return 1;
  }
  const uint32_t bstart = pos, bend = pos + (uint32_t)blen;

  // ---- pass over body: common fields
  uint64_t lo = 0, hi = 0, alt = 0, date = 0;
  bool has_dev = false, has_date = false, has_us = false, us = false, has_elev = false;
  bool req_a = false, req_b = false;  // latitude/longitude | alertType/alertMessage
  uint32_t n_mx = 0;
  double lat = 0, lon = 0, elev = 0;
  // alert type / message; offsets default to the payload start so every record points into its payload
  uint32_t t_off = start, t_len = 0, m_off = start, m_len = 0;
  pos = bstart;
  while (ok && pos < bend) {
    uint32_t f, wt;
    ok = sw_read_tag(buf, &pos, bend, &f, &wt);
    if (!ok) break;
    if (f == 1 && wt == 2) {  // hardwareId in every body message
      ok = sw_read_varint(buf, &pos, bend, &v) && v <= (uint64_t)(bend - pos);
      if (!ok) break;
      if (out) sw_fingerprint(buf + pos, (uint32_t)v, &lo, &hi);  // count pass skips hashing
      has_dev = true;
      pos += (uint32_t)v;
      continue;
    }
    if (f == SW_FIELD_ALTERNATE_ID && wt == 2 &&
        (cmd == SW_CMD_SEND_DEVICE_MEASUREMENTS || cmd == SW_CMD_SEND_DEVICE_LOCATION ||
         cmd == SW_CMD_SEND_DEVICE_ALERT)) {
      ok = sw_read_varint(buf, &pos, bend, &v) && v <= (uint64_t)(bend - pos);
      if (!ok) break;
      if (out) alt = sw_hash64(buf + pos, (uint32_t)v);
      pos += (uint32_t)v;
      continue;
    }
    switch (cmd) {
      case SW_CMD_SEND_DEVICE_MEASUREMENTS:
        if (f == 2 && wt == 2) { n_mx++; ok = trusted ? sw_skip_field(buf, &pos, bend, wt) : sw_check_pair(buf, &pos, bend, 1); }
        else if (f == 3 && wt == 1) { if (pos + 8 > bend) { ok = false; break; } date = sw_load_le64(buf + pos); pos += 8; has_date = true; }
        else if (f == 4 && wt == 2) ok = trusted ? sw_skip_field(buf, &pos, bend, wt) : sw_check_pair(buf, &pos, bend, 2);
        else if (f == 5 && wt == 0) { ok = sw_read_varint(buf, &pos, bend, &v); has_us = true; us = v != 0; }
        else ok = sw_skip_field(buf, &pos, bend, wt);
        break;
      case SW_CMD_SEND_DEVICE_LOCATION:
        if ((f == 2 || f == 3 || f == 4 || f == 5) && wt == 1) {
          if (pos + 8 > bend) { ok = false; break; }
          uint64_t bits = sw_load_le64(buf + pos); pos += 8;
          double d;
          __builtin_memcpy(&d, &bits, 8);
          if (f == 2) { lat = d; req_a = true; } else if (f == 3) { lon = d; req_b = true; }
          else if (f == 4) { elev = d; has_elev = true; }
          else { date = bits; has_date = true; }
        } else if (f == 6 && wt == 2) ok = trusted ? sw_skip_field(buf, &pos, bend, wt) : sw_check_pair(buf, &pos, bend, 2);
        else if (f == 7 && wt == 0) { ok = sw_read_varint(buf, &pos, bend, &v); has_us = true; us = v != 0; }
        else ok = sw_skip_field(buf, &pos, bend, wt);
        break;
      case SW_CMD_SEND_DEVICE_ALERT:
        if ((f == 2 || f == 3) && wt == 2) {
          ok = sw_read_varint(buf, &pos, bend, &v) && v <= (uint64_t)(bend - pos);
          if (!ok) break;
          if (f == 2) { t_off = pos; t_len = (uint32_t)v; req_a = true; } else { m_off = pos; m_len = (uint32_t)v; req_b = true; }
          pos += (uint32_t)v;
        } else if (f == 4 && wt == 1) { if (pos + 8 > bend) { ok = false; break; } date = sw_load_le64(buf + pos); pos += 8; has_date = true; }
        else if (f == 5 && wt == 2) ok = trusted ? sw_skip_field(buf, &pos, bend, wt) : sw_check_pair(buf, &pos, bend, 2);
        else if (f == 6 && wt == 0) { ok = sw_read_varint(buf, &pos, bend, &v); has_us = true; us = v != 0; }
        else ok = sw_skip_field(buf, &pos, bend, wt);
        break;
      default:
        ok = sw_skip_field(buf, &pos, bend, wt);
        break;
    }
  }
  if ((cmd == SW_CMD_SEND_DEVICE_LOCATION || cmd == SW_CMD_SEND_DEVICE_ALERT) && !(req_a && req_b)) ok = false;
  if (!ok || !has_dev) {
    if (!out && verdict) *verdict = SW_DEC_ERROR;
    if (out && max_out) sw_fill_control(out, SW_EV_DECODE_ERROR, abs_base + start, abs_base + end, 0, 0, now_ms, src_rank);
    return 1;
  }
  uint8_t flags = (has_us ? SW_F_HAS_UPDATE_STATE : 0) | (us ? SW_F_UPDATE_STATE : 0) |
                  (has_date ? SW_F_HAS_DATE : 0) | (has_elev ? SW_F_HAS_ELEVATION : 0);
  int64_t edate = has_date ? (int64_t)date : now_ms;

  if (!out && verdict) *verdict = SW_DEC_VALID;
  if (cmd == SW_CMD_SEND_DEVICE_MEASUREMENTS) {
    if (!out) return n_mx;
    if (n_mx > max_out) {
      if (max_out) sw_fill_control(out, SW_EV_DECODE_ERROR, abs_base + start, abs_base + end, lo, hi, now_ms, src_rank);
      return max_out ? 1 : 0;
    }
    uint32_t k = 0;
    pos = bstart;
    while (pos < bend && k < n_mx) {
      uint64_t key;
      if (!sw_read_varint(buf, &pos, bend, &key)) break;
      uint32_t f = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
      if (!(f == 2 && wt == 2)) { if (!sw_skip_field(buf, &pos, bend, wt)) break; continue; }
      sw_read_varint(buf, &pos, bend, &v);
      uint32_t mend = pos + (uint32_t)v;
      uint32_t n_off = start, n_len = 0;
      double val = 0;
      while (pos < mend) {
        uint64_t k2;
        if (!sw_read_varint(buf, &pos, mend, &k2)) { pos = mend; break; }
        uint32_t f2 = (uint32_t)(k2 >> 3), w2 = (uint32_t)(k2 & 7);
        if (f2 == 1 && w2 == 2) {
          uint64_t l2;
          if (!sw_read_varint(buf, &pos, mend, &l2) || l2 > (uint64_t)(mend - pos)) { pos = mend; break; }
          n_off = pos; n_len = (uint32_t)l2; pos += (uint32_t)l2;
        } else if (f2 == 2 && w2 == 1 && pos + 8 <= mend) {
          uint64_t bits = sw_load_le64(buf + pos); pos += 8;
          __builtin_memcpy(&val, &bits, 8);
        } else if (!sw_skip_field(buf, &pos, mend, w2)) { pos = mend; break; }
      }
      pos = mend;
      SwEventRec* r = out + k;
      r->fp_lo = lo; r->fp_hi = hi; r->event_date = edate;
      r->name_hash = n_len ? sw_hash64(buf + n_off, n_len) : 0;
      r->v0 = val; r->v1 = 0; r->v2 = 0;
      r->alt_hash = alt ? sw_mix64(alt + k) | 1 : 0;
      r->aux_off = abs_base + n_off; r->aux2_off = 0;
      r->aux_len = (uint16_t)(n_len > 0xffff ? 0xffff : n_len); r->aux2_len = 0;
      r->etype = SW_EV_MEASUREMENT; r->flags = flags; r->src_rank = src_rank; r->level = 0;
      ++k;
    }
    // A structurally valid message always yields n_mx records; pad defensively.
    for (; k < n_mx; ++k) sw_fill_control(out + k, SW_EV_DECODE_ERROR, abs_base + start, abs_base + end, lo, hi, now_ms, src_rank);
    return n_mx;
  }
  if (!out) return 1;
  if (!max_out) return 0;
  if (cmd == SW_CMD_SEND_DEVICE_LOCATION) {
    out->fp_lo = lo; out->fp_hi = hi; out->event_date = edate; out->name_hash = 0;
    out->v0 = lat; out->v1 = lon; out->v2 = elev; out->alt_hash = alt;
    out->aux_off = abs_base + start; out->aux2_off = 0; out->aux_len = 0; out->aux2_len = 0;
    out->etype = SW_EV_LOCATION; out->flags = flags; out->src_rank = src_rank; out->level = 0;
    return 1;
  }
  if (cmd == SW_CMD_SEND_DEVICE_ALERT) {
    out->fp_lo = lo; out->fp_hi = hi; out->event_date = edate;
    out->name_hash = t_len ? sw_hash64(buf + t_off, t_len) : 0;
    out->v0 = 0; out->v1 = 0; out->v2 = 0; out->alt_hash = alt;
    out->aux_off = abs_base + t_off; out->aux2_off = abs_base + m_off;
    out->aux_len = (uint16_t)(t_len > 0xffff ? 0xffff : t_len);
    out->aux2_len = (uint16_t)(m_len > 0xffff ? 0xffff : m_len);
    out->etype = SW_EV_ALERT; out->flags = flags; out->src_rank = src_rank; out->level = 0;  // AlertLevel.Info
    return 1;
  }
  uint8_t et = cmd == SW_CMD_SEND_REGISTRATION ? SW_EV_REGISTRATION
             : cmd == SW_CMD_SEND_ACKNOWLEDGEMENT ? SW_EV_ACK
             : cmd == SW_CMD_SEND_DEVICE_STREAM ? SW_EV_STREAM_CREATE
             : cmd == SW_CMD_SEND_DEVICE_STREAM_DATA ? SW_EV_STREAM_DATA
             : SW_EV_STREAM_DATA_REQUEST;
  sw_fill_control(out, et, abs_base + start, abs_base + end, lo, hi, now_ms, src_rank);
  return 1;
}
