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

SW_HD void sw_clear_span(SwStrRef* s) {
  s->alt_off = 0; s->meta_off = 0; s->alt_len = 0; s->meta_len = 0; s->k = 0; s->has = 0; s->pad = 0;
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
// (ProtobufDeviceEventDecoder.java:79-95).  Advances the cursor past it; *len1 = the largest
// field-1 string length seen (a measurement name).
SW_HD bool sw_check_pair(const uint8_t* buf, uint32_t* pos, uint32_t end, uint32_t wt2, uint32_t* len1 = nullptr) {
  uint64_t len;
  if (!sw_read_varint(buf, pos, end, &len) || len > (uint64_t)(end - *pos)) return false;
  uint32_t p = *pos;
  const uint32_t e = p + (uint32_t)len;
  bool h1 = false, h2 = false;
  while (p < e) {
    uint32_t f, wt;
    if (!sw_read_tag(buf, &p, e, &f, &wt)) return false;
    const uint32_t vs = p;
    if (!sw_skip_field(buf, &p, e, wt)) return false;
    if (f == 1 && wt == 2) {
      h1 = true;
      if (len1) {                       // value length = field bytes minus its length varint
        uint32_t q = vs;
        uint64_t l;
        sw_read_varint(buf, &q, e, &l);
        if ((uint32_t)l > *len1) *len1 = (uint32_t)l;
      }
    }
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
// pass (out == null) stores SW_DEC_VALID, SW_DEC_ERROR or SW_DEC_OVERSIZE there; an emit pass given
// that verdict writes a known error's (or oversize event's) record without parsing it again and
// skips re-validating the embedded entries of a known-valid payload (the same bytes were checked by
// the count pass).
//
// `spans` (optional, emit pass): one SwStrRef per record written -- where the record's alternate id
// and metadata sit in the batch (the durable-block encoder copies them from there).  An event whose
// strings exceed 16-bit lengths (alternate id, metadata span, alert type / message, measurement
// name) is one SW_EV_OVERSIZE record instead: the host routes the payload to the per-event path.
#define SW_DEC_UNKNOWN 0u
#define SW_DEC_VALID 1u
#define SW_DEC_ERROR 2u
#define SW_DEC_OVERSIZE 3u
SW_HD uint32_t sw_decode_payload(const uint8_t* buf, uint32_t start, uint32_t end, uint32_t abs_base,
                                 int64_t now_ms, uint8_t src_rank, SwEventRec* out, uint32_t max_out,
                                 uint32_t* verdict = nullptr, SwStrRef* spans = nullptr) {
  const uint32_t known = verdict ? *verdict : SW_DEC_UNKNOWN;
  if (out && known == SW_DEC_ERROR) {
    if (max_out) {
      sw_fill_control(out, SW_EV_DECODE_ERROR, abs_base + start, abs_base + end, 0, 0, now_ms, src_rank);
      if (spans) sw_clear_span(spans);
    }
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
    if (out && max_out) {
      sw_fill_control(out, SW_EV_DECODE_ERROR, abs_base + start, abs_base + end, 0, 0, now_ms, src_rank);
      if (spans) sw_clear_span(spans);
    }
    if (!out && verdict) *verdict = SW_DEC_ERROR;
    return 1;
  }
  const uint32_t bstart = pos, bend = pos + (uint32_t)blen;
  const bool event = cmd == SW_CMD_SEND_DEVICE_MEASUREMENTS || cmd == SW_CMD_SEND_DEVICE_LOCATION ||
                     cmd == SW_CMD_SEND_DEVICE_ALERT;
  // metadata entries: field 4 of DeviceMeasurements, 6 of DeviceLocation, 5 of DeviceAlert
  const uint32_t meta_f = cmd == SW_CMD_SEND_DEVICE_MEASUREMENTS ? 4u : cmd == SW_CMD_SEND_DEVICE_LOCATION ? 6u : 5u;

  // ---- pass over body: common fields
  uint64_t lo = 0, hi = 0, date = 0;
  bool has_dev = false, has_date = false, has_us = false, us = false, has_elev = false, has_alt = false;
  bool req_a = false, req_b = false;  // latitude/longitude | alertType/alertMessage
  uint32_t n_mx = 0, name_max = 0;
  double lat = 0, lon = 0, elev = 0;
  // alert type / message; offsets default to the payload start so every record points into its payload
  uint32_t t_off = start, t_len = 0, m_off = start, m_len = 0;
  uint32_t a_off = start, a_len = 0;                  // alternate id (the last occurrence wins)
  uint32_t md_lo = 0, md_hi = 0;                      // metadata entries span [md_lo, md_hi)
  bool has_md = false;
  pos = bstart;
  while (ok && pos < bend) {
    uint32_t f, wt;
    const uint32_t fstart = pos;
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
    if (f == SW_FIELD_ALTERNATE_ID && wt == 2 && event) {
      ok = sw_read_varint(buf, &pos, bend, &v) && v <= (uint64_t)(bend - pos);
      if (!ok) break;
      a_off = pos; a_len = (uint32_t)v; has_alt = true;
      pos += (uint32_t)v;
      continue;
    }
    if (event && f == meta_f && wt == 2) {
      ok = trusted ? sw_skip_field(buf, &pos, bend, wt) : sw_check_pair(buf, &pos, bend, 2);
      if (!has_md) md_lo = fstart;
      md_hi = pos;
      has_md = true;
      continue;
    }
    switch (cmd) {
      case SW_CMD_SEND_DEVICE_MEASUREMENTS:
        if (f == 2 && wt == 2) { n_mx++; ok = trusted ? sw_skip_field(buf, &pos, bend, wt) : sw_check_pair(buf, &pos, bend, 1, &name_max); }
        else if (f == 3 && wt == 1) { if (pos + 8 > bend) { ok = false; break; } date = sw_load_le64(buf + pos); pos += 8; has_date = true; }
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
        } else if (f == 7 && wt == 0) { ok = sw_read_varint(buf, &pos, bend, &v); has_us = true; us = v != 0; }
        else ok = sw_skip_field(buf, &pos, bend, wt);
        break;
      case SW_CMD_SEND_DEVICE_ALERT:
        if ((f == 2 || f == 3) && wt == 2) {
          ok = sw_read_varint(buf, &pos, bend, &v) && v <= (uint64_t)(bend - pos);
          if (!ok) break;
          if (f == 2) { t_off = pos; t_len = (uint32_t)v; req_a = true; } else { m_off = pos; m_len = (uint32_t)v; req_b = true; }
          pos += (uint32_t)v;
        } else if (f == 4 && wt == 1) { if (pos + 8 > bend) { ok = false; break; } date = sw_load_le64(buf + pos); pos += 8; has_date = true; }
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
    if (out && max_out) {
      sw_fill_control(out, SW_EV_DECODE_ERROR, abs_base + start, abs_base + end, 0, 0, now_ms, src_rank);
      if (spans) sw_clear_span(spans);
    }
    return 1;
  }
  // strings past the engine's 16-bit lengths: the whole payload takes the per-event path.  The
  // count pass decides (it alone sees every measurement name); the emit pass follows its verdict.
  const bool oversize = event && (known == SW_DEC_OVERSIZE ||
                                  (!trusted && (a_len > 0xffffu || md_hi - md_lo > 0xffffu || t_len > 0xffffu ||
                                                m_len > 0xffffu || name_max > 0xffffu)));
  if (oversize) {
    if (!out && verdict) *verdict = SW_DEC_OVERSIZE;
    if (!out) return 1;
    if (!max_out) return 0;
    sw_fill_control(out, SW_EV_OVERSIZE, abs_base + start, abs_base + end, lo, hi, now_ms, src_rank);
    if (spans) sw_clear_span(spans);
    return 1;
  }
  uint8_t flags = (has_us ? SW_F_HAS_UPDATE_STATE : 0) | (us ? SW_F_UPDATE_STATE : 0) |
                  (has_date ? SW_F_HAS_DATE : 0) | (has_elev ? SW_F_HAS_ELEVATION : 0);
  int64_t edate = has_date ? (int64_t)date : now_ms;
  SwStrRef sp;
  sp.alt_off = abs_base + a_off; sp.alt_len = (uint16_t)a_len;
  sp.meta_off = has_md ? abs_base + md_lo : abs_base + start; sp.meta_len = has_md ? (uint16_t)(md_hi - md_lo) : 0;
  sp.k = 0; sp.has = (has_alt ? SW_SR_ALT : 0) | (has_md ? SW_SR_META : 0); sp.pad = 0;

  if (!out && verdict) *verdict = SW_DEC_VALID;
  if (!out) return cmd == SW_CMD_SEND_DEVICE_MEASUREMENTS ? n_mx : 1;
  const uint64_t alt = has_alt && (cmd != SW_CMD_SEND_DEVICE_MEASUREMENTS || n_mx == 1) ? sw_hash64(buf + a_off, a_len) : 0;
  if (cmd == SW_CMD_SEND_DEVICE_MEASUREMENTS) {
    if (n_mx > max_out) {
      if (max_out) {
        sw_fill_control(out, SW_EV_DECODE_ERROR, abs_base + start, abs_base + end, lo, hi, now_ms, src_rank);
        if (spans) sw_clear_span(spans);
      }
      return max_out ? 1 : 0;
    }
    const bool multi = n_mx > 1;
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
      // measurement k of a multi-measurement payload has the alternate id "<alt>:<k>"
      r->alt_hash = !has_alt ? 0 : multi ? sw_hash64_sfx(buf + a_off, a_len, k) : alt;
      r->aux_off = abs_base + n_off; r->aux2_off = 0;
      r->aux_len = (uint16_t)n_len; r->aux2_len = 0;
      r->etype = SW_EV_MEASUREMENT; r->flags = flags; r->src_rank = src_rank; r->level = 0;
      if (spans) {
        spans[k] = sp;
        spans[k].k = (uint16_t)(k > 0xffffu ? 0xffffu : k);
        spans[k].has |= multi ? SW_SR_MULTI : 0;
      }
      ++k;
    }
    // A structurally valid message always yields n_mx records; pad defensively.
    for (; k < n_mx; ++k) {
      sw_fill_control(out + k, SW_EV_DECODE_ERROR, abs_base + start, abs_base + end, lo, hi, now_ms, src_rank);
      if (spans) sw_clear_span(spans + k);
    }
    return n_mx;
  }
  if (!max_out) return 0;
  if (spans) *spans = sp;
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
    out->aux_len = (uint16_t)t_len;
    out->aux2_len = (uint16_t)m_len;
    out->etype = SW_EV_ALERT; out->flags = flags; out->src_rank = src_rank; out->level = 0;  // AlertLevel.Info
    return 1;
  }
  if (spans) sw_clear_span(spans);
  uint8_t et = cmd == SW_CMD_SEND_REGISTRATION ? SW_EV_REGISTRATION
             : cmd == SW_CMD_SEND_ACKNOWLEDGEMENT ? SW_EV_ACK
             : cmd == SW_CMD_SEND_DEVICE_STREAM ? SW_EV_STREAM_CREATE
             : cmd == SW_CMD_SEND_DEVICE_STREAM_DATA ? SW_EV_STREAM_DATA
             : SW_EV_STREAM_DATA_REQUEST;
  sw_fill_control(out, et, abs_base + start, abs_base + end, lo, hi, now_ms, src_rank);
  return 1;
}
