// Per-payload routing of the messages an engine step did not persist (the host "slow path").
//
// The MI355X step rejects events of unregistered / unassigned devices, control messages
// (registration, acknowledgement, streams) and undecodable payloads.  Every reject record points
// into its payload (aux_off, csrc/include/swdecode.h), so only the affected payloads are looked at:
// a binary search finds each one, it is parsed once, and the reference's Kafka payloads are written
// straight into one output heap:
//   unregistered / unassigned data -> GInboundEventPayload per event (unregistered-device topic,
//     InboundPayloadProcessingLogic.java:199-218)
//   registration                  -> GDeviceRegistationPayload (registration topic,
//     EventSourcesManager.java:153-182)
//   acknowledgement / streams      -> the payload itself (the tenant decodes those few on the host;
//     the reference message has no member for them)
//   undecodable                    -> the payload itself (failed-decode topic,
//     EventSourcesManager.java:189-197)
// Output records are keyed by device token and carry the Kafka partition of the key.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "swtypes.h"

extern "C" int32_t sw_partition_for_key(const uint8_t* key, int32_t len, int32_t n);

namespace {

enum RouteKind { RK_UNREGISTERED = 0, RK_REGISTRATION = 1, RK_CONTROL = 2, RK_FAILED = 3 };

struct Str {
  const uint8_t* p = nullptr;
  uint32_t n = 0;
  bool has = false;
};

struct Meta {
  Str k, v;
};

struct Mx {
  Str name;
  double value = 0;
};

struct Parsed {
  uint64_t cmd = 0;
  Str originator, token, alt, type, message, dtype, area;
  double lat = 0, lon = 0, elev = 0;
  bool has_lat = false, has_lon = false, has_elev = false;
  uint64_t date = 0;
  bool has_date = false;
  bool us = false, has_us = false;
  std::vector<Mx> mx;
  std::vector<Meta> meta;
};

// ---------------------------------------------------------------- protobuf writer
struct W {
  std::vector<uint8_t> b;
  void varint(uint64_t v) {
    while (v >= 0x80) {
      b.push_back((uint8_t)(v | 0x80));
      v >>= 7;
    }
    b.push_back((uint8_t)v);
  }
  void key(uint32_t f, uint32_t wt) { varint(((uint64_t)f << 3) | wt); }
  void str(uint32_t f, const Str& s) {
    key(f, 2);
    varint(s.n);
    b.insert(b.end(), s.p, s.p + s.n);
  }
  void bytes(uint32_t f, const std::vector<uint8_t>& m) {
    key(f, 2);
    varint(m.size());
    b.insert(b.end(), m.begin(), m.end());
  }
  void dbl(uint32_t f, double d) {
    key(f, 1);
    uint64_t u;
    memcpy(&u, &d, 8);
    for (int i = 0; i < 8; ++i) b.push_back((uint8_t)(u >> (8 * i)));
  }
  void u64(uint32_t f, uint64_t v) {
    key(f, 0);
    varint(v);
  }
};

// proto3 wrappers: GOptionalString / GOptionalDouble / GOptionalBoolean {value = 1}
std::vector<uint8_t> opt_str(const Str& s) {
  W w;
  if (s.n) w.str(1, s);
  return w.b;
}

std::vector<uint8_t> opt_dbl(double d) {
  W w;
  uint64_t u;
  memcpy(&u, &d, 8);
  if (u) w.dbl(1, d);
  return w.b;
}

std::vector<uint8_t> opt_bool(bool v) {
  W w;
  if (v) w.u64(1, 1);
  return w.b;
}

void map_entries(W& w, uint32_t f, const std::vector<Meta>& meta) {
  for (const Meta& m : meta) {
    W e;
    if (m.k.n) e.str(1, m.k);
    if (m.v.n) e.str(2, m.v);
    w.bytes(f, e.b);
  }
}

// GDeviceEventCreateRequest (alternateId = 1, eventDate = 5, updateState = 6, metadata = 7)
std::vector<uint8_t> event_header(const Parsed& p, const Str& alt) {
  W w;
  if (alt.has) w.bytes(1, opt_str(alt));
  if (p.has_date && p.date) w.u64(5, p.date);
  if (p.has_us) w.bytes(6, opt_bool(p.us));
  map_entries(w, 7, p.meta);
  return w.b;
}

// GInboundEventPayload {sourceId = 1, deviceToken = 2, originator = 3, event = 4}
std::vector<uint8_t> inbound(const Str& source, const Parsed& p, uint32_t member, const std::vector<uint8_t>& req) {
  W any;
  any.bytes(member, req);
  W w;
  if (source.n) w.str(1, source);
  if (p.token.n) w.str(2, p.token);
  if (p.originator.has) w.bytes(3, opt_str(p.originator));
  w.bytes(4, any.b);
  return w.b;
}

// ---------------------------------------------------------------- device protocol reader
bool rd_str(const uint8_t* b, uint32_t* pos, uint32_t end, Str* s) {
  uint64_t n;
  if (!sw_read_varint(b, pos, end, &n) || n > (uint64_t)(end - *pos)) return false;
  s->p = b + *pos;
  s->n = (uint32_t)n;
  s->has = true;
  *pos += (uint32_t)n;
  return true;
}

bool rd_dbl(const uint8_t* b, uint32_t* pos, uint32_t end, double* d) {
  if (*pos + 8 > end) return false;
  const uint64_t u = sw_load_le64(b + *pos);
  memcpy(d, &u, 8);
  *pos += 8;
  return true;
}

bool rd_meta(const uint8_t* b, uint32_t* pos, uint32_t end, Meta* m) {
  uint64_t n;
  if (!sw_read_varint(b, pos, end, &n) || n > (uint64_t)(end - *pos)) return false;
  const uint32_t me = *pos + (uint32_t)n;
  while (*pos < me) {
    uint64_t k;
    if (!sw_read_varint(b, pos, me, &k)) return false;
    const uint32_t f = (uint32_t)(k >> 3), wt = (uint32_t)(k & 7);
    if (f == 1 && wt == 2) { if (!rd_str(b, pos, me, &m->k)) return false; }
    else if (f == 2 && wt == 2) { if (!rd_str(b, pos, me, &m->v)) return false; }
    else if (!sw_skip_field(b, pos, me, wt)) return false;
  }
  return true;
}

bool parse(const uint8_t* b, uint32_t s, uint32_t e, Parsed* p) {
  uint32_t pos = s;
  uint64_t hl, bl;
  if (!sw_read_varint(b, &pos, e, &hl) || hl > (uint64_t)(e - pos)) return false;
  const uint32_t he = pos + (uint32_t)hl;
  while (pos < he) {
    uint64_t k;
    if (!sw_read_varint(b, &pos, he, &k)) return false;
    const uint32_t f = (uint32_t)(k >> 3), wt = (uint32_t)(k & 7);
    if (f == 1 && wt == 0) { if (!sw_read_varint(b, &pos, he, &p->cmd)) return false; }
    else if (f == 2 && wt == 2) { if (!rd_str(b, &pos, he, &p->originator)) return false; }
    else if (!sw_skip_field(b, &pos, he, wt)) return false;
  }
  if (!sw_read_varint(b, &pos, e, &bl) || bl > (uint64_t)(e - pos)) return false;
  const uint32_t be = pos + (uint32_t)bl;
  const uint64_t c = p->cmd;
  if (c < 1 || c > 8) return false;
  while (pos < be) {
    uint64_t k, v;
    if (!sw_read_varint(b, &pos, be, &k)) return false;
    const uint32_t f = (uint32_t)(k >> 3), wt = (uint32_t)(k & 7);
    bool ok = true;
    if (f == 1 && wt == 2) ok = rd_str(b, &pos, be, &p->token);
    else if (f == SW_FIELD_ALTERNATE_ID && wt == 2 && c >= 3 && c <= 5) ok = rd_str(b, &pos, be, &p->alt);
    else if (c == SW_CMD_SEND_DEVICE_MEASUREMENTS) {
      if (f == 2 && wt == 2) {
        uint64_t n;
        ok = sw_read_varint(b, &pos, be, &n) && n <= (uint64_t)(be - pos);
        if (ok) {
          const uint32_t me = pos + (uint32_t)n;
          Mx m;
          while (ok && pos < me) {
            uint64_t k2;
            ok = sw_read_varint(b, &pos, me, &k2);
            if (!ok) break;
            const uint32_t f2 = (uint32_t)(k2 >> 3), w2 = (uint32_t)(k2 & 7);
            if (f2 == 1 && w2 == 2) ok = rd_str(b, &pos, me, &m.name);
            else if (f2 == 2 && w2 == 1) ok = rd_dbl(b, &pos, me, &m.value);
            else ok = sw_skip_field(b, &pos, me, w2);
          }
          p->mx.push_back(m);
        }
      } else if (f == 3 && wt == 1) { ok = pos + 8 <= be; if (ok) { p->date = sw_load_le64(b + pos); pos += 8; p->has_date = true; } }
      else if (f == 4 && wt == 2) { Meta m; ok = rd_meta(b, &pos, be, &m); p->meta.push_back(m); }
      else if (f == 5 && wt == 0) { ok = sw_read_varint(b, &pos, be, &v); p->has_us = true; p->us = v != 0; }
      else ok = sw_skip_field(b, &pos, be, wt);
    } else if (c == SW_CMD_SEND_DEVICE_LOCATION) {
      if (f == 2 && wt == 1) { ok = rd_dbl(b, &pos, be, &p->lat); p->has_lat = true; }
      else if (f == 3 && wt == 1) { ok = rd_dbl(b, &pos, be, &p->lon); p->has_lon = true; }
      else if (f == 4 && wt == 1) { ok = rd_dbl(b, &pos, be, &p->elev); p->has_elev = true; }
      else if (f == 5 && wt == 1) { ok = pos + 8 <= be; if (ok) { p->date = sw_load_le64(b + pos); pos += 8; p->has_date = true; } }
      else if (f == 6 && wt == 2) { Meta m; ok = rd_meta(b, &pos, be, &m); p->meta.push_back(m); }
      else if (f == 7 && wt == 0) { ok = sw_read_varint(b, &pos, be, &v); p->has_us = true; p->us = v != 0; }
      else ok = sw_skip_field(b, &pos, be, wt);
    } else if (c == SW_CMD_SEND_DEVICE_ALERT) {
      if (f == 2 && wt == 2) ok = rd_str(b, &pos, be, &p->type);
      else if (f == 3 && wt == 2) ok = rd_str(b, &pos, be, &p->message);
      else if (f == 4 && wt == 1) { ok = pos + 8 <= be; if (ok) { p->date = sw_load_le64(b + pos); pos += 8; p->has_date = true; } }
      else if (f == 5 && wt == 2) { Meta m; ok = rd_meta(b, &pos, be, &m); p->meta.push_back(m); }
      else if (f == 6 && wt == 0) { ok = sw_read_varint(b, &pos, be, &v); p->has_us = true; p->us = v != 0; }
      else ok = sw_skip_field(b, &pos, be, wt);
    } else if (c == SW_CMD_SEND_REGISTRATION) {
      if (f == 2 && wt == 2) ok = rd_str(b, &pos, be, &p->dtype);
      else if (f == 3 && wt == 2) { Meta m; ok = rd_meta(b, &pos, be, &m); p->meta.push_back(m); }
      else if (f == 4 && wt == 2) ok = rd_str(b, &pos, be, &p->area);
      else ok = sw_skip_field(b, &pos, be, wt);
    } else {
      ok = sw_skip_field(b, &pos, be, wt);
    }
    if (!ok) return false;
  }
  return p->token.n > 0;
}

struct Rec {
  int32_t kind, part;
  std::vector<uint8_t> key, val;
};

struct Out {
  std::vector<Rec> recs;
  int32_t parts[4];
  void emit(int kind, const Str& key, const uint8_t* v, int64_t vn) {
    Rec r;
    r.kind = kind;
    r.part = key.n ? sw_partition_for_key(key.p, (int32_t)key.n, parts[kind] > 0 ? parts[kind] : 1) : -1;
    r.key.assign(key.p, key.p + key.n);
    r.val.assign(v, v + vn);
    recs.push_back(std::move(r));
  }
};

}  // namespace

// Route the rejected messages of one raw batch.
//   raw/offs/n_msgs : the batch (payload bytes, n_msgs + 1 offsets)
//   rej_off/rej_st  : n_rej reject records: any byte offset inside their payload + engine status
//                     (1 unregistered, 2 unassigned, 3 duplicate, 4 decode error, 5 control)
//   parts           : partitions of the unregistered, registration, decoded and failed-decode topics
// Output: records grouped by (kind, partition) -- stable, so per-key order is the batch order --
// with rec[i] = (kind, partition, key length, value length) and the keys / values concatenated in
// that order in key_heap / val_heap.  Returns the record count, or -1 when a heap or rec is too
// small (need[0] = records, need[1] = key bytes, need[2] = value bytes: call again with those).
// Duplicates are dropped (dedup).  payloads_out = payloads looked at.
static int64_t route_hits(const uint8_t* raw, std::vector<std::pair<uint64_t, uint8_t>>& hit, const char* source_id,
                          const int32_t* parts, int32_t* rec, int64_t rec_cap, uint8_t* key_heap, int64_t key_cap,
                          uint8_t* val_heap, int64_t val_cap, int64_t* need, int64_t* payloads_out) {
  // hit: ((start << 32 | end), status), one per affected payload after the dedupe below
  std::sort(hit.begin(), hit.end());
  hit.erase(std::unique(hit.begin(), hit.end(),
                        [](const std::pair<uint64_t, uint8_t>& a, const std::pair<uint64_t, uint8_t>& b) {
                          return a.first == b.first;
                        }),
            hit.end());
  Out o;
  for (int k = 0; k < 4; ++k) o.parts[k] = parts[k];
  Str source;
  source.p = (const uint8_t*)source_id;
  source.n = (uint32_t)strlen(source_id);
  for (const auto& h : hit) {
    const uint32_t s = (uint32_t)(h.first >> 32), e = (uint32_t)h.first;
    Parsed p;
    const bool ok = parse(raw, s, e, &p);
    if (!ok || h.second == 4) {
      Str none;
      o.emit(RK_FAILED, none, raw + s, e - s);
      continue;
    }
    if (p.cmd == SW_CMD_SEND_REGISTRATION) {
      W reg;
      if (p.dtype.n) reg.bytes(1, opt_str(p.dtype));
      if (p.area.n) reg.bytes(3, opt_str(p.area));
      map_entries(reg, 4, p.meta);
      W w;                                  // GDeviceRegistationPayload
      if (source.n) w.str(1, source);
      w.str(2, p.token);
      if (p.originator.has) w.bytes(3, opt_str(p.originator));
      if (!reg.b.empty()) w.bytes(4, reg.b);
      o.emit(RK_REGISTRATION, p.token, w.b.data(), (int64_t)w.b.size());
    } else if (p.cmd == SW_CMD_SEND_DEVICE_MEASUREMENTS) {
      const size_t n = p.mx.size();
      for (size_t i = 0; i < n; ++i) {
        Str alt = p.alt;
        std::string suffixed;
        if (alt.has && n > 1) {            // ProtobufDecoder: "<alternateId>:<index>" per measurement
          suffixed.assign((const char*)alt.p, alt.n);
          suffixed += ":" + std::to_string(i);
          alt.p = (const uint8_t*)suffixed.data();
          alt.n = (uint32_t)suffixed.size();
        }
        W m;                                // GDeviceMeasurementCreateRequest
        if (p.mx[i].name.n) m.str(1, p.mx[i].name);
        uint64_t u;
        memcpy(&u, &p.mx[i].value, 8);
        if (u) m.dbl(2, p.mx[i].value);
        m.bytes(3, event_header(p, alt));
        const std::vector<uint8_t> v = inbound(source, p, 1, m.b);
        o.emit(RK_UNREGISTERED, p.token, v.data(), (int64_t)v.size());
      }
    } else if (p.cmd == SW_CMD_SEND_DEVICE_LOCATION) {
      W m;                                  // GDeviceLocationCreateRequest
      m.bytes(1, opt_dbl(p.lat));
      m.bytes(2, opt_dbl(p.lon));
      if (p.has_elev) m.bytes(3, opt_dbl(p.elev));
      m.bytes(4, event_header(p, p.alt));
      const std::vector<uint8_t> v = inbound(source, p, 3, m.b);
      o.emit(RK_UNREGISTERED, p.token, v.data(), (int64_t)v.size());
    } else if (p.cmd == SW_CMD_SEND_DEVICE_ALERT) {
      W m;                                  // GDeviceAlertCreateRequest (source Device, level Info)
      if (p.type.n) m.str(3, p.type);
      if (p.message.n) m.str(4, p.message);
      m.bytes(5, event_header(p, p.alt));
      const std::vector<uint8_t> v = inbound(source, p, 2, m.b);
      o.emit(RK_UNREGISTERED, p.token, v.data(), (int64_t)v.size());
    } else {
      o.emit(RK_CONTROL, p.token, raw + s, e - s);
    }
  }
  if (payloads_out) *payloads_out = (int64_t)hit.size();
  std::stable_sort(o.recs.begin(), o.recs.end(), [](const Rec& a, const Rec& b) {
    return a.kind != b.kind ? a.kind < b.kind : a.part < b.part;
  });
  int64_t kb = 0, vb = 0;
  for (const Rec& r : o.recs) {
    kb += (int64_t)r.key.size();
    vb += (int64_t)r.val.size();
  }
  const int64_t n = (int64_t)o.recs.size();
  need[0] = n;
  need[1] = kb;
  need[2] = vb;
  if (n > rec_cap || kb > key_cap || vb > val_cap) return -1;
  int64_t ko = 0, vo = 0;
  for (int64_t i = 0; i < n; ++i) {
    const Rec& r = o.recs[(size_t)i];
    rec[4 * i] = r.kind;
    rec[4 * i + 1] = r.part;
    rec[4 * i + 2] = (int32_t)r.key.size();
    rec[4 * i + 3] = (int32_t)r.val.size();
    if (!r.key.empty()) memcpy(key_heap + ko, r.key.data(), r.key.size());
    if (!r.val.empty()) memcpy(val_heap + vo, r.val.data(), r.val.size());
    ko += (int64_t)r.key.size();
    vo += (int64_t)r.val.size();
  }
  return n;
}

extern "C" {

// rej_off: any byte offset inside the rejected event's payload (binary search over offs).
int64_t sw_route_rejects(const uint8_t* raw, const uint32_t* offs, int64_t n_msgs, const uint32_t* rej_off,
                         const uint8_t* rej_st, int64_t n_rej, const char* source_id, const int32_t* parts,
                         int32_t* rec, int64_t rec_cap, uint8_t* key_heap, int64_t key_cap, uint8_t* val_heap,
                         int64_t val_cap, int64_t* need, int64_t* payloads_out) {
  std::vector<std::pair<uint64_t, uint8_t>> hit;
  hit.reserve((size_t)n_rej);
  for (int64_t i = 0; i < n_rej; ++i) {
    const uint8_t st = rej_st[i];
    if (st == 3 || st == 0) continue;
    const uint32_t* it = std::upper_bound(offs, offs + n_msgs + 1, rej_off[i]);
    const int64_t m = (int64_t)(it - offs) - 1;
    if (m < 0 || m >= n_msgs) continue;
    hit.push_back({((uint64_t)offs[m] << 32) | offs[m + 1], st});
  }
  return route_hits(raw, hit, source_id, parts, rec, rec_cap, key_heap, key_cap, val_heap, val_cap, need,
                    payloads_out);
}

// refs: n x (payload start, payload end, status | src_rank << 8) as the MI355X step snapshot them
// (k_reject_refs); only refs whose src_rank == rank are routed (their bytes are in `raw`).
int64_t sw_route_refs(const uint8_t* raw, const uint32_t* refs, int64_t n, int32_t rank, const char* source_id,
                      const int32_t* parts, int32_t* rec, int64_t rec_cap, uint8_t* key_heap, int64_t key_cap,
                      uint8_t* val_heap, int64_t val_cap, int64_t* need, int64_t* payloads_out) {
  std::vector<std::pair<uint64_t, uint8_t>> hit;
  hit.reserve((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t s = refs[3 * i], e = refs[3 * i + 1], st = refs[3 * i + 2] & 0xff, src = refs[3 * i + 2] >> 8;
    if (st == 3 || st == 0 || (int32_t)src != rank || e <= s) continue;
    hit.push_back({((uint64_t)s << 32) | e, (uint8_t)st});
  }
  return route_hits(raw, hit, source_id, parts, rec, rec_cap, key_heap, key_cap, val_heap, val_cap, need,
                    payloads_out);
}

}  // extern "C"
