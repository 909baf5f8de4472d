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
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
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
// Appends into a reused buffer (clear() keeps the capacity): no allocation per record once warm.
struct W {
  std::vector<uint8_t> buf;
  size_t n = 0;
  void clear() { n = 0; }
  size_t size() const { return n; }
  const uint8_t* data() const { return buf.data(); }
  uint8_t* at(size_t k) {                    // room for k more bytes, returns the write cursor
    if (n + k > buf.size()) buf.resize(std::max<size_t>(2 * buf.size(), n + k + 4096));
    return buf.data() + n;
  }
  void raw(const uint8_t* p, size_t k) {
    memcpy(at(k), p, k);
    n += k;
  }
  void varint(uint64_t v) {
    uint8_t* o = at(10);
    size_t i = 0;
    while (v >= 0x80) {
      o[i++] = (uint8_t)(v | 0x80);
      v >>= 7;
    }
    o[i++] = (uint8_t)v;
    n += i;
  }
  void key(uint32_t f, uint32_t wt) { varint(((uint64_t)f << 3) | wt); }
  void str(uint32_t f, const Str& s) {
    key(f, 2);
    varint(s.n);
    raw(s.p, s.n);
  }
  void sub(uint32_t f, const W& m) {
    key(f, 2);
    varint(m.n);
    raw(m.buf.data(), m.n);
  }
  void fixed64(uint64_t u) {
    memcpy(at(8), &u, 8);                    // little-endian host
    n += 8;
  }
  void dbl(uint32_t f, double d) {
    key(f, 1);
    uint64_t u;
    memcpy(&u, &d, 8);
    fixed64(u);
  }
  void u64(uint32_t f, uint64_t v) {
    key(f, 0);
    varint(v);
  }
  // proto3 wrappers GOptionalString / GOptionalDouble / GOptionalBoolean {value = 1}, written inline
  void opt_str(uint32_t f, const Str& s) {
    key(f, 2);
    if (!s.n) { varint(0); return; }
    varint(1 + vlen(s.n) + s.n);
    str(1, s);
  }
  void opt_dbl(uint32_t f, double d) {
    uint64_t u;
    memcpy(&u, &d, 8);
    key(f, 2);
    if (!u) { varint(0); return; }
    varint(9);
    dbl(1, d);
  }
  void opt_bool(uint32_t f, bool v) {
    key(f, 2);
    if (!v) { varint(0); return; }
    varint(2);
    u64(1, 1);
  }
  static size_t vlen(uint64_t v) {
    size_t n = 1;
    while (v >= 0x80) { v >>= 7; ++n; }
    return n;
  }
};

void map_entries(W& w, uint32_t f, const std::vector<Meta>& meta) {
  for (const Meta& m : meta) {
    const size_t n = (m.k.n ? 1 + W::vlen(m.k.n) + m.k.n : 0) + (m.v.n ? 1 + W::vlen(m.v.n) + m.v.n : 0);
    w.key(f, 2);
    w.varint(n);
    if (m.k.n) w.str(1, m.k);
    if (m.v.n) w.str(2, m.v);
  }
}

// GDeviceEventCreateRequest (alternateId = 1, eventDate = 5, updateState = 6, metadata = 7)
void event_header(W& w, const Parsed& p, const Str& alt) {
  w.clear();
  if (alt.has) w.opt_str(1, alt);
  if (p.has_date && p.date) w.u64(5, p.date);
  if (p.has_us) w.opt_bool(6, p.us);
  map_entries(w, 7, p.meta);
}

// GInboundEventPayload {sourceId = 1, deviceToken = 2, originator = 3, event = 4 {member = req}}
void inbound(W& out, const Str& source, const Parsed& p, uint32_t member, const W& req) {
  if (source.n) out.str(1, source);
  if (p.token.n) out.str(2, p.token);
  if (p.originator.has) out.opt_str(3, p.originator);
  out.key(4, 2);
  out.varint(1 + W::vlen(req.size()) + req.size());
  out.sub(member, req);
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

// One routed record: key = device token (bytes in the raw batch), value in a worker's arena.
struct RecRef {
  uint64_t order;           // kind << 62 | partition << 46 | payload rank << 14 | sub-record
  const uint8_t* key;
  uint32_t klen;
  uint32_t worker;
  uint64_t voff;
  uint64_t vlen;
};

struct Worker {
  W arena, h, m, reg;       // output values + reused scratch
  std::vector<RecRef> recs;
  Parsed p;
  std::string alt;
};

static inline uint64_t order_of(int kind, int32_t part, uint64_t rank, uint64_t sub) {
  return ((uint64_t)kind << 62) | ((uint64_t)(part < 0 ? 0 : part & 0xffff) << 46) | ((rank & 0xffffffffull) << 14) |
         (sub & 0x3fff);
}

}  // namespace

// Route the rejected messages of one raw batch.
//   raw/offs/n_msgs : the batch (payload bytes, n_msgs + 1 offsets)
//   rej_off/rej_st  : n_rej reject records: any byte offset inside their payload + engine status
//                     (1 unregistered, 2 unassigned, 3 duplicate, 4 decode error, 5 control, 6 recheck)
//   parts           : partitions of the unregistered, registration, decoded and failed-decode topics
// Output: records grouped by (kind, partition) -- stable, so per-key order is the batch order --
// with rec[i] = (kind, partition, key length, value length) and the keys / values concatenated in
// that order in key_heap / val_heap.  Returns the record count, or -1 when a heap or rec is too
// small (need[0] = records, need[1] = key bytes, need[2] = value bytes: call again with those).
// Duplicates are dropped (dedup).  payloads_out = payloads looked at.
static void route_one(Worker& wk, uint32_t wid, const uint8_t* raw, uint32_t s, uint32_t e, uint8_t st,
                      uint64_t rank, const Str& source, const int32_t* parts) {
  Parsed& p = wk.p;
  p.cmd = 0;
  p.originator = p.token = p.alt = p.type = p.message = p.dtype = p.area = Str();
  p.has_lat = p.has_lon = p.has_elev = p.has_date = p.us = p.has_us = false;
  p.lat = p.lon = p.elev = 0;
  p.date = 0;
  p.mx.clear();
  p.meta.clear();
  auto emit = [&](int kind, const Str& key, const uint8_t* v, size_t vn, uint64_t sub, bool in_arena) {
    RecRef r;
    const int32_t part = key.n ? sw_partition_for_key(key.p, (int32_t)key.n, parts[kind] > 0 ? parts[kind] : 1) : -1;
    r.order = order_of(kind, part, rank, sub);
    r.key = key.p;
    r.klen = key.n;
    r.worker = wid;
    if (in_arena) {
      r.voff = (uint64_t)(v - wk.arena.data());
    } else {                                  // raw payload bytes: copy into the arena
      r.voff = wk.arena.size();
      wk.arena.raw(v, vn);
    }
    r.vlen = vn;
    wk.recs.push_back(r);
  };
  const bool ok = parse(raw, s, e, &p);
  if (!ok || st == 4) {
    emit(RK_FAILED, Str(), raw + s, e - s, 0, false);
    return;
  }
  const size_t v0 = wk.arena.size();
  if ((st == SW_ST_CONTROL || st == SW_ST_RECHECK) &&
      (p.cmd == SW_CMD_SEND_DEVICE_MEASUREMENTS || p.cmd == SW_CMD_SEND_DEVICE_LOCATION ||
       p.cmd == SW_CMD_SEND_DEVICE_ALERT)) {
    // an event the engine handed back -- SW_EV_OVERSIZE (strings past its 16-bit lengths) or an
    // alternate id the store-backed filter may hold (SW_ST_RECHECK): the whole payload goes to the
    // host, which decodes it onto the per-event path (stored whole there, deduplicated against the
    // event store by alternate id)
    emit(RK_CONTROL, p.token, raw + s, e - s, 0, false);
    return;
  }
  if (p.cmd == SW_CMD_SEND_REGISTRATION) {
    W& reg = wk.reg;
    reg.clear();
    if (p.dtype.n) reg.opt_str(1, p.dtype);
    if (p.area.n) reg.opt_str(3, p.area);
    map_entries(reg, 4, p.meta);
    W& w = wk.arena;                           // GDeviceRegistationPayload
    if (source.n) w.str(1, source);
    w.str(2, p.token);
    if (p.originator.has) w.opt_str(3, p.originator);
    if (reg.size()) w.sub(4, reg);
    emit(RK_REGISTRATION, p.token, w.data() + v0, w.size() - v0, 0, true);
  } else if (p.cmd == SW_CMD_SEND_DEVICE_MEASUREMENTS) {
    const size_t n = p.mx.size();
    for (size_t i = 0; i < n; ++i) {
      Str alt = p.alt;
      if (alt.has && n > 1) {                // ProtobufDecoder: "<alternateId>:<index>" per measurement
        wk.alt.assign((const char*)alt.p, alt.n);
        wk.alt += ':';
        wk.alt += std::to_string(i);
        alt.p = (const uint8_t*)wk.alt.data();
        alt.n = (uint32_t)wk.alt.size();
      }
      event_header(wk.h, p, alt);
      W& m = wk.m;                            // GDeviceMeasurementCreateRequest
      m.clear();
      if (p.mx[i].name.n) m.str(1, p.mx[i].name);
      uint64_t u;
      memcpy(&u, &p.mx[i].value, 8);
      if (u) m.dbl(2, p.mx[i].value);
      m.sub(3, wk.h);
      const size_t a = wk.arena.size();
      inbound(wk.arena, source, p, 1, m);
      emit(RK_UNREGISTERED, p.token, wk.arena.data() + a, wk.arena.size() - a, i, true);
    }
  } else if (p.cmd == SW_CMD_SEND_DEVICE_LOCATION) {
    event_header(wk.h, p, p.alt);
    W& m = wk.m;                              // GDeviceLocationCreateRequest
    m.clear();
    m.opt_dbl(1, p.lat);
    m.opt_dbl(2, p.lon);
    if (p.has_elev) m.opt_dbl(3, p.elev);
    m.sub(4, wk.h);
    inbound(wk.arena, source, p, 3, m);
    emit(RK_UNREGISTERED, p.token, wk.arena.data() + v0, wk.arena.size() - v0, 0, true);
  } else if (p.cmd == SW_CMD_SEND_DEVICE_ALERT) {
    event_header(wk.h, p, p.alt);
    W& m = wk.m;                              // GDeviceAlertCreateRequest (source Device, level Info)
    m.clear();
    if (p.type.n) m.str(3, p.type);
    if (p.message.n) m.str(4, p.message);
    m.sub(5, wk.h);
    inbound(wk.arena, source, p, 2, m);
    emit(RK_UNREGISTERED, p.token, wk.arena.data() + v0, wk.arena.size() - v0, 0, true);
  } else {
    emit(RK_CONTROL, p.token, raw + s, e - s, 0, false);
  }
}

// Route the rejected messages of one raw batch (see the entry points below for the inputs).
// Output: records grouped by (kind, partition) -- within a group in batch order, so per-key order
// is preserved -- with rec[i] = (kind, partition, key length, value length) and the keys / values
// concatenated in that order in key_heap / val_heap.  Returns the record count, or -1 when a heap or
// rec is too small (need[0] = records, need[1] = key bytes, need[2] = value bytes: call again with
// those).  Payloads are parsed on up to 8 threads; duplicates never get here (dedup drops them).
struct Hit {
  uint64_t key;            // payload start << 32 | end in the batch: order and identity
  uint32_t ps, pe;         // where its bytes are in `raw` (the batch, or a compact copy)
  uint8_t st;
  bool operator<(const Hit& o) const { return key < o.key; }
};

static int64_t route_hits(const uint8_t* raw, std::vector<Hit>& hit, const char* source_id,
                          const int32_t* parts, int32_t* rec, int64_t rec_cap, uint8_t* key_heap, int64_t key_cap,
                          uint8_t* val_heap, int64_t val_cap, int64_t* need, int64_t* payloads_out) {
  // one hit per affected payload after the dedupe below; sorted by batch position, so a payload's
  // rank in `hit` is its batch order
  std::sort(hit.begin(), hit.end());
  hit.erase(std::unique(hit.begin(), hit.end(), [](const Hit& a, const Hit& b) { return a.key == b.key; }),
            hit.end());
  if (payloads_out) *payloads_out = (int64_t)hit.size();
  Str source;
  source.p = (const uint8_t*)source_id;
  source.n = (uint32_t)strlen(source_id);
  const size_t nh = hit.size();
  static const int max_t = getenv("SW_ROUTE_THREADS") ? std::max(1, atoi(getenv("SW_ROUTE_THREADS"))) : 8;
  const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)max_t, nh / 512));
  static thread_local std::vector<Worker> tl_workers;
  std::vector<Worker>& workers = tl_workers;   // the caller's: worker threads must not see their own
  if ((int)workers.size() < T) workers.resize((size_t)T);
  auto work = [&workers, &hit, nh, T, raw, &source, parts](int t) {
    Worker& wk = workers[(size_t)t];
    wk.arena.clear();
    wk.recs.clear();
    const size_t a = nh * (size_t)t / (size_t)T, b = nh * (size_t)(t + 1) / (size_t)T;
    // payloads are scattered over the batch: prefetch a few ahead so their misses overlap
    constexpr size_t AHEAD = 16;
    for (size_t i = a; i < b && i < a + AHEAD; ++i) {
      __builtin_prefetch(raw + hit[i].ps);
      __builtin_prefetch(raw + hit[i].ps + 64);
    }
    for (size_t i = a; i < b; ++i) {
      if (i + AHEAD < b) {
        const uint8_t* q = raw + hit[i + AHEAD].ps;
        __builtin_prefetch(q);
        __builtin_prefetch(q + 64);
      }
      route_one(wk, (uint32_t)t, raw, hit[i].ps, hit[i].pe, hit[i].st, i, source, parts);
    }
  };
  if (T == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
  }
  // stable counting sort into (kind, partition) groups: workers hold consecutive hit ranges and
  // emit in hit order, so walking them in order is batch order
  int32_t pmax = 1;
  for (int k = 0; k < 4; ++k) pmax = std::max(pmax, parts[k]);
  const size_t nb = (size_t)4 * (size_t)pmax;
  std::vector<int64_t> cnt(nb + 1, 0), kbytes(nb + 1, 0), vbytes(nb + 1, 0);
  auto bucket = [pmax](const RecRef& r) {
    const int kind = (int)(r.order >> 62);
    const int32_t part = r.klen ? (int32_t)((r.order >> 46) & 0xffff) : 0;
    return (size_t)kind * (size_t)pmax + (size_t)std::min(part, pmax - 1);
  };
  int64_t n = 0, kb = 0, vb = 0;
  for (int t = 0; t < T; ++t)
    for (const RecRef& r : workers[(size_t)t].recs) {
      const size_t bk = bucket(r);
      ++cnt[bk + 1];
      kbytes[bk + 1] += r.klen;
      vbytes[bk + 1] += (int64_t)r.vlen;
      ++n;
      kb += r.klen;
      vb += (int64_t)r.vlen;
    }
  need[0] = n;
  need[1] = kb;
  need[2] = vb;
  if (n > rec_cap || kb > key_cap || vb > val_cap) return -1;
  for (size_t b = 0; b < nb; ++b) {
    cnt[b + 1] += cnt[b];
    kbytes[b + 1] += kbytes[b];
    vbytes[b + 1] += vbytes[b];
  }
  // every record's slot and byte offsets: a prefix within its bucket
  std::vector<int64_t> ri(cnt.begin(), cnt.end() - 1), ko(kbytes.begin(), kbytes.end() - 1),
      vo(vbytes.begin(), vbytes.end() - 1);
  for (int t = 0; t < T; ++t) {
    const Worker& wk = workers[(size_t)t];
    for (const RecRef& r : wk.recs) {
      const size_t bk = bucket(r);
      const int64_t i = ri[bk]++;
      rec[4 * i] = (int32_t)(r.order >> 62);
      rec[4 * i + 1] = r.klen ? (int32_t)((r.order >> 46) & 0xffff) : -1;
      rec[4 * i + 2] = (int32_t)r.klen;
      rec[4 * i + 3] = (int32_t)r.vlen;
      if (r.klen) memcpy(key_heap + ko[bk], r.key, r.klen);
      memcpy(val_heap + vo[bk], wk.arena.data() + r.voff, r.vlen);
      ko[bk] += r.klen;
      vo[bk] += (int64_t)r.vlen;
    }
  }
  return n;
}

extern "C" {

// rej_off: any byte offset inside the rejected event's payload (binary search over offs).
int64_t sw_route_rejects(const uint8_t* raw, const uint32_t* offs, int64_t n_msgs, const uint32_t* rej_off,
                         const uint8_t* rej_st, int64_t n_rej, const char* source_id, const int32_t* parts,
                         int32_t* rec, int64_t rec_cap, uint8_t* key_heap, int64_t key_cap, uint8_t* val_heap,
                         int64_t val_cap, int64_t* need, int64_t* payloads_out) {
  std::vector<Hit> hit;
  hit.reserve((size_t)n_rej);
  for (int64_t i = 0; i < n_rej; ++i) {
    const uint8_t st = rej_st[i];
    if (st == 3 || st == 0) continue;
    const uint32_t* it = std::upper_bound(offs, offs + n_msgs + 1, rej_off[i]);
    const int64_t m = (int64_t)(it - offs) - 1;
    if (m < 0 || m >= n_msgs) continue;
    hit.push_back({((uint64_t)offs[m] << 32) | offs[m + 1], offs[m], offs[m + 1], st});
  }
  return route_hits(raw, hit, source_id, parts, rec, rec_cap, key_heap, key_cap, val_heap, val_cap, need,
                    payloads_out);
}

// refs: n x (payload start, payload end, status | src_rank << 8, copy offset) as the MI355X step
// snapshot them (k_reject_refs).  Payloads are parsed from `compact` at their copy offset, or from
// the raw batch `raw` (may be null) when the copy did not fit (offset ~0).  Only refs whose
// src_rank == rank are routed; recheck packages (bit 16 of the status word, several ranks:
// pipeline/recheck.py settles them) are not.
int64_t sw_route_refs(const uint8_t* compact, const uint8_t* raw, const uint32_t* refs, int64_t n, int32_t rank,
                      const char* source_id, const int32_t* parts, int32_t* rec, int64_t rec_cap, uint8_t* key_heap,
                      int64_t key_cap, uint8_t* val_heap, int64_t val_cap, int64_t* need, int64_t* payloads_out) {
  std::vector<Hit> hit, spill;
  hit.reserve((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t s = refs[4 * i], e = refs[4 * i + 1], st = refs[4 * i + 2] & 0xff, src = refs[4 * i + 2] >> 8;
    const uint32_t c = refs[4 * i + 3];
    if (refs[4 * i + 2] & 0x10000u) continue;          // a recheck package: settled by its owner
    if (st == 3 || st == 0 || (int32_t)src != rank || e <= s) continue;
    if (c != 0xffffffffu) hit.push_back({((uint64_t)s << 32) | e, c, c + (e - s), (uint8_t)st});
    else spill.push_back({((uint64_t)s << 32) | e, s, e, (uint8_t)st});
  }
  if (spill.empty() || !raw)
    return route_hits(compact, hit, source_id, parts, rec, rec_cap, key_heap, key_cap, val_heap, val_cap, need,
                      payloads_out);
  // rare: the compact buffer overflowed -- those payloads come from the raw batch (routed with the
  // raw base; all offsets rebased onto it by copying the compact ones there is not possible, so
  // the two sets are routed in one pass over a merged view: copies first, then the raw spill)
  std::vector<uint8_t> merged;
  size_t total = 0;
  for (const Hit& h : hit) total = std::max<size_t>(total, h.pe);
  merged.resize(total + 64);
  if (total) memcpy(merged.data(), compact, total);
  for (Hit& h : spill) {
    const size_t at = merged.size();
    merged.insert(merged.end(), raw + h.ps, raw + h.pe);
    h.pe = (uint32_t)(at + (h.pe - h.ps));
    h.ps = (uint32_t)at;
    hit.push_back(h);
  }
  merged.resize(merged.size() + 64);
  return route_hits(merged.data(), hit, source_id, parts, rec, rec_cap, key_heap, key_cap, val_heap, val_cap, need,
                    payloads_out);
}

}  // extern "C"
