// JSON device requests -> the device protobuf wire format, natively.
//
// Reference: JSON payloads are decoded per event (JsonDeviceRequestDecoder, Jackson) and each
// decoded request then travels the per-event inbound path.  Here a JSON event source that
// forwards raw batches to the fused engine transcodes each payload into the same
// `varint(len(Header)) Header varint(len(Body)) Body` bytes a protobuf device sends
// (sitewhere_amd/models/wire.py): the MI355X decoder, dedup, state, rules and durable store then
// handle JSON devices exactly like protobuf ones.
//
// Transcoded: {"deviceToken", "type": DeviceMeasurement | DeviceLocation | DeviceAlert,
// "originator"?, "request": {...}} whose request the engine path represents exactly (integer
// eventDate, metadata of string values, alerts at level Info from source Device).  Anything else returns a
// negative code and the caller keeps the per-event path for that payload, so no request changes
// meaning by being transcoded.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <utility>
#include <vector>

namespace {

// A string value: a span of the payload when it has no escapes, else of the per-thread unescape
// arena (never longer than the payload: every escape shrinks when decoded).
struct Str {
  const char* p = nullptr;
  uint32_t n = 0;
  bool has = false;
  bool eq(const char* w, uint32_t wn) const { return n == wn && memcmp(p, w, wn) == 0; }
};

struct Req {
  Str token, type, originator;
  // request fields
  Str name, alt, atype, message, level, source;
  double value = 0, lat = 0, lon = 0, elev = 0;
  bool has_value = false, has_lat = false, has_lon = false, has_elev = false;
  int64_t date = 0;
  bool has_date = false, date_bad = false;
  int update = -1;          // -1 absent, 0/1
  bool meta_bad = false, bad = false, value_bad = false;
  std::vector<std::pair<Str, Str>>* md = nullptr;   // metadata entries in document order
};

struct P {
  const char* p;
  const char* e;
  char* arena;              // unescaped strings are written here
  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  bool lit(const char* w, size_t n) {
    if ((size_t)(e - p) < n || memcmp(p, w, n) != 0) return false;
    p += n;
    return true;
  }
  static char* utf8(char* o, uint32_t c) {
    if (c < 0x80) {
      *o++ = (char)c;
    } else if (c < 0x800) {
      *o++ = (char)(0xc0 | (c >> 6));
      *o++ = (char)(0x80 | (c & 0x3f));
    } else if (c < 0x10000) {
      *o++ = (char)(0xe0 | (c >> 12));
      *o++ = (char)(0x80 | ((c >> 6) & 0x3f));
      *o++ = (char)(0x80 | (c & 0x3f));
    } else {
      *o++ = (char)(0xf0 | (c >> 18));
      *o++ = (char)(0x80 | ((c >> 12) & 0x3f));
      *o++ = (char)(0x80 | ((c >> 6) & 0x3f));
      *o++ = (char)(0x80 | (c & 0x3f));
    }
    return o;
  }
  bool hex4(uint32_t* v) {
    if (e - p < 4) return false;
    uint32_t x = 0;
    for (int i = 0; i < 4; ++i) {
      char c = p[i];
      x <<= 4;
      if (c >= '0' && c <= '9') x |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') x |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') x |= (uint32_t)(c - 'A' + 10);
      else return false;
    }
    p += 4;
    *v = x;
    return true;
  }
  bool str(Str* out) {
    if (p >= e || *p != '"') return false;
    const char* s = ++p;
    while (p < e && *p != '"' && *p != '\\' && (unsigned char)*p >= 0x20) ++p;   // the common case
    if (p >= e || (unsigned char)*p < 0x20) return false;
    if (*p == '"') {
      if (out) { out->p = s; out->n = (uint32_t)(p - s); }
      ++p;
      return true;
    }
    char* o0 = arena;                     // has escapes: unescape into the arena
    memcpy(o0, s, (size_t)(p - s));
    char* o = o0 + (p - s);
    while (p < e) {
      char c = *p++;
      if (c == '"') {
        if (out) { out->p = o0; out->n = (uint32_t)(o - o0); }
        arena = o;
        return true;
      }
      if ((unsigned char)c < 0x20) return false;
      if (c != '\\') { *o++ = c; continue; }
      if (p >= e) return false;
      char x = *p++;
      uint32_t u;
      switch (x) {
        case '"': case '\\': case '/': *o++ = x; break;
        case 'b': *o++ = '\b'; break;
        case 'f': *o++ = '\f'; break;
        case 'n': *o++ = '\n'; break;
        case 'r': *o++ = '\r'; break;
        case 't': *o++ = '\t'; break;
        case 'u':
          if (!hex4(&u)) return false;
          if (u >= 0xd800 && u < 0xdc00) {           // surrogate pair
            uint32_t lo;
            if (!(e - p >= 2 && p[0] == '\\' && p[1] == 'u')) return false;
            p += 2;
            if (!hex4(&lo) || lo < 0xdc00 || lo >= 0xe000) return false;
            u = 0x10000 + ((u - 0xd800) << 10) + (lo - 0xdc00);
          } else if (u >= 0xdc00 && u < 0xe000) {
            return false;
          }
          o = utf8(o, u);
          break;
        default: return false;
      }
    }
    return false;
  }
  // number: *is_int when it has no fraction / exponent
  bool num(double* d, int64_t* i, bool* is_int) {
    const char* s = p;
    if (p < e && *p == '-') ++p;
    if (p >= e || *p < '0' || *p > '9') return false;
    if (*p == '0') ++p;
    else while (p < e && *p >= '0' && *p <= '9') ++p;
    bool integer = true;
    if (p < e && *p == '.') {
      integer = false;
      ++p;
      if (p >= e || *p < '0' || *p > '9') return false;
      while (p < e && *p >= '0' && *p <= '9') ++p;
    }
    if (p < e && (*p == 'e' || *p == 'E')) {
      integer = false;
      ++p;
      if (p < e && (*p == '+' || *p == '-')) ++p;
      if (p >= e || *p < '0' || *p > '9') return false;
      while (p < e && *p >= '0' && *p <= '9') ++p;
    }
    const size_t len = (size_t)(p - s);
    *is_int = integer && len <= 18;
    if (*is_int) {                      // exact: digits only, at most 18 of them
      int64_t v = 0;
      const char* q = s[0] == '-' ? s + 1 : s;
      for (; q < p; ++q) v = v * 10 + (*q - '0');
      *i = s[0] == '-' ? -v : v;
      *d = (double)*i;
      if (len <= 16) return true;       // |v| < 2^53 when it has at most 15 digits + sign
    }
    char buf[64];                        // the grammar-checked span, NUL-terminated for strtod
    if (len < sizeof(buf)) {
      memcpy(buf, s, len);
      buf[len] = 0;
      *d = strtod(buf, nullptr);
    } else {
      std::string t(s, len);
      *d = strtod(t.c_str(), nullptr);
    }
    return true;
  }
  bool skip(int depth = 0) {          // any value
    if (depth > 64) return false;
    ws();
    if (p >= e) return false;
    if (*p == '"') return str(nullptr);
    if (*p == '{' || *p == '[') {
      const char close = *p == '{' ? '}' : ']';
      const bool obj = *p == '{';
      ++p;
      ws();
      if (p < e && *p == close) { ++p; return true; }
      while (true) {
        ws();
        if (obj) {
          if (!str(nullptr)) return false;
          ws();
          if (p >= e || *p != ':') return false;
          ++p;
        }
        if (!skip(depth + 1)) return false;
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == close) { ++p; return true; }
        return false;
      }
    }
    if (lit("true", 4) || lit("false", 5) || lit("null", 4)) return true;
    double d;
    int64_t i;
    bool it;
    return num(&d, &i, &it);
  }
};

#define KEY(k, lit_) ((k).eq(lit_, sizeof(lit_) - 1))

bool parse_request(P& q, Req& r) {
  q.ws();
  if (q.p >= q.e || *q.p != '{') return false;
  ++q.p;
  q.ws();
  if (q.p < q.e && *q.p == '}') { ++q.p; return true; }
  Str key;
  while (true) {
    q.ws();
    if (!q.str(&key)) return false;
    q.ws();
    if (q.p >= q.e || *q.p != ':') return false;
    ++q.p;
    q.ws();
    Str* target = nullptr;
    double* num_target = nullptr;
    bool* num_has = nullptr;
    if (KEY(key, "name")) target = &r.name;
    else if (KEY(key, "alternateId")) target = &r.alt;
    else if (KEY(key, "type")) target = &r.atype;
    else if (KEY(key, "message")) target = &r.message;
    else if (KEY(key, "level")) target = &r.level;
    else if (KEY(key, "source")) target = &r.source;
    else if (KEY(key, "value")) { num_target = &r.value; num_has = &r.has_value; }
    else if (KEY(key, "latitude")) { num_target = &r.lat; num_has = &r.has_lat; }
    else if (KEY(key, "longitude")) { num_target = &r.lon; num_has = &r.has_lon; }
    else if (KEY(key, "elevation")) { num_target = &r.elev; num_has = &r.has_elev; }
    const bool is_date = !target && !num_target && KEY(key, "eventDate");
    if (target) {
      if (q.lit("null", 4)) {
      } else if (q.str(target)) {
        target->has = true;
      } else {
        return false;
      }
    } else if (num_target || is_date) {
      double d = 0;
      int64_t iv = 0;
      bool it = false;
      if (q.lit("null", 4)) {
      } else if (q.num(&d, &iv, &it)) {
        if (num_target) { *num_target = d; *num_has = true; }
        else if (it) { r.date = iv; r.has_date = true; }
        else r.date_bad = true;
      } else {
        if (num_target == &r.value) r.value_bad = true;   // e.g. a numeric string: the per-event path converts it
        else if (is_date) r.date_bad = true;
        else r.bad = true;
        if (!q.skip()) return false;
      }
    } else if (KEY(key, "updateState")) {
      if (q.lit("true", 4)) r.update = 1;
      else if (q.lit("false", 5)) r.update = 0;
      else if (q.lit("null", 4)) {}
      else { r.bad = true; if (!q.skip()) return false; }
    } else if (KEY(key, "metadata")) {
      // an object of string values -> repeated Metadata{name, value} (the protobuf a device sends);
      // any other value type stays on the per-event path
      r.md->clear();
      r.meta_bad = false;
      if (q.lit("null", 4)) {
      } else if (q.p < q.e && *q.p == '{') {
        ++q.p;
        q.ws();
        if (q.p < q.e && *q.p == '}') {
          ++q.p;
        } else {
          while (true) {
            Str mk, mv;
            q.ws();
            if (!q.str(&mk)) return false;
            q.ws();
            if (q.p >= q.e || *q.p != ':') return false;
            ++q.p;
            q.ws();
            if (q.p < q.e && *q.p == '"') {
              if (!q.str(&mv)) return false;
              r.md->push_back({mk, mv});
            } else {
              r.meta_bad = true;
              if (!q.skip()) return false;
            }
            q.ws();
            if (q.p < q.e && *q.p == ',') { ++q.p; continue; }
            if (q.p < q.e && *q.p == '}') { ++q.p; break; }
            return false;
          }
        }
      } else {
        r.meta_bad = true;
        if (!q.skip()) return false;
      }
    } else {
      if (!q.skip()) return false;                     // fields the engine path does not use
    }
    q.ws();
    if (q.p < q.e && *q.p == ',') { ++q.p; continue; }
    if (q.p < q.e && *q.p == '}') { ++q.p; return true; }
    return false;
  }
}

// strict UTF-8 (the per-event path decodes payloads as UTF-8 and rejects anything else)
bool valid_utf8(const unsigned char* s, int64_t n) {
  int64_t i = 0;
  while (i < n) {
    if (i + 8 <= n) {                                  // 8 ASCII bytes at a time
      uint64_t w;
      memcpy(&w, s + i, 8);
      if ((w & 0x8080808080808080ull) == 0) { i += 8; continue; }
    }
    const unsigned char c = s[i];
    if (c < 0x80) { ++i; continue; }
    const int k = (c & 0xe0) == 0xc0 ? 1 : (c & 0xf0) == 0xe0 ? 2 : (c & 0xf8) == 0xf0 ? 3 : -1;
    if (k < 0 || i + k >= n) return false;
    uint32_t cp = c & (k == 1 ? 0x1f : k == 2 ? 0x0f : 0x07);
    for (int j = 1; j <= k; ++j) {
      if ((s[i + j] & 0xc0) != 0x80) return false;
      cp = (cp << 6) | (s[i + j] & 0x3f);
    }
    if ((k == 1 && cp < 0x80) || (k == 2 && cp < 0x800) || (k == 3 && (cp < 0x10000 || cp > 0x10ffff)) ||
        (cp >= 0xd800 && cp < 0xe000))
      return false;
    i += k + 1;
  }
  return true;
}

bool parse_top(const char* s, int64_t n, Req& r, char* arena) {
  if (!valid_utf8((const unsigned char*)s, n)) return false;
  P q{s, s + n, arena};
  q.ws();
  if (q.p >= q.e || *q.p != '{') return false;
  ++q.p;
  Str key;
  bool have_req = false;
  while (true) {
    q.ws();
    if (q.p < q.e && *q.p == '}' && !have_req && !r.token.has) return false;
    if (!q.str(&key)) return false;
    q.ws();
    if (q.p >= q.e || *q.p != ':') return false;
    ++q.p;
    q.ws();
    Str* t = KEY(key, "deviceToken") ? &r.token : KEY(key, "type") ? &r.type
           : KEY(key, "originator") ? &r.originator : nullptr;
    if (t) {
      if (q.lit("null", 4)) {
        t->has = false;
      } else {
        if (!q.str(t)) return false;
        t->has = true;
      }
    } else if (KEY(key, "request")) {
      if (!parse_request(q, r)) return false;
      have_req = true;
    } else {
      if (!q.skip()) return false;
    }
    q.ws();
    if (q.p < q.e && *q.p == ',') { ++q.p; continue; }
    if (q.p < q.e && *q.p == '}') {
      ++q.p;
      q.ws();
      return q.p == q.e && have_req;
    }
    return false;
  }
}

// ---- protobuf writer: straight into a caller buffer already checked to be large enough
inline int vlen(uint64_t v) {
  int k = 1;
  while (v >= 0x80) { v >>= 7; ++k; }
  return k;
}
struct W {
  uint8_t* o;
  void varint(uint64_t v) {
    while (v >= 0x80) { *o++ = (uint8_t)(v | 0x80); v >>= 7; }
    *o++ = (uint8_t)v;
  }
  void tag(int f, int wt) { varint(((uint64_t)f << 3) | (uint64_t)wt); }
  void bytes(const char* p, uint32_t n) { memcpy(o, p, n); o += n; }
  void str(int f, const Str& s) { tag(f, 2); varint(s.n); bytes(s.p, s.n); }
  void fixed(int f, const void* v) { tag(f, 1); memcpy(o, v, 8); o += 8; }
  void boolean(int f, bool v) { tag(f, 0); *o++ = v ? 1 : 0; }
};
inline int str_size(int f, const Str& s) { return vlen((uint64_t)f << 3) + vlen(s.n) + (int)s.n; }

}  // namespace

extern "C" {

// Transcode one JSON device request.  Returns the protobuf length written to out, or
//   -1 invalid JSON / not a device request (the per-event decoder reports it),
//   -2 valid but not representable on the engine path (non-string metadata, a level, a string date ...),
//   -3 out too small.
int64_t sw_json_to_pb(const char* in, int64_t n, uint8_t* out, int64_t cap) {
  static thread_local std::vector<char> arena;
  if (arena.size() < (size_t)n + 8) arena.resize((size_t)n + 8);
  static thread_local std::vector<std::pair<Str, Str>> md;
  Req r;
  r.md = &md;
  md.clear();
  if (!parse_top(in, n, r, arena.data()) || !r.token.has || r.token.n == 0 || !r.type.has) return -1;
  if (r.bad || r.date_bad || r.value_bad || r.meta_bad) return -2;
  // metadata entries: Metadata{1: name, 2: value}, each a length-delimited field of the body
  int meta = 0;
  for (const auto& kv : md) {
    const int ent = str_size(1, kv.first) + str_size(2, kv.second);
    meta += 1 + vlen((uint64_t)ent) + ent;
  }
  static const Str empty{"", 0, true};
  // sizes first (body, then header), so the message is written once, in place
  int command, body = str_size(1, r.token), meas = 0;
  if (KEY(r.type, "DeviceMeasurement")) {
    if (!r.name.has || !r.has_value) return -2;
    command = 5;
    meas = str_size(1, r.name) + 9;
    body += 1 + vlen((uint64_t)meas) + meas + meta;
    if (r.has_date) body += 9;
    if (r.update >= 0) body += 2;
  } else if (KEY(r.type, "DeviceLocation")) {
    if (!r.has_lat || !r.has_lon) return -2;
    command = 3;
    body += 18 + (r.has_elev ? 9 : 0) + (r.has_date ? 9 : 0) + (r.update >= 0 ? 2 : 0) + meta;
  } else if (KEY(r.type, "DeviceAlert")) {
    if ((r.level.has && !KEY(r.level, "Info")) || (r.source.has && !KEY(r.source, "Device"))) return -2;
    command = 4;
    body += str_size(2, r.atype.has ? r.atype : empty) + str_size(3, r.message.has ? r.message : empty);
    body += (r.has_date ? 9 : 0) + (r.update >= 0 ? 2 : 0) + meta;
  } else {
    return -2;                                         // registrations, acks, streams ...: per-event path
  }
  if (r.alt.has) body += str_size(15, r.alt);
  const int hdr = 2 + (r.originator.has ? str_size(2, r.originator) : 0);
  const int64_t total = vlen((uint64_t)hdr) + hdr + vlen((uint64_t)body) + body;
  if (total > cap) return -3;
  W w{out};
  auto put_meta = [&](int f) {
    for (const auto& kv : md) {
      w.tag(f, 2);
      w.varint((uint64_t)(str_size(1, kv.first) + str_size(2, kv.second)));
      w.str(1, kv.first);
      w.str(2, kv.second);
    }
  };
  w.varint((uint64_t)hdr);
  w.tag(1, 0);
  w.varint((uint64_t)command);
  if (r.originator.has) w.str(2, r.originator);
  w.varint((uint64_t)body);
  w.str(1, r.token);
  if (command == 5) {
    w.tag(2, 2);
    w.varint((uint64_t)meas);
    w.str(1, r.name);
    w.fixed(2, &r.value);
    if (r.has_date) w.fixed(3, &r.date);
    put_meta(4);
    if (r.update >= 0) w.boolean(5, r.update == 1);
  } else if (command == 3) {
    w.fixed(2, &r.lat);
    w.fixed(3, &r.lon);
    if (r.has_elev) w.fixed(4, &r.elev);
    if (r.has_date) w.fixed(5, &r.date);
    put_meta(6);
    if (r.update >= 0) w.boolean(7, r.update == 1);
  } else {
    w.str(2, r.atype.has ? r.atype : empty);
    w.str(3, r.message.has ? r.message : empty);
    if (r.has_date) w.fixed(4, &r.date);
    put_meta(5);
    if (r.update >= 0) w.boolean(6, r.update == 1);
  }
  if (r.alt.has) w.str(15, r.alt);
  return (int64_t)(w.o - out);
}

// Batch form: payloads heap + offsets[n + 1] -> protobuf heap + out_offs[n + 1]; status[i] = 0 when
// payload i was transcoded, else its negative code (its out range is empty).  Returns bytes written,
// or -3 when out_cap is too small.
int64_t sw_json_to_pb_batch(const char* heap, const int64_t* offs, int64_t n, uint8_t* out, int64_t out_cap,
                            int64_t* out_offs, int8_t* status) {
  int64_t pos = 0;
  out_offs[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    int64_t w = sw_json_to_pb(heap + offs[i], offs[i + 1] - offs[i], out + pos, out_cap - pos);
    if (w == -3) return -3;
    status[i] = w < 0 ? (int8_t)w : 0;
    if (w > 0) pos += w;
    out_offs[i + 1] = pos;
  }
  return pos;
}

}  // extern "C"
