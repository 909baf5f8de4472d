// Enriched events of a decoded durable block as the reference's outbound JSON, natively.
//
// Outbound connectors publish every event they keep as {"event": <the event>, "context": <the
// enrichment context>} (services/outbound_connectors.py event_json; reference OutboundPayloadEnrichment
// -Logic.java:54-92 + the connectors' JSON marshalling, e.g. MqttOutboundConnector.java:257-258).
// Materialising each kept row as a Python event object and json.dumps'ing it ran ~8K events/s
// (profiles/r5_consumers); here the selected rows of a decoded block (persistence/segments.py
// decode_block: columns + string heap) are written straight to JSON bytes -- byte for byte what
// json.dumps(event_json(materialize_row(...), context)) gives (tests/test_row_json.py), including
// float repr and ensure_ascii escaping -- plus, per row, an MQTT topic from a template.  MQTT QoS 0
// PUBLISH packets can be framed here too (one socket write per batch).
//
// Dictionaries come in as string tables: offsets (n + 1, int64) into a byte heap, entry k =
// heap[off[k] .. off[k + 1]), a None entry marked in a presence byte array.
#include <stdint.h>
#include <string.h>

#include <charconv>
#include <utility>
#include <vector>

namespace {

struct StrTab {
  const uint8_t* heap;
  const int64_t* off;
  const uint8_t* present;  // null: every entry present
  int64_t n;
  bool has(int64_t k) const { return k >= 0 && k < n && (!present || present[k]); }
  std::pair<const uint8_t*, int64_t> get(int64_t k) const { return {heap + off[k], off[k + 1] - off[k]}; }
};

struct Out {                                    // bounded writer: counts past the end, writes nothing there
  uint8_t* b;
  int64_t cap;
  int64_t n = 0;
  void put(const void* x, size_t k) {
    if (n + (int64_t)k <= cap) memcpy(b + n, x, k);
    n += (int64_t)k;
  }
  void lit(const char* x) { put(x, strlen(x)); }
  void ch(char c) {
    if (n < cap) b[n] = (uint8_t)c;
    ++n;
  }
  void i64(int64_t v) {
    char t[24];
    auto r = std::to_chars(t, t + sizeof(t), v);
    put(t, (size_t)(r.ptr - t));
  }
  // float.__repr__ (shortest round trip; fixed for 1e-4 <= |v| < 1e16, else d.ddde+XX), as json.dumps
  void dbl(double v) {
    if (v != v) { lit("NaN"); return; }
    if (v == __builtin_inf()) { lit("Infinity"); return; }
    if (v == -__builtin_inf()) { lit("-Infinity"); return; }
    char b[64];
    auto r = std::to_chars(b, b + sizeof(b), v, std::chars_format::scientific);
    const char* p = b;
    const char* end = r.ptr;
    bool neg = false;
    if (*p == '-') { neg = true; ++p; }
    char dig[32];
    int nd = 0;
    const char* q = p;
    for (; q < end && *q != 'e'; ++q)
      if (*q != '.') dig[nd++] = *q;
    int e = 0;
    if (q < end) {
      ++q;
      std::from_chars(*q == '+' ? q + 1 : q, end, e);
    }
    while (nd > 1 && dig[nd - 1] == '0') --nd;  // to_chars is already shortest; defensive
    if (neg) ch('-');
    if (e >= -5 && e < 16) {                     // repr switches to exponent below 1e-4 (e < -4)
      if (e < -4) goto sci;
      if (e < 0) {
        lit("0.");
        for (int k = 0; k < -e - 1; ++k) ch('0');
        put(dig, (size_t)nd);
      } else {
        for (int k = 0; k <= e; ++k) ch(k < nd ? dig[k] : '0');
        ch('.');
        if (nd > e + 1) put(dig + e + 1, (size_t)(nd - e - 1));
        else ch('0');
      }
      return;
    }
  sci:
    ch(dig[0]);
    if (nd > 1) {
      ch('.');
      put(dig + 1, (size_t)(nd - 1));
    }
    ch('e');
    ch(e < 0 ? '-' : '+');
    const int ae = e < 0 ? -e : e;
    if (ae < 10) ch('0');
    i64(ae);
  }
  void hex4(uint32_t u) {
    static const char* H = "0123456789abcdef";
    lit("\\u");
    ch(H[(u >> 12) & 15]); ch(H[(u >> 8) & 15]); ch(H[(u >> 4) & 15]); ch(H[u & 15]);
  }
  void cp(uint32_t c) {  // one code point, ensure_ascii
    if (c == '"') lit("\\\"");
    else if (c == '\\') lit("\\\\");
    else if (c == '\n') lit("\\n");
    else if (c == '\r') lit("\\r");
    else if (c == '\t') lit("\\t");
    else if (c == '\b') lit("\\b");
    else if (c == '\f') lit("\\f");
    else if (c < 0x20 || (c >= 0x7f && c < 0x10000)) {
      if (c < 0x7f) hex4(c);
      else hex4(c);
    } else if (c < 0x7f) ch((char)c);
    else {                                       // astral: a UTF-16 surrogate pair
      const uint32_t v = c - 0x10000;
      hex4(0xd800 | (v >> 10));
      hex4(0xdc00 | (v & 0x3ff));
    }
  }
  // UTF-8 bytes as a JSON string; invalid sequences -> U+FFFD per maximal subpart (Python's
  // decode("utf-8", "replace"))
  void str(const uint8_t* p, int64_t n) {
    ch('"');
    int64_t i = 0;
    while (i < n) {
      int64_t r = i;                               // a run of printable ASCII needing no escape
      while (r < n && p[r] >= 0x20 && p[r] < 0x7f && p[r] != '"' && p[r] != '\\') ++r;
      if (r > i) {
        put(p + i, (size_t)(r - i));
        i = r;
        if (i >= n) break;
      }
      const uint8_t b = p[i];
      if (b < 0x80) { cp(b); ++i; continue; }
      int need = 0;
      uint32_t c = 0, lo = 0x80, hi = 0xbf;
      if (b >= 0xc2 && b <= 0xdf) { need = 1; c = b & 0x1f; }
      else if (b >= 0xe0 && b <= 0xef) {
        need = 2; c = b & 0x0f;
        if (b == 0xe0) lo = 0xa0;
        if (b == 0xed) hi = 0x9f;
      } else if (b >= 0xf0 && b <= 0xf4) {
        need = 3; c = b & 0x07;
        if (b == 0xf0) lo = 0x90;
        if (b == 0xf4) hi = 0x8f;
      } else { cp(0xfffd); ++i; continue; }
      int64_t j = i + 1;
      int got = 0;
      for (; got < need && j < n; ++got, ++j) {
        const uint8_t x = p[j];
        const uint32_t l = got == 0 ? lo : 0x80, h = got == 0 ? hi : 0xbf;
        if (x < l || x > h) break;
        c = (c << 6) | (x & 0x3f);
      }
      if (got == need) { cp(c); i = j; }
      else { cp(0xfffd); i = j; }               // the maximal subpart read so far becomes one U+FFFD
    }
    ch('"');
  }
  void str(const std::pair<const uint8_t*, int64_t>& x) { str(x.first, x.second); }
  void tab(const StrTab& t, int64_t k) {
    if (t.has(k)) str(t.get(k));
    else lit("null");
  }
};

// protobuf varint
bool varint(const uint8_t*& p, const uint8_t* end, uint64_t* v) {
  uint64_t x = 0;
  for (int s = 0; s < 64 && p < end; s += 7) {
    const uint8_t b = *p++;
    x |= (uint64_t)(b & 0x7f) << s;
    if (!(b & 0x80)) { *v = x; return true; }
  }
  return false;
}

// the metadata map of a body's wire span (segments.parse_metadata): Metadata {name = 1; value = 2}
// entries of field `field`; a repeated name keeps its first position and takes the last value
void metadata(Out& o, const uint8_t* p, int64_t n, uint32_t field) {
  struct Ent { const uint8_t* k; int64_t kn; const uint8_t* v; int64_t vn; bool hv; };
  std::vector<Ent> ents;
  const uint8_t* end = p + n;
  while (p < end) {
    uint64_t key, len;
    if (!varint(p, end, &key)) break;
    const uint32_t f = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
    if (wt == 0) { uint64_t d; if (!varint(p, end, &d)) break; continue; }
    if (wt == 1) { p += 8; continue; }
    if (wt == 5) { p += 4; continue; }
    if (wt != 2 || !varint(p, end, &len) || (int64_t)len > end - p) break;
    const uint8_t* e = p;
    p += len;
    if (f != field) continue;
    const uint8_t* ee = e + len;
    const uint8_t* k = nullptr; int64_t kn = 0; const uint8_t* v = nullptr; int64_t vn = 0; bool hv = false;
    while (e < ee) {
      uint64_t k2, l2;
      if (!varint(e, ee, &k2)) break;
      const uint32_t f2 = (uint32_t)(k2 >> 3), w2 = (uint32_t)(k2 & 7);
      if (w2 == 0) { uint64_t d; if (!varint(e, ee, &d)) break; continue; }
      if (w2 == 1) { e += 8; continue; }
      if (w2 == 5) { e += 4; continue; }
      if (w2 != 2 || !varint(e, ee, &l2) || (int64_t)l2 > ee - e) break;
      if (f2 == 1) { k = e; kn = (int64_t)l2; }
      else if (f2 == 2) { v = e; vn = (int64_t)l2; hv = true; }
      e += l2;
    }
    if (!k) continue;
    bool dup = false;
    for (auto& x : ents)
      if (x.kn == kn && !memcmp(x.k, k, (size_t)kn)) { x.v = v; x.vn = vn; x.hv = hv; dup = true; break; }
    if (!dup) ents.push_back({k, kn, v, vn, hv});
  }
  o.ch('{');
  for (size_t i = 0; i < ents.size(); ++i) {
    if (i) o.lit(", ");
    o.str(ents[i].k, ents[i].kn);
    o.lit(": ");
    if (ents[i].hv) o.str(ents[i].v, ents[i].vn);
    else o.lit("\"\"");
  }
  o.ch('}');
}

const char* kTypes[] = {"Measurement", "Location", "Alert", "CommandInvocation", "CommandResponse", "StateChange"};
const char* kLevels[] = {"Info", "Warning", "Error", "Critical"};

}  // namespace

extern "C" {

// Rows `rows[0 .. n)` of decoded block columns (persistence/segments.py decode_block) as outbound
// JSON documents, back to back into `out` (offsets in out_off[n + 1]), and, with a topic template
// (`tpl`: literal bytes with the markers \x01 = device token, \x02 = event type), each row's topic into
// `tout` (offsets tout_off[n + 1]); `block_rows` (optional): each row's row in its block, for its
// event id (default row0 + rows[j]).  asg: 7 strings per assignment index (assignment, device,
// customer, area, asset, device token, device type); names: per name id; rules: per name id, the
// message of a rule-generated alert of that type.  Returns the bytes written to `out`, or -needed
// when `out` / `tout` are too small (nothing usable then), or -1 - i when row i cannot be written
// here (an API-added JSON row: the caller's Python path).
int64_t swjson_rows(const int64_t* rows, int64_t n, const uint8_t* etype, const uint8_t* level, const int64_t* date,
                    const int32_t* asg, const uint16_t* name, const double* v0, const double* v1, const double* v2,
                    const uint8_t* flags, const uint8_t* heap, const int64_t* soff,
                    int64_t boot, int64_t first_seq, int64_t world, int64_t rank, int64_t recv_ms, int64_t row0,
                    const uint8_t* a_heap, const int64_t* a_off, const uint8_t* a_present, int64_t n_asg,
                    const uint8_t* n_heap, const int64_t* n_off, const uint8_t* n_present, int64_t n_names,
                    const uint8_t* r_heap, const int64_t* r_off, const uint8_t* r_present,
                    const uint8_t* tpl, int64_t tpl_len,
                    uint8_t* out, int64_t cap, int64_t* out_off, uint8_t* tout, int64_t tcap, int64_t* tout_off,
                    const int64_t* block_rows) {
  const StrTab A{a_heap, a_off, a_present, n_asg * 7};
  const StrTab N{n_heap, n_off, n_present, n_names};
  const StrTab R{r_heap, r_off, r_present, n_names};
  Out o{out, cap}, t{tout, tout ? tcap : 0};
  char bootx[24];
  const int bl = (int)(std::to_chars(bootx, bootx + sizeof(bootx), (unsigned long long)boot, 16).ptr - bootx);
  for (int64_t j = 0; j < n; ++j) {
    const int64_t i = rows[j];
    const uint8_t f = flags[i];
    const int et = etype[i];
    if ((f & 0x80) || et == 3 || et == 4 || et > 5) return -1 - j;   // SEGF_JSON rows: the Python path
    const int64_t a = asg[i];
    const bool ha = a >= 0 && a < n_asg && A.has(7 * a);   // the assignment's context is known
    auto ctxs = [&](int k) {
      if (ha && A.has(7 * a + k)) o.str(A.get(7 * a + k));
      else o.lit("null");
    };
    out_off[j] = o.n;
    o.lit("{\"event\": {\"id\": \"");
    o.put(bootx, (size_t)bl);
    o.ch('-');
    o.i64((first_seq + (block_rows ? block_rows[j] : row0 + i)) * world + rank);
    o.lit("\", \"alternateId\": ");
    if (f & 0x8) o.str(heap + soff[3 * i], soff[3 * i + 1] - soff[3 * i]);
    else o.lit("null");
    o.lit(", \"eventType\": \"");
    o.lit(kTypes[et]);
    o.lit("\", \"deviceId\": "); ctxs(1);
    o.lit(", \"deviceAssignmentId\": "); ctxs(0);
    o.lit(", \"customerId\": "); ctxs(2);
    o.lit(", \"areaId\": "); ctxs(3);
    o.lit(", \"assetId\": "); ctxs(4);
    o.lit(", \"eventDate\": "); o.i64(date[i]);
    o.lit(", \"receivedDate\": "); o.i64(recv_ms);
    o.lit(", \"metadata\": ");
    if ((f & 0x10) && (et == 0 || et == 1 || et == 2))
      metadata(o, heap + soff[3 * i + 2], soff[3 * i + 3] - soff[3 * i + 2], et == 0 ? 4 : et == 1 ? 6 : 5);
    else o.lit("{}");
    const int64_t nid = name[i];
    const bool named = nid != 0xffff && N.has(nid);
    if (et == 0) {
      o.lit(", \"name\": ");
      if (named) o.str(N.get(nid)); else o.lit("\"\"");
      o.lit(", \"value\": "); o.dbl(v0[i]);
    } else if (et == 1) {
      o.lit(", \"latitude\": "); o.dbl(v0[i]);
      o.lit(", \"longitude\": "); o.dbl(v1[i]);
      o.lit(", \"elevation\": ");
      if (f & 0x4) o.dbl(v2[i]); else o.lit("null");
    } else if (et == 2) {
      const bool gen = (f & 0x20) != 0;
      o.lit(", \"source\": \"");
      o.lit(gen || (f & 0x40) ? "System" : "Device");
      o.lit("\", \"level\": \"");
      o.lit(kLevels[level[i] < 3 ? level[i] : 3]);
      o.lit("\", \"type\": ");
      if (named) o.str(N.get(nid)); else o.lit("\"\"");
      o.lit(", \"message\": ");
      if (gen) {
        if (nid != 0xffff && R.has(nid)) o.str(R.get(nid)); else o.lit("\"\"");
      } else o.str(heap + soff[3 * i + 1], soff[3 * i + 2] - soff[3 * i + 1]);
    } else {
      o.lit(", \"attribute\": \"presence\", \"type\": \"presence\", \"previousState\": \"PRESENT\", "
            "\"newState\": \"NOT_PRESENT\"");
    }
    o.lit("}, \"context\": {\"deviceId\": "); ctxs(1);
    o.lit(", \"deviceToken\": "); ctxs(5);
    o.lit(", \"deviceTypeId\": "); ctxs(6);
    o.lit(", \"assignmentStatus\": \"Active\", \"engine\": \"batch\"}}");
    if (tout) {
      tout_off[j] = t.n;
      for (int64_t k = 0; k < tpl_len; ++k) {
        if (tpl[k] == 1) {
          if (ha && A.has(7 * a + 5)) { auto x = A.get(7 * a + 5); t.put(x.first, (size_t)x.second); }
          else t.lit("None");
        } else if (tpl[k] == 2) t.lit(kTypes[et]);
        else t.ch((char)tpl[k]);
      }
    }
  }
  out_off[n] = o.n;
  if (tout) tout_off[n] = t.n;
  if (o.n > cap || (tout && t.n > tcap)) return -(o.n > t.n ? o.n : t.n) - (int64_t)1 - n;
  return o.n;
}

// MQTT 3.1.1 QoS 0 PUBLISH packets of n (topic, payload) pairs, back to back into `out` (one socket
// write for a connector's batch).  Returns the bytes written, or -needed.
int64_t swmqtt_publish_qos0(const uint8_t* topics, const int64_t* t_off, const uint8_t* payloads, const int64_t* p_off,
                            int64_t n, uint8_t retain, uint8_t* out, int64_t cap) {
  int64_t need = 0;
  for (int64_t j = 0; j < n; ++j) {
    const int64_t rl = 2 + (t_off[j + 1] - t_off[j]) + (p_off[j + 1] - p_off[j]);
    need += 1 + (rl < 128 ? 1 : rl < 16384 ? 2 : rl < 2097152 ? 3 : 4) + rl;
  }
  if (need > cap) return -need;
  uint8_t* w = out;
  for (int64_t j = 0; j < n; ++j) {
    const int64_t tl = t_off[j + 1] - t_off[j], pl = p_off[j + 1] - p_off[j];
    int64_t rl = 2 + tl + pl;
    *w++ = (uint8_t)(0x30 | (retain ? 1 : 0));
    do {
      uint8_t b = (uint8_t)(rl & 0x7f);
      rl >>= 7;
      if (rl) b |= 0x80;
      *w++ = b;
    } while (rl);
    *w++ = (uint8_t)(tl >> 8);
    *w++ = (uint8_t)(tl & 0xff);
    memcpy(w, topics + t_off[j], (size_t)tl);
    w += tl;
    memcpy(w, payloads + p_off[j], (size_t)pl);
    w += pl;
  }
  return w - out;
}

// Complete MQTT packets at the front of buf[0 .. n): per packet (first byte, start, body start, end)
// into out[4 k ..], at most cap packets.  Returns the packets found; *used = the end of the last one.
// -1: a malformed remaining length (more than 4 bytes), -2: a packet longer than max_len.
int64_t swmqtt_scan(const uint8_t* buf, int64_t n, int64_t* out, int64_t cap, int64_t max_len, int64_t* used) {
  int64_t p = 0, k = 0;
  while (k < cap && n - p >= 2) {
    int64_t len = 0, mult = 1, i = p + 1;
    bool done = false;
    for (int b = 0; b < 4 && i < n; ++b) {
      const uint8_t x = buf[i++];
      len += (int64_t)(x & 0x7f) * mult;
      mult <<= 7;
      if (!(x & 0x80)) { done = true; break; }
    }
    if (!done) {
      if (i - p > 4) return -1;
      break;                                     // the length bytes are not all here yet
    }
    if (len > max_len) return -2;
    if (n - i < len) break;
    out[4 * k] = buf[p];
    out[4 * k + 1] = p;
    out[4 * k + 2] = i;
    out[4 * k + 3] = i + len;
    ++k;
    p = i + len;
  }
  *used = p;
  return k;
}

// When every one of the k packets swmqtt_scan found in buf (hdr: its 4 words per packet) is a QoS 0,
// non-retained PUBLISH: the distinct topics (the first packet of each, in first-seen order) into
// first[] and each packet's topic number into tix[]; returns how many distinct topics, -1 when some
// packet is of another kind, -2 beyond `cap` topics.  A broker forwards such a batch whole when all
// its topics have the same subscribers; a client hands each topic's payloads over together.
int64_t swmqtt_qos0_topics(const uint8_t* buf, const int64_t* hdr, int64_t k, int64_t* first, int64_t cap,
                           int32_t* tix) {
  int64_t nd = 0;
  std::vector<int64_t> t0s, tls;
  int64_t last = -1;
  for (int64_t i = 0; i < k; ++i) {
    const int64_t fb = hdr[4 * i], bs = hdr[4 * i + 2], e = hdr[4 * i + 3];
    if ((fb >> 4) != 3 || (fb & 0x07) || e - bs < 2) return -1;
    const int64_t tl = ((int64_t)buf[bs] << 8) | buf[bs + 1];
    if (bs + 2 + tl > e) return -1;
    const uint8_t* t = buf + bs + 2;
    int64_t m = -1;
    if (last >= 0 && tls[last] == tl && memcmp(buf + t0s[last], t, (size_t)tl) == 0) m = last;
    for (int64_t q = 0; m < 0 && q < nd; ++q)
      if (tls[q] == tl && memcmp(buf + t0s[q], t, (size_t)tl) == 0) m = q;
    if (m < 0) {
      if (nd >= cap) return -2;
      m = nd++;
      t0s.push_back(bs + 2);
      tls.push_back(tl);
      first[m] = i;
    }
    tix[i] = (int32_t)m;
    last = m;
  }
  return nd;
}

}  // extern "C"
