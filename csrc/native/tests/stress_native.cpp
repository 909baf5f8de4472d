// Concurrency stress driver for the host runtime, built with the host sanitizers
// (tests/test_native_sanitizers.py: -fsanitize=thread, and -fsanitize=address,undefined).
//
// The reference ships no race detection at all and its shared structures raced
// (GrpcUtils' static claims HashMap, LifecycleComponent's child map).  Here the shared native state
// is the commit log (swnative.cpp: partitions appended by producer threads while consumer threads
// wait / read / view records in place, retention drops segments and recycles them between
// partitions, adopted external buffers are released, consumer-group offsets are saved) and the CPU
// engine's fork-join pool (swcpuengine.cpp).  This program drives all of those from several threads
// at once and checks every record it reads back, and feeds the device-protocol decoder corrupted
// payloads; the sanitizers check the memory accesses.
//
//   stress_native [durable_dir]      exit 0 = all checks passed
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "swtypes.h"

extern "C" {
void* swlog_open(const char* dir, int32_t fsync_each);
void swlog_close(void* h);
int32_t swlog_topic(void* h, const char* name, int32_t partitions);
int64_t swlog_append_batch(void* h, int32_t topic, int32_t p, const uint8_t* keys, const int64_t* koff,
                           const uint8_t* vals, const int64_t* voff, const int64_t* ts, int64_t n);
int64_t swlog_end_offset(void* h, int32_t topic, int32_t p);
int64_t swlog_begin_offset(void* h, int32_t topic, int32_t p);
int64_t swlog_wait(void* h, int32_t topic, int32_t p, int64_t offset, int32_t timeout_ms);
int64_t swlog_read(void* h, int32_t topic, int32_t p, int64_t offset, int64_t max_records, uint8_t* out,
                   int64_t out_cap, int64_t* n_out);
int64_t swlog_retain_from(void* h, int32_t topic, int32_t p, int64_t offset);
int64_t swlog_append_external(void* h, int32_t topic, int32_t p, const uint8_t* body, int64_t len, int64_t klen,
                              int64_t ts, int64_t ext_id);
int32_t swlog_view(void* h, int32_t topic, int32_t p, int64_t offset, const uint8_t** val, int64_t* vlen,
                   int64_t* ts);
int32_t swlog_hold(void* h, int32_t topic, int32_t p, int64_t offset);
int64_t swlog_take_released(void* h, int64_t* out, int64_t max);
int32_t swlog_set_retention(void* h, int32_t topic, int64_t bytes);
int32_t swlog_commit(void* h, const char* group, int32_t topic, int32_t p, int64_t offset);
int64_t swlog_committed(void* h, const char* group, int32_t topic, int32_t p);
int32_t swlog_flush(void* h);
void sw_memcpy_mt(void* dst, const void* src, int64_t n, int32_t threads);
uint32_t sw_crc32c(const uint8_t* p, int64_t n);
void* swce_create(int32_t n_threads);
void swce_destroy(void* p);
void swce_reserve(void* p, int64_t state_slots, int64_t dedup_slots);
int64_t swce_capture_names(void* p, const SwEventRec* recs, int64_t n, uint8_t* refs, int64_t cap);
int64_t sw_cpu_decode(const uint8_t* raw, const uint32_t* off, int64_t n_msgs, int64_t now_ms, int32_t rank,
                      SwEventRec* out, SwStrRef* spans, int64_t cap, int32_t n_threads);
int64_t sw_gen_payloads(int64_t n_msgs, const char* prefix, int64_t n_devices, double p_loc, double p_alert,
                        double p_unreg, int32_t mx_per_msg, int32_t n_names, int64_t ts0, uint64_t seed,
                        int32_t with_alt_id, double lat0, double lon0, double span_deg, double p_meta, uint8_t* out,
                        int64_t out_cap, uint32_t* offs, uint64_t alt_base);
int64_t swseg_encode(const SwOutRec* rows, const SwEventRec* recs, const SwStrRef* spans, const uint8_t* raw,
                     int64_t raw_bytes, int64_t n, uint8_t* out, int64_t cap);
void swseg_seal(uint8_t* block, int64_t first_seq, int64_t recv_ms, int64_t boot, int32_t rank, int32_t world);
int32_t swseg_verify(const uint8_t* b, int64_t len);
int64_t swseg_index_append(uint8_t* block, int64_t cap, const int32_t* ctx, int64_t n_ctx);
int64_t swseg_ix_max_bytes(int64_t n_rows);
int64_t swseg_ix_offset(const uint8_t* block);
void swseg_ix_alt_find(const uint8_t* const* t, int64_t n, const uint64_t* want, int64_t n_want, int64_t* out_blk,
                       int64_t* out_page);
void swseg_ix_ctx_find(const uint8_t* const* t, int64_t n, int32_t d, uint32_t key, int64_t* out);
int64_t swseg_string_bytes(const uint8_t* b, int64_t p0, int64_t p1);
int64_t swseg_decode(const uint8_t* b, int64_t p0, int64_t p1, uint8_t* etype, uint8_t* level, int64_t* date,
                     int32_t* asg, uint16_t* name, double* v0, double* v1, double* v2, uint8_t* flags,
                     uint8_t* str_heap, int64_t str_cap, int64_t* str_off);
int64_t swjson_select_block(const uint8_t* b, int32_t etmask, const uint8_t* keep, int64_t n_keep, int32_t keep_default,
                            const uint8_t* a_known, int64_t n_asg, const uint8_t* a_heap, const int64_t* a_off,
                            const uint8_t* a_present, const uint8_t* n_heap, const int64_t* n_off,
                            const uint8_t* n_present, int64_t n_names, const uint8_t* r_heap, const int64_t* r_off,
                            const uint8_t* r_present, const uint8_t* tpl, int64_t tpl_len, int32_t threads,
                            uint8_t* scratch, int64_t scap, uint8_t* tscratch, int64_t tscap, uint8_t* out,
                            int64_t cap, int64_t* out_off, uint8_t* tout, int64_t tcap, int64_t* tout_off,
                            int64_t* counts, int64_t* miss, int64_t miss_cap);
int64_t swseg_threshold_rows(const uint8_t* b, const uint8_t* name_mask, int64_t n_mask, double lo, double hi,
                             int32_t has_lo, int32_t has_hi, int32_t threads, int64_t* out_rows, int32_t* out_asg,
                             double* out_val, int64_t cap);
int64_t swmqtt_publish_qos0(const uint8_t* topics, const int64_t* t_off, const uint8_t* payloads, const int64_t* p_off,
                            int64_t n, uint8_t retain, uint8_t* out, int64_t cap);
int64_t swmqtt_scan(const uint8_t* buf, int64_t n, int64_t* out, int64_t cap, int64_t max_len, int64_t* used);
}

static std::atomic<int> g_fail{0};
#define CHECK(c, ...)                                      \
  do {                                                     \
    if (!(c)) {                                            \
      fprintf(stderr, "CHECK failed %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                        \
      fprintf(stderr, "\n");                               \
      g_fail++;                                            \
    }                                                      \
  } while (0)

// value = [u32 producer][u32 seq][u32 len][u32 crc of body][body: len bytes of (producer*7+seq)&0xff]
static size_t make_value(uint8_t* v, uint32_t prod, uint32_t seq) {
  const uint32_t len = 8 + (seq * 13 + prod * 5) % 200;
  memset(v + 16, (int)((prod * 7 + seq) & 0xff), len);
  const uint32_t c = sw_crc32c(v + 16, len);
  memcpy(v, &prod, 4);
  memcpy(v + 4, &seq, 4);
  memcpy(v + 8, &len, 4);
  memcpy(v + 12, &c, 4);
  return 16 + len;
}

static bool check_value(const uint8_t* v, int64_t vlen, uint32_t* prod, uint32_t* seq) {
  if (vlen < 16) return false;
  uint32_t len, c;
  memcpy(prod, v, 4);
  memcpy(seq, v + 4, 4);
  memcpy(&len, v + 8, 4);
  memcpy(&c, v + 12, 4);
  if ((int64_t)len + 16 != vlen) return false;
  for (uint32_t i = 0; i < len; ++i)
    if (v[16 + i] != (uint8_t)((*prod * 7 + *seq) & 0xff)) return false;
  return sw_crc32c(v + 16, len) == c;
}

constexpr int kProducers = 4, kParts = 2, kBatches = 600, kPerBatch = 8, kExternal = 300;

// Producers 0..kProducers-1 append batches (each to partition prod % kParts); producer kProducers
// adopts external buffers into partition 0.  One reader per partition follows with swlog_wait +
// swlog_read and checks per-producer order; one viewer per partition reads in place under a hold.
static void log_stress(const char* dir) {
  void* L = swlog_open(dir, 0);
  const int32_t t = swlog_topic(L, "stress", kParts);
  const bool durable = dir && dir[0];
  if (!durable) swlog_set_retention(L, t, 48 << 10);   // memory-only: retention recycles segments
  std::atomic<int> producers_left{kProducers + (durable ? 0 : 1)};
  std::vector<std::vector<uint8_t>> ext(kExternal);
  std::atomic<int64_t> released{0};

  std::vector<std::thread> th;
  for (int pr = 0; pr < kProducers; ++pr)
    th.emplace_back([&, pr] {
      std::vector<uint8_t> keys, vals(kPerBatch * 256);
      std::vector<int64_t> koff(kPerBatch + 1), voff(kPerBatch + 1), ts(kPerBatch);
      uint32_t seq = 0;
      for (int b = 0; b < kBatches; ++b) {
        keys.clear();
        koff[0] = voff[0] = 0;
        for (int i = 0; i < kPerBatch; ++i) {
          char k[32];
          const int kl = snprintf(k, sizeof k, "dev-%d-%u", pr, seq);
          keys.insert(keys.end(), k, k + kl);
          koff[i + 1] = (int64_t)keys.size();
          voff[i + 1] = voff[i] + (int64_t)make_value(vals.data() + voff[i], (uint32_t)pr, seq++);
          ts[i] = 1700000000000 + seq;
        }
        const int64_t off = swlog_append_batch(L, t, pr % kParts, keys.data(), koff.data(), vals.data(),
                                               voff.data(), ts.data(), kPerBatch);
        CHECK(off >= 0, "append_batch failed");
        if (b % 64 == 0) swlog_commit(L, "stress-group", t, pr % kParts, off);
      }
      producers_left--;
    });
  if (!durable)
    th.emplace_back([&] {            // zero-copy adoption of caller-owned buffers
      for (int i = 0; i < kExternal; ++i) {
        ext[i].resize(8 + 256);
        memcpy(ext[i].data(), "extkey!!", 8);
        const size_t n = make_value(ext[i].data() + 8, 1000, (uint32_t)i);
        CHECK(swlog_append_external(L, t, 0, ext[i].data(), (int64_t)(8 + n), 8, i, i) >= 0, "append_external");
        int64_t ids[16];
        released += swlog_take_released(L, ids, 16);
      }
      producers_left--;
    });

  for (int p = 0; p < kParts; ++p) {
    th.emplace_back([&, p] {         // copying reader: swlog_wait + swlog_read
      std::vector<uint8_t> buf(1 << 16);
      std::vector<int64_t> last(kProducers + 1, -1);
      int64_t next = 0;
      for (;;) {
        const bool done = producers_left.load() == 0;
        const int64_t end = swlog_wait(L, t, p, next, 5);
        if (end <= next && done) break;
        const int64_t begin = swlog_begin_offset(L, t, p);
        if (next < begin) next = begin;            // retention overtook the reader: skip ahead
        int64_t n = 0;
        const int64_t w = swlog_read(L, t, p, next, 64, buf.data(), (int64_t)buf.size(), &n);
        CHECK(w >= 0, "read returned %lld", (long long)w);
        int64_t pos = 0;
        for (int64_t i = 0; i < n; ++i) {
          int64_t off;
          uint32_t kl, vl, prod, seq;
          memcpy(&off, buf.data() + pos, 8);
          memcpy(&kl, buf.data() + pos + 16, 4);
          memcpy(&vl, buf.data() + pos + 20, 4);
          CHECK(off >= next, "offset went backwards");
          CHECK(check_value(buf.data() + pos + 24 + kl, vl, &prod, &seq), "corrupt record at %lld", (long long)off);
          const int slot = prod == 1000 ? kProducers : (int)prod;
          if (slot <= kProducers) {
            CHECK((int64_t)seq > last[slot], "producer %u out of order", prod);
            last[slot] = seq;
          }
          next = off + 1;
          pos += 24 + kl + vl;
        }
      }
    });
    th.emplace_back([&, p] {         // in-place viewer: hold, view, verify, release the hold
      int64_t rounds = 0;
      while (producers_left.load() > 0 || rounds < 50) {
        ++rounds;
        const int64_t b = swlog_begin_offset(L, t, p), e = swlog_end_offset(L, t, p);
        if (e <= b) { std::this_thread::yield(); continue; }
        const int64_t o = b + (e - b) / 2;
        swlog_hold(L, t, p, o);
        const uint8_t* v;
        int64_t vl, ts;
        if (swlog_view(L, t, p, o, &v, &vl, &ts) == 0) {
          uint32_t prod, seq;
          CHECK(check_value(v, vl, &prod, &seq), "corrupt in-place view at %lld", (long long)o);
        }
        swlog_hold(L, t, p, INT64_MAX);
      }
    });
  }
  th.emplace_back([&] {              // retention / group-offset traffic beside the data path
    while (producers_left.load() > 0) {
      for (int p = 0; p < kParts; ++p) {
        const int64_t e = swlog_end_offset(L, t, p);
        if (!durable && e > 4000) swlog_retain_from(L, t, p, e - 4000);
        (void)swlog_committed(L, "stress-group", t, p);
      }
      if (durable) swlog_flush(L);
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  });
  for (auto& x : th) x.join();
  for (int p = 0; p < kParts; ++p)
    CHECK(swlog_committed(L, "stress-group", t, p) >= 0, "group offset missing on partition %d", p);
  const int64_t total = swlog_end_offset(L, t, 0) + swlog_end_offset(L, t, 1);
  CHECK(total == (int64_t)kProducers * kBatches * kPerBatch + (durable ? 0 : kExternal), "end offsets %lld",
        (long long)total);
  swlog_close(L);
  printf("log stress (%s): %lld records, %lld external buffers released\n", durable ? "durable" : "memory",
         (long long)total, (long long)released.load());
}

// Two CPU engines (each with its own fork-join pool) capturing names from concurrent threads.
static void engine_stress() {
  std::vector<std::thread> th;
  for (int e = 0; e < 2; ++e)
    th.emplace_back([e] {
      void* eng = swce_create(4);
      swce_reserve(eng, 1 << 12, 1 << 12);
      const int64_t n = 4096;
      std::vector<SwEventRec> recs(n);
      std::vector<uint8_t> refs(16 * n);
      int64_t total = 0;
      for (int round = 0; round < 40; ++round) {
        for (int64_t i = 0; i < n; ++i) {
          memset(&recs[i], 0, sizeof(SwEventRec));
          recs[i].name_hash = 1 + (uint64_t)((i * 2654435761u + round * 977 + e) % 3000);
          recs[i].etype = (uint8_t)(i % 3);
          recs[i].aux_off = (uint32_t)i;
          recs[i].aux_len = 4;
        }
        total += swce_capture_names(eng, recs.data(), n, refs.data(), n);
      }
      CHECK(total == 3000, "engine %d captured %lld distinct names", e, (long long)total);
      swce_destroy(eng);
    });
  for (auto& x : th) x.join();
  std::vector<uint8_t> a(1 << 22), b(1 << 22);
  for (size_t i = 0; i < a.size(); ++i) a[i] = (uint8_t)(i * 31);
  sw_memcpy_mt(b.data(), a.data(), (int64_t)a.size(), 6);
  CHECK(memcmp(a.data(), b.data(), a.size()) == 0, "sw_memcpy_mt mismatch");
  printf("engine pool stress ok\n");
}

// The decoder parses untrusted device bytes: decode generated payloads, then thousands of
// corrupted ones (flipped bytes, truncations, garbage), each from an exactly sized heap block so
// the address sanitizer sees any read past the message.
static void decode_fuzz() {
  const int64_t n = 2000;
  std::vector<uint8_t> raw(n * 256);
  std::vector<uint32_t> off(n + 1);
  const int64_t bytes = sw_gen_payloads(n, "dev-", 500, 0.3, 0.1, 0.05, 3, 16, 1700000000000, 7, 1, 33.0, -85.0, 1.0,
                                        0.3, raw.data(), (int64_t)raw.size(), off.data(), 0);
  CHECK(bytes > 0, "payload generation failed");
  std::vector<SwEventRec> out(n * 8);
  std::vector<SwStrRef> spans(n * 8);
  const int64_t good = sw_cpu_decode(raw.data(), off.data(), n, 1700000001000, 0, out.data(), spans.data(),
                                     (int64_t)out.size(), 4);
  CHECK(good >= n, "decoded %lld events from %lld messages", (long long)good, (long long)n);
  // the lossless durable block of the decoded events: encode from an exactly sized batch, verify,
  // decode every column and string (the sanitizer sees any read past the batch or the block)
  {
    std::vector<uint8_t> exact(raw.begin(), raw.begin() + bytes);
    std::vector<SwOutRec> rows((size_t)good);
    for (int64_t i = 0; i < good; ++i) {
      rows[i].event_date = out[i].event_date;
      rows[i].v0 = out[i].v0;
      rows[i].v1 = out[i].v1;
      rows[i].assignment = (int32_t)(i % 97);
      rows[i].name_id = out[i].etype == SW_EV_LOCATION ? 0xffff : 1;
      rows[i].etype = out[i].etype < 16 ? out[i].etype : SW_EV_MEASUREMENT;
      rows[i].level = 0;
    }
    std::vector<uint8_t> blk((size_t)(good * 600 + (1 << 20)));
    const int64_t nb = swseg_encode(rows.data(), out.data(), spans.data(), exact.data(), (int64_t)exact.size(), good,
                                    blk.data(), (int64_t)blk.size());
    CHECK(nb > 0, "block encode failed (%lld)", (long long)nb);
    if (nb > 0) {
      swseg_seal(blk.data(), 0, 1700000001000, 1, 0, 1);
      std::vector<uint8_t> b2(blk.begin(), blk.begin() + nb);
      CHECK(swseg_verify(b2.data(), nb) == 0, "block does not verify");
      const int64_t cap = swseg_string_bytes(b2.data(), 0, 1 << 30);
      std::vector<uint8_t> et(good), lv(good), fl(good), heap((size_t)cap);
      std::vector<int64_t> dt(good), so(3 * good + 1);
      std::vector<int32_t> as(good);
      std::vector<uint16_t> nm(good);
      std::vector<double> a0(good), a1(good), a2(good);
      const int64_t got = swseg_decode(b2.data(), 0, 1 << 30, et.data(), lv.data(), dt.data(), as.data(), nm.data(),
                                       a0.data(), a1.data(), a2.data(), fl.data(), heap.data(), cap, so.data());
      CHECK(got == good, "block decode returned %lld of %lld rows", (long long)got, (long long)good);
      // connector selection + JSON straight from the block (worker slices, then concatenated), on 3
      // threads; first with slices too small (measured only), then sized from the answer
      {
        const int64_t na = 97;
        std::string ah;
        std::vector<int64_t> ao(7 * na + 1);
        std::vector<uint8_t> ap(7 * na, 1), known(na, 1), keep(na);
        for (int64_t i = 0; i < 7 * na; ++i) { ao[i] = (int64_t)ah.size(); ah += "ctx-\"" + std::to_string(i); }
        ao[7 * na] = (int64_t)ah.size();
        for (int64_t i = 0; i < na; ++i) keep[i] = (uint8_t)(i % 3 != 0);
        const std::string nh = "namemx";
        std::vector<int64_t> no = {0, 4, 6};
        std::vector<uint8_t> np = {1, 1};
        const char* tpl = "t/\x01/\x02";
        int64_t counts[3], miss[64];
        int64_t scap = 64, tscap = 64;
        for (int round = 0; round < 3; ++round) {
          std::vector<uint8_t> sc((size_t)scap), tsc((size_t)tscap), o((size_t)scap), to((size_t)tscap);
          std::vector<int64_t> oo(good + 1), too(good + 1);
          const int64_t r = swjson_select_block(b2.data(), 0x7, keep.data(), na, 0, known.data(), na,
                                                (const uint8_t*)ah.data(), ao.data(), ap.data(),
                                                (const uint8_t*)nh.data(), no.data(), np.data(), 2,
                                                (const uint8_t*)nh.data(), no.data(), np.data(), (const uint8_t*)tpl,
                                                (int64_t)strlen(tpl), 3, sc.data(), scap, tsc.data(), tscap, o.data(),
                                                scap, oo.data(), to.data(), tscap, too.data(), counts, miss, 64);
          if (r >= 0) {
            CHECK(counts[0] > 0 && counts[0] < good && oo[counts[0]] == r, "selection wrote %lld bytes for %lld rows",
                  (long long)r, (long long)counts[0]);
            break;
          }
          CHECK(r > -(int64_t(1) << 40), "selection failed (%lld)", (long long)r);
          scap = tscap = -r + 4096;
        }
        std::vector<uint8_t> nmask = {1, 1};
        std::vector<int64_t> rr(good);
        std::vector<int32_t> ra(good);
        std::vector<double> rv(good);
        const int64_t k = swseg_threshold_rows(b2.data(), nmask.data(), 2, -1e300, 50.0, 0, 1, 3, rr.data(), ra.data(),
                                               rv.data(), good);
        CHECK(k >= 0 && k <= good, "threshold rows returned %lld", (long long)k);
      }
    }
    // the same block with its index trailer (csrc/native/swindex.cpp) built into an exactly sized
    // buffer, verified, and queried through the alternate-id and context-key lookups
    if (nb > 0) {
      std::vector<int32_t> ctx(97 * 4);
      for (int i = 0; i < 97; ++i) { ctx[4 * i] = i; ctx[4 * i + 1] = i % 7; ctx[4 * i + 2] = i % 5; ctx[4 * i + 3] = -1; }
      std::vector<uint8_t> ib((size_t)(nb + swseg_ix_max_bytes(good)));
      std::copy(blk.begin(), blk.begin() + nb, ib.begin());
      const int64_t ni = swseg_index_append(ib.data(), (int64_t)ib.size(), ctx.data(), 97);
      CHECK(ni > nb, "index append returned %lld", (long long)ni);
      if (ni > nb) {
        swseg_seal(ib.data(), 0, 1700000001000, 1, 0, 1);
        std::vector<uint8_t> b3(ib.begin(), ib.begin() + ni);
        CHECK(swseg_verify(b3.data(), ni) == 0, "indexed block does not verify");
        const int64_t toff = swseg_ix_offset(b3.data());
        CHECK(toff > 0 && toff < ni, "bad trailer offset %lld", (long long)toff);
        std::vector<uint8_t> tr(b3.begin() + toff, b3.end());     // exact: the lookups stay inside it
        const uint8_t* tp = tr.data();
        uint64_t want[3] = {0x0123456789abcdefull, 0, ~0ull};
        int64_t ob[3], op[3], cf[7];
        swseg_ix_alt_find(&tp, 1, want, 3, ob, op);
        swseg_ix_ctx_find(&tp, 1, 0, (3u << 3) | 1u, cf);
      }
    }
  }
  uint64_t s = 12345;
  auto rnd = [&] { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
  int64_t events = 0;
  for (int it = 0; it < 20000; ++it) {
    const int64_t m = (int64_t)(rnd() % n);
    uint32_t len = off[m + 1] - off[m];
    std::vector<uint8_t> msg(raw.begin() + off[m], raw.begin() + off[m] + len);
    switch (it % 4) {
      case 0: msg[rnd() % len] ^= (uint8_t)(1 + rnd() % 255); break;
      case 1: msg.resize(1 + rnd() % len); break;
      case 2: for (int k = 0; k < 4; ++k) msg[rnd() % len] = (uint8_t)rnd(); break;
      default: for (auto& b : msg) b = (uint8_t)rnd(); break;
    }
    std::vector<uint8_t> heap(msg);              // exact size: no slack for an over-read to hide in
    const uint32_t o[2] = {0, (uint32_t)heap.size()};
    SwEventRec ev[64];
    SwStrRef sp[64];
    const int64_t k = sw_cpu_decode(heap.data(), o, 1, 1700000001000, 0, ev, sp, 64, 1);
    CHECK(k >= 0 && k <= 64, "decode of a corrupt message returned %lld", (long long)k);
    events += k;
  }
  printf("decode fuzz: %lld events from 2000 valid messages, %lld from 20000 corrupted ones\n", (long long)good,
         (long long)events);
}

// MQTT framing and the packet scanner, whole and cut at every byte boundary of a short stream
static void mqtt_frames() {
  const std::string topics = "a/bt/longer/topic", pay = std::string(300, 'x') + "{}";
  const int64_t t_off[4] = {0, 3, 3, (int64_t)topics.size()}, p_off[4] = {0, 1, 300, (int64_t)pay.size()};
  std::vector<uint8_t> out(4096);
  const int64_t n = swmqtt_publish_qos0((const uint8_t*)topics.data(), t_off, (const uint8_t*)pay.data(), p_off, 3, 0,
                                        out.data(), (int64_t)out.size());
  CHECK(n > 0, "framing failed (%lld)", (long long)n);
  for (int64_t cut = 0; cut <= n; ++cut) {
    std::vector<uint8_t> part(out.begin(), out.begin() + cut);     // exact size
    int64_t hdr[4 * 8], used = -1;
    const int64_t k = swmqtt_scan(part.data(), cut, hdr, 8, 1 << 20, &used);
    CHECK(k >= 0 && k <= 3 && used <= cut, "scan of %lld bytes: %lld packets, %lld used", (long long)cut,
          (long long)k, (long long)used);
  }
}

int main(int argc, char** argv) {
  mqtt_frames();
  decode_fuzz();
  log_stress("");
  if (argc > 1) log_stress(argv[1]);
  engine_stress();
  if (g_fail) {
    fprintf(stderr, "%d check(s) failed\n", g_fail.load());
    return 1;
  }
  printf("all native stress checks passed\n");
  return 0;
}
