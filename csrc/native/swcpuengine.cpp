// Native CPU engine shard: the fused inbound pipeline of csrc/hip/swgpu.hip on host cores.
//
// Stage semantics are those of the Python oracle (sitewhere_amd/pipeline/cpu_engine.py), bit for
// bit: registry lookup + assignment validation, alternate-id dedup, name interning, persist +
// enrichment into the columnar event ring, device-state merge, zone-test rules, presence scan.
// Reference counterparts: InboundPayloadProcessingLogic.java:101-218 (validation),
// AlternateIdDeduplicator.java (dedup), KafkaEventPersistenceTriggers / OutboundPayloadEnrichmentLogic
// (persist + enrich), DeviceStateProcessingLogic.java:116-200 (state), ZoneTestRuleProcessor.java:47-62
// (rules), DevicePresenceManager.java:110-200 (presence).
//
// Memory layout follows the GPU engine: the registry probe reads one packed 32-byte slot
// (fingerprint, device, *active* assignment), enrichment one 16-byte assignment-context row and the
// state merge one 32-byte state row, so each stage costs about one cache miss per event.
//
// Parallel design (one persistent fork-join pool per engine):
//   * lookup, persist, zone tests and the presence scan are data-parallel over record chunks; results
//     are concatenated in chunk order so every output row lands where the sequential oracle puts it;
//   * dedup is sharded by alternate-id hash: each shard thread walks its records in batch order, so
//     "first occurrence wins" holds exactly;
//   * the device-state merge is sharded by assignment.  Every state update is a lexicographic max
//     over (date, event id) -- order independent -- so per-shard processing equals the oracle;
//   * name interning assigns ids in first-occurrence order: a parallel read-only probe finds the
//     (rare) unknown names and a short sequential pass numbers them.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <new>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "swtypes.h"
#include "swengine.h"   // SW_STAT_* slots

namespace {

// ------------------------------------------------------------------------------------ hash map
// Open addressing, linear probing, key 0 = empty, grows at 1/2 load.  V is trivially copyable.
// Zero-initialised array on anonymous pages, transparent huge pages requested: the state map of a
// million-device shard spans gigabytes, and with 4 KB pages every random probe is also a TLB miss.
template <typename T>
struct PageArray {
  T* p = nullptr;
  size_t n = 0;
  PageArray() = default;
  PageArray(const PageArray&) = delete;
  PageArray& operator=(const PageArray&) = delete;
  PageArray(PageArray&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
  PageArray& operator=(PageArray&& o) noexcept {
    if (this != &o) { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
    return *this;
  }
  ~PageArray() { release(); }
  void assign_zero(size_t count) {
    release();
    n = count;
    const size_t bytes = std::max<size_t>(count * sizeof(T), 1);
    void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) { p = nullptr; n = 0; throw std::bad_alloc(); }
    if (bytes >= (2u << 20)) madvise(m, bytes, MADV_HUGEPAGE);
    p = static_cast<T*>(m);   // anonymous pages read as zero
  }
  void release() {
    if (p) munmap(p, std::max<size_t>(n * sizeof(T), 1));
    p = nullptr;
    n = 0;
  }
  size_t size() const { return n; }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
};

template <typename V>
struct U64Map {
  PageArray<uint64_t> keys;
  PageArray<V> vals;
  size_t n = 0, mask = 0;

  U64Map() { reset(64); }
  void reset(size_t cap) {
    size_t c = 64;
    while (c < cap) c <<= 1;
    keys.assign_zero(c);
    vals.assign_zero(c);
    mask = c - 1;
    n = 0;
  }
  static inline size_t mix(uint64_t k) { return (size_t)sw_mix64(k); }
  const V* find(uint64_t k) const {
    for (size_t s = mix(k) & mask;; s = (s + 1) & mask) {
      if (keys[s] == k) return &vals[s];
      if (keys[s] == 0) return nullptr;
    }
  }
  // returns (slot value, inserted)
  std::pair<V*, bool> insert(uint64_t k) {
    if (2 * (n + 1) > keys.size()) grow();
    for (size_t s = mix(k) & mask;; s = (s + 1) & mask) {
      if (keys[s] == k) return {&vals[s], false};
      if (keys[s] == 0) {
        keys[s] = k;
        vals[s] = V{};
        ++n;
        return {&vals[s], true};
      }
    }
  }
  void grow() {
    PageArray<uint64_t> ok = std::move(keys);
    PageArray<V> ov = std::move(vals);
    reset(ok.size() * 2);
    for (size_t i = 0; i < ok.size(); ++i)
      if (ok[i]) *insert(ok[i]).first = ov[i];
  }
  template <typename F>
  void for_each(F&& f) const {
    for (size_t i = 0; i < keys.size(); ++i)
      if (keys[i]) f(keys[i], vals[i]);
  }
};

struct MsVal {
  int64_t date;
  int64_t eid1;
};

// ------------------------------------------------------------------------------------ fork-join pool
class Pool {
 public:
  explicit Pool(int n) : n_(std::max(1, std::min(n, 64))) {
    for (int t = 1; t < n_; ++t) th_.emplace_back([this, t] { loop(t); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return n_; }
  // fn(t) on every worker t in [0, n); the caller runs t = 0.
  void run(const std::function<void(int)>& fn) {
    if (n_ == 1) { fn(0); return; }
    {
      std::lock_guard<std::mutex> g(m_);
      fn_ = &fn;
      pending_ = n_ - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return pending_ == 0; });
    fn_ = nullptr;
  }

 private:
  void loop(int t) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* fn;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        fn = fn_;
      }
      (*fn)(t);
      {
        std::lock_guard<std::mutex> g(m_);
        if (--pending_ == 0) done_.notify_one();
      }
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* fn_ = nullptr;
  uint64_t gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
};

inline void chunk_of(int64_t n, int t, int T, int64_t* b, int64_t* e) {
  int64_t c = (n + T - 1) / T;
  *b = std::min<int64_t>(n, (int64_t)t * c);
  *e = std::min<int64_t>(n, *b + c);
}

}  // namespace

extern "C" {

// Packed host tables (numpy-owned; sitewhere_amd/pipeline/native_engine.py keeps them current
// through the EngineBase dirty hooks, exactly like the GPU engine patches its HBM copies).
typedef struct SwCeReg {   // REG_SLOT
  uint64_t lo, hi;
  int32_t dev, asg;        // asg = the device's active assignment, -1 if none
  uint64_t pad;
} SwCeReg;

typedef struct SwCeCtx {   // assignment context for enrichment + generated events
  int32_t device, customer, area, asset;
} SwCeCtx;

typedef struct SwCeState { // per-assignment device state
  uint64_t last, missing, loc_date;
  int64_t loc_eid;         // event id + 1 of the newest location (0 = none)
} SwCeState;

typedef struct SwCeTables {
  const SwCeReg* reg;
  int64_t reg_mask;
  const SwCeCtx* ctx;
  const uint8_t* asg_active;
  int64_t n_assignments;
  SwCeState* st;
  // event store ring (struct of arrays, cpu_engine.STORE_COLS order)
  uint8_t* s_etype;
  uint8_t* s_level;
  int64_t* s_date;
  int64_t* s_recv;
  int32_t* s_dev;
  int32_t* s_asg;
  int32_t* s_cust;
  int32_t* s_area;
  int32_t* s_asset;
  uint64_t* s_name;
  double* s_v0;
  double* s_v1;
  double* s_v2;
  uint64_t* s_alt;
  uint64_t* s_aux;
  int32_t* s_batch;
  int64_t store_cap;
  // zones: vtx [2V] (lat, lon), zoff [Z+1], bbox [4Z], tests [T], alert hashes [T]
  const double* zone_vtx;
  const int32_t* zone_off;
  const double* zone_bbox;  // min lat, min lon, max lat, max lon
  const SwZoneTest* tests;
  const uint64_t* test_hash;
  int32_t n_tests;
  int32_t rank;
  int32_t world;
  int32_t batch_seq;
  int64_t gen_cap;
  uint64_t presence_hash;
  int64_t presence_missing_ms;
  uint64_t* stats;  // [SW_N_STATS], SW_STAT_* slots
  int32_t cluster;  // persist each step stable-sorted by assignment (EngineConfig.cluster)
  int32_t pad0;
} SwCeTables;

typedef struct SwCeStep {
  int64_t cursor;     // in/out: store sequence of the next persisted event
  int64_t seq_base;   // in/out: dedup sequence of work[0]
  int64_t n_ok;       // out
  int64_t n_gen;      // out
  int64_t n_rule;     // out
  int64_t n_rej;      // out
} SwCeStep;

}  // extern "C"

// Zeroed words from calloc: pages the filter never touches are never committed (a multi-GB filter
// of a small tenant costs what its ids touch).
struct LazyWords {
  uint64_t* p = nullptr;
  size_t n = 0;
  LazyWords() = default;
  LazyWords(const LazyWords&) = delete;
  LazyWords& operator=(const LazyWords&) = delete;
  ~LazyWords() { free(p); }
  void assign_zero(size_t count) {
    free(p);
    p = count ? static_cast<uint64_t*>(calloc(count, sizeof(uint64_t))) : nullptr;
    n = p ? count : 0;
  }
  bool empty() const { return n == 0; }
  size_t size() const { return n; }
  uint64_t* data() { return p; }
  const uint64_t* data() const { return p; }
  uint64_t& operator[](size_t i) { return p[i]; }
  const uint64_t& operator[](size_t i) const { return p[i]; }
};

struct SwCpuEngine {
  Pool pool;
  std::vector<U64Map<int64_t>> dedup;       // current generation of the alternate-id window, by hash % T
  std::vector<U64Map<int64_t>> dedup_prev;  // previous generation (see the rotation in swce_process)
  int64_t dd_slots = 0, dd_batch = 0;       // window slots and the largest batch (rotation rule)
  // store-backed dedup filter (generational fingerprint tables, swtypes.h SW_FF_*), empty: off
  LazyWords ff;                             // [buckets][gens][SW_FF_SLOTS] u32, as 64-bit words
  int64_t ff_bmask = 0, ff_gens = 0;
  int64_t ff_meta[SW_FF_META + SW_FF_MAX_GENS] = {};
  uint32_t* ff_tab() { return reinterpret_cast<uint32_t*>(ff.data()); }
  const uint32_t* ff_tab() const { return reinterpret_cast<const uint32_t*>(ff.data()); }
  U64Map<int32_t> intern;
  int32_t n_intern = 0;
  std::vector<U64Map<MsVal>> ms;       // sharded by assignment % T
  U64Map<uint8_t> seen;                // names already reported by the decode phase
  // per-step scratch, kept across steps (no page-faulting fresh buffers every batch)
  std::vector<int32_t> asg, dev;
  std::vector<int64_t> ok_idx;
  std::vector<int64_t> ok_tmp;      // clustering sort scratch
  std::vector<std::vector<int32_t>> lists;  // [chunk * T + shard] -> record / row indices
  std::vector<std::vector<int64_t>> scratch64;
  explicit SwCpuEngine(int n) : pool(n), dedup(pool.size()), dedup_prev(pool.size()), ms(pool.size()) {
    const int T = pool.size();
    lists.resize((size_t)T * T);
    scratch64.resize(T);
  }
  int T() const { return pool.size(); }
};

static inline int32_t nid_of(const SwCpuEngine* e, uint64_t h) {
  if (!h) return -1;
  const int32_t* v = e->intern.find(h);
  return v ? *v : -1;
}

// Does a live generation of the filter hold the id (ff_has in csrc/hip/swgpu.hip)?
static inline bool ff_has(const SwCpuEngine* e, uint64_t h) {
  const uint64_t m = sw_ff_mix(h);
  const uint32_t fp = sw_ff_fp(m);
  const int gens = (int)e->ff_gens;
  int64_t b = (int64_t)sw_ff_bucket(m, e->ff_bmask);
  uint32_t open = (1u << gens) - 1u;
  const uint32_t* t = e->ff_tab();
  for (int p = 0; p < SW_FF_MAX_PROBE && open; ++p) {
    for (int g = 0; g < gens; ++g) {
      if (!((open >> g) & 1u)) continue;
      const uint32_t* s = t + (b * gens + g) * SW_FF_SLOTS;
      bool empty = false;
      for (int k = 0; k < SW_FF_SLOTS; ++k) {
        const uint32_t v = __atomic_load_n(&s[k], __ATOMIC_RELAXED);
        if (v == fp) return true;
        empty |= v == 0;
      }
      if (empty) open &= ~(1u << g);
    }
    b = (b + 1) & e->ff_bmask;
  }
  return false;
}

// Add the id to generation g: one CAS into the first free slot of its chain (ff_add on the GPU).
static inline bool ff_add(SwCpuEngine* e, int g, uint64_t h) {
  const uint64_t m = sw_ff_mix(h);
  const uint32_t fp = sw_ff_fp(m);
  const int gens = (int)e->ff_gens;
  int64_t b = (int64_t)sw_ff_bucket(m, e->ff_bmask);
  uint32_t* t = e->ff_tab();
  for (int p = 0; p < SW_FF_MAX_PROBE; ++p) {
    uint32_t* s = t + (b * gens + g) * SW_FF_SLOTS;
    for (int k = 0; k < SW_FF_SLOTS; ++k) {
      uint32_t v = __atomic_load_n(&s[k], __ATOMIC_RELAXED);
      if (v == fp) return true;
      if (v == 0) {
        if (__atomic_compare_exchange_n(&s[k], &v, fp, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) return true;
        if (v == fp) return true;       // the same id, added by another thread
      }
    }
    b = (b + 1) & e->ff_bmask;
  }
  return false;
}

// Clear generation g.  Only buckets that hold something are written: untouched pages of the lazily
// committed table stay uncommitted.
static void ff_clear(SwCpuEngine* e, int g) {
  const int64_t nb = e->ff_bmask + 1, gens = e->ff_gens;
  uint32_t* t = e->ff_tab();
  for (int64_t b = 0; b < nb; ++b) {
    uint64_t* w = reinterpret_cast<uint64_t*>(t + (b * gens + g) * SW_FF_SLOTS);
    uint64_t any = 0;
    for (int k = 0; k < SW_FF_SLOTS / 2; ++k) any |= w[k];
    if (any) memset(w, 0, SW_FF_SLOTS * sizeof(uint32_t));
  }
}

static inline bool pip(const double* v, int32_t n, double x, double y) {
  bool inside = false;
  for (int32_t i = 0, j = n - 1; i < n; j = i++) {
    const double xi = v[2 * i], yi = v[2 * i + 1], xj = v[2 * j], yj = v[2 * j + 1];
    if (((yi > y) != (yj > y)) && (x < (xj - xi) * (y - yi) / (yj - yi) + xi)) inside = !inside;
  }
  return inside;
}

// Stable LSD radix sort (11-bit digits) of the ok indices by their assignment index.
static void cluster_by_assignment(int64_t* idx, int64_t n, const int32_t* asg, int64_t n_asg,
                                  std::vector<int64_t>& tmp) {
  int bits = 1;
  while (bits < 31 && (int64_t(1) << bits) < n_asg) ++bits;
  if ((int64_t)tmp.size() < n) tmp.resize(n);
  int64_t* src = idx;
  int64_t* dst = tmp.data();
  std::vector<int64_t> cnt(1 << 11);
  for (int shift = 0; shift < bits; shift += 11) {
    std::fill(cnt.begin(), cnt.end(), 0);
    for (int64_t j = 0; j < n; ++j) ++cnt[((uint32_t)asg[src[j]] >> shift) & 2047u];
    int64_t sum = 0;
    for (auto& c : cnt) { const int64_t x = c; c = sum; sum += x; }
    for (int64_t j = 0; j < n; ++j) dst[cnt[((uint32_t)asg[src[j]] >> shift) & 2047u]++] = src[j];
    std::swap(src, dst);
  }
  if (src != idx) memcpy(idx, src, sizeof(int64_t) * n);
}

// Persist rows [b, end) -- record idx[j] (or j) with assignment asg_of(j) -- at store sequence
// cursor + j and write the enriched outbound rows.  Safe on disjoint ranges concurrently.
template <typename AsgOf>
static void persist_range(const SwCpuEngine* e, const SwCeTables* t, const SwEventRec* recs, const int64_t* idx,
                          const int32_t* dev, AsgOf asg_of, int64_t cursor, int64_t now_ms, SwOutRec* out, int64_t b,
                          int64_t end, const SwStrRef* spans, SwEventRec* prec, SwStrRef* pspans) {
  int64_t row = (cursor + b) % t->store_cap;
  for (int64_t j = b; j < end; ++j) {
    const SwEventRec& r = recs[idx ? idx[j] : j];
    // the persisted record and its string refs, row-aligned with `out` (durable-block encoder input)
    if (prec) prec[j] = r;
    if (pspans) {
      if (spans) pspans[j] = spans[idx ? idx[j] : j];
      else memset(&pspans[j], 0, sizeof(SwStrRef));
    }
    const int32_t a = asg_of(j);
    const SwCeCtx c = t->ctx[a];
    t->s_etype[row] = r.etype;
    t->s_level[row] = r.level;
    t->s_date[row] = r.event_date;
    t->s_recv[row] = now_ms;
    t->s_dev[row] = dev ? dev[idx ? idx[j] : j] : c.device;
    t->s_asg[row] = a;
    t->s_cust[row] = c.customer;
    t->s_area[row] = c.area;
    t->s_asset[row] = c.asset;
    t->s_name[row] = r.name_hash;
    t->s_v0[row] = r.v0;
    t->s_v1[row] = r.v1;
    t->s_v2[row] = r.v2;
    t->s_alt[row] = r.alt_hash;
    t->s_aux[row] = ((uint64_t)r.src_rank << 48) | ((uint64_t)r.aux_len << 32) | (uint64_t)r.aux_off;
    t->s_batch[row] = t->batch_seq;
    const int32_t nid = nid_of(e, r.name_hash);
    SwOutRec& o = out[j];
    o.event_date = r.event_date;
    o.v0 = r.v0;
    o.v1 = r.v1;
    o.assignment = a;
    o.name_id = (nid >= 0 && nid < 0xFFFF) ? (uint16_t)nid : (uint16_t)0xFFFF;
    o.etype = r.etype;
    o.level = r.level;
    if (++row == t->store_cap) row = 0;
  }
}

// Device-state merge of one record (oracle: CpuInboundEngine._state).
static inline void state_one(const SwCpuEngine* e, const SwCeTables* t, const SwEventRec& r, int32_t a, int64_t eid1,
                             int64_t now_ms, U64Map<MsVal>& ms) {
  const int et = r.etype;
  if (et != SW_EV_MEASUREMENT && et != SW_EV_LOCATION && et != SW_EV_ALERT) return;
  SwCeState& s = t->st[a];
  if ((int64_t)s.last < now_ms) s.last = (uint64_t)now_ms;
  s.missing = 0;
  const int64_t d = r.event_date;
  if (et == SW_EV_LOCATION) {
    const int64_t cd = (int64_t)s.loc_date;
    if (d > cd) {
      s.loc_date = (uint64_t)d;
      s.loc_eid = eid1;
    } else if (d == cd) {
      s.loc_eid = std::max<int64_t>(s.loc_eid, eid1);
    }
  } else if (r.name_hash) {
    const int32_t nid = nid_of(e, r.name_hash);
    const uint64_t key = (((uint64_t)(uint32_t)a << 32) | ((uint64_t)(uint32_t)nid << 1) | (et == SW_EV_ALERT ? 1u : 0u)) + 1;
    auto ins = ms.insert(key);
    MsVal& v = *ins.first;
    if (ins.second || d > v.date) {
      v.date = d;
      v.eid1 = eid1;
    } else if (d == v.date) {
      v.eid1 = std::max(v.eid1, eid1);
    }
  }
}

// Give every unknown name hash of recs[idx[k]] (k in [0, n)) the next id, in first-occurrence
// order: a parallel read-only probe, then a sequential pass over the (rare) misses.
template <typename Map, typename OnNew>
static void first_occurrence(SwCpuEngine* e, Map& map, const SwEventRec* recs, const int64_t* idx, int64_t n,
                             bool names_only, OnNew on_new) {
  const int T = e->T();
  for (auto& v : e->scratch64) v.clear();
  e->pool.run([&](int w) {
    int64_t b, end;
    chunk_of(n, w, T, &b, &end);
    uint64_t last = 0;
    for (int64_t k = b; k < end; ++k) {
      const SwEventRec& r = recs[idx ? idx[k] : k];
      const uint64_t h = r.name_hash;
      if (!h || h == last || (names_only && r.etype >= 16)) continue;
      last = h;
      if (!map.find(h)) e->scratch64[w].push_back(k);
    }
  });
  for (int w = 0; w < T; ++w)
    for (int64_t k : e->scratch64[w]) {
      const SwEventRec& r = recs[idx ? idx[k] : k];
      auto ins = map.insert(r.name_hash);
      if (ins.second) on_new(r, ins.first);
    }
}

static void intern_in_order(SwCpuEngine* e, const SwEventRec* recs, const int64_t* idx, int64_t n) {
  first_occurrence(e, e->intern, recs, idx, n, false, [e](const SwEventRec&, int32_t* v) { *v = e->n_intern++; });
}

extern "C" {

void* swce_create(int32_t n_threads) { return new SwCpuEngine(n_threads); }

void swce_destroy(void* p) { delete static_cast<SwCpuEngine*>(p); }

int32_t swce_threads(void* p) { return static_cast<SwCpuEngine*>(p)->T(); }

// Pre-size the state and dedup maps (total slots over all shards), like the GPU engine's fixed
// HBM tables: no rehash pauses while a fleet's (assignment, name) keys accumulate.
void swce_reserve(void* p, int64_t state_slots, int64_t dedup_slots) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  const int64_t T = e->T();
  for (auto& m : e->ms)
    if (m.n == 0) m.reset((size_t)std::max<int64_t>(64, state_slots / (2 * T)));
  for (auto& m : e->dedup)
    if (m.n == 0) m.reset((size_t)std::max<int64_t>(64, dedup_slots / T));
}

// Decode-phase name capture: report hashes (etype < 16) not reported before, in record order.
// refs rows are NAME_REF {hash, off, len, src_rank, etype}.  Returns the number written.
int64_t swce_capture_names(void* p, const SwEventRec* recs, int64_t n, uint8_t* refs, int64_t cap) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  int64_t k = 0;
  first_occurrence(e, e->seen, recs, nullptr, n, true, [&](const SwEventRec& r, uint8_t*) {
    if (k >= cap) return;
    uint8_t* o = refs + 16 * k++;
    const uint64_t h = r.name_hash;
    const uint32_t off = r.aux_off;
    const uint16_t len = r.aux_len;
    memcpy(o, &h, 8);
    memcpy(o + 8, &off, 4);
    memcpy(o + 12, &len, 2);
    o[14] = r.src_rank;
    o[15] = r.etype;
  });
  return k;
}

// One process phase over the (already exchanged) work records.  status [n] receives each record's
// validation outcome; out [n + gen_cap] the enriched rows (persisted first, then generated).
// spans [n] (nullable): the work records' string refs; prec / pspans [n + gen_cap] (nullable) receive
// the persisted records and their string refs, row-aligned with out.
int32_t swce_process(void* p, const SwCeTables* t, SwCeStep* st, const SwEventRec* work, int64_t n, int64_t now_ms,
                     int32_t presence, uint8_t* status, SwOutRec* out, const SwStrRef* spans, SwEventRec* prec,
                     SwStrRef* pspans) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  const int T = e->T();
  const bool any_rank = t->world > 1 && spans != nullptr;   // the work batch's strings were exchanged
  static const bool trace = getenv("SW_CE_TRACE") != nullptr;
  auto tp = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!trace) return;
    auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[swce] %-9s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(now - tp).count());
    tp = now;
  };
  if ((int64_t)e->asg.size() < n + 1) { e->asg.resize(n + 1); e->dev.resize(n + 1); }
  int32_t* asg = e->asg.data();
  int32_t* dev = e->dev.data();
  int64_t has_alt[64] = {};

  // 1. registry lookup + assignment validation (InboundPayloadProcessingLogic.validateAssignment)
  e->pool.run([&](int w) {
    int64_t b, end;
    chunk_of(n, w, T, &b, &end);
    for (int64_t i = b; i < end; ++i) {
      const SwEventRec& r = work[i];
      asg[i] = -1;
      dev[i] = -1;
      if (r.etype == SW_EV_DECODE_ERROR) { status[i] = SW_ST_DECODE_ERROR; continue; }
      int64_t s = (int64_t)(r.fp_lo & (uint64_t)t->reg_mask);
      int32_t d = -1, a = -1;
      for (int64_t q = 0; q <= t->reg_mask; ++q) {
        const SwCeReg& g = t->reg[s];
        if (g.lo == r.fp_lo && g.hi == r.fp_hi) { d = g.dev; a = g.asg; break; }
        if (g.lo == 0 && g.hi == 0) break;
        s = (s + 1) & t->reg_mask;
      }
      dev[i] = d;
      if (r.etype >= 16) { status[i] = SW_ST_CONTROL; continue; }
      if (d < 0) { status[i] = SW_ST_UNREGISTERED; continue; }
      asg[i] = a;
      status[i] = a >= 0 ? SW_ST_OK : SW_ST_UNASSIGNED;
      if (a >= 0 && r.alt_hash) has_alt[w] = 1;
    }
  });
  lap("lookup");

  // 2. alternate-id dedup, sharded by hash; each shard walks its records in batch order.  The window
  // is generational like the GPU's (k_dedup_rotate): before a batch that could push the current
  // generation past half the window's slots, the previous generation is forgotten.
  if (e->dd_slots > 0) {
    int64_t cur = 0;
    for (auto& m : e->dedup) cur += (int64_t)m.n;
    if (cur + e->dd_batch > e->dd_slots / 2) {
      std::swap(e->dedup, e->dedup_prev);
      for (auto& m : e->dedup) m.reset((size_t)std::max<int64_t>(64, e->dd_slots / T));
      t->stats[SW_STAT_DEDUP_ROTATIONS] += 1;
    }
  }
  bool any_alt = false;
  for (int w = 0; w < T; ++w) any_alt |= has_alt[w] != 0;
  if (any_alt) {
    e->pool.run([&](int w) {
      for (int sh = 0; sh < T; ++sh) e->lists[(size_t)w * T + sh].clear();
      int64_t b, end;
      chunk_of(n, w, T, &b, &end);
      for (int64_t i = b; i < end; ++i)
        // a settled recheck skips the window: its id was claimed when it came back as a recheck
        if (work[i].alt_hash && status[i] == SW_ST_OK && !(work[i].flags & SW_F_SETTLED))
          e->lists[(size_t)w * T + sw_mix64(work[i].alt_hash) % (uint64_t)T].push_back((int32_t)i);
    });
    const int64_t seq_base = st->seq_base;
    e->pool.run([&](int sh) {
      U64Map<int64_t>& m = e->dedup[sh];
      const U64Map<int64_t>& prev = e->dedup_prev[sh];
      for (int w = 0; w < T; ++w)
        for (int32_t i : e->lists[(size_t)w * T + sh]) {
          if (prev.n && prev.find(work[i].alt_hash)) {
            status[i] = SW_ST_DUPLICATE;
            continue;
          }
          auto ins = m.insert(work[i].alt_hash);
          if (ins.second) {
            *ins.first = seq_base + i;
            // first sight in the window: the store may still hold it (filter from earlier steps).
            // Every record this rank owns goes through it when its strings came along (the host
            // settles a recheck by its alternate id); without the string exchange only records
            // decoded here do (the host path re-reads their payload).  A settled record skips it.
            if (!e->ff.empty() && !(work[i].flags & SW_F_SETTLED) &&
                (any_rank || work[i].src_rank == (uint8_t)t->rank) && ff_has(e, work[i].alt_hash))
              status[i] = SW_ST_RECHECK;
          } else {
            status[i] = SW_ST_DUPLICATE;
          }
        }
    });
  }
  lap("dedup");

  // 3. ok index list in batch order; per-status counts
  int64_t nok[65] = {};
  uint64_t cnt[64][8] = {};
  e->pool.run([&](int w) {
    int64_t b, end;
    chunk_of(n, w, T, &b, &end);
    int64_t k = 0;
    for (int64_t i = b; i < end; ++i) {
      ++cnt[w][status[i] & 7];
      k += status[i] == SW_ST_OK;
    }
    nok[w + 1] = k;
  });
  for (int w = 0; w < T; ++w) nok[w + 1] += nok[w];
  const int64_t n_ok = nok[T];
  if ((int64_t)e->ok_idx.size() < n_ok + 1) e->ok_idx.resize(n_ok + 1);
  int64_t* ok_idx = e->ok_idx.data();
  e->pool.run([&](int w) {
    int64_t b, end;
    chunk_of(n, w, T, &b, &end);
    int64_t k = nok[w];
    for (int64_t i = b; i < end; ++i)
      if (status[i] == SW_ST_OK) ok_idx[k++] = i;
  });
  lap("compact");

  // 4. name interning in first-occurrence order over the persisted records
  intern_in_order(e, work, ok_idx, n_ok);
  lap("intern");

  // 4b. persist order: stable by assignment (the durable block's clustering, csrc/include/swindex.h;
  // the MI355X engine radix-sorts the same pairs)
  if (t->cluster && n_ok > 1) cluster_by_assignment(ok_idx, n_ok, asg, t->n_assignments, e->ok_tmp);
  lap("cluster");

  // 5. persist + enrich (parallel rows); rows bucketed by assignment shard for the state merge
  const int64_t cursor0 = st->cursor;
  const bool ff_on = !e->ff.empty();
  const int ff_live = ff_on ? (int)e->ff_meta[0] : 0;
  std::atomic<int64_t> ff_dropped{0}, ff_ids{0};
  e->pool.run([&](int w) {
    int64_t b, end;
    chunk_of(n_ok, w, T, &b, &end);
    persist_range(e, t, work, ok_idx, dev, [&](int64_t j) { return asg[ok_idx[j]]; }, cursor0, now_ms, out, b, end,
                  spans, prec, pspans);
    if (ff_on) {                              // persisted ids join the filter's live generation
      int64_t dropped = 0, ids = 0;
      for (int64_t j = b; j < end; ++j)
        if (work[ok_idx[j]].alt_hash) {
          ++ids;
          if (!ff_add(e, ff_live, work[ok_idx[j]].alt_hash)) ++dropped;
        }
      if (dropped) ff_dropped += dropped;
      if (ids) ff_ids += ids;
    }
    if (T > 1) {
      for (int sh = 0; sh < T; ++sh) e->lists[(size_t)w * T + sh].clear();
      for (int64_t j = b; j < end; ++j) e->lists[(size_t)w * T + (uint32_t)out[j].assignment % (uint32_t)T].push_back((int32_t)j);
    }
  });
  lap("persist");

  // 6. device state (sharded by assignment)
  const int64_t W = t->world, R = t->rank;
  e->pool.run([&](int sh) {
    if (T == 1) {
      for (int64_t j = 0; j < n_ok; ++j)
        state_one(e, t, work[ok_idx[j]], out[j].assignment, (cursor0 + j) * W + R + 1, now_ms, e->ms[0]);
      return;
    }
    for (int w = 0; w < T; ++w)
      for (int32_t j : e->lists[(size_t)w * T + sh])
        state_one(e, t, work[ok_idx[j]], out[j].assignment, (cursor0 + j) * W + R + 1, now_ms, e->ms[sh]);
  });
  int64_t cursor = cursor0 + n_ok;
  lap("state");

  // 7. zone-test rules over the persisted locations, generated in (row, test) order
  std::vector<SwEventRec> gen;
  std::vector<int32_t> gen_asg;
  int64_t n_rule = 0;
  if (t->n_tests > 0) {
    e->pool.run([&](int w) {
      std::vector<int64_t>& hits = e->scratch64[w];
      hits.clear();
      int64_t b, end;
      chunk_of(n_ok, w, T, &b, &end);
      for (int64_t j = b; j < end; ++j) {
        if (out[j].etype != SW_EV_LOCATION) continue;
        const double x = out[j].v0, y = out[j].v1;
        for (int32_t k = 0; k < t->n_tests; ++k) {
          const SwZoneTest& zt = t->tests[k];
          const int32_t z = zt.zone;
          // strict longitude-band reject is exact: no edge can straddle a point outside it
          const bool out_band = y < t->zone_bbox[4 * z + 1] || y > t->zone_bbox[4 * z + 3];
          const bool inside = !out_band &&
                              pip(t->zone_vtx + 2 * (int64_t)t->zone_off[z], t->zone_off[z + 1] - t->zone_off[z], x, y);
          if ((zt.condition == 0) == inside) hits.push_back(j * t->n_tests + k);
        }
      }
    });
    for (int w = 0; w < T && (int64_t)gen.size() < t->gen_cap; ++w)
      for (int64_t hk : e->scratch64[w]) {
        if ((int64_t)gen.size() >= t->gen_cap) break;
        const int64_t j = hk / t->n_tests;
        const int32_t k = (int32_t)(hk % t->n_tests);
        SwEventRec g;
        memset(&g, 0, sizeof(g));
        g.event_date = now_ms;
        g.name_hash = t->test_hash[k];
        g.aux_off = (uint32_t)k;
        g.etype = SW_EV_ALERT;
        g.src_rank = (uint8_t)t->rank;
        g.level = (uint8_t)t->tests[k].level;
        gen.push_back(g);
        gen_asg.push_back(out[j].assignment);
      }
    n_rule = (int64_t)gen.size();
  }
  lap("zones");

  // 8. presence scan (DevicePresenceManager): assignments silent for presence_missing_ms
  if (presence && t->presence_missing_ms > 0) {
    const int64_t lim = std::max<int64_t>(now_ms - t->presence_missing_ms, 0);
    const int64_t na = t->n_assignments;
    e->pool.run([&](int w) {
      std::vector<int64_t>& miss = e->scratch64[w];
      miss.clear();
      int64_t b, end;
      chunk_of(na, w, T, &b, &end);
      for (int64_t a = b; a < end; ++a) {
        SwCeState& s = t->st[a];
        if (t->asg_active[a] && s.last > 0 && s.last < (uint64_t)lim && s.missing == 0) {
          s.missing = (uint64_t)now_ms;
          miss.push_back(a);
        }
      }
    });
    for (int w = 0; w < T; ++w)
      for (int64_t a : e->scratch64[w]) {
        if ((int64_t)gen.size() >= t->gen_cap) break;
        SwEventRec g;
        memset(&g, 0, sizeof(g));
        g.event_date = now_ms;
        g.name_hash = t->presence_hash;
        g.etype = SW_EV_STATE_CHANGE;
        g.src_rank = (uint8_t)t->rank;
        gen.push_back(g);
        gen_asg.push_back((int32_t)a);
      }
  }
  lap("presence");

  // 9. generated events: intern, persist (parallel rows), state (sharded by assignment)
  const int64_t n_gen = (int64_t)gen.size();
  if (n_gen) {
    intern_in_order(e, gen.data(), nullptr, n_gen);
    SwOutRec* gout = out + n_ok;
    e->pool.run([&](int w) {
      int64_t b, end;
      chunk_of(n_gen, w, T, &b, &end);
      persist_range(e, t, gen.data(), nullptr, nullptr, [&](int64_t j) { return gen_asg[j]; }, cursor, now_ms, gout, b,
                    end, nullptr, prec ? prec + n_ok : nullptr, pspans ? pspans + n_ok : nullptr);
    });
    e->pool.run([&](int sh) {
      for (int64_t j = 0; j < n_gen; ++j)
        if ((uint32_t)gen_asg[j] % (uint32_t)T == (uint32_t)sh)
          state_one(e, t, gen[j], gen_asg[j], (cursor + j) * W + R + 1, now_ms, e->ms[sh]);
    });
    cursor += n_gen;
  }
  lap("gen");
  if (ff_on) {
    e->ff_meta[5] += ff_dropped.load();
    e->ff_meta[6] += ff_ids.load();
    if (e->ff_meta[6] >= e->ff_meta[2]) {     // the live generation has taken its ids: the oldest is
      const int nxt = (int)((ff_live + 1) % e->ff_gens);   // cleared and becomes the live one
      ff_clear(e, nxt);
      e->ff_meta[0] = nxt;
      e->ff_meta[SW_FF_META + nxt] = cursor;
      e->ff_meta[6] = 0;
      e->ff_meta[4] += 1;
    }
  }

  // 10. bookkeeping (SW_STAT_* slots; messages and new names are counted by the caller)
  uint64_t c[8] = {};
  for (int w = 0; w < T; ++w)
    for (int s = 0; s < 8; ++s) c[s] += cnt[w][s];
  uint64_t* S = t->stats;
  S[1] += (uint64_t)n;
  S[2] += (uint64_t)(n_ok + n_gen);
  S[3] += c[SW_ST_UNREGISTERED];
  S[4] += c[SW_ST_UNASSIGNED];
  S[5] += c[SW_ST_DUPLICATE];
  S[6] += c[SW_ST_DECODE_ERROR];
  S[7] += c[SW_ST_CONTROL];
  S[SW_STAT_DEDUP_RECHECKS] += c[SW_ST_RECHECK];
  S[8] += (uint64_t)n_rule;
  S[9] += (uint64_t)(n_gen - n_rule);
  st->cursor = cursor;
  st->seq_base += n;
  st->n_ok = n_ok;
  st->n_gen = n_gen;
  st->n_rule = n_rule;
  st->n_rej = n - n_ok;
  return 0;
}

// Store-backed dedup filter: `buckets` per generation (a power of two, 0 = off), `gens` generations
// (2..SW_FF_MAX_GENS) of `ids_per_gen` persisted ids; cleared, generation 0 live.
int32_t swce_ff_init(void* p, int64_t buckets, int64_t gens, int64_t ids_per_gen) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  if (buckets > 0 && ((buckets & (buckets - 1)) || gens < 2 || gens > SW_FF_MAX_GENS || ids_per_gen <= 0)) return -1;
  e->ff.assign_zero(buckets > 0 ? (size_t)(buckets * gens * SW_FF_SLOTS / 2) : 0);
  if (buckets > 0 && e->ff.empty()) return -2;
  e->ff_bmask = buckets > 0 ? buckets - 1 : 0;
  e->ff_gens = buckets > 0 ? gens : 0;
  memset(e->ff_meta, 0, sizeof(e->ff_meta));
  e->ff_meta[2] = ids_per_gen;
  e->ff_meta[3] = e->ff_gens;
  return 0;
}

// Add ids to generation g (warm start from the store; EngineBase.filter_seed).
void swce_ff_add(void* p, int64_t g, const uint64_t* h, int64_t n) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  if (e->ff.empty() || g < 0 || g >= e->ff_gens) return;
  for (int64_t i = 0; i < n; ++i)
    if (h[i] && !ff_add(e, (int)g, h[i])) e->ff_meta[5] += 1;
}

void swce_ff_clear(void* p, int64_t g) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  if (!e->ff.empty() && g >= 0 && g < e->ff_gens) ff_clear(e, (int)g);
}

// The filter's meta words (SW_FF_META + SW_FF_MAX_GENS): read into `out`, then, with `in`, replaced.
void swce_ff_meta(void* p, int64_t* out, const int64_t* in) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  if (out) memcpy(out, e->ff_meta, sizeof(e->ff_meta));
  if (in) memcpy(e->ff_meta, in, sizeof(e->ff_meta));
}

// Checkpoints keep the filter sparse: the non-empty 64-byte buckets (index into [buckets * gens]
// and their 16 fingerprints).  A multi-GB filter of a small tenant is a few KB.  Returns the count
// of non-empty buckets; writes them only when cap >= count.
int64_t swce_ff_export(void* p, int64_t* idx, uint32_t* rows, int64_t cap) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  if (e->ff.empty()) return 0;
  const int64_t nb = (e->ff_bmask + 1) * e->ff_gens;
  const uint64_t* w = e->ff.data();
  int64_t k = 0;
  for (int64_t b = 0; b < nb; ++b) {
    uint64_t any = 0;
    for (int j = 0; j < SW_FF_SLOTS / 2; ++j) any |= w[b * (SW_FF_SLOTS / 2) + j];
    if (!any) continue;
    if (idx && k < cap) {
      idx[k] = b;
      memcpy(rows + k * SW_FF_SLOTS, w + b * (SW_FF_SLOTS / 2), SW_FF_SLOTS * sizeof(uint32_t));
    }
    ++k;
  }
  return k;
}

// Replace the table by the sparse buckets (everything else empty).
int32_t swce_ff_import(void* p, const int64_t* idx, const uint32_t* rows, int64_t n) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  if (e->ff.empty()) return n ? -1 : 0;
  const int64_t nb = (e->ff_bmask + 1) * e->ff_gens;
  for (int g = 0; g < e->ff_gens; ++g) ff_clear(e, g);
  uint32_t* t = e->ff_tab();
  for (int64_t k = 0; k < n; ++k) {
    if (idx[k] < 0 || idx[k] >= nb) return -2;
    memcpy(t + idx[k] * SW_FF_SLOTS, rows + k * SW_FF_SLOTS, SW_FF_SLOTS * sizeof(uint32_t));
  }
  return 0;
}

// Window sizing of the generational dedup (slots per generation, largest batch in records).
void swce_dedup_window(void* p, int64_t slots, int64_t batch) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  e->dd_slots = slots;
  e->dd_batch = batch;
}

// Previous dedup generation (checkpoints carry both).
int64_t swce_dedup_prev_size(void* p) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  int64_t n = 0;
  for (auto& m : e->dedup_prev) n += (int64_t)m.n;
  return n;
}

int64_t swce_dedup_prev_export(void* p, uint64_t* keys, int64_t* seqs) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  int64_t k = 0;
  for (auto& m : e->dedup_prev) m.for_each([&](uint64_t key, int64_t v) { keys[k] = key; seqs[k] = v; ++k; });
  return k;
}

void swce_dedup_prev_import(void* p, const uint64_t* keys, const int64_t* seqs, int64_t n) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  for (auto& m : e->dedup_prev) m.reset(64);
  for (int64_t i = 0; i < n; ++i)
    *e->dedup_prev[sw_mix64(keys[i]) % (uint64_t)e->T()].insert(keys[i]).first = seqs[i];
}

// ---------------------------------------------------------------- checkpoint export / import
int64_t swce_dedup_size(void* p) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  int64_t n = 0;
  for (auto& m : e->dedup) n += (int64_t)m.n;
  return n;
}

int64_t swce_dedup_export(void* p, uint64_t* keys, int64_t* seqs) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  int64_t k = 0;
  for (auto& m : e->dedup) m.for_each([&](uint64_t key, int64_t v) { keys[k] = key; seqs[k] = v; ++k; });
  return k;
}

void swce_dedup_import(void* p, const uint64_t* keys, const int64_t* seqs, int64_t n) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  for (auto& m : e->dedup) m.reset(64);
  for (int64_t i = 0; i < n; ++i) *e->dedup[sw_mix64(keys[i]) % (uint64_t)e->T()].insert(keys[i]).first = seqs[i];
}

int64_t swce_intern_size(void* p) { return (int64_t)static_cast<SwCpuEngine*>(p)->intern.n; }

int64_t swce_intern_export(void* p, uint64_t* keys, int32_t* ids) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  int64_t k = 0;
  e->intern.for_each([&](uint64_t key, int32_t v) { keys[k] = key; ids[k] = v; ++k; });
  return k;
}

void swce_intern_import(void* p, const uint64_t* keys, const int32_t* ids, int64_t n) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  e->intern.reset(64);
  e->n_intern = 0;
  for (int64_t i = 0; i < n; ++i) {
    *e->intern.insert(keys[i]).first = ids[i];
    e->n_intern = std::max(e->n_intern, ids[i] + 1);
  }
}

int64_t swce_seen_size(void* p) { return (int64_t)static_cast<SwCpuEngine*>(p)->seen.n; }

int64_t swce_seen_export(void* p, uint64_t* keys) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  int64_t k = 0;
  e->seen.for_each([&](uint64_t key, uint8_t) { keys[k++] = key; });
  return k;
}

void swce_seen_import(void* p, const uint64_t* keys, int64_t n) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  e->seen.reset(64);
  for (int64_t i = 0; i < n; ++i) e->seen.insert(keys[i]);
}

int64_t swce_ms_size(void* p) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  int64_t n = 0;
  for (auto& m : e->ms) n += (int64_t)m.n;
  return n;
}

// rows: [asg, name_id, kind, date, eid1] x n (int64)
int64_t swce_ms_export(void* p, int64_t* rows) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  int64_t k = 0;
  for (auto& m : e->ms)
    m.for_each([&](uint64_t key, const MsVal& v) {
      const uint64_t x = key - 1;
      int64_t* o = rows + 5 * k++;
      o[0] = (int64_t)(x >> 32);
      o[1] = (int64_t)((x & 0xFFFFFFFFull) >> 1);
      o[2] = (int64_t)(x & 1);
      o[3] = v.date;
      o[4] = v.eid1;
    });
  return k;
}

void swce_ms_import(void* p, const int64_t* rows, int64_t n) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  for (auto& m : e->ms) m.reset(64);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t* r = rows + 5 * i;
    const uint64_t key = (((uint64_t)(uint32_t)r[0] << 32) | ((uint64_t)(uint32_t)r[1] << 1) | (uint64_t)(r[2] & 1)) + 1;
    MsVal& v = *e->ms[(uint32_t)r[0] % (uint32_t)e->T()].insert(key).first;
    v.date = r[3];
    v.eid1 = r[4];
  }
}

// Last-value state of one assignment: rows [name_id, kind, date, eid1] (int64); returns count.
int64_t swce_ms_of(void* p, int32_t a, int64_t* rows, int64_t cap) {
  SwCpuEngine* e = static_cast<SwCpuEngine*>(p);
  int64_t k = 0;
  e->ms[(uint32_t)a % (uint32_t)e->T()].for_each([&](uint64_t key, const MsVal& v) {
    const uint64_t x = key - 1;
    if ((int64_t)(x >> 32) != a || k >= cap) return;
    int64_t* o = rows + 4 * k++;
    o[0] = (int64_t)((x & 0xFFFFFFFFull) >> 1);
    o[1] = (int64_t)(x & 1);
    o[2] = v.date;
    o[3] = v.eid1;
  });
  return k;
}

}  // extern "C"
