// engine.cpp -- host side of the MI355X causal-log engine (implements include/clonos_engine.h).
//
// Owns: the HBM segment pool (components of determinantBufferSize bytes), the per-log
// metadata with exactly the reference's semantics, host staging of appends, and the
// batching of all byte work into gfx950 kernels (kernels.hip) on one HIP stream.
//
// R/ = /root/reference/flink-runtime/src/main/java/org/apache/flink/runtime/causal/.
// The log metadata mirrors R/log/thread/ThreadCausalLogImpl.java:51-527 line for line in
// behaviour (EpochStartOffset objects shared by reference with ConsumerOffset, Netty
// component-granular discardReadComponents), but the bytes never leave HBM.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <optional>
#include <vector>

#include "../../include/clonos_engine.h"
#include "kernels.h"

static_assert(sizeof(clg_delta_req) == 32, "clg_delta_req layout");

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) return fail(CLG_E_DEVICE, "%s failed: %s", #x, hipGetErrorString(e_)); \
  } while (0)

// A launch helper's CLG_E_DEVICE carries the HIP error into the error text.
void note_launch_error(const char* what) {
  if (const char* m = clg::take_launch_error()) fail(CLG_E_DEVICE, "%s: %s", what, m);
}
#define CHK(x)                                          \
  do {                                                  \
    int r_ = (x);                                       \
    if (r_ != CLG_OK) {                                 \
      if (r_ == CLG_E_DEVICE) note_launch_error(#x);    \
      return r_;                                        \
    }                                                   \
  } while (0)

struct EpochStart {
  int64_t id;
  int32_t offset;
};
struct Consumer {
  std::shared_ptr<EpochStart> es;  // ConsumerOffset.epochStart (a reference, may go stale)
  int32_t offset;
};

// EpochStart objects (with their shared_ptr control blocks) come from a per-thread free
// list: a config-4 step opens an epoch in, and truncates one out of, each of 66 k logs.
template <class T>
struct EpochAlloc {
  using value_type = T;
  EpochAlloc() = default;
  template <class U>
  EpochAlloc(const EpochAlloc<U>&) {}
  struct FreeList : std::vector<void*> {  // a thread's pooled blocks go back at its exit
    ~FreeList() {
      for (void* p : *this) ::operator delete(p);
    }
  };
  static FreeList& free_list() {
    static thread_local FreeList f;
    return f;
  }
  T* allocate(size_t n) {
    auto& f = free_list();
    if (n == 1 && !f.empty()) {
      void* p = f.back();
      f.pop_back();
      return static_cast<T*>(p);
    }
    return static_cast<T*>(::operator new(n * sizeof(T)));
  }
  void deallocate(T* p, size_t n) {
    auto& f = free_list();
    if (n == 1 && f.size() < (1u << 20)) f.push_back(p);
    else ::operator delete(p);
  }
  template <class U>
  bool operator==(const EpochAlloc<U>&) const { return true; }
  template <class U>
  bool operator!=(const EpochAlloc<U>&) const { return false; }
};

// A log's epochs: epoch id -> its start offset, in id order (the reference's
// epochStartOffsets map).  A log holds few epochs between checkpoints, appended in
// increasing order, so they live in a small sorted array, the first kInline inside the Log
// itself: a config-4 step opens an epoch in, and truncates one out of, each of 66 k logs,
// and per-log work is bound by cache misses.  The offset is kept inline; the shared
// EpochStart object (Java's EpochStartOffset, which a ConsumerOffset references) exists
// only once a consumer refers to the epoch (ref()), and rebase() keeps both in step.
struct EpochEnt {
  int64_t id = 0;
  int32_t offset = 0;
  std::shared_ptr<EpochStart> shared;  // null until a ConsumerOffset refers to the epoch
};
class EpochMap {
 public:
  EpochEnt* begin() { return data(); }
  EpochEnt* end() { return data() + n_; }
  const EpochEnt* begin() const { return data(); }
  const EpochEnt* end() const { return data() + n_; }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  EpochEnt* find(int64_t k) {
    EpochEnt* it = lower(k);
    return it != end() && it->id == k ? it : end();
  }
  const EpochEnt* find(int64_t k) const { return const_cast<EpochMap*>(this)->find(k); }
  // computeIfAbsent(k -> offset); the entry stays valid until the next insert or erase
  EpochEnt* emplace(int64_t k, int32_t offset) {
    EpochEnt* it = lower(k);
    if (it != end() && it->id == k) return it;
    const size_t i = size_t(it - begin());
    if (big_.empty() && n_ < kInline) {
      for (size_t j = n_; j > i; --j) inl_[j] = std::move(inl_[j - 1]);
      inl_[i] = EpochEnt{k, offset, nullptr};
    } else {
      if (big_.empty()) {  // spill the inline entries
        big_.reserve(2 * kInline);
        for (uint32_t j = 0; j < n_; ++j) big_.push_back(std::move(inl_[j]));
        for (auto& x : inl_) x.shared.reset();
      }
      big_.insert(big_.begin() + long(i), EpochEnt{k, offset, nullptr});
    }
    ++n_;
    return begin() + i;
  }
  // drop every epoch with id < k (checkpoint completion)
  void erase_below(int64_t k) {
    const size_t d = size_t(lower(k) - begin());
    if (!d) return;
    if (big_.empty()) {
      for (size_t j = d; j < n_; ++j) inl_[j - d] = std::move(inl_[j]);
      for (size_t j = n_ - d; j < n_; ++j) inl_[j].shared.reset();
    } else {
      big_.erase(big_.begin(), big_.begin() + long(d));
    }
    n_ -= uint32_t(d);
  }
  // every offset -= move (the shared objects too: consumers see the rebased offset)
  void rebase(int32_t move) {
    for (EpochEnt& x : *this) {
      x.offset -= move;
      if (x.shared) x.shared->offset = x.offset;
    }
  }
  // the EpochStart object a ConsumerOffset holds (created on first reference)
  static std::shared_ptr<EpochStart> ref(EpochEnt& x) {
    if (!x.shared) x.shared = std::allocate_shared<EpochStart>(EpochAlloc<EpochStart>(), EpochStart{x.id, x.offset});
    return x.shared;
  }

 private:
  static constexpr uint32_t kInline = 2;
  EpochEnt* data() { return big_.empty() ? inl_ : big_.data(); }
  const EpochEnt* data() const { return big_.empty() ? inl_ : big_.data(); }
  EpochEnt* lower(int64_t k) {
    if (n_ == 0 || end()[-1].id < k) return end();  // the common case: a new epoch
    return std::lower_bound(begin(), end(), k, [](const EpochEnt& a, int64_t b) { return a.id < b; });
  }
  uint32_t n_ = 0;
  EpochEnt inl_[kInline];
  std::vector<EpochEnt> big_;  // all entries once more than kInline were held
};

// A log's segments (Netty components), the first kInline inside the Log itself.
class SegList {
 public:
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  uint32_t operator[](size_t i) const { return data()[i]; }
  const uint32_t* begin() const { return data(); }
  const uint32_t* end() const { return data() + n_; }
  void push_back(uint32_t v) {
    if (big_.empty() && n_ < kInline) {
      inl_[n_++] = v;
      return;
    }
    if (big_.empty()) big_.assign(inl_, inl_ + n_);
    big_.push_back(v);
    ++n_;
  }
  // drop the first k (discardReadComponents)
  void erase_front(size_t k) {
    if (!k) return;
    if (big_.empty()) {
      for (size_t j = k; j < n_; ++j) inl_[j - k] = inl_[j];
    } else {
      big_.erase(big_.begin(), big_.begin() + long(k));
      if (big_.size() <= kInline) {  // back inline
        std::copy(big_.begin(), big_.end(), inl_);
        big_.clear();
        big_.shrink_to_fit();
      }
    }
    n_ -= uint32_t(k);
  }

 private:
  static constexpr uint32_t kInline = 6;
  const uint32_t* data() const { return big_.empty() ? inl_ : big_.data(); }
  uint32_t n_ = 0;
  uint32_t inl_[kInline] = {};
  std::vector<uint32_t> big_;  // all segments once more than kInline were held
};
struct ChKey {
  uint64_t lo, hi;
  bool operator==(const ChKey& o) const { return lo == o.lo && hi == o.hi; }
};
struct ChKeyHash {
  size_t operator()(const ChKey& k) const { return std::hash<uint64_t>()(k.lo * 0x9E3779B97F4A7C15ull ^ k.hi); }
};

// JobCausalLogImpl (one per job per TaskManager, JobCausalLogFactory.java:56-67): the
// job's sharing depth (ExecutionConfig.determinantSharingDepth) and its
// latestCompletedCheckpoint, whose CAS gates the fan-out of truncation (:230-246).
struct Job {
  bool open = false;
  uint64_t lo = 0, hi = 0;  // JobID (an AbstractID)
  int32_t depth = CLG_FULL_SHARING;
  int64_t latest_cp = 0;  // JobCausalLogImpl.latestCompletedCheckpoint (:92, :117)
};

struct Log {
  clg_causal_log_id id{};
  uint32_t job = 0;
  int32_t depth = CLG_FULL_SHARING;  // the owning job's sharing depth
  bool open = false;
  SegList segs;                // composite components
  int32_t writer = 0;          // visibleWriterIndex (== composite writerIndex)
  int32_t flushed = 0;         // physical bytes [0, flushed) are resident in HBM
  // Host copy of physical bytes [tail_start, writer): the staged bytes [flushed, writer)
  // plus the most recent flushed ones (clg_config.host_tail_bytes), so a slice of the log's
  // tail -- a consumer keeping up with its producer -- is served without a GPU round trip.
  // tail_start <= flushed <= writer.
  std::vector<uint8_t> tail;
  int32_t tail_start = 0;
  uint32_t pending_bytes() const { return uint32_t(writer - flushed); }
  const uint8_t* pending_data() const { return tail.data() + (flushed - tail_start); }
  EpochMap epochs;
  std::unordered_map<ChKey, Consumer, ChKeyHash> consumers;
};

// In-flight (data) log of one subpartition (InMemorySubpartitionInFlightLogger.java:28-207):
// SortedMap<epoch, List<Buffer>>; each buffer's bytes occupy whole pool segments.
struct IflBuf {
  std::vector<uint32_t> segs;
  uint32_t len;
};
// The spillable logger's replay iterator (SpilledReplayIterator.java:60-401): a consumer and a
// prefetch EpochCursor (:306-394) over the live view tailMap(view) of the epochs.
struct IflCursor {
  int64_t ne = 0;    // nextEpoch
  int64_t off = 0;   // nextEpochOffset
  int64_t last = 0;  // lastEpoch
  int64_t rem = 0;   // remaining
};
struct IflIter {
  bool exists = false;  // currentIterator != null
  int64_t view = 0;     // the tailMap's lower bound (getInFlightIterator's epochID)
  IflCursor con, pre;
};
struct InFlight {
  bool open = false;
  uint32_t type = CLG_IFL_IN_MEMORY;
  bool replaying = false;  // spillable: isReplaying (:58)
  IflIter it;              // spillable: currentIterator (:60)
  std::map<int64_t, std::vector<IflBuf>> epochs;
};

struct IdKey {  // (job, CausalLogID): logs of different jobs never alias
  uint32_t job;
  int16_t v;
  uint8_t main;
  int8_t sub;
  int64_t lo, hi;
  bool operator<(const IdKey& o) const {
    if (job != o.job) return job < o.job;
    if (v != o.v) return v < o.v;
    if (main != o.main) return main < o.main;
    if (main) return false;  // CausalLogID.equals: main logs compare by vertex only
    if (lo != o.lo) return lo < o.lo;
    if (hi != o.hi) return hi < o.hi;
    return sub < o.sub;
  }
};
IdKey key_of(uint32_t job, const clg_causal_log_id& id) {
  IdKey k{job, id.vertex_id, uint8_t(id.is_main ? 1 : 0), id.is_main ? int8_t(0) : id.subpartition,
          id.is_main ? 0 : id.irp_lower, id.is_main ? 0 : id.irp_upper};
  return k;
}

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t n) {
    if (n <= cap) return CLG_OK;
    if (p) hipFree(p);
    p = nullptr;
    size_t c = std::max(n, cap * 2);
    c = (c + 255) & ~size_t(255);
    hipError_t e = hipMalloc(&p, c + 64);
    if (e != hipSuccess) {
      cap = 0;
      return fail(CLG_E_DEVICE, "hipMalloc(%zu) failed: %s", c, hipGetErrorString(e));
    }
    cap = c;
    return CLG_OK;
  }
  ~DevBuf() {
    if (p) hipFree(p);
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

struct PinBuf {
  void* p = nullptr;
  size_t cap = 0;
  unsigned flags = hipHostMallocDefault;  // hipHostMallocCoherent: device atomics reach the host at once
  int ensure(size_t n) {
    if (n <= cap) return CLG_OK;
    if (p) hipHostFree(p);
    p = nullptr;
    size_t c = std::max(n, cap * 2);
    c = (c + 255) & ~size_t(255);
    hipError_t e = hipHostMalloc(&p, c, flags);
    if (e != hipSuccess) {
      cap = 0;
      return fail(CLG_E_DEVICE, "hipHostMalloc(%zu) failed: %s", c, hipGetErrorString(e));
    }
    cap = c;
    return CLG_OK;
  }
  ~PinBuf() {
    if (p) hipHostFree(p);
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

struct Stat {
  uint64_t launches = 0;
  double ms = 0;
  uint64_t bytes = 0;
};
struct PendingTiming {
  std::string name;
  hipEvent_t a, b;
  uint64_t bytes;
};

// Guard bytes either side of the segment pool: the gather and decode kernels issue aligned
// 16-B loads that may start before a piece's first byte or end past its last.
constexpr size_t kPoolGuard = 256;

// Two-level engine lock.  The per-call ThreadCausalLog operations of the drop-in (append,
// hasDelta, offset, slices the host tail holds, logLength, a host-input upstream delta) take
// only the stripe of their log, so task threads appending and Netty threads slicing
// different logs run in parallel -- as on the reference's per-log objects -- without
// touching a shared cache line.  Everything that touches the GPU, the log table or several
// logs at once takes the engine mutex and then every stripe (EXCLUSIVE).  Exclusive is
// re-entrant (clg_job_close -> clg_log_close), and a per-log request from the exclusive
// holder passes through.
constexpr uint32_t kLogStripes = 64;
struct alignas(64) Stripe {
  std::mutex m;
};
struct EngineLock {
  std::mutex m;
  std::atomic<std::thread::id> owner{};
  int depth = 0;
  Stripe stripe[kLogStripes];
  bool owned() const { return owner.load(std::memory_order_relaxed) == std::this_thread::get_id(); }
  void lock() {
    if (owned()) {
      ++depth;
      return;
    }
    m.lock();
    for (auto& s : stripe) s.m.lock();
    owner.store(std::this_thread::get_id(), std::memory_order_relaxed);
    depth = 1;
  }
  void unlock() {
    if (--depth == 0) {
      owner.store(std::thread::id(), std::memory_order_relaxed);
      for (uint32_t i = kLogStripes; i-- > 0;) stripe[i].m.unlock();
      m.unlock();
    }
  }
};
struct XGuard {
  EngineLock& l;
  explicit XGuard(EngineLock& l_) : l(l_) { l.lock(); }
  ~XGuard() { l.unlock(); }
};

// A few host threads for the per-log loops of very large batches (config 4: 66 k logs per
// decode, truncation): run(fn) calls fn(part, parts) once per part, the calling thread taking
// part 0; workers spin briefly for the next job, then sleep.  Jobs only ever come from the
// holder of the engine lock, one at a time.
class WorkPool {
 public:
  explicit WorkPool(unsigned n) : n_(n ? n : 1) {
    for (unsigned i = 1; i < n_; ++i) th_.emplace_back([this, i] { loop(i); });
  }
  ~WorkPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  unsigned size() const { return n_; }
  void run(const std::function<void(unsigned, unsigned)>& fn) {
    if (n_ == 1) {
      fn(0, 1);
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = &fn;
      left_.store(n_ - 1, std::memory_order_relaxed);
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    fn(0, n_);
    while (left_.load(std::memory_order_acquire) != 0) std::this_thread::yield();
  }

 private:
  void loop(unsigned i) {
    uint64_t seen = 0;
    for (;;) {
      // a short spin (the next job of a batch comes within microseconds), then sleep: a longer
      // one burns the box's CPU quota between batches
      const auto t0 = std::chrono::steady_clock::now();
      while (gen_.load(std::memory_order_acquire) == seen &&
             std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(50))
        std::this_thread::yield();
      const std::function<void(unsigned, unsigned)>* job;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || gen_.load(std::memory_order_acquire) != seen; });
        if (stop_) return;
        seen = gen_.load(std::memory_order_acquire);
        job = job_;
      }
      (*job)(i, n_);
      left_.fetch_sub(1, std::memory_order_acq_rel);
    }
  }
  unsigned n_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<unsigned> left_{0};
  const std::function<void(unsigned, unsigned)>* job_ = nullptr;
  bool stop_ = false;
};

}  // namespace

// clg_host_register's ranges: host base -> device address (for CLG_MEM_MAPPED outputs)
namespace {
struct Mapped {
  uintptr_t host;
  uint64_t bytes;
  uintptr_t dev;
};
std::mutex g_map_mu;
std::vector<Mapped> g_mapped;
// The device address of registered host memory [h, h + n) (0: not wholly inside one
// registered range).
uintptr_t clg_mapped_device_address(const void* h, uint64_t n) {
  std::lock_guard<std::mutex> g(g_map_mu);
  for (const Mapped& m : g_mapped)
    if (uintptr_t(h) >= m.host && uintptr_t(h) < m.host + m.bytes && n <= m.host + m.bytes - uintptr_t(h))
      return m.dev + (uintptr_t(h) - m.host);
  return 0;
}
}  // namespace

namespace clg_internal {  // error text for the host-only translation units (response.cpp)
int set_error(int code, const char* msg) { return fail(code, "%s", msg); }
}  // namespace clg_internal

struct clg_engine {
  clg_config cfg{};
  hipStream_t stream = nullptr;
  void* pool_alloc = nullptr;  // pool minus the guard bytes either side
  uint8_t* pool = nullptr;
  std::vector<uint32_t> free_segs;
  // The write path's Serializable candidates per segment (kernels.h SideCar; hdr null: none,
  // every decode tile is scanned), and each segment's life stamp: bumped whenever the segment
  // leaves the free list, carried by the chunks written into it.
  clg::SideCar side{};
  void* side_alloc = nullptr;
  std::vector<uint32_t> seg_life;
  const clg::SideCar* side_arg() const { return side.hdr ? &side : nullptr; }
  // a chunk's life word: the segment's life (31 bits) | 1 << 31 when the request's bytes go on
  // in the next chunk (contiguous in the source: the writer measures streams across it)
  uint32_t life_word(uint32_t seg, bool more) const { return (seg_life[seg] & 0x7FFFFFFFu) | (more ? 0x80000000u : 0u); }
  // the in-flight (data) log's own pool (clg_config.ifl_*)
  void* ifl_alloc = nullptr;
  uint8_t* ifl_pool = nullptr;
  uint32_t ifl_C = 0;
  std::vector<uint32_t> ifl_free;
  uint8_t* ifl_addr(uint32_t s) const { return ifl_pool + size_t(s) * ifl_C; }
  std::vector<Log> logs;
  std::vector<InFlight> ifls;
  std::map<IdKey, uint32_t> by_id;
  std::vector<Job> jobs;  // jobs[0]: the default job (cfg.sharing_depth)
  std::vector<uint32_t> dirty;  // logs with staged (unflushed) bytes: flush() visits only these
  EngineLock mu;
  std::mutex pool_mu;   // free_segs, taken by appends holding only their stripe
  std::mutex dirty_mu;  // dirty, idem

  // staging / scratch
  PinBuf h_stage, h_desc, h_sres, h_outs;
  // Per decode slot (0: synchronous calls; 1, 2: the asynchronous decodes in flight): the
  // read-back of span ranges and abort words, the staged plan, the end-of-read-back event.
  static constexpr uint32_t kSlots = 1 + CLG_DECODE_MAX_INFLIGHT;
  PinBuf h_zres_s[kSlots], h_plan_s[kSlots];
  hipEvent_t zdone[kSlots] = {};
  uint32_t plan_slot = 0;  // the slot stage_plan / enqueue_plan use (launch_fused sets it)
  DevBuf d_stage, d_desc, d_pieces, d_tiles, d_spans, d_agg, d_conv, d_tres, d_sres, d_totals, d_out;
  std::vector<uint64_t> tab_at;  // clg_get_determinants_batch: a log's place in the segment table (UINT64_MAX: none)
  DevBuf d_fconv, d_lanes, d_sums, d_fres, d_flags, d_dbg, d_prof, d_rprof, d_prof2, d_jpos, d_jlen, d_jn, d_defer;
  DevBuf d_o_off, d_o_tag, d_o_v0, d_o_widx, d_o_wrc, d_o_wv1, d_o_wvo, d_o_wvl, d_o_wsub;
  DevBuf d_zctl, d_ztiles, d_zbits;  // fast decode: control words, tiles, record-start bitmaps
  DevBuf d_zjpos, d_zjlen, d_zjn, d_zjwork;  // fast decode: Serializable length tables (phase 3)
  uint32_t zjovf_cap = 1u << 16;  // their overflow arena's entries (grown on demand)
  uint32_t zjwork_min = 0;        // the general walker's work list: at least this many items
  DevBuf d_zbad;                     // fast decode: per-span "chain went wrong" flags
  DevBuf d_sf_meta, d_sf_rec, d_sf_wide;  // per-span fallback: bad-span list, robust outputs
  bool jser_hint = false;            // the last batches held Serializable records: build tables first
  // The count pass's lean speculative walk (decode_fused.hip lean_walk) while the last fast
  // decode's records were almost all fixed-length (wide rows under 1/16): its result is the
  // same either way, its cost grows with wide records.  CLONOS_LEAN=0/1 forces it (developer).
  bool lean_hint = true;
  static int lean_env() {
    static const int v = getenv("CLONOS_LEAN") ? atoi(getenv("CLONOS_LEAN")) : -1;
    return v;
  }
  DevBuf d_rmeta, d_rsizes;          // replay-prep: subpartition span tables / BufferBuilt sizes
  DevBuf d_encin, d_encw, d_encout;  // encode: staged host input, block prefixes, host-output staging
  DevBuf d_hdr;                      // piggyback: delta headers staged for the gather
  // The Serializable walker's spill arena (kernels.h JArena): [used u64 | pad to 256 | bytes].
  // Grown (doubled) whenever a decode reports CLG_E_NOSPACE, i.e. a walk found it full.
  DevBuf d_jarena;
  size_t jarena_bytes = size_t(16) << 20;
  PinBuf h_jused;  // read-backs of the arena's bump counter: [0] decode, [1] replay classification
  // Slices into device memory run on their own stream, overlapping the next decode: the
  // gather only reads log segments, so every pool write (flush / upstream scatter) and
  // every full sync first waits for it (gwait).
  hipStream_t gstream = nullptr;
  hipEvent_t gready = nullptr;
  bool g_pending = false;
  // two descriptor sets, so a gather can be queued while the previous one still runs;
  // gdone[s] marks the end of the last gather that used set s
  PinBuf h_gdesc[2];
  DevBuf d_gdesc[2], d_gpieces[2];
  hipEvent_t gdone[2] = {nullptr, nullptr};
  uint32_t gseq = 0;
  PinBuf h_rmeta;
  PinBuf h_rout;  // replay-prep: the subpartition results, read back in one place (pinned)
  DevBuf d_plan;
  bool fused_decode = true;  // CLG_F_ROBUST_DECODE / CLONOS_DECODE=robust: robust pipeline only
  bool small_decode = true;  // CLG_F_NO_SMALL_DECODE / CLONOS_SMALL=0: no single-launch small batches

  // timing
  std::map<std::string, Stat> stats;
  // Developer host-phase timing (CLONOS_HOST_PROF set): the wall time of host-side work as
  // pseudo-stats "host_*" beside the kernels' (launches = calls, ms = host wall time).
  const bool host_prof = getenv("CLONOS_HOST_PROF") != nullptr;
  struct HostTimer {
    clg_engine* e;
    const char* name;
    std::chrono::steady_clock::time_point t0;
    HostTimer(clg_engine* en, const char* n) : e(en && en->host_prof ? en : nullptr), name(n) {
      if (e) t0 = std::chrono::steady_clock::now();
    }
    ~HostTimer() {
      if (!e) return;
      Stat& s = e->stats[name];
      s.launches++;
      s.ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    // (sections of one call: the time since the last lap, under `lap_name`)
    void lap(const char* lap_name) {
      if (!e) return;
      const auto now = std::chrono::steady_clock::now();
      Stat& s = e->stats[lap_name];
      s.launches++;
      s.ms += std::chrono::duration<double, std::milli>(now - t0).count();
      t0 = now;
    }
  };
  std::vector<PendingTiming> timings;
  std::vector<hipEvent_t> ev_pool;

  uint32_t C() const { return cfg.segment_bytes; }
  uint8_t* seg_addr(uint32_t s) const { return pool + size_t(s) * C(); }

  // ---------------------------------------------------------------- timing helpers
  hipEvent_t get_event() {
    if (!ev_pool.empty()) {
      hipEvent_t e = ev_pool.back();
      ev_pool.pop_back();
      return e;
    }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
  }
  template <class F>
  int timed(const char* name, uint64_t bytes, F&& launch, hipStream_t on = nullptr) {
    if (!(cfg.flags & CLG_F_TIMING)) return launch();
    hipEvent_t a = get_event(), b = get_event();
    hipEventRecord(a, on ? on : stream);
    int r = launch();
    hipEventRecord(b, on ? on : stream);
    timings.push_back(PendingTiming{name, a, b, bytes});
    return r;
  }
  // ready_only: only the timings whose end event has completed (the rest stay pending)
  void collect_timings(bool ready_only = false) {
    if (ready_only) {
      std::vector<PendingTiming> later;
      for (auto& t : timings)
        if (hipEventQuery(t.b) == hipErrorNotReady) later.push_back(t);
      if (!later.empty()) {
        std::vector<PendingTiming> done;
        for (auto& t : timings)
          if (hipEventQuery(t.b) != hipErrorNotReady) done.push_back(t);
        timings.swap(done);
        collect_timings();
        timings.swap(later);
        return;
      }
    }
    for (auto& t : timings) {
      float ms = 0;
      hipEventSynchronize(t.b);
      hipEventElapsedTime(&ms, t.a, t.b);
      Stat& s = stats[t.name];
      s.launches++;
      s.ms += ms;
      s.bytes += t.bytes;
      ev_pool.push_back(t.a);
      ev_pool.push_back(t.b);
    }
    timings.clear();
  }
  int gwait() {
    if (g_pending) {
      g_pending = false;
      HIPCHK(hipStreamSynchronize(gstream));
    }
    return CLG_OK;
  }
  // The arena for kernels queued next on `stream`, its bump counter reset first.
  int jarena_reset(clg::JArena* a) {
    CHK(d_jarena.ensure(jarena_bytes + 256));
    HIPCHK(hipMemsetAsync(d_jarena.p, 0, 8, stream));
    *a = clg::JArena{d_jarena.as<uint8_t>() + 256, jarena_bytes, d_jarena.as<unsigned long long>()};
    return CLG_OK;
  }
  // Queues a read-back of the arena's bump counter into slot k, after the walks queued so
  // far; jarena_spilled(k) (after a sync) says whether any of them found the arena full --
  // then some walk returned kJsSpill and whatever the kernels derived from it is void.
  int jarena_note(int k) {
    CHK(h_jused.ensure(64));
    HIPCHK(hipMemcpyAsync(h_jused.as<uint64_t>() + k, d_jarena.p, 8, hipMemcpyDeviceToHost, stream));
    return CLG_OK;
  }
  int jarena_clear_note(int k) {
    CHK(h_jused.ensure(64));
    h_jused.as<uint64_t>()[k] = 0;
    return CLG_OK;
  }
  bool jarena_spilled(int k) const { return h_jused.p && h_jused.as<uint64_t>()[k] > jarena_bytes; }
  int jarena_grow() {
    CHK(sync());  // kernels still using the old arena
    if (jarena_bytes >= (size_t(1) << 36))
      return fail(CLG_E_DEVICE, "Serializable walker spill arena would exceed 64 GiB");
    jarena_bytes *= 2;
    stats["jser_arena_grow"].launches++;
    return CLG_OK;
  }

  int sync() {
    CHK(gwait());
    HIPCHK(hipStreamSynchronize(stream));
    collect_timings();
    return CLG_OK;
  }

  // ---------------------------------------------------------------- segments
  int32_t capacity(const Log& l) const { return int32_t(l.segs.size()) * int32_t(C()); }
  // notEnoughSpaceFor / addComponent (:351-353, :438-452): all-or-nothing.
  int ensure_space(Log& l, int32_t n) {
    if (int64_t(l.writer) + n <= capacity(l)) return CLG_OK;
    std::lock_guard<std::mutex> g(pool_mu);
    return ensure_space_locked(l, n);
  }
  int ensure_space_locked(Log& l, int32_t n) {  // pool_mu held
    int64_t need_bytes = int64_t(l.writer) + n - capacity(l);
    if (need_bytes <= 0) return CLG_OK;
    size_t need = size_t((need_bytes + C() - 1) / C());
    if (need > free_segs.size())
      return fail(CLG_E_NOSPACE, "segment pool exhausted (need %zu, free %zu)", need, free_segs.size());
    for (size_t i = 0; i < need; ++i) {
      l.segs.push_back(free_segs.back());
      ++seg_life[free_segs.back()];
      free_segs.pop_back();
    }
    return CLG_OK;
  }
  void write_pending(Log& l, const uint8_t* b, uint32_t n) {
    if (l.flushed == l.writer && n) {
      std::lock_guard<std::mutex> g(dirty_mu);
      dirty.push_back(uint32_t(&l - logs.data()));
    }
    l.tail.insert(l.tail.end(), b, b + n);
    l.writer += int32_t(n);
  }
  // epochStartOffsets.computeIfAbsent(e -> visibleWriterIndex); valid until the next insert
  static EpochEnt* compute_if_absent(Log& l, int64_t e) { return l.epochs.emplace(e, l.writer); }
  int32_t bytes_to_send(const Log& l, int64_t epoch, int32_t phys) const {  // :384-395
    auto it = l.epochs.find(epoch + 1);
    return (it != l.epochs.end() ? it->offset : l.writer) - phys;
  }

  int get_log(uint32_t h, Log** out) {
    if (h >= logs.size() || !logs[h].open) return fail(CLG_E_NO_LOG, "unknown log handle %u", h);
    *out = &logs[h];
    return CLG_OK;
  }

  // ---------------------------------------------------------------- flush (append scatter)
  // Drops flushed bytes from the front of a log's host tail beyond the configured keep.
  void trim_tail(Log& l) {
    const size_t keep = cfg.host_tail_bytes;
    const size_t flushed_in_tail = size_t(l.flushed - l.tail_start);
    if (flushed_in_tail <= 2 * keep) return;  // amortised: trim to `keep` once it doubled
    const size_t drop = flushed_in_tail - keep;
    l.tail.erase(l.tail.begin(), l.tail.begin() + long(drop));
    l.tail_start += int32_t(drop);
  }
  // Staged (unflushed) bytes of one log are bounded: past this the append that crossed it
  // flushes (the host holds at most ~this + host_tail_bytes per log).
  bool over_stage_limit(uint32_t h) const {
    const uint32_t lim = std::max<uint32_t>(65536u, 2u * cfg.host_tail_bytes);
    return h < logs.size() && logs[h].open && logs[h].pending_bytes() > lim;
  }
  // Forget the host tail (bytes were written to HBM behind its back).
  static void reset_tail(Log& l) {
    l.tail.clear();
    l.tail_start = l.writer;
  }

  int flush() {
    size_t total = 0, nchunks = 0;
    for (uint32_t h : dirty) {
      const Log& l = logs[h];
      if (l.open && l.pending_bytes()) {
        total += l.pending_bytes();
        nchunks += l.pending_bytes() / C() + 2;
      }
    }
    if (total == 0) {
      dirty.clear();
      return CLG_OK;
    }
    CHK(gwait());  // an in-flight gather may still read the segments about to be written
    const size_t desc_bytes = nchunks * sizeof(clg::ScatterChunk);
    CHK(h_stage.ensure(total));
    CHK(h_desc.ensure(desc_bytes));
    CHK(d_stage.ensure(total));
    CHK(d_desc.ensure(desc_bytes));
    uint8_t* hs = h_stage.as<uint8_t>();
    clg::ScatterChunk* ch = h_desc.as<clg::ScatterChunk>();
    size_t off = 0, n = 0;
    for (uint32_t h : dirty) {
      Log& l = logs[h];
      const uint32_t pb = l.open ? l.pending_bytes() : 0u;
      if (!pb) continue;
      memcpy(hs + off, l.pending_data(), pb);
      int32_t p = l.flushed;
      size_t src = off;
      size_t left = pb;
      while (left) {
        const uint32_t si = uint32_t(p) / C(), so = uint32_t(p) % C();
        const uint32_t take = uint32_t(std::min<size_t>(left, C() - so));
        ch[n++] = clg::ScatterChunk{seg_addr(l.segs[si]) + so, src, take, life_word(l.segs[si], left > take)};
        p += int32_t(take);
        src += take;
        left -= take;
      }
      off += pb;
      l.flushed = l.writer;
      trim_tail(l);
    }
    dirty.clear();
    HIPCHK(hipMemcpyAsync(d_stage.p, hs, total, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(d_desc.p, ch, n * sizeof(clg::ScatterChunk), hipMemcpyHostToDevice, stream));
    CHK(timed("append_scatter", 2 * total, [&] {
      return clg::launch_scatter(d_desc.as<clg::ScatterChunk>(), uint32_t(n), d_stage.as<uint8_t>(), stream, side_arg());
    }));
    // the pinned staging buffers are reused by the next flush: wait for the copies
    HIPCHK(hipStreamSynchronize(stream));
    return CLG_OK;
  }

  // ---------------------------------------------------------------- ThreadCausalLog ops
  int append(uint32_t h, int64_t epoch, const uint8_t* b, uint32_t n) {  // :158-177
    Log* l;
    CHK(get_log(h, &l));
    if (l->depth == 0) return CLG_OK;
    if (n && !b) return fail(CLG_E_INVALID_ARG, "null record");
    CHK(ensure_space(*l, int32_t(n)));
    compute_if_absent(*l, epoch);
    write_pending(*l, b, n);
    return CLG_OK;
  }

  int upstream(uint32_t h, int64_t epoch, int32_t off_from_epoch, const uint8_t* d, uint32_t n) {  // :117-154
    Log* l;
    CHK(get_log(h, &l));
    if (n == 0) return CLG_OK;
    if (!d) return fail(CLG_E_INVALID_ARG, "null delta");
    auto es = compute_if_absent(*l, epoch);
    const int32_t cur = l->writer - es->offset;
    const int32_t num_new = (off_from_epoch + int32_t(n)) - cur;
    if (num_new > 0) {
      // :136-137 add components before delta.readerIndex(<0) throws (:143): capacity grows
      CHK(ensure_space(*l, num_new));
      if (num_new > int32_t(n))
        return fail(CLG_E_GAP, "upstream delta leaves a gap: offsetFromEpoch %d, %u bytes, log at %d", off_from_epoch,
                    n, cur);
      write_pending(*l, d + (n - uint32_t(num_new)), uint32_t(num_new));
    }
    return CLG_OK;
  }

  // Batched processUpstreamDelta (:117-154) over one input buffer.  Device input (e.g.
  // an RCCL receive buffer) is scattered straight into the log segments: pending host
  // bytes are flushed first, so the logs' byte order is preserved.
  int upstream_batch(clg_delta_req* r, uint32_t n, const uint8_t* bytes, uint32_t in_kind) {
    HostTimer ht(this, "host_upstream_batch");
    if (in_kind != CLG_MEM_DEVICE) {
      for (uint32_t i = 0; i < n; ++i) {
        r[i].status = upstream(r[i].log, r[i].epoch, r[i].offset_from_epoch, bytes + r[i].src_off, r[i].len);
      }
      return CLG_OK;
    }
    std::optional<HostTimer> hsub(std::in_place, this, "host_up_wait");  // (CLONOS_HOST_PROF sub-stages)
    CHK(flush());
    CHK(gwait());  // the scatter below writes segments an in-flight gather may read
    hsub.reset();
    if (n >= kParallelLogs) {
      int st = CLG_OK;
      if (upstream_parallel(r, n, bytes, &st)) return st;
    }
    // the chunks go straight into the pinned descriptor buffer (a config-4 batch has 66 k of
    // them: a fresh vector per call cost page faults, and a copy)
    size_t bound = 0;
    for (uint32_t i = 0; i < n; ++i) bound += r[i].len / C() + 2;
    CHK(h_desc.ensure(std::max<size_t>(1, bound) * sizeof(clg::ScatterChunk)));
    clg::ScatterChunk* ch = h_desc.as<clg::ScatterChunk>();
    size_t nch = 0, total = 0;
    std::unique_lock<std::mutex> pool_guard(pool_mu);  // once for the batch, not per log
    for (uint32_t i = 0; i < n; ++i) {
      r[i].status = CLG_OK;
      Log* l;
      if ((r[i].status = get_log(r[i].log, &l)) != CLG_OK || r[i].len == 0) continue;
      auto es = compute_if_absent(*l, r[i].epoch);
      const int32_t cur = l->writer - es->offset;
      const int32_t num_new = (r[i].offset_from_epoch + int32_t(r[i].len)) - cur;
      if (num_new <= 0) continue;
      if ((r[i].status = ensure_space_locked(*l, num_new)) != CLG_OK) continue;  // before the gap check (:136-143)
      if (num_new > int32_t(r[i].len)) {
        r[i].status = fail(CLG_E_GAP, "upstream delta leaves a gap: offsetFromEpoch %d, %u bytes, log at %d",
                           r[i].offset_from_epoch, r[i].len, cur);
        continue;
      }
      int32_t p = l->writer;
      uint64_t src = r[i].src_off + (r[i].len - uint32_t(num_new));
      uint32_t left = uint32_t(num_new);
      while (left) {
        const uint32_t si = uint32_t(p) / C(), so = uint32_t(p) % C();
        const uint32_t take = std::min<uint32_t>(left, C() - so);
        ch[nch++] = clg::ScatterChunk{seg_addr(l->segs[si]) + so, src, take, life_word(l->segs[si], left > take)};
        p += int32_t(take);
        src += take;
        left -= take;
      }
      l->writer += num_new;
      l->flushed = l->writer;
      reset_tail(*l);  // these bytes go to HBM only
      total += size_t(num_new);
    }
    pool_guard.unlock();
    if (!nch) return CLG_OK;
    const size_t db = nch * sizeof(clg::ScatterChunk);
    CHK(d_desc.ensure(db));
    HIPCHK(hipMemcpyAsync(d_desc.p, h_desc.p, db, hipMemcpyHostToDevice, stream));
    CHK(timed("upstream_scatter", 2 * total, [&] {
      return clg::launch_scatter(d_desc.as<clg::ScatterChunk>(), uint32_t(nch), bytes, stream, side_arg());
    }));
    return sync();  // the caller's buffer and the pinned descriptors are free again
  }

  // upstream_batch's device-input loop on the host threads, for batches of many distinct logs
  // (config 4: 66 k): per part each request's new bytes and the segments it needs; then, in
  // request order, the segments taken from the pool (a request the pool cannot serve gets
  // CLG_E_NOSPACE with nothing taken, a gap CLG_E_GAP after its segments were added -- as one by
  // one) and each request's place among the scatter chunks; then per part the segments
  // attached, the chunks written and the logs advanced.  false: not applicable (a log twice).
  std::vector<uint8_t> up_seen;
  struct UpPlan {
    int32_t num_new, writer, cur;  // (the log's writer and offset in the epoch, read in the first pass)
    uint32_t need, chunks;
    uint64_t seg_from, ch_from;
  };
  std::vector<UpPlan> up_plan;
  bool upstream_parallel(clg_delta_req* r, uint32_t n, const uint8_t* bytes, int* out_st) {
    std::optional<HostTimer> hsub(std::in_place, this, "host_up_seen");
    up_seen.assign(logs.size(), 0);
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t h = r[i].log;
      if (h < logs.size()) {
        if (up_seen[h]) return false;  // two deltas of one log apply in order: the serial loop
        up_seen[h] = 1;
      }
    }
    WorkPool* wp = workers();
    const unsigned P = wp->size();
    const uint32_t per = (n + P - 1) / P, Cb = C();
    up_plan.resize(n);
    // per part: segments, chunks and bytes it needs, and whether a request leaves a gap
    struct UpPart {
      uint64_t need = 0, chunks = 0, bytes = 0;
      bool gap = false;
    };
    std::vector<UpPart> upart(P + 1);
    hsub.emplace(this, "host_up_pass1");
    wp->run([&](unsigned k, unsigned) {
      UpPart q;
      for (uint32_t i = k * per; i < std::min(n, (k + 1) * per); ++i) {
        UpPlan& u = up_plan[i];
        u = UpPlan{0, 0, 0, 0, 0, 0, 0};
        r[i].status = CLG_OK;
        Log* l;
        if ((r[i].status = get_log(r[i].log, &l)) != CLG_OK || r[i].len == 0) continue;
        auto es = compute_if_absent(*l, r[i].epoch);
        const int32_t cur = l->writer - es->offset;
        const int32_t num_new = (r[i].offset_from_epoch + int32_t(r[i].len)) - cur;
        if (num_new <= 0) continue;
        const int64_t need_bytes = int64_t(l->writer) + num_new - capacity(*l);
        u.num_new = num_new;
        u.writer = l->writer;
        u.cur = cur;
        u.need = need_bytes > 0 ? uint32_t((need_bytes + Cb - 1) / Cb) : 0u;
        q.need += u.need;
        if (num_new > int32_t(r[i].len)) {
          q.gap = true;
        } else {
          const uint32_t p = uint32_t(u.writer);
          u.chunks = (p + uint32_t(num_new) - 1) / Cb - p / Cb + 1;
          q.chunks += u.chunks;
          q.bytes += uint64_t(num_new);
        }
      }
      upart[k + 1] = q;
    });
    hsub.emplace(this, "host_up_serial");
    std::unique_lock<std::mutex> pool_guard(pool_mu);
    const size_t top = free_segs.size();
    size_t taken = 0, nch = 0, total = 0;
    bool any_gap = false;
    for (unsigned k = 0; k < P; ++k) {
      any_gap |= upart[k + 1].gap;
      upart[k + 1].need += upart[k].need;
      upart[k + 1].chunks += upart[k].chunks;
      upart[k + 1].bytes += upart[k].bytes;
    }
    // every request served (the usual batch): each part places its own segments and chunks
    // from the parts' prefix in the second pass, as the request-order loop below would
    const bool placed_in_parts = !any_gap && upart[P].need <= top;
    if (placed_in_parts) {
      taken = upart[P].need;
      nch = upart[P].chunks;
      total = upart[P].bytes;
    } else for (uint32_t i = 0; i < n; ++i) {  // request order: the pool and the chunk list
      UpPlan& u = up_plan[i];
      if (!u.num_new) continue;
      if (u.need > top - taken) {
        r[i].status = fail(CLG_E_NOSPACE, "segment pool exhausted (need %u, free %zu)", u.need, top - taken);
        u.num_new = 0;
        u.need = 0;
        continue;
      }
      u.seg_from = taken;
      taken += u.need;
      if (u.num_new > int32_t(r[i].len)) {  // the segments stay (:136-143), nothing is written
        r[i].status = fail(CLG_E_GAP, "upstream delta leaves a gap: offsetFromEpoch %d, %u bytes, log at %d",
                           r[i].offset_from_epoch, r[i].len, u.cur);
        u.num_new = 0;
        continue;
      }
      u.ch_from = nch;  // (u.chunks from the first pass: no log record touched here)
      nch += u.chunks;
      total += size_t(u.num_new);
    }
    if (int st = h_desc.ensure(std::max<size_t>(1, nch) * sizeof(clg::ScatterChunk)); st != CLG_OK) {
      *out_st = st;
      return true;
    }
    clg::ScatterChunk* ch = h_desc.as<clg::ScatterChunk>();
    hsub.emplace(this, "host_up_pass2");
    wp->run([&](unsigned k, unsigned) {
      uint64_t sf = upart[k].need, cf = upart[k].chunks;
      for (uint32_t i = k * per; i < std::min(n, (k + 1) * per); ++i) {
        UpPlan& u = up_plan[i];
        if (placed_in_parts && u.num_new) {
          u.seg_from = sf;
          sf += u.need;
          u.ch_from = cf;
          cf += u.chunks;
        }
        if (!u.need && !u.num_new) continue;
        Log& l = logs[r[i].log];
        for (uint32_t j = 0; j < u.need; ++j) {  // pop order
          const uint32_t sg = free_segs[top - 1 - (u.seg_from + j)];
          l.segs.push_back(sg);
          ++seg_life[sg];  // (each segment is taken by one part)
        }
        if (!u.num_new) continue;
        int32_t p = l.writer;
        uint64_t src = r[i].src_off + (r[i].len - uint32_t(u.num_new));
        uint32_t left = uint32_t(u.num_new);
        uint64_t c = u.ch_from;
        while (left) {
          const uint32_t si = uint32_t(p) / Cb, so = uint32_t(p) % Cb;
          const uint32_t take = std::min<uint32_t>(left, Cb - so);
          ch[c++] = clg::ScatterChunk{seg_addr(l.segs[si]) + so, src, take, life_word(l.segs[si], left > take)};
          p += int32_t(take);
          src += take;
          left -= take;
        }
        l.writer += u.num_new;
        l.flushed = l.writer;
        reset_tail(l);  // these bytes go to HBM only
      }
    });
    free_segs.resize(top - taken);
    pool_guard.unlock();
    hsub.emplace(this, "host_up_gpu");
    *out_st = CLG_OK;
    if (!nch) return true;
    const size_t db = nch * sizeof(clg::ScatterChunk);
    if ((*out_st = d_desc.ensure(db)) != CLG_OK) return true;
    if (hipMemcpyAsync(d_desc.p, h_desc.p, db, hipMemcpyHostToDevice, stream) != hipSuccess) {
      *out_st = fail(CLG_E_DEVICE, "hipMemcpyAsync failed");
      return true;
    }
    if ((*out_st = timed("upstream_scatter", 2 * total, [&] {
           return clg::launch_scatter(d_desc.as<clg::ScatterChunk>(), uint32_t(nch), bytes, stream, side_arg());
         })) != CLG_OK)
      return true;
    *out_st = sync();
    return true;
  }

  int has_delta(uint32_t h, ChKey k, int64_t epoch, int32_t* out) {  // :196-240
    Log* l;
    CHK(get_log(h, &l));
    *out = 0;
    if (l->depth == 0) return CLG_OK;
    auto it = l->epochs.find(epoch);
    if (it == l->epochs.end()) return CLG_OK;
    auto ci = l->consumers.find(k);
    if (ci == l->consumers.end()) ci = l->consumers.emplace(k, Consumer{EpochMap::ref(*it), 0}).first;
    Consumer& c = ci->second;
    if (c.es->id != epoch) {
      if (c.es->id > epoch)
        return fail(CLG_E_CONSUMER_BACKWARDS, "Consumer went backwards, current epoch %lld requested %lld",
                    (long long)c.es->id, (long long)epoch);
      c.es = EpochMap::ref(*it);
      c.offset = 0;
    }
    *out = bytes_to_send(*l, epoch, c.es->offset + c.offset) != 0;
    return CLG_OK;
  }

  int offset_from_epoch(uint32_t h, ChKey k, int32_t* out) {  // :243-246
    Log* l;
    CHK(get_log(h, &l));
    auto ci = l->consumers.find(k);
    if (ci == l->consumers.end()) return fail(CLG_E_NO_CONSUMER, "consumer not registered on log %u", h);
    *out = ci->second.offset;
    return CLG_OK;
  }

  // getDeltaForConsumer :249-277, metadata half: returns (phys, nb) and advances.
  int take_delta(uint32_t h, ChKey k, int64_t epoch, int32_t* phys, int32_t* nb) {
    Log* l;
    CHK(get_log(h, &l));
    auto ci = l->consumers.find(k);
    if (ci == l->consumers.end()) return fail(CLG_E_NO_CONSUMER, "consumer not registered on log %u", h);
    Consumer& c = ci->second;
    const int32_t p = c.es->offset + c.offset;
    const int32_t n = bytes_to_send(*l, epoch, p);
    if (n < 0 || p < 0 || int64_t(p) + n > capacity(*l))
      return fail(CLG_E_STATE, "delta [%d, %d) outside log of capacity %d", p, p + n, capacity(*l));
    c.offset += n;
    *phys = p;
    *nb = n;
    return CLG_OK;
  }

  // Pieces of [phys, phys+n) of a log, split at segment boundaries.
  void add_pieces(const Log& l, int32_t phys, int32_t n, uint64_t dst, std::vector<clg::GatherPiece>& out) {
    while (n > 0) {
      const uint32_t si = uint32_t(phys) / C(), so = uint32_t(phys) % C();
      const uint32_t take = std::min<uint32_t>(uint32_t(n), C() - so);
      out.push_back(clg::GatherPiece{seg_addr(l.segs[si]) + so, dst, take, 0});
      phys += int32_t(take);
      dst += take;
      n -= int32_t(take);
    }
  }

  int run_gather(const std::vector<clg::GatherPiece>& pieces, uint64_t total, void* out, uint32_t out_kind,
                 const char* stat = "slice_gather", bool wait = true) {
    if (pieces.empty()) return CLG_OK;
    const size_t db = pieces.size() * sizeof(clg::GatherPiece);
    CHK(h_desc.ensure(db));
    CHK(d_desc.ensure(db));
    memcpy(h_desc.p, pieces.data(), db);
    HIPCHK(hipMemcpyAsync(d_desc.p, h_desc.p, db, hipMemcpyHostToDevice, stream));
    uint8_t* dout;
    if (out_kind == CLG_MEM_DEVICE) {
      dout = static_cast<uint8_t*>(out);
    } else {
      CHK(d_out.ensure(total));
      dout = d_out.as<uint8_t>();
    }
    CHK(timed(stat, 2 * total, [&] {
      return clg::launch_gather(d_desc.as<clg::GatherPiece>(), uint32_t(pieces.size()), dout, stream);
    }));
    if (out_kind != CLG_MEM_DEVICE) HIPCHK(hipMemcpyAsync(out, dout, total, hipMemcpyDeviceToHost, stream));
    return wait || out_kind != CLG_MEM_DEVICE ? sync() : CLG_OK;
  }

  // The gather's descriptors, staged: runs | segment table; *o: where each part starts.
  // (Tried and removed: pieces in source order -- every consumer's piece of one segment back
  // to back on one XCD, for L2 hits -- took the isolated config-2 gather from 0.39 to 0.43 ms
  // and cost 0.1 ms of host grouping per step.  Round 5: a segment-major gather, one block per
  // log segment copying it for every consumer of that log (each segment read from HBM once):
  // in the config-2 step the gather fell from 0.68 to 0.54 ms but the decode beside it rose
  // from 0.62 to 0.75 and the step from 0.732 to 0.786 ms; isolated 0.46 against 0.39 ms.
  // The re-reads are not what bounds the step.)
  static size_t al16(size_t x) { return (x + 15) & ~size_t(15); }
  static size_t gather_desc_layout(const std::vector<clg::SegSpan>& runs, const std::vector<uint32_t>& segtab,
                                   size_t o[2]) {
    o[0] = 0;
    o[1] = al16(runs.size() * sizeof(clg::SegSpan));
    return o[1] + segtab.size() * 4;
  }
  static void gather_desc_fill(uint8_t* h, const std::vector<clg::SegSpan>& runs, const std::vector<uint32_t>& segtab,
                               const size_t o[2]) {
    memcpy(h + o[0], runs.data(), runs.size() * sizeof(clg::SegSpan));
    memcpy(h + o[1], segtab.data(), segtab.size() * 4);
  }
  int gather_expand(const uint8_t* d, const std::vector<clg::SegSpan>& runs, const size_t o[2], uint32_t n_pieces,
                    clg::GatherPiece* pieces, hipStream_t on) {
    return clg::launch_expand_pieces(reinterpret_cast<const clg::SegSpan*>(d), uint32_t(runs.size()), n_pieces,
                                     reinterpret_cast<const uint32_t*>(d + o[1]), pool, C(), pieces, on);
  }

  // Batched gather from runs: pieces are generated on the device (k_expand_pieces).
  int run_gather_runs(const std::vector<clg::SegSpan>& runs, const std::vector<uint32_t>& segtab, uint32_t n_pieces,
                      uint64_t total, void* out, uint32_t out_kind) {
    if (runs.empty() || !n_pieces) return CLG_OK;
    if (out_kind == CLG_MEM_DEVICE && (cfg.flags & CLG_F_ASYNC_SLICE))
      return gather_runs_async(runs, segtab, n_pieces, total, out);
    size_t o[2];
    const size_t hb = gather_desc_layout(runs, segtab, o);
    CHK(h_desc.ensure(hb));
    CHK(d_desc.ensure(hb));
    CHK(d_pieces.ensure(size_t(n_pieces) * sizeof(clg::GatherPiece)));
    gather_desc_fill(h_desc.as<uint8_t>(), runs, segtab, o);
    HIPCHK(hipMemcpyAsync(d_desc.p, h_desc.p, hb, hipMemcpyHostToDevice, stream));
    CHK(gather_expand(d_desc.as<uint8_t>(), runs, o, n_pieces, d_pieces.as<clg::GatherPiece>(), stream));
    uint8_t* dout;
    if (out_kind == CLG_MEM_DEVICE) {
      dout = static_cast<uint8_t*>(out);
    } else {
      CHK(d_out.ensure(total));
      dout = d_out.as<uint8_t>();
    }
    CHK(timed("slice_gather", 2 * total, [&] {
      return clg::launch_gather(d_pieces.as<clg::GatherPiece>(), n_pieces, dout, stream);
    }));
    if (out_kind != CLG_MEM_DEVICE) HIPCHK(hipMemcpyAsync(out, dout, total, hipMemcpyDeviceToHost, stream));
    return sync();
  }

  // Device-output slice gather on gstream, after everything already queued on `stream`
  // (appends); returns without waiting.  Its own descriptor buffers, so the next decode
  // on `stream` does not touch them; the next gather waits for this one first.
  int gather_runs_async(const std::vector<clg::SegSpan>& runs, const std::vector<uint32_t>& segtab, uint32_t n_pieces,
                        uint64_t total, void* out) {
    const uint32_t set = gseq++ & 1u;
    if (gdone[set]) HIPCHK(hipEventSynchronize(gdone[set]));  // the gather two calls ago released this set
    else HIPCHK(hipEventCreateWithFlags(&gdone[set], hipEventDisableTiming));
    size_t o[2];
    const size_t hb = gather_desc_layout(runs, segtab, o);
    PinBuf& hd = h_gdesc[set];
    DevBuf& dd = d_gdesc[set];
    DevBuf& dp = d_gpieces[set];
    CHK(hd.ensure(hb));
    CHK(dd.ensure(hb));
    CHK(dp.ensure(size_t(n_pieces) * sizeof(clg::GatherPiece)));
    gather_desc_fill(hd.as<uint8_t>(), runs, segtab, o);
    // no wait on `stream`: every pool write (flush, upstream scatter) has completed when
    // its call returned, and decodes only read the pool
    HIPCHK(hipMemcpyAsync(dd.p, hd.p, hb, hipMemcpyHostToDevice, gstream));
    CHK(gather_expand(dd.as<uint8_t>(), runs, o, n_pieces, dp.as<clg::GatherPiece>(), gstream));
    CHK(timed("slice_gather", 2 * total, [&] {
      return clg::launch_gather(dp.as<clg::GatherPiece>(), n_pieces, static_cast<uint8_t*>(out), gstream);
    }, gstream));
    HIPCHK(hipEventRecord(gdone[set], gstream));
    g_pending = true;
    return CLG_OK;
  }

  // host_only: serve the slice from the host tail or return kNeedGpu with nothing changed
  // (the caller holds only the shared lock and retries under the exclusive one).
  static constexpr int kNeedGpu = 1;
  int get_delta(uint32_t h, ChKey k, int64_t epoch, void* out, uint32_t cap, uint32_t kind, uint32_t* n,
                bool host_only = false) {
    *n = 0;
    Log* l;
    CHK(get_log(h, &l));
    auto ci = l->consumers.find(k);
    if (ci == l->consumers.end()) return fail(CLG_E_NO_CONSUMER, "consumer not registered on log %u", h);
    {
      const int32_t p = ci->second.es->offset + ci->second.offset;
      const int32_t nb = bytes_to_send(*l, epoch, p);
      if (nb < 0 || p < 0 || int64_t(p) + nb > capacity(*l))
        return fail(CLG_E_STATE, "delta [%d, %d) outside log of capacity %d", p, p + nb, capacity(*l));
      if (uint32_t(nb) > cap) {
        *n = uint32_t(nb);  // required size (the consumer does not advance)
        return fail(CLG_E_CAPACITY, "delta needs %d bytes", nb);
      }
      if (kind == CLG_MEM_HOST && p >= l->tail_start && p + nb <= l->writer) {  // the host tail holds it
        int32_t phys, nb2;
        CHK(take_delta(h, k, epoch, &phys, &nb2));
        if (nb2) memcpy(out, l->tail.data() + (phys - l->tail_start), size_t(nb2));
        *n = uint32_t(nb2);
        return CLG_OK;
      }
    }
    if (host_only) return kNeedGpu;
    CHK(flush());
    int32_t phys, nb;
    CHK(take_delta(h, k, epoch, &phys, &nb));
    std::vector<clg::GatherPiece> pieces;
    add_pieces(*l, phys, nb, 0, pieces);
    CHK(run_gather(pieces, uint64_t(nb), out, kind));
    *n = uint32_t(nb);
    return CLG_OK;
  }

  int determinants_range(const Log& l, int64_t start_epoch, int32_t* start, int32_t* nb) {  // :285-313
    int32_t s = 0;
    auto it = l.epochs.find(start_epoch);
    if (it != l.epochs.end())
      s = it->offset;
    else if (!l.epochs.empty())
      s = l.epochs.begin()->offset;
    *start = s;
    *nb = l.writer - s;
    if (*nb < 0 || s < 0 || l.writer > capacity(l))  // makeDeltaUnsafe IndexOutOfBounds
      return fail(CLG_E_STATE, "determinant range [%d, %d) outside the log", s, l.writer);
    return CLG_OK;
  }

  int get_determinants(uint32_t h, int64_t start_epoch, void* out, uint32_t cap, uint32_t kind, uint32_t* n,
                       bool host_only = false) {
    *n = 0;
    Log* l;
    CHK(get_log(h, &l));
    if (l->depth == 0) return CLG_OK;
    int32_t s, nb;
    CHK(determinants_range(*l, start_epoch, &s, &nb));
    if (uint32_t(nb) > cap) {
      *n = uint32_t(nb);  // required size
      return fail(CLG_E_CAPACITY, "getDeterminants needs %d bytes", nb);
    }
    if (kind == CLG_MEM_HOST && s >= l->tail_start) {  // the host tail holds it
      if (nb) memcpy(out, l->tail.data() + (s - l->tail_start), size_t(nb));
      *n = uint32_t(nb);
      return CLG_OK;
    }
    if (host_only) return kNeedGpu;
    CHK(flush());
    std::vector<clg::GatherPiece> pieces;
    add_pieces(*l, s, nb, 0, pieces);
    CHK(run_gather(pieces, uint64_t(nb), out, kind));
    *n = uint32_t(nb);
    return CLG_OK;
  }

  // notifyCheckpointComplete :398-435 (flushes first so no staged byte lives in a dropped
  // component).
  int checkpoint_complete(Log& l, int64_t cp) { return checkpoint_complete(l, cp, free_segs); }
  // (freed: where the dropped segments go -- a host thread's own list in the parallel truncation)
  int checkpoint_complete(Log& l, int64_t cp, std::vector<uint32_t>& freed) {
    const int32_t R = compute_if_absent(l, cp)->offset;  // (read before the erase moves entries)
    l.epochs.erase_below(cp);
    if (R < 0 || R > l.writer) return fail(CLG_E_STATE, "readerIndex %d outside [0, %d]", R, l.writer);
    int32_t move = 0;
    if (R != 0) {
      size_t drop;
      if (R == l.writer && l.writer == capacity(l)) {  // discard-all case
        drop = l.segs.size();
        move = R;
      } else {
        drop = size_t(R) / C();
        move = int32_t(drop * C());
      }
      for (size_t i = 0; i < drop; ++i) freed.push_back(l.segs[i]);
      l.segs.erase_front(drop);
    }
    l.epochs.rebase(move);
    l.writer -= move;
    l.flushed -= move;
    l.tail_start -= move;
    if (l.tail_start < 0) {  // bytes of dropped components
      l.tail.erase(l.tail.begin(), l.tail.begin() + std::min<long>(long(l.tail.size()), long(-l.tail_start)));
      l.tail_start = 0;
      if (l.tail_start + int32_t(l.tail.size()) != l.writer) reset_tail(l);
    }
    return CLG_OK;
  }

  // ---------------------------------------------------------------- decode
  struct DecodePlan {
    std::vector<clg::TileDesc> tiles;   // host-built tiles (staged host input)
    std::vector<clg::SpanDesc> spans;
    std::vector<clg::SegSpan> runs;     // log spans: tiles generated on the device
    std::vector<uint32_t> segtab;       // concatenated segment indices of the runs' logs
    uint32_t n_tiles = 0;
    uint32_t n_tiny = 0;                // whole spans of one tile and at most kZTinySpan bytes
    uint32_t unit = 0;                  // device-planning tile window
    const std::vector<uint32_t>* only = nullptr;  // plan only these spans (ascending), as spans 0, 1, ...
    // a builder that could not plan a log (a queued decode's re-plan after a rebase found its
    // range gone): the decode fails with this status instead of decoding an empty span
    int status = CLG_OK;
    // plan_parallel wrote the runs, segment table and spans straight into the pinned plan
    // buffer of decode slot stage_slot (stage_plan then adds only the chunk table); runs and
    // segtab stay empty, their sizes are n_runs / n_segs.  A re-launch of the plan (an abort's
    // fallbacks) re-plans it from its builder first (unstage).
    bool staged = false;
    uint32_t stage_slot = 0;
    size_t n_runs = 0, n_segs = 0;
    size_t run_count() const { return staged ? n_runs : runs.size(); }
    size_t seg_count() const { return staged ? n_segs : segtab.size(); }
    void reset() {  // empty, capacity kept (a config-4 plan is ~4 MB: fresh pages cost page faults)
      status = CLG_OK;
      staged = false;
      stage_slot = 0;
      n_runs = n_segs = 0;
      tiles.clear();
      spans.clear();
      runs.clear();
      segtab.clear();
      n_tiles = n_tiny = unit = 0;
      only = nullptr;
    }
  };
  // clg_decode_logs' plan and log ranges, kept between calls for their capacity
  DecodePlan zplan;
  // host threads for batches of very many logs (CLONOS_HOST_THREADS, default 8; 1: none)
  std::unique_ptr<WorkPool> host_pool;
  // The CPUs this process may use: its affinity mask, capped by a cgroup CPU quota (a GPU box
  // shares its host between GPUs: 16 CPUs per GPU on the MI355X pool).
  static int usable_cpus() {
    int n = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) n = int(std::thread::hardware_concurrency());
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long long period = 0;
      if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0)
        n = std::min<long long>(n, std::max<long long>(1, atoll(q) / period));
      fclose(f);
    }
    return std::max(1, n);
  }
  // Host threads for the per-log loops: CLONOS_HOST_THREADS, else up to 16 of the usable CPUs.
  // Config 4's step on one box (round 5): 2.49 ms with 16 against 3.1-3.4 ms with 8; round 6,
  // median of four each: 2.09 / 2.20 / 2.40 ms with 16 / 14 / 12.
  WorkPool* workers() {
    if (!host_pool) {
      const char* v = getenv("CLONOS_HOST_THREADS");
      const int n = std::max(1, std::min(v ? atoi(v) : 16, usable_cpus()));
      host_pool = std::make_unique<WorkPool>(unsigned(n));
    }
    return host_pool.get();
  }
  static constexpr uint32_t kParallelLogs = 8192;  // logs per batch from which the loops split
  std::vector<int32_t> zst, znb;
  // Span filter of a plan (the per-span fallback re-decodes single spans): false = skip.
  static bool plan_keep(const DecodePlan& p, uint32_t* s) {
    if (!p.only) return true;
    const auto it = std::lower_bound(p.only->begin(), p.only->end(), *s);
    if (it == p.only->end() || *it != *s) return false;
    *s = uint32_t(it - p.only->begin());
    return true;
  }

  // Tile window for device planning: min(segment, tile) when one divides the other.
  uint32_t tile_unit(uint32_t k) const {
    const uint32_t c = C();
    if (c <= k) return (k % c == 0) ? c : 0;
    return (c % k == 0) ? k : 0;
  }

  void plan_host_span(DecodePlan& p, const uint8_t* dbase, uint64_t len, uint32_t s, uint32_t T) {
    if (!plan_keep(p, &s)) return;
    clg::SpanDesc sd{uint32_t(p.tiles.size()), 0, len};
    uint64_t o = 0;
    while (o < len) {
      const uintptr_t addr = uintptr_t(dbase + o);
      const uint32_t delta = uint32_t(addr & 15);
      const uint32_t take = uint32_t(std::min<uint64_t>(len - o, uint64_t(T - delta)));
      p.tiles.push_back(clg::TileDesc{reinterpret_cast<const uint8_t*>(addr & ~uintptr_t(15)), delta, take, s, 0, o});
      o += take;
      sd.n_tiles++;
    }
    p.n_tiny += (sd.n_tiles == 1 && len <= clg::kZTinySpan) ? 1u : 0u;
    p.spans.push_back(sd);
    p.n_tiles = uint32_t(p.tiles.size());
  }

  void plan_log_span(DecodePlan& p, const Log& l, int32_t start, int32_t len, uint32_t s, uint32_t T) {
    if (!plan_keep(p, &s)) return;
    p.unit = tile_unit(T);
    if (const uint32_t U = p.unit) {  // device planning
      const uint32_t cnt = len > 0 ? (uint32_t(start + len - 1) / U - uint32_t(start) / U + 1) : 0;
      p.spans.push_back(clg::SpanDesc{p.n_tiles, cnt, uint64_t(len)});
      p.n_tiny += (cnt == 1 && uint32_t(len) <= clg::kZTinySpan) ? 1u : 0u;
      if (cnt) {  // only the segments the span covers go into the table (phys rebased on them)
        const uint32_t s0 = uint32_t(start) / C(), s1 = uint32_t(start + len - 1) / C() + 1;
        p.runs.push_back(clg::SegSpan{p.segtab.size(), uint32_t(start) - s0 * C(), uint32_t(len), s, p.n_tiles, 0});
        p.segtab.insert(p.segtab.end(), l.segs.begin() + s0, l.segs.begin() + s1);
      }
      p.n_tiles += cnt;
      return;
    }
    clg::SpanDesc sd{uint32_t(p.tiles.size()), 0, uint64_t(len)};
    int32_t ph = start;
    const int32_t end = start + len;
    while (ph < end) {
      const uint32_t si = uint32_t(ph) / C(), so = uint32_t(ph) % C();
      const uint32_t take = std::min<uint32_t>(uint32_t(end - ph), C() - so);
      // tiles never exceed kTile aligned bytes: split large segments
      uint32_t done = 0;
      while (done < take) {
        const uint32_t o = so + done;
        const uint32_t delta = o & 15;
        const uint32_t t = std::min<uint32_t>(take - done, T - delta);
        p.tiles.push_back(clg::TileDesc{seg_addr(l.segs[si]) + (o & ~15u), delta, t, s, 0, uint64_t(ph - start + int32_t(done))});
        done += t;
        sd.n_tiles++;
      }
      ph += int32_t(take);
    }
    p.n_tiny += (sd.n_tiles == 1 && uint32_t(len) <= clg::kZTinySpan) ? 1u : 0u;
    p.spans.push_back(sd);
    p.n_tiles = uint32_t(p.tiles.size());
  }

  // clg_decode_logs' ranges and device-planned fast plan (plan_log_span's spans, runs and
  // segment table, in the same order) on the host threads: per part of the logs their ranges
  // and sizes, then the parts' offsets, then each part writes its entries in place.  false:
  // not applicable (no device planning) or a log failed -- the caller runs the serial loop,
  // which reports the error.
  // stage >= 0: the runs, segment table and spans go straight into that decode slot's pinned
  // plan buffer (DecodePlan::staged; the spans into p.spans too, which the host reads), so the
  // launch copies nothing on the host but the chunk table.
  bool plan_parallel(DecodePlan& p, const uint32_t* log, const int64_t* start_epoch, uint32_t n, uint64_t* total,
                     int stage = -1) {
    const uint32_t U = tile_unit(clg::kZTile), Cb = C();
    if (!U) return false;
    WorkPool* wp = workers();
    const unsigned P = wp->size();
    struct Part {
      uint64_t bytes = 0, tiles = 0, runs = 0, segs = 0, tiny = 0;
      bool bad = false;
    };
    std::vector<Part> part(P);
    std::optional<HostTimer> hsub(std::in_place, this, "host_plan_pass1");
    std::vector<int32_t>& st = zst;
    std::vector<int32_t>& nb = znb;
    const uint32_t per = (n + P - 1) / P;
    auto cnt_of = [&](int32_t start, int32_t len) -> uint32_t {
      return len > 0 ? uint32_t(start + len - 1) / U - uint32_t(start) / U + 1 : 0u;
    };
    wp->run([&](unsigned k, unsigned) {
      Part& q = part[k];
      for (uint32_t i = k * per; i < std::min(n, (k + 1) * per); ++i) {
        Log* l;
        if (get_log(log[i], &l) != CLG_OK ||
            (l->depth != 0 && determinants_range(*l, start_epoch[i], &st[i], &nb[i]) != CLG_OK)) {
          q.bad = true;
          return;
        }
        const uint32_t c = cnt_of(st[i], nb[i]);
        q.bytes += uint64_t(nb[i]);
        q.tiles += c;
        q.tiny += (c == 1 && uint32_t(nb[i]) <= clg::kZTinySpan) ? 1u : 0u;
        if (c) {
          ++q.runs;
          q.segs += uint32_t(st[i] + nb[i] - 1) / Cb - uint32_t(st[i]) / Cb + 1;
        }
      }
    });
    std::vector<Part> at(P + 1);
    for (unsigned k = 0; k < P; ++k) {
      if (part[k].bad) return false;
      at[k + 1].bytes = at[k].bytes + part[k].bytes;
      at[k + 1].tiles = at[k].tiles + part[k].tiles;
      at[k + 1].runs = at[k].runs + part[k].runs;
      at[k + 1].segs = at[k].segs + part[k].segs;
      at[k + 1].tiny = at[k].tiny + part[k].tiny;
    }
    if (at[P].tiles >= (1ull << 32)) return false;
    hsub.emplace(this, "host_plan_pass2");
    p.reset();
    p.unit = U;
    p.spans.resize(n);
    p.n_tiles = uint32_t(at[P].tiles);
    p.n_tiny = uint32_t(at[P].tiny);
    clg::SegSpan* runs_out;
    uint32_t* seg_out;
    clg::SpanDesc* spans_copy = nullptr;
    if (stage >= 0) {  // the layout stage_plan computes, room for the count pass's chunk table after it
      PlanLayout L;
      plan_layout(0, at[P].runs * sizeof(clg::SegSpan), at[P].segs * sizeof(uint32_t), size_t(n) * sizeof(clg::SpanDesc),
                  (size_t(p.n_tiles) + 2) * sizeof(uint32_t), &L);
      PinBuf& h = h_plan_s[stage];
      if (h.ensure(L.hb + 64) != CLG_OK) return false;
      uint8_t* hd = h.as<uint8_t>();
      runs_out = reinterpret_cast<clg::SegSpan*>(hd + L.o_runs);
      seg_out = reinterpret_cast<uint32_t*>(hd + L.o_seg);
      spans_copy = reinterpret_cast<clg::SpanDesc*>(hd + L.o_spans);
      p.staged = true;
      p.stage_slot = uint32_t(stage);
      p.n_runs = at[P].runs;
      p.n_segs = at[P].segs;
    } else {
      p.runs.resize(at[P].runs);
      p.segtab.resize(at[P].segs);
      runs_out = p.runs.data();
      seg_out = p.segtab.data();
    }
    wp->run([&](unsigned k, unsigned) {
      uint64_t tile = at[k].tiles, run = at[k].runs, seg = at[k].segs;
      for (uint32_t i = k * per; i < std::min(n, (k + 1) * per); ++i) {
        const Log& l = logs[log[i]];
        const int32_t start = st[i], len = nb[i];
        const uint32_t c = cnt_of(start, len);
        p.spans[i] = clg::SpanDesc{uint32_t(tile), c, uint64_t(len)};
        if (spans_copy) spans_copy[i] = p.spans[i];
        if (c) {  // plan_log_span's device-planning entries
          const uint32_t s0 = uint32_t(start) / Cb, s1 = uint32_t(start + len - 1) / Cb + 1;
          runs_out[run++] = clg::SegSpan{seg, uint32_t(start) - s0 * Cb, uint32_t(len), i, uint32_t(tile), 0};
          std::copy(l.segs.begin() + s0, l.segs.begin() + s1, seg_out + seg);
          seg += s1 - s0;
        }
        tile += c;
      }
    });
    *total = at[P].bytes;
    return true;
  }

  static void reset_result(clg_decoded* out) {
    out->n_rec = out->n_wide = 0;
    out->err_status = CLG_OK;
    out->err_span = 0;
    out->err_off = -1;
    out->err_tag = 0;
  }

  // Uploads the plan's descriptors (spans into d_spans) and materialises its tiles in
  // `dtiles` (device planning from the segment table, or the host-built list).
  int upload_plan(DecodePlan& p, DevBuf& dtiles) {
    PlanLayout L;
    CHK(stage_plan(p, dtiles, &L));
    return enqueue_plan(p, L, dtiles);
  }
  // Where a staged plan lies in h_plan / d_plan (byte offsets).
  struct PlanLayout {
    size_t tb = 0, sb = 0, o_runs = 0, o_seg = 0, o_spans = 0, o_chunk = 0, hb = 0;
  };
  // Host half: the plan's descriptors (and the count pass's chunk table, if any) into the
  // pinned plan buffer (its own: an asynchronous decode may still be uploading it while later
  // calls -- flush, slices -- stage theirs).
  static void plan_layout(size_t tb, size_t rb, size_t gb, size_t sb, size_t cb, PlanLayout* L) {
    L->tb = tb;
    L->sb = sb;
    L->o_runs = (tb + 15) & ~size_t(15);
    L->o_seg = (L->o_runs + rb + 15) & ~size_t(15);
    L->o_spans = (L->o_seg + gb + 15) & ~size_t(15);
    L->o_chunk = (L->o_spans + sb + 15) & ~size_t(15);
    L->hb = L->o_chunk + cb;
  }
  int stage_plan(const DecodePlan& p, DevBuf& dtiles, PlanLayout* L, const std::vector<uint32_t>* chunk = nullptr) {
    const uint32_t nt = p.n_tiles, ns = uint32_t(p.spans.size());
    CHK(dtiles.ensure(std::max<size_t>(1, nt) * sizeof(clg::TileDesc)));
    CHK(d_spans.ensure(ns * sizeof(clg::SpanDesc)));
    const size_t cb = chunk ? chunk->size() * sizeof(uint32_t) : 0;
    plan_layout(p.tiles.size() * sizeof(clg::TileDesc), p.run_count() * sizeof(clg::SegSpan),
                p.seg_count() * sizeof(uint32_t), ns * sizeof(clg::SpanDesc), cb, L);
    PinBuf& h_plan = h_plan_s[plan_slot];
    if (p.staged) {  // runs, segment table and spans are in place (plan_parallel): the chunk table
      if (p.stage_slot != plan_slot || h_plan.cap < L->hb + 64)
        return fail(CLG_E_STATE, "staged decode plan in slot %u, launched in slot %u", p.stage_slot, plan_slot);
      CHK(d_plan.ensure(L->hb));
      if (cb) memcpy(h_plan.as<uint8_t>() + L->o_chunk, chunk->data(), cb);
      return CLG_OK;
    }
    const size_t tb = L->tb, rb = p.runs.size() * sizeof(clg::SegSpan), gb = p.segtab.size() * sizeof(uint32_t),
                 sb = L->sb;
    CHK(h_plan.ensure(L->hb + 64));
    CHK(d_plan.ensure(L->hb));
    uint8_t* hd = h_plan.as<uint8_t>();
    if (L->hb >= kParallelCopy) {  // a config-4 plan is ~3 MB: the host threads copy it
      const std::pair<const void*, size_t> part[5] = {
          {p.tiles.data(), tb}, {p.runs.data(), rb}, {p.segtab.data(), gb}, {p.spans.data(), sb},
          {cb ? chunk->data() : nullptr, cb}};
      const size_t dst[5] = {0, L->o_runs, L->o_seg, L->o_spans, L->o_chunk};
      workers()->run([&](unsigned k, unsigned P) {
        for (int j = 0; j < 5; ++j) {
          const size_t n = part[j].second, a = n * k / P, b = n * (k + 1) / P;
          if (b > a) memcpy(hd + dst[j] + a, static_cast<const uint8_t*>(part[j].first) + a, b - a);
        }
      });
      return CLG_OK;
    }
    memcpy(hd, p.tiles.data(), tb);
    memcpy(hd + L->o_runs, p.runs.data(), rb);
    memcpy(hd + L->o_seg, p.segtab.data(), gb);
    memcpy(hd + L->o_spans, p.spans.data(), sb);
    if (cb) memcpy(hd + L->o_chunk, chunk->data(), cb);
    return CLG_OK;
  }
  static constexpr size_t kParallelCopy = 1u << 20;
  // The count pass's chunks of about equal cost: a tile costs its bytes plus a fixed 1 KiB
  // (tiles of one span are taken as equally long; a small whole span that pass 0 counted, a
  // skip), and block b takes the tiles whose cumulative cost passes b / G of the total.
  // ch[0 .. G]: boundaries, ch[G] = n_tiles.
  // Batches of many spans: the cost sums per part of the spans on the host threads, then
  // each part places the boundaries that fall in it (the same boundaries as one pass).
  void count_chunks(const DecodePlan& p, uint32_t G, bool tiny, std::vector<uint32_t>& ch) {
    ch.assign(size_t(G) + 1, p.n_tiles);
    ch[0] = 0;
    constexpr double kTileCost = 1024.0, kTinyCost = 64.0;  // (pass 0 counted the small whole spans)
    auto cost = [&](const clg::SpanDesc& s) {
      return tiny && s.n_tiles == 1 && s.len <= clg::kZTinySpan ? kTinyCost : double(s.len) / s.n_tiles + kTileCost;
    };
    const size_t ns = p.spans.size();
    const unsigned P = ns >= kParallelLogs ? workers()->size() : 1u;
    std::vector<double> part(P + 1, 0.0);
    auto range = [&](unsigned k, size_t* a, size_t* b) {
      *a = ns * k / P;
      *b = ns * (k + 1) / P;
    };
    auto sums = [&](unsigned k, unsigned) {
      size_t a, b;
      range(k, &a, &b);
      double t = 0;
      for (size_t i = a; i < b; ++i)
        if (p.spans[i].n_tiles) t += cost(p.spans[i]) * p.spans[i].n_tiles;
      part[k + 1] = t;
    };
    if (P > 1) workers()->run(sums); else sums(0, 1);
    for (unsigned k = 0; k < P; ++k) part[k + 1] += part[k];
    if (!(part[P] > 0)) return;  // (no tiles)
    const double target = part[P] / G;
    // part k places boundaries [bstart(k), bstart(k + 1)): those past the cost before it
    auto bstart = [&](unsigned k) -> uint32_t {
      if (k == 0) return 1u;
      if (k >= P) return G;
      uint32_t b = uint32_t(std::min<double>(double(G), std::max(1.0, std::floor(part[k] / target))));
      while (b > 1 && target * (b - 1) > part[k]) --b;
      while (b < G && target * b <= part[k]) ++b;
      return b;
    };
    auto place = [&](unsigned k, unsigned) {
      size_t a, e;
      range(k, &a, &e);
      double acc = part[k];
      uint32_t b = bstart(k);
      const uint32_t bend = bstart(k + 1);
      double next = target * b;
      for (size_t i = a; i < e && b < bend; ++i) {
        const auto& s = p.spans[i];
        if (!s.n_tiles) continue;
        const double c = cost(s), end = acc + c * s.n_tiles;
        while (b < bend && next <= end) {  // boundary inside this span: the first tile past it
          const double kk = (next - acc) / c;
          ch[b++] = s.first_tile + std::min<uint32_t>(s.n_tiles, uint32_t(kk) + (kk > double(uint32_t(kk)) ? 1u : 0u));
          next = target * b;
        }
        acc = end;
      }
      const uint32_t past = e < ns ? p.spans[e].first_tile : p.n_tiles;  // (rounding: the part's end)
      while (b < bend) ch[b++] = past;
    };
    if (P > 1) workers()->run(place); else place(0, 1);
  }
  std::vector<uint32_t> chunk_buf;
  // Device half: upload, span table, tiles (expanded on the device from the runs).
  int enqueue_plan(const DecodePlan& p, const PlanLayout& L, DevBuf& dtiles) {
    HIPCHK(hipMemcpyAsync(d_plan.p, h_plan_s[plan_slot].p, L.hb, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(d_spans.p, d_plan.as<uint8_t>() + L.o_spans, L.sb, hipMemcpyDeviceToDevice, stream));
    if (!p.runs.empty()) {
      CHK(clg::launch_expand_tiles(reinterpret_cast<const clg::SegSpan*>(d_plan.as<uint8_t>() + L.o_runs),
                                   uint32_t(p.runs.size()), p.n_tiles,
                                   reinterpret_cast<const uint32_t*>(d_plan.as<uint8_t>() + L.o_seg), pool, C(),
                                   p.unit, dtiles.as<clg::TileDesc>(), stream));
    } else if (L.tb) {
      HIPCHK(hipMemcpyAsync(dtiles.p, d_plan.p, L.tb, hipMemcpyDeviceToDevice, stream));
    }
    return CLG_OK;
  }

  // Output arrays the kernels write: the caller's device arrays, or engine scratch that
  // finish_out copies to the caller's host arrays.
  // Registered host outputs (CLG_MEM_MAPPED) of at most kMappedDirect bytes: the kernels write
  // them through their device addresses, so no read-back copy and no host memcpy follow (for
  // config 5's replay-prep decode, 1.7 MB of rows: 0.12 ms of finish_out).
  static constexpr uint64_t kMappedDirect = 8ull << 20;
  static bool mapped_direct(const clg_decoded& out) {
    return out.out_kind == CLG_MEM_MAPPED && out.cap * 13 + out.wcap * 25 <= kMappedDirect &&
           mapped_outputs(out, nullptr);
  }
  int prep_out(clg_decoded* out, clg::DecodeOut* o) {
    const bool dev = out->out_kind == CLG_MEM_DEVICE;
    if (mapped_direct(*out)) {
      mapped_outputs(*out, o);
      return CLG_OK;
    }
    if (dev) {
      *o = clg::DecodeOut{out->off, out->tag, out->v0, out->w_idx, out->w_rc, out->w_v1, out->w_var_off,
                         out->w_var_len, out->w_sub, out->cap, out->wcap};
    } else {
      const size_t cap = std::max<uint64_t>(1, out->cap), wcap = std::max<uint64_t>(1, out->wcap);
      CHK(d_o_off.ensure(cap * 4));
      CHK(d_o_tag.ensure(cap));
      CHK(d_o_v0.ensure(cap * 8));
      CHK(d_o_widx.ensure(wcap * 4));
      CHK(d_o_wrc.ensure(wcap * 4));
      CHK(d_o_wv1.ensure(wcap * 8));
      CHK(d_o_wvo.ensure(wcap * 4));
      CHK(d_o_wvl.ensure(wcap * 4));
      CHK(d_o_wsub.ensure(wcap));
      *o = clg::DecodeOut{d_o_off.as<uint32_t>(), d_o_tag.as<uint8_t>(), d_o_v0.as<int64_t>(), d_o_widx.as<uint32_t>(),
                         d_o_wrc.as<int32_t>(), d_o_wv1.as<int64_t>(), d_o_wvo.as<uint32_t>(), d_o_wvl.as<uint32_t>(),
                         d_o_wsub.as<uint8_t>(), out->cap, out->wcap};
    }
    return CLG_OK;
  }

  // An asynchronous decode into device memory completes on its own stream only: slices still
  // running on gstream only read log segments, and every call that writes segments waits for
  // gstream first (flush, upstream deltas, the in-flight pool).  Measured on MI355X (config-2
  // step, 3 runs each, tools/ab_env.sh): 0.79 ms against 0.83 ms when the completion also
  // drained gstream.
  bool settling = false;  // settle() is completing an asynchronous decode
  int finish_out(clg_decoded* out, uint64_t nrec, uint64_t nwide) {
    out->n_rec = nrec;
    out->n_wide = nwide;
    if (out->out_kind != CLG_MEM_DEVICE && !mapped_direct(*out)) {
      // the used part of each array into one pinned staging buffer (asynchronous copies; into
      // the caller's pageable arrays each copy was a synchronous staged transfer: 0.17 ms for
      // config 1's 44-log decode), then into the caller's arrays
      const uint64_t r = std::min(nrec, out->cap), w = std::min(nwide, out->wcap);
      struct Part {
        void* dst;
        const void* src;
        uint64_t n;
      } parts[9] = {{out->off, d_o_off.p, r * 4},          {out->tag, d_o_tag.p, r},
                    {out->v0, d_o_v0.p, r * 8},            {out->w_idx, d_o_widx.p, w * 4},
                    {out->w_rc, d_o_wrc.p, w * 4},         {out->w_v1, d_o_wv1.p, w * 8},
                    {out->w_var_off, d_o_wvo.p, w * 4},    {out->w_var_len, d_o_wvl.p, w * 4},
                    {out->w_sub, d_o_wsub.p, w}};
      uint64_t at[10] = {0};
      for (int i = 0; i < 9; ++i) at[i + 1] = (at[i] + parts[i].n + 15) & ~uint64_t(15);
      if (at[9] <= (uint64_t(64) << 20)) {
        CHK(h_outs.ensure(at[9] + 16));
        uint8_t* hb = h_outs.as<uint8_t>();
        for (int i = 0; i < 9; ++i)
          if (parts[i].n) HIPCHK(hipMemcpyAsync(hb + at[i], parts[i].src, parts[i].n, hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        for (int i = 0; i < 9; ++i)
          if (parts[i].n) memcpy(parts[i].dst, hb + at[i], parts[i].n);
      } else {  // large outputs: straight into the caller's arrays (no 64 MB+ pinned buffer)
        for (int i = 0; i < 9; ++i)
          if (parts[i].n) HIPCHK(hipMemcpyAsync(parts[i].dst, parts[i].src, parts[i].n, hipMemcpyDeviceToHost, stream));
      }
    }
    if (settling && out->out_kind == CLG_MEM_DEVICE) {
      collect_timings(true);  // (finish_fused waited for the run's read-back, which follows emit)
    } else {
      CHK(sync());
    }
    if (nrec > out->cap || nwide > out->wcap)
      return fail(CLG_E_CAPACITY, "decode produced %llu records / %llu wide rows, capacity %llu / %llu",
                  (unsigned long long)nrec, (unsigned long long)nwide, (unsigned long long)out->cap,
                  (unsigned long long)out->wcap);
    return CLG_OK;
  }

  // Speculative warm-up bytes before each lane's region (CLONOS_WARM overrides; tuning aid).
  // Measured on MI355X (tools/r3_warm.sh): 96 B is best for short fixed-length records
  // (config 2: count 0.176 ms at 96 B, 0.194 at 64, 0.182 at 128; round 6, with the lean walk
  // and the staggered starts, 64-128 B within 2 %: pipeline 0.430-0.437 ms).  With Serializable
  // tables the count pass walks the step-code map, whose steps no longer diverge on wide
  // records, and 48-128 B are best too (config-3 subset: 0.43-0.44 ms, 0.451 at 16 B).
  static uint32_t spec_warm(bool /*jser*/) {
    static const int w = [] {
      const char* v = getenv("CLONOS_WARM");
      return v ? atoi(v) : -1;
    }();
    return w >= 0 ? uint32_t(w) : 96u;
  }

  // Fast three-pass decode (decode_fused.hip).  *aborted = true when the kernels met
  // anything outside its fast path; the caller then runs the robust pipeline.
  // jser: build the Serializable tables first (phase 3).  *need_jser: the batch aborted
  // only because it met Serializable records without tables.
  int run_fused(DecodePlan& p, uint64_t log_bytes, clg_decoded* out, uint64_t* span_rec_base, bool* aborted,
                bool jser, bool* need_jser) {
    *aborted = false;
    *need_jser = false;
    reset_result(out);
    if (p.spans.empty()) return CLG_OK;
    if (!fused_fits(p)) {
      *aborted = true;
      return CLG_OK;
    }
    FusedRun r;
    CHK(launch_fused(p, log_bytes, out, jser, &r));
    return finish_fused(p, r, out, span_rec_base, aborted, need_jser);
  }
  // Records and wide rows per span from the read-back span_hi words (hz[ns + s], packed
  // wide << 31 | records): spans hold consecutive record ranges in span order, so a span's
  // range starts where the previous span with tiles ended.  span_rec_base[0 .. ns].
  static void span_totals(const DecodePlan& p, const uint64_t* hz, uint64_t* span_rec_base, uint64_t* nrec,
                          uint64_t* nwide) {
    constexpr uint64_t kRecMask = (1ull << 31) - 1;
    const uint32_t ns = uint32_t(p.spans.size());
    uint64_t prev = 0;
    for (uint32_t s = 0; s < ns; ++s) {
      if (span_rec_base) span_rec_base[s] = prev & kRecMask;
      if (p.spans[s].n_tiles) prev = hz[ns + s];
    }
    if (span_rec_base) span_rec_base[ns] = prev & kRecMask;
    *nrec = prev & kRecMask;
    *nwide = prev >> 31;
  }
  static constexpr uint32_t kHostResSpans = 1024;  // spans up to which the scan writes the host read-back
  // more than 8 GiB in one batch: the offsets pass covers 2^20 tiles
  static bool fused_fits(const DecodePlan& p) { return p.n_tiles <= (1u << 20); }

  // One queued three-pass decode: launch_fused queues everything up to the read-back of the
  // span ranges and abort words; finish_fused waits for it and turns it into the result.
  struct FusedRun {
    uint64_t log_bytes = 0;
    bool jser = false;
    hipEvent_t ea = nullptr, eb = nullptr;  // emit's timing events
    hipEvent_t pa = nullptr, pb = nullptr;  // the whole pipeline's (count start .. emit end)
    // for the per-span fallback: the run's control words and outputs, and whether only
    // span-local reasons aborted it (chains that went wrong, not a timeout / table overflow)
    clg::FusedCtl ctl{};
    clg::DecodeOut o{};
    bool span_local = false;
    bool lookback_bad = false;  // emit found a scan offset other than its predecessor's prefix
    bool one = false;           // the one-pass decode (k_decode_one) ran, not the three passes
    // its decode slot (read-back buffer, staged plan, jser arena note), and for a queued
    // decode the event after its read-back, which its completion waits for (not the stream:
    // a later decode may be queued behind it)
    uint32_t slot = 0;
    hipEvent_t done = nullptr;
    int note() const { return slot ? int(1 + slot) : 0; }
  };
  FusedRun zlast;  // the last finished fast run
  // The one-pass decode (k_decode_one, decode_fused.hip): off by default, since on MI355X it is
  // slower than the three passes (config 2: 0.58 against 0.43 ms, DESIGN.md section 4, "One
  // pass").  CLONOS_ONE_PASS=1 uses it for batches of more than kZSmallTilesMax tiles without
  // tables or small whole spans; =2 for every batch the three passes would take (the tests).
  // An abort goes to the three passes (after_abort), and so does a run with allow_one cleared.
  const int one_pass = [] {
    const char* v = getenv("CLONOS_ONE_PASS");
    return v ? atoi(v) : 0;
  }();
  bool allow_one = true;
  int launch_fused(DecodePlan& p, uint64_t log_bytes, clg_decoded* out, bool jser, FusedRun* r) {
    HostTimer ht(this, "host_decode_launch");
    const uint32_t nt = p.n_tiles, ns = uint32_t(p.spans.size());
    r->log_bytes = log_bytes;
    r->jser = jser;
    // chunks of equal cost when blocks take several tiles of spans of different sizes
    const bool zdbg = getenv("CLONOS_FUSED_DEBUG") != nullptr;
    const char* prof_path = getenv("CLONOS_SCAN_PHASES");  // developer diagnostics: phase stamps
    // pass 0 (small whole spans, a lane each) for batches without Serializable tables
    const bool tiny = p.n_tiny && !jser && !prof_path;
    // (default: logs in segments of at least two tiles, or host input -- tiles of a few hundred
    // bytes give canonical exits from too few bytes, which often miss, and the batch goes again)
    const bool one = one_pass && allow_one && !jser && !p.n_tiny && !zdbg &&
                     ((nt > clg::kZSmallTilesMax && (!p.run_count() || C() >= 2 * clg::kZTile)) || one_pass == 2);
    r->one = one;
    const uint32_t G = clg::decode_count_grid(jser, nt);
    const bool chunked = G && nt > G && ns > 1 && !one;
    std::optional<HostTimer> hsub(std::in_place, this, "host_launch_chunks");  // (CLONOS_HOST_PROF sub-stages)
    if (chunked) count_chunks(p, G, tiny, chunk_buf);
    PlanLayout L;
    hsub.emplace(this, "host_launch_stage");
    struct SlotScope {  // stage_plan / enqueue_plan use this run's slot
      uint32_t& s;
      SlotScope(uint32_t& s_, uint32_t v) : s(s_) { s = v; }
      ~SlotScope() { s = 0; }
    } slot_scope(plan_slot, r->slot);
    CHK(stage_plan(p, d_ztiles, &L, chunked ? &chunk_buf : nullptr));
    hsub.emplace(this, "host_launch_enqueue");
    clg::DecodeOut o{};
    CHK(prep_out(out, &o));
    hsub->lap("host_enq_out");
    // words: st_x[nt] ex[nt] rep_flag[nt] (u8) cnt[nt] base[nt] boff[nb] | span_lo[ns] span_hi[ns] |
    // abort[8] rep[4] (u32) | lb: ticket, look-back[nb] | ent[G]; bits apart.  st_x, ex,
    // rep_flag, the abort and repair words, lb and ent are zeroed per batch.
    const size_t nbk = (size_t(nt) + 1023) / 1024, fw = (size_t(nt) + 7) / 8;
    const size_t o_cnt = 2 * size_t(nt) + fw, n_ab = clg::kZAbortWords / 2;
    const size_t o_span = o_cnt + 2 * size_t(nt) + nbk, o_ab = o_span + 2 * size_t(ns), o_lb = o_ab + n_ab;
    // (ent: G words for the count pass's chunks, or the one-pass decode's 65 counters, 128 B apart)
    const size_t n_ent = std::max<size_t>(one ? 65 * 16 : 1, G);
    const size_t o_ent = o_lb + 1 + nbk, words = o_ent + n_ent;
    CHK(d_zctl.ensure(words * 8));
    CHK(d_zbits.ensure(std::max<size_t>(1, nt) * 64 * 16));
    CHK(d_zbad.ensure(std::max<size_t>(1, ns) * 4));
    CHK(d_zerr.ensure(std::max<size_t>(1, ns) * 8));
    PinBuf& h_zres = h_zres_s[r->slot];
    CHK(h_zres.ensure((2 * size_t(ns) + n_ab + 1) * 8));  // (+ the table work counters)
    hsub->lap("host_enq_bufs");
    uint64_t* w = d_zctl.as<uint64_t>();
    uint32_t* ab = reinterpret_cast<uint32_t*>(w + o_ab);
    if (zdbg) CHK(d_dbg.ensure(clg::kZDbgTiles * 4 + size_t(nt) * 16));
    if (prof_path) CHK(d_prof.ensure(size_t(nt) * (one ? 128 : 64)));  // (one pass: its phase stamps too)
    const uint32_t jwork_cap = std::max<uint32_t>(uint32_t(nt) * 16 + 1024, zjwork_min);
    if (jser) {
      CHK(d_zjpos.ensure((size_t(nt) * clg::kZJCap + zjovf_cap) * 4));
      CHK(d_zjlen.ensure((size_t(nt) * clg::kZJCap + zjovf_cap) * 4));
      CHK(d_zjn.ensure(size_t(nt) * 8));  // jn, jbase
      CHK(d_zjwork.ensure((2 * size_t(jwork_cap) + 3 + size_t(nt)) * 4));  // (+ the sidecar's scan list)
    }
    clg::FusedCtl ctl{w, w + o_cnt, w + o_cnt + nt, w + o_cnt + 2 * size_t(nt), d_zbits.as<uint64_t>(), w + o_span,
                      w + o_span + ns, ab,
                      zdbg ? d_dbg.as<uint32_t>() : nullptr, prof_path ? d_prof.as<uint64_t>() : nullptr, nt,
                      jser ? d_zjpos.as<uint32_t>() : nullptr, jser ? d_zjlen.as<uint32_t>() : nullptr,
                      jser ? d_zjn.as<uint32_t>() : nullptr, jser ? 1u : 0u, jwork_cap,
                      jser ? d_zjwork.as<uint32_t>() : nullptr, spec_warm(jser), clg::JArena{}};
    if (jser) CHK(jarena_reset(&ctl.jar));
    ctl.jbase = jser ? d_zjn.as<uint32_t>() + nt : nullptr;
    ctl.jovf_cap = zjovf_cap;
    ctl.span_bad = d_zbad.as<uint32_t>();
    ctl.skip_bad = 0;
    ctl.span_err = keep_errors && !one ? d_zerr.as<uint64_t>() : nullptr;  // (one pass: errors abort it)
    ctl.chunk = chunked ? reinterpret_cast<const uint32_t*>(d_plan.as<uint8_t>() + L.o_chunk) : nullptr;
    ctl.tiny = tiny ? 1u : 0u;
    ctl.ex = w + nt;
    ctl.rep_flag = reinterpret_cast<uint8_t*>(w + 2 * size_t(nt));
    ctl.rep = ab + 8;
    ctl.ent = w + o_ent;
    ctl.perturb = fused_perturb;
    ctl.lb_check = 1;
    ctl.n_spans = ns;
    ctl.lb = w + o_lb;
    ctl.lean = !jser && (lean_env() >= 0 ? lean_env() != 0 : lean_hint) ? 1u : 0u;
    ctl.side = side;
    // the scan writes the result into the pinned read-back buffer itself (no copy queued after
    // emit) while the spans are few: each span_hi is its own write across the bus, and for
    // config 4's 66 k spans those took 2.5 ms -- there one copy after emit reads them back
    const bool host_res = ns <= kHostResSpans;
    ctl.h_res = host_res ? h_zres.as<uint64_t>() : nullptr;
    memset(h_zres.p, 0, (2 * size_t(ns) + n_ab + 1) * 8);  // (a batch without tiles runs no scan)
    hsub->lap("host_enq_memset");
    r->ctl = ctl;
    r->o = o;
    auto* zt = d_ztiles.as<clg::TileDesc>();
    auto* zs = d_spans.as<clg::SpanDesc>();
    const bool timing = (cfg.flags & CLG_F_TIMING) != 0;
    // The whole sequence, enqueued on `stream`; `ev` (timing) brackets jser, count, offsets
    // and emit, `evp` the whole pipeline.  (Captured as a hipGraph and replayed per batch
    // shape it was no faster: 197 us for a 16-log decode either way, and the bench step
    // unchanged.  Split into parts whose count ran beside the previous part's emit on a second
    // stream it was slower: config 2 0.44 -> 0.46 / 0.53 ms in 2 / 4 parts.)
    auto enqueue = [&](hipEvent_t* ev, hipEvent_t* evp) -> int {
      // the plan up in one copy, then one launch for the set-up: tiles from the runs, the span
      // table, and the zeroed control words (st_x, ex, rep_flag; abort words and repair
      // counters; bad-span flags; kept-error offsets ~0; the jser work counters)
      HIPCHK(hipMemcpyAsync(d_plan.p, h_plan_s[plan_slot].p, L.hb, hipMemcpyHostToDevice, stream));
      hsub->lap("host_enq_h2d");
      {
        clg::PrepArgs pa{};
        const bool runs = p.run_count() != 0;
        pa.runs = reinterpret_cast<const clg::SegSpan*>(d_plan.as<uint8_t>() + L.o_runs);
        pa.n_runs = uint32_t(p.run_count());
        pa.n_tiles = runs ? nt : 0;
        pa.segtab = reinterpret_cast<const uint32_t*>(d_plan.as<uint8_t>() + L.o_seg);
        pa.pool = pool;
        pa.C = C();
        pa.U = p.unit;
        pa.tiles = d_ztiles.as<clg::TileDesc>();
        const size_t nsw = std::max<size_t>(1, ns);
        pa.r[0] = clg::PrepRange{d_spans.as<uint32_t>(), reinterpret_cast<const uint32_t*>(d_plan.as<uint8_t>() + L.o_spans),
                                 L.sb / 4, 0, 0};
        pa.r[1] = clg::PrepRange{reinterpret_cast<uint32_t*>(w), nullptr, o_cnt * 2, 0, 0};
        pa.r[2] = clg::PrepRange{ab, nullptr, clg::kZAbortWords + 2 * (1 + nbk + n_ent), 0, 0};  // abort words, repair counters, look-back, entries
        pa.r[3] = clg::PrepRange{d_zbad.as<uint32_t>(), nullptr, nsw, 0, 0};
        pa.r[4] = clg::PrepRange{d_zerr.as<uint32_t>(), nullptr, keep_errors ? nsw * 2 : 0, 0xFFFFFFFFu, 0};
        pa.r[5] = clg::PrepRange{jser ? d_zjwork.as<uint32_t>() : nullptr, nullptr, jser ? 2u : 0u, 0, 0};
        pa.r[6] = clg::PrepRange{d_ztiles.as<uint32_t>(), reinterpret_cast<const uint32_t*>(d_plan.p), runs ? 0 : L.tb / 4, 0, 0};
        pa.r[7] = clg::PrepRange{jser ? d_zjwork.as<uint32_t>() + 2 + 2 * size_t(jwork_cap) : nullptr, nullptr,
                                 jser && side.hdr ? 1u : 0u, 0, 0};  // the sidecar's scan-list count
        CHK(clg::launch_decode_prep(pa, stream));
      }
      hsub->lap("host_enq_prep");
      if (zdbg) HIPCHK(hipMemsetAsync(d_dbg.p, 0, clg::kZDbgTiles * 4 + size_t(nt) * 16, stream));
      if (prof_path) HIPCHK(hipMemsetAsync(d_prof.p, 0, size_t(nt) * (one ? 128 : 64), stream));
      if (evp) HIPCHK(hipEventRecord(evp[0], stream));
      if (tiny) CHK(clg::launch_decode_fused(zt, nt, zs, ns, ctl, o, stream, 4));  // small whole spans
      if (one) {  // count, look-back and emit in one launch
        if (ev) HIPCHK(hipEventRecord(ev[2], stream));
        CHK(clg::launch_decode_fused(zt, nt, zs, ns, ctl, o, stream, 6));
        if (ev) HIPCHK(hipEventRecord(ev[3], stream));
      }
      for (int ph : {3, 0, 5, 2}) {  // jser tables, count, offsets (one launch), emit
        if (one) break;
        if (ph == 3 && !jser) continue;
        const int k = ph == 3 ? 0 : ph == 0 ? 1 : ph == 5 ? 2 : 3;
        if (ev) HIPCHK(hipEventRecord(ev[2 * k], stream));
        CHK(clg::launch_decode_fused(zt, nt, zs, ns, ctl, o, stream, uint32_t(ph)));
        if (ev) HIPCHK(hipEventRecord(ev[2 * k + 1], stream));
      }
      if (evp) HIPCHK(hipEventRecord(evp[1], stream));
      hsub->lap("host_enq_kernels");
      // the span ranges and abort words: in h_zres already (the scan wrote them) or read back
      // now (emit ran right behind the scan: it returns at once when the batch aborted, and its
      // stores are bounded by the output capacity)
      if (!host_res) {  // span_hi and the abort words (adjacent; the host derives the ranges from span_hi)
        HIPCHK(hipMemcpyAsync(h_zres.as<uint64_t>() + ns, ctl.span_hi, (size_t(ns) + n_ab) * 8, hipMemcpyDeviceToHost,
                              stream));
        if (jser)  // the table work counters beside them (the scan copies them when it writes h_res)
          HIPCHK(hipMemcpyAsync(h_zres.as<uint64_t>() + 2 * size_t(ns) + n_ab, ctl.jwork, 8, hipMemcpyDeviceToHost, stream));
      }
      hsub->lap("host_enq_d2h");
      if (jser) CHK(jarena_note(r->note()));
      if (r->slot) {
        if (!zdone[r->slot]) HIPCHK(hipEventCreateWithFlags(&zdone[r->slot], hipEventDisableTiming));
        HIPCHK(hipEventRecord(zdone[r->slot], stream));
        r->done = zdone[r->slot];
      }
      return CLG_OK;
    };
    hipEvent_t ev[8] = {}, evp[2] = {};
    if (timing) {
      for (auto& e : ev) e = get_event();
      for (auto& e : evp) e = get_event();
    }
    CHK(enqueue(timing ? ev : nullptr, timing ? evp : nullptr));
    if (timing && one) {  // the one kernel's duration: its bytes need the record count (finish_fused)
      ev_pool.insert(ev_pool.end(), {ev[0], ev[1], ev[4], ev[5], ev[6], ev[7]});
      r->ea = ev[2];
      r->eb = ev[3];
    } else if (timing) {  // per-kernel durations, read back by sync(); emit's bytes need the record count
      if (jser) timings.push_back(PendingTiming{"decode_jser", ev[0], ev[1], log_bytes});
      else ev_pool.insert(ev_pool.end(), {ev[0], ev[1]});
      timings.push_back(PendingTiming{"decode_count", ev[2], ev[3], log_bytes});
      timings.push_back(PendingTiming{"decode_offsets", ev[4], ev[5], 24 * uint64_t(nt)});
      r->ea = ev[6];
      r->eb = ev[7];
    }
    if (timing) {
      r->pa = evp[0];
      r->pb = evp[1];
    }
    return CLG_OK;
  }
  int finish_fused(const DecodePlan& p, FusedRun& r, clg_decoded* out, uint64_t* span_rec_base, bool* aborted,
                   bool* need_jser) {
    *aborted = false;
    *need_jser = false;
    const uint32_t nt = p.n_tiles, ns = uint32_t(p.spans.size());
    const bool jser = r.jser, zdbg = getenv("CLONOS_FUSED_DEBUG") != nullptr;
    const uint64_t log_bytes = r.log_bytes;
    hipEvent_t ea = r.ea, eb = r.eb;
    uint64_t* hz = h_zres_s[r.slot].as<uint64_t>();
    {
      HostTimer hw(this, "host_decode_wait");
      if (r.done) HIPCHK(hipEventSynchronize(r.done));  // (a later decode may be queued behind it)
      else HIPCHK(hipStreamSynchronize(stream));
    }
    HostTimer ht(this, "host_decode_finish");
    if (const char* prof_path = getenv("CLONOS_SCAN_PHASES")) {
      std::vector<uint64_t> hp(size_t(nt) * (r.one ? 16 : 8));
      hipMemcpy(hp.data(), d_prof.p, hp.size() * 8, hipMemcpyDeviceToHost);
      if (FILE* fp = fopen(prof_path, "wb")) {
        fwrite(hp.data(), 8, hp.size(), fp);
        fclose(fp);
      }
    }
    const uint32_t* hab = reinterpret_cast<const uint32_t*>(hz + 2 * size_t(ns));
    if (jser) jser_hint = hab[7] != 0;  // keep building tables while batches hold Serializable records
    if (hab[9]) stats["decode_chunk_repair"].launches += hab[9];  // repair requests the count pass served
    if (hab[8]) stats["decode_entry_repair"].launches += hab[8];  // chunks walked again for a wrong entry
    if (hab[11]) stats["decode_canon_before_end"].launches += hab[11];  // canonical exits inside their tile
    const bool spilled = jser && jarena_spilled(r.note());  // a stream walk found the spill arena full
    if (spilled) CHK(jarena_grow());
    // Serializable tables: the overflow arena or the walker's work list was full (reason 6)
    bool grown = false;
    if (jser && hab[6]) {
      // the work list's and the overflow arena's use, from this run's own read-back (a later
      // decode queued behind it may have zeroed the device words already)
      const uint32_t used[2] = {hab[clg::kZAbortWords], hab[clg::kZAbortWords + 1]};
      if (used[0] > r.ctl.jwork_cap) zjwork_min = std::max(zjwork_min, 2 * used[0]);
      if (used[1] > zjovf_cap) zjovf_cap = std::max<uint32_t>(2 * used[1], 2 * zjovf_cap);
      grown = used[0] > r.ctl.jwork_cap || used[1] > r.ctl.jovf_cap;
      stats["decode_jser_grow"].launches++;
    }
    if (zdbg) {  // count-pass chunk entries read as published but before their tile (not taken)
      uint32_t w8[8];
      hipMemcpy(w8, d_dbg.as<uint32_t>() + 16, sizeof(w8), hipMemcpyDeviceToHost);
      if (w8[0])
        fprintf(stderr, "[clonos] %u chunk-entry reads not taken; first: tile %u word %08x%08x tile span offset %u (poll %u)\n",
                w8[0], w8[1], w8[3], w8[2], w8[4], w8[5]);
    }
    if (hab[0] || spilled) {
      if (ea) {
        ev_pool.push_back(ea);
        ev_pool.push_back(eb);
      }
      if (r.pa) {
        ev_pool.push_back(r.pa);
        ev_pool.push_back(r.pb);
      }
      *aborted = true;
      static const char* kWhy[7] = {nullptr, "decode_abort_bad", "decode_abort_end", "decode_abort_exit",
                                    "decode_abort_timeout", "decode_abort_serializable", "decode_abort_overflow"};
      for (int k = 1; k <= 6; ++k)  // (which reasons: the bench line lists them beside the kernels)
        if (hab[k]) stats[kWhy[k]].launches++;
      // Serializable records were met without tables: other aborts may be consequences
      // (entries guessed across them), so the tables decide; a second abort goes robust
      // (a table arena that was full, now grown: the same, once)
      *need_jser = (!jser && hab[5] && !spilled) || (jser && (spilled || grown));
      r.span_local = !r.one && !*need_jser && !spilled && !hab[4] && !hab[6] && !hab[10];
      if (r.one) stats["decode_one_abort"].launches++;  // (the three passes decode it again)
      r.lookback_bad = hab[10] != 0;
      if (hab[10]) stats["decode_lookback_check"].launches++;  // a look-back read gave a wrong offset
      zlast = r;
      if (getenv("CLONOS_FUSED_DEBUG"))
        fprintf(stderr, "[clonos] fused decode aborted (%u tiles, jser %d): first tile per reason bad=%d end=%d exit=%d "
                "timeout=%d serializable=%d overflow=%d\n", nt, int(jser), int(~hab[1]), int(~hab[2]), int(~hab[3]),
                int(~hab[4]), int(~hab[5]), int(~hab[6]));
      if (zdbg) {
        std::vector<uint32_t> hd(clg::kZDbgTiles);
        hipMemcpy(hd.data(), d_dbg.p, hd.size() * 4, hipMemcpyDeviceToHost);
        fprintf(stderr, "[clonos] tile %u reason %u x_pub %u x_true %u e_true %u lo %u hi %u end_a %u\n", hd[1], hd[2],
                hd[3], hd[4], hd[5], hd[6], hd[7], hd[8]);
        if (hd[9] == 0xD15A) {
          fprintf(stderr, "[clonos] repair walk from tile %u gave up at tile %u (entry %u exit %u, span %u, %u disagreements)\n",
                  hd[10], hd[11], hd[12], hd[13], hd[14], hd[15]);
          {  // who wrote the exits before the walk (site 1 the count pass, 2 a repair walk)
            const uint32_t f = hd[10];
            std::vector<uint64_t> pp(size_t(p.n_tiles) * 2);
            hipMemcpy(pp.data(), d_dbg.as<uint8_t>() + clg::kZDbgTiles * 4, pp.size() * 8, hipMemcpyDeviceToHost);
            for (uint32_t t = f >= 10 ? f - 10 : 0; t <= std::min(hd[11] + 1, p.n_tiles - 1); ++t) {
              const uint64_t w = pp[size_t(t) * 2 + 1];
              uint64_t exv = 0, stx = 0;
              hipMemcpy(&exv, r.ctl.ex + t, 8, hipMemcpyDeviceToHost);
              hipMemcpy(&stx, r.ctl.st_x + t, 8, hipMemcpyDeviceToHost);
              fprintf(stderr, "[clonos]   tile %u: ex writer site %llu block %llu (chunk first / walk start %llu, why/old %llu) "
                      "entry %llu ex %llx st_x %llx\n",
                      t, (unsigned long long)(w >> 60), (unsigned long long)((w >> 32) & 0xFFFFFFF),
                      (unsigned long long)((w >> 4) & 0xFFFFFF), (unsigned long long)(w & 15),
                      (unsigned long long)pp[size_t(t) * 2], (unsigned long long)exv, (unsigned long long)stx);
            }
          }
        }
        for (int l = 0; l < 64; ++l) {
          const uint32_t* d = &hd[24 + 8 * l];
          fprintf(stderr, "  lane %2d rs %5u re %5u spec_exit %5u spec_bad %5u canon_exit %5u canon_bad %u entry %5u exit %5u bad %u\n",
                  l, d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7] & 0x7FFFFFFFu, d[7] >> 31);
        }
      }
      return CLG_OK;
    }
    uint64_t nrec = 0, nwide = 0;
    span_totals(p, hz, span_rec_base, &nrec, &nwide);
    if (!jser) lean_hint = nwide * 16 < nrec;
    if (ea) timings.push_back(PendingTiming{r.one ? "decode_one" : "decode_emit", ea, eb, log_bytes + 13 * nrec + 25 * nwide});
    // the pipeline's algorithmic bytes: log bytes read + the SoA rows
    if (r.pa) timings.push_back(PendingTiming{"decode_pipeline", r.pa, r.pb, log_bytes + 13 * nrec + 25 * nwide});
    return finish_out(out, nrec, nwide);
  }
  // ---------------------------------------------------------------- small batches
  // A batch of at most kSmallBytes and clg::kZSmallTilesMax tiles, without Serializable
  // tables, decodes in ONE launch (k_decode_small_tiles, decode_fused.hip): the plan
  // goes up in one copy, and the kernel writes host outputs straight into pinned memory, so
  // the call is copy + launch + one wait -- the three-pass sequence is about 15 queue
  // operations, which for config 1 (44 logs, 73 KB) cost more than the decode.  A span that
  // goes wrong sends the batch down the usual path.  CLG_F_NO_SMALL_DECODE (or CLONOS_SMALL=0,
  // a developer switch) turns it off.
  static constexpr uint64_t kSmallBytes = 1u << 20;
  static constexpr uint32_t kSmallSpans = clg::kZSmallSpans;
  static constexpr uint64_t kSmallHostOut = 32u << 20;  // pinned output bytes at most (cap-sized)
  PinBuf h_small_out, h_small_res;
  // Decode errors kept on the fast path (FusedCtl::span_err; CLONOS_KEEP_ERRORS=0 turns it off,
  // a developer switch): a span whose error the full rules confirm keeps the fast run's records
  // before it, and only spans whose chains went wrong otherwise go to the robust pipeline.
  // Test switch (CLONOS_FUSED_PERTURB, FusedCtl::perturb): wrong chunk entries and a wrong
  // look-back result, which the checks must catch (k_decode_repair, run_small, emit).
  const uint32_t fused_perturb = [] {
    const char* v = getenv("CLONOS_FUSED_PERTURB");
    return v ? uint32_t(strtoul(v, nullptr, 0)) : 0u;
  }();
  const bool keep_errors = [] {
    const char* v = getenv("CLONOS_KEEP_ERRORS");
    return !(v && atoi(v) == 0);
  }();
  DevBuf d_zerr, d_sf_cls;
  DevBuf d_small;
  clg::SmallPlanArg small_arg;
  bool small_flip = false;
  bool small_ok(const DecodePlan& p, uint64_t log_bytes, const clg_decoded* out) const {
    if (!small_decode || jser_hint || p.spans.empty() || p.spans.size() > kSmallSpans || log_bytes > kSmallBytes ||
        p.only || p.staged)
      return false;
    if (out->out_kind == CLG_MEM_HOST && out->cap * 13 + out->wcap * 25 > kSmallHostOut) return false;
    if (out->out_kind == CLG_MEM_MAPPED && !mapped_outputs(*out, nullptr)) return false;
    return p.n_tiles <= clg::kZSmallTilesMax;
  }
  // CLG_MEM_MAPPED outputs: every array's device address (false: one is not registered, or
  // its cap / wcap elements reach past its registered range -- the caller's staging path then)
  static bool mapped_outputs(const clg_decoded& out, clg::DecodeOut* o) {
    void* h[9] = {out.off, out.tag, out.v0, out.w_idx, out.w_rc, out.w_v1, out.w_var_off, out.w_var_len, out.w_sub};
    const uint64_t c = std::max<uint64_t>(1, out.cap), w = std::max<uint64_t>(1, out.wcap);
    const uint64_t n[9] = {c * 4, c, c * 8, w * 4, w * 4, w * 8, w * 4, w * 4, w};
    uintptr_t d[9];
    for (int i = 0; i < 9; ++i)
      if (!(d[i] = clg_mapped_device_address(h[i], n[i]))) return false;
    if (o)
      *o = clg::DecodeOut{reinterpret_cast<uint32_t*>(d[0]), reinterpret_cast<uint8_t*>(d[1]), reinterpret_cast<int64_t*>(d[2]),
                          reinterpret_cast<uint32_t*>(d[3]), reinterpret_cast<int32_t*>(d[4]), reinterpret_cast<int64_t*>(d[5]),
                          reinterpret_cast<uint32_t*>(d[6]), reinterpret_cast<uint32_t*>(d[7]), reinterpret_cast<uint8_t*>(d[8]),
                          out.cap, out.wcap};
    return true;
  }
  // The plan's device-planned runs as host-built tiles (k_expand_tiles' rule, on the host).
  void host_tiles(DecodePlan& p) {
    if (p.runs.empty()) return;
    const uint32_t U = p.unit, Cb = C();
    p.tiles.resize(p.n_tiles);
    for (const auto& r : p.runs) {
      const uint32_t w0 = r.phys / U, w1 = (r.phys + r.len - 1) / U;
      for (uint32_t w = w0; w <= w1; ++w) {
        const uint32_t s0 = std::max(w * U, r.phys), e1 = std::min((w + 1) * U, r.phys + r.len);
        const uint32_t si = s0 / Cb, so = s0 % Cb;
        p.tiles[r.first + (w - w0)] = clg::TileDesc{seg_addr(segtab_at(p, r.segtab_off + si)) + (so & ~15u), so & 15u,
                                                    e1 - s0, uint32_t(r.dst), 0, uint64_t(s0 - r.phys)};
      }
    }
    p.runs.clear();
    p.segtab.clear();
    p.unit = 0;
  }
  static uint32_t segtab_at(const DecodePlan& p, uint64_t i) { return p.segtab[size_t(i)]; }
  // The small path's hand-offs, checked once its kernel is done: every tile but a span's first
  // entered at the exit the tile before it published, and every tile's base is the one before
  // it plus that tile's counts (the kernel's per-tile words: entry | exit << 32, base, counts).
  // A mismatch -- a poll that read a wrong word -- sends the batch the usual way.
  bool small_handoffs_ok(const DecodePlan& p, const uint64_t* res) {
    const uint32_t nt = p.n_tiles, ns = uint32_t(p.spans.size());
    const uint64_t* ck = res + 3 + ns;
    for (uint32_t t = 0; t < nt; ++t) {
      const uint64_t* k = ck + 3 * size_t(t);
      const bool first = p.tiles[t].span_off == 0;
      if ((t == 0 ? k[1] != 0 : k[1] != k[-2] + k[-1]) || (!first && uint32_t(k[0]) != uint32_t(k[-3] >> 32))) {
        stats["decode_small_handoff"].launches++;
        return false;
      }
    }
    return true;
  }
  int run_small(DecodePlan& p, uint64_t log_bytes, clg_decoded* out, uint64_t* span_rec_base, bool* aborted) {
    HostTimer ht(this, "host_decode_small");
    *aborted = false;
    reset_result(out);
    host_tiles(p);
    const uint32_t nt = p.n_tiles, ns = uint32_t(p.spans.size());
    if (nt == 0) {  // every span empty: no records, and no launch (a grid of zero blocks is invalid)
      if (span_rec_base) std::fill(span_rec_base, span_rec_base + ns + 1, uint64_t(0));
      out->n_rec = out->n_wide = 0;
      return CLG_OK;
    }
    // the plan: in the launch's arguments when it fits (no copy queued), else one copy
    const bool arg_plan = nt <= clg::kZSmallArgTiles && ns <= clg::kZSmallArgSpans;
    PlanLayout L;
    if (arg_plan) {
      memcpy(small_arg.tiles, p.tiles.data(), size_t(nt) * sizeof(clg::TileDesc));
      memcpy(small_arg.spans, p.spans.data(), size_t(ns) * sizeof(clg::SpanDesc));
    } else {
      CHK(stage_plan(p, d_ztiles, &L));
    }
    // outputs: the caller's device arrays, or pinned host memory the kernel writes directly
    clg::DecodeOut o{};
    const bool host = out->out_kind == CLG_MEM_HOST;
    const uint64_t cap = std::max<uint64_t>(1, out->cap), wcap = std::max<uint64_t>(1, out->wcap);
    uint64_t at[10] = {0};
    const uint64_t sz[9] = {cap * 4, cap, cap * 8, wcap * 4, wcap * 4, wcap * 8, wcap * 4, wcap * 4, wcap};
    for (int i = 0; i < 9; ++i) at[i + 1] = (at[i] + sz[i] + 15) & ~uint64_t(15);
    if (host) {
      CHK(h_small_out.ensure(at[9] + 16));
      uint8_t* hb = h_small_out.as<uint8_t>();
      o = clg::DecodeOut{reinterpret_cast<uint32_t*>(hb + at[0]), hb + at[1], reinterpret_cast<int64_t*>(hb + at[2]),
                         reinterpret_cast<uint32_t*>(hb + at[3]), reinterpret_cast<int32_t*>(hb + at[4]),
                         reinterpret_cast<int64_t*>(hb + at[5]), reinterpret_cast<uint32_t*>(hb + at[6]),
                         reinterpret_cast<uint32_t*>(hb + at[7]), hb + at[8], out->cap, out->wcap};
    } else if (out->out_kind == CLG_MEM_MAPPED) {  // registered host memory: written from the GPU directly
      mapped_outputs(*out, &o);
    } else {
      o = clg::DecodeOut{out->off, out->tag, out->v0, out->w_idx, out->w_rc, out->w_v1, out->w_var_off,
                         out->w_var_len, out->w_sub, out->cap, out->wcap};
    }
    // scratch: per-tile counts and record-start bitmaps, per-span look-back words
    CHK(d_zbits.ensure(std::max<size_t>(1, nt) * 64 * 16));
    CHK(h_small_res.ensure((3 + size_t(ns) + 3 * size_t(nt)) * 8));  // (+ the per-tile hand-off words)
    uint64_t* res = h_small_res.as<uint64_t>();
    res[0] = res[1] = res[2] = 0;
    // look-back words: two buffers of kZSmallAggWords, zeroed once; each call zeroes the other;
    // then the per-tile counts
    constexpr size_t kAgg = clg::kZSmallAggWords;
    if (!d_small.p) {
      CHK(d_small.ensure((2 * kAgg + clg::kZSmallTilesMax) * 8));
      HIPCHK(hipMemsetAsync(d_small.p, 0, 2 * kAgg * 8, stream));
    }
    uint64_t* agg = d_small.as<uint64_t>() + (small_flip ? kAgg : 0);
    uint64_t* agg_next = d_small.as<uint64_t>() + (small_flip ? 0 : kAgg);
    small_flip = !small_flip;
    uint64_t* cnt = d_small.as<uint64_t>() + 2 * kAgg;
    clg::FusedCtl ctl{};
    ctl.cnt = cnt;
    ctl.bits = d_zbits.as<uint64_t>();
    ctl.n_tiles = nt;
    ctl.n_spans = ns;
    ctl.perturb = fused_perturb;
    // warm-up 32 B, not staggered: a lone wave per span waits on every step, and shorter
    // warm-ups cost fewer merges than they save (config 1: the kernel 65 -> 62 us at 32 or 16 B,
    // 63 at 48)
    ctl.warm = 32u | (1u << 31);
    const bool sprof = getenv("CLONOS_SMALL_PROF") != nullptr;  // developer diagnostics: phase stamps
    if (sprof) {
      CHK(d_prof.ensure(size_t(nt) * 64));
      HIPCHK(hipMemsetAsync(d_prof.p, 0, size_t(nt) * 64, stream));
      ctl.prof = d_prof.as<uint64_t>();
    }
    std::optional<HostTimer> hsub(std::in_place, this, "host_small_submit");  // (CLONOS_HOST_PROF sub-stages)
    if (!arg_plan) HIPCHK(hipMemcpyAsync(d_plan.p, h_plan_s[0].p, L.hb, hipMemcpyHostToDevice, stream));
    const bool timing = (cfg.flags & CLG_F_TIMING) != 0;
    hipEvent_t ea = nullptr, eb = nullptr;
    if (timing) {
      ea = get_event();
      eb = get_event();
      HIPCHK(hipEventRecord(ea, stream));
    }
    CHK(clg::launch_decode_small(reinterpret_cast<const clg::TileDesc*>(d_plan.p), nt,
                                 reinterpret_cast<const clg::SpanDesc*>(d_plan.as<uint8_t>() + L.o_spans), ns, ctl, o,
                                 agg, agg_next, res, stream, arg_plan ? &small_arg : nullptr));
    if (timing) HIPCHK(hipEventRecord(eb, stream));
    hsub.emplace(this, "host_small_wait");
    HIPCHK(hipStreamSynchronize(stream));
    hsub.emplace(this, "host_small_finish");
    if (sprof) {  // per tile (count_tile's stamps): walk, merge, counts ticks; merge steps, passes
      std::vector<uint64_t> hp(size_t(nt) * 8);
      HIPCHK(hipMemcpy(hp.data(), d_prof.p, hp.size() * 8, hipMemcpyDeviceToHost));
      for (uint32_t t = 0; t < nt; ++t) {
        const uint64_t* q = &hp[size_t(t) * 8];
        fprintf(stderr, "[clonos] small decode tile %u: walk %llu  merge %llu  counts %llu  steps %llu/%llu  passes %llu\n", t,
                (unsigned long long)(q[2] - q[1]), (unsigned long long)(q[3] - q[2]), (unsigned long long)(q[4] - q[3]),
                (unsigned long long)(q[5] & 0xFFFFF), (unsigned long long)((q[5] >> 20) & 0xFFFFF),
                (unsigned long long)(q[5] >> 40));
      }
    }
    if (res[2] || !small_handoffs_ok(p, res)) {
      if (timing) timings.push_back(PendingTiming{"decode_small", ea, eb, 0});
      *aborted = true;
      return CLG_OK;
    }
    constexpr uint64_t kRecMask = (1ull << 31) - 1;
    const uint64_t nrec = res[0], nwide = res[1];
    if (span_rec_base) {
      for (uint32_t s = 0; s < ns; ++s) span_rec_base[s] = res[3 + s] & kRecMask;
      span_rec_base[ns] = nrec;
      for (uint32_t s = ns; s-- > 0;)  // (the kernel writes the spans with tiles: an empty one starts where the next does)
        if (!p.spans[s].n_tiles) span_rec_base[s] = span_rec_base[s + 1];
    }
    if (timing) timings.push_back(PendingTiming{"decode_small", ea, eb, log_bytes + 13 * nrec + 25 * nwide});
    out->n_rec = nrec;
    out->n_wide = nwide;
    if (host) {
      const uint64_t r = std::min(nrec, out->cap), w = std::min(nwide, out->wcap);
      const uint8_t* hb = h_small_out.as<uint8_t>();
      void* dst[9] = {out->off, out->tag, out->v0, out->w_idx, out->w_rc, out->w_v1, out->w_var_off, out->w_var_len,
                      out->w_sub};
      const uint64_t n[9] = {r * 4, r, r * 8, w * 4, w * 4, w * 8, w * 4, w * 4, w};
      for (int i = 0; i < 9; ++i)
        if (n[i]) memcpy(dst[i], hb + at[i], n[i]);
    }
    if (nrec > out->cap || nwide > out->wcap)
      return fail(CLG_E_CAPACITY, "decode produced %llu records / %llu wide rows, capacity %llu / %llu",
                  (unsigned long long)nrec, (unsigned long long)nwide, (unsigned long long)out->cap,
                  (unsigned long long)out->wcap);
    return CLG_OK;
  }

  // Decode dispatcher: fused single pass first, robust pipeline on abort.  `build(plan,
  // tile_bytes)` fills a plan for the given tile geometry.
  template <class Build>
  int decode(Build&& build, uint64_t log_bytes, clg_decoded* out, uint64_t* span_rec_base,
             DecodePlan* prebuilt = nullptr) {
    // fused counts are packed in 31-bit fields: at most log_bytes / 2 records
    if (fused_decode && log_bytes / 2 < (1ull << 31)) {
      DecodePlan own;
      DecodePlan& pf = prebuilt ? *prebuilt : own;  // (prebuilt: the fast plan, kZTile tiles)
      if (!prebuilt) {
        HostTimer hp(this, "host_decode_plan");
        build(pf, clg::kZTile);
      }
      CHK(plan_ok(pf));
      bool aborted = false, need_jser = false;
      if (small_ok(pf, log_bytes, out)) {
        CHK(run_small(pf, log_bytes, out, span_rec_base, &aborted));
        if (!aborted) return CLG_OK;
        stats["decode_small_fallback"].launches++;
      }
      CHK(run_fused(pf, log_bytes, out, span_rec_base, &aborted, jser_hint, &need_jser));
      if (!aborted) return CLG_OK;
      return after_abort(pf, build, log_bytes, out, span_rec_base, need_jser);
    }
    DecodePlan p;
    build(p, uint32_t(clg::kTile));
    CHK(plan_ok(p));
    return run_decode(p, log_bytes, out, span_rec_base);
  }
  int plan_ok(const DecodePlan& p) {
    return p.status == CLG_OK ? CLG_OK
                              : fail(p.status, "a queued decode's log range is gone (truncated past its start epoch)");
  }

  // Per-span fallback after a fast run whose chains went wrong in some spans only (a
  // decode error, a record the fast rules cannot place): those spans are decoded together in
  // one robust run into scratch, their counts injected into the fast run's per-tile counts,
  // scan and emit re-run for the other spans (emit skips the bad ones), and the robust
  // records placed by one kernel (k_sf_place; their wide rows' record indices moved to the
  // batch's).  *done = false: not applicable (too many or too large bad spans), the
  // caller decodes the whole batch robustly.  The result equals the whole-batch robust
  // decode's: every span's records, the first error of the lowest span.
  // at most this many bad spans, and three quarters of the bytes: past that the whole batch
  // goes robust (one run either way; the fast run's second half is the saving)
  static constexpr uint32_t kSfMaxSpans = 8192;
  template <class Build>
  int span_fallback(DecodePlan& pf, Build&& build, uint64_t log_bytes, clg_decoded* out, uint64_t* span_rec_base,
                    bool* done) {
    *done = false;
    const uint32_t ns = uint32_t(pf.spans.size()), nt = pf.n_tiles;
    std::vector<uint32_t> flag(ns);
    HIPCHK(hipMemcpy(flag.data(), d_zbad.p, size_t(ns) * 4, hipMemcpyDeviceToHost));
    // spans with an error position (kept errors): the full rules classify the record there on
    // the GPU; a confirmed error keeps the fast run's records before it (k_err_classify)
    std::vector<uint32_t> kept;
    std::vector<uint64_t> kept_off;
    std::vector<int32_t> kept_res;
    if (zlast.ctl.span_err) {
      std::vector<uint64_t> err(ns);
      HIPCHK(hipMemcpy(err.data(), zlast.ctl.span_err, size_t(ns) * 8, hipMemcpyDeviceToHost));
      std::vector<uint32_t> cand;
      for (uint32_t s = 0; s < ns; ++s)
        if (flag[s] && err[s] != ~0ull) cand.push_back(s);
      if (!cand.empty()) {
        const uint32_t nc = uint32_t(cand.size());
        CHK(d_sf_cls.ensure(size_t(nc) * 12 + 64));
        HIPCHK(hipMemcpyAsync(d_sf_cls.p, cand.data(), size_t(nc) * 4, hipMemcpyHostToDevice, stream));
        auto* cres = reinterpret_cast<int32_t*>(d_sf_cls.as<uint8_t>() + ((size_t(nc) * 4 + 15) & ~size_t(15)));
        clg::JArena jar;
        CHK(jarena_reset(&jar));
        CHK(clg::launch_err_classify(d_ztiles.as<clg::TileDesc>(), d_spans.as<clg::SpanDesc>(), d_sf_cls.as<uint32_t>(),
                                     nc, zlast.ctl, cres, jar, stream));
        std::vector<int32_t> cr(size_t(nc) * 2);
        HIPCHK(hipMemcpyAsync(cr.data(), cres, cr.size() * 4, hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        for (uint32_t i = 0; i < nc; ++i)
          if (cr[2 * i] < 0) {  // confirmed: not a bad span any more
            flag[cand[i]] = 0;
            kept.push_back(cand[i]);
            kept_off.push_back(err[cand[i]]);
            kept_res.push_back(cr[2 * i]);
            kept_res.push_back(cr[2 * i + 1]);
          }
      }
    }
    std::vector<uint32_t> bad;
    uint64_t bad_bytes = 0;
    for (uint32_t s = 0; s < ns; ++s)
      if (flag[s]) {
        bad.push_back(s);
        bad_bytes += pf.spans[s].len;
      }
    if ((bad.empty() && kept.empty()) || bad.size() > kSfMaxSpans || bad_bytes > log_bytes / 4 * 3) return CLG_OK;
    if (!kept.empty()) stats["decode_kept_errors"].launches++;
    if (!bad.empty()) stats["decode_span_fallback"].launches++;
    const uint32_t nb = uint32_t(bad.size());
    // scratch: the robust decode's records (13 B) and wide rows (25 B) of the bad spans
    const uint64_t RC = bad_bytes / 2 + nb + 1, WC = bad_bytes / 6 + nb + 1;  // (records are >= 2 B, wide >= 6 B)
    CHK(d_sf_rec.ensure(RC * 13 + 64));
    CHK(d_sf_wide.ensure(WC * 25 + 64));
    uint8_t* rb = d_sf_rec.as<uint8_t>();
    uint8_t* wb = d_sf_wide.as<uint8_t>();
    auto* s_off = reinterpret_cast<uint32_t*>(rb);
    auto* s_v0 = reinterpret_cast<int64_t*>(rb + RC * 4 + 7 - (RC * 4 + 7) % 8);
    auto* s_tag = reinterpret_cast<uint8_t*>(s_v0 + RC);
    auto* s_widx = reinterpret_cast<uint32_t*>(wb);
    auto* s_wrc = reinterpret_cast<int32_t*>(s_widx + WC);
    auto* s_wvo = reinterpret_cast<uint32_t*>(s_wrc + WC);
    auto* s_wvl = s_wvo + WC;
    auto* s_wv1 = reinterpret_cast<int64_t*>(reinterpret_cast<uint8_t*>(s_wvl + WC) + 8 - (uintptr_t(s_wvl + WC) & 7));
    auto* s_wsub = reinterpret_cast<uint8_t*>(s_wv1 + WC);
    std::vector<uint64_t> packed(nb), nrec(nb), nwide(nb), rbase(nb), wbase(nb);
    int e_status = CLG_OK, e_tag = 0;
    uint32_t e_span = 0;
    int64_t e_off = -1;
    if (nb) {  // every bad span in ONE robust run (spans 0 .. nb-1 of its plan), into scratch
      DecodePlan sp;
      sp.only = &bad;
      build(sp, uint32_t(clg::kTile));
      CHK(plan_ok(sp));
      clg_decoded so{};
      so.off = s_off;
      so.tag = s_tag;
      so.v0 = s_v0;
      so.w_idx = s_widx;
      so.w_rc = s_wrc;
      so.w_v1 = s_wv1;
      so.w_var_off = s_wvo;
      so.w_var_len = s_wvl;
      so.w_sub = s_wsub;
      so.cap = RC;
      so.wcap = WC;
      so.out_kind = CLG_MEM_DEVICE;
      const int st = run_decode(sp, bad_bytes, &so, nullptr);
      if (st != CLG_OK && so.err_status == CLG_OK) return st;  // an engine failure, not a decode error
      if (so.err_status != CLG_OK) {  // the lowest bad span's error (bad[] ascends)
        e_status = so.err_status;
        e_span = bad[so.err_span];
        e_off = so.err_off;
        e_tag = so.err_tag;
      }
      // per span: records, wide rows and their places in the scratch (run_decode's span results)
      const clg::SpanRes* hres = h_sres.as<clg::SpanRes>();
      for (uint32_t i = 0; i < nb; ++i) {
        nrec[i] = hres[i].n_rec;
        nwide[i] = hres[i].n_wide;
        rbase[i] = hres[i].rec_base;
        wbase[i] = hres[i].wide_base;
        if (nrec[i] >= (1ull << 31) || nwide[i] >= (1ull << 32)) return CLG_OK;  // past the fast counts' packing
        packed[i] = nwide[i] << 31 | nrec[i];
      }
    }
    // the lowest span's error: the robust run's or a kept one's (kept[] ascends)
    if (!kept.empty() && (e_status == CLG_OK || kept[0] < e_span)) {
      e_status = kept_res[0];
      e_span = kept[0];
      e_off = int64_t(kept_off[0]);
      e_tag = kept_res[1];
    }
    // the fast run again over the good spans: its plan back in place (the robust runs used
    // the shared span table), the bad spans' counts injected, scan and emit (kept errors: the
    // tiles past the error hold no records, emit stops there)
    PlanLayout L;
    if (nb) {
      CHK(stage_plan(pf, d_ztiles, &L));
      CHK(enqueue_plan(pf, L, d_ztiles));
    }
    // meta: the packed counts, the bad spans, then the placement rows (16-byte aligned)
    const size_t o_place = (size_t(nb) * 12 + 15) & ~size_t(15), mb = o_place + size_t(nb) * sizeof(clg::SfPlace);
    CHK(d_sf_meta.ensure(mb + 64));
    std::vector<uint8_t> meta(mb + 8);
    memcpy(meta.data(), packed.data(), size_t(nb) * 8);
    memcpy(meta.data() + size_t(nb) * 8, bad.data(), size_t(nb) * 4);
    auto* pl = reinterpret_cast<clg::SfPlace*>(meta.data() + o_place);
    for (uint32_t i = 0; i < nb; ++i) pl[i] = clg::SfPlace{rbase[i], nrec[i], wbase[i], nwide[i], bad[i], 0};
    HIPCHK(hipMemcpyAsync(d_sf_meta.p, meta.data(), mb, hipMemcpyHostToDevice, stream));
    clg::FusedCtl ctl = zlast.ctl;
    ctl.skip_bad = 1;
    ctl.lb_check = 0;  // (the three-launch scan below: no look-back words)
    ctl.chunk = nullptr;  // (the count pass's chunk table is not staged again: scan and emit never read it)
    auto* zt = d_ztiles.as<clg::TileDesc>();
    auto* zs = d_spans.as<clg::SpanDesc>();
    CHK(clg::launch_decode_inject(zs, reinterpret_cast<const uint32_t*>(d_sf_meta.as<uint8_t>() + size_t(nb) * 8),
                                  d_sf_meta.as<uint64_t>(), nb, ctl, stream));
    HIPCHK(hipMemsetAsync(ctl.abort, 0, 32, stream));
    CHK(clg::launch_decode_fused(zt, nt, zs, ns, ctl, zlast.o, stream, 1));
    CHK(clg::launch_decode_fused(zt, nt, zs, ns, ctl, zlast.o, stream, 2));
    // the robust records into place, at the bases the scan gave the bad spans (one launch)
    const clg::DecodeOut sc{s_off, s_tag, s_v0, s_widx, s_wrc, s_wv1, s_wvo, s_wvl, s_wsub, RC, WC};
    CHK(clg::launch_sf_place(reinterpret_cast<const clg::SfPlace*>(d_sf_meta.as<uint8_t>() + o_place), nb, sc, zlast.o,
                             ctl, stream));
    CHK(h_zres_s[0].ensure((2 * size_t(ns) + clg::kZAbortWords / 2) * 8));
    uint64_t* hz = h_zres_s[0].as<uint64_t>();
    HIPCHK(hipMemcpyAsync(hz, ctl.span_lo, (2 * size_t(ns) + 4) * 8, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    if (reinterpret_cast<const uint32_t*>(hz + 2 * size_t(ns))[0]) return CLG_OK;  // (cannot happen) whole batch
    uint64_t tr = 0, tw = 0;
    span_totals(pf, hz, span_rec_base, &tr, &tw);
    *done = true;
    CHK(finish_out(out, tr, tw));
    if (e_status != CLG_OK) {
      out->err_status = e_status;
      out->err_span = e_span;
      out->err_off = e_off;
      out->err_tag = e_tag;
      return fail(e_status, "decode error %d in span %u at offset %lld (tag %d)", e_status, e_span, (long long)e_off,
                  e_tag);
    }
    return CLG_OK;
  }

  // The fast path aborted: again with the Serializable length tables when that was the
  // reason; then, when only some spans' chains went wrong, those spans alone through the
  // robust pipeline (span_fallback); else the whole batch through it.
  template <class Build>
  int after_abort(DecodePlan& pf, Build&& build, uint64_t log_bytes, clg_decoded* out, uint64_t* span_rec_base,
                  bool need_jser) {
    bool aborted = true, nj = false;
    if (pf.staged) {  // its runs and segment table live only in the pinned buffer: planned again
      pf.reset();
      build(pf, clg::kZTile);
      CHK(plan_ok(pf));
    }
    // the one-pass decode aborted (a case its rules leave to the three passes): those
    if (zlast.one) {
      allow_one = false;
      const int st = run_fused(pf, log_bytes, out, span_rec_base, &aborted, zlast.jser || need_jser, &nj);
      allow_one = true;
      CHK(st);
      if (!aborted) return CLG_OK;
      need_jser = nj;
    }
    // a look-back read gave a wrong offset (emit's check): the fast path once more, as it was
    if (zlast.lookback_bad && !need_jser) {
      CHK(run_fused(pf, log_bytes, out, span_rec_base, &aborted, zlast.jser, &nj));
      if (!aborted) return CLG_OK;
      need_jser = nj;
    }
    // with the tables; again (at most twice) while a table arena was full and has grown
    for (int tries = 0; need_jser && tries < 3; ++tries) {
      stats["decode_jser_retry"].launches++;
      CHK(run_fused(pf, log_bytes, out, span_rec_base, &aborted, true, &nj));
      if (!aborted) return CLG_OK;
      need_jser = nj;
    }
    if (zlast.span_local && !nj) {
      bool done = false;
      const int st = span_fallback(pf, build, log_bytes, out, span_rec_base, &done);
      if (done) return st;
    }
    stats["decode_fallback"].launches++;
    DecodePlan p;
    build(p, uint32_t(clg::kTile));
    CHK(plan_ok(p));
    return run_decode(p, log_bytes, out, span_rec_base);
  }

  // ---------------------------------------------------------------- asynchronous decode
  // clg_decode_logs_async: the three-pass decode is queued and the call returns; settle()
  // completes it (result, fallbacks) in clg_decode_wait or first thing in any other call
  // that needs the engine exclusively (see ENGINE_GUARD), so a pending decode never sees
  // its inputs change.  Slices into device memory on the gather stream and consumer seeks
  // leave it pending: they only read log segments and move consumer offsets.
  // Up to CLG_DECODE_MAX_INFLIGHT decodes are queued at once, each with its own slot (read-
  // back words, staged plan, completion event), so decode i+1's kernels are on the stream
  // before the host completes decode i and the GPU never waits for the host in between.
  // The device scratch (control words, bitmaps, tables) is shared and stream-ordered: the
  // fast path of decode i only needs its read-back.  A decode whose fast run aborted while a
  // later one was already queued has lost its scratch to that one, so it is decoded again
  // from its plan builder, and so are the later ones (rare: they may share its outputs).
  struct PendingDecode {
    bool active = false;  // queued on the GPU, not yet completed
    bool redo = false;    // its fast run's scratch is void: decode again when completed
    DecodePlan plan;
    FusedRun run;
    uint64_t log_bytes = 0;
    clg_decoded* out = nullptr;
    uint64_t* span_rec_base = nullptr;
    std::function<void(DecodePlan&, uint32_t)> build;
    int status = CLG_OK;  // its result, for the clg_decode_wait that pairs with it
    std::string err;      // and its error text
    int64_t min_epoch = INT64_MIN;  // the smallest start epoch it decodes from (INT64_MIN: unknown)
  };
  // clg_truncate_all while decodes are queued (their ranges start at or above the checkpoint):
  // the segments it frees wait here until no decode is queued (the queued kernels may still
  // read them), and the logs' rebase generation tells a queued decode that re-plans (an abort's
  // fallback) to look its ranges up again
  std::vector<uint32_t> free_later;
  uint64_t rebase_gen = 0;
  int64_t q_min_epoch = INT64_MIN;  // clg_decode_logs_async -> decode_async: the call's smallest start epoch
  void release_later() {
    if (free_later.empty() || any_active()) return;
    free_segs.insert(free_segs.end(), free_later.begin(), free_later.end());
    free_later.clear();
  }
  std::deque<PendingDecode> pq;  // queued by clg_decode_logs_async, not yet waited for (oldest first)
  // the largest queued plan so far (the scratch is sized for it): a larger one is queued only
  // once nothing is in flight, since growing a buffer frees the one the GPU may still read
  uint64_t hw_tiles = 0, hw_spans = 0, hw_runs = 0, hw_segs = 0;
  bool hw_jser = false;

  bool any_active(size_t from = 0) const {
    for (size_t i = from; i < pq.size(); ++i)
      if (pq[i].active) return true;
    return false;
  }
  // A decode the async call completed at once (not queued): its status goes to the wait.
  // Engine failures (not a decode result) return from the call instead, with nothing queued.
  int push_settled(int st, clg_decoded* out) {
    if (st != CLG_OK && st != CLG_E_CAPACITY && out->err_status == CLG_OK) return st;
    PendingDecode d;
    d.status = st;
    if (st != CLG_OK) d.err = g_err;
    pq.push_back(std::move(d));
    return CLG_OK;
  }
  // queued decodes' plans, recycled (a config-4 plan is ~4 MB: fresh pages cost page faults)
  std::vector<DecodePlan> plan_pool;
  int decode_async(std::function<void(DecodePlan&, uint32_t)> build, uint64_t log_bytes, clg_decoded* out,
                   uint64_t* span_rec_base, DecodePlan* prebuilt = nullptr) {
    const bool fast = fused_decode && log_bytes / 2 < (1ull << 31);
    DecodePlan pf;
    if (prebuilt) {
      pf = std::move(*prebuilt);  // (the fast plan, kZTile tiles)
    } else if (fast) {
      HostTimer hp(this, "host_decode_plan");
      build(pf, clg::kZTile);
    }
    CHK(plan_ok(pf));
    const bool queue = fast && !pf.spans.empty() && fused_fits(pf);
    // what the queued decodes' completions need must not be overwritten by this one's kernels:
    // host outputs go through shared staging arrays, and a scratch buffer that has to grow
    // frees the old one
    bool clash = !queue;
    for (const auto& d : pq)
      if (d.active && d.out->out_kind != CLG_MEM_DEVICE) clash = true;
    if (queue && (pf.n_tiles > hw_tiles || pf.spans.size() > hw_spans || pf.run_count() > hw_runs ||
                  pf.seg_count() > hw_segs || (jser_hint && !hw_jser)))
      clash = true;
    if (clash) CHK(settle());
    if (!queue) {  // nothing to queue, or too large for the fast path: decoded now
      if (fast && pf.spans.empty()) {
        reset_result(out);
        return push_settled(CLG_OK, out);
      }
      return push_settled(decode(build, log_bytes, out, span_rec_base), out);
    }
    reset_result(out);
    // a slot no queued decode holds: the one the plan was staged for (free still: planned in
    // this call, and a settle above only frees slots)
    const uint32_t slot = pf.staged ? pf.stage_slot : free_slot();
    if (slot == 0 || slot >= kSlots || slot_used(slot))
      return fail(CLG_E_STATE, "no free decode slot");  // (cannot happen: bounded by the caller)
    FusedRun r;
    r.slot = slot;
    CHK(launch_fused(pf, log_bytes, out, jser_hint, &r));
    hw_tiles = std::max<uint64_t>(hw_tiles, pf.n_tiles);
    hw_spans = std::max<uint64_t>(hw_spans, pf.spans.size());
    hw_runs = std::max<uint64_t>(hw_runs, pf.run_count());
    hw_segs = std::max<uint64_t>(hw_segs, pf.seg_count());
    hw_jser = hw_jser || r.jser;
    PendingDecode d;
    d.active = true;
    d.plan = std::move(pf);
    d.run = r;
    d.log_bytes = log_bytes;
    d.out = out;
    d.span_rec_base = span_rec_base;
    d.build = std::move(build);
    d.min_epoch = q_min_epoch;
    pq.push_back(std::move(d));
    return CLG_OK;
  }

  bool slot_used(uint32_t slot) const {
    for (const auto& d : pq)
      if (d.active && d.run.slot == slot) return true;
    return false;
  }
  uint32_t free_slot() const {  // the first asynchronous decode slot no queued decode holds (kSlots: none)
    uint32_t slot = 1;
    while (slot < kSlots && slot_used(slot)) ++slot;
    return slot;
  }
  // Completes the queued decodes [0, upto] (all: upto = SIZE_MAX), oldest first.
  int settle(size_t upto = SIZE_MAX) {
    for (size_t i = 0; i < pq.size() && i <= upto; ++i) {
      PendingDecode& d = pq[i];
      if (!d.active) continue;
      d.active = false;
      int st;
      if (d.redo) {  // a decode before it aborted after this one was queued
        CHK(sync());
        st = decode(d.build, d.log_bytes, d.out, d.span_rec_base);
      } else {
        bool aborted = false, need_jser = false;
        settling = true;
        st = finish_fused(d.plan, d.run, d.out, d.span_rec_base, &aborted, &need_jser);
        settling = false;
        if (st == CLG_OK && aborted) {
          if (any_active(i + 1)) {  // its scratch went to the later decodes: all of them again
            stats["decode_async_redo"].launches++;
            CHK(sync());
            for (size_t j = i + 1; j < pq.size(); ++j)
              if (pq[j].active) pq[j].redo = true;
            st = decode(d.build, d.log_bytes, d.out, d.span_rec_base);
          } else {
            st = after_abort(d.plan, d.build, d.log_bytes, d.out, d.span_rec_base, need_jser);
          }
        }
      }
      d.status = st;
      if (st != CLG_OK) d.err = g_err;
      d.build = nullptr;
      if (plan_pool.size() < kSlots) {
        d.plan.reset();
        plan_pool.push_back(std::move(d.plan));
      }
      d.plan = DecodePlan();
    }
    release_later();
    return CLG_OK;  // the decodes' own statuses go to clg_decode_wait
  }
  // clg_decode_wait: the oldest queued decode, completed; its status
  int wait_oldest(std::string* err) {
    if (pq.empty()) return CLG_OK;
    CHK(settle(0));
    const int st = pq.front().status;
    if (st != CLG_OK) *err = pq.front().err;
    pq.pop_front();
    release_later();
    return st;
  }

  // The robust pipeline; again with a grown spill arena while a Serializable stream walk
  // found the arena full (CLG_E_NOSPACE is never a decode result).
  int run_decode(DecodePlan& p, uint64_t log_bytes, clg_decoded* out, uint64_t* span_rec_base) {
    for (;;) {
      CHK(jarena_clear_note(0));
      const int st = run_decode_once(p, log_bytes, out, span_rec_base);
      if (!jarena_spilled(0)) return st;
      CHK(jarena_grow());
    }
  }
  int run_decode_once(DecodePlan& p, uint64_t log_bytes, clg_decoded* out, uint64_t* span_rec_base) {
    reset_result(out);
    const uint32_t nt = p.n_tiles, ns = uint32_t(p.spans.size());
    if (ns == 0) return CLG_OK;
    CHK(d_agg.ensure(std::max<size_t>(1, nt) * clg::kEntries * sizeof(uint64_t)));
    CHK(d_conv.ensure(std::max<size_t>(1, nt) * sizeof(clg::TileConv)));
    CHK(d_tres.ensure(std::max<size_t>(1, nt) * sizeof(clg::TileRes)));
    CHK(d_sres.ensure(ns * sizeof(clg::SpanRes)));
    CHK(d_totals.ensure(2 * sizeof(uint64_t)));
    CHK(d_fconv.ensure(std::max<size_t>(1, nt) * clg::kFPoints * sizeof(uint32_t)));
    CHK(d_lanes.ensure(std::max<size_t>(1, nt) * clg::kFPoints * sizeof(clg::LaneSeg)));
    CHK(d_sums.ensure(std::max<size_t>(1, nt) * sizeof(clg::TileSum)));
    CHK(d_fres.ensure(std::max<size_t>(1, nt) * sizeof(clg::FastRes)));
    CHK(d_flags.ensure(ns * sizeof(uint32_t)));
    CHK(d_jpos.ensure(std::max<size_t>(1, nt) * clg::kJserCap * sizeof(uint32_t)));
    CHK(d_jlen.ensure(std::max<size_t>(1, nt) * clg::kJserCap * sizeof(uint32_t)));
    CHK(d_jn.ensure(std::max<size_t>(1, nt) * sizeof(uint32_t)));
    CHK(d_defer.ensure(std::max<size_t>(1, nt) * sizeof(uint32_t)));
    CHK(upload_plan(p, d_tiles));
    CHK(h_sres.ensure(ns * sizeof(clg::SpanRes) + 64));
    clg::DecodeOut o{};
    CHK(prep_out(out, &o));
    auto* dt = d_tiles.as<clg::TileDesc>();
    auto* ds = d_spans.as<clg::SpanDesc>();
    auto* flags = d_flags.as<uint32_t>();
    // fast path: fused scan (points + segments) -> per-span resolution -> emit
    clg::JArena jar;
    CHK(jarena_reset(&jar));
    clg::JserTabs J{d_jpos.as<uint32_t>(), d_jlen.as<uint32_t>(), d_jn.as<uint32_t>(), d_defer.as<uint32_t>(), jar};
    J.side = side;  // (k_jser_fill takes a tile's table from the sidecar where it can)
    const char* rprof_path = getenv("CLONOS_ROBUST_PHASES");  // developer diagnostics (stamps per tile)
    if (rprof_path && d_rprof.ensure(std::max<size_t>(1, nt) * 16 * 8) == CLG_OK) {
      J.prof = d_rprof.as<uint64_t>();
      hipMemsetAsync(J.prof, 0, size_t(nt) * 128, stream);
    }
    uint32_t* dbg = nullptr;
    if (getenv("CLONOS_DEBUG_DUMP") && d_dbg.ensure(std::max<size_t>(1, nt) * clg::kFPoints * 4) == CLG_OK)
      dbg = d_dbg.as<uint32_t>();
    uint64_t* prof = nullptr;  // developer diagnostics: per-phase s_memtime stamps of the scan
    const char* prof_path = getenv("CLONOS_SCAN_PHASES");
    if (prof_path && d_prof.ensure(std::max<size_t>(1, nt) * 8 * 8) == CLG_OK) {
      prof = d_prof.as<uint64_t>();
      hipMemsetAsync(prof, 0, size_t(nt) * 64, stream);
    }
    CHK(timed("robust_scan", log_bytes, [&] {
      return clg::launch_fast_scan(dt, nt, ds, d_fconv.as<uint32_t>(), J, 0, d_lanes.as<clg::LaneSeg>(),
                                   d_sums.as<clg::TileSum>(), dbg, prof, stream);
    }));
    if (prof) {
      std::vector<uint64_t> hp(size_t(nt) * 8);
      hipMemcpyAsync(hp.data(), prof, hp.size() * 8, hipMemcpyDeviceToHost, stream);
      hipStreamSynchronize(stream);
      if (FILE* fp = fopen(prof_path, "wb")) {
        fwrite(hp.data(), 8, hp.size(), fp);
        fclose(fp);
      }
    }
    CHK(timed("robust_jser", 0, [&] { return clg::launch_jser_fill(dt, nt, ds, J, stream); }));
    uint64_t* prof2 = nullptr;  // developer diagnostics: the deferred scan's phase stamps (CLONOS_ROBUST_PHASES)
    if (J.prof && d_prof2.ensure(std::max<size_t>(1, nt) * 64) == CLG_OK) {
      prof2 = d_prof2.as<uint64_t>();
      hipMemsetAsync(prof2, 0, size_t(nt) * 64, stream);
    }
    CHK(timed("robust_scan_deferred", 0, [&] {
      return clg::launch_fast_scan(dt, nt, ds, d_fconv.as<uint32_t>(), J, 1, d_lanes.as<clg::LaneSeg>(),
                                   d_sums.as<clg::TileSum>(), dbg, prof2, stream);
    }));
    if (prof2) {
      std::vector<uint64_t> hp(size_t(nt) * 8);
      hipMemcpyAsync(hp.data(), prof2, hp.size() * 8, hipMemcpyDeviceToHost, stream);
      hipStreamSynchronize(stream);
      if (FILE* fp = fopen((std::string(rprof_path) + ".scan").c_str(), "wb")) {
        fwrite(hp.data(), 8, hp.size(), fp);
        fclose(fp);
      }
    }
    CHK(timed("robust_resolve", uint64_t(nt) * 32, [&] {
      return clg::launch_fast_resolve(dt, ds, ns, d_fconv.as<uint32_t>(), d_lanes.as<clg::LaneSeg>(),
                                      d_sums.as<clg::TileSum>(), J, d_fres.as<clg::FastRes>(),
                                      d_sres.as<clg::SpanRes>(), flags, jar, stream);
    }));
    if (cfg.flags & CLG_F_TIMING) {  // diagnostics: spans the convergence-point tier leaves to the DP
      std::vector<uint32_t> hf(ns);
      HIPCHK(hipMemcpyAsync(hf.data(), flags, size_t(ns) * 4, hipMemcpyDeviceToHost, stream));
      HIPCHK(hipStreamSynchronize(stream));
      uint64_t nf = 0, no = 0;
      for (uint32_t f : hf) {
        nf += f != 0;
        no += f == 2;
      }
      stats["robust_dp_spans"].launches += nf;
      stats["robust_dp_spans_overflow"].launches += no;
      stats["robust_spans"].launches += ns;
    }
    // robust DP pipeline for flagged spans only (early exit elsewhere)
    CHK(timed("robust_dp_tables", 0, [&] {
      return clg::launch_decode_tables(dt, nt, ds, d_agg.as<uint64_t>(), d_conv.as<clg::TileConv>(), flags, jar, stream);
    }));
    CHK(timed("robust_dp_resolve", 0, [&] {
      return clg::launch_decode_resolve(dt, ds, ns, d_agg.as<uint64_t>(), d_conv.as<clg::TileConv>(),
                                        d_tres.as<clg::TileRes>(), d_sres.as<clg::SpanRes>(), flags, jar, stream);
    }));
    CHK(timed("robust_spanscan", uint64_t(ns) * 48, [&] {
      return clg::launch_decode_spanscan(d_sres.as<clg::SpanRes>(), ns, d_totals.as<uint64_t>(), stream);
    }));
    // emit bytes are attributed after the counts are known (below)
    hipEvent_t ea = nullptr, eb = nullptr;
    if (cfg.flags & CLG_F_TIMING) {
      ea = get_event();
      eb = get_event();
      hipEventRecord(ea, stream);
    }
    CHK(clg::launch_fast_emit(dt, nt, ds, d_fconv.as<uint32_t>(), J, d_lanes.as<clg::LaneSeg>(),
                              d_fres.as<clg::FastRes>(), d_sres.as<clg::SpanRes>(), flags, o, stream));
    if (cfg.flags & CLG_F_TIMING) hipEventRecord(eb, stream);
    CHK(timed("robust_dp_emit", 0, [&] {
      return clg::launch_decode_emit(dt, nt, ds, d_conv.as<clg::TileConv>(), d_tres.as<clg::TileRes>(),
                                     d_sres.as<clg::SpanRes>(), flags, o, jar, stream);
    }));
    if (J.prof) {
      std::vector<uint64_t> hp(size_t(nt) * 16);
      hipMemcpyAsync(hp.data(), J.prof, hp.size() * 8, hipMemcpyDeviceToHost, stream);
      hipStreamSynchronize(stream);
      if (FILE* fp = fopen(rprof_path, "wb")) {
        fwrite(hp.data(), 8, hp.size(), fp);
        fclose(fp);
      }
    }
    if (const char* dump = getenv("CLONOS_DEBUG_DUMP")) {  // developer diagnostics only
      std::vector<uint32_t> hc(size_t(nt) * clg::kFPoints), hf(ns);
      std::vector<clg::TileSum> hs(nt);
      hipMemcpyAsync(hc.data(), d_fconv.p, hc.size() * 4, hipMemcpyDeviceToHost, stream);
      hipMemcpyAsync(hs.data(), d_sums.p, hs.size() * sizeof(clg::TileSum), hipMemcpyDeviceToHost, stream);
      hipMemcpyAsync(hf.data(), d_flags.p, hf.size() * 4, hipMemcpyDeviceToHost, stream);
      hipStreamSynchronize(stream);
      if (FILE* fp = fopen(dump, "wb")) {
        fwrite(&nt, 4, 1, fp);
        fwrite(&ns, 4, 1, fp);
        fwrite(hc.data(), 4, hc.size(), fp);
        fwrite(hs.data(), sizeof(clg::TileSum), hs.size(), fp);
        fwrite(hf.data(), 4, hf.size(), fp);
        std::vector<clg::TileDesc> ht(nt);
        hipMemcpy(ht.data(), d_tiles.p, nt * sizeof(clg::TileDesc), hipMemcpyDeviceToHost);
        fwrite(ht.data(), sizeof(clg::TileDesc), nt, fp);
        std::vector<uint32_t> hd(size_t(nt) * clg::kFPoints);
        hipMemcpy(hd.data(), d_dbg.p, hd.size() * 4, hipMemcpyDeviceToHost);
        fwrite(hd.data(), 4, hd.size(), fp);
        std::vector<clg::LaneSeg> hl(size_t(nt) * clg::kFPoints);
        hipMemcpy(hl.data(), d_lanes.p, hl.size() * sizeof(clg::LaneSeg), hipMemcpyDeviceToHost);
        fwrite(hl.data(), sizeof(clg::LaneSeg), hl.size(), fp);
        fclose(fp);
      }
    }
    clg::SpanRes* hres = h_sres.as<clg::SpanRes>();
    HIPCHK(hipMemcpyAsync(hres, d_sres.p, ns * sizeof(clg::SpanRes), hipMemcpyDeviceToHost, stream));
    CHK(jarena_note(0));
    HIPCHK(hipStreamSynchronize(stream));
    uint64_t nrec = 0, nwide = 0;
    for (uint32_t s = 0; s < ns; ++s) {
      if (span_rec_base) span_rec_base[s] = hres[s].rec_base;
      nrec += hres[s].n_rec;
      nwide += hres[s].n_wide;
      if (hres[s].status != CLG_OK && out->err_status == CLG_OK) {
        out->err_status = hres[s].status;
        out->err_span = s;
        out->err_off = hres[s].err_off;
        out->err_tag = hres[s].err_tag;
      }
    }
    if (span_rec_base) span_rec_base[ns] = nrec;
    if (cfg.flags & CLG_F_TIMING)
      timings.push_back(PendingTiming{"robust_emit", ea, eb, log_bytes + 13 * nrec + 25 * nwide});
    CHK(finish_out(out, nrec, nwide));
    if (out->err_status != CLG_OK)
      return fail(out->err_status, "decode error %d in span %u at offset %lld (tag %d)", out->err_status, out->err_span,
                  (long long)out->err_off, out->err_tag);
    return CLG_OK;
  }
};

// =======================================================================================
// C-ABI
// =======================================================================================
extern "C" {

// Exclusive calls first complete a pending asynchronous decode (clg_decode_logs_async);
// ENGINE_GUARD_KEEP leaves it pending (calls that only read log segments on the gather
// stream or move consumer offsets).
#define ENGINE_GUARD_KEEP(e)                                        \
  if (!(e)) return fail(CLG_E_INVALID_ARG, "null engine");          \
  XGuard guard_((e)->mu)
#define ENGINE_GUARD(e) \
  ENGINE_GUARD_KEEP(e); \
  (e)->settle()

// A per-log call: only the log's stripe (see EngineLock).
struct LogGuard {
  std::mutex* s;
  LogGuard(clg_engine* e, uint32_t h) : s(e->mu.owned() ? nullptr : &e->mu.stripe[h % kLogStripes].m) {
    if (s) s->lock();
  }
  ~LogGuard() {
    if (s) s->unlock();
  }
};
#define LOG_GUARD(e, h)                                    \
  if (!(e)) return fail(CLG_E_INVALID_ARG, "null engine"); \
  LogGuard lguard_((e), (h))

void clg_config_default(clg_config* cfg) {
  memset(cfg, 0, sizeof *cfg);
  cfg->segment_bytes = 16384;  // NettyConfig.java:86-89
  cfg->pool_segments = 16384;  // 256 MiB
  cfg->device = 0;
  cfg->sharing_depth = CLG_FULL_SHARING;
  cfg->host_tail_bytes = 16384;    // one component of each log's tail kept on the host
  cfg->ifl_segment_bytes = 32768;  // the in-flight log's pool: Flink's 32 KiB memory segments
  cfg->ifl_pool_segments = 4096;   // 128 MiB
}

int clg_abi_version(void) { return CLG_ABI_VERSION; }


int clg_host_register(void* p, uint64_t bytes) {
  if (!p || !bytes) return fail(CLG_E_INVALID_ARG, "null or empty range");
  hipError_t er = hipHostRegister(p, size_t(bytes), hipHostRegisterMapped);
  if (er != hipSuccess) return fail(CLG_E_DEVICE, "hipHostRegister(%llu bytes): %s", (unsigned long long)bytes,
                                     hipGetErrorString(er));
  void* d = nullptr;
  er = hipHostGetDevicePointer(&d, p, 0);
  if (er != hipSuccess) {
    (void)hipHostUnregister(p);
    return fail(CLG_E_DEVICE, "hipHostGetDevicePointer: %s", hipGetErrorString(er));
  }
  std::lock_guard<std::mutex> g(g_map_mu);
  g_mapped.push_back(Mapped{uintptr_t(p), bytes, uintptr_t(d)});
  return CLG_OK;
}

int clg_host_unregister(void* p) {
  {
    std::lock_guard<std::mutex> g(g_map_mu);
    auto it = std::find_if(g_mapped.begin(), g_mapped.end(), [&](const Mapped& m) { return m.host == uintptr_t(p); });
    if (it == g_mapped.end()) return fail(CLG_E_INVALID_ARG, "range not registered");
    g_mapped.erase(it);
  }
  const hipError_t er = hipHostUnregister(p);
  return er == hipSuccess ? CLG_OK : fail(CLG_E_DEVICE, "hipHostUnregister: %s", hipGetErrorString(er));
}


const char* clg_last_error(void) { return g_err.c_str(); }

int clg_engine_create(const clg_config* cfg, clg_engine** out) {
  if (!cfg || !out) return fail(CLG_E_INVALID_ARG, "null argument");
  *out = nullptr;
  if (cfg->segment_bytes < 16 || (cfg->segment_bytes & 15) || cfg->pool_segments == 0)
    return fail(CLG_E_INVALID_ARG, "segment_bytes must be a positive multiple of 16 and pool_segments > 0");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(CLG_E_DEVICE, "no HIP device visible (the engine has no CPU fallback)");
  if (cfg->device < 0 || cfg->device >= ndev) return fail(CLG_E_INVALID_ARG, "device %d out of range", cfg->device);
  std::unique_ptr<clg_engine> e(new clg_engine());
  e->cfg = *cfg;
  const char* dm = getenv("CLONOS_DECODE");
  e->fused_decode = !(cfg->flags & CLG_F_ROBUST_DECODE) && !(dm && !strcmp(dm, "robust"));
  e->small_decode = !(cfg->flags & CLG_F_NO_SMALL_DECODE) && !(getenv("CLONOS_SMALL") && atoi(getenv("CLONOS_SMALL")) == 0);
  if (const char* ja = getenv("CLONOS_JSER_ARENA"))  // initial spill arena bytes (tests: force its growth)
    e->jarena_bytes = std::max<size_t>(256, size_t(strtoull(ja, nullptr, 0)));
  HIPCHK(hipSetDevice(cfg->device));
  {
    // The device-output slice gather (HBM-bound) runs beside the next decode (VALU-bound):
    // its queue gets the higher priority so its workgroups are dispatched first
    // (CLONOS_GATHER_PRIO=0: same priority as the decode stream; 2: the decode stream's
    // queue higher instead, so the decode's short set-up, scan and read-back launches do not
    // wait behind the gather's workgroups).
    const char* gp = getenv("CLONOS_GATHER_PRIO");
    const int mode = gp ? atoi(gp) : 1;
    int lo = 0, hi = 0;
    const bool prio = hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess && hi != lo;
    if (prio && mode == 2) HIPCHK(hipStreamCreateWithPriority(&e->stream, hipStreamNonBlocking, hi));
    else HIPCHK(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    if (prio && mode == 1) HIPCHK(hipStreamCreateWithPriority(&e->gstream, hipStreamNonBlocking, hi));
    else HIPCHK(hipStreamCreateWithFlags(&e->gstream, hipStreamNonBlocking));
  }
  HIPCHK(hipEventCreateWithFlags(&e->gready, hipEventDisableTiming));
  const size_t pool_bytes = size_t(cfg->segment_bytes) * cfg->pool_segments;
  void* p = nullptr;
  HIPCHK(hipMalloc(&p, pool_bytes + 2 * kPoolGuard));  // guards: aligned over-reads either side
  e->pool_alloc = p;
  e->pool = static_cast<uint8_t*>(p) + kPoolGuard;
  e->free_segs.resize(cfg->pool_segments);
  for (uint32_t i = 0; i < cfg->pool_segments; ++i) e->free_segs[i] = cfg->pool_segments - 1 - i;
  e->seg_life.assign(cfg->pool_segments, 0u);
  // the sidecar: C / 64 entries per segment (256 for 16 KiB: config 3 averages ~100), its
  // positions 16 bits (segments up to 64 KiB); CLONOS_SIDECAR=0 turns it off (developer A/B)
  const char* sc = getenv("CLONOS_SIDECAR");
  if (cfg->segment_bytes <= 65536u && cfg->pool_segments && !(sc && atoi(sc) == 0)) {
    const uint32_t cap = std::min<uint32_t>(clg::kSideCapMax, std::max<uint32_t>(8u, cfg->segment_bytes / 64u));
    const size_t hb = size_t(cfg->pool_segments) * 8, eb = size_t(cfg->pool_segments) * cap * 4;
    // (no room beside a pool sized to the HBM: the engine runs without it, the decode scans)
    if (hipMalloc(&p, hb + eb) == hipSuccess) {
      e->side_alloc = p;
      HIPCHK(hipMemset(p, 0, hb));  // life 0: every segment's first chunk starts its list
      e->side = clg::SideCar{static_cast<uint64_t*>(p), reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(p) + hb),
                             e->pool, pool_bytes, cfg->segment_bytes, cap};
    } else {
      (void)hipGetLastError();  // (the failed allocation is not the engine's error)
    }
  }
  e->ifl_C = cfg->ifl_segment_bytes ? cfg->ifl_segment_bytes : 32768u;
  const uint32_t ifl_n = cfg->ifl_pool_segments ? cfg->ifl_pool_segments : 4096u;
  if (e->ifl_C % 16) return fail(CLG_E_INVALID_ARG, "ifl_segment_bytes must be a multiple of 16");
  e->cfg.ifl_segment_bytes = e->ifl_C;
  e->cfg.ifl_pool_segments = ifl_n;
  HIPCHK(hipMalloc(&p, size_t(e->ifl_C) * ifl_n + 2 * kPoolGuard));
  e->ifl_alloc = p;
  e->ifl_pool = static_cast<uint8_t*>(p) + kPoolGuard;
  e->ifl_free.resize(ifl_n);
  for (uint32_t i = 0; i < ifl_n; ++i) e->ifl_free[i] = ifl_n - 1 - i;
  e->jobs.emplace_back();  // job 0: the default job
  e->jobs[0].open = true;
  e->jobs[0].depth = cfg->sharing_depth;
  *out = e.release();
  return CLG_OK;
}

void clg_engine_destroy(clg_engine* e) {
  if (!e) return;
  hipSetDevice(e->cfg.device);
  e->settle();  // a pending asynchronous decode: its events go back to the pool
  hipStreamSynchronize(e->stream);
  e->gwait();
  for (auto& t : e->timings) {
    hipEventDestroy(t.a);
    hipEventDestroy(t.b);
  }
  for (auto ev : e->ev_pool) hipEventDestroy(ev);
  for (auto ev : e->zdone)
    if (ev) hipEventDestroy(ev);
  if (e->pool_alloc) hipFree(e->pool_alloc);
  if (e->side_alloc) hipFree(e->side_alloc);
  if (e->ifl_alloc) hipFree(e->ifl_alloc);
  hipStreamDestroy(e->stream);
  if (e->gstream) hipStreamDestroy(e->gstream);
  if (e->gready) hipEventDestroy(e->gready);
  for (auto ev : e->gdone)
    if (ev) hipEventDestroy(ev);
  delete e;
}

void* clg_engine_stream(clg_engine* e) { return e ? (void*)e->stream : nullptr; }
void* clg_gather_stream(clg_engine* e) { return e ? (void*)e->gstream : nullptr; }

int clg_sync(clg_engine* e) {
  ENGINE_GUARD(e);
  CHK(e->flush());
  return e->sync();
}

int clg_pool_stats(clg_engine* e, uint32_t* used, uint32_t* free_segments) {
  ENGINE_GUARD(e);
  *free_segments = uint32_t(e->free_segs.size());
  *used = e->cfg.pool_segments - *free_segments;
  return CLG_OK;
}

int clg_job_open(clg_engine* e, uint64_t job_lo, uint64_t job_hi, int32_t sharing_depth, uint32_t* job) {
  ENGINE_GUARD(e);
  if (!job) return fail(CLG_E_INVALID_ARG, "null argument");
  for (uint32_t j = 0; j < e->jobs.size(); ++j)
    if (e->jobs[j].open && e->jobs[j].lo == job_lo && e->jobs[j].hi == job_hi && j != 0)
      return fail(CLG_E_INVALID_ARG, "job already open");
  Job nj;
  nj.open = true;
  nj.lo = job_lo;
  nj.hi = job_hi;
  nj.depth = sharing_depth;
  for (uint32_t j = 1; j < e->jobs.size(); ++j)
    if (!e->jobs[j].open) {
      e->jobs[j] = nj;
      *job = j;
      return CLG_OK;
    }
  e->jobs.push_back(nj);
  *job = uint32_t(e->jobs.size() - 1);
  return CLG_OK;
}

int clg_job_close(clg_engine* e, uint32_t job) {
  ENGINE_GUARD(e);
  if (job >= e->jobs.size() || !e->jobs[job].open) return fail(CLG_E_NO_LOG, "unknown job %u", job);
  for (uint32_t h = 0; h < e->logs.size(); ++h)
    if (e->logs[h].open && e->logs[h].job == job) CHK(clg_log_close(e, h));
  if (job != 0) e->jobs[job] = Job();
  else e->jobs[0].latest_cp = 0;
  return CLG_OK;
}

int clg_ifl_pool_stats(clg_engine* e, uint32_t* used, uint32_t* free_segments) {
  ENGINE_GUARD(e);
  *free_segments = uint32_t(e->ifl_free.size());
  *used = e->cfg.ifl_pool_segments - *free_segments;
  return CLG_OK;
}

int clg_log_open(clg_engine* e, uint32_t job, const clg_causal_log_id* id, uint32_t* handle) {
  ENGINE_GUARD(e);
  if (!id || !handle) return fail(CLG_E_INVALID_ARG, "null argument");
  if (job >= e->jobs.size() || !e->jobs[job].open) return fail(CLG_E_NO_LOG, "unknown job %u", job);
  const IdKey k = key_of(job, *id);
  if (e->by_id.count(k)) return fail(CLG_E_INVALID_ARG, "log already open");
  Log l;
  l.id = *id;
  l.job = job;
  l.depth = e->jobs[job].depth;
  l.open = true;
  if (e->free_segs.empty()) return fail(CLG_E_NOSPACE, "segment pool exhausted");
  l.segs.push_back(e->free_segs.back());  // ctor addComponent() :102
  ++e->seg_life[e->free_segs.back()];
  e->free_segs.pop_back();
  const uint32_t h = uint32_t(e->logs.size());  // handles are never reused: a stale one is CLG_E_NO_LOG
  e->logs.push_back(std::move(l));
  e->by_id[k] = h;
  *handle = h;
  return CLG_OK;
}

int clg_log_close(clg_engine* e, uint32_t h) {
  ENGINE_GUARD(e);
  Log* l;
  CHK(e->get_log(h, &l));
  CHK(e->sync());
  for (uint32_t s : l->segs) e->free_segs.push_back(s);
  e->by_id.erase(key_of(l->job, l->id));
  *l = Log();
  return CLG_OK;
}

int clg_log_find(clg_engine* e, uint32_t job, const clg_causal_log_id* id, uint32_t* handle) {
  ENGINE_GUARD(e);
  auto it = e->by_id.find(key_of(job, *id));
  if (it == e->by_id.end()) return fail(CLG_E_NO_LOG, "log not found");
  *handle = it->second;
  return CLG_OK;
}

int clg_log_get_id(clg_engine* e, uint32_t h, clg_causal_log_id* id, uint32_t* job) {
  ENGINE_GUARD(e);
  Log* l;
  CHK(e->get_log(h, &l));
  if (id) *id = l->id;
  if (job) *job = l->job;
  return CLG_OK;
}

int clg_append(clg_engine* e, uint32_t log, int64_t epoch, const uint8_t* rec, uint32_t n) {
  bool spill;
  {
    LOG_GUARD(e, log);
    CHK(e->append(log, epoch, rec, n));
    spill = e->over_stage_limit(log);
  }
  if (!spill) return CLG_OK;
  ENGINE_GUARD(e);  // bounded write-behind: this log's staged bytes go to HBM now
  return e->flush();
}

int clg_append_batch(clg_engine* e, const uint32_t* log, const int64_t* epoch, const uint64_t* off,
                     const uint32_t* len, uint32_t n, const uint8_t* bytes) {
  ENGINE_GUARD(e);
  for (uint32_t i = 0; i < n; ++i) CHK(e->append(log[i], epoch[i], bytes + off[i], len[i]));
  return CLG_OK;
}

int clg_upstream_delta(clg_engine* e, uint32_t log, int64_t epoch, int32_t off, const uint8_t* d, uint32_t n) {
  bool spill;
  {
    LOG_GUARD(e, log);
    CHK(e->upstream(log, epoch, off, d, n));
    spill = e->over_stage_limit(log);
  }
  if (!spill) return CLG_OK;
  ENGINE_GUARD(e);
  return e->flush();
}

int clg_log_length(clg_engine* e, uint32_t h, int32_t* out) {  // :180-192
  LOG_GUARD(e, h);
  Log* l;
  CHK(e->get_log(h, &l));
  *out = l->epochs.empty() ? l->writer : l->writer - l->epochs.begin()->offset;
  return CLG_OK;
}

int clg_log_length_batch(clg_engine* e, const uint32_t* log, uint32_t n, int32_t* out, uint64_t* total) {
  ENGINE_GUARD(e);
  if (n && !log) return fail(CLG_E_INVALID_ARG, "null argument");
  uint64_t t = 0;
  for (uint32_t i = 0; i < n; ++i) {
    Log* l;
    CHK(e->get_log(log[i], &l));
    const int32_t v = l->epochs.empty() ? l->writer : l->writer - l->epochs.begin()->offset;
    if (out) out[i] = v;
    t += uint64_t(v);
  }
  if (total) *total = t;
  return CLG_OK;
}

int clg_has_delta(clg_engine* e, uint32_t log, clg_channel_id c, int64_t epoch, int32_t* out) {
  LOG_GUARD(e, log);
  return e->has_delta(log, ChKey{c.lo, c.hi}, epoch, out);
}

int clg_offset_from_epoch(clg_engine* e, uint32_t log, clg_channel_id c, int32_t* out) {
  LOG_GUARD(e, log);
  return e->offset_from_epoch(log, ChKey{c.lo, c.hi}, out);
}

int clg_get_delta(clg_engine* e, uint32_t log, clg_channel_id c, int64_t epoch, void* out, uint32_t cap,
                  uint32_t kind, uint32_t* n) {
  {  // the host tail holds it: no GPU, only this log's stripe
    LOG_GUARD(e, log);
    const int r = e->get_delta(log, ChKey{c.lo, c.hi}, epoch, out, cap, kind, n, true);
    if (r != clg_engine::kNeedGpu) return r;
  }
  ENGINE_GUARD(e);
  return e->get_delta(log, ChKey{c.lo, c.hi}, epoch, out, cap, kind, n);
}

int clg_get_determinants(clg_engine* e, uint32_t log, int64_t start_epoch, void* out, uint32_t cap, uint32_t kind,
                         uint32_t* n) {
  {
    LOG_GUARD(e, log);
    const int r = e->get_determinants(log, start_epoch, out, cap, kind, n, true);
    if (r != clg_engine::kNeedGpu) return r;
  }
  ENGINE_GUARD(e);
  return e->get_determinants(log, start_epoch, out, cap, kind, n);
}

int clg_notify_checkpoint_complete(clg_engine* e, uint32_t h, int64_t cp) {
  ENGINE_GUARD(e);
  Log* l;
  CHK(e->get_log(h, &l));
  CHK(e->flush());
  return e->checkpoint_complete(*l, cp);
}

int clg_unregister_consumer(clg_engine* e, uint32_t h, clg_channel_id c) {
  LOG_GUARD(e, h);
  Log* l;
  CHK(e->get_log(h, &l));
  l->consumers.erase(ChKey{c.lo, c.hi});
  return CLG_OK;
}

int clg_log_get_state(clg_engine* e, uint32_t h, clg_log_state* st, int64_t* ids, int32_t* offs, int32_t cap) {
  ENGINE_GUARD(e);
  Log* l;
  CHK(e->get_log(h, &l));
  st->writer = l->writer;
  st->capacity = e->capacity(*l);
  st->n_components = int32_t(l->segs.size());
  st->n_epochs = int32_t(l->epochs.size());
  int32_t i = 0;
  for (auto& ep : l->epochs) {
    if (i < cap) {
      if (ids) ids[i] = ep.id;
      if (offs) offs[i] = ep.offset;
    }
    ++i;
  }
  return i > cap && (ids || offs) ? fail(CLG_E_CAPACITY, "%d epochs", i) : CLG_OK;
}

int clg_consumer_state(clg_engine* e, uint32_t h, clg_channel_id c, int32_t* exists, int64_t* epoch, int32_t* offset) {
  ENGINE_GUARD(e);
  Log* l;
  CHK(e->get_log(h, &l));
  auto ci = l->consumers.find(ChKey{c.lo, c.hi});
  *exists = ci != l->consumers.end();
  if (*exists) {
    *epoch = ci->second.es->id;
    *offset = ci->second.offset;
  }
  return CLG_OK;
}

int clg_log_read_phys(clg_engine* e, uint32_t h, int32_t phys, uint32_t n, uint8_t* host_out) {
  ENGINE_GUARD(e);
  Log* l;
  CHK(e->get_log(h, &l));
  if (phys < 0 || int64_t(phys) + n > e->capacity(*l)) return fail(CLG_E_STATE, "range outside log");
  CHK(e->flush());
  std::vector<clg::GatherPiece> pieces;
  e->add_pieces(*l, phys, int32_t(n), 0, pieces);
  return e->run_gather(pieces, n, host_out, CLG_MEM_HOST);
}

// getDeterminants(startEpoch) of many logs (respondToDeterminantRequest's copies for a
// replay-prep merge, JobCausalLogImpl.java:188-204): the ranges on the host, the bytes by
// one device gather, back to back in request order.
int clg_get_determinants_batch(clg_engine* e, const uint32_t* log, const int64_t* start_epoch, uint32_t n, void* out,
                               uint64_t cap, uint32_t out_kind, uint64_t* out_off, uint32_t* len, uint64_t* total) {
  ENGINE_GUARD(e);
  if (n && (!log || !start_epoch || !len)) return fail(CLG_E_INVALID_ARG, "null argument");
  std::vector<clg::SegSpan> runs;
  std::vector<uint32_t> segtab;
  uint32_t n_pieces = 0;
  const uint32_t C = e->C();
  uint64_t dst = 0;
  if (!out) {  // sizes only (the merge measures every copy first): no gather plan
    for (uint32_t i = 0; i < n; ++i) {
      Log* l;
      CHK(e->get_log(log[i], &l));
      int32_t s = 0, nb = 0;
      if (l->depth != 0) CHK(e->determinants_range(*l, start_epoch[i], &s, &nb));
      len[i] = uint32_t(nb);
      if (out_off) out_off[i] = dst;
      dst += uint64_t(nb);
    }
    if (total) *total = dst;
    return CLG_OK;
  }
  runs.reserve(n);
  // each log's segment indices once in segtab: the log's place there, by handle (a hash map
  // took 0.1 ms for config 5's 2 064 logs)
  std::vector<uint64_t>& tab_at = e->tab_at;
  if (tab_at.size() < e->logs.size()) tab_at.resize(e->logs.size(), UINT64_MAX);
  std::vector<uint32_t> touched;
  touched.reserve(n);
  int st = CLG_OK;
  for (uint32_t i = 0; i < n && st == CLG_OK; ++i) {
    Log* l;
    if ((st = e->get_log(log[i], &l)) != CLG_OK) break;
    int32_t s = 0, nb = 0;
    if (l->depth != 0 && (st = e->determinants_range(*l, start_epoch[i], &s, &nb)) != CLG_OK) break;
    len[i] = uint32_t(nb);
    if (out_off) out_off[i] = dst;
    if (nb > 0) {
      uint64_t& at = tab_at[log[i]];
      if (at == UINT64_MAX) {
        at = segtab.size();
        touched.push_back(log[i]);
        segtab.insert(segtab.end(), l->segs.begin(), l->segs.end());
      }
      runs.push_back(clg::SegSpan{at, uint32_t(s), uint32_t(nb), dst, n_pieces, 0});
      n_pieces += uint32_t(s + nb - 1) / C - uint32_t(s) / C + 1;
    }
    dst += uint64_t(nb);
  }
  for (uint32_t h : touched) tab_at[h] = UINT64_MAX;
  if (st != CLG_OK) return st;
  if (total) *total = dst;
  if (dst > cap) return fail(CLG_E_CAPACITY, "getDeterminants batch needs %llu bytes", (unsigned long long)dst);
  CHK(e->flush());
  return e->run_gather_runs(runs, segtab, n_pieces, dst, out, out_kind);
}

int clg_slice_batch(clg_engine* e, const clg_slice_req* reqs, uint32_t n, clg_slice_res* res, void* out, uint64_t cap,
                    uint32_t out_kind, uint64_t* total) {
  ENGINE_GUARD_KEEP(e);
  if (!(out_kind == CLG_MEM_DEVICE && (e->cfg.flags & CLG_F_ASYNC_SLICE))) e->settle();
  if (n && (!reqs || !res)) return fail(CLG_E_INVALID_ARG, "null argument");
  CHK(e->flush());
  std::vector<clg::SegSpan> runs;
  std::vector<uint32_t> segtab;
  std::unordered_map<uint32_t, uint64_t> tab_of;  // log -> its segment indices in segtab
  runs.reserve(n);
  uint32_t n_pieces = 0;
  const uint32_t C = e->C();
  uint64_t dst = 0;
  for (uint32_t i = 0; i < n; ++i) {
    clg_slice_res& r = res[i];
    r = clg_slice_res{CLG_OK, 0, 0, 0, dst};
    const ChKey k{reqs[i].consumer.lo, reqs[i].consumer.hi};
    int32_t has = 0;
    int st = e->has_delta(reqs[i].log, k, reqs[i].epoch, &has);
    if (st != CLG_OK) {
      r.status = st;
      continue;
    }
    r.has_delta = has;
    if (!has) continue;
    st = e->offset_from_epoch(reqs[i].log, k, &r.offset_from_epoch);  // Abstract...:199 before :201
    if (st != CLG_OK) {
      r.status = st;
      continue;
    }
    int32_t phys, nb;
    st = e->take_delta(reqs[i].log, k, reqs[i].epoch, &phys, &nb);
    if (st != CLG_OK) {
      r.status = st;
      continue;
    }
    if (dst + uint64_t(nb) > cap) {
      // undo the consumer advance so the request can be retried with a bigger buffer
      e->logs[reqs[i].log].consumers[k].offset -= nb;
      r.status = CLG_E_CAPACITY;
      continue;
    }
    r.len = nb;
    if (nb > 0) {
      auto ti = tab_of.find(reqs[i].log);
      if (ti == tab_of.end()) {
        const auto& segs = e->logs[reqs[i].log].segs;
        ti = tab_of.emplace(reqs[i].log, segtab.size()).first;
        segtab.insert(segtab.end(), segs.begin(), segs.end());
      }
      runs.push_back(clg::SegSpan{ti->second, uint32_t(phys), uint32_t(nb), dst, n_pieces, 0});
      n_pieces += uint32_t(phys + nb - 1) / C - uint32_t(phys) / C + 1;
    }
    dst += uint64_t(nb);
  }
  if (total) *total = dst;
  return e->run_gather_runs(runs, segtab, n_pieces, dst, out, out_kind);
}

int clg_consumer_seek(clg_engine* e, uint32_t h, clg_channel_id c, int64_t epoch, int32_t offset) {
  ENGINE_GUARD_KEEP(e);
  Log* l;
  CHK(e->get_log(h, &l));
  auto it = l->epochs.find(epoch);
  if (it == l->epochs.end()) return fail(CLG_E_STATE, "epoch %lld not in log", (long long)epoch);
  l->consumers[ChKey{c.lo, c.hi}] = Consumer{EpochMap::ref(*it), offset};
  return CLG_OK;
}

int clg_upstream_delta_batch(clg_engine* e, clg_delta_req* reqs, uint32_t n, const uint8_t* bytes, uint32_t in_kind) {
  ENGINE_GUARD_KEEP(e);
  clg_engine::HostTimer ht(e, "host_abi_upstream");  // (CLONOS_HOST_PROF: lock held to here; settle and the call)
  e->settle();
  if (n && (!reqs || !bytes)) return fail(CLG_E_INVALID_ARG, "null argument");
  return e->upstream_batch(reqs, n, bytes, in_kind);
}

int clg_consumer_seek_batch(clg_engine* e, const clg_slice_req* reqs, const int32_t* offsets, uint32_t n) {
  ENGINE_GUARD_KEEP(e);
  if (n && (!reqs || !offsets)) return fail(CLG_E_INVALID_ARG, "null argument");
  for (uint32_t i = 0; i < n; ++i) {
    Log* l;
    CHK(e->get_log(reqs[i].log, &l));
    auto it = l->epochs.find(reqs[i].epoch);
    if (it == l->epochs.end()) return fail(CLG_E_STATE, "epoch %lld not in log", (long long)reqs[i].epoch);
    l->consumers[ChKey{reqs[i].consumer.lo, reqs[i].consumer.hi}] = Consumer{EpochMap::ref(*it), offsets[i]};
  }
  return CLG_OK;
}

int clg_truncate_all(clg_engine* e, uint32_t job, int64_t cp, int32_t* applied) {  // JobCausalLogImpl :230-246
  // Beside queued asynchronous decodes whose ranges start at or above cp (config 4's step:
  // the host truncates while the GPU decodes the new epoch): the truncation only drops bytes
  // below cp, so the queued kernels read nothing it frees -- its segments return to the pool
  // once those decodes complete.  Otherwise (a decode from below cp, appends not yet flushed)
  // the queued decodes complete first.
  ENGINE_GUARD_KEEP(e);
  bool defer = false;
  if (e->any_active()) {
    int64_t mn = INT64_MAX;
    for (const auto& d : e->pq)
      if (d.active) mn = std::min(mn, d.min_epoch);
    const bool dirty = !e->dirty.empty();  // (appends not yet flushed: the flush below writes segments)
    if (cp > mn || dirty) CHK(e->settle());
    else defer = true;
  } else {
    e->release_later();
  }
  if (applied) *applied = 0;
  if (job >= e->jobs.size() || !e->jobs[job].open) return fail(CLG_E_NO_LOG, "unknown job %u", job);
  Job& j = e->jobs[job];
  if (j.latest_cp >= cp) return CLG_OK;  // the CAS: only a newer checkpoint fans out
  j.latest_cp = cp;
  ++e->rebase_gen;
  std::vector<uint32_t>& to = defer ? e->free_later : e->free_segs;
  CHK(e->flush());
  clg_engine::HostTimer ht(e, "host_truncate_all");
  if (e->logs.size() >= clg_engine::kParallelLogs) {
    // 66 k logs (config 4): the host threads take parts of the log table.  A log whose epochs
    // below cp hold shared EpochStart objects (a consumer refers to them) is left to this
    // thread (their blocks go back to a per-thread free list); each part collects its freed
    // segments, which join the pool after.
    WorkPool* wp = e->workers();
    const unsigned P = wp->size();
    const size_t nl = e->logs.size(), per = (nl + P - 1) / P;
    std::vector<std::vector<uint32_t>> freed(P), later(P);
    std::vector<int> st(P, CLG_OK);
    wp->run([&](unsigned k, unsigned) {
      const size_t i1 = std::min(nl, (k + 1) * per);
      for (size_t i = k * per; i < i1; ++i) {
        if (i + 8 < i1) {  // the Log objects ahead (per-log work is bound by their cache misses)
          const char* q = reinterpret_cast<const char*>(&e->logs[i + 8]);
          for (size_t b = 0; b < sizeof(Log); b += 64) __builtin_prefetch(q + b, 1);
        }
        Log& l = e->logs[i];
        if (!l.open || l.job != job) continue;
        bool shared = false;
        for (const EpochEnt& x : l.epochs) {
          if (x.id >= cp) break;
          shared |= x.shared != nullptr;
        }
        if (shared) {
          later[k].push_back(uint32_t(i));
          continue;
        }
        if ((st[k] = e->checkpoint_complete(l, cp, freed[k])) != CLG_OK) return;
      }
    });
    ht.lap("host_trunc_pool");
    for (unsigned k = 0; k < P; ++k) to.insert(to.end(), freed[k].begin(), freed[k].end());
    for (unsigned k = 0; k < P; ++k)
      if (st[k] != CLG_OK) return fail(st[k], "checkpoint completion failed on a log (state outside its bounds)");
    size_t n_later = 0;
    for (unsigned k = 0; k < P; ++k) {
      n_later += later[k].size();
      for (uint32_t i : later[k]) CHK(e->checkpoint_complete(e->logs[i], cp, to));
    }
    ht.lap(n_later ? "host_trunc_later" : "host_trunc_free");
  } else {
    for (auto& l : e->logs)
      if (l.open && l.job == job) CHK(e->checkpoint_complete(l, cp, to));
  }
  if (applied) *applied = 1;
  return CLG_OK;
}

int clg_decode_host(clg_engine* e, const uint8_t* bytes, const uint64_t* span_off, const uint64_t* span_len, uint32_t n,
                    clg_decoded* out, uint64_t* span_rec_base) {
  ENGINE_GUARD(e);
  if (!out || (n && (!span_off || !span_len))) return fail(CLG_E_INVALID_ARG, "null argument");
  uint64_t lo = UINT64_MAX, hi = 0, total = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (span_len[i] == 0) continue;
    lo = std::min(lo, span_off[i]);
    hi = std::max(hi, span_off[i] + span_len[i]);
    total += span_len[i];
  }
  if (lo == UINT64_MAX) lo = hi = 0;
  CHK(e->d_stage.ensure(hi - lo + 16));
  CHK(e->h_stage.ensure(hi - lo + 16));
  if (hi > lo) {
    memcpy(e->h_stage.p, bytes + lo, hi - lo);
    HIPCHK(hipMemcpyAsync(e->d_stage.p, e->h_stage.p, hi - lo, hipMemcpyHostToDevice, e->stream));
  }
  auto build = [&](clg_engine::DecodePlan& p, uint32_t T) {
    for (uint32_t i = 0; i < n; ++i)
      e->plan_host_span(p, e->d_stage.as<uint8_t>() + (span_len[i] ? span_off[i] - lo : 0), span_len[i], i, T);
  };
  return e->decode(build, total, out, span_rec_base);
}

int clg_decode_logs(clg_engine* e, const uint32_t* log, const int64_t* start_epoch, uint32_t n, clg_decoded* out,
                    uint64_t* span_rec_base) {
  ENGINE_GUARD(e);
  if (!out || (n && (!log || !start_epoch))) return fail(CLG_E_INVALID_ARG, "null argument");
  CHK(e->flush());
  std::vector<int32_t>& st = e->zst;
  std::vector<int32_t>& nb = e->znb;
  st.assign(n, 0);
  nb.assign(n, 0);
  uint64_t total = 0;
  // the ranges and the fast decode's plan in one pass over the logs (per-log work of a
  // 66 k-log batch is bound by the cache misses on the log records)
  clg_engine::DecodePlan& pf = e->zplan;
  pf.reset();
  if (e->fused_decode) {
    pf.spans.reserve(n);
    pf.runs.reserve(n);
  }
  {
    clg_engine::HostTimer ht(e, "host_decode_plan");
    if (!(n >= clg_engine::kParallelLogs && e->fused_decode && e->plan_parallel(pf, log, start_epoch, n, &total, 0))) {
      total = 0;
      pf.reset();
      for (uint32_t i = 0; i < n; ++i) {
        Log* l;
        CHK(e->get_log(log[i], &l));
        if (l->depth != 0) CHK(e->determinants_range(*l, start_epoch[i], &st[i], &nb[i]));
        total += uint64_t(nb[i]);
        if (e->fused_decode) e->plan_log_span(pf, *l, st[i], nb[i], i, clg::kZTile);
      }
    }
  }
  auto build = [&](clg_engine::DecodePlan& p, uint32_t T) {  // re-plans (fallbacks)
    p.spans.reserve(n);
    p.runs.reserve(n);
    for (uint32_t i = 0; i < n; ++i) e->plan_log_span(p, e->logs[log[i]], st[i], nb[i], i, T);
  };
  return e->decode(build, total, out, span_rec_base, e->fused_decode ? &pf : nullptr);
}

int clg_decode_logs_async(clg_engine* e, const uint32_t* log, const int64_t* start_epoch, uint32_t n,
                          clg_decoded* out, uint64_t* span_rec_base) {
  ENGINE_GUARD_KEEP(e);  // (the queued decodes stay queued)
  if (!out || (n && (!log || !start_epoch))) return fail(CLG_E_INVALID_ARG, "null argument");
  // every queued decode's status is kept for its wait
  if (e->pq.size() >= CLG_DECODE_MAX_INFLIGHT)
    return fail(CLG_E_STATE, "%d asynchronous decodes are not waited for (clg_decode_wait)", CLG_DECODE_MAX_INFLIGHT);
  CHK(e->flush());  // (stream-ordered after the queued decodes, past their ranges)
  std::vector<uint32_t> hs(log, log + n);
  std::vector<int32_t> st, nb;
  uint64_t total = 0;
  // many logs: the ranges and the fast plan on the host threads (clg_decode_logs' way), into
  // a recycled plan
  clg_engine::DecodePlan pf;
  if (!e->plan_pool.empty()) {
    pf = std::move(e->plan_pool.back());
    e->plan_pool.pop_back();
  }
  pf.reset();
  bool planned = false;
  if (n >= clg_engine::kParallelLogs && e->fused_decode) {
    clg_engine::HostTimer ht(e, "host_decode_plan");
    e->zst.assign(n, 0);  // (plan_parallel's ranges go here)
    e->znb.assign(n, 0);
    const uint32_t fs = e->free_slot();  // (the plan is staged for that slot)
    planned = e->plan_parallel(pf, log, start_epoch, n, &total, fs < clg_engine::kSlots ? int(fs) : -1);
  }
  if (planned) {
    st.assign(e->zst.begin(), e->zst.begin() + n);
    nb.assign(e->znb.begin(), e->znb.begin() + n);
  } else {
    total = 0;
    st.assign(n, 0);
    nb.assign(n, 0);
    for (uint32_t i = 0; i < n; ++i) {
      Log* l;
      CHK(e->get_log(log[i], &l));
      if (l->depth != 0) CHK(e->determinants_range(*l, start_epoch[i], &st[i], &nb[i]));
      total += uint64_t(nb[i]);
    }
  }
  // by value: the robust fallback may re-plan when the decode is settled.  Only a checkpoint
  // truncation at or below every start epoch runs before that (clg_truncate_all settles
  // otherwise); it rebases the logs, and a re-plan after it looks the ranges up again (the
  // same bytes at their new offsets)
  int64_t mn = INT64_MAX;
  for (uint32_t i = 0; i < n; ++i) mn = std::min(mn, start_epoch[i]);
  std::vector<int64_t> eps(start_epoch, start_epoch + n);
  auto build = [e, hs = std::move(hs), st = std::move(st), nb = std::move(nb), eps = std::move(eps),
                gen = e->rebase_gen](clg_engine::DecodePlan& p, uint32_t T) {
    p.spans.reserve(hs.size());
    p.runs.reserve(hs.size());
    for (uint32_t i = 0; i < uint32_t(hs.size()); ++i) {
      int32_t s = st[i], b = nb[i];
      const Log& l = e->logs[hs[i]];
      if (gen != e->rebase_gen && l.depth != 0 && e->determinants_range(l, eps[i], &s, &b) != CLG_OK) {
        p.status = CLG_E_STATE;  // (the settle-on-truncate rule makes this unreachable)
        s = b = 0;
      }
      e->plan_log_span(p, l, s, b, i, T);
    }
  };
  e->q_min_epoch = n ? mn : INT64_MAX;
  const int rc = e->decode_async(build, total, out, span_rec_base, planned ? &pf : nullptr);
  e->q_min_epoch = INT64_MIN;
  if (pf.spans.capacity() && e->plan_pool.size() < clg_engine::kSlots) {  // (not queued: the plan back)
    pf.reset();
    e->plan_pool.push_back(std::move(pf));
  }
  return rc;
}

int clg_decode_wait(clg_engine* e) {
  ENGINE_GUARD_KEEP(e);
  std::string err;
  const int st = e->wait_oldest(&err);
  return st == CLG_OK ? CLG_OK : fail(st, "%s", err.c_str());
}

int clg_replay_prep(clg_engine* e, const uint64_t* key, const uint8_t* bytes, const uint64_t* off, const uint64_t* len,
                    uint32_t n, uint32_t* winner, uint32_t* n_keys, clg_decoded* out, uint64_t* span_rec_base) {
  ENGINE_GUARD(e);
  if (n && (!key || !off || !len || !winner || !n_keys)) return fail(CLG_E_INVALID_ARG, "null argument");
  // DeterminantResponseEvent.merge :136-146: per CausalLogID keep the longer buffer,
  // ties -> the later one (v2).  Keys keep first-appearance order.
  std::unordered_map<uint64_t, uint32_t> best;
  std::vector<uint64_t> order;
  for (uint32_t i = 0; i < n; ++i) {
    auto it = best.find(key[i]);
    if (it == best.end()) {
      best.emplace(key[i], i);
      order.push_back(key[i]);
    } else if (!(len[it->second] > len[i])) {
      it->second = i;
    }
  }
  *n_keys = uint32_t(order.size());
  std::vector<uint64_t> so(order.size()), sl(order.size());
  for (size_t k = 0; k < order.size(); ++k) {
    winner[k] = best[order[k]];
    so[k] = off[winner[k]];
    sl[k] = len[winner[k]];
  }
  if (!out) return CLG_OK;
  return clg_decode_host(e, bytes, so.data(), sl.data(), uint32_t(order.size()), out, span_rec_base);
}

// ReplayingState (:58-66, :108-130) + SubpartitionRecoveryThread.run (:157-188) +
// LogReplayerImpl (:51-158), batched over failed vertices.  Main logs go through the
// batched decode; subpartition recovery buffers through k_bufsizes (5-byte BufferBuilt
// records, no chain walk).  All inputs are staged to HBM in one copy.
static int replay_prepare(clg_engine* e, const clg_replay_vertex* v, uint32_t n, clg_replay_out* out, bool dev_in);
int clg_replay_prepare(clg_engine* e, const clg_replay_vertex* v, uint32_t n, clg_replay_out* out) {
  return replay_prepare(e, v, n, out, false);
}
int clg_replay_prepare_device(clg_engine* e, const clg_replay_vertex* v, uint32_t n, clg_replay_out* out) {
  return replay_prepare(e, v, n, out, true);
}
// Pinned read-back of replay-prep's subpartition results: sizes, then count, err_off (8 B
// each), status, err_tag (4 B each) per subpartition, as they lie on the device.
static size_t o_rout_cnt(uint64_t n_sizes) { return (size_t(n_sizes) * 4 + 15) & ~size_t(15); }
static size_t o_rout_end(uint32_t ns, uint64_t n_sizes) { return o_rout_cnt(n_sizes) + size_t(ns) * 24 + 64; }
static int replay_prepare(clg_engine* e, const clg_replay_vertex* v, uint32_t n, clg_replay_out* out, bool dev_in) {
  ENGINE_GUARD(e);
  if (!out || !out->main || !out->main_rec_base || (n && !v)) return fail(CLG_E_INVALID_ARG, "null argument");
  clg_engine::HostTimer lap(e, "host_replay_rest");  // (laps below: the sections)
  struct Piece {
    const uint8_t* p;
    uint64_t len;
  };
  std::vector<Piece> mains(n), subs;
  // the accumulated map's entries by CausalLogID (equals :128-149), per vertex: an
  // open-addressing table, O(entries + subpartitions) (a std::map took 0.16 ms for config 5's
  // 16 vertices x 129 entries)
  std::vector<IdKey> keys;
  std::vector<uint32_t> slot;  // entry index + 1 (0: empty)
  uint64_t mask = 0;
  const clg_response* indexed = nullptr;
  auto hkey = [](const IdKey& k) {  // splitmix64 finaliser over the fields (a vertex's keys differ in sub only)
    auto mix = [](uint64_t z) {
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      return z ^ (z >> 31);
    };
    return mix(mix(uint64_t(uint16_t(k.v)) | uint64_t(k.main) << 16 | (uint64_t(uint8_t(k.sub)) << 24 ^ uint64_t(k.lo))) ^
               uint64_t(k.hi));
  };
  auto same = [](const IdKey& a, const IdKey& b) {
    return a.v == b.v && a.main == b.main && a.sub == b.sub && a.lo == b.lo && a.hi == b.hi;
  };
  auto lookup = [&](const clg_response* r, const clg_causal_log_id& id) -> Piece {
    if (!r) return Piece{nullptr, 0};
    if (r != indexed) {
      uint64_t size = 16;
      while (size < 2ull * r->n) size <<= 1;
      mask = size - 1;
      slot.assign(size, 0u);
      keys.resize(r->n);
      for (uint32_t i = 0; i < r->n; ++i) {
        keys[i] = key_of(0, r->entries[i].id);
        uint64_t h = hkey(keys[i]) & mask;
        while (slot[h] && !same(keys[slot[h] - 1], keys[i])) h = (h + 1) & mask;
        if (!slot[h]) slot[h] = i + 1;  // the first of equal keys
      }
      indexed = r;
    }
    const IdKey k = key_of(0, id);
    for (uint64_t h = hkey(k) & mask; slot[h]; h = (h + 1) & mask)
      if (same(keys[slot[h] - 1], k)) return Piece{r->entries[slot[h] - 1].bytes, r->entries[slot[h] - 1].len};
    return Piece{nullptr, 0};
  };
  subs.reserve(1024);
  for (uint32_t i = 0; i < n; ++i) {
    if (v[i].n_subpartitions && !v[i].subpartitions) return fail(CLG_E_INVALID_ARG, "null subpartition table");
    clg_causal_log_id mid{};
    mid.vertex_id = v[i].vertex_id;
    mid.is_main = 1;
    mains[i] = lookup(v[i].acc, mid);
    for (uint32_t j = 0; j < v[i].n_subpartitions; ++j) {
      clg_causal_log_id sid = v[i].subpartitions[j];
      sid.vertex_id = v[i].vertex_id;  // id.replace(lower, upper, index) keeps the vertex (:114, :121)
      sid.is_main = 0;
      subs.push_back(lookup(v[i].acc, sid));
    }
  }
  lap.lap("host_replay_index");
  const uint32_t ns = uint32_t(subs.size());
  if (ns && (!out->sizes_base || !out->sub_count || !out->sub_status || !out->sub_err_off || !out->sub_err_tag))
    return fail(CLG_E_INVALID_ARG, "null subpartition output");
  // sizes capacity: one slot per whole 5-byte record
  uint64_t n_sizes = 0;
  for (uint32_t j = 0; j < ns; ++j) {
    out->sizes_base[j] = n_sizes;
    n_sizes += subs[j].len / 5;
  }
  if (ns) out->sizes_base[ns] = n_sizes;
  if (n_sizes > out->sizes_cap || (n_sizes && !out->buffer_sizes))
    return fail(CLG_E_CAPACITY, "buffer_sizes needs %llu entries", (unsigned long long)n_sizes);
  // stage main logs then subpartition buffers (16-byte aligned pieces) in one copy
  std::vector<uint64_t> at(n + ns);
  uint64_t total = 0, main_bytes = 0, sub_bytes = 0;
  for (uint32_t i = 0; i < n + ns; ++i) {
    const Piece& pc = i < n ? mains[i] : subs[i - n];
    at[i] = total;
    total += (pc.len + 15) & ~uint64_t(15);
    (i < n ? main_bytes : sub_bytes) += pc.len;
  }
  CHK(e->d_stage.ensure(total + 16));
  if (dev_in) {  // the winners already in HBM (e.g. an RCCL receive buffer): one device gather
    std::vector<clg::GatherPiece> pieces;
    for (uint32_t i = 0; i < n + ns; ++i) {
      const Piece& pc = i < n ? mains[i] : subs[i - n];
      for (uint64_t o = 0; o < pc.len; o += 1u << 30)  // a piece's length is 32-bit
        pieces.push_back(clg::GatherPiece{pc.p + o, at[i] + o, uint32_t(std::min<uint64_t>(pc.len - o, 1u << 30)), 0});
    }
    // (no wait: the kernels below read the staged bytes on the same stream)
    CHK(e->run_gather(pieces, total, e->d_stage.p, CLG_MEM_DEVICE, "replay_stage", false));
  } else {
    CHK(e->h_stage.ensure(total + 16));
    for (uint32_t i = 0; i < n + ns; ++i) {
      const Piece& pc = i < n ? mains[i] : subs[i - n];
      if (pc.len) memcpy(e->h_stage.as<uint8_t>() + at[i], pc.p, pc.len);
    }
    if (total) HIPCHK(hipMemcpyAsync(e->d_stage.p, e->h_stage.p, total, hipMemcpyHostToDevice, e->stream));
  }
  lap.lap("host_replay_stage");
  const uint8_t* dst = e->d_stage.as<uint8_t>();
  // subpartition buffers first (their kernels only read the staged bytes)
  std::function<int(clg::JArena)> classify;
  const int32_t* d_sub_status = nullptr;
  if (ns) {
    std::vector<clg::BufSpan> bs(ns);
    std::vector<clg::BufChunk> bc;
    constexpr uint64_t kRecPerChunk = 256;
    for (uint32_t j = 0; j < ns; ++j) {
      bs[j] = clg::BufSpan{dst + at[n + j], subs[j].len, out->sizes_base[j]};
      const uint64_t nk = (subs[j].len + 4) / 5;  // records incl. a partial tail
      for (uint64_t k = 0; k < nk; k += kRecPerChunk)
        bc.push_back(clg::BufChunk{j, 0, k, std::min(nk, k + kRecPerChunk)});
    }
    const size_t o_spans = 0, o_chunks = (ns * sizeof(clg::BufSpan) + 15) & ~size_t(15);
    const size_t o_res = (o_chunks + bc.size() * sizeof(clg::BufChunk) + 15) & ~size_t(15);
    const size_t res_bytes = size_t(ns) * (8 + 8 + 4 + 8 + 4);  // first_bad, count, status, err_off, err_tag
    CHK(e->h_rmeta.ensure(o_res + res_bytes + 64));
    CHK(e->d_rmeta.ensure(o_res + res_bytes + 64));
    uint8_t* hm = e->h_rmeta.as<uint8_t>();
    memcpy(hm + o_spans, bs.data(), ns * sizeof(clg::BufSpan));
    memcpy(hm + o_chunks, bc.data(), bc.size() * sizeof(clg::BufChunk));
    HIPCHK(hipMemcpyAsync(e->d_rmeta.p, hm, o_res, hipMemcpyHostToDevice, e->stream));
    uint8_t* dm = e->d_rmeta.as<uint8_t>();
    uint64_t* d_first = reinterpret_cast<uint64_t*>(dm + o_res);
    uint64_t* d_count = d_first + ns;
    int64_t* d_eoff = reinterpret_cast<int64_t*>(d_count + ns);
    int32_t* d_status = reinterpret_cast<int32_t*>(d_eoff + ns);
    int32_t* d_etag = d_status + ns;
    HIPCHK(hipMemsetAsync(d_first, 0xFF, ns * 8, e->stream));
    CHK(e->d_rsizes.ensure(std::max<uint64_t>(1, n_sizes) * 4));
    const auto* d_spans = reinterpret_cast<const clg::BufSpan*>(dm + o_spans);
    CHK(e->timed("replay_bufsizes", sub_bytes + 4 * n_sizes, [&] {
      return clg::launch_bufsizes(reinterpret_cast<const clg::BufChunk*>(dm + o_chunks), uint32_t(bc.size()), d_spans,
                                  e->d_rsizes.as<int32_t>(), d_first, e->stream);
    }));
    clg::JArena jar;
    CHK(e->jarena_reset(&jar));
    CHK(clg::launch_bufsizes_classify(d_spans, ns, d_first, d_count, d_status, d_eoff, d_etag, jar, e->stream));
    CHK(e->jarena_clear_note(1));
    CHK(e->jarena_note(1));
    classify = [=](clg::JArena a) {
      return clg::launch_bufsizes_classify(d_spans, ns, d_first, d_count, d_status, d_eoff, d_etag, a, e->stream);
    };
    d_sub_status = d_status;
    // read back into pinned memory (asynchronous; into the caller's pageable arrays each copy
    // was a staged synchronous one), copied out after the decode's sync below
    CHK(e->h_rout.ensure(o_rout_end(ns, n_sizes)));
    uint8_t* hr = e->h_rout.as<uint8_t>();
    if (n_sizes) HIPCHK(hipMemcpyAsync(hr, e->d_rsizes.p, n_sizes * 4, hipMemcpyDeviceToHost, e->stream));
    // count, err_off, status, err_tag: adjacent on the device (d_first's block): one copy
    HIPCHK(hipMemcpyAsync(hr + o_rout_cnt(n_sizes), d_count, size_t(ns) * 24, hipMemcpyDeviceToHost, e->stream));
  }
  lap.lap("host_replay_sizes");
  // main logs: the batched decode (span i = vertex i)
  auto build = [&](clg_engine::DecodePlan& p, uint32_t T) {
    for (uint32_t i = 0; i < n; ++i) e->plan_host_span(p, dst + at[i], mains[i].len, i, T);
  };
  CHK(e->decode(build, main_bytes, out->main, out->main_rec_base));
  lap.lap("host_replay_decode");
  CHK(e->sync());
  // a Serializable walk in a subpartition buffer found the spill arena full: again, larger
  uint8_t* hr = e->h_rout.as<uint8_t>();
  const size_t oc = o_rout_cnt(n_sizes);
  while (ns && e->jarena_spilled(1)) {
    CHK(e->jarena_grow());
    clg::JArena jar;
    CHK(e->jarena_reset(&jar));
    CHK(classify(jar));
    CHK(e->jarena_note(1));
    HIPCHK(hipMemcpyAsync(hr + oc + size_t(ns) * 16, d_sub_status, size_t(ns) * 4, hipMemcpyDeviceToHost, e->stream));
    CHK(e->sync());
  }
  if (ns) {
    if (n_sizes) memcpy(out->buffer_sizes, hr, n_sizes * 4);
    memcpy(out->sub_count, hr + oc, size_t(ns) * 8);
    memcpy(out->sub_err_off, hr + oc + size_t(ns) * 8, size_t(ns) * 8);
    memcpy(out->sub_status, hr + oc + size_t(ns) * 16, size_t(ns) * 4);
    memcpy(out->sub_err_tag, hr + oc + size_t(ns) * 20, size_t(ns) * 4);
  }
  lap.lap("host_replay_finish");
  return CLG_OK;
}

// SimpleDeterminantEncoder.encodeTo over a batch (encode.hip): sizes pass, one host read
// of the total, write pass.
int clg_encode_batch(clg_engine* e, const clg_encode_in* in, void* out, uint64_t cap, uint32_t out_kind,
                     uint64_t* n_out, uint64_t* bad_index) {
  ENGINE_GUARD(e);
  if (!in || !n_out || (in->n && (!in->tag || !in->v0)) ||
      (in->n_wide && (!in->w_idx || !in->w_rc || !in->w_v1 || !in->w_var_off || !in->w_var_len || !in->w_sub)) ||
      (in->var_len && !in->var))
    return fail(CLG_E_INVALID_ARG, "null argument");
  *n_out = 0;
  if (bad_index) *bad_index = UINT64_MAX;
  if (in->n == 0) return CLG_OK;
  const uint64_t n = in->n, nw = in->n_wide;
  clg::EncodeIn d{in->tag, in->v0, in->w_idx, in->w_rc, in->w_v1, in->w_var_off, in->w_var_len, in->w_sub, in->var, n, nw};
  if (in->in_kind != CLG_MEM_DEVICE) {  // stage the host arrays in one device buffer
    const size_t sz[9] = {n, 8 * n, 4 * nw, 4 * nw, 8 * nw, 4 * nw, 4 * nw, nw, size_t(in->var_len)};
    const void* src[9] = {in->tag, in->v0, in->w_idx, in->w_rc, in->w_v1, in->w_var_off, in->w_var_len, in->w_sub, in->var};
    size_t off[9], tot = 0;
    for (int i = 0; i < 9; ++i) {
      off[i] = tot;
      tot += (sz[i] + 15) & ~size_t(15);
    }
    CHK(e->d_encin.ensure(tot + 16));
    uint8_t* b = e->d_encin.as<uint8_t>();
    for (int i = 0; i < 9; ++i)
      if (sz[i]) HIPCHK(hipMemcpyAsync(b + off[i], src[i], sz[i], hipMemcpyHostToDevice, e->stream));
    d = clg::EncodeIn{b + off[0], reinterpret_cast<const int64_t*>(b + off[1]), reinterpret_cast<const uint32_t*>(b + off[2]),
                      reinterpret_cast<const int32_t*>(b + off[3]), reinterpret_cast<const int64_t*>(b + off[4]),
                      reinterpret_cast<const uint32_t*>(b + off[5]), reinterpret_cast<const uint32_t*>(b + off[6]),
                      b + off[7], b + off[8], n, nw};
  }
  const uint64_t nb = (n + 1023) / 1024;
  const size_t o_wsum = 0, o_wbase = (nb * 4 + 15) & ~size_t(15), o_bsum = o_wbase + (((nb + 1) * 8 + 15) & ~size_t(15)),
               o_bbase = o_bsum + ((nb * 8 + 15) & ~size_t(15)), o_bad = o_bbase + (((nb + 1) * 8 + 15) & ~size_t(15));
  CHK(e->d_encw.ensure(o_bad + 16));
  uint8_t* w = e->d_encw.as<uint8_t>();
  auto* wsum = reinterpret_cast<uint32_t*>(w + o_wsum);
  auto* wbase = reinterpret_cast<uint64_t*>(w + o_wbase);
  auto* bsum = reinterpret_cast<uint64_t*>(w + o_bsum);
  auto* bbase = reinterpret_cast<uint64_t*>(w + o_bbase);
  auto* bad = reinterpret_cast<uint32_t*>(w + o_bad);
  HIPCHK(hipMemsetAsync(bad, 0xFF, 4, e->stream));
  CHK(clg::launch_encode(d, wsum, wbase, bsum, bbase, bad, nullptr, 0, e->stream));
  uint64_t hres[2] = {0, 0};  // total bytes, wide rows used
  uint32_t hbad = 0;
  HIPCHK(hipMemcpyAsync(&hres[0], bbase + nb, 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&hres[1], wbase + nb, 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, e->stream));
  CHK(e->sync());
  if (hbad != 0xFFFFFFFFu || hres[1] != nw) {
    if (bad_index) *bad_index = hbad != 0xFFFFFFFFu ? hbad : n;
    return fail(CLG_E_INVALID_ARG, "record %llu: invalid tag or side-table row (%llu wide rows given, %llu used)",
                (unsigned long long)(hbad != 0xFFFFFFFFu ? hbad : n), (unsigned long long)nw,
                (unsigned long long)hres[1]);
  }
  *n_out = hres[0];
  if (hres[0] > cap || !out) return fail(CLG_E_CAPACITY, "encode needs %llu bytes", (unsigned long long)hres[0]);
  uint8_t* dst = static_cast<uint8_t*>(out);
  if (out_kind != CLG_MEM_DEVICE) {
    CHK(e->d_encout.ensure(hres[0] + 16));
    dst = e->d_encout.as<uint8_t>();
  }
  CHK(e->timed("encode_write", hres[0] + 9 * n + 25 * nw + in->var_len,
               [&] { return clg::launch_encode(d, wsum, wbase, bsum, bbase, bad, dst, 1, e->stream); }));
  if (out_kind != CLG_MEM_DEVICE) HIPCHK(hipMemcpyAsync(out, dst, hres[0], hipMemcpyDeviceToHost, e->stream));
  return e->sync();
}

namespace {
void wr16(std::vector<uint8_t>& b, uint16_t v) { b.push_back(uint8_t(v >> 8)); b.push_back(uint8_t(v)); }
void wr32(std::vector<uint8_t>& b, uint32_t v) { wr16(b, uint16_t(v >> 16)); wr16(b, uint16_t(v)); }
void wr64(std::vector<uint8_t>& b, uint64_t v) { wr32(b, uint32_t(v >> 32)); wr32(b, uint32_t(v)); }
uint32_t rd32(const uint8_t* p) { return uint32_t(p[0]) << 24 | uint32_t(p[1]) << 16 | uint32_t(p[2]) << 8 | p[3]; }
uint64_t rd64(const uint8_t* p) { return uint64_t(rd32(p)) << 32 | rd32(p + 4); }
}  // namespace

// enrichWithCausalLogDelta (AbstractDeltaSerializerDeserializer.java:89-115) for a batch of
// channels: host metadata (hasDelta / offset / take) and header bytes, then one gather
// kernel writes headers and deltas into the output.
int clg_enrich_batch(clg_engine* e, uint32_t strategy, clg_enrich_req* reqs, uint32_t n, const uint32_t* log,
                     const uint8_t* flags, void* out, uint64_t cap, uint32_t out_kind, uint64_t* total) {
  ENGINE_GUARD(e);
  if ((n && (!reqs || !log)) || !total || strategy > CLG_DELTA_HIERARCHICAL)
    return fail(CLG_E_INVALID_ARG, "null argument or unknown strategy");
  CHK(e->flush());
  struct Adv {
    uint32_t log;
    ChKey k;
    int32_t nb;
  };
  struct Sent {
    uint32_t log;
    int32_t phys, nb;
    uint64_t dst;
  };
  std::vector<Adv> advs;
  std::vector<Sent> sent;
  std::vector<uint8_t> hdr;          // all headers back to back
  std::vector<uint64_t> hdr_at(n);   // request -> its header offset in hdr
  uint64_t dst = 0;
  for (uint32_t i = 0; i < n; ++i) {
    clg_enrich_req& r = reqs[i];
    r.status = CLG_OK;
    r.out_off = dst;
    const ChKey k{r.consumer.lo, r.consumer.hi};
    const size_t h0 = hdr.size();
    hdr_at[i] = h0;
    wr32(hdr, 0);  // header size, patched below (:98, :103)
    wr64(hdr, uint64_t(r.epoch));
    uint64_t dlen = 0;
    auto one = [&](uint32_t j, bool* has_out, int32_t* ofe, int32_t* nb) -> int {  // hasDelta, then take if sent
      int32_t has = 0;
      *has_out = false;
      CHK(e->has_delta(log[j], k, r.epoch, &has));
      if (!has || !(flags ? (flags[j] & CLG_DE_SEND) : 1)) return CLG_OK;
      CHK(e->offset_from_epoch(log[j], k, ofe));
      int32_t phys;
      CHK(e->take_delta(log[j], k, r.epoch, &phys, nb));
      advs.push_back(Adv{log[j], k, *nb});
      sent.push_back(Sent{log[j], phys, *nb, dlen});  // dst relative to the request's deltas, fixed below
      dlen += uint64_t(*nb);
      *has_out = true;
      return CLG_OK;
    };
    const size_t sent0 = sent.size();
    int st = CLG_OK;
    if (strategy == CLG_DELTA_FLAT) {  // [CausalLogID][offsetFromEpoch i32][len i32] per sent log (:80-84, :91-99)
      for (uint32_t j = r.first; j < r.first + r.count && st == CLG_OK; ++j) {
        bool has;
        int32_t ofe = 0, nb = 0;
        st = one(j, &has, &ofe, &nb);
        if (st != CLG_OK || !has) continue;
        const clg_causal_log_id& id = e->logs[log[j]].id;
        wr16(hdr, uint16_t(id.vertex_id));
        hdr.push_back(id.is_main ? 1 : 0);
        if (!id.is_main) {
          wr64(hdr, uint64_t(id.irp_lower));
          wr64(hdr, uint64_t(id.irp_upper));
          hdr.push_back(uint8_t(id.subpartition));
        }
        wr32(hdr, uint32_t(ofe));
        wr32(hdr, uint32_t(nb));
      }
    } else {  // Grouping: per vertex [vertex i16][hasMain]{main}[numPartitions u8]{[lo][hi][numSub u8]{[sub][ofe][len]}}
      uint32_t j = r.first;
      const uint32_t end = r.first + r.count;
      while (j < end && st == CLG_OK) {
        const int16_t v = e->logs[log[j]].id.vertex_id;
        const size_t vstart = hdr.size();
        int updates = 0;
        wr16(hdr, uint16_t(v));  // :113-115
        bool has = false;
        int32_t ofe = 0, nb = 0;
        if (e->logs[log[j]].id.is_main) {  // :116-121
          st = one(j, &has, &ofe, &nb);
          ++j;
        }
        if (st != CLG_OK) break;
        hdr.push_back(has ? 1 : 0);
        if (has) {
          wr32(hdr, uint32_t(ofe));
          wr32(hdr, uint32_t(nb));
          ++updates;
        }
        const size_t np_at = hdr.size();
        hdr.push_back(0);  // numPartitionDeltas (:134-141)
        int parts = 0;
        while (j < end && st == CLG_OK && e->logs[log[j]].id.vertex_id == v && !e->logs[log[j]].id.is_main) {
          const int64_t lo = e->logs[log[j]].id.irp_lower, hi = e->logs[log[j]].id.irp_upper;
          const size_t pstart = hdr.size();
          wr64(hdr, uint64_t(lo));  // :146-148
          wr64(hdr, uint64_t(hi));
          const size_t ns_at = hdr.size();
          hdr.push_back(0);
          int subs = 0;
          while (j < end && e->logs[log[j]].id.vertex_id == v && !e->logs[log[j]].id.is_main &&
                 e->logs[log[j]].id.irp_lower == lo && e->logs[log[j]].id.irp_upper == hi) {
            bool hs;
            int32_t o2 = 0, n2 = 0;
            st = one(j, &hs, &o2, &n2);
            if (st != CLG_OK) break;
            if (hs) {  // :150-154
              hdr.push_back(uint8_t(e->logs[log[j]].id.subpartition));
              wr32(hdr, uint32_t(o2));
              wr32(hdr, uint32_t(n2));
              ++subs;
            }
            ++j;
          }
          if (subs == 0) {
            hdr.resize(pstart);  // :156-158
          } else {
            hdr[ns_at] = uint8_t(subs);
            ++parts;
          }
        }
        hdr[np_at] = uint8_t(parts);
        updates += parts;
        if (updates == 0) hdr.resize(vstart);  // :125-126
        if (j < end && st == CLG_OK && e->logs[log[j]].id.vertex_id != v) continue;
        if (j < end && st == CLG_OK && e->logs[log[j]].id.vertex_id == v && e->logs[log[j]].id.is_main) {
          st = fail(CLG_E_INVALID_ARG, "hierarchical entries: vertex %d repeats", int(v));
        }
      }
    }
    if (st != CLG_OK) {  // undo this request's takes; the request reports the error
      for (size_t q = sent0; q < sent.size(); ++q) e->logs[sent[q].log].consumers[k].offset -= sent[q].nb;
      advs.resize(advs.size() - (sent.size() - sent0));
      sent.resize(sent0);
      hdr.resize(h0);
      r.status = st;
      r.header_bytes = 0;
      r.out_len = 0;
      continue;
    }
    const uint32_t hb = uint32_t(hdr.size() - h0);
    hdr[h0] = uint8_t(hb >> 24), hdr[h0 + 1] = uint8_t(hb >> 16), hdr[h0 + 2] = uint8_t(hb >> 8), hdr[h0 + 3] = uint8_t(hb);
    for (size_t q = sent0; q < sent.size(); ++q) sent[q].dst += dst + hb;
    r.header_bytes = hb;
    r.out_len = hb + dlen;
    dst += r.out_len;
  }
  *total = dst;
  if (dst > cap || (dst && !out)) {  // nothing moves: undo every take
    for (auto& a : advs) e->logs[a.log].consumers[a.k].offset -= a.nb;
    return fail(CLG_E_CAPACITY, "enrich needs %llu bytes", (unsigned long long)dst);
  }
  if (dst == 0) return CLG_OK;
  // headers staged in HBM (guard bytes either side for the gather's aligned reads)
  constexpr size_t kG = 32;
  CHK(e->d_hdr.ensure(hdr.size() + 2 * kG));
  CHK(e->h_stage.ensure(hdr.size() + 16));
  memcpy(e->h_stage.p, hdr.data(), hdr.size());
  uint8_t* dh = e->d_hdr.as<uint8_t>() + kG;
  HIPCHK(hipMemcpyAsync(dh, e->h_stage.p, hdr.size(), hipMemcpyHostToDevice, e->stream));
  std::vector<clg::GatherPiece> pieces;
  for (uint32_t i = 0; i < n; ++i)
    if (reqs[i].status == CLG_OK && reqs[i].header_bytes)
      pieces.push_back(clg::GatherPiece{dh + hdr_at[i], reqs[i].out_off, reqs[i].header_bytes, 0});
  for (auto& q : sent)
    if (q.nb > 0) e->add_pieces(e->logs[q.log], q.phys, q.nb, q.dst, pieces);
  return e->run_gather(pieces, dst, out, out_kind);
}

// processCausalLogDelta (:117-163): header parsed on the host, deltas applied by the
// batched upstream scatter straight from the message buffer.
int clg_process_delta(clg_engine* e, uint32_t job, uint32_t strategy, const uint8_t* msg, uint64_t n,
                      uint32_t in_kind, int64_t* epoch, uint32_t* handles, uint32_t cap, uint32_t* n_logs,
                      uint64_t* consumed) {
  ENGINE_GUARD(e);
  if (job >= e->jobs.size() || !e->jobs[job].open) return fail(CLG_E_NO_LOG, "unknown job %u", job);
  if (!msg || !epoch || !n_logs || strategy > CLG_DELTA_HIERARCHICAL) return fail(CLG_E_INVALID_ARG, "null argument");
  *n_logs = 0;
  if (n < 12) return fail(CLG_E_TRUNCATED, "delta header truncated");
  std::vector<uint8_t> hb(12);
  if (in_kind == CLG_MEM_DEVICE) HIPCHK(hipMemcpy(hb.data(), msg, 12, hipMemcpyDeviceToHost));
  else memcpy(hb.data(), msg, 12);
  const int32_t hsize = int32_t(rd32(hb.data()));
  if (hsize < 12 || uint64_t(hsize) > n) return fail(CLG_E_TRUNCATED, "delta header size %d", hsize);
  hb.resize(size_t(hsize));
  if (in_kind == CLG_MEM_DEVICE) HIPCHK(hipMemcpy(hb.data(), msg, size_t(hsize), hipMemcpyDeviceToHost));
  else memcpy(hb.data(), msg, size_t(hsize));
  *epoch = int64_t(rd64(hb.data() + 4));
  size_t p = 12;
  uint64_t delta_at = uint64_t(hsize);
  std::vector<clg_delta_req> reqs;
  auto need = [&](size_t k) { return p + k <= size_t(hsize); };
  auto apply = [&](const clg_causal_log_id& id) -> int {  // processThreadDelta :129-163
    if (!need(8)) return fail(CLG_E_TRUNCATED, "delta record truncated");
    const int32_t ofe = int32_t(rd32(&hb[p])), len = int32_t(rd32(&hb[p + 4]));
    p += 8;
    if (len < 0 || delta_at + uint64_t(len) > n) return fail(CLG_E_TRUNCATED, "delta past the message");
    uint32_t h;
    const IdKey key = key_of(job, id);
    auto it = e->by_id.find(key);
    if (it == e->by_id.end()) {
      CHK(clg_log_open(e, job, &id, &h));  // insertNewUpstreamLog
    } else {
      h = it->second;
    }
    reqs.push_back(clg_delta_req{h, ofe, *epoch, delta_at, uint32_t(len), 0});
    delta_at += uint64_t(len);
    if (*n_logs < cap && handles) handles[*n_logs] = h;
    ++*n_logs;
    return CLG_OK;
  };
  while (p < size_t(hsize)) {
    clg_causal_log_id id{};
    if (!need(3)) return fail(CLG_E_TRUNCATED, "CausalLogID truncated");
    id.vertex_id = int16_t(uint16_t(hb[p]) << 8 | hb[p + 1]);
    const bool main = hb[p + 2] != 0;
    p += 3;
    if (strategy == CLG_DELTA_FLAT) {  // deserializeCausalLogID (Flat :107-119)
      id.is_main = main ? 1 : 0;
      if (!main) {
        if (!need(17)) return fail(CLG_E_TRUNCATED, "CausalLogID truncated");
        id.irp_lower = int64_t(rd64(&hb[p]));
        id.irp_upper = int64_t(rd64(&hb[p + 8]));
        id.subpartition = int8_t(hb[p + 16]);
        p += 17;
      }
      CHK(apply(id));
    } else {  // Grouping deserializeStrategyStep :66-88
      if (main) {
        id.is_main = 1;
        CHK(apply(id));
      }
      if (!need(1)) return fail(CLG_E_TRUNCATED, "partition count truncated");
      const int np = int(int8_t(hb[p++]));
      for (int q = 0; q < np; ++q) {
        if (!need(17)) return fail(CLG_E_TRUNCATED, "partition truncated");
        clg_causal_log_id sid{};
        sid.vertex_id = id.vertex_id;
        sid.irp_lower = int64_t(rd64(&hb[p]));
        sid.irp_upper = int64_t(rd64(&hb[p + 8]));
        const int ns = int(int8_t(hb[p + 16]));
        p += 17;
        for (int t = 0; t < ns; ++t) {
          if (!need(1)) return fail(CLG_E_TRUNCATED, "subpartition truncated");
          sid.subpartition = int8_t(hb[p++]);
          CHK(apply(sid));
        }
      }
    }
  }
  if (consumed) *consumed = delta_at;
  if (reqs.empty()) return CLG_OK;
  CHK(e->upstream_batch(reqs.data(), uint32_t(reqs.size()), msg, in_kind));
  for (auto& r : reqs)
    if (r.status != CLG_OK) return fail(r.status, "processUpstreamDelta failed on log %u", r.log);
  return CLG_OK;
}

// ---- in-flight (data) log (inflightlogging/InMemorySubpartitionInFlightLogger.java) ------
static int ifl_get(clg_engine* e, uint32_t h, InFlight** out) {
  if (h >= e->ifls.size() || !e->ifls[h].open) return fail(CLG_E_NO_LOG, "unknown in-flight log handle %u", h);
  *out = &e->ifls[h];
  return CLG_OK;
}

static void ifl_release(clg_engine* e, std::vector<IflBuf>& bufs) {  // Buffer.recycleBuffer
  for (auto& b : bufs) e->ifl_free.insert(e->ifl_free.end(), b.segs.rbegin(), b.segs.rend());
  bufs.clear();
}

int clg_ifl_open(clg_engine* e, uint32_t* handle) { return clg_ifl_open_typed(e, CLG_IFL_IN_MEMORY, handle); }

int clg_ifl_open_typed(clg_engine* e, uint32_t type, uint32_t* handle) {
  ENGINE_GUARD(e);
  if (!handle) return fail(CLG_E_INVALID_ARG, "null argument");
  if (type != CLG_IFL_IN_MEMORY && type != CLG_IFL_SPILLABLE) return fail(CLG_E_INVALID_ARG, "bad in-flight log type %u", type);
  uint32_t i = 0;
  while (i < e->ifls.size() && e->ifls[i].open) ++i;
  if (i == e->ifls.size()) e->ifls.emplace_back();
  e->ifls[i] = InFlight{};
  e->ifls[i].open = true;
  e->ifls[i].type = type;
  *handle = i;
  return CLG_OK;
}

int clg_ifl_close(clg_engine* e, uint32_t h) {  // close() :90-94
  ENGINE_GUARD(e);
  InFlight* f;
  CHK(ifl_get(e, h, &f));
  for (auto& kv : f->epochs) ifl_release(e, kv.second);
  f->epochs.clear();
  f->open = false;
  return CLG_OK;
}

// log(buffer, epochID, isFinished) :44-48 -- computeIfAbsent(epoch).add(buffer), batched.
// Segments are taken for the whole batch first (all-or-nothing), then one scatter copies
// every buffer into its segments.
int clg_ifl_log_batch(clg_engine* e, const uint32_t* ifl, const int64_t* epoch, const uint64_t* off,
                      const uint32_t* len, uint32_t n, const uint8_t* bytes, uint32_t in_kind) {
  ENGINE_GUARD(e);
  if (n == 0) return CLG_OK;
  if (!ifl || !epoch || !off || !len || !bytes) return fail(CLG_E_INVALID_ARG, "null argument");
  if (in_kind != CLG_MEM_HOST && in_kind != CLG_MEM_DEVICE) return fail(CLG_E_INVALID_ARG, "bad in_kind");
  const uint32_t C = e->ifl_C;
  size_t need = 0, total = 0;
  for (uint32_t i = 0; i < n; ++i) {
    InFlight* f;
    CHK(ifl_get(e, ifl[i], &f));
    need += (size_t(len[i]) + C - 1) / C;
    total += len[i];
  }
  if (need > e->ifl_free.size())
    return fail(CLG_E_NOSPACE, "in-flight pool exhausted (needs %zu segments, free %zu)", need, e->ifl_free.size());
  CHK(e->gwait());  // a queued gather may still read segments that were freed and are reused now
  std::vector<clg::ScatterChunk> ch;
  ch.reserve(need);
  const uint8_t* dsrc = bytes;
  if (in_kind == CLG_MEM_HOST) {  // pack the buffers into pinned staging, one upload
    CHK(e->h_stage.ensure(total ? total : 1));
    CHK(e->d_stage.ensure(total ? total : 1));
    dsrc = e->d_stage.as<uint8_t>();
  }
  uint64_t packed = 0;
  uint32_t npe = 0;  // 1 + the first buffer whose spillable log() throws after appending
  for (uint32_t i = 0; i < n; ++i) {
    IflBuf b{{}, len[i]};
    const uint64_t src = in_kind == CLG_MEM_HOST ? packed : off[i];
    if (in_kind == CLG_MEM_HOST && len[i]) memcpy(e->h_stage.as<uint8_t>() + packed, bytes + off[i], len[i]);
    for (uint32_t o = 0; o < len[i]; o += C) {
      const uint32_t s = e->ifl_free.back();
      e->ifl_free.pop_back();
      b.segs.push_back(s);
      ch.push_back(clg::ScatterChunk{e->ifl_addr(s), src + o, std::min(C, len[i] - o), 0});
    }
    packed += len[i];
    InFlight& f = e->ifls[ifl[i]];
    f.epochs[epoch[i]].push_back(std::move(b));
    if (f.type == CLG_IFL_SPILLABLE && f.replaying) {  // :98-99
      if (!f.it.exists) {
        npe = npe ? npe : i + 1;  // currentIterator is null: notifyNewBufferAdded throws
      } else {                    // SpilledReplayIterator.notifyNewBufferAdded :262-277
        for (IflCursor* c : {&f.it.pre, &f.it.con}) {
          ++c->rem;
          c->last = std::max(c->last, epoch[i]);
        }
      }
    }
  }
  if (ch.empty())
    return npe ? fail(CLG_E_STATE, "log() of buffer %u while replaying without an iterator (NullPointerException)", npe - 1)
               : CLG_OK;
  const size_t db = ch.size() * sizeof(clg::ScatterChunk);
  CHK(e->h_desc.ensure(db));
  CHK(e->d_desc.ensure(db));
  memcpy(e->h_desc.p, ch.data(), db);
  if (in_kind == CLG_MEM_HOST)
    HIPCHK(hipMemcpyAsync(e->d_stage.p, e->h_stage.p, total, hipMemcpyHostToDevice, e->stream));
  HIPCHK(hipMemcpyAsync(e->d_desc.p, e->h_desc.p, db, hipMemcpyHostToDevice, e->stream));
  CHK(e->timed("ifl_scatter", 2 * total, [&] {
    return clg::launch_scatter(e->d_desc.as<clg::ScatterChunk>(), uint32_t(ch.size()), dsrc, e->stream);
  }));
  HIPCHK(hipStreamSynchronize(e->stream));  // staging buffers are reused; device input is the caller's
  if (npe) return fail(CLG_E_STATE, "log() of buffer %u while replaying without an iterator (NullPointerException)", npe - 1);
  return CLG_OK;
}

int clg_ifl_notify_checkpoint_complete(clg_engine* e, uint32_t h, int64_t cp) {  // :51-70
  ENGINE_GUARD(e);
  InFlight* f;
  CHK(ifl_get(e, h, &f));
  for (auto it = f->epochs.begin(); it != f->epochs.end() && it->first < cp;) {
    ifl_release(e, it->second);
    it = f->epochs.erase(it);
  }
  return CLG_OK;
}

int clg_ifl_state(clg_engine* e, uint32_t h, int64_t* ids, uint32_t* nb, uint32_t cap, uint32_t* n_epochs) {
  ENGINE_GUARD(e);
  InFlight* f;
  CHK(ifl_get(e, h, &f));
  uint32_t k = 0;
  for (auto& kv : f->epochs) {
    if (k < cap) {
      if (ids) ids[k] = kv.first;
      if (nb) nb[k] = uint32_t(kv.second.size());
    }
    ++k;
  }
  if (n_epochs) *n_epochs = k;
  return CLG_OK;
}

// ---- the spillable logger's iterator (SpilledReplayIterator.java), on host metadata ---------
// Every EpochCursor step that reads the map through the live view tailMap(view) fails (returns
// false) where the Java code throws: an epoch missing from the view (NullPointerException) or an
// offset past its buffers (IndexOutOfBoundsException).
static bool ifl_size(const InFlight& f, int64_t view, int64_t ep, int64_t* n) {  // log.get(ep).getEpochSize()
  if (ep < view) return false;
  const auto it = f.epochs.find(ep);
  if (it == f.epochs.end()) return false;
  *n = int64_t(it->second.size());
  return true;
}
static bool ifl_advance(const InFlight& f, int64_t view, IflCursor& c) {  // advanceEpochIfNeeded :353-358
  int64_t n;
  if (!ifl_size(f, view, c.ne, &n)) return false;
  if (c.off == n && c.ne != c.last) {
    ++c.ne;
    c.off = 0;
  }
  return true;
}
static bool ifl_cnext(const InFlight& f, int64_t view, IflCursor& c, const IflBuf** out) {  // next() :342-351
  if (!ifl_advance(f, view, c)) return false;
  const auto it = c.ne >= view ? f.epochs.find(c.ne) : f.epochs.end();
  if (it == f.epochs.end() || c.off < 0 || c.off >= int64_t(it->second.size())) return false;
  if (out) *out = &it->second[size_t(c.off)];
  ++c.off;
  --c.rem;
  return ifl_advance(f, view, c);
}
static bool ifl_behind(const InFlight& f, int64_t view, IflCursor& a, IflCursor& b, bool* res) {  // behind() :364-367
  if (!ifl_advance(f, view, a) || !ifl_advance(f, view, b)) return false;
  *res = a.ne < b.ne || (a.ne == b.ne && a.off < b.off);
  return true;
}
static void ifl_prefetch(const InFlight& f, IflIter& it) {  // prefetchNextBuffers :126-158 (exceptions swallowed)
  while (it.pre.rem > 0)
    if (!ifl_advance(f, it.view, it.pre) || !ifl_cnext(f, it.view, it.pre, nullptr)) return;
}

// getInFlightIterator(start, ignore) and the drain of its iterator, per logger type:
//   in-memory (:73-82, ReplayIterator :114-167): walks tailMap(start) by ++currentKey, so it only
//     yields contiguous epochs from `start`; a missing key throws inside next() right after the
//     last buffer before it was taken (:156 -> :133), so that buffer is lost to the caller;
//   spillable (:126-142, SpilledReplayIterator): the iterator is the logger's current one, its
//     cursors stepped literally (above); max_buffers / CLG_IFL_CONTINUE drain it in parts.
// Iterator state is worked on in copies and committed only when the gather runs, so a sizing
// call (CLG_E_CAPACITY) changes nothing.
int clg_ifl_replay_batch(clg_engine* e, const clg_ifl_replay_req* reqs, uint32_t n, clg_ifl_replay_res* res,
                         void* out, uint64_t cap, uint32_t out_kind, uint32_t* sizes, int64_t* epochs,
                         uint64_t sizes_cap, uint64_t* total, uint64_t* total_buffers) {
  ENGINE_GUARD(e);
  if (n && (!reqs || !res)) return fail(CLG_E_INVALID_ARG, "null argument");
  if (out_kind != CLG_MEM_HOST && out_kind != CLG_MEM_DEVICE) return fail(CLG_E_INVALID_ARG, "bad out_kind");
  struct Pick {
    const IflBuf* b;
    uint64_t dst;
  };
  struct Work {  // a spillable logger's iterator state during this call
    IflIter it;
    bool replaying;
  };
  std::map<uint32_t, Work> work;
  std::vector<Pick> picks;
  uint64_t dst = 0, nbuf = 0;
  auto take = [&](clg_ifl_replay_res& r, const IflBuf& b, int64_t ep) {
    picks.push_back(Pick{&b, dst});
    if (nbuf < sizes_cap) {
      if (sizes) sizes[nbuf] = b.len;
      if (epochs) epochs[nbuf] = ep;  // getEpoch() before this next()
    }
    dst += b.len;
    r.len += b.len;
    ++nbuf;
    ++r.n_buffers;
  };
  for (uint32_t i = 0; i < n; ++i) {
    clg_ifl_replay_res& r = res[i];
    const int64_t start = reqs[i].start_epoch;
    r = clg_ifl_replay_res{CLG_OK, 0, 0, 0, dst, 0, nbuf, start};
    InFlight* f;
    int st = ifl_get(e, reqs[i].ifl, &f);
    if (st != CLG_OK) {
      r.status = st;
      continue;
    }
    const uint64_t ign = reqs[i].ignore_buffers;
    if (f->type == CLG_IFL_SPILLABLE) {
      auto wi = work.find(reqs[i].ifl);
      if (wi == work.end()) wi = work.emplace(reqs[i].ifl, Work{f->it, f->replaying}).first;
      Work& w = wi->second;
      if (!(reqs[i].flags & CLG_IFL_CONTINUE)) {  // getInFlightIterator :126-142
        w.replaying = true;
        const auto first = f->epochs.lower_bound(start);
        if (first == f->epochs.end()) {  // tailMap empty: null (the current iterator stays)
          r.flags = CLG_IFL_NULL_ITERATOR | CLG_IFL_REPLAYING;
          continue;
        }
        IflIter it;
        it.exists = true;
        it.view = start;
        it.con.ne = first->first;
        it.con.last = f->epochs.rbegin()->first;
        for (auto jt = first; jt != f->epochs.end(); ++jt) it.con.rem += int64_t(jt->second.size());
        it.pre = it.con;
        bool ok = true;
        for (uint64_t k = 0; k < ign && ok; ++k)  // the constructor's skip :98-101
          ok = ifl_cnext(*f, it.view, it.con, nullptr) && ifl_cnext(*f, it.view, it.pre, nullptr);
        if (!ok) {  // the constructor throws: no new iterator, isReplaying stays set
          r.status = fail(CLG_E_STATE, "skip of %llu buffers fails inside the iterator's constructor",
                          (unsigned long long)ign);
          r.flags = CLG_IFL_REPLAYING;
          continue;
        }
        ifl_prefetch(*f, it);  // :123
        w.it = it;
      } else if (!w.it.exists) {
        r.status = fail(CLG_E_STATE, "no current in-flight iterator to continue");
        r.flags = w.replaying ? CLG_IFL_REPLAYING : 0u;
        continue;
      }
      IflIter& it = w.it;
      r.remaining = uint32_t(std::max<int64_t>(it.con.rem, 0));
      const uint32_t cap_n = reqs[i].max_buffers;
      bool thrown = false;
      while (it.con.rem > 0 && (cap_n == 0 || r.n_buffers < cap_n)) {  // next() :171-203
        bool bh;
        if (!ifl_behind(*f, it.view, it.con, it.pre, &bh)) {
          thrown = true;
          break;
        }
        if (!bh) {
          ifl_prefetch(*f, it);
          if (!ifl_behind(*f, it.view, it.con, it.pre, &bh) || !bh) {  // (not behind: it would wait forever)
            thrown = true;
            break;
          }
        }
        const IflBuf* b = nullptr;
        if (!ifl_advance(*f, it.view, it.con)) {  // getEpoch() :166-168
          thrown = true;
          break;
        }
        const int64_t ep = it.con.ne;
        if (!ifl_cnext(*f, it.view, it.con, &b)) {
          thrown = true;
          break;
        }
        if (it.con.rem <= 0) w.replaying = false;  // :186-193
        ifl_prefetch(*f, it);
        take(r, *b, ep);
      }
      if (thrown) r.status = CLG_E_EPOCH_GAP;
      IflCursor c = it.con;
      r.end_epoch = ifl_advance(*f, it.view, c) ? c.ne : it.con.ne;
      r.flags = w.replaying ? CLG_IFL_REPLAYING : 0u;
      continue;
    }
    if (reqs[i].max_buffers || reqs[i].flags) {
      r.status = fail(CLG_E_INVALID_ARG, "max_buffers / CLG_IFL_CONTINUE need a spillable in-flight log");
      continue;
    }
    auto it = f->epochs.find(start);
    if (it == f->epochs.end()) {  // :121-127 -- currentIterator == null, nothing left, currentKey = start
      if (ign) r.status = fail(CLG_E_STATE, "skip of %llu buffers on an empty iterator", (unsigned long long)ign);
      continue;
    }
    uint64_t tail = 0, k = 0;  // tail: numberOfBuffersLeft (:123); k: buffers before a gap
    bool gap = false;
    int64_t expect = start;
    for (auto jt = it; jt != f->epochs.end(); ++jt) {
      tail += jt->second.size();
      if (!gap && jt->first == expect) {
        k += jt->second.size();
        ++expect;
      } else {
        gap = true;
      }
    }
    const uint64_t deliver = gap ? k - 1 : k;  // buffers next() returns
    if (ign > deliver) {  // the skip loop inside getInFlightIterator throws (:78-79)
      r.status = gap ? fail(CLG_E_STATE, "skip of %llu buffers reaches an epoch gap after %llu", (unsigned long long)ign,
                            (unsigned long long)deliver)
                     : fail(CLG_E_STATE, "skip of %llu buffers past the end (%llu)", (unsigned long long)ign,
                            (unsigned long long)deliver);
      continue;
    }
    if (gap) r.status = CLG_E_EPOCH_GAP;  // the next() after the last delivered buffer throws (:156 -> :133)
    // after the last successful next() the iterator sits on the last contiguous epoch: that
    // epoch holds the final buffer (no gap) or the K-th buffer the gap swallows
    r.end_epoch = expect - 1;
    r.remaining = uint32_t(tail - ign);
    uint64_t idx = 0;
    for (auto jt = it; jt != f->epochs.end() && idx < deliver; ++jt)
      for (const IflBuf& b : jt->second) {
        if (idx >= deliver) break;
        if (idx++ < ign) continue;
        take(r, b, jt->first);
      }
  }
  if (total) *total = dst;
  if (total_buffers) *total_buffers = nbuf;
  if (dst > cap || nbuf > sizes_cap || (nbuf && !sizes) || (dst && !out))
    return fail(CLG_E_CAPACITY, "in-flight replay needs %llu bytes / %llu sizes (cap %llu / %llu)",
                (unsigned long long)dst, (unsigned long long)nbuf, (unsigned long long)cap,
                (unsigned long long)sizes_cap);
  for (auto& kv : work) {  // commit the spillable iterators
    e->ifls[kv.first].it = kv.second.it;
    e->ifls[kv.first].replaying = kv.second.replaying;
  }
  std::vector<clg::GatherPiece> pieces;
  const uint32_t C = e->ifl_C;
  for (const Pick& p : picks)
    for (size_t s = 0; s < p.b->segs.size(); ++s) {
      const uint32_t o = uint32_t(s) * C;
      pieces.push_back(clg::GatherPiece{e->ifl_addr(p.b->segs[s]), p.dst + o, std::min(C, p.b->len - o), 0});
    }
  CHK(e->flush());
  return e->run_gather(pieces, dst, out, out_kind, "ifl_gather");
}

int clg_kernel_stats(clg_engine* e, clg_kernel_stat* out, uint32_t cap, uint32_t* n) {
  ENGINE_GUARD(e);
  CHK(e->sync());
  uint32_t i = 0;
  for (auto& kv : e->stats) {
    if (i < cap) {
      memset(&out[i], 0, sizeof out[i]);
      snprintf(out[i].name, sizeof out[i].name, "%s", kv.first.c_str());
      out[i].launches = kv.second.launches;
      out[i].total_ms = kv.second.ms;
      out[i].bytes = kv.second.bytes;
    }
    ++i;
  }
  *n = i;
  return CLG_OK;
}

int clg_kernel_stats_reset(clg_engine* e) {
  ENGINE_GUARD(e);
  CHK(e->sync());
  e->stats.clear();
  return CLG_OK;
}

}  // extern "C"
