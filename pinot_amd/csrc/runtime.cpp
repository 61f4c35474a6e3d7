// runtime.cpp — host runtime of libpinotgpu.so: tables, pinned segments, global dictionaries, query plans and
// results behind the C ABI of include/pinotgpu.h.
//
// What runs where:
//   host  : per-segment predicate translation into dictId space (the PredicateEvaluators of
//           core/operator/filter/predicate/, once per segment per query, O(log card) each), filter constant
//           folding (FilterPlanNode.java:146-247), group-key layout (DictionaryBasedGroupKeyGenerator key math
//           over the table-global dictionaries), result decoding;
//   device: everything per document (kernels.hip).
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <execinfo.h>
#include <pthread.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <thread>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <list>
#include <map>
#include <unordered_map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/pinotgpu.h"
#include "comm.h"
#include "filter_stats.h"
#include "host_common.h"
#include "host_result.h"
#include "internal.h"
#include "range_index.h"

using namespace pgpu;

// ================================================================================================ errors
namespace {

// PGPU_TRACE=crash (diagnostics): on SIGSEGV / SIGBUS / SIGABRT print the faulting address and the native frames
// (backtrace_symbols_fd: object, symbol or offset -- resolve offsets with addr2line -f -C -e <object>), then hand the
// signal to the previously installed handler (Python's faulthandler prints the Python stacks).
struct sigaction g_prev_segv, g_prev_bus, g_prev_abrt;
void crash_trace_handler(int sig, siginfo_t* si, void* uc) {
  char line[160];
  int len = snprintf(line, sizeof line, "[pgpu] fatal signal %d at address %p (thread %lu)\n", sig,
                     si ? si->si_addr : nullptr, (unsigned long)pthread_self());
  if (len > 0) { ssize_t w = write(2, line, (size_t)len); (void)w; }
  void* frames[64];
  const int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  for (int i = 0; i < n; ++i) {  // offsets into their objects, for addr2line
    Dl_info info;
    if (dladdr(frames[i], &info) && info.dli_fname) {
      len = snprintf(line, sizeof line, "[pgpu]   #%d %s +0x%lx\n", i, info.dli_fname,
                     (unsigned long)((uintptr_t)frames[i] - (uintptr_t)info.dli_fbase));
      if (len > 0) { ssize_t w = write(2, line, (size_t)len); (void)w; }
    }
  }
  const struct sigaction* prev = sig == SIGSEGV ? &g_prev_segv : sig == SIGBUS ? &g_prev_bus : &g_prev_abrt;
  if (prev->sa_flags & SA_SIGINFO) {
    if (prev->sa_sigaction) { prev->sa_sigaction(sig, si, uc); return; }
  } else if (prev->sa_handler != SIG_DFL && prev->sa_handler != SIG_IGN && prev->sa_handler) {
    prev->sa_handler(sig);
    return;
  }
  signal(sig, SIG_DFL);
  raise(sig);
}
// Diagnostics: PGPU_TRACE, the one environment variable the library reads -- comma-separated words, none of which
// changes a result: "1" (per-phase host times of every plan, execution and finalize on stderr), "crash" (on
// SIGSEGV / SIGBUS / SIGABRT print the native frames), "check" (a scan launch's records and tile map are read back
// and checked before the launch), "serialize" (entry points run one at a time: isolates host races from device ones).
// Executor settings are pgpu_config's (pgpu_table_set_config), never the environment.
bool diag(const char* word) {
  static const std::string v = [] {
    const char* e = getenv("PGPU_TRACE");
    return "," + std::string(e ? e : "") + ",";
  }();
  return v.find("," + std::string(word) + ",") != std::string::npos;
}

struct CrashTraceInstaller {
  void install() {
    if (!diag("crash")) return;
    void* warm[2];
    backtrace(warm, 2);  // loads the unwinder now, not inside the handler
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = crash_trace_handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &g_prev_segv);
    sigaction(SIGBUS, &sa, &g_prev_bus);
    sigaction(SIGABRT, &sa, &g_prev_abrt);
    static const char msg[] = "[pgpu] crash trace installed\n";
    ssize_t w = write(2, msg, sizeof msg - 1);
    (void)w;
  }
};
void install_crash_trace() {
  static std::once_flag once;
  std::call_once(once, [] { CrashTraceInstaller().install(); });
}

thread_local std::string g_err;

// PGPU_TRACE=1: per-phase host timings on stderr (diagnostics only).
bool trace_on() {
  static const bool on = diag("1");
  return on;
}
double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

}  // namespace

int pgpu::host_fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int pgpu::abi_exception() noexcept {
  try {
    throw;
  } catch (const std::bad_alloc&) {
    g_err = "host allocation failed";
    return PGPU_ERR_OUT_OF_MEMORY;
  } catch (const std::exception& e) {
    return host_fail(PGPU_ERR_INVALID_ARGUMENT, "internal error: %s", e.what());
  } catch (...) {
    return host_fail(PGPU_ERR_INVALID_ARGUMENT, "internal error");
  }
}

namespace {

#define HIP_TRY(expr)                                                                               \
  do {                                                                                              \
    hipError_t _e = (expr);                                                                         \
    if (_e != hipSuccess)                                                                           \
      return fail(_e == hipErrorOutOfMemory ? PGPU_ERR_OUT_OF_MEMORY : PGPU_ERR_DEVICE, "%s: %s (%s:%d)", \
                  #expr, hipGetErrorString(_e), __FILE__, __LINE__);                                \
  } while (0)

#define TRY(expr)          \
  do {                     \
    int _rc = (expr);      \
    if (_rc) return _rc;   \
  } while (0)

// The execution's timing events (pgpu_plan_timing).  PGPU_NO_TIMING_EVENTS (an A/B build of the library only): none
// recorded -- each event is a marker packet between two dependent dispatches of the stream.
#ifdef PGPU_NO_TIMING_EVENTS
#define PGPU_TIMING_RECORD(ev, stream) ((void)0)
#else
#define PGPU_TIMING_RECORD(ev, stream) HIP_TRY(hipEventRecord(ev, stream))
#endif

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    hipGetDevice(&prev);
    if (prev != dev) hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) hipSetDevice(prev);
  }
};

// Device buffer that only grows (hipFree synchronises the device; growth is rare after warm-up).
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t n) {
    if (n <= cap) return 0;
    if (p && trace_on()) fprintf(stderr, "[pgpu] device buffer grows %zu -> %zu bytes\n", cap, n + n / 4);
    if (p) HIP_TRY(hipFree(p));
    p = nullptr;
    size_t c = std::max<size_t>(n + n / 4, 4096);
    HIP_TRY(hipMalloc(&p, c));
    cap = c;
    return 0;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

// Device memory owned through shared_ptr: freed with its last owner.  A column's LUT is rebuilt out of place when
// the table-global dictionary grows, so a plan still running keeps reading the LUT it was planned with.
struct DevMem {
  void* p = nullptr;
  DevMem() = default;
  DevMem(const DevMem&) = delete;
  DevMem& operator=(const DevMem&) = delete;
  ~DevMem() { if (p) hipFree(p); }
};

// Host worker pool for per-query planning of long segment lists (the per-segment predicate translation that
// Pinot runs on its query worker threads, one task per segment: BaseCombineOperator.java:85-115).  Workers are
// started once and parked on a condition variable; run() executes fn(0..n-1) on the workers and the caller.
class HostPool {
 public:
  explicit HostPool(int workers) {
    for (int i = 0; i < workers; ++i) threads_.emplace_back([this] { loop(); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& th : threads_) th.join();
  }
  int size() const { return (int)threads_.size(); }
  void run(int n, const std::function<void(int)>& fn) {
    std::lock_guard<std::mutex> serial(run_mu_);  // one batch at a time
    {
      std::lock_guard<std::mutex> g(mu_);
      fn_ = &fn;
      n_ = n;
      next_.store(0);
      done_ = 0;
      ++gen_;
    }
    cv_.notify_all();
    int mine = 0;
    for (int i; (i = next_.fetch_add(1)) < n;) { fn(i); ++mine; }
    std::unique_lock<std::mutex> g(mu_);
    done_ += mine;
    // every worker that joined this batch must have left its claim loop before the next batch resets next_ (a
    // straggler's fetch_add would otherwise claim an index of the next batch and call this batch's fn)
    done_cv_.wait(g, [&] { return done_ >= n_ && active_ == 0; });
    fn_ = nullptr;
  }

 private:
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* fn;
      int n;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        fn = fn_;
        n = n_;
        if (!fn) continue;  // the batch already completed
        ++active_;
      }
      int mine = 0;
      for (int i; (i = next_.fetch_add(1)) < n;) { (*fn)(i); ++mine; }
      std::lock_guard<std::mutex> g(mu_);
      done_ += mine;
      --active_;
      if (done_ >= n_ && active_ == 0) done_cv_.notify_all();
    }
  }
  std::vector<std::thread> threads_;
  std::mutex mu_, run_mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0, done_ = 0, active_ = 0;
  std::atomic<int> next_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};

HostPool& host_pool() {
  static HostPool pool(std::max(1, std::min(7, (int)std::thread::hardware_concurrency() - 1)));
  return pool;
}
// Segments per planning task.  Measured on MI355X hosts: translating the 1000 segments of C3 takes ~90 us on one
// thread, and waking pool workers costs more than it saves below a few thousand segments, so lists shorter than
// this are planned on the calling thread.  pgpu_config.plan_chunk_segments sets it (tests).
// Launches of a streamed plan: equal chunks, so every launch of the scan kernel covers the same work (the
// roofline's per-launch bytes and rocprof's average launch agree).  Measured on MI355X (C3, 1000 segments): four
// streamed launches took 1.115 ms per query against 0.950 ms for one -- each launch boundary costs the scan's
// ramp and tail (~33 us) plus the in-stream record upload, more than the ~130 us of planning it hides -- so plans
// run as one launch unless pgpu_config.stream_chunks asks for more (tests exercise the streamed path with it).
int stream_chunk_count(const pgpu_config& cfg, size_t nseg) {
  if (cfg.stream_chunks > 1) return std::min<int>(cfg.stream_chunks, (int)std::max<size_t>(nseg, 1));
  return 1;
}

size_t plan_chunk_segs(const pgpu_config& cfg) {
  return cfg.plan_chunk_segments > 0 ? (size_t)cfg.plan_chunk_segments : 4096;
}

// ================================================================================================ values
inline uint32_t rd_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
inline uint64_t rd_be64(const uint8_t* p) { return ((uint64_t)rd_be32(p) << 32) | rd_be32(p + 4); }
inline void wr_be32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}
inline void wr_be64(uint8_t* p, uint64_t v) { wr_be32(p, (uint32_t)(v >> 32)); wr_be32(p + 4, (uint32_t)v); }

// Double.doubleToLongBits's NaN (0x7ff8000000000000): raw values and IN-set literals use it for every NaN.
const double kCanonicalNaN = [] {
  const uint64_t b = 0x7ff8000000000000ull;
  double d;
  memcpy(&d, &b, 8);
  return d;
}();
// Raw (no-dictionary) columns: per-doc value arrays padded to whole 32-doc groups (the raw filter leaves read a
// lane's whole group).
inline int64_t raw_padded_docs(int64_t n) { return std::max<int64_t>((n + 31) & ~int64_t(31), 32); }

// Order-preserving int64 key of a double (MIN/MAX operand on the device).
inline int64_t double_key(double d) {
  int64_t b;
  memcpy(&b, &d, 8);
  return b >= 0 ? b : (b ^ INT64_MAX);
}
inline double key_double(int64_t k) {
  int64_t b = k >= 0 ? k : (k ^ INT64_MAX);
  double d;
  memcpy(&d, &b, 8);
  return d;
}

constexpr int64_t kHostCompactBytes = 512 * 1024;  // dense tables up to this size are compacted on the host
constexpr int64_t kPartMinBytes = 32ll << 20;        // dense tables this large use the partitioned group-by
#ifndef PGPU_PART_LDS_KB
#define PGPU_PART_LDS_KB 64
#endif
constexpr int64_t kPartLds = PGPU_PART_LDS_KB * 1024;  // K8d accumulators per partition (LDS)
constexpr int64_t kMaxParts = 16384;                 // K8a/K8c LDS histogram entries
constexpr int64_t kHashPartLdsMax = 64 * 1024;       // K8h LDS hash table per partition, at most
constexpr int64_t kPartMaxRecordBytes = 32ll << 30;  // scratch for the partitioned records
constexpr int kDocIdColumn = -2;                     // query column of the virtual $docId (hidden first-doc slot)

bool is_int_type(int t) { return t == PGPU_INT || t == PGPU_LONG; }
bool is_fp_type(int t) { return t == PGPU_FLOAT || t == PGPU_DOUBLE; }

// PinotDataBitSet.getNumBitsPerValue (seglocal/io/util/PinotDataBitSet.java:59-70): bit length, at least 1.
int num_bits_per_value(int max_value) {
  if (max_value <= 1) return 1;
  int n = 0;
  while (max_value) { n++; max_value >>= 1; }
  return n;
}

// Strict decimal conversion of Integer.parseInt / Long.parseLong.
bool parse_long(const char* s, int64_t lo, int64_t hi, int64_t* out) {
  const char* p = s;
  bool neg = false;
  if (*p == '+' || *p == '-') { neg = *p == '-'; ++p; }
  if (!*p) return false;
  unsigned __int128 v = 0;
  for (; *p; ++p) {
    if (*p < '0' || *p > '9') return false;
    v = v * 10 + (unsigned)(*p - '0');
    if (v > ((unsigned __int128)1 << 64)) return false;
  }
  __int128 sv = neg ? -(__int128)v : (__int128)v;
  if (sv < lo || sv > hi) return false;
  *out = (int64_t)sv;
  return true;
}
// Double.parseDouble / Float.parseFloat (decimal and the Java 'd'/'f' suffixes).
bool parse_double(const char* s, double* out) {
  char* end = nullptr;
  errno = 0;
  double d = strtod(s, &end);
  if (end == s) return false;
  while (*end == 'd' || *end == 'D' || *end == 'f' || *end == 'F' || *end == ' ') ++end;
  if (*end) return false;
  *out = d;
  return true;
}

int cmp_bytes(const uint8_t* a, size_t na, const uint8_t* b, size_t nb) {
  int c = memcmp(a, b, std::min(na, nb));
  if (c) return c;
  return na < nb ? -1 : (na > nb ? 1 : 0);
}

// ================================================================================================ model
// Host copy of one dictionary (segment-local or table-global), sorted ascending.  A table-global dictionary is an
// immutable snapshot (copy on growth, `id` unique per snapshot): plans and their results keep the snapshot their
// group ids index, so a pin that grows the dictionary while a query runs never re-labels that query's groups.
std::atomic<uint64_t> g_dict_ids{1};
struct Dict {
  int type = PGPU_INT;
  uint64_t id = 0;
  uint64_t digest = 0;           // content hash, computed on first use (dict_digest; 0 = not yet)
  std::vector<int64_t> iv;       // INT / LONG
  std::vector<double> dv;        // FLOAT / DOUBLE
  std::vector<std::string> sv;   // STRING (unpadded)
  size_t size() const { return is_int_type(type) ? iv.size() : is_fp_type(type) ? dv.size() : sv.size(); }
};

// A pinned bitmap inverted index (pgpu_attach_inverted_index; BitmapInvertedIndexReader): the Roaring containers
// of every dictId in one device block (ARRAY / BITMAP payloads, internal.h), their directory kept on the host.
struct InvIndex {
  struct Cont { int64_t word; int32_t type, n, key; };
  // Owned: freed with the last owner (the segment column, or a plan whose bitmap tasks point into it), so a
  // re-attach or an unpin never frees memory an existing plan still reads.
  ~InvIndex() { if (d_block) hipFree(d_block); }
  void* d_block = nullptr;
  int64_t bytes = 0;
  // Per dictId, in one 16-byte record so planning takes one cache miss per (segment, dictId): its containers
  // [begin, begin + count) and its docs (Roaring cardinality).
  struct Entry { int32_t begin, count; int64_t docs; };
  std::vector<Entry> ids;
  std::vector<Cont> conts;
};

struct Column {
  int32_t card = 0, bits = 0, entry_width = 0, padding = 0;
  int64_t fwd_bytes = 0;            // Pinot byte length of the forward index
  uint32_t* d_fwd = nullptr;        // inside the segment's allocation
  int64_t fwd_words = 0;            // padded words
  Dict dict;                        // parsed local dictionary
  bool sorted = false;              // SortedIndexReaderImpl column: docIds of dictId i are [sorted_start[i], sorted_start[i+1])
  std::vector<int32_t> sorted_start;
  std::vector<uint8_t> raw_dict;    // BIG_ENDIAN bytes as pinned (string padding semantics, column_bytes)
  // lazily built device arrays (under the table mutex)
  std::shared_ptr<DevMem> lut;      // int32 local -> global dictId; replaced, never rewritten, on dictionary growth
  uint64_t lut_version = ~0ull;
  int32_t lut_off = -1;             // >= 0: the LUT is lut[i] = lut_off + i (KCol.lut_off)
  // accumulator operand read through the table-global value arrays (ensure_value_map): the global dictId of local
  // id 0 (-1: the segment's own arrays) and the KCol.gaps thresholds
  uint64_t vmap_version = ~0ull;
  int32_t vgap_first = -1;
  std::vector<uint32_t> vgaps;
  int64_t* d_key = nullptr;
  double* d_val = nullptr;
  bool key_affine = false;          // INT / LONG dictionary of consecutive values: d_key[i] = key_base + i
  int64_t key_base = 0;
  std::shared_ptr<InvIndex> inv;    // bitmap inverted index, if attached
  std::shared_ptr<const RangeIdx> rng;  // range index, if attached (RANGE leaves: RangeIndexBasedFilterOperator)
  // raw (no-dictionary) column: d_key / d_val hold the values per doc (read through the table's identity $docId
  // forward index), raw_min / raw_max bound integer sums
  bool raw = false;
  int64_t raw_min = 0, raw_max = 0;
};

// A pinned star-tree (pgpu_attach_startree): one device block holding the nodes, the star-tree documents'
// dimension forward indexes and the pre-aggregated metric arrays.
struct StarTreeDev {
  int32_t num_dims = 0, num_nodes = 0, num_docs = 0;
  std::vector<int32_t> dim_cols, dim_bits;
  std::vector<pgpu_agg> metrics;
  void* d_block = nullptr;
  int64_t bytes = 0;
  const int32_t* d_nodes = nullptr;
  std::vector<const uint32_t*> d_dim_fwd;
  std::vector<const double*> d_mf;
  std::vector<const int64_t*> d_mc;
  int dim_of(int col) const {
    for (int d = 0; d < num_dims; ++d) if (dim_cols[d] == col) return d;
    return -1;
  }
  int pair(int fn, int col) const {  // AggregationFunctionColumnPair lookup (COUNT: column ignored)
    for (size_t m = 0; m < metrics.size(); ++m)
      if (metrics[m].fn == fn && (fn == PGPU_AGG_COUNT || metrics[m].column == col)) return (int)m;
    return -1;
  }
};

// A pinned segment.  Reference-counted like Pinot's SegmentDataManager (acquire / release per query,
// BaseTableDataManager.java:245-258): the table and every plan that references the segment hold it, so an unpin
// while a query still runs defers the device free until that query's plan is destroyed.
struct Segment {
  int64_t handle = 0;
  int32_t num_docs = 0;
  void* d_block = nullptr;
  std::vector<Column> cols;
  std::unique_ptr<StarTreeDev> star;
  Segment() = default;
  Segment(const Segment&) = delete;
  Segment& operator=(const Segment&) = delete;
  ~Segment() {
    for (auto& c : cols) {
      if (c.d_key) hipFree(c.d_key);
      if (c.d_val) hipFree(c.d_val);
    }
    if (d_block) hipFree(d_block);
    if (star && star->d_block) hipFree(star->d_block);
  }
};

// What a plan keeps alive while it exists (shared by the copies a plan-cache hit makes): its segments and the LUT
// versions its records point at.
struct PlanRefs {
  std::vector<std::shared_ptr<Segment>> segs;
  std::vector<std::shared_ptr<DevMem>> luts;  // LUTs, value maps and table-global value arrays the records point at
};
// An accumulator column's value arrays in one plan segment, as planned (ensure_value_map): the segment's own (keys /
// vals null), or the table's from the segment's first value on, with the gap thresholds (KCol.gaps).
struct ValMap {
  const int64_t* keys = nullptr;
  const double* vals = nullptr;
  int32_t ngaps = 0;
  std::array<uint32_t, kMaxValueGaps> gaps{};
};
// A group-by key column's LUT in one plan segment, as planned: lut null = consecutive run (global = id + off).
struct KeyLut {
  const int32_t* lut = nullptr;
  int32_t off = 0;
};

// Device copy of a cached plan's launch inputs: the per-segment records (SET pointers patched to its own bitset
// words) and the tile -> record map.  A repeated query (a cache hit) launches straight from it -- no record upload,
// no tile expansion -- so its GPU timeline starts with the scan.  The first execution of the cached plan builds it
// on its stream and records `built`; later executions (any stream) wait on that event.
struct DeviceImage {
  std::mutex mu;
  std::atomic<bool> uploaded{false};
  bool ready = false;  // `built` has completed: later executions need no stream wait (under mu)
  hipEvent_t built = nullptr;
  DevBuf segrec, sets, tile_seg;
  ~DeviceImage() {
    if (built) hipEventDestroy(built);
    segrec.release();
    sets.release();
    tile_seg.release();
  }
};

struct Scratch {
  DevBuf docbits, bittasks, bitblocks;  // inverted-index leaves: materialised docId bitmaps and their container tasks
  DevBuf rawtasks;                      // raw-value leaves: tasks, jobs, IN keys (one buffer)
  HostPinned rawstage;
  DevBuf segrec, sets, slab, table, hash_keys, stats, ckeys, cslots, counter, bitmap, tile_seg, starrec, starwork;
  DevBuf part_start, block_off, rec_key, rec_val;  // partitioned group-by (large dense key spaces)
  DevBuf rec_key32;                                // hashed partitions: whole record keys
  DevBuf stage_keys;  // ARRAY_MAP key spaces: the prefix hash table
  DevBuf coarse_fill, fine_fill, mid_key, mid_val;
  DevBuf leap_maps, mask_jobs, leaf_masks;  // numEntriesScannedInFilter: LEAP2 maps, GENERIC leaf bitmaps
  DevBuf xcursor;                       // cross-GPU exchange: per-owner record cursors
  DevBuf xsend, xrecv, xshard;          // pgpu_plan_combine: exported / received records, the reduce-scattered shard
  DevBuf hsort;                         // hash-mode finalize: the decoded columns / compact form
  DevBuf part_mm;                       // hashed partitions: each partition's slot ranges (KPartParams.out_mm)
  HostPinned xstage;                    // their initial values (pinned: the upload is asynchronous)
  // Pinned staging: `stage` is the source of the execution's asynchronous uploads (records, bitsets); `readback`
  // receives finalize's copies.  Separate buffers, because a finalize that had to grow the upload buffer would
  // free it while its uploads may still be queued behind other queries' work on a shared stream.
  HostPinned stage, readback, starstage, bitstage, maskstage;
  std::vector<uint8_t> starrec_sent;  // the star-tree records last uploaded to `starrec` (a repeat skips the copy)
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  std::vector<hipEvent_t> cev;  // per scan launch: (start, end)
  // A query that timed out returns while its device work may still run (wait_plan): the scratch goes back to the
  // pool marked abandoned and is not handed out again before `busy` (recorded after that work) has completed.
  hipEvent_t busy = nullptr;
  bool abandoned = false;
  std::shared_ptr<DeviceImage> image;  // the plan image the last execution read (kept while it may still run)
  // device bytes held (acquire_scratch prefers the scratch that has grown the most)
  size_t footprint() const {
    size_t n = 0;
    for (const DevBuf* b : {&docbits, &bittasks, &bitblocks, &rawtasks, &segrec, &sets, &slab, &table, &hash_keys,
                            &stats, &ckeys, &cslots, &counter, &bitmap, &tile_seg, &starrec, &starwork, &part_start,
                            &block_off, &rec_key, &rec_val, &rec_key32, &stage_keys, &coarse_fill, &fine_fill,
                            &mid_key, &mid_val, &leap_maps, &mask_jobs, &leaf_masks, &hsort, &part_mm})
      n += b->cap;
    return n;
  }
  void release() {
    if (busy) { hipEventDestroy(busy); busy = nullptr; }
    abandoned = false;
    for (auto& e : cev) if (e) hipEventDestroy(e);
    cev.clear();
    docbits.release(); bittasks.release(); bitblocks.release(); rawtasks.release(); rawstage.release();
    segrec.release(); tile_seg.release(); sets.release(); slab.release(); table.release(); hash_keys.release(); stats.release();
    ckeys.release(); cslots.release(); counter.release(); bitmap.release(); stage.release(); readback.release();
    starrec.release();
    starrec_sent.clear();
    starstage.release();
    bitstage.release();
    starwork.release();
    part_start.release(); block_off.release(); rec_key.release(); rec_val.release(); stage_keys.release();
    coarse_fill.release(); fine_fill.release(); mid_key.release(); mid_val.release();
    leap_maps.release(); mask_jobs.release(); leaf_masks.release(); maskstage.release();
    xcursor.release(); xstage.release(); xsend.release(); xrecv.release(); xshard.release(); hsort.release(); part_mm.release();
    for (auto& e : ev) if (e) { hipEventDestroy(e); e = nullptr; }
  }
};

struct GenScratch {
  DevBuf pos, presence, code_to_pos, cdf, pos_to_id;
};

}  // namespace

// pgpu_config_default: the library's settings (include/pinotgpu.h documents each field).
pgpu_config default_config() {
  pgpu_config c;
  memset(&c, 0, sizeof c);
  c.struct_size = (int32_t)sizeof(pgpu_config);
  c.plan_cache = 1;
  c.partitioned_group_by = 1;
  c.hash_partitions = 1;
  c.hash_partition_bits = 14;
  c.hash_partition_lds_kb = 0;
  c.lds_table_kb = 112;
  c.plan_chunk_segments = 4096;
  c.stream_chunks = 1;
  c.compact_results = 1;
  c.star_tree_workgroups = 0;
  c.dense_selectivity = 0.25;
  return c;
}

struct pgpu_table_s {
  int device = 0;
  // executor settings (pgpu_table_set_config); plans copy them when they are made
  mutable std::mutex cfg_mu;
  pgpu_config cfg = default_config();
  std::vector<std::string> names;
  std::vector<int32_t> types;
  std::mutex mu;
  std::unordered_map<int64_t, std::shared_ptr<Segment>> segments;
  std::vector<std::shared_ptr<Segment>> by_handle;  // handle -> segment (handles are dense), null once unpinned
  int64_t next_handle = 1;
  std::vector<std::shared_ptr<const Dict>> global;  // current snapshot per column (replaced under mu)
  std::vector<uint64_t> global_version;
  // Table-global value arrays of accumulator columns (ensure_global_values): the global dictionary's values as
  // order-preserving int64 keys and as doubles, indexed by global dictId -- one array every segment's gathers share,
  // instead of each segment's own (C2's md: 100 dictionaries of 800 KB competing for the XCD L2s)
  struct GlobalValues {
    uint64_t version = ~0ull;
    std::shared_ptr<DevMem> keys, vals;
  };
  std::vector<GlobalValues> gvalues;
  hipStream_t stream = nullptr;
  std::vector<std::unique_ptr<Scratch>> scratch_pool;
  GenScratch gen;
  std::shared_ptr<ResultPool> result_pool = std::make_shared<ResultPool>();
  int64_t device_bytes = 0;
  int num_cus = 256;
  // The virtual $docId column (identity forward index + values, docs [0, docid_n)): the hidden MIN($docId) slot of
  // the first-seen numGroupsLimit emulation reads it like any other column.
  uint32_t* d_docid_fwd = nullptr;
  int64_t* d_docid_key = nullptr;
  int docid_bits = 0;
  int64_t docid_n = 0;
  std::vector<void*> retired;  // replaced $docId buffers (plans built earlier may still point at them)
  // Compiled-plan cache (pgpu_plan_create / _create_execute): the host image of a plan -- per-segment records with
  // the predicate literals translated to dictId ranges / sets, launch configuration, statistics classification --
  // keyed by the query bytes, the segment list and `version`, which every change of pinned state bumps (pin, unpin,
  // index attach, dictionary growth).  A repeated query (a dashboard refresh) skips the host translation; the
  // device work runs in full every time.
  std::atomic<uint64_t> version{1};
  std::mutex cache_mu;
  std::list<std::pair<std::string, std::shared_ptr<pgpu_plan_s>>> plan_cache;  // most recent first
  // Query deadlines on the device (pgpu_query.end_time_ms): one reading `clock_ticks` of the device's constant-rate
  // wall clock, taken no earlier than host epoch time `clock_host_us`, maps epoch time to clock ticks; refreshed
  // every 10 s (calibrate_clock).
  std::mutex clock_mu;
  hipStream_t clock_stream = nullptr;
  uint64_t* clock_pinned = nullptr;
  double clock_rate_khz = 0;
  double clock_host_us = 0;
  uint64_t clock_ticks = 0;
  double clock_steady_us = -1;
};

int pgpu::table_dict_view(pgpu_table t, int col, DictView* out) {
  if (!t || col < 0 || col >= (int)t->names.size()) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad column %d", col);
  std::shared_ptr<const Dict> d;
  {
    std::lock_guard<std::mutex> g(t->mu);
    d = t->global[col];
  }
  out->keep = d;
  out->type = d->type;
  out->iv = &d->iv;
  out->dv = &d->dv;
  out->sv = &d->sv;
  out->name = t->names[col];
  return 0;
}

int pgpu::result_key_dict_view(const pgpu_result_s* r, pgpu_table t, int key, DictView* out) {
  if (!r || key < 0 || key >= r->num_keys) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad group-by key %d", key);
  if ((int)r->key_dicts.size() <= key || !r->key_dicts[key]) return table_dict_view(t, r->key_cols[key], out);
  auto d = std::static_pointer_cast<const Dict>(r->key_dicts[key]);
  out->keep = d;
  out->type = d->type;
  out->iv = &d->iv;
  out->dv = &d->dv;
  out->sv = &d->sv;
  out->name = t && r->key_cols[key] >= 0 && r->key_cols[key] < (int)t->names.size() ? t->names[r->key_cols[key]] : "";
  return 0;
}

namespace {

// ------------------------------------------------------------------------------------------------ dictionaries
int parse_dictionary(int type, const pgpu_column_buffers& cb, Dict* d) {
  d->type = type;
  const int64_t card = cb.cardinality;
  if (card < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "negative cardinality");
  const int w = cb.entry_width;
  if (card > 0 && (!cb.dict || cb.dict_len < card * (int64_t)w))
    return fail(PGPU_ERR_INVALID_ARGUMENT, "dictionary buffer too small (%lld < %lld x %d)", (long long)cb.dict_len,
                (long long)card, w);
  switch (type) {
    case PGPU_INT:
      if (w != 4) return fail(PGPU_ERR_INVALID_ARGUMENT, "INT dictionary entry width %d", w);
      d->iv.resize(card);
      for (int64_t i = 0; i < card; ++i) d->iv[i] = (int32_t)rd_be32(cb.dict + i * 4);
      break;
    case PGPU_LONG:
      if (w != 8) return fail(PGPU_ERR_INVALID_ARGUMENT, "LONG dictionary entry width %d", w);
      d->iv.resize(card);
      for (int64_t i = 0; i < card; ++i) d->iv[i] = (int64_t)rd_be64(cb.dict + i * 8);
      break;
    case PGPU_FLOAT:
      if (w != 4) return fail(PGPU_ERR_INVALID_ARGUMENT, "FLOAT dictionary entry width %d", w);
      d->dv.resize(card);
      for (int64_t i = 0; i < card; ++i) {
        uint32_t u = rd_be32(cb.dict + i * 4);
        float f;
        memcpy(&f, &u, 4);
        d->dv[i] = f;
      }
      break;
    case PGPU_DOUBLE:
      if (w != 8) return fail(PGPU_ERR_INVALID_ARGUMENT, "DOUBLE dictionary entry width %d", w);
      d->dv.resize(card);
      for (int64_t i = 0; i < card; ++i) {
        uint64_t u = rd_be64(cb.dict + i * 8);
        memcpy(&d->dv[i], &u, 8);
      }
      break;
    case PGPU_STRING:
      d->sv.resize(card);
      for (int64_t i = 0; i < card; ++i) {  // FixedByteValueReaderWriter.getUnpaddedString (:57-95)
        const uint8_t* s = cb.dict + i * w;
        int n = 0;
        while (n < w && s[n] != (uint8_t)cb.padding_byte) ++n;
        d->sv[i].assign(reinterpret_cast<const char*>(s), n);
      }
      break;
    default:
      return fail(PGPU_ERR_INVALID_ARGUMENT, "unsupported data type %d", type);
  }
  return 0;
}

bool dbl_less(double a, double b) {  // Double.compare order for the sorted global dictionary
  if (a < b) return true;
  if (a > b) return false;
  int64_t x, y;
  memcpy(&x, &a, 8);
  memcpy(&y, &b, 8);
  return x < y;
}

// Merges sorted `src` into the global dictionary snapshot `g`: a new snapshot replaces it when the union grew.
// Returns true if it grew.
bool merge_dict(std::shared_ptr<const Dict>& g, const Dict& src) {
  const Dict& dst = *g;
  auto out = std::make_shared<Dict>();
  out->type = dst.type;
  if (is_int_type(dst.type)) {
    out->iv.reserve(dst.iv.size() + src.iv.size());
    std::set_union(dst.iv.begin(), dst.iv.end(), src.iv.begin(), src.iv.end(), std::back_inserter(out->iv));
  } else if (is_fp_type(dst.type)) {
    std::vector<double> s = src.dv;
    std::sort(s.begin(), s.end(), dbl_less);
    out->dv.reserve(dst.dv.size() + s.size());
    std::set_union(dst.dv.begin(), dst.dv.end(), s.begin(), s.end(), std::back_inserter(out->dv), dbl_less);
  } else {
    std::vector<std::string> s = src.sv;
    std::sort(s.begin(), s.end());
    out->sv.reserve(dst.sv.size() + s.size());
    std::set_union(dst.sv.begin(), dst.sv.end(), s.begin(), s.end(), std::back_inserter(out->sv));
  }
  if (out->size() == dst.size()) return false;
  out->id = g_dict_ids.fetch_add(1);
  g = std::move(out);
  return true;
}

// BaseImmutableDictionary.insertionIndexOf behind PredicateUtils.getStoredValue (Dictionary.java:49-100,
// BaseImmutableDictionary.java:97-230).  Returns false when the literal does not convert (BadQueryRequest).
int64_t global_index_of(const Dict& g, const Dict& local, size_t i) {
  if (is_int_type(g.type)) {
    auto it = std::lower_bound(g.iv.begin(), g.iv.end(), local.iv[i]);
    return (it != g.iv.end() && *it == local.iv[i]) ? it - g.iv.begin() : -1;
  }
  if (is_fp_type(g.type)) {
    auto it = std::lower_bound(g.dv.begin(), g.dv.end(), local.dv[i], dbl_less);
    return (it != g.dv.end() && !dbl_less(local.dv[i], *it)) ? it - g.dv.begin() : -1;
  }
  auto it = std::lower_bound(g.sv.begin(), g.sv.end(), local.sv[i]);
  return (it != g.sv.end() && *it == local.sv[i]) ? it - g.sv.begin() : -1;
}

// Makes the local->global LUT of (seg, col) current.
int ensure_lut(pgpu_table_s* t, Segment& s, int col, hipStream_t stream) {
  Column& c = s.cols[col];
  if (c.lut_version == t->global_version[col] && c.lut) return 0;
  std::vector<int32_t> lut(std::max<int32_t>(c.card, 1));
  for (int32_t i = 0; i < c.card; ++i) {
    int64_t g = global_index_of(*t->global[col], c.dict, i);
    if (g < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "value missing from the global dictionary (column %d)", col);
    lut[i] = (int32_t)g;
  }
  auto m = std::make_shared<DevMem>();
  HIP_TRY(hipMalloc(&m->p, sizeof(int32_t) * lut.size()));
  if (!c.lut) t->device_bytes += sizeof(int32_t) * lut.size();
  HIP_TRY(hipMemcpyAsync(m->p, lut.data(), sizeof(int32_t) * lut.size(), hipMemcpyHostToDevice, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  c.lut = std::move(m);  // the previous version lives on in the plans that reference it
  c.lut_version = t->global_version[col];
  // strictly increasing (both dictionaries sorted), so the ends decide whether it is a contiguous run
  c.lut_off = c.card > 0 && lut[c.card - 1] - lut[0] == c.card - 1 ? lut[0] : -1;
  return 0;
}

// Dictionary values for aggregation (Dictionary.readDoubleValues, DataFetcher.java:469-478).
int ensure_values(pgpu_table_s* t, Segment& s, int col, hipStream_t stream) {
  Column& c = s.cols[col];
  if (c.d_key) return 0;
  const size_t n = std::max<int32_t>(c.card, 1);
  std::vector<int64_t> key(n, 0);
  std::vector<double> val(n, 0.0);
  for (int32_t i = 0; i < c.card; ++i) {
    if (is_int_type(c.dict.type)) {
      key[i] = c.dict.iv[i];
      val[i] = (double)c.dict.iv[i];
    } else {
      key[i] = double_key(c.dict.dv[i]);
      val[i] = c.dict.dv[i];
    }
  }
  HIP_TRY(hipMalloc(&c.d_key, sizeof(int64_t) * n));
  HIP_TRY(hipMalloc(&c.d_val, sizeof(double) * n));
  t->device_bytes += 16 * n;
  HIP_TRY(hipMemcpyAsync(c.d_key, key.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipMemcpyAsync(c.d_val, val.data(), sizeof(double) * n, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  if (is_int_type(c.dict.type) && c.card > 0) {  // sorted distinct integers: consecutive iff the ends span card
    const __int128 span = (__int128)c.dict.iv[c.card - 1] - (__int128)c.dict.iv[0];
    c.key_affine = span == (__int128)(c.card - 1);
    c.key_base = c.dict.iv[0];
  }
  return 0;
}

// Dictionaries of at least this many entries are read through the table-global value arrays when their segment's
// dictionary lacks at most kMaxValueGaps of the global values (smaller ones stay L2-resident on their own).
#ifndef PGPU_NO_GLOBAL_VALUES  // (defined only by an A/B build of the library: every segment's own arrays)
constexpr int32_t kGlobalValuesMinCard = 8192;
#else
constexpr int32_t kGlobalValuesMinCard = INT32_MAX;
#endif

// The table-global value arrays of `col` for its current global dictionary (under the table mutex).
int ensure_global_values(pgpu_table_s* t, int col, hipStream_t stream) {
  auto& gv = t->gvalues[col];
  if (gv.version == t->global_version[col] && gv.keys) return 0;
  const Dict& g = *t->global[col];
  const size_t n = std::max<size_t>(g.size(), 1);
  std::vector<int64_t> key(n, 0);
  std::vector<double> val(n, 0.0);
  for (size_t i = 0; i < g.size(); ++i) {
    if (is_int_type(g.type)) {
      key[i] = g.iv[i];
      val[i] = (double)g.iv[i];
    } else {
      key[i] = double_key(g.dv[i]);
      val[i] = g.dv[i];
    }
  }
  auto k = std::make_shared<DevMem>(), v = std::make_shared<DevMem>();
  HIP_TRY(hipMalloc(&k->p, sizeof(int64_t) * n));
  HIP_TRY(hipMalloc(&v->p, sizeof(double) * n));
  HIP_TRY(hipMemcpyAsync(k->p, key.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipMemcpyAsync(v->p, val.data(), sizeof(double) * n, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  if (!gv.keys) t->device_bytes += 16 * (int64_t)n;
  gv.keys = std::move(k);  // the previous arrays live on in the plans that reference them
  gv.vals = std::move(v);
  gv.version = t->global_version[col];
  return 0;
}

// How (seg, col)'s local dictIds index the table-global value arrays (under the table mutex): from the global id of
// local id 0 on, skipping the global values the segment's dictionary lacks -- at most kMaxValueGaps of them, as
// thresholds (KCol.gaps, vidx) -- or not at all (dictionaries below kGlobalValuesMinCard, or more missing values: the
// segment's own arrays).
int ensure_value_map(pgpu_table_s* t, Segment& s, int col) {
  Column& c = s.cols[col];
  if (c.vmap_version == t->global_version[col]) return 0;
  c.vgap_first = -1;
  c.vgaps.clear();
  c.vmap_version = t->global_version[col];
  if (c.raw || c.card < kGlobalValuesMinCard) return 0;
  const Dict& g = *t->global[col];
  int64_t prev = -1, first = -1;
  std::vector<uint32_t> gaps;
  for (int32_t i = 0; i < c.card; ++i) {
    const int64_t gi = global_index_of(g, c.dict, i);
    if (gi < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "value missing from the global dictionary (column %d)", col);
    if (i == 0) first = gi;
    // each global id skipped before local id i: a threshold at i, in mapped space (+ the thresholds before it)
    for (int64_t d = i == 0 ? 0 : gi - prev - 1; d > 0; --d) {
      if ((int)gaps.size() == kMaxValueGaps) return 0;
      gaps.push_back((uint32_t)(i + (int64_t)gaps.size()));
    }
    prev = gi;
  }
  c.vgap_first = (int32_t)first;
  c.vgaps = std::move(gaps);
  return 0;
}

int64_t padded_fwd_words(int64_t num_docs, int bits);
int scan_variant(const pgpu_plan_s* P);

// Identity forward index of the virtual $docId column over docs [0, n): Pinot's MSB-first fixed-bit layout of the
// values 0..n-1 (a sorted "dictionary" of docIds), and the values as int64 (the MIN slot's keys).
int ensure_docid(pgpu_table_s* t, int64_t n, hipStream_t stream) {
  if (n <= t->docid_n) return 0;
  int bits = 1;
  while (bits < 31 && (int64_t(1) << bits) < n) ++bits;
  const int64_t words = padded_fwd_words(n, bits);
  std::vector<uint8_t> fwd((size_t)words * 4, 0);
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t bit = (uint64_t)i * bits;
    for (int b = 0; b < bits; ++b)
      if ((i >> (bits - 1 - b)) & 1) fwd[(bit + b) >> 3] |= (uint8_t)(0x80u >> ((bit + b) & 7));
  }
  std::vector<int64_t> key(n);
  for (int64_t i = 0; i < n; ++i) key[i] = i;
  if (t->d_docid_fwd) t->retired.push_back(t->d_docid_fwd);
  if (t->d_docid_key) t->retired.push_back(t->d_docid_key);
  t->d_docid_fwd = nullptr;
  t->d_docid_key = nullptr;
  t->docid_n = 0;
  HIP_TRY(hipMalloc(&t->d_docid_fwd, fwd.size()));
  HIP_TRY(hipMalloc(&t->d_docid_key, (size_t)n * 8));
  HIP_TRY(hipMemcpyAsync(t->d_docid_fwd, fwd.data(), fwd.size(), hipMemcpyHostToDevice, stream));
  HIP_TRY(hipMemcpyAsync(t->d_docid_key, key.data(), (size_t)n * 8, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  t->docid_bits = bits;
  t->docid_n = n;
  t->device_bytes += (int64_t)fwd.size() + n * 8;
  return 0;
}

// Unpin accounting: the segment's device bytes leave the table's total now; the memory itself goes with the last
// reference (~Segment).
void account_unpin(pgpu_table_s* t, const Segment* s) {
  int64_t fwd_words = 0;
  for (const auto& c : s->cols) {
    if (c.inv) t->device_bytes -= c.inv->bytes;
    t->device_bytes -= (c.lut ? 4 * std::max(c.card, 1) : 0) +
                       (c.d_key ? 16 * (c.raw ? raw_padded_docs(s->num_docs) : std::max(c.card, 1)) : 0);
    if (!c.raw) fwd_words += (c.fwd_words + 63) & ~int64_t(63);
  }
  if (s->d_block) t->device_bytes -= std::max<int64_t>(fwd_words, 64) * 4;
  if (s->star) t->device_bytes -= s->star->bytes;
}

int64_t padded_fwd_words(int64_t num_docs, int bits) {
  return ((num_docs + kTileDocs - 1) / kTileDocs) * (int64_t)kBlock * bits + kFwdPadWords;
}

// LZ4 block decoder (the LZ4 block format of lz4-java's LZ4SafeDecompressor, behind Pinot's LZ4Decompressor /
// LZ4WithLengthDecompressor, seglocal/io/compression/LZ4Decompressor.java:40-50).  Every length and offset is
// checked against both buffers; returns the decoded length or -1.
int64_t lz4_decode_block(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap) {
  const uint8_t* ip = src;
  const uint8_t* const iend = src + n;
  uint8_t* op = dst;
  uint8_t* const oend = dst + cap;
  auto ext_len = [&](int64_t& len) -> bool {  // 255-continued length bytes
    uint32_t b;
    do {
      if (ip >= iend) return false;
      b = *ip++;
      len += b;
    } while (b == 255);
    return true;
  };
  while (ip < iend) {
    const uint32_t token = *ip++;
    int64_t lit = token >> 4;
    if (lit == 15 && !ext_len(lit)) return -1;
    if (lit > iend - ip || lit > oend - op) return -1;
    memcpy(op, ip, (size_t)lit);
    ip += lit;
    op += lit;
    if (ip == iend) return op - dst;  // last sequence: literals only
    if (iend - ip < 2) return -1;
    const int64_t off = (int64_t)ip[0] | ((int64_t)ip[1] << 8);
    ip += 2;
    int64_t ml = token & 15;
    if (ml == 15 && !ext_len(ml)) return -1;
    ml += 4;
    if (off == 0 || off > op - dst || ml > oend - op) return -1;
    const uint8_t* m = op - off;
    if (off >= ml) {
      memcpy(op, m, (size_t)ml);
      op += ml;
    } else {  // overlapping: the last `off` bytes repeat
      for (int64_t k = 0; k < ml; ++k) op[k] = m[k];
      op += ml;
    }
  }
  return -1;  // an empty block has no token
}

// A raw fixed-width forward index (FixedByteChunkSVForwardIndexWriter; BaseChunkSVForwardIndexReader.java:56-154):
// the header (version, numChunks, numDocsPerChunk, sizeOfEntry; versions 2-3: totalDocs, compression type,
// dataHeaderStart), the chunk offsets (int / long), the chunks -- PASS_THROUGH (read in place), LZ4 or
// LZ4_LENGTH_PREFIXED (ChunkCompressionType 3 / 4, each chunk decoded on its own: getChunkPosition, the last
// chunk to the end of the buffer).  Out: per doc the int64 key the kernels read (integer value, or the
// order-preserving key of the double; NaN canonical, as Double.doubleToLongBits) and the double value.
struct RawValues {
  std::vector<int64_t> key;
  std::vector<double> val;
  int64_t lo = 0, hi = 0;  // integer range (sum bounds)
};
int decode_raw_forward_index(int type, const uint8_t* b, int64_t n, int32_t num_docs, int c, RawValues* out) {
  if (type == PGPU_STRING) return fail(PGPU_ERR_UNSUPPORTED, "column %d: raw STRING columns are not on the GPU path", c);
  if (!b || n < 16) return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: raw forward index too short", c);
  const int32_t version = (int32_t)rd_be32(b), num_chunks = (int32_t)rd_be32(b + 4);
  const int32_t per_chunk = (int32_t)rd_be32(b + 8), size = (int32_t)rd_be32(b + 12);
  if (version != 2 && version != 3)
    return fail(PGPU_ERR_UNSUPPORTED, "column %d: raw forward index version %d (2 and 3 are read)", c, version);
  if (n < 28) return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: raw forward index header truncated", c);
  const int32_t total = (int32_t)rd_be32(b + 16), compression = (int32_t)rd_be32(b + 20);
  const int32_t header_start = (int32_t)rd_be32(b + 24);
  // ChunkCompressionType: PASS_THROUGH 0, SNAPPY 1, ZSTANDARD 2, LZ4 3, LZ4_LENGTH_PREFIXED 4
  if (compression != 0 && compression != 3 && compression != 4)
    return fail(PGPU_ERR_UNSUPPORTED, "column %d: raw chunk compression type %d (PASS_THROUGH, LZ4 and "
                "LZ4_LENGTH_PREFIXED are read)", c, compression);
  const int want = (type == PGPU_INT || type == PGPU_FLOAT) ? 4 : 8;
  if (size != want) return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: raw entry size %d, type needs %d", c, size, want);
  if (num_chunks < 0 || per_chunk <= 0 || total < num_docs || (int64_t)num_chunks * per_chunk < num_docs)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: raw forward index covers %d docs, segment has %d", c, total,
                num_docs);
  const int entry = version == 2 ? 4 : 8;
  const int64_t data = (int64_t)header_start + (int64_t)num_chunks * entry;
  if (header_start < 28 || data > n || (compression == 0 && data + (int64_t)num_docs * size > n))
    return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: raw forward index too short for %d docs", c, num_docs);
  // A chunk decodes to at most min(numDocsPerChunk, totalDocs) entries, and an LZ4 block expands at most ~255x
  // (each sequence byte of a match length stands for <= 255 output bytes): a header claiming more is rejected
  // before anything is allocated.
  const int64_t chunk_bytes = compression ? std::min<int64_t>(per_chunk, total) * size : 0;
  if (compression && chunk_bytes > (n - data) * 256 + 64)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: raw chunk of %d docs cannot come from a %lld-byte index", c,
                per_chunk, (long long)n);
  std::vector<uint8_t> chunk;
  try {
    out->key.assign(std::max<int32_t>(num_docs, 1), 0);
    out->val.assign(std::max<int32_t>(num_docs, 1), 0.0);
    chunk.resize((size_t)chunk_bytes);
  } catch (const std::bad_alloc&) {
    return fail(PGPU_ERR_OUT_OF_MEMORY, "column %d: host memory for %d raw values", c, num_docs);
  }
  int64_t lo = INT64_MAX, hi = INT64_MIN;
  for (int64_t k = 0, d0 = 0; d0 < num_docs; ++k, d0 += per_chunk) {
    const int64_t nd = std::min<int64_t>(per_chunk, num_docs - d0);
    const uint8_t* v = b + data + d0 * size;
    if (compression) {
      auto chunk_pos = [&](int64_t i) {
        const uint8_t* e = b + header_start + i * entry;
        return entry == 4 ? (int64_t)rd_be32(e) : (int64_t)rd_be64(e);
      };
      const int64_t pos = chunk_pos(k), end = k + 1 < num_chunks ? chunk_pos(k + 1) : n;
      if (pos < data || end < pos || end > n)
        return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: chunk %lld outside the forward index", c, (long long)k);
      int64_t skip = compression == 4 ? 4 : 0;  // LZ4WithLength: little-endian decompressed length first
      if (end - pos < skip) return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: chunk %lld truncated", c, (long long)k);
      const int64_t got = lz4_decode_block(b + pos + skip, end - pos - skip, chunk.data(), (int64_t)chunk.size());
      if (got < nd * size)
        return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: LZ4 chunk %lld is malformed or short", c, (long long)k);
      v = chunk.data();
    }
    for (int64_t i = 0; i < nd; ++i, v += size) {
      const int64_t d = d0 + i;
      switch (type) {
        case PGPU_INT: { const int64_t x = (int32_t)rd_be32(v); out->key[d] = x; out->val[d] = (double)x; lo = std::min(lo, x); hi = std::max(hi, x); break; }
        case PGPU_LONG: { const int64_t x = (int64_t)rd_be64(v); out->key[d] = x; out->val[d] = (double)x; lo = std::min(lo, x); hi = std::max(hi, x); break; }
        case PGPU_FLOAT: {
          const uint32_t u = rd_be32(v);
          float f;
          memcpy(&f, &u, 4);
          out->val[d] = (double)f;
          out->key[d] = double_key(std::isnan(out->val[d]) ? kCanonicalNaN : out->val[d]);
          break;
        }
        default: {
          const uint64_t u = rd_be64(v);
          double x;
          memcpy(&x, &u, 8);
          out->val[d] = x;
          out->key[d] = double_key(std::isnan(x) ? kCanonicalNaN : x);
        }
      }
    }
  }
  out->lo = num_docs > 0 && lo <= hi ? lo : 0;
  out->hi = num_docs > 0 && lo <= hi ? hi : 0;
  return 0;
}

int parse_raw_column(int type, const pgpu_column_buffers& cb, int32_t num_docs, int c, Column* col, RawValues* out) {
  TRY(decode_raw_forward_index(type, cb.fwd, cb.fwd_len, num_docs, c, out));
  col->raw = true;
  col->card = 0;
  col->bits = 0;
  col->fwd_bytes = cb.fwd_len;
  col->raw_min = out->lo;
  col->raw_max = out->hi;
  return 0;
}

// Registers a segment whose columns have parsed dictionaries and device forward indexes.
void plan_cache_clear(pgpu_table_s* t);

int64_t register_segment(pgpu_table_s* t, std::unique_ptr<Segment> seg_in) {
  std::shared_ptr<Segment> seg(std::move(seg_in));
  t->version++;
  for (size_t c = 0; c < seg->cols.size(); ++c)
    if (merge_dict(t->global[c], seg->cols[c].dict)) t->global_version[c]++;
  int64_t h = t->next_handle++;
  seg->handle = h;
  if ((int64_t)t->by_handle.size() <= h) t->by_handle.resize(h + 1);
  t->by_handle[h] = seg;
  t->segments[h] = std::move(seg);
  plan_cache_clear(t);
  return h;
}

// ------------------------------------------------------------------------------------------------ plans
struct LeafHost {
  int32_t kind = LEAF_NONE, negate = 0;
  uint32_t lo = 0, span = 0;
  uint32_t dict_lo = 0, dict_span = 0;  // LEAF_DOCRANGE: the dictId range it came from (star-tree matching)
  std::vector<uint32_t> set;  // bitset words for LEAF_SET
  std::vector<int32_t> inv_ids;  // LEAF_BITMAP: matching dictIds whose inverted-index bitmaps are ORed
  std::vector<int64_t> raw;      // LEAF_RAW_RANGE: inclusive key bounds {lo, hi}; LEAF_RAW_IN: sorted distinct keys
  double inv_frac = 0;           // LEAF_BITMAP: fraction of the segment's docs in those bitmaps
};

enum Tri { T_NONE = 0, T_ALL = 1, T_VAR = 2 };

// One scan launch of a plan: a contiguous run of segment records (tile_base relative to tile_begin), the set_fix
// entries and SET bitset words they own.
struct LaunchChunk {
  int64_t rec_begin = 0, num_recs = 0, tile_begin = 0, num_tiles = 0;
  int64_t fix_begin = 0, fix_end = 0, set_begin = 0, set_end = 0;
};

// Streamed execution requested by pgpu_plan_create_execute.
struct StreamExec {
  hipStream_t stream = nullptr;
  void* d_table = nullptr;
};

}  // namespace

pgpu_config table_config(const pgpu_table_s* t) {
  std::lock_guard<std::mutex> g(t->cfg_mu);
  return t->cfg;
}

struct pgpu_plan_s {
  pgpu_config cfg = default_config();  // the table's settings when the plan was made
  pgpu_table_s* table = nullptr;
  std::vector<Segment*> segs;
  std::shared_ptr<PlanRefs> refs;         // keeps segs and the LUTs the records point at alive
  std::vector<KeyLut> key_lut;            // [segment][group-by column] LUT as planned (taken under the table mutex)
  std::vector<int32_t> val_cols;          // accumulator table columns with table-global value arrays somewhere
  std::vector<ValMap> val_map;            // [segment][val_cols index] as planned
  const uint32_t* docid_fwd = nullptr;    // the $docId column as planned (identity forward index + values)
  const int64_t* docid_key = nullptr;
  int docid_bits = 0;
  std::vector<int32_t> query_cols;        // table column of each query column slot
  int num_leaves = 0;
  std::vector<int32_t> leaf_slot;         // query column slot of each leaf
  std::vector<int32_t> ops;               // encoded postfix program
  bool pure_and = false;
  int max_depth = 0;
  std::vector<int32_t> key_cols;          // table columns of group-by expressions
  std::vector<std::shared_ptr<const Dict>> key_dicts;  // global dictionary snapshots the key space is built on
  std::vector<int64_t> key_card;          // key digit ranges (global cardinalities, or the filter's bound)
  std::vector<int64_t> key_off;           // first global id of each key digit (filter-restricted key spaces)
  int64_t key_bias = 0;                   // sum key_off[j] * key_stride[j]: subtracted from composite keys
  std::vector<int64_t> key_stride;
  int64_t num_keys = 0;                   // dense G or hash capacity
  int mode = MODE_LDS;
  std::vector<int32_t> slot_kind, slot_col, slot_tcol;
  std::vector<int32_t> agg_fn, agg_slot, agg_col;   // per aggregation: fn, value slot (or -1), table column
  int num_projected = 0;
  // per-segment compiled data
  std::vector<uint8_t> segrec;            // host image of the KSeg records
  int seg_stride = 0;
  std::vector<uint32_t> set_words;        // all SET bitsets back to back
  std::vector<std::pair<int64_t, int64_t>> set_fix;  // (offset of KLeaf.set field in segrec, word offset)
  bool no_inverted = false;               // keep scan leaves (pgpu_filter_bitmap's single-segment path)
  int64_t docbit_words = 0;               // LEAF_BITMAP docId bitmaps of the plan (device words)
  std::vector<std::pair<int64_t, int64_t>> bit_fix;  // (offset of KLeaf.set field in segrec, docbits word offset)
  std::vector<KBitTask> bit_tasks;        // containers ORed into the docbits by inv_materialize_kernel
  std::vector<KBitBlock> bit_blocks;      // every 65536-doc block of the docbits, with its tasks
  std::vector<KRawTask> raw_tasks;        // raw-value leaves evaluated into docbits regions (raw_leaf_bitmap_kernel)
  std::vector<int64_t> raw_vals;          // their IN / NOT_IN keys
  std::vector<std::shared_ptr<InvIndex>> inv_refs;  // inverted indexes the bit tasks point into (kept alive)
  std::shared_ptr<DeviceImage> image;     // cached plans: device-resident records / tile map (one-launch plans)
  int64_t num_tiles = 0;
  int tile_shift = 0;                     // small plans: 8192-doc tiles split in 2^tile_shift (KParams.tile_shift)
  int64_t total_docs = 0;
  int64_t scanned_entries_model = 0;      // numEntriesScannedInFilter of the STATS_CONST segments (host)
  bool in_kernel_stats = false;           // the scan kernel counts STATS_CHAIN / STATS_LEAP2 segments
  bool any_leap2 = false;
  bool leap_reserved = false;             // the scan's LDS holds the LEAP2 bytes (configure); maps allocated
  // STATS_GENERIC segments: their filter tree, replayed on the host over the leaves' device bitmaps
  struct GenericStat { int64_t rec; int32_t num_docs; StatTree tree; int64_t out_word; };
  std::vector<GenericStat> generic;
  int64_t generic_words = 0;
  std::vector<int> leaf_perm;             // evaluation position -> predicate index
  int64_t post_exempt_docs = 0;           // aggregation-only: docs of segments answered from metadata / dictionary
  int segments_matched_filter = 0;
  int64_t leaf_kinds[kLeafKinds] = {};     // (segment, leaf) pairs of the scanned segments by kernel leaf kind
  std::vector<uint8_t> seg_scanned;       // per plan segment: 1 = scanned (filter not folded to empty)
  int grid = 0;
  size_t lds_bytes = 0;
  bool dense = false;                     // direct kernel instance with whole-group decode (dense tiles)
  // dense plans whose group-by columns need no LUT and whose operands no dictionary lookup in any segment, with no
  // double sums: the dense instance compiled without those gathers (aggregate_batch's SIMPLE; fewer registers)
  bool dense_simple = false;
  bool gathers = false;                   // some segment's key LUT or operand dictionary is read (not simple)
  bool pair_variant = false;              // sparse instance with the index + scan pair (variant 3)
  bool fast_variant = false;              // sparse instance for pure-AND plans of <= kFastLeaves leaves (variant 4)
  bool fast_wide = false;                 // ... with 4-doc lane batches: estimated selectivity >= 1/16 (variant 5)
  bool partitioned = false;               // large dense table: partitioned group-by (partition.h) instead of atomics
  std::vector<LaunchChunk> chunks;        // scan launches (one unless the plan was streamed)
  int launches_done = 0;
  int64_t set_words_bound = 0;            // streamed plans: upper bound of the SET bitset words
  int64_t tile_bound = 0;                 // streamed plans: upper bound of the tiles
  int part_shift = 0, num_parts = 0, part_grid = 0;
  int part_grid_staged[2] = {0, 0};  // the grid when K8c runs staged (u32 / u64 records): set at the first execution
  size_t part_lds = 0;
  std::vector<int32_t> stream_col, stream_f64, slot_stream;
  bool part_val32 = false;  // KPartParams.val32
  // MODE_HASH plans over key spaces < 2^31: hashed partitions (KPartParams.hashed, K8h) instead of the global hash
  // table.  part_hash_live: the last execution's groups are the compacted records in Scratch::ckeys (count in
  // Scratch::counter) and no table was built; finalize reads them as is, an exchange first materialises the table.
  bool part_hash = false, part_hash_live = false;
  int part_pbits = 0, part_sbits = 0;
  int64_t part_pack_min = 0, part_pack_range = -1;  // the single stream's value range (-1: none)
  double sel_estimate = 1.0;              // estimated filter selectivity (uniform dictIds)
  int64_t sel_docs = 0;
  Scratch* scratch = nullptr;
  hipStream_t last_stream = nullptr;
  bool executed = false;
  const void* d_table_used = nullptr;
  bool hash = false;
  // numGroupsLimit (InstancePlanMakerImplV2.java:70): a segment whose group-key space (product of its local
  // cardinalities) exceeds the limit may drop groups in first-seen docId order (DictionaryBasedGroupKeyGenerator
  // IntGroupIdMap :1101-1113).  If such a plan produces more than `limit` groups in total, Pinot's truncation could
  // apply and the GPU result is not reported (PGPU_ERR_UNSUPPORTED: the caller runs Pinot's own operator).
  int64_t num_groups_limit = 0;
  bool limit_sensitive = false;
  // pgpu_query.end_time_ms (QueryContext.getEndTimeMs) of the query being run: set per query, not cached
  int64_t end_time_ms = 0;
  int64_t exec_start_ms = 0;
  int cancel = 0;                         // pgpu_plan_cancel (__atomic_* access: another thread sets it)
  // key spaces beyond 64 bits (KParams.num_stages): per stage its end column, table slots, the next group's key
  // space; stage_space holds every group's key space (the last group's too)
  std::vector<int32_t> stage_end;
  std::vector<int64_t> stage_cap, stage_mult, stage_space;
  unsigned long long* d_stats = nullptr;  // statistics words of the last execution (scratch)
  // cross-GPU exchange of a hash-mode table (pgpu_plan_exchange_*): per-owner group counts of the local table, and
  // the records merged into the owner's table (-1: the table holds the local groups)
  std::vector<int64_t> xchg_counts;
  int64_t merged_records = -1;
  // hash-mode plans: the bound on their groups (table sizing), and the groups the plan's executions found (shared
  // with the plan cache's image and every copy of it: -1 = none yet)
  int64_t group_bound = 0;
  std::shared_ptr<std::atomic<int64_t>> groups_seen;
  // MODE_LDS / MODE_HASH plans: KParams.pack_slot (the COUNT rides in an integer SUM's word; an LDS table has no
  // COUNT row, a hash table's is filled by hash_unpack after the scan)
  int32_t pack_slot = -1;
  int pack_shift = kLdsPackShift;   // the COUNT's bits start here (MODE_HASH: 64 - bits(total docs))
  // pgpu_plan_combine REDUCE_SCATTER: this rank's merged key range [shard_begin, shard_begin + shard_count), slot rows
  // of shard_count words at `shard`; pgpu_plan_finalize reads it
  const void* shard = nullptr;
  int64_t shard_begin = 0, shard_count = 0;
  // pgpu_plan_combine: the slot kinds the plan was planned with, when the combine's agreement changed them (an int64
  // SUM merged as float64), and the communicator whose stream-ordered collectives this execution's finalize waits on
  // (an expired wait aborts it: a peer that never joined leaves them pending).  exec_prologue resets all three, so a
  // plan executed again after a combine runs and finalizes as planned.
  std::vector<int32_t> slot_kind_planned;
  std::shared_ptr<pgpu::Comm> comm_used;  // the communicator of the last combine (shared: outlives pgpu_comm_destroy)
  // First-seen emulation (composite plans, see split_for_groups_limit): parts executed and finalized one after
  // another at finalize, their rows truncated / capped and merged on the host.
  bool first_doc_slot = false;            // this plan carries the hidden MIN($docId) slot (last slot)
  bool composite = false;
  bool pql_cap = false;                   // GroupByCombineOperator's inter-segment cap of 2 x numGroupsLimit
  struct Part {
    std::shared_ptr<pgpu_plan_s> plan;
    std::vector<int32_t> seg_index;       // plan segment positions of the part's segments
    bool first_seen = false;              // rows in first-seen order (map holder)
    bool truncate = false;                // keep the first numGroupsLimit groups (segment key space > the limit)
  };
  std::vector<Part> parts;
  // star-tree segments (StarTreeFilterOperator + StarTreeGroupByExecutor instead of the scan)
  std::vector<KStarSeg> star;                                // host images; pointers patched at execute
  std::vector<std::tuple<int, int, int64_t>> star_match_fix; // (star seg, dim, word offset in set_words)
  std::vector<int64_t> star_work_off;                        // per star seg: byte offset of its scratch
  int64_t star_work_bytes = 0;
  int star_chunks = 1;                    // K6 workgroups per launch batch (persistent)
  int star_batches = 0;                   // K6 launches (kStarMaxSegs segments each)
  int32_t star_range_cache = 0;           // ranges per segment K6 stages in LDS
  size_t star_lds_bytes = 0;
  int32_t star_cache_ints = 0;  // K6 LDS cache of key LUTs + match sets (max over the star-tree segments; 0: off)
  int64_t star_segments = 0;
  int64_t star_docs_read = 0;                                // star-tree documents K6 read (after finalize)
};



namespace {

// Open-addressing table slots for at most `groups` groups: load <= 1/2, a power of two, >= 1024.
int64_t hash_capacity(int64_t groups) {
  const int64_t want = std::max<int64_t>(2 * std::max<int64_t>(groups, 1), 1024);
  int64_t cap = 1;
  while (cap < want) cap <<= 1;
  return cap;
}

// The free scratch that has grown the most: a query then finds its buffers at size, where handing out the first free
// one had a steady stream of repeated queries take a scratch that a smaller query had sized and grow it -- hipFree
// waits for the whole device (C4's star path at 3 queries in flight: one launch of 7 ms in a 20-query run).
Scratch* acquire_scratch(pgpu_table_s* t) {
  std::lock_guard<std::mutex> g(t->mu);
  std::unique_ptr<Scratch>* best = nullptr;
  size_t best_bytes = 0;
  for (auto& s : t->scratch_pool)
    if (s && (!s->abandoned || hipEventQuery(s->busy) != hipErrorNotReady)) {
      const size_t b = s->footprint();
      if (!best || b > best_bytes) {
        best = &s;
        best_bytes = b;
      }
    }
  if (!best) return new Scratch();
  Scratch* r = best->release();
  best->reset();
  r->abandoned = false;
  return r;
}
void release_scratch(pgpu_table_s* t, Scratch* s) {
  if (!s) return;
  std::lock_guard<std::mutex> g(t->mu);
  for (auto& p : t->scratch_pool)
    if (!p) { p.reset(s); return; }
  t->scratch_pool.emplace_back(s);
}

// A predicate literal converted once per query to the column's stored type (PredicateUtils.getStoredValue): the
// per-segment translation below then only binary-searches.  `star` = RangePredicate.UNBOUNDED ("*").
struct Literal {
  bool star = false;
  int64_t i = 0;
  double d = 0.0;
  std::string s;
};
struct ParsedPred {
  std::vector<Literal> lits;
};

// Literal conversion per column type; false = BadQueryRequestException (PredicateEvaluatorProvider.java:85-88).
bool parse_literal(int type, const char* lit, bool allow_star, Literal* out) {
  if (allow_star && strcmp(lit, "*") == 0) { out->star = true; return true; }
  switch (type) {
    case PGPU_INT: return parse_long(lit, INT32_MIN, INT32_MAX, &out->i);
    case PGPU_LONG: return parse_long(lit, INT64_MIN, INT64_MAX, &out->i);
    case PGPU_FLOAT:
      if (!parse_double(lit, &out->d)) return false;
      out->d = (double)(float)out->d;
      return true;
    case PGPU_DOUBLE: return parse_double(lit, &out->d);
    default: out->s = lit; return true;
  }
}

// Dictionary.insertionIndexOf (BaseImmutableDictionary.java:86-120) of a converted literal: index if present,
// else -(insertion point + 1).
// Search of a sorted, duplicate-free numeric dictionary: up to 3 interpolation probes narrow [lo, hi] (dictionaries
// of dense ids / days / uniformly spread values resolve in one probe, touching one cache line instead of the ~14
// of a cold binary search -- planning does one lookup per predicate per segment), then the binary search of
// BaseImmutableDictionary.insertionIndexOf on what is left.  Same result as the plain binary search: probes only
// move the bounds past values known to be smaller / larger.
template <class T>
int sorted_search(const std::vector<T>& a, T v) {
  int lo = 0, hi = (int)a.size() - 1;
  for (int round = 0; round < 3 && lo < hi; ++round) {
    const T a_lo = a[lo], a_hi = a[hi];
    if (!(v > a_lo) || !(v < a_hi)) break;  // at or outside the ends (NaN-free dictionaries)
    // LONG values past 2^53 can round to equal doubles, and +-inf ends give inf / inf: interpolation only while
    // the fraction is a finite number in [0, 1] (the binary search below finishes the job either way).
    const double f = ((double)v - (double)a_lo) / ((double)a_hi - (double)a_lo);
    if (!(f >= 0.0 && f <= 1.0)) break;
    int pos = lo + (int)(f * (double)(hi - lo));
    pos = pos < lo + 1 ? lo + 1 : (pos > hi - 1 ? hi - 1 : pos);
    if (a[pos] < v) lo = pos + 1;
    else if (a[pos] > v) hi = pos - 1;
    else return pos;
  }
  while (lo <= hi) {
    const int mid = (int)(((unsigned)lo + (unsigned)hi) >> 1);
    if (a[mid] < v) lo = mid + 1;
    else if (a[mid] > v) hi = mid - 1;
    else return mid;
  }
  return -(lo + 1);
}

int insertion_index(const Column& c, const Literal& v) {
  const Dict& d = c.dict;
  int lo = 0, hi = (int)d.size() - 1;
  switch (d.type) {
    case PGPU_INT: case PGPU_LONG:
      return sorted_search<int64_t>(d.iv, v.i);
    case PGPU_FLOAT: case PGPU_DOUBLE:
      return sorted_search<double>(d.dv, v.d);
    default: {
      const uint8_t* lv = reinterpret_cast<const uint8_t*>(v.s.data());
      const size_t ln = v.s.size();
      if (c.padding == 0) {
        while (lo <= hi) {
          const int mid = (int)(((unsigned)lo + (unsigned)hi) >> 1);
          const std::string& m = d.sv[mid];
          const int r = cmp_bytes(reinterpret_cast<const uint8_t*>(m.data()), m.size(), lv, ln);
          if (r < 0) lo = mid + 1;
          else if (r > 0) hi = mid - 1;
          else return mid;
        }
      } else {  // legacy non-zero padding: padded comparison (BaseImmutableDictionary.java:215-228)
        std::string padded(v.s);
        if ((int)padded.size() < c.entry_width) padded.append(c.entry_width - padded.size(), (char)c.padding);
        while (lo <= hi) {
          const int mid = (int)(((unsigned)lo + (unsigned)hi) >> 1);
          const uint8_t* m = c.raw_dict.data() + (int64_t)mid * c.entry_width;
          const int r = cmp_bytes(m, c.entry_width, reinterpret_cast<const uint8_t*>(padded.data()), padded.size());
          if (r < 0) lo = mid + 1;
          else if (r > 0) hi = mid - 1;
          else return mid;
        }
      }
      return -(lo + 1);
    }
  }
}

// Converts the literals of predicate `p` for a column of `type`.
int parse_predicate(int type, const pgpu_predicate& p, ParsedPred* out) {
  const int need = p.type == PGPU_PRED_RANGE ? 2 : 1;
  if (p.num_values < need) return fail(PGPU_ERR_INVALID_ARGUMENT, "predicate on column %d needs %d value(s)", p.column, need);
  out->lits.resize(p.num_values);
  for (int i = 0; i < p.num_values; ++i)
    if (!parse_literal(type, p.values[i], p.type == PGPU_PRED_RANGE, &out->lits[i]))
      return fail(PGPU_ERR_BAD_QUERY, "BadQueryRequestException: cannot convert '%s' to the type of column %d",
                  p.values[i], p.column);
  return 0;
}

// FilterOperatorUtils.getLeafFilterOperator (FilterOperatorUtils.java:72-79): an EQ / NOT_EQ / IN / NOT_IN
// predicate on a column with an inverted index (and not sorted: the sorted index wins) becomes a
// BitmapBasedFilterOperator.  The leaf keeps its negate flag: flip(OR(bitmaps of the literals' dictIds)) over
// [0, numDocs) equals the reference's OR over the non-matching dictIds (BitmapBasedFilterOperator.java:73-98).
void to_inverted_leaf(const Column& c, const pgpu_predicate& p, const Segment& s, LeafHost* L) {
  if (!c.inv || c.sorted || (L->kind != LEAF_RANGE && L->kind != LEAF_SET)) return;
  if (p.type != PGPU_PRED_EQ && p.type != PGPU_PRED_NOT_EQ && p.type != PGPU_PRED_IN && p.type != PGPU_PRED_NOT_IN)
    return;
  L->inv_ids.clear();
  if (L->kind == LEAF_RANGE) {
    for (uint32_t i = 0; i < L->span; ++i) L->inv_ids.push_back((int32_t)(L->lo + i));
  } else {
    for (size_t w = 0; w < L->set.size(); ++w)
      for (uint32_t bits = L->set[w]; bits; bits &= bits - 1)
        L->inv_ids.push_back((int32_t)(w * 32 + __builtin_ctz(bits)));
  }
  int64_t docs = 0;
  for (int32_t id : L->inv_ids) docs += c.inv->ids[id].docs;
  L->inv_frac = (double)docs / std::max(1, s.num_docs);
  L->kind = LEAF_BITMAP;
}

// Translates predicate `p` against one segment's column dictionary (dictionary-based PredicateEvaluators).
// `ids` is caller-owned scratch.
int translate_predicate_dict(const Column& c, const pgpu_predicate& p, const ParsedPred& pp, LeafHost* L,
                             std::vector<int>& ids);

// Dictionary-space translation, then on a sorted column a dictId range becomes the docId range of the
// SortedIndexBasedFilterOperator (SortedIndexBasedFilterOperator.java:51-125; dictIds [lo, hi) own docs
// [start(lo), start(hi)) of the SortedIndexReaderImpl pairs).
int translate_predicate(const Column& c, const pgpu_predicate& p, const ParsedPred& pp, LeafHost* L,
                        std::vector<int>& ids) {
  TRY(translate_predicate_dict(c, p, pp, L, ids));
  if (c.sorted && L->kind == LEAF_RANGE) {
    const int32_t d0 = c.sorted_start[L->lo], d1 = c.sorted_start[L->lo + L->span];
    L->dict_lo = L->lo;
    L->dict_span = L->span;
    L->kind = LEAF_DOCRANGE;
    L->lo = (uint32_t)d0;
    L->span = (uint32_t)std::max(0, d1 - d0);
  }
  return 0;
}

int translate_predicate_dict(const Column& c, const pgpu_predicate& p, const ParsedPred& pp, LeafHost* L,
                             std::vector<int>& ids) {
  const int32_t card = c.card;
  switch (p.type) {
    case PGPU_PRED_EQ: {  // EqualsPredicateEvaluatorFactory.java:86-99
      const int ins = insertion_index(c, pp.lits[0]);
      if (ins < 0) L->kind = LEAF_NONE;
      else if (card == 1) L->kind = LEAF_ALL;
      else { L->kind = LEAF_RANGE; L->lo = ins; L->span = 1; }
      return 0;
    }
    case PGPU_PRED_NOT_EQ: {  // NotEqualsPredicateEvaluatorFactory.java:88-102
      const int ins = insertion_index(c, pp.lits[0]);
      if (ins < 0) L->kind = LEAF_ALL;
      else if (card == 1) L->kind = LEAF_NONE;
      else { L->kind = LEAF_RANGE; L->lo = ins; L->span = 1; L->negate = 1; }
      return 0;
    }
    case PGPU_PRED_IN: case PGPU_PRED_NOT_IN: {  // InPredicateEvaluatorFactory.java:138-154, NotIn...:140-160
      ids.clear();
      for (const Literal& v : pp.lits) {
        const int ins = insertion_index(c, v);
        if (ins >= 0) ids.push_back(ins);
      }
      std::sort(ids.begin(), ids.end());
      ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
      const int n = (int)ids.size();
      const bool in = p.type == PGPU_PRED_IN;
      if (n == 0) { L->kind = in ? LEAF_NONE : LEAF_ALL; return 0; }
      if (n == card) { L->kind = in ? LEAF_ALL : LEAF_NONE; return 0; }
      L->negate = in ? 0 : 1;
      if (ids.back() - ids.front() + 1 == n) {  // contiguous dictIds: a range test
        L->kind = LEAF_RANGE;
        L->lo = ids.front();
        L->span = n;
      } else {
        L->kind = LEAF_SET;
        L->set.assign(((size_t)card + 31) / 32, 0u);
        for (int id : ids) L->set[id >> 5] |= 1u << (id & 31);
      }
      return 0;
    }
    case PGPU_PRED_RANGE: {  // SortedDictionaryBasedRangePredicateEvaluator (RangePredicateEvaluatorFactory.java:115-159)
      int start, end;
      if (pp.lits[0].star) start = 0;
      else {
        const int ins = insertion_index(c, pp.lits[0]);
        start = ins < 0 ? -(ins + 1) : (p.lower_inclusive ? ins : ins + 1);
      }
      if (pp.lits[1].star) end = card;
      else {
        const int ins = insertion_index(c, pp.lits[1]);
        end = ins < 0 ? -(ins + 1) : (p.upper_inclusive ? ins + 1 : ins);
      }
      const int nm = end - start;
      if (nm <= 0) L->kind = LEAF_NONE;
      else if (nm == card) L->kind = LEAF_ALL;
      else { L->kind = LEAF_RANGE; L->lo = start; L->span = nm; }
      return 0;
    }
    default:
      return fail(PGPU_ERR_UNSUPPORTED, "predicate type %d is not on the GPU path", p.type);
  }
}

// Raw-value predicate evaluators (no dictionary; BaseRawValueBasedPredicateEvaluator subclasses, never always-true /
// -false for FilterPlanNode): the leaf tests the column's per-doc int64 keys -- the value for INT / LONG, the
// order-preserving key of the double for FLOAT / DOUBLE (NaN canonical) -- against
//   RANGE (RangePredicateEvaluatorFactory.java:60-102, 268-448): unbounded = inclusive MIN / MAX (+-inf); Java's
//          comparisons turned into inclusive key bounds (exclusive: the next representable value; 0.0 and -0.0
//          compare equal, NaN never matches);
//   EQ / NOT_EQ (EqualsPredicateEvaluatorFactory.java:60-70 `==`, NotEquals `!=`): the range [v, v] (negated);
//   IN / NOT_IN (InPredicateEvaluatorFactory.java:69-126): fastutil Int/Long/Float/DoubleOpenHashSet.contains --
//          bit equality (Float.floatToIntBits / Double.doubleToLongBits: 0.0 != -0.0, NaN == NaN).
void translate_raw_predicate(int type, const pgpu_predicate& p, const ParsedPred& pp, LeafHost* L) {
  L->raw.clear();
  L->negate = 0;
  const bool fp = is_fp_type(type);
  auto empty = [&] { L->kind = LEAF_RAW_RANGE; L->raw = {1, 0}; };
  auto fkey = [](double v) { return double_key(std::isnan(v) ? kCanonicalNaN : v); };
  switch (p.type) {
    case PGPU_PRED_EQ: case PGPU_PRED_NOT_EQ: {
      L->negate = p.type == PGPU_PRED_NOT_EQ;
      L->kind = LEAF_RAW_RANGE;
      if (!fp) { L->raw = {pp.lits[0].i, pp.lits[0].i}; return; }
      const double v = pp.lits[0].d;
      if (std::isnan(v)) { empty(); L->negate = p.type == PGPU_PRED_NOT_EQ; return; }
      if (v == 0.0) L->raw = {fkey(-0.0), fkey(0.0)};
      else L->raw = {fkey(v), fkey(v)};
      return;
    }
    case PGPU_PRED_IN: case PGPU_PRED_NOT_IN: {
      L->negate = p.type == PGPU_PRED_NOT_IN;
      L->kind = LEAF_RAW_IN;
      for (const Literal& v : pp.lits) L->raw.push_back(fp ? fkey(v.d) : v.i);
      std::sort(L->raw.begin(), L->raw.end());
      L->raw.erase(std::unique(L->raw.begin(), L->raw.end()), L->raw.end());
      L->span = (uint32_t)L->raw.size();
      return;
    }
    default: {  // RANGE
      L->kind = LEAF_RAW_RANGE;
      const Literal& a = pp.lits[0];
      const Literal& b = pp.lits[1];
      if (!fp) {
        const int64_t tmin = type == PGPU_INT ? INT32_MIN : INT64_MIN, tmax = type == PGPU_INT ? INT32_MAX : INT64_MAX;
        int64_t lo = a.star ? tmin : a.i, hi = b.star ? tmax : b.i;
        if (!a.star && !p.lower_inclusive) { if (lo == INT64_MAX) { empty(); return; } ++lo; }
        if (!b.star && !p.upper_inclusive) { if (hi == INT64_MIN) { empty(); return; } --hi; }
        L->raw = {lo, hi};
        return;
      }
      const double inf = std::numeric_limits<double>::infinity();
      double lo = a.star ? -inf : a.d, hi = b.star ? inf : b.d;
      if (std::isnan(lo) || std::isnan(hi)) { empty(); return; }
      int64_t klo, khi;
      if (a.star || p.lower_inclusive) klo = lo == 0.0 ? fkey(-0.0) : fkey(lo);
      else if (lo == inf) { empty(); return; }
      else klo = fkey(lo == 0.0 ? std::nextafter(0.0, inf) : std::nextafter(lo, inf));
      if (b.star || p.upper_inclusive) khi = hi == 0.0 ? fkey(0.0) : fkey(hi);
      else if (hi == -inf) { empty(); return; }
      else khi = fkey(hi == 0.0 ? std::nextafter(-0.0, -inf) : std::nextafter(hi, -inf));
      L->raw = {klo, khi};
      return;
    }
  }
}

// Constant folding of the program against the leaves' constants (FilterPlanNode.java:146-176).
// Fraction of docs the filter program passes if every dictId were equally frequent (leaf fractions combined as
// independent events).  Only picks the scan kernel instance (dense / sparse): never affects results.
double estimate_selectivity(const std::vector<int32_t>& ops, const std::vector<double>& leaf) {
  double st[kMaxOps];
  int sp = 0;
  for (int32_t e : ops) {
    const int op = e >> 16, arg = e & 0xFFFF;
    if (op == OP_LEAF) st[sp++] = leaf[arg];
    else if (op == OP_NOT) st[sp - 1] = 1.0 - st[sp - 1];
    else {
      double x = op == OP_AND ? 1.0 : 0.0;
      for (int j = sp - arg; j < sp; ++j) x = op == OP_AND ? x * st[j] : 1.0 - (1.0 - x) * (1.0 - st[j]);
      sp -= arg;
      st[sp++] = x;
    }
  }
  return sp == 0 ? 1.0 : st[sp - 1];
}

Tri fold_program(const std::vector<int32_t>& ops, const std::vector<Tri>& leaf) {
  Tri st[kMaxOps];
  int sp = 0;
  for (int32_t e : ops) {
    const int op = e >> 16, arg = e & 0xFFFF;
    if (op == OP_LEAF) st[sp++] = leaf[arg];
    else if (op == OP_NOT) {
      Tri& x = st[sp - 1];
      x = x == T_ALL ? T_NONE : x == T_NONE ? T_ALL : T_VAR;
    } else {
      bool any_none = false, any_all = false, all_all = true, all_none = true;
      for (int j = sp - arg; j < sp; ++j) {
        any_none |= st[j] == T_NONE;
        any_all |= st[j] == T_ALL;
        all_all &= st[j] == T_ALL;
        all_none &= st[j] == T_NONE;
      }
      sp -= arg;
      if (op == OP_AND) st[sp++] = any_none ? T_NONE : all_all ? T_ALL : T_VAR;
      else st[sp++] = any_all ? T_ALL : all_none ? T_NONE : T_VAR;
    }
  }
  return sp == 0 ? T_ALL : st[sp - 1];
}

// ------------------------------------------------------------------------------------------------ star-tree plans
// The filter as a star-tree sees it: composites (one leaf, or an OR of leaves on one column) that are ANDed
// (StarTreeUtils.extractPredicateEvaluatorsMap / isOrClauseValidForStarTree, core/startree/StarTreeUtils.java:
// 88-218).  False for other shapes (NOT, AND under OR, OR across columns): those segments use the scan path, which
// returns the same result.
bool star_composites(const std::vector<int32_t>& ops, const pgpu_query* q, std::vector<std::vector<int>>* out) {
  struct Node {
    int type;  // 0 leaf, 1 OR on one column, 2 AND
    int col;
    std::vector<int> leaves;
    std::vector<std::vector<int>> comps;
  };
  std::vector<Node> st;
  for (int32_t e : ops) {
    const int op = e >> 16, arg = e & 0xFFFF;
    if (op == OP_LEAF) {
      st.push_back({0, q->predicates[arg].column, {arg}, {}});
    } else if (op == OP_NOT) {
      return false;
    } else if (op == OP_OR) {
      Node n{1, -1, {}, {}};
      for (int j = (int)st.size() - arg; j < (int)st.size(); ++j) {
        if (st[j].type == 2) return false;
        if (n.col >= 0 && st[j].col != n.col) return false;
        n.col = st[j].col;
        n.leaves.insert(n.leaves.end(), st[j].leaves.begin(), st[j].leaves.end());
      }
      st.resize(st.size() - arg);
      st.push_back(std::move(n));
    } else {
      Node n{2, -1, {}, {}};
      for (int j = (int)st.size() - arg; j < (int)st.size(); ++j) {
        if (st[j].type == 2) n.comps.insert(n.comps.end(), st[j].comps.begin(), st[j].comps.end());
        else n.comps.push_back(st[j].leaves);
      }
      st.resize(st.size() - arg);
      st.push_back(std::move(n));
    }
  }
  out->clear();
  if (st.empty()) return true;
  if (st.back().type == 2) *out = st.back().comps;
  else out->push_back(st.back().leaves);
  return true;
}

// Matching dictIds of one translated leaf over [0, card) as a bitset (PredicateEvaluator.getMatchingDictIds).
void leaf_bitset(const LeafHost& L, int32_t card, std::vector<uint32_t>& w) {
  const size_t nw = ((size_t)card + 31) / 32;
  w.assign(nw, 0u);
  for (int32_t i = 0; i < card; ++i) {
    bool m;
    switch (L.kind) {
      case LEAF_ALL: m = true; break;
      case LEAF_NONE: m = false; break;
      case LEAF_RANGE: m = (uint32_t)i >= L.lo && (uint32_t)i < L.lo + L.span; break;
      case LEAF_DOCRANGE: m = (uint32_t)i >= L.dict_lo && (uint32_t)i < L.dict_lo + L.dict_span; break;
      default: m = (L.set[i >> 5] >> (i & 31)) & 1u; break;
    }
    if (L.kind == LEAF_RANGE || L.kind == LEAF_SET || L.kind == LEAF_DOCRANGE) m ^= L.negate != 0;
    if (m) w[i >> 5] |= 1u << (i & 31);
  }
}

// Plans segment `s` on its star-tree when the query fits it (StarTreeUtils.isFitForStarTree, :151-176, and the
// function-column pairs of the aggregations, :67-86).  *used = false leaves the segment to the scan path.
int plan_star_segment(pgpu_plan_s* P, size_t seg_index, Segment* s, const pgpu_query* q,
                      const std::vector<std::vector<int>>& comps, const std::vector<LeafHost>& leaves, bool* used) {
  *used = false;
  const StarTreeDev* st = s->star.get();
  if (!st || st->num_dims > kMaxStarDims || st->num_nodes < 1 || P->first_doc_slot) return 0;
  bool has_avg = false;
  int avg_col = -1;
  for (int i = 0; i < q->num_aggs; ++i) {
    if (st->pair(q->aggs[i].fn, q->aggs[i].column) < 0) return 0;
    if (q->aggs[i].fn == PGPU_AGG_AVG) { has_avg = true; avg_col = q->aggs[i].column; }
  }
  for (int c : P->key_cols)
    if (st->dim_of(c) < 0) return 0;
  for (int l = 0; l < q->num_predicates; ++l)
    if (st->dim_of(q->predicates[l].column) < 0) return 0;
  KStarSeg k;
  memset(&k, 0, sizeof k);
  k.nodes = st->d_nodes;
  k.num_nodes = st->num_nodes;
  k.num_docs = st->num_docs;
  k.num_dims = st->num_dims;
  for (int d = 0; d < st->num_dims; ++d) {
    k.dim_fwd[d] = st->d_dim_fwd[d];
    k.dim_bits[d] = st->dim_bits[d];
  }
  // slot sources
  const int cnt_pair = st->pair(PGPU_AGG_COUNT, -1);
  if (cnt_pair >= 0) k.src_c[0] = st->d_mc[cnt_pair];
  else if (has_avg) k.src_c[0] = st->d_mc[st->pair(PGPU_AGG_AVG, avg_col)];
  for (size_t sl = 1; sl < P->slot_kind.size(); ++sl) {
    const int col = P->slot_tcol[sl];
    int m = -1;
    switch (P->slot_kind[sl]) {
      case SLOT_SUM_I64: case SLOT_SUM_F64:
        m = st->pair(PGPU_AGG_SUM, col);
        if (m < 0) m = st->pair(PGPU_AGG_AVG, col);
        break;
      case SLOT_MIN_KEY: m = st->pair(PGPU_AGG_MIN, col); break;
      default: m = st->pair(PGPU_AGG_MAX, col); break;
    }
    if (m < 0 || !st->d_mf[m]) return 0;
    k.src_f[sl] = st->d_mf[m];
  }
  // predicate dims: AND of the composites' matching dictIds; always-true composites are dropped
  std::vector<std::vector<uint32_t>> match(st->num_dims);
  std::vector<uint32_t> cw, lw;
  for (const auto& comp : comps) {
    const int col = q->predicates[comp[0]].column;
    const int d = st->dim_of(col);
    const int32_t card = s->cols[col].card;
    const size_t nw = ((size_t)card + 31) / 32;
    cw.assign(nw, 0u);
    for (int l : comp) {
      leaf_bitset(leaves[l], card, lw);
      for (size_t i = 0; i < nw; ++i) cw[i] |= lw[i];
    }
    int64_t ones = 0;
    for (uint32_t x : cw) ones += __builtin_popcount(x);
    if (ones == card) continue;  // isAlwaysTrue: not a predicate column for the traversal
    if (match[d].empty()) match[d].assign(nw, ~0u);
    for (size_t i = 0; i < nw; ++i) match[d][i] &= cw[i];
    k.pred_mask |= 1 << d;
  }
  *used = true;
  for (int d = 0; d < st->num_dims; ++d) {
    if (!(k.pred_mask & (1 << d))) continue;
    int64_t ones = 0;
    for (uint32_t x : match[d]) ones += __builtin_popcount(x);
    if (ones == 0) return 0;  // no matching dictId: the traversal returns null (empty result for the segment)
  }
  for (size_t j = 0; j < P->key_cols.size(); ++j) {
    const int c = P->key_cols[j];
    // K6 always gathers through the LUT (the planned version, taken under the table mutex)
    k.key_lut[j] = reinterpret_cast<const int32_t*>(P->refs->luts[seg_index * P->key_cols.size() + j]->p);
    k.key_dim[j] = st->dim_of(c);
    k.dim_card[k.key_dim[j]] = s->cols[c].card;
    if (!(k.pred_mask & (1 << k.key_dim[j]))) k.group_mask |= 1 << k.key_dim[j];
  }
  for (const auto& comp : comps) {
    const int col = q->predicates[comp[0]].column;
    k.dim_card[st->dim_of(col)] = s->cols[col].card;
  }
  {  // K6 LDS cache: the key LUTs and the match sets of the predicate dims (a superset of the residual dims)
    int64_t ints = 0;
    for (size_t j = 0; j < P->key_cols.size(); ++j) ints += k.dim_card[k.key_dim[j]];
    for (int d = 0; d < st->num_dims; ++d)
      if (k.pred_mask & (1 << d)) ints += (k.dim_card[d] + 31) / 32;
    constexpr int64_t kStarCacheMax = 8192;  // 32 KB
    if (P->star_cache_ints >= 0)
      P->star_cache_ints = ints > kStarCacheMax ? -1 : std::max<int32_t>(P->star_cache_ints, (int32_t)ints);
  }
  const int idx = (int)P->star.size();
  for (int d = 0; d < st->num_dims; ++d) {
    if (!(k.pred_mask & (1 << d))) continue;
    if (P->set_words.size() & 1) P->set_words.push_back(0);
    P->star_match_fix.emplace_back(idx, d, (int64_t)P->set_words.size());
    P->set_words.insert(P->set_words.end(), match[d].begin(), match[d].end());
  }
  const int64_t nn = st->num_nodes;
  P->star_work_off.push_back(P->star_work_bytes);
  P->star_work_bytes += ((2 * nn * 4 + (nn + 1) * 8 + 6 * nn * 4 + 8) + 15) & ~int64_t(15);
  P->star.push_back(k);
  return 0;
}

struct ExecCtx {
  KParams kp;
  // PGPU_TRACE=1: host time marks of the execution, printed when it took over a millisecond
  std::vector<std::pair<const char*, double>> marks;
  void mark(const char* what) { if (trace_on()) marks.emplace_back(what, now_us()); }
  // where this execution's records, bitsets and tile map live: the scratch, or the cached plan's DeviceImage
  uint8_t* segrec = nullptr;
  uint32_t* sets = nullptr;
  int32_t* tile_seg = nullptr;
  bool from_image = false;
  // one-launch LDS plans: the leap-frog statistics run in the slab fold's launch (launch_epilogue)
  const uint8_t* leap_segs = nullptr;
  int32_t leap_nsegs = 0;
  uint64_t* table = nullptr;
  int64_t words = 0;
  int nslots = 0;
  double t_start = 0;
  int64_t slabs_used = 0;  // MODE_LDS: slabs written by the scan launches so far (launches pack them back to back)
};

// numEntriesScannedInFilter method of a segment whose leaves have the Pinot operator kinds `sig` (base-5 digits,
// predicate 0 first; filter_stats.h): the folded tree, and the scan-kernel record bits of CHAIN / LEAP2.
struct SegStats {
  StatTree tree;
  int kind = STATS_CONST;
  int64_t const_per_doc = 0;
  int32_t rec_stats = KSTATS_NONE;
  std::vector<int32_t> range_leaves;  // range-index leaves whose partial-match scan counts (range_index_leaves)
};
SegStats classify_segment_stats(const pgpu_plan_s* P, uint64_t sig) {
  std::vector<int32_t> lt(P->num_leaves);
  for (int l = P->num_leaves - 1; l >= 0; --l) { lt[l] = (int32_t)(sig % kStatLeafKinds); sig /= kStatLeafKinds; }
  SegStats ss;
  ss.tree = build_stat_tree(P->ops, lt);
  const StatsPlan sp = classify_stat_tree(ss.tree, 1);
  ss.kind = sp.kind;
  ss.const_per_doc = sp.constant;
  ss.range_leaves = range_index_leaves(ss.tree);
  std::vector<int> pos(P->num_leaves);  // predicate index -> evaluation position in the kernel
  for (int k = 0; k < P->num_leaves; ++k) pos[P->leaf_perm[k]] = k;
  if (sp.kind == STATS_CHAIN && P->in_kernel_stats) {
    // counted in the kernel when its evaluation order is Pinot's: index leaves, then the scans in order
    int last_idx = -1, prev_scan = -1;
    bool ok = true;
    for (int l : sp.index_leaves) last_idx = std::max(last_idx, pos[l]);
    for (int l : sp.scan_leaves) { ok &= pos[l] > last_idx && pos[l] > prev_scan; prev_scan = pos[l]; }
    if (ok) {
      ss.rec_stats = KSTATS_CHAIN;
      for (int l : sp.scan_leaves) ss.rec_stats |= 1 << (4 + pos[l]);
    } else {
      ss.kind = STATS_GENERIC;
    }
  } else if (sp.kind == STATS_LEAP2 && P->in_kernel_stats) {
    ss.rec_stats = KSTATS_LEAP2 | (pos[sp.scan_leaves[0]] << 8) | (pos[sp.scan_leaves[1]] << 10);
  } else if (sp.kind != STATS_CONST) {
    ss.kind = STATS_GENERIC;
  }
  return ss;
}

// True when an int64 accumulator cannot overflow for SUM / AVG over integer column `col` of these segments.
bool int_sum_fits(const std::vector<Segment*>& segs, int col) {
  long double bound = 0;
  for (const Segment* s : segs) {
    const Column& c = s->cols[col];
    const Dict& d = c.dict;
    if (!c.raw && d.iv.empty()) continue;
    const long double lo = c.raw ? (long double)c.raw_min : (long double)d.iv.front();
    const long double hi = c.raw ? (long double)c.raw_max : (long double)d.iv.back();
    const long double m = std::max(std::fabs(lo), std::fabs(hi));
    bound += m * (long double)s->num_docs;
  }
  return bound < 0x1p62L;
}

int exec_prologue(pgpu_plan_s* P, hipStream_t stream, void* d_table, int max_chunks, ExecCtx& X);
int exec_upload_chunk(pgpu_plan_s* P, hipStream_t stream, const ExecCtx& X, const LaunchChunk& C);
int exec_launch_chunk(pgpu_plan_s* P, hipStream_t stream, ExecCtx& X, const LaunchChunk& C, int c);
int exec_epilogue(pgpu_plan_s* P, hipStream_t stream, ExecCtx& X);

// The slot whose table word also carries the COUNT (KParams.pack_slot), or -1: the first integer SUM over a column
// whose values are >= 0 in every segment, when `max_count` (the most docs one word can see) bounds both halves of the
// word -- count < 2^(64 - shift), sum < 2^shift.  Not with star-tree segments (K6 keeps its own table layout).
int32_t pack_slot_for(const pgpu_table_s* t, const pgpu_plan_s* P, const pgpu_query* q, int64_t max_count,
                      int shift) {
  if (P->slot_kind.empty() || P->slot_kind[0] != SLOT_COUNT || shift <= 0 || shift >= 64) return -1;
  if (max_count >= (INT64_C(1) << (64 - shift))) return -1;
  for (const Segment* s : P->segs)
    if (s->star && !(q->options & PGPU_OPT_NO_STAR_TREE)) return -1;
  for (size_t sl = 1; sl < P->slot_kind.size(); ++sl) {
    const int c = P->slot_tcol[sl];
    if (P->slot_kind[sl] != SLOT_SUM_I64 || c < 0 || c == kDocIdColumn || !is_int_type(t->types[c])) continue;
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    bool known = true;
    for (const Segment* seg : P->segs) {
      const Column& col = seg->cols[c];
      if (col.raw) { lo = std::min(lo, col.raw_min); hi = std::max(hi, col.raw_max); }
      else if (!col.dict.iv.empty()) { lo = std::min(lo, col.dict.iv.front()); hi = std::max(hi, col.dict.iv.back()); }
      else if (col.dict.size() != 0) { known = false; break; }
    }
    if (known && lo <= hi && lo >= 0 && (long double)max_count * (long double)hi < ldexpl(1.0L, shift))
      return (int32_t)sl;
  }
  return -1;
}

// LDS-table plans (shift 40): a workgroup scans at most ceil(tiles / grid) + 2 tiles under either tile order, and the
// grid is at least min(tiles, CUs).
int32_t lds_pack_slot(const pgpu_table_s* t, const pgpu_plan_s* P, const pgpu_query* q, int64_t G) {
  if (G <= 1) return -1;
  int64_t tiles = 0;
  for (const Segment* s : P->segs) tiles += ((int64_t)s->num_docs + kTileDocs - 1) / kTileDocs;
  const int64_t min_grid = std::max<int64_t>(1, std::min<int64_t>(tiles, t->num_cus));
  const int64_t wg_docs = ((tiles + min_grid - 1) / min_grid + 2) * kTileDocs;
  return pack_slot_for(t, P, q, wg_docs, kLdsPackShift);
}

// Hash-table plans: one word sees at most every doc of the plan, so the COUNT takes bits(total_docs) high bits; the
// scan's adds stay packed and hash_unpack splits the occupied words after it (exec_epilogue).  Single-stage keys only.
int32_t hash_pack_slot(const pgpu_table_s* t, const pgpu_plan_s* P, const pgpu_query* q, int* shift) {
  if (!P->stage_end.empty() || P->total_docs <= 0) return -1;
  int bits = 0;
  while (bits < 63 && (INT64_C(1) << bits) <= P->total_docs) ++bits;
  *shift = 64 - bits;
  return pack_slot_for(t, P, q, P->total_docs, *shift);
}

// Hashed partitions (KPartParams.hashed) for a MODE_HASH plan: single-stage keys whose composite key fits int32
// (part_keys' arithmetic and the records' u32 keys), unless pgpu_config.hash_partitions is 0 (the global hash table).
bool part_hash_eligible(const pgpu_plan_s* P, int64_t G) {
  return P->cfg.hash_partitions && P->mode == MODE_HASH && P->stage_end.empty() && G > 0 && G < (INT64_C(1) << 31) && P->key_bias == 0;
}

// Hashed partitions' shape for `groups` expected groups: 2^pbits partitions (K8a / K8c's LDS histogram: at most
// kMaxParts) of LDS hash tables of 2^sbits entries (4 + 8 x slots bytes each).  Small tables keep more K8h
// workgroups on a CU, so the tables are 2^10 entries at a load of at most ~0.6 and partitions are added first; past
// kMaxParts partitions the tables grow, up to kHashPartLdsMax (more groups than that take further K8h rounds).
// Measured on c5_hash (10^7 groups, r04, ms per query): 2^14 x 2^10 (20 KB) 3.69-3.72, 2^13 x 2^11 (40 KB)
// 4.06-4.17, 2^13 x 2^12 (80 KB) 7.67, 2^14 x 2^12 11.7-12.7; the global hash table 14.8.  pgpu_config's
// hash_partition_lds_kb / hash_partition_bits (tests force K8h's extra rounds with them) cap the table bytes and the
// partition bits.
void hash_part_bits(const pgpu_config& cfg, int64_t groups, int nslots, int* pbits, int* sbits) {
  const int64_t lds_cap = cfg.hash_partition_lds_kb > 0
                              ? std::min<int64_t>((int64_t)cfg.hash_partition_lds_kb * 1024, 128 * 1024)
                              : kHashPartLdsMax;
  const int max_pbits = std::max(0, std::min(14, cfg.hash_partition_bits));
  auto fits = [&](int p, int sb) { return (long double)groups <= 0.6L * (long double)(int64_t(1) << (p + sb)); };
  int sb = 10;
  while (sb > 8 && (int64_t)part_hash_lds(sb, nslots) > lds_cap) --sb;
  int p = 0;
  while (p < max_pbits && !fits(p, sb)) ++p;
  while (!fits(p, sb) && sb < 14 && (int64_t)part_hash_lds(sb + 1, nslots) <= lds_cap) ++sb;
  *pbits = p;
  *sbits = sb;
}

// Coarse runs of the two-level scatter: 2^cshift consecutive partitions each, at most 64 (KPartParams.cshift).
int part_coarse_shift(int num_parts) {
  int cshift = 0;
  while ((num_parts + (1 << cshift) - 1) >> cshift > 64) ++cshift;
  return cshift;
}
int part_coarse_runs(int num_parts) {
  const int cshift = part_coarse_shift(num_parts);
  return (num_parts + (1 << cshift) - 1) >> cshift;
}

// A cached hashed-partition plan re-shaped for the groups its last execution found (plan_cache_get): the partition
// count, the pass kernels' LDS and grid follow.
void hash_part_resize(pgpu_plan_s* P, int64_t groups) {
  const int nslots = (int)P->slot_kind.size();
  int pbits = 0, sbits = 0;
  hash_part_bits(P->cfg, groups, nslots, &pbits, &sbits);
  const int64_t parts = int64_t(1) << pbits;
  const size_t pass_lds = (size_t)((parts + 3) & ~int64_t(3)) * 4 + (P->pure_and ? 0 : (size_t)kMaxStack * kBlock * 4);
  if (pass_lds > 96 * 1024) return;
  P->part_pbits = pbits;
  P->part_sbits = sbits;
  P->num_parts = (int)parts;
  P->part_lds = pass_lds;
  P->part_grid_staged[0] = P->part_grid_staged[1] = 0;
  int per_cu = occupancy_part_pass(pass_lds, (int)parts, part_coarse_runs((int)parts), 0);
  per_cu = std::max(1, std::min(per_cu, 4));
  P->part_grid = (int)std::max<int64_t>(1, std::min<int64_t>(P->num_tiles, (int64_t)P->table->num_cus * per_cu));
}

// Records K8h may append (the groups): as finalize's compaction of a hash table sizes its output.
int64_t part_hash_out_cap(const pgpu_plan_s* P) {
  return std::max<int64_t>(1, std::min<int64_t>(P->num_keys, std::max<int64_t>(P->total_docs, 1)));
}

// K8h found more groups than its record buffer holds (the bound above is exact for the plan's key space and docs, so
// this is a planning bug, reported instead of a truncated result)
int part_hash_overflow(const pgpu_plan_s* P, uint64_t groups) {
  return fail(PGPU_ERR_DEVICE, "hashed partitions found %llu groups, past their record buffer of %lld",
              (unsigned long long)groups, (long long)part_hash_out_cap(P));
}

int plan_create_impl(pgpu_table_s* t, const int64_t* handles, int32_t nsegs, const pgpu_query* q, pgpu_plan_s* P,
                     const StreamExec* se = nullptr) {
  if (!q) return fail(PGPU_ERR_INVALID_ARGUMENT, "null query");
  const double t_start = trace_on() ? now_us() : 0;
  P->cfg = table_config(t);
  const int ncols = (int)t->names.size();
  // num_group_by == 0: aggregation-only (AggregationOperator, core/operator/query/AggregationOperator.java:58-95):
  // one accumulator row (key space G = 1), reduced per wave before any atomic.
  if (q->num_group_by < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "negative group-by count");
  if (q->num_group_by > kMaxKeys) return fail(PGPU_ERR_UNSUPPORTED, "more than %d group-by columns", kMaxKeys);
  if (q->num_predicates > kMaxLeaves) return fail(PGPU_ERR_UNSUPPORTED, "more than %d predicates", kMaxLeaves);
  if (q->num_filter_ops > kMaxOps) return fail(PGPU_ERR_UNSUPPORTED, "filter program longer than %d", kMaxOps);
  P->table = t;
  P->end_time_ms = q->end_time_ms;
  double tr[8] = {0};
  int ntr = 0;
  auto mark = [&] { if (trace_on() && ntr < 8) tr[ntr++] = now_us(); };
  // Segment references (SegmentDataManager acquire): the table mutex is held only to take them here and, below, to
  // build the lazily made LUT / value arrays and snapshot the global dictionary sizes -- the per-segment translation
  // runs unlocked, so concurrent queries on one table plan in parallel.
  P->refs = std::make_shared<PlanRefs>();
  {
    std::lock_guard<std::mutex> g(t->mu);
    P->segs.reserve(nsegs);
    P->refs->segs.reserve(nsegs);
    for (int i = 0; i < nsegs; ++i) {
      const int64_t h = handles[i];
      const std::shared_ptr<Segment>* sp = h > 0 && h < (int64_t)t->by_handle.size() ? &t->by_handle[h] : nullptr;
      if (!sp || !*sp) return fail(PGPU_ERR_NOT_FOUND, "unknown segment handle %lld", (long long)h);
      P->segs.push_back(sp->get());
      P->refs->segs.push_back(*sp);
    }
  }
  // query columns
  auto slot_of = [&](int col) -> int {
    for (size_t i = 0; i < P->query_cols.size(); ++i)
      if (P->query_cols[i] == col) return (int)i;
    P->query_cols.push_back(col);
    return (int)P->query_cols.size() - 1;
  };
  for (int i = 0; i < q->num_predicates; ++i) {
    const int c = q->predicates[i].column;
    if (c < 0 || c >= ncols) return fail(PGPU_ERR_INVALID_ARGUMENT, "predicate %d: bad column %d", i, c);
    P->leaf_slot.push_back(slot_of(c));
  }
  P->num_leaves = q->num_predicates;
  for (int i = 0; i < q->num_group_by; ++i) {
    const int c = q->group_by[i];
    if (c < 0 || c >= ncols) return fail(PGPU_ERR_INVALID_ARGUMENT, "group-by %d: bad column %d", i, c);
    P->key_cols.push_back(c);
    slot_of(c);
  }
  // raw (no-dictionary) columns: aggregation operands and raw-value predicate leaves (below); a group-by on one runs
  // on Pinot's NoDictionary*GroupKeyGenerator, not here
  bool any_raw_leaf = false;
  for (Segment* s : P->segs) {
    for (int i = 0; i < q->num_predicates; ++i) {
      const Column& c = s->cols[q->predicates[i].column];
      any_raw_leaf |= c.raw;
      if (c.raw && t->types[q->predicates[i].column] == PGPU_STRING)
        return fail(PGPU_ERR_UNSUPPORTED, "predicate on raw STRING column %d", q->predicates[i].column);
    }
    for (int i = 0; i < q->num_group_by; ++i)
      if (s->cols[q->group_by[i]].raw)
        return fail(PGPU_ERR_UNSUPPORTED, "group-by on raw (no-dictionary) column %d", q->group_by[i]);
  }
  // program
  int depth = 0, max_depth = 0;
  bool pure_and = q->num_filter_ops > 0;
  int leaves_seen = 0;
  for (int i = 0; i < q->num_filter_ops; ++i) {
    const pgpu_filter_op& o = q->filter[i];
    if (o.op == PGPU_OP_PRED) {
      if (o.arg < 0 || o.arg >= q->num_predicates) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad predicate index");
      if (o.arg != leaves_seen) pure_and = false;
      ++leaves_seen;
      ++depth;
      P->ops.push_back((OP_LEAF << 16) | o.arg);
    } else if (o.op == PGPU_OP_NOT) {
      if (depth < 1) return fail(PGPU_ERR_INVALID_ARGUMENT, "malformed filter program");
      pure_and = false;
      P->ops.push_back(OP_NOT << 16);
    } else if (o.op == PGPU_OP_AND || o.op == PGPU_OP_OR) {
      if (o.arg < 1 || o.arg > depth) return fail(PGPU_ERR_INVALID_ARGUMENT, "malformed filter program");
      if (o.op == PGPU_OP_OR || i != q->num_filter_ops - 1) pure_and = false;
      depth -= o.arg - 1;
      P->ops.push_back(((o.op == PGPU_OP_AND ? OP_AND : OP_OR) << 16) | o.arg);
    } else {
      return fail(PGPU_ERR_INVALID_ARGUMENT, "bad filter opcode %d", o.op);
    }
    max_depth = std::max(max_depth, depth);
  }
  if (q->num_filter_ops > 0 && depth != 1) return fail(PGPU_ERR_INVALID_ARGUMENT, "malformed filter program");
  if (max_depth > kMaxStack) return fail(PGPU_ERR_UNSUPPORTED, "filter nesting deeper than %d", kMaxStack);
  if (q->num_filter_ops == 1) pure_and = true;  // a single leaf
  if (pure_and && leaves_seen != q->num_predicates) pure_and = false;
  P->pure_and = pure_and;
  P->max_depth = max_depth;

  // aggregations -> accumulator slots (slot 0 = COUNT)
  P->slot_kind.push_back(SLOT_COUNT);
  P->slot_col.push_back(0);
  P->slot_tcol.push_back(-1);
  auto add_slot = [&](int kind, int tcol) -> int {
    for (size_t s = 1; s < P->slot_kind.size(); ++s)
      if (P->slot_kind[s] == kind && P->slot_tcol[s] == tcol) return (int)s;
    P->slot_kind.push_back(kind);
    P->slot_tcol.push_back(tcol);
    P->slot_col.push_back(slot_of(tcol));
    return (int)P->slot_kind.size() - 1;
  };
  for (int i = 0; i < q->num_aggs; ++i) {
    const pgpu_agg& a = q->aggs[i];
    P->agg_fn.push_back(a.fn);
    P->agg_col.push_back(a.column);
    if (a.fn == PGPU_AGG_COUNT) { P->agg_slot.push_back(0); continue; }
    if (a.column < 0 || a.column >= ncols) return fail(PGPU_ERR_INVALID_ARGUMENT, "aggregation %d: bad column", i);
    const int type = t->types[a.column];
    if (type == PGPU_STRING) return fail(PGPU_ERR_UNSUPPORTED, "numeric aggregation over a STRING column");
    int kind;
    switch (a.fn) {
      case PGPU_AGG_SUM: case PGPU_AGG_AVG:
        // Integer columns sum exactly in int64 unless the plan could overflow it: |sum| <= sum over segments of
        // numDocs x max |value| (the sorted dictionary's ends).  Past 2^62 the slot accumulates the doubles of
        // the values (Pinot's own arithmetic, SumAggregationFunction.java:66-73) instead of wrapping.
        kind = is_int_type(type) && int_sum_fits(P->segs, a.column) ? SLOT_SUM_I64 : SLOT_SUM_F64;
        break;
      case PGPU_AGG_MIN: kind = SLOT_MIN_KEY; break;
      case PGPU_AGG_MAX: kind = SLOT_MAX_KEY; break;
      default: return fail(PGPU_ERR_UNSUPPORTED, "aggregation function %d", a.fn);
    }
    P->agg_slot.push_back(add_slot(kind, a.column));
  }
  if (P->first_doc_slot) {  // hidden MIN($docId): each group's first matching doc (its IntGroupIdMap id order)
    P->slot_kind.push_back(SLOT_MIN_KEY);
    P->slot_tcol.push_back(kDocIdColumn);
    P->slot_col.push_back(slot_of(kDocIdColumn));
  }
  if ((int)P->slot_kind.size() > kMaxSlots) return fail(PGPU_ERR_UNSUPPORTED, "too many accumulators");
  if ((int)P->query_cols.size() > kMaxQueryCols) return fail(PGPU_ERR_UNSUPPORTED, "too many columns");
  {  // TransformOperator.getNumColumnsProjected: distinct group-by and aggregation columns
    std::vector<int> proj(P->key_cols.begin(), P->key_cols.end());
    for (int i = 0; i < q->num_aggs; ++i) if (q->aggs[i].column >= 0) proj.push_back(q->aggs[i].column);
    std::sort(proj.begin(), proj.end());
    P->num_projected = (int)(std::unique(proj.begin(), proj.end()) - proj.begin());
  }

  P->num_groups_limit = q->num_groups_limit;
  P->pql_cap = !(q->options & PGPU_OPT_SQL_GROUP_BY);
  if (q->num_groups_limit > 0) {
    for (Segment* s : P->segs) {
      int64_t prod = 1;
      for (int c : P->key_cols) {
        const int64_t card = std::max<int64_t>(s->cols[c].card, 1);
        prod = prod > INT64_MAX / card ? INT64_MAX : prod * card;
      }
      if (prod > q->num_groups_limit) P->limit_sensitive = true;
    }
  }
  // Under the table mutex: the global dictionary sizes the key layout is built on, and every segment's device LUT /
  // value arrays of the referenced columns (built once per segment, rebuilt out of place when the global dictionary
  // grows) -- taken together, so the LUTs the plan points at map into exactly the key space it sizes.
  std::vector<int64_t> gcard(P->key_cols.size());
  {
    const hipStream_t stream = t->stream;
    const size_t nk = P->key_cols.size();
    std::lock_guard<std::mutex> table_lock(t->mu);
    P->key_dicts.resize(nk);
    for (size_t j = 0; j < nk; ++j) {
      P->key_dicts[j] = t->global[P->key_cols[j]];
      gcard[j] = (int64_t)P->key_dicts[j]->size();
    }
    P->key_lut.resize(P->segs.size() * nk);
    P->refs->luts.reserve(P->segs.size() * nk);
    for (size_t i = 0; i < P->segs.size(); ++i) {
      Segment* s = P->segs[i];
      for (size_t j = 0; j < nk; ++j) {
        const int c = P->key_cols[j];
        TRY(ensure_lut(t, *s, c, stream));
        const Column& col = s->cols[c];
        P->refs->luts.push_back(col.lut);
        KeyLut& kl = P->key_lut[i * nk + j];
        kl.lut = col.lut_off >= 0 ? nullptr : reinterpret_cast<const int32_t*>(col.lut->p);
        kl.off = col.lut_off;
      }
      for (size_t k = 1; k < P->slot_kind.size(); ++k)
        if (P->slot_tcol[k] != kDocIdColumn) TRY(ensure_values(t, *s, P->slot_tcol[k], stream));
      if (P->first_doc_slot) TRY(ensure_docid(t, s->num_docs, stream));
    }
    // accumulator columns whose values are gathered (FLOAT / DOUBLE, or integers not consecutive): the table-global
    // arrays where a segment's dictionary maps onto the global one
    P->val_cols.clear();
    for (size_t k = 1; k < P->slot_kind.size(); ++k) {
      const int c = P->slot_tcol[k];
      if (c == kDocIdColumn || std::find(P->val_cols.begin(), P->val_cols.end(), c) != P->val_cols.end()) continue;
      bool any = false;
      for (Segment* s : P->segs) {
        const Column& col = s->cols[c];
        if (col.raw || col.card < kGlobalValuesMinCard || (is_int_type(t->types[c]) && col.key_affine)) continue;
        TRY(ensure_value_map(t, *s, c));
        any |= col.vgap_first >= 0;
      }
      if (any) {
        TRY(ensure_global_values(t, c, stream));
        P->val_cols.push_back(c);
      }
    }
    P->val_map.assign(P->segs.size() * P->val_cols.size(), ValMap{});
    for (size_t v = 0; v < P->val_cols.size(); ++v) {
      const int c = P->val_cols[v];
      const auto& gv = t->gvalues[c];
      P->refs->luts.push_back(gv.keys);
      P->refs->luts.push_back(gv.vals);
      for (size_t i = 0; i < P->segs.size(); ++i) {
        const Column& col = P->segs[i]->cols[c];
        ValMap& vm = P->val_map[i * P->val_cols.size() + v];
        if (col.raw || col.card < kGlobalValuesMinCard || (is_int_type(t->types[c]) && col.key_affine) ||
            col.vmap_version != t->global_version[c] || col.vgap_first < 0)
          continue;
        vm.keys = reinterpret_cast<const int64_t*>(gv.keys->p) + col.vgap_first;
        vm.vals = reinterpret_cast<const double*>(gv.vals->p) + col.vgap_first;
        vm.ngaps = (int32_t)col.vgaps.size();
        std::copy(col.vgaps.begin(), col.vgaps.end(), vm.gaps.begin());
      }
    }
    P->docid_fwd = t->d_docid_fwd;
    P->docid_key = t->d_docid_key;
    P->docid_bits = t->docid_bits;
  }
  // Key space restricted by the filter: a group-by column that a top-level conjunct of the filter bounds (EQ / IN /
  // RANGE on the same numeric column) can only produce the global ids inside that bound -- C3's GROUP BY
  // daysSinceEpoch under "daysSinceEpoch BETWEEN 17849 AND 17856" has 8 possible keys, not 365.  Column j's key
  // digit becomes (global id - key_off[j]); the kernels subtract key_bias = sum key_off[j] * stride[j] once.  Same
  // groups, a table (and slab fold, and compaction) sized by what the filter admits.
  std::vector<int64_t> klo(P->key_cols.size(), 0), kspan(gcard);
  if (P->pure_and) {
    for (size_t j = 0; j < P->key_cols.size(); ++j) {
      const int c = P->key_cols[j];
      const Dict& gd = *P->key_dicts[j];
      if (!is_int_type(gd.type) && !is_fp_type(gd.type)) continue;
      int64_t lo = 0, hi = (int64_t)gd.size();
      for (int l = 0; l < q->num_predicates; ++l) {
        const pgpu_predicate& pr = q->predicates[l];
        if (pr.column != c || (pr.type != PGPU_PRED_EQ && pr.type != PGPU_PRED_IN && pr.type != PGPU_PRED_RANGE)) continue;
        ParsedPred pp;
        TRY(parse_predicate(t->types[c], pr, &pp));
        auto search = [&](const Literal& v) {
          return is_int_type(gd.type) ? sorted_search<int64_t>(gd.iv, v.i) : sorted_search<double>(gd.dv, v.d);
        };
        int64_t a = 0, b = 0;
        if (pr.type == PGPU_PRED_RANGE) {  // as translate_predicate_dict's RANGE, on the global dictionary
          if (pp.lits[0].star) a = 0;
          else { const int ins = search(pp.lits[0]); a = ins < 0 ? -(ins + 1) : (pr.lower_inclusive ? ins : ins + 1); }
          if (pp.lits[1].star) b = (int64_t)gd.size();
          else { const int ins = search(pp.lits[1]); b = ins < 0 ? -(ins + 1) : (pr.upper_inclusive ? ins + 1 : ins); }
        } else {
          a = INT64_MAX;
          b = INT64_MIN;
          for (const Literal& v : pp.lits) {
            const int ins = search(v);
            if (ins >= 0) { a = std::min<int64_t>(a, ins); b = std::max<int64_t>(b, ins + 1); }
          }
          if (a > b) a = b = 0;
        }
        lo = std::max(lo, a);
        hi = std::min(hi, b);
      }
      if (hi <= lo) { lo = 0; hi = 1; }  // nothing admitted: no doc can match, keep a one-key digit
      klo[j] = lo;
      kspan[j] = hi - lo;
    }
    int64_t prod = 1;  // ARRAY_MAP stage plans keep the full key space (their stages restart the strides)
    bool ovf = false;
    for (size_t j = 0; j < P->key_cols.size(); ++j) {
      const int64_t card = std::max<int64_t>(kspan[j], 1);
      if (prod > INT64_MAX / card) ovf = true;
      else prod *= card;
    }
    if (ovf) { std::fill(klo.begin(), klo.end(), 0); kspan = gcard; }
  }
  P->key_off = klo;
  // group-key layout over the table-global dictionaries (mixed radix, first column fastest: ArrayBasedHolder)
  bool overflow = false;
  int64_t G = 1;
  for (size_t j = 0; j < P->key_cols.size(); ++j) {
    const int64_t card = std::max<int64_t>(kspan[j], 1);
    P->key_card.push_back(card);
    P->key_stride.push_back(G);
    if (!overflow && G > INT64_MAX / card) overflow = true;
    else if (!overflow) G *= card;
  }
  P->key_bias = 0;
  if (!overflow)
    for (size_t j = 0; j < P->key_cols.size(); ++j) P->key_bias += P->key_off[j] * P->key_stride[j];
  if (overflow) {
    // ArrayMapBasedHolder (DictionaryBasedGroupKeyGenerator.java:127-137: the cardinality product overflows a long).
    // The key columns split into consecutive groups whose keys fit 62 bits: group s's key (the previous group's slot x
    // its own key space + the mixed-radix key of its columns) is mapped on the device to its slot in hash table s --
    // a dense id below 2^31 -- and the last group's key is the group key of the plan's hash table.  Exact, like the
    // IntArray map it replaces; the tables are decoded back to dictIds at finalize.
    const int nk = (int)P->key_cols.size();
    constexpr int64_t kLim = INT64_C(1) << 62;
    int64_t docs = 0;
    for (Segment* s : P->segs) docs += s->num_docs;
    std::vector<int> ends;
    std::vector<int64_t> spaces, caps;
    int64_t capp = 1;  // slots of the previous group's table (1: none)
    for (int j = 0; j < nk;) {
      int64_t l = 1;
      int k = j;
      while (k < nk && l <= kLim / capp / P->key_card[k]) l *= P->key_card[k++];
      if (k == j) return fail(PGPU_ERR_UNSUPPORTED, "group key space beyond the staged ARRAY_MAP keys");
      for (int i = j; i < k; ++i)  // strides restart within each group
        P->key_stride[i] = i == j ? 1 : P->key_stride[i - 1] * P->key_card[i - 1];
      ends.push_back(k);
      spaces.push_back(l);
      if (k == nk) break;
      const int64_t want = std::max<int64_t>(2 * std::min<int64_t>(capp * l, std::max<int64_t>(docs, 1)), 1024);
      int64_t cap = 1;
      while (cap < want) cap <<= 1;
      if (cap > (INT64_C(1) << 31)) return fail(PGPU_ERR_UNSUPPORTED, "ARRAY_MAP key stage beyond 2^31 slots");
      caps.push_back(cap);
      capp = cap;
      j = k;
    }
    P->stage_end.assign(ends.begin(), ends.end() - 1);
    P->stage_cap = caps;
    P->stage_space = spaces;  // per group (the last one included)
    P->stage_mult.assign(spaces.begin() + 1, spaces.end());
    G = INT64_C(1) << 40;  // beyond every dense table: the hash table below (no overflow in the sizing products)
  }
  const int nslots = (int)P->slot_kind.size();
  constexpr int64_t kDenseGlobalMax = int64_t(1) << 26;
  // LDS-privatised tables up to 112 KB (one workgroup per CU at the top end): measured on MI355X, an 80 KB table
  // (C4: 5000 groups x 2 slots) runs 2.1x faster in LDS than with global atomics.  pgpu_config.lds_table_kb.
  const int64_t kLdsBudget = (int64_t)std::max(1, P->cfg.lds_table_kb) * 1024;
  // direct kernel LDS: [table (MODE_LDS)] [filter stack (general programs)] [per-wave match queues]
  const size_t stack_bytes = (pure_and ? 0 : (size_t)kMaxStack * kBlock * 4) + (size_t)(kBlock / 64) * 2 * kWaveQ * 4;
  for (Segment* s : P->segs) P->total_docs += s->num_docs;
  P->pack_slot = lds_pack_slot(t, P, q, G);
  const int lds_rows = nslots - (P->pack_slot >= 0 ? 1 : 0);
  if ((int64_t)lds_rows * G * 8 <= kLdsBudget) {
    P->mode = MODE_LDS;
    P->num_keys = G;
    P->lds_bytes = (size_t)lds_rows * G * 8 + stack_bytes;
  } else if (G <= kDenseGlobalMax) {
    P->pack_slot = -1;
    P->mode = MODE_GLOBAL;
    P->num_keys = G;
    P->lds_bytes = stack_bytes;
  } else {
    P->mode = MODE_HASH;
    P->hash = true;
    P->pack_slot = hash_pack_slot(t, P, q, &P->pack_shift);
    // Groups are bounded by the key space and, per segment, by min(its local key space, its docs): C5-style keys of
    // small per-segment cardinalities need far fewer slots than 2 x docs.  A cached plan re-sizes from the group
    // count its last execution found (hash_capacity, plan_cache_get): same query, same segments, same groups.
    int64_t bound = 0;
    for (Segment* s : P->segs) {
      int64_t local = 1;
      for (int c : P->key_cols) {
        const int64_t card = std::max<int64_t>(s->cols[c].card, 1);
        local = local > (int64_t)s->num_docs / card ? (int64_t)s->num_docs + 1 : local * card;
      }
      bound += std::min<int64_t>(local, s->num_docs);
    }
    P->group_bound = std::max<int64_t>(1, std::min<int64_t>(G, bound));
    P->groups_seen = std::make_shared<std::atomic<int64_t>>(-1);
    P->num_keys = hash_capacity(P->group_bound);
    P->lds_bytes = stack_bytes;
  }

  // per-segment records
  const int nqc = (int)P->query_cols.size();
  P->seg_scanned.reserve(P->segs.size());
  P->seg_stride = (int)(sizeof(KSegHdr) + sizeof(KCol) * nqc + sizeof(KLeaf) * std::max(P->num_leaves, 0));
  P->seg_stride = (P->seg_stride + 15) & ~15;
  P->segrec.reserve(P->segs.size() * (size_t)P->seg_stride);
  std::vector<ParsedPred> parsed(P->num_leaves);
  for (int l = 0; l < P->num_leaves; ++l)
    TRY(parse_predicate(t->types[q->predicates[l].column], q->predicates[l], &parsed[l]));
  std::vector<std::vector<int>> star_comps;
  const bool star_allowed = q->num_group_by > 0 && !(q->options & PGPU_OPT_NO_STAR_TREE) && P->stage_end.empty() &&
                            star_composites(P->ops, q, &star_comps);
  // Aggregation-only over a match-all segment: COUNT-only is answered from metadata, MIN/MAX-only from the
  // dictionaries (AggregationPlanNode.java:165-183) -- same values, numEntriesScannedPostFilter 0
  // (MetadataBasedAggregationOperator.java:89-92, DictionaryBasedAggregationOperator.java:171-173).
  bool exempt_kind = false, minmax_kind = false;
  if (q->num_group_by == 0 && q->num_aggs > 0) {
    bool all_count = true, all_minmax = true;
    for (int i = 0; i < q->num_aggs; ++i) {
      all_count &= q->aggs[i].fn == PGPU_AGG_COUNT;
      all_minmax &= q->aggs[i].fn == PGPU_AGG_MIN || q->aggs[i].fn == PGPU_AGG_MAX;
    }
    exempt_kind = all_count || all_minmax;
    minmax_kind = all_minmax && !all_count;
  }
  // DictionaryBasedAggregationOperator needs a dictionary on every MIN / MAX column (AggregationPlanNode.java:196-213)
  auto raw_minmax = [&](const Segment* s) {
    if (!minmax_kind) return false;
    for (int i = 0; i < q->num_aggs; ++i)
      if (q->aggs[i].column >= 0 && s->cols[q->aggs[i].column].raw) return true;
    return false;
  };
  bool any_star = false, any_inv = false;
  mark();
  for (Segment* s : P->segs) {
    any_star |= star_allowed && s->star != nullptr;
    for (int l = 0; l < q->num_predicates; ++l)
      any_inv |= s->cols[q->predicates[l].column].inv != nullptr;
  }
  // per query column: its group-by key index (-1: none) and whether an accumulator reads its values
  std::vector<int> qcol_key(P->query_cols.size(), -1);
  std::vector<char> qcol_val(P->query_cols.size(), 0);
  for (size_t j = 0; j < P->key_cols.size(); ++j)
    for (size_t i = 0; i < P->query_cols.size(); ++i)
      if (P->query_cols[i] == P->key_cols[j]) qcol_key[i] = (int)j;
  for (size_t k = 1; k < P->slot_col.size(); ++k) qcol_val[P->slot_col[k]] = 1;
  // Per-segment translation (PredicateEvaluatorProvider + FilterPlanNode per segment) in contiguous chunks,
  // on the host worker pool for large segment lists; records carry chunk-relative tile / set offsets, fixed up
  // when the chunks are concatenated in segment order.
  struct Chunk {
    bool gathers = false;  // pgpu_plan_s::gathers
    std::vector<uint8_t> rec;
    std::vector<uint32_t> set_words;
    std::vector<std::pair<int64_t, int64_t>> set_fix;
    std::vector<std::pair<int64_t, int64_t>> bit_fix;
    std::vector<KBitTask> bit_tasks;
    std::vector<KBitBlock> bit_blocks;
    std::vector<KRawTask> raw_tasks;
    std::vector<int64_t> raw_vals;
    std::vector<std::shared_ptr<InvIndex>> inv_refs;
    std::vector<pgpu_plan_s::GenericStat> generic;  // rec: chunk-relative record index
    bool any_leap2 = false;
    int64_t docbit_words = 0;
    std::vector<uint8_t> scanned;
    int64_t tiles = 0, entries = 0, matched = 0, sel_docs = 0, exempt = 0;
    int64_t leaf_kinds[kLeafKinds] = {};
    double sel = 1.0;
    int rc = 0;
    std::string err;
  };
  // Pure-AND programs evaluate their leaves in order with a wave-uniform early exit (AndDocIdIterator); leaves on
  // columns sorted in every segment go first (FilterOperatorUtils orders index-based children first,
  // FilterOperatorUtils.java:143-178) -- their docId-range masks cost no memory traffic and let whole waves skip
  // the scan leaves' bytes.
  std::vector<int> perm(P->num_leaves);
  for (int l = 0; l < P->num_leaves; ++l) perm[l] = l;
  if (P->pure_and && P->num_leaves > 1) {
    // FilterOperatorUtils.reorderAndFilterChildOperators (:143-178): sorted-index leaves, then bitmap
    // (inverted-index) leaves, then range-index leaves, then scans.
    std::vector<int> first, second, third, rest;
    for (int l = 0; l < P->num_leaves; ++l) {
      const pgpu_predicate& pr = q->predicates[l];
      const bool eq_in = pr.type == PGPU_PRED_EQ || pr.type == PGPU_PRED_NOT_EQ || pr.type == PGPU_PRED_IN ||
                         pr.type == PGPU_PRED_NOT_IN;
      bool all_sorted = !P->segs.empty(), all_inv = !P->segs.empty() && eq_in && !P->no_inverted;
      bool all_rng = !P->segs.empty() && pr.type == PGPU_PRED_RANGE;
      for (Segment* s : P->segs) {
        all_sorted &= s->cols[pr.column].sorted;
        all_inv &= s->cols[pr.column].inv != nullptr && !s->star;
        all_rng &= s->cols[pr.column].rng != nullptr;
      }
      (all_sorted ? first : all_inv ? second : all_rng ? third : rest).push_back(l);
    }
    first.insert(first.end(), second.begin(), second.end());
    first.insert(first.end(), third.begin(), third.end());
    first.insert(first.end(), rest.begin(), rest.end());
    perm = first;
    std::vector<int32_t> slots(P->num_leaves);
    for (int k = 0; k < P->num_leaves; ++k) slots[k] = P->leaf_slot[perm[k]];
    P->leaf_slot = slots;
  }
  auto plan_range = [&](size_t b, size_t e, Chunk& C) -> int {
    std::vector<LeafHost> leaves(P->num_leaves);
    std::vector<Tri> tri(P->num_leaves);
    std::vector<int> ids_scratch;
    std::vector<uint8_t> rec(P->seg_stride);
    std::unordered_map<uint64_t, SegStats> stat_cache;
    for (size_t i = b; i < e; ++i) {
      Segment* s = P->segs[i];
      for (int l = 0; l < P->num_leaves; ++l) {
        LeafHost& lh = leaves[l];
        lh.kind = LEAF_NONE; lh.negate = 0; lh.lo = 0; lh.span = 0;
        const Column& pc = s->cols[q->predicates[l].column];
        if (pc.raw) translate_raw_predicate(t->types[q->predicates[l].column], q->predicates[l], parsed[l], &lh);
        else TRY(translate_predicate(pc, q->predicates[l], parsed[l], &lh, ids_scratch));
        if (!P->no_inverted && !s->star) to_inverted_leaf(s->cols[q->predicates[l].column], q->predicates[l], *s, &lh);
        tri[l] = leaves[l].kind == LEAF_NONE ? T_NONE : leaves[l].kind == LEAF_ALL ? T_ALL : T_VAR;
      }
      const Tri whole = P->num_leaves ? fold_program(P->ops, tri) : T_ALL;
      C.scanned.push_back(0);
      if (whole == T_NONE || s->num_docs == 0) continue;  // EmptyFilterOperator: the segment is not scanned
      C.scanned.back() = 1;
      C.matched++;
      if (exempt_kind && whole == T_ALL && !raw_minmax(s)) C.exempt += s->num_docs;
      if (star_allowed && s->star) {  // only on the sequential path (any_star)
        bool used = false;
        TRY(plan_star_segment(P, i, s, q, star_comps, leaves, &used));
        if (used) continue;
      }
      // numEntriesScannedInFilter (filter_stats.h): Pinot's leaf operators in this segment, its folded operator
      // tree, and how the count is taken
      int32_t rec_stats = KSTATS_NONE;
      {
        // the tree depends only on the leaves' operator kinds: classified once per distinct kind vector of the
        // chunk (no per-segment allocation)
        uint64_t sig = 0;
        for (int l = 0; l < P->num_leaves; ++l) {
          const pgpu_predicate& pr = q->predicates[l];
          const Column& col = s->cols[pr.column];
          // FilterOperatorUtils.getLeafFilterOperator (:42-82): sorted column -> SortedIndexBasedFilterOperator;
          // RANGE with a range index -> RangeIndexBasedFilterOperator; other predicates with an inverted index ->
          // BitmapBasedFilterOperator; else a scan
          const int k = tri[l] == T_NONE ? SL_EMPTY : tri[l] == T_ALL ? SL_ALL : col.sorted ? SL_SORTED :
                        (pr.type != PGPU_PRED_RANGE && col.inv) ? SL_BITMAP :
                        (pr.type == PGPU_PRED_RANGE && col.rng && leaves[l].kind == LEAF_RANGE) ? SL_RANGEIDX : SL_SCAN;
          sig = sig * kStatLeafKinds + (uint64_t)k;
        }
        auto it = stat_cache.find(sig);
        if (it == stat_cache.end()) it = stat_cache.emplace(sig, classify_segment_stats(P, sig)).first;
        const SegStats& ss = it->second;
        rec_stats = ss.rec_stats;
        C.any_leap2 |= (rec_stats & 3) == KSTATS_LEAP2;
        if (ss.kind == STATS_CONST) C.entries += ss.const_per_doc * s->num_docs;
        for (int l : ss.range_leaves) {  // RangeIndexBasedFilterOperator's own partial-match scan
          const LeafHost& lh = leaves[l];
          C.entries += s->cols[q->predicates[l].column].rng->partial_entries(lh.lo, (int64_t)lh.lo + lh.span - 1);
        }
        if (ss.kind == STATS_GENERIC)
          C.generic.push_back({(int64_t)(C.rec.size() / P->seg_stride), s->num_docs, ss.tree, 0});
      }
      if (C.sel_docs == 0) {  // selectivity estimate from the first scanned segment's translated leaves
        std::vector<double> frac(P->num_leaves, 1.0);
        for (int l = 0; l < P->num_leaves; ++l) {
          const LeafHost& lh = leaves[l];
          const double card = std::max(1, s->cols[q->predicates[l].column].card);
          double f = lh.kind == LEAF_ALL ? 1.0 : lh.kind == LEAF_NONE ? 0.0 : lh.kind == LEAF_RANGE ? lh.span / card : 0.0;
          if (lh.kind == LEAF_DOCRANGE) f = (double)lh.span / std::max(1, s->num_docs);
          if (lh.kind == LEAF_BITMAP) f = lh.inv_frac;
          if (lh.kind == LEAF_RAW_RANGE || lh.kind == LEAF_RAW_IN) f = 0.5;  // no dictionary to estimate from
          if (lh.kind == LEAF_SET) {
            int64_t ones = 0;
            for (uint32_t w : lh.set) ones += __builtin_popcount(w);
            f = ones / card;
          }
          frac[l] = lh.negate ? 1.0 - f : f;
        }
        C.sel = P->num_leaves ? estimate_selectivity(P->ops, frac) : 1.0;
        C.sel_docs = s->num_docs;
      }
      std::fill(rec.begin(), rec.end(), 0);
      KSegHdr* h = reinterpret_cast<KSegHdr*>(rec.data());
      h->num_docs = s->num_docs;
      h->tile_base = (int32_t)C.tiles;  // chunk-relative
      h->num_tiles = (int32_t)((s->num_docs + kTileDocs - 1) / kTileDocs);
      h->stats = rec_stats;
      KCol* kc = reinterpret_cast<KCol*>(rec.data() + sizeof(KSegHdr));
      for (int j = 0; j < nqc; ++j) {
        if (P->query_cols[j] == kDocIdColumn) {
          kc[j].fwd = P->docid_fwd;
          kc[j].lut = nullptr;
          kc[j].dkey = P->docid_key;
          kc[j].dval = nullptr;
          kc[j].bits = P->docid_bits;
          continue;
        }
        const Column& c = s->cols[P->query_cols[j]];
        if (c.raw) {  // values per doc, addressed through the identity docId index
          kc[j].fwd = P->docid_fwd;
          kc[j].lut = nullptr;
          kc[j].dkey = c.d_key;
          kc[j].dval = c.d_val;
          kc[j].bits = P->docid_bits;
          continue;
        }
        kc[j].fwd = c.d_fwd;
        kc[j].bits = c.bits;
        if (qcol_key[j] >= 0) {  // group-by key: the LUT version planned (the segment's current one may be newer)
          const KeyLut& kl = P->key_lut[i * P->key_cols.size() + qcol_key[j]];
          kc[j].lut = kl.lut;
          kc[j].lut_off = kl.off;
        }
        if (qcol_val[j]) {  // accumulator operand: value arrays, built once (ensure_values) and never replaced
          kc[j].dkey = c.key_affine ? nullptr : c.d_key;
          kc[j].key_base = c.key_base;
          kc[j].dval = c.d_val;
          // or the table-global ones, as planned under the table mutex (ensure_value_map)
          const int tc = P->query_cols[j];
          for (size_t v = 0; v < P->val_cols.size(); ++v) {
            if (P->val_cols[v] != tc) continue;
            const ValMap& vm = P->val_map[i * P->val_cols.size() + v];
            if (vm.keys) {
              kc[j].dkey = vm.keys;
              kc[j].dval = vm.vals;
              kc[j].ngaps = vm.ngaps;
              std::copy(vm.gaps.begin(), vm.gaps.end(), kc[j].gaps);
            }
          }
        }
      }
      for (int j = 0; j < nqc; ++j)
        C.gathers |= (qcol_key[j] >= 0 && kc[j].lut != nullptr) || (qcol_val[j] && kc[j].dkey != nullptr);
      KLeaf* kl = reinterpret_cast<KLeaf*>(rec.data() + sizeof(KSegHdr) + sizeof(KCol) * nqc);
      const int64_t rec_off = (int64_t)C.rec.size();
      for (int k = 0; k < P->num_leaves; ++k) {
        const LeafHost& lh = leaves[perm[k]];
        kl[k].kind = lh.kind;
        kl[k].negate = lh.negate;
        kl[k].lo = lh.lo;
        kl[k].span = lh.span;
        kl[k].set = nullptr;
        if (lh.kind == LEAF_SET) {
          const int64_t field = rec_off + (int64_t)((uint8_t*)&kl[k].set - rec.data());
          C.set_fix.emplace_back(field, (int64_t)C.set_words.size());
          C.set_words.insert(C.set_words.end(), lh.set.begin(), lh.set.end());
          if (C.set_words.size() & 1) C.set_words.push_back(0);  // every leaf's words 8-byte aligned
        }
        if (lh.kind == LEAF_RAW_RANGE || lh.kind == LEAF_RAW_IN) {
          // raw-value leaf: evaluated per query into a docId bitmap region (raw_leaf_bitmap_kernel, negation
          // included) that the scan reads as a LEAF_BITMAP
          const int64_t field = rec_off + (int64_t)((uint8_t*)&kl[k].set - rec.data());
          C.bit_fix.emplace_back(field, C.docbit_words);
          KRawTask rt;
          memset(&rt, 0, sizeof rt);
          rt.keys = s->cols[q->predicates[perm[k]].column].d_key;
          rt.dst = C.docbit_words;
          rt.num_docs = s->num_docs;
          rt.kind = lh.kind;
          rt.negate = lh.negate;
          if (lh.kind == LEAF_RAW_RANGE) {
            rt.lo = lh.raw[0];
            rt.hi = lh.raw[1];
          } else {
            rt.lo = (int64_t)C.raw_vals.size();
            rt.hi = (int64_t)lh.raw.size();
            C.raw_vals.insert(C.raw_vals.end(), lh.raw.begin(), lh.raw.end());
          }
          C.raw_tasks.push_back(rt);
          C.docbit_words += ((((int64_t)s->num_docs + 31) / 32) + 1) & ~int64_t(1);
          kl[k].kind = LEAF_BITMAP;
          kl[k].negate = 0;
        }
        bool bitdir = false;
        if (lh.kind == LEAF_BITMAP && lh.inv_ids.size() == 1) {
          // one dictId (no OR to compute): the scan reads its containers in place through a block directory --
          // BITMAP containers word by word, ARRAY containers (< 4096 docs of a block, e.g. a segment's partial last
          // block) by a binary search of their sorted offsets (array_group_mask); entry = payload address, | 1 and
          // the entry count in bits 48..63 for an ARRAY
          const InvIndex& inv = *s->cols[q->predicates[perm[k]].column].inv;
          const InvIndex::Entry& e = inv.ids[lh.inv_ids[0]];
          bitdir = true;
          for (int32_t ci = e.begin; ci < e.begin + e.count && bitdir; ++ci) {
            const InvIndex::Cont& ct = inv.conts[ci];
            const uint64_t a = reinterpret_cast<uint64_t>(reinterpret_cast<const uint32_t*>(inv.d_block) + ct.word);
            bitdir = ct.type == CONT_BITMAP || (ct.type == CONT_ARRAY && ct.n >= 0 && ct.n < 65536 && (a >> 47) == 0);
          }
          if (bitdir) {
            const int64_t nblk = ((int64_t)s->num_docs + 65535) >> 16;
            std::vector<uint64_t> dir((size_t)nblk, 0);
            for (int32_t ci = e.begin; ci < e.begin + e.count; ++ci) {
              const InvIndex::Cont& ct = inv.conts[ci];
              if (ct.key < 0 || ct.key >= nblk) continue;
              const uint64_t a = reinterpret_cast<uint64_t>(reinterpret_cast<const uint32_t*>(inv.d_block) + ct.word);
              dir[ct.key] = ct.type == CONT_BITMAP ? a : (ct.n > 0 ? (a | 1ull | ((uint64_t)ct.n << 48)) : 0);
            }
            C.inv_refs.push_back(s->cols[q->predicates[perm[k]].column].inv);
            const int64_t field = rec_off + (int64_t)((uint8_t*)&kl[k].set - rec.data());
            C.set_fix.emplace_back(field, (int64_t)C.set_words.size());
            for (uint64_t d : dir) {
              C.set_words.push_back((uint32_t)d);
              C.set_words.push_back((uint32_t)(d >> 32));
            }
            kl[k].kind = LEAF_BITDIR;
          }
        }
        if (kl[k].kind >= 0 && kl[k].kind < kLeafKinds) C.leaf_kinds[kl[k].kind]++;
        if (lh.kind == LEAF_BITMAP && !bitdir) {  // docId bitmap region: whole 65536-doc containers
          const int64_t field = rec_off + (int64_t)((uint8_t*)&kl[k].set - rec.data());
          const InvIndex& inv = *s->cols[q->predicates[perm[k]].column].inv;
          C.inv_refs.push_back(s->cols[q->predicates[perm[k]].column].inv);
          C.bit_fix.emplace_back(field, C.docbit_words);
          const int64_t nblk = ((int64_t)s->num_docs + 65535) >> 16;
          const size_t t0 = C.bit_tasks.size();
          for (int32_t id : lh.inv_ids) {
            const InvIndex::Entry& e = inv.ids[id];
            for (int32_t ci = e.begin; ci < e.begin + e.count; ++ci) {
              const InvIndex::Cont& ct = inv.conts[ci];
              KBitTask task;
              task.payload = reinterpret_cast<const uint32_t*>(inv.d_block) + ct.word;
              task.type = ct.type;
              task.n = ct.n;
              task.dst = C.docbit_words + (int64_t)ct.key * kContainerWords;
              C.bit_tasks.push_back(task);
            }
          }
          if (lh.inv_ids.size() > 1)  // one dictId's containers are already in key order
            std::stable_sort(C.bit_tasks.begin() + t0, C.bit_tasks.end(),
                             [](const KBitTask& x, const KBitTask& y) { return x.dst < y.dst; });
          size_t ti = t0;
          for (int64_t kb = 0; kb < nblk; ++kb) {
            KBitBlock blk;
            blk.dst = C.docbit_words + kb * kContainerWords;
            blk.task_begin = (int32_t)ti;
            while (ti < C.bit_tasks.size() && C.bit_tasks[ti].dst == blk.dst) ++ti;
            blk.num_tasks = (int32_t)(ti - blk.task_begin);
            C.bit_blocks.push_back(blk);
          }
          C.docbit_words += nblk * kContainerWords;
        }
      }
      C.rec.insert(C.rec.end(), rec.begin(), rec.end());
      C.tiles += h->num_tiles;
    }
    return 0;
  };
  // Launch configuration once the tiles are known (tile_base: their number, or an upper bound for streamed plans).
  auto configure = [&](int64_t tile_base) -> int {
    P->num_tiles = tile_base;
    if (tile_base > INT32_MAX) return fail(PGPU_ERR_UNSUPPORTED, "too many tiles in one plan");
    P->star_segments = (int64_t)P->star.size();
    if (!P->star.empty()) {
      if (P->star_cache_ints < 0) P->star_cache_ints = 0;  // some segment's LUTs do not fit: global reads
      int64_t max_nodes = 0;
      for (const KStarSeg& k : P->star) max_nodes = std::max<int64_t>(max_nodes, k.num_nodes);
      P->star_range_cache = max_nodes * 16 <= 32 * 1024 ? (int32_t)max_nodes : 0;
      const int64_t nseg_launch = std::min<int64_t>((int64_t)P->star.size(), kStarMaxSegs);
      P->star_batches = (int)(((int64_t)P->star.size() + kStarMaxSegs - 1) / kStarMaxSegs);
      const int64_t rc = P->star_range_cache;
      const size_t table_bytes = P->mode == MODE_LDS ? (size_t)((nslots * G + 1) & ~int64_t(1)) * 8 : 0;
      P->star_lds_bytes = table_bytes + (size_t)((nseg_launch + 2) & ~int64_t(1)) * 8 + (size_t)((rc + 2) & ~int64_t(1)) * 8 +
                          (size_t)((2 * rc + 3) & ~int64_t(3)) * 4 + (size_t)P->star_cache_ints * 4;
      // K6: persistent workgroups (1024 threads in MODE_LDS, 256 otherwise), one resident wave of them over the
      // CUs; each flushes its table slab once
      const int64_t per_cu = P->mode == MODE_LDS ? std::max<int64_t>(1, std::min<int64_t>(2, (160 * 1024) /
                                                      std::max<size_t>(P->star_lds_bytes, 1))) : 8;
      const int64_t want = P->cfg.star_tree_workgroups;  // pgpu_config
      P->star_chunks = (int)(want > 0 ? want : (int64_t)t->num_cus * per_cu);
    }
    // Dense instance when tiles are expected to hold >= 8 matches per 32-doc group on average: below that the sparse
    // instance's per-match batches win (measured on MI355X, r04 session x: the C4 scan path at 15 % selectivity
    // 195 -> 170 us with the sparse instance; C2 at 50 % 577 us dense vs 1468 sparse).  pgpu_config.dense_selectivity.
    {
      P->dense = P->mode != MODE_HASH && P->sel_estimate >= P->cfg.dense_selectivity;
    }
    {
      bool f64 = false;
      for (int k : P->slot_kind) f64 |= k == SLOT_SUM_F64;
      // (a streamed plan configures before its later chunks are planned: never simple)
      P->dense_simple = P->dense && !P->gathers && !f64 && P->tile_bound == 0;
    }
    // the sparse instance with the index + scan pair: two-leaf AND plans with an in-place index leaf
    P->pair_variant = !P->dense && P->pure_and && P->num_leaves == 2 && P->leaf_kinds[LEAF_BITDIR] > 0;
    P->fast_variant = !P->dense && !P->pair_variant && P->pure_and && P->num_leaves <= kFastLeaves;
    P->fast_wide = P->fast_variant && P->sel_estimate >= 1.0 / 16;
    const int variant = scan_variant(P);
    int per_cu;  // resident workgroups per CU
    {
      static std::mutex occ_mu;
      static std::map<std::tuple<int, int, int, size_t>, int> occ_cache;  // (device, mode, dense, lds) -> per CU
      {
        std::lock_guard<std::mutex> g(occ_mu);
        const auto k = std::make_tuple(t->device, (int)P->mode, variant, P->lds_bytes);
        auto it = occ_cache.find(k);
        if (it == occ_cache.end()) it = occ_cache.emplace(k, occupancy_filter_groupby(P->mode, variant, P->lds_bytes)).first;
        per_cu = it->second;
      }
      if (per_cu <= 0) per_cu = 1;
      per_cu = std::min(per_cu, 4);
      P->grid = (int)std::max<int64_t>(1, std::min<int64_t>(tile_base, (int64_t)t->num_cus * per_cu));
    }
    // a multiple of the 8 XCDs (the kernel's XCD-aware tile order): rounded up when every tile has a workgroup of its
    // own and the resident capacity allows -- rounded down, an XCD's eighth of the tiles would outnumber its
    // workgroups and one of them would scan two tiles in a row (C1: 492 tiles on 488 workgroups)
    if (P->grid >= 64)
      P->grid = (P->grid == tile_base && ((P->grid + 7) & ~7) <= (int64_t)t->num_cus * per_cu) ? (P->grid + 7) & ~7
                                                                                                  : P->grid & ~7;
    if (P->any_leap2 || (se && P->in_kernel_stats)) {
      P->leap_reserved = true;
      // STATS_LEAP2 bytes of a workgroup's tiles are buffered in LDS (one per tile and wave) until the end of the
      // scan: at most kLeapLdsTiles tiles per workgroup (more workgroups than resident ones for huge plans)
      constexpr int64_t kLeapLdsTiles = 4096;
      const int64_t need = (tile_base + kLeapLdsTiles - 4) / (kLeapLdsTiles - 3);
      if (P->grid < need) P->grid = (int)((need + 7) & ~int64_t(7));
      const int64_t per_wg = (tile_base + P->grid - 1) / std::max(P->grid, 1) + 3;
      P->lds_bytes += (size_t)((per_wg * (kBlock / 64) + 15) & ~int64_t(15));
    }
    // Large dense tables: partitioned group-by (partition.h) instead of random global atomics; sparse hash key
    // spaces below 2^31: the same passes over hashed partitions (K8h) instead of the global hash table.
    const bool dense_part = P->mode == MODE_GLOBAL && (int64_t)nslots * G * 8 >= kPartMinBytes;
    const bool hash_part = part_hash_eligible(P, G);
    if ((dense_part || hash_part) && P->star.empty() && tile_base > 0 && P->total_docs < (int64_t)UINT32_MAX &&
        P->cfg.partitioned_group_by) {
      int shift = 16;
      while (shift > 8 && ((int64_t)nslots << shift) * 8 > kPartLds) --shift;
      int64_t parts = (G + (int64_t(1) << shift) - 1) >> shift;
      int pbits = 0, sbits = 0;
      if (hash_part) {
        hash_part_bits(P->cfg, P->group_bound, nslots, &pbits, &sbits);
        shift = 0;
        parts = int64_t(1) << pbits;
      }
      std::vector<int32_t> scol, sf64, sstream(nslots, -1);
      for (int sl = 1; sl < nslots; ++sl) {
        const int f64 = P->slot_kind[sl] == SLOT_SUM_F64 ? 1 : 0;
        int k = -1;
        for (size_t j = 0; j < scol.size(); ++j)
          if (scol[j] == P->slot_col[sl] && sf64[j] == f64) k = (int)j;
        if (k < 0) { scol.push_back(P->slot_col[sl]); sf64.push_back(f64); k = (int)scol.size() - 1; }
        sstream[sl] = k;
      }
      const int64_t rec_bytes = P->total_docs * ((hash_part ? 4 : 2) + 8 * (int64_t)scol.size());
      const size_t pass_lds = (size_t)((parts + 3) & ~int64_t(3)) * 4 + (pure_and ? 0 : (size_t)kMaxStack * kBlock * 4);
      if (parts <= kMaxParts && rec_bytes <= kPartMaxRecordBytes && pass_lds <= 96 * 1024 &&
          (!hash_part || (int)scol.size() <= kHashPartStreams)) {
        P->partitioned = true;
        P->part_hash = hash_part;
        if (hash_part) P->pack_slot = -1;  // K8h accumulates every slot itself (no packed global words)
        P->part_pbits = pbits;
        P->part_sbits = sbits;
        P->part_shift = shift;
        P->num_parts = (int)parts;
        P->stream_col = scol;
        P->stream_f64 = sf64;
        P->slot_stream = sstream;
        // u32 record values when every stream is an integer column whose values fit int32 in every segment
        // (sorted dictionaries: the first and last entries bound them)
        bool v32 = true;
        for (size_t j = 0; j < scol.size() && v32; ++j) {
          const int c = P->query_cols[scol[j]];
          if (sf64[j]) v32 = false;
          else if (c != kDocIdColumn)
            for (const Segment* s : P->segs) {
              const Column& col = s->cols[c];
              int64_t lo, hi;
              if (col.raw) { lo = col.raw_min; hi = col.raw_max; }
              else if (!col.dict.iv.empty()) { lo = col.dict.iv.front(); hi = col.dict.iv.back(); }
              else if (col.dict.size() == 0) continue;
              else { v32 = false; break; }
              if (lo < INT32_MIN || hi > INT32_MAX) { v32 = false; break; }
            }
        }
        P->part_val32 = v32;
        // one integer stream: its value range, for packing values into the coarse records (KPartParams.pack_bits)
        P->part_pack_range = -1;
        if (v32 && scol.size() == 1 && P->query_cols[scol[0]] != kDocIdColumn) {
          int64_t lo = INT64_MAX, hi = INT64_MIN;
          for (const Segment* s : P->segs) {
            const Column& col = s->cols[P->query_cols[scol[0]]];
            if (col.raw) { lo = std::min(lo, col.raw_min); hi = std::max(hi, col.raw_max); }
            else if (!col.dict.iv.empty()) { lo = std::min(lo, col.dict.iv.front()); hi = std::max(hi, col.dict.iv.back()); }
          }
          if (lo <= hi) {
            P->part_pack_min = lo;
            P->part_pack_range = hi - lo;
          }
        }
        P->part_lds = pass_lds;
        int per_cu = occupancy_part_pass(pass_lds, (int)parts, part_coarse_runs((int)parts), 0);
        per_cu = std::max(1, std::min(per_cu, 4));
        P->part_grid = (int)std::max<int64_t>(1, std::min<int64_t>(tile_base, (int64_t)t->num_cus * per_cu));
      }
    }
    return 0;
  };
  // Appends a planned chunk to the plan; tile_shift is added to its records' chunk-relative tile_base (0 keeps
  // them relative, as a streamed launch of the chunk reads them).
  auto merge_chunk = [&](Chunk& C, int64_t tile_shift) {
    if (P->set_words.size() & 1) P->set_words.push_back(0);  // chunk words keep their 8-byte alignment
    const int64_t rec0 = (int64_t)P->segrec.size(), set0 = (int64_t)P->set_words.size();
    if (tile_shift)
      for (size_t r = 0; r < C.rec.size(); r += P->seg_stride)
        reinterpret_cast<KSegHdr*>(C.rec.data() + r)->tile_base += (int32_t)tile_shift;
    for (auto& f : C.set_fix) P->set_fix.emplace_back(rec0 + f.first, set0 + f.second);
    for (auto& f : C.bit_fix) P->bit_fix.emplace_back(rec0 + f.first, P->docbit_words + f.second);
    for (KBitBlock blk : C.bit_blocks) {
      blk.dst += P->docbit_words;
      blk.task_begin += (int32_t)P->bit_tasks.size();
      P->bit_blocks.push_back(blk);
    }
    P->bit_tasks.insert(P->bit_tasks.end(), C.bit_tasks.begin(), C.bit_tasks.end());
    for (KRawTask rt : C.raw_tasks) {
      rt.dst += P->docbit_words;
      if (rt.kind == LEAF_RAW_IN) rt.lo += (int64_t)P->raw_vals.size();
      P->raw_tasks.push_back(rt);
    }
    P->raw_vals.insert(P->raw_vals.end(), C.raw_vals.begin(), C.raw_vals.end());
    P->inv_refs.insert(P->inv_refs.end(), C.inv_refs.begin(), C.inv_refs.end());
    for (auto& g : C.generic) {
      g.rec += rec0 / std::max(P->seg_stride, 1);
      g.out_word = P->generic_words;
      P->generic_words += (int64_t)P->num_leaves * (((int64_t)g.num_docs + 31) / 32);
      P->generic.push_back(std::move(g));
    }
    P->any_leap2 |= C.any_leap2;
    P->gathers |= C.gathers;
    P->docbit_words += C.docbit_words;
    P->segrec.insert(P->segrec.end(), C.rec.begin(), C.rec.end());
    P->set_words.insert(P->set_words.end(), C.set_words.begin(), C.set_words.end());
    P->seg_scanned.insert(P->seg_scanned.end(), C.scanned.begin(), C.scanned.end());
    P->segments_matched_filter += C.matched;
    P->scanned_entries_model += C.entries;
    P->post_exempt_docs += C.exempt;
    for (int k = 0; k < kLeafKinds; ++k) P->leaf_kinds[k] += C.leaf_kinds[k];
    if (P->sel_docs == 0 && C.sel_docs) { P->sel_estimate = C.sel; P->sel_docs = C.sel_docs; }
  };
  const size_t nseg = P->segs.size();
  // Streamed plan (pgpu_plan_create_execute): equal chunks of segments, each launched as soon as it is planned,
  // so the GPU scans chunk c while the host translates chunk c + 1 (Pinot plans and runs each segment's
  // operator on its own worker thread, BaseCombineOperator.java:85-115).
  const bool part_eligible = ((P->mode == MODE_GLOBAL && (int64_t)nslots * G * 8 >= kPartMinBytes) ||
                              part_hash_eligible(P, G)) &&
                             P->cfg.partitioned_group_by;
  // CHAIN / LEAP2 statistics need the direct kernel's register fast path (a pure AND of <= kFastLeaves leaves)
  P->in_kernel_stats = P->pure_and && P->num_leaves <= kFastLeaves && !part_eligible;
  P->leaf_perm = perm;
  const int stream_chunks = se ? stream_chunk_count(P->cfg, nseg) : 1;
  if (se && !any_star && !any_inv && !any_raw_leaf && !part_eligible && stream_chunks > 1) {
    for (Segment* s : P->segs) {
      P->tile_bound += (s->num_docs + kTileDocs - 1) / kTileDocs;
      for (int l = 0; l < P->num_leaves; ++l) {
        const int ty = q->predicates[l].type;
        if (ty == PGPU_PRED_IN || ty == PGPU_PRED_NOT_IN)
          P->set_words_bound += ((int64_t)s->cols[q->predicates[l].column].card + 31) / 32;
      }
    }
    if (!P->scratch) return fail(PGPU_ERR_INVALID_ARGUMENT, "streamed plan without scratch");
    ExecCtx X;
    int64_t tile_off = 0;
    mark();
    for (int c = 0; c < stream_chunks; ++c) {
      Chunk C;
      C.rec.reserve((nseg / stream_chunks + 1) * (size_t)P->seg_stride);
      TRY(plan_range(nseg * c / stream_chunks, nseg * (c + 1) / stream_chunks, C));
      LaunchChunk L;
      L.rec_begin = (int64_t)(P->segrec.size() / P->seg_stride);
      L.fix_begin = (int64_t)P->set_fix.size();
      L.set_begin = (int64_t)P->set_words.size();
      L.tile_begin = tile_off;
      merge_chunk(C, 0);
      L.num_recs = (int64_t)(P->segrec.size() / P->seg_stride) - L.rec_begin;
      L.fix_end = (int64_t)P->set_fix.size();
      L.set_end = (int64_t)P->set_words.size();
      L.num_tiles = C.tiles;
      tile_off += C.tiles;
      P->chunks.push_back(L);
      if (c == 0) {
        TRY(configure(P->tile_bound));
        TRY(exec_prologue(P, se->stream, se->d_table, stream_chunks, X));
      }
      TRY(exec_upload_chunk(P, se->stream, X, L));
      TRY(exec_launch_chunk(P, se->stream, X, L, c));
    }
    mark();
    P->num_tiles = tile_off;
    TRY(exec_epilogue(P, se->stream, X));
    if (trace_on())
      fprintf(stderr, "[pgpu] plan_create (streamed, %d launches): %.1f us (%zu segments)\n", stream_chunks,
              now_us() - t_start, P->segs.size());
    return 0;
  }
  const int nchunks = any_star ? 1 : (int)std::min<size_t>(host_pool().size() + 1, (nseg + plan_chunk_segs(P->cfg) - 1) / plan_chunk_segs(P->cfg));
  std::vector<Chunk> chunks(std::max(nchunks, 1));
  auto run_chunk = [&](int c) {
    Chunk& C = chunks[c];
    C.rec.reserve((nseg / chunks.size() + 1) * (size_t)P->seg_stride);
    C.rc = plan_range(nseg * c / chunks.size(), nseg * (c + 1) / chunks.size(), C);
    if (C.rc) C.err = g_err;
  };
  mark();
  if (chunks.size() == 1) run_chunk(0);
  else host_pool().run((int)chunks.size(), run_chunk);
  mark();
  int64_t tile_base = 0;
  for (Chunk& C : chunks) {
    if (C.rc) return fail(C.rc, "%s", C.err.c_str());
    merge_chunk(C, tile_base);
    tile_base += C.tiles;
  }
  // Small plans (C1: one 1M-doc segment = 123 tiles on 256 CUs): split every tile into 2 or 4 so that at least two
  // tiles per CU run.  The scan kernel's direct path only: not with leap-frog statistics (their per-(tile, wave)
  // bytes are whole 32-doc groups) nor the partitioned group-by (its own passes).
  if (tile_base > 0 && tile_base < 2 * (int64_t)t->num_cus && !P->any_leap2 && P->star.empty() &&
      !(P->mode == MODE_GLOBAL && (int64_t)nslots * G * 8 >= kPartMinBytes)) {
    int sh = 1;
    while (sh < 2 && (tile_base << sh) < 2 * (int64_t)t->num_cus) ++sh;
    P->tile_shift = sh;
    for (size_t r = 0; r + sizeof(KSegHdr) <= P->segrec.size(); r += P->seg_stride) {
      KSegHdr* h = reinterpret_cast<KSegHdr*>(P->segrec.data() + r);
      h->tile_base <<= sh;
      h->num_tiles <<= sh;
    }
    tile_base <<= sh;
  }
  TRY(configure(tile_base));
  P->chunks.assign(1, LaunchChunk{0, (int64_t)(P->segrec.size() / std::max(P->seg_stride, 1)), 0, P->num_tiles, 0,
                                  (int64_t)P->set_fix.size(), 0, (int64_t)P->set_words.size()});
  if (trace_on())
    fprintf(stderr, "[pgpu] plan_create: %.1f us (%zu segments; setup %.1f, ensure %.1f, translate %.1f, rest %.1f)\n",
            now_us() - t_start, P->segs.size(), tr[0] - t_start, tr[1] - tr[0], tr[2] - tr[1], now_us() - tr[2]);
  return 0;
}

// ---- query deadlines (BaseCombineOperator.java:79-132: the combine waits until QueryContext.getEndTimeMs and then
// returns a timeout block; GroupByCombineOperator.java:193-203 for group-by).  The persistent scans compare the
// device wall clock against the deadline converted to clock ticks and stop taking tiles past it.
double epoch_us() {
  return (double)std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::system_clock::now().time_since_epoch()).count();
}

// Device clock ticks at host epoch time end_ms, never earlier than the true reading (the calibration pairs a clock
// value with a host time taken before the kernel that read it, so queueing delay only makes deadlines later).
int deadline_ticks(pgpu_table_s* t, int64_t end_ms, uint64_t* out) {
  std::lock_guard<std::mutex> g(t->clock_mu);
  if (!t->clock_stream) {
    int khz = 0;
    HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, t->device));
    if (khz <= 0) return fail(PGPU_ERR_DEVICE, "device wall clock rate unavailable");
    t->clock_rate_khz = khz;
    HIP_TRY(hipStreamCreateWithFlags(&t->clock_stream, hipStreamNonBlocking));
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&t->clock_pinned), 64, hipHostMallocDefault));
  }
  const double steady = now_us();
  if (t->clock_steady_us < 0 || steady - t->clock_steady_us > 10e6) {
    double best = 1e300;
    for (int i = 0; i < 3 && best > 200.0; ++i) {  // the tightest of up to 3 readings
      const double h0 = epoch_us();
      if (launch_read_clock(t->clock_pinned, t->clock_stream))
        return fail(PGPU_ERR_DEVICE, "clock read launch failed: %s", hipGetErrorString(hipGetLastError()));
      HIP_TRY(hipStreamSynchronize(t->clock_stream));
      const double h1 = epoch_us();
      if (h1 - h0 < best) {
        best = h1 - h0;
        t->clock_host_us = h0;
        t->clock_ticks = *reinterpret_cast<volatile uint64_t*>(t->clock_pinned);
      }
    }
    t->clock_steady_us = steady;
  }
  const double dt_us = (double)end_ms * 1000.0 - t->clock_host_us;
  *out = t->clock_ticks + (dt_us > 0 ? (uint64_t)(dt_us * t->clock_rate_khz / 1000.0) : 0);
  if (*out == 0) *out = 1;
  return 0;
}

// The combine's timeout: aggregation-only plans report BaseCombineOperator's EXECUTION_TIMEOUT_ERROR (250),
// group-by plans GroupByCombineOperator's QUERY_EXECUTION_ERROR (200) wrapping a TimeoutException.
int timeout_fail(const pgpu_plan_s* P) {
  if (P->key_cols.empty())
    return fail(PGPU_ERR_TIMEOUT, "QueryException 250 (EXECUTION_TIMEOUT_ERROR): Timed out while polling results block");
  return fail(PGPU_ERR_TIMEOUT, "QueryException 200 (QUERY_EXECUTION_ERROR): Timed out while combining group-by results "
              "after %lldms", (long long)(P->end_time_ms - P->exec_start_ms));
}

// Leaves the plan's scratch to the device work still queued on `stream` (see Scratch::busy).
int abandon_scratch(Scratch* sc, hipStream_t stream) {
  if (!sc) return 0;
  if (!sc->busy) HIP_TRY(hipEventCreateWithFlags(&sc->busy, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(sc->busy, stream));
  sc->abandoned = true;
  return 0;
}

// Waits for the plan's work on `stream`.  With an end time the wait gives up at it, as the combine's
// _blockingQueue.poll(endTimeMs - now) / _operatorLatch.await(timeoutMs) do (BaseCombineOperator.java:193-203,
// GroupByCombineOperator.java:193-203): the query returns PGPU_ERR_TIMEOUT at its deadline and the device work
// left running keeps its scratch out of the pool until it completes.
int cancel_fail() {
  return fail(PGPU_ERR_CANCELLED, "QueryException 503 (QUERY_CANCELLATION_ERROR): Query was cancelled");
}

bool cancelled(const pgpu_plan_s* P) { return __atomic_load_n(&P->cancel, __ATOMIC_ACQUIRE) != 0; }

int wait_plan(pgpu_plan_s* P, hipStream_t stream) {
  if (!P->scratch) {
    HIP_TRY(hipStreamSynchronize(stream));
    return 0;
  }
  Scratch* sc = P->scratch;
  if (cancelled(P)) return abandon_scratch(sc, stream) ? PGPU_ERR_DEVICE : cancel_fail();
  if (!sc->busy) HIP_TRY(hipEventCreateWithFlags(&sc->busy, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(sc->busy, stream));
  // Polled, not a blocking synchronise: a pgpu_plan_cancel from another thread must end the wait.  Spinning (as the
  // HIP runtime's own synchronise does) for the first ~2 ms keeps the wake-up latency of short queries at the
  // poll interval; longer waits back off to 20 us sleeps.
  const auto t0 = std::chrono::steady_clock::now();
  // a combined plan's stream holds collectives that complete only when every peer joins them: the wait also ends at
  // the communicator's timeout, and an expired wait aborts the communicator (the collectives' kernels exit)
  const int64_t comm_lim = P->comm_used ? P->comm_used->timeout_ms.load(std::memory_order_relaxed) : 0;
  for (int spin = 0;; ++spin) {
    const hipError_t e = hipEventQuery(sc->busy);
    if (e == hipSuccess) return 0;
    if (e != hipErrorNotReady) return fail(PGPU_ERR_DEVICE, "query wait failed: %s", hipGetErrorString(e));
    if (cancelled(P)) {
      sc->abandoned = true;
      if (P->comm_used) P->comm_used->abort();
      return cancel_fail();
    }
    if (P->end_time_ms > 0 && epoch_us() >= (double)P->end_time_ms * 1000.0) {
      sc->abandoned = true;
      if (P->comm_used) P->comm_used->abort();
      return timeout_fail(P);
    }
    if (comm_lim > 0 && (spin & 63) == 63 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(comm_lim)) {
      sc->abandoned = true;
      P->comm_used->abort();
      return fail(PGPU_ERR_TIMEOUT, "the combine's collectives did not complete within the communicator's timeout "
                  "(%lld ms): a peer rank never joined them; communicator aborted", (long long)comm_lim);
    }
    if ((spin & 63) == 63 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2))
      std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

// Raw-value leaves of a plan: its tasks, their 256-group jobs and IN keys staged through pinned memory in one device
// buffer, then raw_leaf_bitmap_kernel writes the leaves' docbits regions (sc->docbits, sized by the caller).
int launch_raw_leaves(const pgpu_plan_s* P, Scratch* sc, hipStream_t stream) {
  if (P->raw_tasks.empty()) return 0;
  std::vector<KRawJob> jobs;
  for (size_t i = 0; i < P->raw_tasks.size(); ++i) {
    const int64_t ngroups = ((int64_t)P->raw_tasks[i].num_docs + 31) / 32;
    for (int64_t g0 = 0; g0 < ngroups; g0 += kBlock) jobs.push_back(KRawJob{(int32_t)i, (int32_t)g0});
  }
  const size_t tb = P->raw_tasks.size() * sizeof(KRawTask), jb = (jobs.size() * sizeof(KRawJob) + 15) & ~size_t(15);
  const size_t vb = std::max<size_t>(P->raw_vals.size(), 1) * 8;
  TRY(sc->rawtasks.ensure(tb + jb + vb));
  TRY(sc->rawstage.ensure(tb + jb + vb));
  uint8_t* hs = reinterpret_cast<uint8_t*>(sc->rawstage.p);
  memcpy(hs, P->raw_tasks.data(), tb);
  if (!jobs.empty()) memcpy(hs + tb, jobs.data(), jobs.size() * sizeof(KRawJob));
  if (!P->raw_vals.empty()) memcpy(hs + tb + jb, P->raw_vals.data(), P->raw_vals.size() * 8);
  HIP_TRY(hipMemcpyAsync(sc->rawtasks.p, hs, tb + jb + vb, hipMemcpyHostToDevice, stream));
  uint8_t* d = sc->rawtasks.as<uint8_t>();
  if (launch_raw_leaf_bitmaps(reinterpret_cast<const KRawJob*>(d + tb), (int64_t)jobs.size(),
                              reinterpret_cast<const KRawTask*>(d), reinterpret_cast<const int64_t*>(d + tb + jb),
                              sc->docbits.as<uint32_t>(), stream))
    return fail(PGPU_ERR_DEVICE, "raw-value filter launch failed: %s", hipGetErrorString(hipGetLastError()));
  return 0;
}

// ---- execution, in three phases so that plan_create can launch segment chunks while it still plans the rest
// (streamed plans): prologue (buffers, table init, stats), one launch per chunk of segment records, epilogue
// (star-tree kernels, slab reduce).  A plan that is not streamed is one chunk.
// KParams.pack_slot (planned with the LDS table's rows, lds_pack_slot) and narrow of a dense LDS plan, from the value
// ranges of its integer columns in every segment (sorted dictionaries: first and last entries; raw columns: their
// decoded range).  PGPU_NO_DENSE_NARROW=1: no 32-bit min / max (A/B).
void dense_lds_forms(const pgpu_plan_s* P, int32_t* pack_slot, uint32_t* narrow) {
  *pack_slot = P->mode == MODE_LDS || P->mode == MODE_HASH ? P->pack_slot : -1;  // planned with the table layout
  *narrow = 0;
  if (!P->dense || P->mode != MODE_LDS || P->num_keys <= 1 || !P->star.empty() || P->grid <= 0) return;
  for (size_t s = 0; s < P->slot_kind.size() && s < 32; ++s) {
    const int kind = P->slot_kind[s], c = P->slot_tcol[s];
    if ((kind != SLOT_MIN_KEY && kind != SLOT_MAX_KEY) || c < 0 || c == kDocIdColumn) continue;
    if (!is_int_type(P->table->types[c])) continue;
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    bool known = true;
    for (const Segment* seg : P->segs) {
      const Column& col = seg->cols[c];
      if (col.raw) { lo = std::min(lo, col.raw_min); hi = std::max(hi, col.raw_max); }
      else if (!col.dict.iv.empty()) { lo = std::min(lo, col.dict.iv.front()); hi = std::max(hi, col.dict.iv.back()); }
      else if (col.dict.size() != 0) { known = false; break; }
    }
    if (!known || lo > hi || lo < 0) continue;
    if (hi < INT64_C(0xFFFFFFFF)) *narrow |= 1u << s;
  }
}

int exec_prologue(pgpu_plan_s* P, hipStream_t stream, void* d_table, int max_chunks, ExecCtx& X) {
  X.t_start = trace_on() ? now_us() : 0;
  if (cancelled(P)) return cancel_fail();  // nothing is launched for a cancelled query
  uint64_t deadline = 0;
  if (P->end_time_ms > 0) {  // past the end time already: nothing is launched
    P->exec_start_ms = (int64_t)(epoch_us() / 1000.0);
    if (P->exec_start_ms >= P->end_time_ms) return timeout_fail(P);
    TRY(deadline_ticks(P->table, P->end_time_ms, &deadline));
  }
  // the state a previous execution's combine left (pgpu_plan_combine): planned slot kinds, no shard, no merged table
  if (!P->slot_kind_planned.empty()) {
    P->slot_kind = P->slot_kind_planned;
    P->slot_kind_planned.clear();
  }
  P->shard = nullptr;
  P->shard_begin = P->shard_count = 0;
  P->comm_used = nullptr;
  P->merged_records = -1;
  Scratch* sc = P->scratch;
  X.nslots = (int)P->slot_kind.size();
  const int nslots = X.nslots;
  X.words = P->part_hash ? 0 : (int64_t)nslots * P->num_keys;  // hashed partitions: records, no table
  for (auto& e : sc->ev)
    if (!e) HIP_TRY(hipEventCreate(&e));
  if ((int)sc->cev.size() < 2 * max_chunks) {
    const size_t old = sc->cev.size();
    sc->cev.resize(2 * max_chunks, nullptr);
    for (size_t i = old; i < sc->cev.size(); ++i) HIP_TRY(hipEventCreate(&sc->cev[i]));
  }
  X.mark("events");
  PGPU_TIMING_RECORD(sc->ev[0], stream);
  X.mark("event 0 recorded");
  TRY(sc->sets.ensure(std::max<size_t>(std::max<size_t>(P->set_words.size(), (size_t)P->set_words_bound) * 4, 16)));
  const size_t rec_cap = std::max<size_t>((size_t)P->segs.size() * P->seg_stride, P->segrec.size());
  TRY(sc->segrec.ensure(std::max<size_t>(rec_cap, 16)));
  TRY(sc->stage.ensure(std::max<size_t>(rec_cap + (size_t)std::max<int64_t>(P->set_words_bound,
                                                                             (int64_t)P->set_words.size()) * 4, 16)));
  // Statistics words (docs matched, entries scanned, star-tree docs, timeout flag): right after the group table when
  // the table is internal, so finalize reads both with one copy
  constexpr size_t kStatsBytes = 64;
  unsigned long long* stats;
  if (!d_table) {
    TRY(sc->table.ensure((size_t)X.words * 8 + kStatsBytes));
    stats = reinterpret_cast<unsigned long long*>(sc->table.as<uint8_t>() + (size_t)X.words * 8);
  } else {
    TRY(sc->stats.ensure(kStatsBytes));
    stats = sc->stats.as<unsigned long long>();
  }
  P->d_stats = stats;
  X.mark("buffers");
  HIP_TRY(hipMemsetAsync(stats, 0, kStatsBytes, stream));
  X.mark("statistics memset queued");
  X.segrec = sc->segrec.as<uint8_t>();
  X.sets = sc->sets.as<uint32_t>();
  TRY(sc->tile_seg.ensure((size_t)std::max<int64_t>(std::max<int64_t>(P->num_tiles, P->tile_bound), 1) * 4));
  X.tile_seg = sc->tile_seg.as<int32_t>();
  X.from_image = P->image && P->chunks.size() == 1 && P->docbit_words == 0 && !P->set_words_bound && !P->tile_bound;
  sc->image = X.from_image ? P->image : nullptr;
  if (X.from_image) {  // build the cached plan's device image once; later executions wait for it
    DeviceImage& im = *P->image;
    std::lock_guard<std::mutex> g(im.mu);
    if (!im.uploaded) {
      const size_t rn = P->segrec.size(), sn = P->set_words.size() * 4;
      TRY(im.segrec.ensure(std::max<size_t>(rn, 16)));
      TRY(im.sets.ensure(std::max<size_t>(sn, 16)));
      TRY(im.tile_seg.ensure((size_t)std::max<int64_t>(P->num_tiles, 1) * 4));
      if (!im.built) HIP_TRY(hipEventCreateWithFlags(&im.built, hipEventDisableTiming));
      uint8_t* stage = reinterpret_cast<uint8_t*>(sc->stage.p);
      if (rn) memcpy(stage, P->segrec.data(), rn);
      for (const auto& f : P->set_fix) {
        const uint32_t* ptr = im.sets.as<uint32_t>() + f.second;
        memcpy(stage + f.first, &ptr, sizeof ptr);
      }
      if (sn) memcpy(stage + rn, P->set_words.data(), sn);
      if (rn) HIP_TRY(hipMemcpyAsync(im.segrec.p, stage, rn, hipMemcpyHostToDevice, stream));
      if (sn) HIP_TRY(hipMemcpyAsync(im.sets.p, stage + rn, sn, hipMemcpyHostToDevice, stream));
      // the plan's scan records (segments its filter prunes or its star-trees answer have none)
      const int32_t nrec = P->seg_stride > 0 ? (int32_t)(P->segrec.size() / P->seg_stride) : 0;
      if (nrec > 0 &&
          launch_expand_tiles(im.segrec.as<uint8_t>(), P->seg_stride, nrec, im.tile_seg.as<int32_t>(), 0,
                              stats, stream))
        return fail(PGPU_ERR_DEVICE, "expand launch failed: %s", hipGetErrorString(hipGetLastError()));
      HIP_TRY(hipEventRecord(im.built, stream));
      im.uploaded = true;
    } else if (!im.ready) {
      if (hipEventQuery(im.built) == hipSuccess) im.ready = true;
      else HIP_TRY(hipStreamWaitEvent(stream, im.built, 0));
    }
    X.segrec = im.segrec.as<uint8_t>();
    X.sets = im.sets.as<uint32_t>();
    X.tile_seg = im.tile_seg.as<int32_t>();
  }
  if (P->docbit_words > 0) TRY(sc->docbits.ensure((size_t)P->docbit_words * 4));
  if (!P->bit_blocks.empty()) {  // BitmapBasedFilterOperator leaves: OR the matching dictIds' containers
    TRY(sc->bittasks.ensure(std::max<size_t>(P->bit_tasks.size(), 1) * sizeof(KBitTask)));
    TRY(sc->bitblocks.ensure(P->bit_blocks.size() * sizeof(KBitBlock)));
    // staged through pinned memory: asynchronous copies (pageable sources would block the host)
    const size_t tb = P->bit_tasks.size() * sizeof(KBitTask), bb = P->bit_blocks.size() * sizeof(KBitBlock);
    TRY(sc->bitstage.ensure(tb + bb));
    uint8_t* hs = reinterpret_cast<uint8_t*>(sc->bitstage.p);
    if (tb) memcpy(hs, P->bit_tasks.data(), tb);
    memcpy(hs + tb, P->bit_blocks.data(), bb);
    if (tb) HIP_TRY(hipMemcpyAsync(sc->bittasks.p, hs, tb, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipMemcpyAsync(sc->bitblocks.p, hs + tb, bb, hipMemcpyHostToDevice, stream));
    if (launch_inv_materialize(sc->bitblocks.as<KBitBlock>(), (int64_t)P->bit_blocks.size(),
                               sc->bittasks.as<KBitTask>(), sc->docbits.as<uint32_t>(), stream))
      return fail(PGPU_ERR_DEVICE, "inverted-index materialise launch failed: %s",
                  hipGetErrorString(hipGetLastError()));
  }
  TRY(launch_raw_leaves(P, sc, stream));  // raw-value leaves' docbits regions
  uint64_t* table = d_table ? reinterpret_cast<uint64_t*>(d_table) : sc->table.as<uint64_t>();
  X.table = table;
  P->d_table_used = table;
  KParams& kp = X.kp;
  memset(&kp, 0, sizeof kp);
  kp.pack_slot = -1;
  kp.deadline = deadline;
  kp.seg_stride = P->seg_stride;
  kp.num_cols = (int)P->query_cols.size();
  kp.num_ops = (int)P->ops.size();
  kp.pure_and = P->pure_and ? 1 : 0;
  for (size_t i = 0; i < P->ops.size(); ++i) kp.ops[i] = P->ops[i];
  kp.num_leaves = P->num_leaves;
  for (int i = 0; i < P->num_leaves; ++i) kp.leaf_col[i] = P->leaf_slot[i];
  kp.num_keys = (int)P->key_cols.size();
  for (size_t j = 0; j < P->key_cols.size(); ++j) {
    int slot = 0;
    for (size_t i = 0; i < P->query_cols.size(); ++i) if (P->query_cols[i] == P->key_cols[j]) slot = (int)i;
    kp.key_col[j] = slot;
    kp.key_stride[j] = P->key_stride[j];
  }
  kp.num_keys_total = P->num_keys;
  kp.key_bias = P->key_bias;
  kp.tile_shift = P->tile_shift;
  // Tile order: interleaved (the tiles in flight on an XCD come from ~one segment: its dictionaries stay in that
  // XCD's L2 for the per-doc gathers) or chunked (a workgroup's tiles follow each other in one segment: its records
  // and leaf registers are loaded once per run).  Plans with many matches (dense, and the sparse ones of estimated
  // selectivity >= 1/16) gather enough to want the former: C4's scan path 151 -> 141 us interleaved, where C3
  // (0.18 %) loses 7 % and the indexed C3 15 % (profiles/r05_ab_summary.txt, session za).
  kp.tile_chunks = P->dense || P->fast_wide ? 0 : 1;
  kp.num_slots = nslots;
  for (int sl = 0; sl < nslots; ++sl) { kp.slot_kind[sl] = P->slot_kind[sl]; kp.slot_col[sl] = P->slot_col[sl]; }
  kp.pair_leaves = 1;
  dense_lds_forms(P, &kp.pack_slot, &kp.narrow);
  kp.pack_shift = P->pack_shift;
  kp.stats = stats;
  if (P->leap_reserved) {  // one byte per (tile, wave) of the plan, written by the scan kernel for LEAP2 segments
    TRY(sc->leap_maps.ensure((size_t)std::max<int64_t>(std::max<int64_t>(P->num_tiles, P->tile_bound), 1) *
                             (kBlock / 64)));
    kp.leap_maps = sc->leap_maps.as<uint8_t>();
  }
  const int star_blocks = P->star_batches * P->star_chunks;
  if (P->mode == MODE_LDS) {
    TRY(sc->slab.ensure((size_t)std::max(max_chunks * P->grid + star_blocks, 1) * X.words * 8));
    kp.slab = sc->slab.as<uint64_t>();
  } else {
    if (P->mode == MODE_HASH && !P->part_hash) {
      TRY(sc->hash_keys.ensure((size_t)P->num_keys * 8));
      kp.hash_keys = sc->hash_keys.as<unsigned long long>();
      if (!P->stage_end.empty()) {
        int64_t total = 0;
        kp.num_stages = (int)P->stage_end.size();
        for (int s = 0; s < kp.num_stages; ++s) {
          kp.stage_end[s] = P->stage_end[s];
          kp.stage_cap[s] = P->stage_cap[s];
          kp.stage_mult[s] = P->stage_mult[s];
          kp.stage_off[s] = total;
          total += P->stage_cap[s];
        }
        TRY(sc->stage_keys.ensure((size_t)total * 8));
        HIP_TRY(hipMemsetAsync(sc->stage_keys.p, 0xFF, (size_t)total * 8, stream));  // every slot empty (~0)
        kp.stage_keys = sc->stage_keys.as<unsigned long long>();
      }
    }
    if (!P->partitioned &&  // the partitioned path stores every table word itself
        launch_table_init(table, P->slot_kind.data(), nslots, P->num_keys, kp.hash_keys, stream))
      return fail(PGPU_ERR_DEVICE, "table init launch failed: %s", hipGetErrorString(hipGetLastError()));
    kp.table = table;
  }
  P->launches_done = 0;
  return 0;
}

// Uploads chunk c's records (SET pointers patched to the device bitsets) and its bitset words.
int exec_upload_chunk(pgpu_plan_s* P, hipStream_t stream, const ExecCtx& X, const LaunchChunk& C) {
  if (X.from_image) return 0;  // the cached plan's device image holds the records
  Scratch* sc = P->scratch;
  uint8_t* stage = reinterpret_cast<uint8_t*>(sc->stage.p);
  const size_t r0 = (size_t)C.rec_begin * P->seg_stride, rn = (size_t)C.num_recs * P->seg_stride;
  if (rn) memcpy(stage + r0, P->segrec.data() + r0, rn);
  for (int64_t i = C.fix_begin; i < C.fix_end; ++i) {
    const auto& f = P->set_fix[i];
    const uint32_t* ptr = sc->sets.as<uint32_t>() + f.second;
    memcpy(stage + f.first, &ptr, sizeof ptr);
  }
  for (const auto& f : P->bit_fix)
    if (f.first >= (int64_t)r0 && f.first < (int64_t)(r0 + rn)) {
      const uint32_t* ptr = sc->docbits.as<uint32_t>() + f.second;
      memcpy(stage + f.first, &ptr, sizeof ptr);
    }
  if (rn) HIP_TRY(hipMemcpyAsync(sc->segrec.as<uint8_t>() + r0, stage + r0, rn, hipMemcpyHostToDevice, stream));
  if (C.set_end > C.set_begin) {
    const size_t set_off = (size_t)P->segs.size() * P->seg_stride + (size_t)C.set_begin * 4;
    const size_t bytes = (size_t)(C.set_end - C.set_begin) * 4;
    if (set_off + bytes > sc->stage.cap) return fail(PGPU_ERR_DEVICE, "set staging overflow");
    memcpy(stage + set_off, P->set_words.data() + C.set_begin, bytes);
    HIP_TRY(hipMemcpyAsync(sc->sets.as<uint32_t>() + C.set_begin, stage + set_off, bytes, hipMemcpyHostToDevice,
                           stream));
  }
  return 0;
}

// Launches the scan of chunk c (records already uploaded): tile map of its records, then the scan kernel (or the
// partitioned group-by) over its tiles into slab region c.
// PGPU_TRACE=check (diagnostics): before a scan launch, the records and tile map the kernel will read are copied
// back and compared with the plan's host records (pointer fields patched at upload skipped); a mismatch fails the
// query (PGPU_ERR_DEVICE) instead of launching on them.
bool check_launch_on() {
  static const bool on = diag("check");
  return on;
}
int check_launch_inputs(const pgpu_plan_s* P, hipStream_t stream, const ExecCtx& X, const LaunchChunk& C) {
  HIP_TRY(hipStreamSynchronize(stream));
  const size_t r0 = (size_t)C.rec_begin * P->seg_stride, rn = (size_t)C.num_recs * P->seg_stride;
  std::vector<uint8_t> dev(rn);
  std::vector<int32_t> tiles((size_t)std::max<int64_t>(C.num_tiles, 0));
  if (rn) HIP_TRY(hipMemcpy(dev.data(), X.segrec + r0, rn, hipMemcpyDeviceToHost));
  if (!tiles.empty()) HIP_TRY(hipMemcpy(tiles.data(), X.tile_seg + C.tile_begin, tiles.size() * 4, hipMemcpyDeviceToHost));
  if (P->segrec.size() >= r0 + rn) {
    std::vector<char> skip(rn, 0);
    auto mark = [&](int64_t off) {
      if (off >= (int64_t)r0 && off + 8 <= (int64_t)(r0 + rn)) memset(skip.data() + (off - r0), 1, 8);
    };
    for (const auto& f : P->set_fix) mark(f.first);
    for (const auto& f : P->bit_fix) mark(f.first);
    for (size_t i = 0; i < rn; ++i)
      if (!skip[i] && dev[i] != P->segrec[r0 + i])
        return fail(PGPU_ERR_DEVICE, "launch check: device record byte %zu differs from the plan (%u vs %u)", r0 + i,
                    dev[i], P->segrec[r0 + i]);
  }
  int32_t prev = 0;
  for (size_t i = 0; i < tiles.size(); ++i) {
    if (tiles[i] < prev || tiles[i] >= C.num_recs)
      return fail(PGPU_ERR_DEVICE, "launch check: tile %zu maps to record %d of %lld", i, tiles[i],
                  (long long)C.num_recs);
    prev = tiles[i];
  }
  return 0;
}

// The scan instance a plan launches (k_direct.hip): 2 dense "simple", 1 dense, 3 index + scan pair, 5 / 4 pure-AND
// sparse with 4 / 2-doc lane batches, 0 the general sparse one.
int scan_variant(const pgpu_plan_s* P) {
  return P->dense_simple ? 2 : P->dense ? 1 : P->pair_variant ? 3 : P->fast_wide ? 5 : P->fast_variant ? 4 : 0;
}

// PGPU_TRACE=wgtimes with a PGPU_DIAG_WG_TIMES build: every scan launch is synchronised and its workgroups' start /
// tile-loop end / end times (wall clock, relative to the earliest start) summarised on stderr -- how much of a launch
// is its ramp, its tail and the imbalance of the static tile split.
unsigned long long* g_diag_times = nullptr;
int diag_wg_times_begin(KParams& kp, int grid, hipStream_t stream) {
  constexpr int kMaxWgs = 1 << 16;
  if (grid > kMaxWgs) return 0;
  if (!g_diag_times) HIP_TRY(hipMalloc(&g_diag_times, (size_t)kMaxWgs * 32));
  HIP_TRY(hipMemsetAsync(g_diag_times, 0, (size_t)grid * 32, stream));
  kp.diag_times = g_diag_times;
  return 0;
}

int diag_wg_times_report(pgpu_table_s* t, const KParams& kp, int grid, hipStream_t stream) {
  if (!kp.diag_times) return 0;
  std::vector<unsigned long long> h((size_t)grid * 4);
  HIP_TRY(hipMemcpyAsync(h.data(), kp.diag_times, h.size() * 8, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  int khz = 100000;
  hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, t->device);
  const double us = 1000.0 / khz;
  unsigned long long t0 = ~0ull;
  for (int b = 0; b < grid; ++b) if (h[4 * b + 2]) t0 = std::min(t0, h[4 * b]);
  if (t0 == ~0ull) return 0;
  std::vector<double> st, le, en, tiles;
  double xcd_end[8] = {0};
  for (int b = 0; b < grid; ++b) {
    if (!h[4 * b + 2]) continue;
    st.push_back((h[4 * b] - t0) * us);
    le.push_back((h[4 * b + 1] - t0) * us);
    en.push_back((h[4 * b + 2] - t0) * us);
    tiles.push_back((double)h[4 * b + 3]);
    xcd_end[b & 7] = std::max(xcd_end[b & 7], en.back());
  }
  auto pct = [](std::vector<double> v, double q) {
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(q * (v.size() - 1) + 0.5))];
  };
  fprintf(stderr, "[pgpu] wgtimes grid %d tiles %d: start p50 %.1f max %.1f | loop end p0 %.1f p10 %.1f p50 %.1f p90 %.1f "
          "max %.1f | end max %.1f us | tiles/wg %.0f..%.0f | xcd end %.1f %.1f %.1f %.1f %.1f %.1f %.1f %.1f\n",
          grid, kp.num_tiles, pct(st, 0.5), pct(st, 1.0), pct(le, 0.0), pct(le, 0.1), pct(le, 0.5), pct(le, 0.9),
          pct(le, 1.0), pct(en, 1.0), pct(tiles, 0.0), pct(tiles, 1.0), xcd_end[0], xcd_end[1], xcd_end[2], xcd_end[3],
          xcd_end[4], xcd_end[5], xcd_end[6], xcd_end[7]);
  return 0;
}

// Run-time claims of a chunked scan launch (KParams.claim; library builds with -DPGPU_TILE_CLAIMS only): the static
// runs cover the first PGPU_CLAIM_STATIC_PM / 1000 of the tiles and the rest is claimed in runs of 1/PGPU_CLAIM_DIV
// of a workgroup's share.  The counters are u32 words 12..15 of the statistics block (zeroed per execution): launches
// 0-3 of a plan.  Measured on MI355X and not the default (r06 session b, profiles/r06_ab_summary.txt): C3's scan
// 729 -> 711 us at 1000 segments but its pipelined step 0.687 -> 0.719 ms, and at 125 segments 119 -> 145 us (every
// claimed tile reloads its segment's records behind a workgroup barrier).
#ifndef PGPU_CLAIM_STATIC_PM
#define PGPU_CLAIM_STATIC_PM 750
#endif
#ifndef PGPU_CLAIM_DIV
#define PGPU_CLAIM_DIV 16
#endif
void set_tile_claims(KParams& kp, unsigned long long* d_stats, int grid, int launch) {
  kp.claim = nullptr;
#ifdef PGPU_TILE_CLAIMS
  const int64_t share = (int64_t)kp.num_tiles / std::max(grid, 1);
  if (!kp.tile_chunks || grid < 64 || (grid & 7) || launch >= 4 || share < 8) return;
  kp.claim = reinterpret_cast<unsigned int*>(d_stats + 6) + launch;
  kp.claim_base = (int32_t)((int64_t)kp.num_tiles * PGPU_CLAIM_STATIC_PM / 1000);
  kp.claim_tiles = (int32_t)std::max<int64_t>(1, share / PGPU_CLAIM_DIV);
#endif
}

int exec_launch_chunk(pgpu_plan_s* P, hipStream_t stream, ExecCtx& X, const LaunchChunk& C, int c) {
  Scratch* sc = P->scratch;
  KParams kp = X.kp;
  kp.segs = X.segrec + (size_t)C.rec_begin * P->seg_stride;
  kp.num_segs = (int)C.num_recs;
  kp.num_tiles = (int32_t)C.num_tiles;
  kp.tile_seg = X.tile_seg + C.tile_begin;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(P->grid, C.num_tiles));
  if (P->mode == MODE_LDS) kp.slab = X.kp.slab + X.slabs_used * X.words;
  if (kp.leap_maps) kp.leap_maps += C.tile_begin * (kBlock / 64);
  if (X.from_image) {  // the tile map is in the image; only the deadline gate remains (and only with a deadline)
    if (C.num_tiles > 0 && kp.deadline && launch_deadline_gate(kp.deadline, kp.stats, stream))
      return fail(PGPU_ERR_DEVICE, "gate launch failed: %s", hipGetErrorString(hipGetLastError()));
  } else if (C.num_recs > 0 && launch_expand_tiles(kp.segs, kp.seg_stride, kp.num_segs, X.tile_seg + C.tile_begin,
                                                   kp.deadline, kp.stats, stream)) {
    return fail(PGPU_ERR_DEVICE, "expand launch failed: %s", hipGetErrorString(hipGetLastError()));
  }
  if (check_launch_on()) TRY(check_launch_inputs(P, stream, X, C));
  if (c == 0) PGPU_TIMING_RECORD(sc->ev[1], stream);
  PGPU_TIMING_RECORD(sc->cev[2 * c], stream);
  if (C.num_tiles > 0 && P->partitioned) {
    const int nslots = X.nslots;
    KPartParams pp;
    memset(&pp, 0, sizeof pp);
    pp.base = kp;
    pp.pshift = P->part_shift;
    pp.num_parts = P->num_parts;
    pp.num_streams = (int)P->stream_col.size();
    for (size_t j = 0; j < P->stream_col.size(); ++j) { pp.stream_col[j] = P->stream_col[j]; pp.stream_f64[j] = P->stream_f64[j]; }
    for (int sl = 0; sl < nslots; ++sl) pp.slot_stream[sl] = P->slot_stream[sl];
    const int64_t cap = std::max<int64_t>(P->total_docs, 1);
    TRY(sc->part_start.ensure((size_t)(P->num_parts + 1) * 4));
    const int cshift = part_coarse_shift(P->num_parts);
    pp.cshift = cshift;
    pp.num_coarse = part_coarse_runs(P->num_parts);
    pp.chunks_per_coarse = std::max(1, 1024 / pp.num_coarse);
    {  // K8e batch: as many records as fit 96 KB of LDS beside the per-partition counters, a multiple of kBlock
      const int kb = P->part_hash ? 4 : 2;  // staged key bytes
      const int64_t fixed = (int64_t)part_split_lds(cshift, pp.num_streams, 0, kb);
      const int64_t b = (96 * 1024 - fixed) / (8 * pp.num_streams + 4 + kb) / kBlock * kBlock;
      pp.split_batch = (int)std::max<int64_t>(kBlock, std::min<int64_t>(kSplitBatch, b));
    }
    TRY(sc->coarse_fill.ensure((size_t)pp.num_coarse * 4));
    TRY(sc->fine_fill.ensure((size_t)P->num_parts * 4));
    if (cshift > 0) {
      TRY(sc->mid_key.ensure((size_t)cap * 4));
      TRY(sc->mid_val.ensure(std::max<size_t>((size_t)cap * 8 * pp.num_streams, 8)));
      pp.mid_key = sc->mid_key.as<uint32_t>();
      pp.mid_val = sc->mid_val.as<uint64_t>();
    }
    pp.coarse_fill = sc->coarse_fill.as<uint32_t>();
    pp.fine_fill = sc->fine_fill.as<uint32_t>();
    if (P->part_hash) {
      pp.hashed = 1;
      pp.mid_pair = cshift > 0 && pp.num_streams == 1 && P->part_val32 && !P->stream_f64[0] ? 1 : 0;
      pp.pbits = P->part_pbits;
      pp.sbits = P->part_sbits;
      TRY(sc->rec_key32.ensure((size_t)cap * 4));
      pp.rec_key32 = sc->rec_key32.as<uint32_t>();
      // the groups' compacted records, where finalize's compaction of a hash table would put them
      const int64_t ocap = part_hash_out_cap(P);
      TRY(sc->ckeys.ensure((size_t)ocap * 8 * (1 + nslots)));
      TRY(sc->counter.ensure(64));
      HIP_TRY(hipMemsetAsync(sc->counter.p, 0, 8, stream));
      pp.out_rec = sc->ckeys.as<uint64_t>();
      pp.out_count = sc->counter.as<unsigned long long>();
      pp.out_cap = ocap;
      TRY(sc->part_mm.ensure((size_t)P->num_parts * 2 * nslots * 8));
      pp.out_mm = sc->part_mm.as<unsigned long long>();
      P->part_hash_live = true;
    } else {
      TRY(sc->rec_key.ensure((size_t)cap * 2));
    }
    TRY(sc->rec_val.ensure(std::max<size_t>((size_t)cap * 8 * pp.num_streams, 8)));
    pp.part_start = sc->part_start.as<uint32_t>();
    pp.rec_key = sc->rec_key.as<uint16_t>();
    pp.rec_val = sc->rec_val.as<uint64_t>();
    pp.rec_cap = cap;
    pp.val32 = P->part_val32 ? 1 : 0;
    if (P->part_hash && P->part_pack_range >= 0 && pp.num_streams == 1 && pp.val32 && P->part_pbits >= 1) {
      // hashed partitions: K8e's records packed as hk below the partition bits | (value - pack_min) above them
      int vb = 0;
      while (vb < 32 && (P->part_pack_range >> vb) != 0) ++vb;
      if (vb <= P->part_pbits) {
        pp.fine_pack = 1;
        pp.pack_min = P->part_pack_min;
        pp.pack_range = P->part_pack_range;
        pp.cs_pack = nslots == 2 && P->slot_kind[0] == SLOT_COUNT && P->slot_kind[1] == SLOT_SUM_I64 &&
                     P->slot_stream[1] == 0 ? 1 : 0;
      }
    } else if (!P->part_hash && cshift > 0 && P->part_pack_range >= 0) {
      const int free_bits = 32 - (pp.pshift + cshift);
      int vb = 0;
      while (vb < free_bits && (P->part_pack_range >> vb) != 0) ++vb;
      if ((P->part_pack_range >> vb) == 0) {
        pp.pack_bits = std::max(vb, 1);
        pp.pack_min = P->part_pack_min;
        pp.fine_pack = pp.pshift + pp.pack_bits <= 32 && pp.num_streams == 1 ? 1 : 0;
        pp.cs_pack = pp.fine_pack && nslots == 2 && P->slot_kind[0] == SLOT_COUNT &&
                     P->slot_kind[1] == SLOT_SUM_I64 && P->slot_stream[1] == 0 ? 1 : 0;
        pp.pack_range = P->part_pack_range;
      }
    }
    int grid = P->part_grid;
#ifndef PGPU_PART_NO_STAGE  // (defined only by an A/B build of the library: every record stored from its lane)
    // one-word records with <= 64 coarse runs: K8c stages each wave's records by run in LDS and stores them in runs;
    // the grid (K8a's too) follows that instance's occupancy
    pp.staged = pp.cshift > 0 && pp.num_coarse <= 64 ? (pp.pack_bits > 0 ? 1 : pp.mid_pair ? 2 : 0) : 0;
    if (pp.staged) {
      if (P->part_grid_staged[pp.staged - 1] <= 0) {
        const int per_cu =
            std::max(1, std::min(occupancy_part_pass(P->part_lds, P->num_parts, pp.num_coarse, pp.staged), 4));
        P->part_grid_staged[pp.staged - 1] =
            (int)std::max<int64_t>(1, std::min<int64_t>(P->num_tiles, (int64_t)P->table->num_cus * per_cu));
      }
      grid = P->part_grid_staged[pp.staged - 1];
    }
#endif
    TRY(sc->block_off.ensure((size_t)grid * pp.num_coarse * 4));
    pp.block_off = sc->block_off.as<uint32_t>();
    if (launch_partitioned(pp, grid, P->part_lds, stream))
      return fail(PGPU_ERR_DEVICE, "partitioned group-by launch failed: %s", hipGetErrorString(hipGetLastError()));
  } else if (C.num_tiles > 0) {
    static const bool wg_times = diag("wgtimes");
    if (wg_times) TRY(diag_wg_times_begin(kp, grid, stream));
    set_tile_claims(kp, P->d_stats, grid, c);
    const int rc = launch_filter_groupby(kp, P->mode,
                                         scan_variant(P),
                                         grid, P->lds_bytes, stream);
    if (rc) return fail(PGPU_ERR_DEVICE, "scan launch failed: %s", hipGetErrorString(hipGetLastError()));
    if (wg_times) TRY(diag_wg_times_report(P->table, kp, grid, stream));
  }
  PGPU_TIMING_RECORD(sc->cev[2 * c + 1], stream);
  if (C.num_tiles > 0 && P->any_leap2 && P->leap_reserved && !P->partitioned) {
    if (P->chunks.size() == 1 && P->mode == MODE_LDS) {  // folded into the epilogue's launch
      X.leap_segs = kp.segs;
      X.leap_nsegs = kp.num_segs;
    } else if (launch_leap2_compose(kp.segs, kp.seg_stride, kp.num_segs, kp.leap_maps, kp.stats, stream)) {
      return fail(PGPU_ERR_DEVICE, "filter statistics launch failed: %s", hipGetErrorString(hipGetLastError()));
    }
  }
  if (C.num_tiles > 0 && !P->partitioned && P->mode == MODE_LDS) X.slabs_used += grid;
  P->launches_done = c + 1;
  return 0;
}

int exec_epilogue(pgpu_plan_s* P, hipStream_t stream, ExecCtx& X) {
  Scratch* sc = P->scratch;
  const int nslots = X.nslots;
  const int64_t words = X.words;
  KParams& kp = X.kp;
  const int nl = P->launches_done;
  if (nl == 0) PGPU_TIMING_RECORD(sc->ev[1], stream);
  if (!P->star.empty()) {
    // star-tree segments: K5 traversal then K6 residual scan + aggregation into the same group table
    X.mark("before star buffers");
    TRY(sc->starwork.ensure((size_t)P->star_work_bytes + P->star.size() * 8 + 16));
    int64_t* seg_total = reinterpret_cast<int64_t*>(sc->starwork.as<uint8_t>() + P->star_work_bytes);
    {
      const void* before = sc->starrec.p;
      TRY(sc->starrec.ensure(P->star.size() * sizeof(KStarSeg)));
      if (sc->starrec.p != before) sc->starrec_sent.clear();  // a new buffer holds nothing yet
    }
    std::vector<KStarSeg> recs = P->star;
    for (size_t i = 0; i < recs.size(); ++i) {
      uint8_t* base = sc->starwork.as<uint8_t>() + P->star_work_off[i];
      const int64_t nn = recs[i].num_nodes;
      recs[i].ranges = reinterpret_cast<int32_t*>(base);
      recs[i].prefix = reinterpret_cast<int64_t*>(base + ((2 * nn * 4 + 7) & ~int64_t(7)));
      recs[i].frontier = reinterpret_cast<int32_t*>(base + ((2 * nn * 4 + 7) & ~int64_t(7)) + (nn + 1) * 8);
      recs[i].out = recs[i].frontier + 6 * nn;
    }
    for (auto& f : P->star_match_fix)
      recs[std::get<0>(f)].match[std::get<1>(f)] = X.sets + std::get<2>(f);
    // The records (this scratch's work buffers, the plan's match sets) are the same for every execution of a cached
    // plan on this scratch: uploaded when they differ from the last upload.  A small host-to-device copy could block
    // the host for milliseconds behind other streams' work (C4 at 3 queries in flight: 5.4 ms in one execution).
    const size_t rbytes = recs.size() * sizeof(KStarSeg);
    X.mark("star buffers + records built");
    if (sc->starrec_sent.size() != rbytes || memcmp(sc->starrec_sent.data(), recs.data(), rbytes) != 0) {
      TRY(sc->starstage.ensure(rbytes));
      memcpy(sc->starstage.p, recs.data(), rbytes);
      HIP_TRY(hipMemcpyAsync(sc->starrec.p, sc->starstage.p, rbytes, hipMemcpyHostToDevice, stream));
      sc->starrec_sent.assign(reinterpret_cast<const uint8_t*>(recs.data()),
                              reinterpret_cast<const uint8_t*>(recs.data()) + rbytes);
    }
    X.mark("star records copy queued");
    if (launch_startree_traverse(sc->starrec.as<KStarSeg>(), (int)recs.size(), seg_total, kp.deadline, kp.stats,
                                 stream))
      return fail(PGPU_ERR_DEVICE, "star-tree traversal launch failed: %s", hipGetErrorString(hipGetLastError()));
    X.mark("K5 launched");
    KStarParams sp;
    memset(&sp, 0, sizeof sp);
    sp.num_wgs = P->star_chunks;
    sp.range_cache = P->star_range_cache;
    sp.num_keys = (int)P->key_cols.size();
    for (size_t j = 0; j < P->key_cols.size(); ++j) sp.key_stride[j] = P->key_stride[j];
    sp.key_bias = P->key_bias;
    sp.num_keys_total = P->num_keys;
    sp.num_slots = nslots;
    for (int sl = 0; sl < nslots; ++sl) {
      sp.slot_kind[sl] = P->slot_kind[sl];
      sp.slot_int[sl] = sl > 0 && P->slot_tcol[sl] >= 0 && is_int_type(P->table->types[P->slot_tcol[sl]]) ? 1 : 0;
    }
    sp.table = kp.table;
    sp.slab = P->mode == MODE_LDS ? kp.slab + X.slabs_used * words : nullptr;
    sp.hash_keys = kp.hash_keys;
    sp.stats = kp.stats;
    sp.deadline = kp.deadline;
    sp.cache_ints = P->star_cache_ints;
    for (int b = 0; b < P->star_batches; ++b) {  // kStarMaxSegs segments per launch, slabs back to back
      const int s0 = b * kStarMaxSegs;
      sp.segs = sc->starrec.as<KStarSeg>() + s0;
      sp.num_segs = (int)std::min<int64_t>(kStarMaxSegs, (int64_t)recs.size() - s0);
      sp.seg_total = seg_total + s0;
      if (P->mode == MODE_LDS) sp.slab = kp.slab + (X.slabs_used + (int64_t)b * P->star_chunks) * words;
      if (launch_startree_scan(sp, P->mode, P->star_lds_bytes, stream))
        return fail(PGPU_ERR_DEVICE, "star-tree scan launch failed: %s", hipGetErrorString(hipGetLastError()));
      X.mark("K6 launched");
    }
  }
  if (!P->generic.empty()) {
    // STATS_GENERIC segments: the leaves' match bitmaps, read back and replayed on the host at finalize
    std::vector<KMaskJob> jobs;
    for (const auto& g : P->generic)
      for (int64_t g0 = 0; g0 < ((int64_t)g.num_docs + 31) / 32; g0 += kBlock)
        jobs.push_back(KMaskJob{(int32_t)g.rec, (int32_t)g0, g.out_word});
    TRY(sc->mask_jobs.ensure(std::max<size_t>(jobs.size(), 1) * sizeof(KMaskJob)));
    TRY(sc->leaf_masks.ensure((size_t)std::max<int64_t>(P->generic_words, 1) * 4));
    TRY(sc->maskstage.ensure(std::max<size_t>(jobs.size() * sizeof(KMaskJob), (size_t)P->generic_words * 4) + 16));
    memcpy(sc->maskstage.p, jobs.data(), jobs.size() * sizeof(KMaskJob));
    HIP_TRY(hipMemcpyAsync(sc->mask_jobs.p, sc->maskstage.p, jobs.size() * sizeof(KMaskJob), hipMemcpyHostToDevice,
                           stream));
    KParams mp = kp;
    mp.segs = X.segrec;
    if (launch_leaf_masks(mp, sc->mask_jobs.as<KMaskJob>(), (int32_t)jobs.size(), sc->leaf_masks.as<uint32_t>(),
                          stream))
      return fail(PGPU_ERR_DEVICE, "leaf mask launch failed: %s", hipGetErrorString(hipGetLastError()));
    HIP_TRY(hipMemcpyAsync(sc->maskstage.p, sc->leaf_masks.p, (size_t)P->generic_words * 4, hipMemcpyDeviceToHost,
                           stream));
  }
  PGPU_TIMING_RECORD(sc->ev[2], stream);
  X.mark("event 2 recorded");
  if (P->mode == MODE_LDS) {
    // fold every slab written: the scan launches' (back to back) and the star-tree chunks' after them
    const int64_t all = X.slabs_used + (int64_t)P->star_batches * P->star_chunks;
    if (all == 0) {
      if (launch_table_init(X.table, P->slot_kind.data(), nslots, P->num_keys, nullptr, stream))
        return fail(PGPU_ERR_DEVICE, "table init launch failed");
    } else if (launch_epilogue(kp.slab, P->slot_kind.data(), nslots, P->num_keys, (int32_t)all, X.table, X.leap_segs,
                               P->seg_stride, X.leap_nsegs, kp.leap_maps, kp.stats, stream)) {
      return fail(PGPU_ERR_DEVICE, "reduce launch failed: %s", hipGetErrorString(hipGetLastError()));
    }
    X.leap_nsegs = 0;
  }
  if (P->mode == MODE_HASH && !P->part_hash && kp.pack_slot >= 0 &&
      launch_hash_unpack(X.table, kp.hash_keys, P->num_keys, kp.pack_slot, kp.pack_shift, stream))
    return fail(PGPU_ERR_DEVICE, "hash unpack launch failed: %s", hipGetErrorString(hipGetLastError()));
  if (X.leap_nsegs > 0 &&  // deferred but no fold ran (cannot happen for a plan with scan tiles; kept exact)
      launch_leap2_compose(X.leap_segs, P->seg_stride, X.leap_nsegs, kp.leap_maps, kp.stats, stream))
    return fail(PGPU_ERR_DEVICE, "filter statistics launch failed: %s", hipGetErrorString(hipGetLastError()));
  PGPU_TIMING_RECORD(sc->ev[3], stream);
  P->last_stream = stream;
  P->executed = true;
  if (trace_on()) {
    const double end = now_us();
    fprintf(stderr, "[pgpu] execute: %.1f us host\n", end - X.t_start);
    if (end - X.t_start > 1000.0) {
      double prev = X.t_start;
      for (const auto& m : X.marks) {
        fprintf(stderr, "[pgpu]   %s +%.1f us\n", m.first, m.second - prev);
        prev = m.second;
      }
      fprintf(stderr, "[pgpu]   (end) +%.1f us\n", end - prev);
    }
  }
  return 0;
}

int plan_execute_impl(pgpu_plan_s* P, hipStream_t stream, void* d_table) {
  const int nl = (int)P->chunks.size();
  ExecCtx X;
  TRY(exec_prologue(P, stream, d_table, std::max(nl, 1), X));
  for (int c = 0; c < nl; ++c) {
    TRY(exec_upload_chunk(P, stream, X, P->chunks[c]));
    TRY(exec_launch_chunk(P, stream, X, P->chunks[c], c));
  }
  return exec_epilogue(P, stream, X);
}

// Group-by dictIds of composite key k: (k / stride[j]) % card[j] (DictionaryBasedGroupKeyGenerator.java:276-323).
void decode_keys(const pgpu_plan_s* P, pgpu_result_s* R, int64_t row, uint64_t key) {
  for (int j = 0; j < R->num_keys; ++j)
    R->gid(j)[row] = (int32_t)((key / (uint64_t)P->key_stride[j]) % (uint64_t)P->key_card[j] + P->key_off[j]);
}

// key_begin / key_count: a shard [slots][key_count] of the dense table holding keys [key_begin, key_begin +
// key_count) (after a reduce-scatter across GPUs); the whole table is (0, num_keys).
int plan_finalize_impl(pgpu_plan_s* P, hipStream_t stream, const void* d_table, int64_t key_begin, int64_t key_count,
                       pgpu_result_s* R) {
  Scratch* sc = P->scratch;
  const double t_start = trace_on() ? now_us() : 0;
  if (!P->executed) return fail(PGPU_ERR_INVALID_ARGUMENT, "plan not executed");
  const uint64_t* table = reinterpret_cast<const uint64_t*>(d_table ? d_table : P->d_table_used);
  const int nslots = (int)P->slot_kind.size();
  const int nk = (int)P->key_cols.size();
  const int64_t G = key_count;
  int64_t n = 0;
  uint64_t matched = 0, star_scanned = 0;
  const int64_t words = (int64_t)nslots * G;
  double t_sync1 = 0;
  R->pool = P->table->result_pool;
  {
    // The buffers filled before the wait below: growing one frees the old one, and hipFree waits for the whole
    // device -- it would hold the wait (and a pgpu_plan_cancel or the query's deadline) until the scan is done.  When
    // one must grow, the plan's work is waited for first (cancel- and deadline-aware), then the buffers grow.
    bool grow = sc->counter.cap < 64 + (size_t)kMaxSlots * 16 || sc->readback.cap < 64 + (size_t)nslots * 16;
    if (!P->hash && words * 8 <= kHostCompactBytes) grow |= sc->readback.cap < (size_t)words * 8 + 64;
    else if (!P->hash) grow |= sc->cslots.cap < compact_scratch_bytes(G, nslots);
    else if (!P->part_hash_live)
      grow |= sc->ckeys.cap < (size_t)std::max<int64_t>(1, std::min<int64_t>(G, P->merged_records >= 0
                                                                                 ? P->merged_records
                                                                                 : std::max<int64_t>(P->total_docs, 1))) *
                                 8 * (1 + nslots);
    if (grow) {
      TRY(wait_plan(P, stream));
      TRY(sc->counter.ensure(64 + (size_t)kMaxSlots * 16));
    }
  }
  if (!P->hash && words * 8 <= kHostCompactBytes) {
    // small dense table: one copy (table + stats) and one sync, compacted on the host in key order
    TRY(sc->readback.ensure((size_t)words * 8 + 64));
    uint64_t* st = reinterpret_cast<uint64_t*>(sc->readback.p);
    if (reinterpret_cast<const uint8_t*>(P->d_stats) == reinterpret_cast<const uint8_t*>(table) + words * 8) {
      HIP_TRY(hipMemcpyAsync(st, table, (size_t)words * 8 + 48, hipMemcpyDeviceToHost, stream));  // table + stats
    } else {
      HIP_TRY(hipMemcpyAsync(st, table, (size_t)words * 8, hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipMemcpyAsync(st + words, P->d_stats, 48, hipMemcpyDeviceToHost, stream));
    }
    TRY(wait_plan(P, stream));
    t_sync1 = trace_on() ? now_us() : 0;
    if (st[words + 5]) return timeout_fail(P);
    matched = st[words];
    star_scanned = st[words + 1] + st[words + 2];
    P->star_docs_read = (int64_t)st[words + 3];
    for (int64_t k = 0; k < G; ++k) n += st[k] != 0;
    TRY(R->alloc(nk, nslots, n));
    int64_t j = 0;
    for (int64_t k = 0; k < G; ++k) {
      if (!st[k]) continue;
      decode_keys(P, R, j, (uint64_t)(key_begin + k));
      for (int s = 0; s < nslots; ++s) R->slot(s)[j] = st[(int64_t)s * G + k];
      ++j;
    }
  } else if (!P->hash) {
    // large dense table: ordered compaction on the device (count / scan, then a scatter in key order), copied back
    // into the pinned result buffer.  Two forms: the columnar dictIds + 8-byte words, or -- when it moves fewer
    // bytes, as for C5's 10M groups of 10M keys -- a presence bitmap over the keys plus each slot's words at the
    // narrowest width their range allows (decoded on the host on first access).
    const int64_t nch = compact_ordered_chunks(G);
    TRY(sc->counter.ensure(64 + (size_t)nslots * 16));
    TRY(sc->cslots.ensure(compact_scratch_bytes(G, nslots)));
    long long* d_minmax = reinterpret_cast<long long*>(sc->counter.as<uint8_t>() + 64);
    if (launch_compact_dense_count(table, nslots, G, sc->cslots.as<uint32_t>(), sc->counter.as<unsigned long long>(),
                                   d_minmax, stream))
      return fail(PGPU_ERR_DEVICE, "compact count launch failed: %s", hipGetErrorString(hipGetLastError()));
    TRY(sc->readback.ensure(64 + (size_t)nslots * 16));
    uint64_t* st = reinterpret_cast<uint64_t*>(sc->readback.p);
    HIP_TRY(hipMemcpyAsync(st, sc->counter.p, 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(st + 1, P->d_stats, 48, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(st + 8, d_minmax, (size_t)nslots * 16, hipMemcpyDeviceToHost, stream));
    TRY(wait_plan(P, stream));
    t_sync1 = trace_on() ? now_us() : 0;
    if (st[6]) return timeout_fail(P);
    n = (int64_t)std::min<uint64_t>(st[0], (uint64_t)G);
    matched = st[1];
    star_scanned = st[2] + st[3];
    P->star_docs_read = (int64_t)st[4];
    std::vector<int32_t> width(nslots, 8);
    int64_t narrow_bytes = 0;
    for (int s = 0; s < nslots; ++s) {
      const long long lo = (long long)st[8 + s], hi = (long long)st[8 + nslots + s];
      width[s] = n > 0 ? compact_slot_width(lo, hi, P->slot_kind[s]) : 8;
      narrow_bytes += n * width[s];
    }
    const int64_t bitmap_words = (G + 63) / 64;
    const bool compact = P->cfg.compact_results && n > 0 && bitmap_words * 8 + narrow_bytes < n * (4 * nk + 8 * nslots);
    if (compact) {
      const int64_t cap = n;
      TRY(sc->ckeys.ensure((size_t)bitmap_words * 8 + (size_t)nslots * cap * 8));
      uint8_t* dev = sc->ckeys.as<uint8_t>();
      if (launch_compact_dense_scatter(table, nslots, G, P->slot_kind.data(), sc->cslots.as<uint32_t>(), d_minmax,
                                       reinterpret_cast<uint64_t*>(dev), dev + bitmap_words * 8, cap, stream))
        return fail(PGPU_ERR_DEVICE, "compact scatter launch failed: %s", hipGetErrorString(hipGetLastError()));
      R->num_keys = nk;
      R->num_slots = nslots;
      R->n = n;
      R->ckey_base = key_begin;
      R->cbits = G;
      R->cstride = P->key_stride;
      R->ccard = P->key_card;
      R->coff = P->key_off;
      R->cwidth = width;
      R->cslot_off.assign(nslots, 0);
      size_t off = (size_t)bitmap_words * 8;
      for (int s = 0; s < nslots; ++s) {
        R->cslot_off[s] = off;
        off += ((size_t)n * width[s] + 7) & ~size_t(7);
      }
      if (R->pool) R->cbuf = R->pool->take();
      TRY(R->cbuf.ensure(off));
      uint8_t* h = reinterpret_cast<uint8_t*>(R->cbuf.p);
      HIP_TRY(hipMemcpyAsync(h, dev, (size_t)bitmap_words * 8, hipMemcpyDeviceToHost, stream));
      for (int s = 0; s < nslots; ++s)
        HIP_TRY(hipMemcpyAsync(h + R->cslot_off[s], dev + bitmap_words * 8 + (size_t)s * cap * 8, (size_t)n * width[s],
                               hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
      R->compact.store(true, std::memory_order_release);
    } else {
      const int64_t cap = std::max<int64_t>(2, (n + 1) & ~int64_t(1));
      TRY(sc->ckeys.ensure((size_t)cap * (4 * nk + 8 * nslots) + 8));
      if (launch_compact_ordered_scatter(table, nslots, G, key_begin, P->key_stride.data(), P->key_card.data(),
                                         P->key_off.data(), nk, sc->cslots.as<uint32_t>(), sc->ckeys.p, cap, stream))
        return fail(PGPU_ERR_DEVICE, "compact launch failed: %s", hipGetErrorString(hipGetLastError()));
      TRY(R->alloc(nk, nslots, n));
      if (n > 0) {
        const uint8_t* dev = sc->ckeys.as<uint8_t>();
        for (int j = 0; j < nk; ++j)
          HIP_TRY(hipMemcpyAsync(R->gid_raw(j), dev + (size_t)j * cap * 4, (size_t)n * 4, hipMemcpyDeviceToHost, stream));
        for (int s = 0; s < nslots; ++s)
          HIP_TRY(hipMemcpyAsync(R->slot_raw(s), dev + (size_t)nk * cap * 4 + (size_t)s * cap * 8, (size_t)n * 8,
                                 hipMemcpyDeviceToHost, stream));
      }
      HIP_TRY(hipStreamSynchronize(stream));
    }
  } else {
    // hash table: unordered compaction, then key order on the host
    const int64_t rec = 1 + nslots;  // entry-major compact record: key, then the slot words
    int64_t cap;
    const bool k8h = P->part_hash_live;
    if (k8h) {  // K8h wrote the compacted records and their count at execute
      cap = part_hash_out_cap(P);
    } else {
      cap = std::max<int64_t>(1, std::min<int64_t>(G, P->merged_records >= 0 ? P->merged_records
                                                                            : std::max<int64_t>(P->total_docs, 1)));
      TRY(sc->counter.ensure(64));
      TRY(sc->ckeys.ensure((size_t)cap * 8 * rec));
      HIP_TRY(hipMemsetAsync(sc->counter.p, 0, 8, stream));
      if (launch_compact(table, sc->hash_keys.as<unsigned long long>(), nslots, G, sc->counter.as<unsigned long long>(),
                         sc->ckeys.as<uint64_t>(), cap, stream))
        return fail(PGPU_ERR_DEVICE, "compact launch failed");
    }
    // each slot's range over the records, read back with their count (the compact form's widths, below)
    const bool want_compact = P->stage_end.empty() && P->cfg.compact_results;
    TRY(sc->counter.ensure(64 + (size_t)kMaxSlots * 16));  // (no regrowth: the first allocation is 4 KB)
    unsigned long long* d_mm = reinterpret_cast<unsigned long long*>(sc->counter.as<uint8_t>() + 64);
    if (want_compact &&
        (k8h ? launch_hash_minmax_parts(sc->part_mm.as<unsigned long long>(), P->num_parts, nslots, d_mm, stream)
             : launch_hash_minmax(sc->ckeys.as<uint64_t>(), sc->counter.as<unsigned long long>(), cap, nslots, d_mm,
                                  stream)))
      return fail(PGPU_ERR_DEVICE, "slot range launch failed: %s", hipGetErrorString(hipGetLastError()));
    TRY(sc->readback.ensure(64 + (size_t)nslots * 16));
    uint64_t* st = reinterpret_cast<uint64_t*>(sc->readback.p);
    HIP_TRY(hipMemcpyAsync(st, sc->counter.p, 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(st + 1, P->d_stats, 48, hipMemcpyDeviceToHost, stream));
    if (want_compact) HIP_TRY(hipMemcpyAsync(st + 8, d_mm, (size_t)nslots * 16, hipMemcpyDeviceToHost, stream));
    TRY(wait_plan(P, stream));
    t_sync1 = trace_on() ? now_us() : 0;
    if (st[6]) return timeout_fail(P);
    if (st[5])  // stats[4]: a probe found no free slot (hash_slot) -- the table was sized below the plan's groups
      return fail(PGPU_ERR_DEVICE, "group hash table of %lld slots overflowed (plan bound %lld groups)",
                  (long long)G, (long long)P->group_bound);
    if (k8h && st[0] > (uint64_t)cap) return part_hash_overflow(P, st[0]);
    n = (int64_t)std::min<uint64_t>(st[0], (uint64_t)cap);
    matched = st[1];
    star_scanned = st[2] + st[3];
    P->star_docs_read = (int64_t)st[4];
    if (P->groups_seen && P->merged_records < 0) P->groups_seen->store(n, std::memory_order_relaxed);
    if (n >= 4096 && P->stage_end.empty()) {
      // Decoded on the device in one streaming pass over the records, in their (hash / partition) order -- the
      // LONG_MAP holder's iteration order is fastutil's hash order (DictionaryBasedGroupKeyGenerator.java:693, :719)
      // and no consumer depends on group order -- held in compact form when that moves fewer bytes (C5-sized
      // results: 10M groups): composite keys at 4 or 8 bytes instead of the decoded dictIds, and each slot at the
      // narrowest width of its range (as the dense compact form); the host decodes it on first access
      // (result_expand).
      int key_bits = 1;
      {
        const long double space = (long double)P->key_stride[nk - 1] * (long double)P->key_card[nk - 1];
        while (key_bits < 64 && (long double)(INT64_C(1) << key_bits) < space) ++key_bits;
      }
      const int32_t key_width = key_bits <= 32 ? 4 : 8;
      std::vector<int32_t> width(nslots, 8);
      std::vector<int64_t> woff(nslots, 0);
      size_t cbytes = ((size_t)n * key_width + 7) & ~size_t(7);
      for (int s2 = 0; s2 < nslots; ++s2) {
        const long long lo = (long long)(st[8 + s2] ^ (1ull << 63)), hi = (long long)(st[8 + nslots + s2] ^ (1ull << 63));
        width[s2] = compact_slot_width(lo, hi, P->slot_kind[s2]);
        woff[s2] = (int64_t)cbytes;
        cbytes += ((size_t)n * width[s2] + 7) & ~size_t(7);
      }
      if (want_compact && cbytes < (size_t)n * (4 * nk + 8 * nslots)) {
        TRY(sc->hsort.ensure(cbytes + 256));
        uint8_t* out = sc->hsort.as<uint8_t>();
        if (launch_hash_compact(sc->ckeys.as<uint64_t>(), n, nslots, key_width, width.data(), woff.data(), out, stream))
          return fail(PGPU_ERR_DEVICE, "hash compact launch failed: %s", hipGetErrorString(hipGetLastError()));
        R->num_keys = nk;
        R->num_slots = nslots;
        R->n = n;
        R->ckey_width = key_width;
        R->cstride = P->key_stride;
        R->ccard = P->key_card;
        R->coff = P->key_off;
        R->cwidth = width;
        R->cslot_off.assign(woff.begin(), woff.end());
        if (R->pool) R->cbuf = R->pool->take();
        TRY(R->cbuf.ensure(cbytes));
        HIP_TRY(hipMemcpyAsync(R->cbuf.p, out, cbytes, hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        R->compact.store(true, std::memory_order_release);
        n = -1;  // held compact
      }
    }
    if (n >= 4096 && P->stage_end.empty()) {
      // decoded into the columnar result on the device: one copy back
      const size_t slot_off = pgpu_result_s::slot_offset(nk, n);
      const size_t out_bytes = slot_off + (size_t)nslots * n * 8;
      TRY(sc->hsort.ensure(out_bytes + 256));
      uint8_t* out = sc->hsort.as<uint8_t>();
      if (launch_hash_decode(sc->ckeys.as<uint64_t>(), n, nslots, nk, P->key_stride.data(), P->key_card.data(),
                             P->key_off.data(), out, slot_off, stream))
        return fail(PGPU_ERR_DEVICE, "hash decode launch failed: %s", hipGetErrorString(hipGetLastError()));
      TRY(R->alloc(nk, nslots, n));
      HIP_TRY(hipMemcpyAsync(R->buf.p, out, out_bytes, hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
      n = -1;  // decoded
    } else if (n > 0) {
      TRY(sc->readback.ensure((size_t)n * rec * 8));
      st = reinterpret_cast<uint64_t*>(sc->readback.p);
      HIP_TRY(hipMemcpyAsync(st, sc->ckeys.p, (size_t)n * rec * 8, hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
    }
    if (n < 0) {
      n = R->n;
    } else {
    std::vector<uint64_t> stages;  // ARRAY_MAP: the stage tables (slot -> that group's key), back to back
    std::vector<int64_t> stage_off;
    if (!P->stage_end.empty() && n > 0) {
      int64_t total = 0;
      for (int64_t c : P->stage_cap) { stage_off.push_back(total); total += c; }
      stages.resize((size_t)total);
      HIP_TRY(hipMemcpyAsync(stages.data(), sc->stage_keys.p, (size_t)total * 8, hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
    }
    std::vector<int64_t> order(n);
    for (int64_t i = 0; i < n; ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return st[a * rec] < st[b * rec]; });
    TRY(R->alloc(nk, nslots, n));
    for (int64_t r = 0; r < n; ++r) {
      const uint64_t* e = st + order[r] * rec;
      if (!P->stage_end.empty()) {  // last group first: its key's slot part names the previous group's key
        uint64_t cur = e[0];
        for (int g = (int)P->stage_space.size() - 1; g >= 0; --g) {
          const uint64_t local = cur % (uint64_t)P->stage_space[g], slot = cur / (uint64_t)P->stage_space[g];
          const int j0 = g == 0 ? 0 : P->stage_end[g - 1], j1 = g < (int)P->stage_end.size() ? P->stage_end[g] : nk;
          for (int j = j0; j < j1; ++j)
            R->gid(j)[r] = (int32_t)((local / (uint64_t)P->key_stride[j]) % (uint64_t)P->key_card[j]);
          if (g > 0) {
            if (slot >= (uint64_t)P->stage_cap[g - 1]) return fail(PGPU_ERR_DEVICE, "ARRAY_MAP stage slot out of range");
            cur = stages[(size_t)(stage_off[g - 1] + (int64_t)slot)];
          }
        }
      } else {
        decode_keys(P, R, r, e[0]);
      }
      for (int s = 0; s < nslots; ++s) R->slot(s)[r] = e[1 + s];
    }
    }
  }
  const double t_sync2 = trace_on() ? now_us() : 0;
  const int na = (int)P->agg_fn.size();
  R->num_aggs = na;
  R->agg_slot = P->agg_slot;
  R->slot_kind = P->slot_kind;
  R->key_cols = P->key_cols;
  R->key_dicts.assign(P->key_dicts.begin(), P->key_dicts.end());
  R->key_types.clear();
  for (int c : P->key_cols) R->key_types.push_back(P->table->types[c]);
  R->agg_fn = P->agg_fn;
  R->agg_col = P->agg_col;
  R->agg_conv.assign(na, RCONV_I64);
  for (int a = 0; a < na; ++a) {
    const int fn = P->agg_fn[a];
    if (fn == PGPU_AGG_COUNT) continue;  // CountAggregationFunction: exact count (held as double by Pinot)
    if (fn == PGPU_AGG_SUM || fn == PGPU_AGG_AVG)
      R->agg_conv[a] = P->slot_kind[P->agg_slot[a]] == SLOT_SUM_I64 ? RCONV_I64 : RCONV_F64;
    else
      R->agg_conv[a] = is_int_type(P->table->types[P->agg_col[a]]) ? RCONV_I64 : RCONV_KEY_F64;
  }
  int64_t generic_entries = 0;
  if (!P->generic.empty()) {  // the leaves' bitmaps were copied into maskstage by the (synchronised) stream
    const uint32_t* words = reinterpret_cast<const uint32_t*>(P->scratch->maskstage.p);
    std::vector<int64_t> part(P->generic.size(), 0);
    auto replay = [&](int i) {
      const auto& g = P->generic[i];
      const int64_t ngroups = ((int64_t)g.num_docs + 31) / 32;
      std::vector<const uint32_t*> masks(P->num_leaves);
      for (int k = 0; k < P->num_leaves; ++k) masks[P->leaf_perm[k]] = words + g.out_word + (int64_t)k * ngroups;
      part[i] = simulate_entries_scanned(g.tree, masks, g.num_docs);
    };
    if (P->generic.size() > 4) host_pool().run((int)P->generic.size(), replay);
    else for (size_t i = 0; i < P->generic.size(); ++i) replay((int)i);
    for (int64_t v : part) generic_entries += v;
  }
  // GroupByCombineOperator.mergeResults (:215-219): the merged map holds >= numGroupsLimit groups (PQL mode only)
  R->groups_limit_reached = P->pql_cap && nk > 0 && P->num_groups_limit > 0 && n >= P->num_groups_limit;
  R->stats[0] = (int64_t)matched;
  R->stats[1] = P->scanned_entries_model + (int64_t)star_scanned + generic_entries;
  R->stats[2] = ((int64_t)matched - P->post_exempt_docs) * P->num_projected;
  R->stats[3] = P->total_docs;
  R->stats[4] = (int64_t)P->segs.size();
  R->stats[5] = P->segments_matched_filter;
  if (trace_on())
    fprintf(stderr, "[pgpu] finalize: launch+sync1 %.1f us, copy+sync2 %.1f us, decode %.1f us (n=%lld)\n",
            t_sync1 - t_start, t_sync2 - t_sync1, now_us() - t_sync2, (long long)n);
  return 0;
}

}  // namespace

// Columnar form of a compact result: rows are the bitmap's set bits in key order; each block of 4096 bitmap words is
// decoded by one task of the host pool (a prefix of its popcounts gives its first row).
int pgpu::result_expand(pgpu_result_s* R) {
  std::lock_guard<std::mutex> g(R->expand_mu);
  if (!R->compact.load(std::memory_order_acquire)) return 0;
  const int nk = R->num_keys, ns = R->num_slots;
  const int64_t n = R->n;
  TRY(R->alloc(nk, ns, n));
  if (R->ckey_width) {  // composite keys (hash-mode results): decode each row's key
    const uint8_t* kb = reinterpret_cast<const uint8_t*>(R->cbuf.p);
    constexpr int64_t kRowsPerTask = 1 << 20;
    const int64_t ktasks = (n + kRowsPerTask - 1) / kRowsPerTask;
    auto keys = [&](int t) {
      const int64_t r0 = t * kRowsPerTask, r1 = std::min(n, r0 + kRowsPerTask);
      for (int64_t r = r0; r < r1; ++r) {
        const uint64_t key = R->ckey_width == 4 ? (uint64_t)reinterpret_cast<const uint32_t*>(kb)[r]
                                                : reinterpret_cast<const uint64_t*>(kb)[r];
        for (int j = 0; j < nk; ++j)
          R->gid_raw(j)[r] = (int32_t)((key / (uint64_t)R->cstride[j]) % (uint64_t)R->ccard[j] + R->coff[j]);
      }
    };
    if (ktasks > 1) host_pool().run((int)ktasks, keys);
    else if (ktasks == 1) keys(0);
  }
  const uint64_t* bm = reinterpret_cast<const uint64_t*>(R->cbuf.p);
  const int64_t words = R->ckey_width ? 0 : (R->cbits + 63) / 64;
  constexpr int64_t kBlockWords = 4096;
  const int64_t nb = (words + kBlockWords - 1) / kBlockWords;
  std::vector<int64_t> first(nb + 1, 0);
  auto count = [&](int b) {
    int64_t c = 0;
    for (int64_t w = b * kBlockWords; w < std::min(words, (b + 1) * kBlockWords); ++w) c += __builtin_popcountll(bm[w]);
    first[b + 1] = c;
  };
  auto decode = [&](int b) {
    int64_t row = first[b];
    std::vector<int32_t*> gid(nk);
    for (int j = 0; j < nk; ++j) gid[j] = R->gid_raw(j);
    for (int64_t w = b * kBlockWords; w < std::min(words, (b + 1) * kBlockWords); ++w) {
      for (uint64_t bits = bm[w]; bits; bits &= bits - 1, ++row) {
        if (row >= n) return;
        const uint64_t key = (uint64_t)(R->ckey_base + w * 64 + __builtin_ctzll(bits));
        for (int j = 0; j < nk; ++j)
          gid[j][row] = (int32_t)((key / (uint64_t)R->cstride[j]) % (uint64_t)R->ccard[j] + R->coff[j]);
      }
    }
  };
  if (nb > 1) host_pool().run((int)nb, count);
  else if (nb == 1) count(0);
  for (int64_t b = 0; b < nb; ++b) first[b + 1] += first[b];
  if (nb > 1) host_pool().run((int)nb, decode);
  else if (nb == 1) decode(0);
  // the words, sign-extended from their compact widths
  const uint8_t* base = reinterpret_cast<const uint8_t*>(R->cbuf.p);
  constexpr int64_t kRows = 1 << 20;
  const int64_t tasks = (n + kRows - 1) / kRows;
  auto widen = [&](int t) {
    const int64_t r0 = t * kRows, r1 = std::min(n, r0 + kRows);
    for (int s = 0; s < ns; ++s) {
      const uint8_t* src = base + R->cslot_off[s];
      uint64_t* dst = R->slot_raw(s);
      switch (R->cwidth[s]) {
        case 1: for (int64_t r = r0; r < r1; ++r) dst[r] = (uint64_t)(int64_t)reinterpret_cast<const int8_t*>(src)[r]; break;
        case 2: for (int64_t r = r0; r < r1; ++r) dst[r] = (uint64_t)(int64_t)reinterpret_cast<const int16_t*>(src)[r]; break;
        case 3:  // 24-bit little-endian, sign-extended
          for (int64_t r = r0; r < r1; ++r) {
            const uint32_t u = (uint32_t)src[3 * r] | (uint32_t)src[3 * r + 1] << 8 | (uint32_t)src[3 * r + 2] << 16;
            dst[r] = (uint64_t)(int64_t)((int32_t)(u << 8) >> 8);
          }
          break;
        case 4: for (int64_t r = r0; r < r1; ++r) dst[r] = (uint64_t)(int64_t)reinterpret_cast<const int32_t*>(src)[r]; break;
        default: memcpy(dst + r0, reinterpret_cast<const uint64_t*>(src) + r0, (size_t)(r1 - r0) * 8); break;
      }
    }
  };
  if (tasks > 1) host_pool().run((int)tasks, widen);
  else if (tasks == 1) widen(0);
  R->compact.store(false, std::memory_order_release);
  return 0;
}

namespace {

// ------------------------------------------------------------------------------------------ numGroupsLimit
// Pinot's group-key generators admit a segment's groups in first-seen docId order until numGroupsLimit and drop the
// docs of later groups (DictionaryBasedGroupKeyGenerator.java:97-161 holder choice, IntGroupIdMap :1101-1113 limit;
// DoubleGroupByResultHolder.java:89-93 ignores INVALID_ID); the PQL combine admits at most 2 x numGroupsLimit
// groups across segments (GroupByCombineOperator.java:61,78-80,138).  A plan where either can bind is split into
// parts: every segment whose key space (product of its local cardinalities) exceeds the limit becomes its own part
// with a hidden MIN($docId) slot -- each group's first matching doc, i.e. its group-id order -- and keeps the
// `limit` groups seen first; the other segments form one part.  When the 2x cap can bind (PQL mode, sum over
// segments of min(key space, limit) > 2 x limit) every segment is a part and groups are admitted segment by
// segment, each segment's groups in its holder's order (ArrayBasedHolder: key order; map holders: first-seen
// order) -- one of the orders Pinot's combine threads can produce, the one its single-threaded run produces.
int split_for_groups_limit(pgpu_table_s* t, const int64_t* handles, int32_t nsegs, const pgpu_query* q,
                           pgpu_plan_s* P, bool* composite) {
  *composite = false;
  if (!q || q->num_group_by <= 0 || q->num_groups_limit <= 0 || nsegs <= 0) return 0;
  const int64_t L = q->num_groups_limit;
  const int64_t threshold = std::min<int64_t>(10000, L);  // maxInitialResultHolderCapacity (ARRAY holder bound)
  std::vector<int64_t> prod(nsegs, 1);
  int64_t global_keys = 1;  // the table-global key space bounds the distinct groups of any segment set
  {
    std::lock_guard<std::mutex> g(t->mu);
    for (int k = 0; k < q->num_group_by; ++k) {
      const int c = q->group_by[k];
      if (c < 0 || c >= (int)t->names.size()) return 0;
      const int64_t card = std::max<int64_t>((int64_t)t->global[c]->size(), 1);
      global_keys = global_keys > INT64_MAX / card ? INT64_MAX : global_keys * card;
    }
    for (int i = 0; i < nsegs; ++i) {
      const int64_t h = handles[i];
      const Segment* sp = h > 0 && h < (int64_t)t->by_handle.size() ? t->by_handle[h].get() : nullptr;
      if (!sp) return 0;  // plan_create_impl reports it
      for (int k = 0; k < q->num_group_by; ++k) {
        const int c = q->group_by[k];
        if (c < 0 || c >= (int)t->names.size()) return 0;
        const int64_t card = std::max<int64_t>(sp->cols[c].card, 1);
        prod[i] = prod[i] > INT64_MAX / card ? INT64_MAX : prod[i] * card;
      }
    }
  }
  const bool pql = !(q->options & PGPU_OPT_SQL_GROUP_BY);
  bool any_sensitive = false;
  int64_t bound = 0;
  for (int i = 0; i < nsegs; ++i) {
    any_sensitive |= prod[i] > L;
    bound = std::min<int64_t>(INT64_MAX / 2, bound + std::min<int64_t>(prod[i], L));
  }
  const bool cap_may_bind = pql && std::min(bound, global_keys) > 2 * L;
  if (!any_sensitive && !cap_may_bind) return 0;
  std::vector<int32_t> rest;
  auto add_part = [&](const std::vector<int32_t>& idx, bool first_seen, bool truncate) -> int {
    pgpu_plan_s::Part part;
    part.plan = std::make_shared<pgpu_plan_s>();
    part.plan->first_doc_slot = first_seen;
    part.seg_index = idx;
    part.first_seen = first_seen;
    part.truncate = truncate;
    std::vector<int64_t> hs;
    for (int32_t i : idx) hs.push_back(handles[i]);
    TRY(plan_create_impl(t, hs.data(), (int32_t)hs.size(), q, part.plan.get()));
    P->parts.push_back(std::move(part));
    return 0;
  };
  for (int i = 0; i < nsegs; ++i) {
    if (cap_may_bind) TRY(add_part({i}, prod[i] > threshold, prod[i] > L));
    else if (prod[i] > L) TRY(add_part({i}, true, true));
    else rest.push_back(i);
  }
  if (!rest.empty()) TRY(add_part(rest, false, false));
  P->composite = true;
  *composite = true;
  P->table = t;
  P->num_groups_limit = L;
  P->pql_cap = pql;
  P->seg_scanned.assign(nsegs, 0);
  for (const auto& part : P->parts)
    for (size_t k = 0; k < part.seg_index.size() && k < part.plan->seg_scanned.size(); ++k)
      P->seg_scanned[part.seg_index[k]] = part.plan->seg_scanned[k];
  P->executed = false;
  return 0;
}

// Executes and finalizes the parts one after another (one part's group table in memory at a time) and merges their
// rows on the host: first-seen truncation per part, the 2x cap in admission order, AggregationFunction.merge.
int composite_finalize(pgpu_plan_s* P, hipStream_t stream, pgpu_result_s* R) {
  pgpu_table_s* t = P->table;
  const int64_t L = P->num_groups_limit;
  std::vector<std::unique_ptr<pgpu_result_s>> rs;
  for (auto& part : P->parts) {
    pgpu_plan_s* Q = part.plan.get();
    Q->scratch = acquire_scratch(t);
    auto Ri = std::make_unique<pgpu_result_s>();
    int rc = plan_execute_impl(Q, stream, nullptr);
    if (!rc) rc = plan_finalize_impl(Q, stream, nullptr, 0, Q->num_keys, Ri.get());
    if (rc && !Q->scratch->abandoned) hipStreamSynchronize(stream);
    release_scratch(t, Q->scratch);
    Q->scratch = nullptr;
    TRY(rc);
    rs.push_back(std::move(Ri));
  }
  const pgpu_plan_s* P0 = P->parts[0].plan.get();
  const int nk = (int)P0->key_cols.size();
  const int ns = (int)P0->slot_kind.size() - (P0->first_doc_slot ? 1 : 0);
  std::vector<int32_t> kind(P0->slot_kind.begin(), P0->slot_kind.begin() + ns);
  for (const auto& part : P->parts)
    for (int s = 0; s < ns; ++s)
      if (part.plan->slot_kind[s] == SLOT_SUM_F64) kind[s] = SLOT_SUM_F64;
  const int64_t cap = P->pql_cap ? std::min<int64_t>(2 * L, INT32_MAX) : INT64_MAX;
  // a group's key: the mixed-radix key, or for ARRAY_MAP plans (prefix key, rest key) -- never a slot number, which
  // is local to one part's tables
  using Key = std::array<int32_t, kMaxKeys>;  // the group-by dictIds (slot numbers are local to one part's tables)
  struct KeyHash {
    size_t operator()(const Key& k) const {
      uint64_t h = 0;
      for (int32_t v : k) h = (h ^ (uint32_t)v) * 0x9E3779B97F4A7C15ull;
      return (size_t)(h ^ (h >> 29));
    }
  };
  std::unordered_map<Key, int64_t, KeyHash> index;
  std::vector<Key> keys;
  std::vector<uint64_t> vals;
  int64_t counter = 0;
  // The parts were planned one after another: a pin in between may have grown a global dictionary, so their group
  // ids can index different snapshots.  Merge in the newest (largest: dictionaries only grow) and re-label the
  // other parts' ids through their values.
  std::vector<std::shared_ptr<const Dict>> kd(nk);
  for (const auto& part : P->parts)
    for (int j = 0; j < nk; ++j)
      if (!kd[j] || part.plan->key_dicts[j]->size() > kd[j]->size()) kd[j] = part.plan->key_dicts[j];
  for (size_t i = 0; i < P->parts.size(); ++i) {
    const auto& part = P->parts[i];
    pgpu_result_s* Ri = rs[i].get();
    const pgpu_plan_s* Q = part.plan.get();
    for (int j = 0; j < nk; ++j) {
      if (Q->key_dicts[j] == kd[j]) continue;
      const Dict& old = *Q->key_dicts[j];
      std::vector<int32_t> relabel(old.size());
      for (size_t x = 0; x < old.size(); ++x) relabel[x] = (int32_t)global_index_of(*kd[j], old, x);
      for (int64_t r = 0; r < Ri->n; ++r) Ri->gid(j)[r] = relabel[Ri->gid(j)[r]];
    }
    std::vector<int64_t> order(Ri->n);
    std::iota(order.begin(), order.end(), 0);
    if (part.first_seen) {
      const uint64_t* fd = Ri->slot(Ri->num_slots - 1);
      std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return (int64_t)fd[a] < (int64_t)fd[b]; });
      if (part.truncate && (int64_t)order.size() > L) order.resize(L);
    }
    for (int64_t r : order) {
      Key key{};
      for (int j = 0; j < nk; ++j) key[j] = Ri->gid(j)[r];
      auto it = index.find(key);
      if (it == index.end()) {
        if (counter++ >= cap) continue;  // _numGroups.getAndIncrement() < _interSegmentNumGroupsLimit
        index.emplace(key, (int64_t)keys.size());
        keys.push_back(key);
        for (int s = 0; s < ns; ++s) {
          uint64_t w = Ri->slot(s)[r];
          if (kind[s] == SLOT_SUM_F64 && Q->slot_kind[s] == SLOT_SUM_I64) {
            const double d = (double)(int64_t)w;
            memcpy(&w, &d, 8);
          }
          vals.push_back(w);
        }
        continue;
      }
      uint64_t* dst = vals.data() + it->second * ns;
      for (int s = 0; s < ns; ++s) {
        const uint64_t w = Ri->slot(s)[r];
        switch (kind[s]) {
          case SLOT_COUNT: case SLOT_SUM_I64: dst[s] += w; break;
          case SLOT_SUM_F64: {
            double a, b;
            memcpy(&a, &dst[s], 8);
            if (Q->slot_kind[s] == SLOT_SUM_I64) b = (double)(int64_t)w;
            else memcpy(&b, &w, 8);
            a += b;
            memcpy(&dst[s], &a, 8);
            break;
          }
          case SLOT_MIN_KEY: if ((int64_t)w < (int64_t)dst[s]) dst[s] = w; break;
          default: if ((int64_t)w > (int64_t)dst[s]) dst[s] = w; break;
        }
      }
    }
  }
  std::vector<int64_t> rows(keys.size());
  std::iota(rows.begin(), rows.end(), 0);
  // ascending mixed-radix key order: the last group-by column is the most significant
  std::sort(rows.begin(), rows.end(), [&](int64_t a, int64_t b) {
    for (int j = nk - 1; j >= 0; --j)
      if (keys[a][j] != keys[b][j]) return keys[a][j] < keys[b][j];
    return false;
  });
  const int64_t n = (int64_t)rows.size();
  R->pool = t->result_pool;
  TRY(R->alloc(nk, ns, n));
  for (int64_t r = 0; r < n; ++r) {
    const Key& k = keys[rows[r]];
    for (int j = 0; j < nk; ++j) R->gid(j)[r] = k[j];
    for (int s = 0; s < ns; ++s) R->slot(s)[r] = vals[rows[r] * ns + s];
  }
  const pgpu_result_s* R0 = rs[0].get();
  R->num_aggs = R0->num_aggs;
  R->agg_slot = R0->agg_slot;
  R->slot_kind = kind;
  R->key_cols = R0->key_cols;
  R->key_dicts.assign(kd.begin(), kd.end());
  R->key_types = R0->key_types;
  R->agg_fn = R0->agg_fn;
  R->agg_col = R0->agg_col;
  R->agg_conv = R0->agg_conv;
  for (int a = 0; a < R->num_aggs; ++a)
    if ((R->agg_fn[a] == PGPU_AGG_SUM || R->agg_fn[a] == PGPU_AGG_AVG) && kind[R->agg_slot[a]] == SLOT_SUM_F64)
      R->agg_conv[a] = RCONV_F64;
  for (const auto& Ri : rs)
    for (int k = 0; k < 6; ++k) R->stats[k] += Ri->stats[k];
  R->groups_limit_reached = P->pql_cap && n >= L;
  return 0;
}

// ------------------------------------------------------------------------------------------ plan cache
constexpr size_t kPlanCacheEntries = 16;

bool plan_cache_enabled(const pgpu_table_s* t, const pgpu_query* q) {
  return table_config(t).plan_cache && q && !(q->options & PGPU_OPT_NO_PLAN_CACHE);
}

// The bytes that determine a compiled plan: table version, segment handles, and every field of the query
// (predicate literals included).
std::string plan_cache_key(pgpu_table_s* t, const int64_t* handles, int32_t nsegs, const pgpu_query* q) {
  std::string k;
  auto put = [&](const void* p, size_t n) { k.append(reinterpret_cast<const char*>(p), n); };
  const uint64_t v = t->version.load();
  put(&v, 8);
  put(&nsegs, 4);
  if (nsegs > 0) put(handles, sizeof(int64_t) * (size_t)nsegs);
  put(&q->num_predicates, 4);
  for (int i = 0; i < q->num_predicates; ++i) {
    const pgpu_predicate& pr = q->predicates[i];
    const int32_t f[5] = {pr.type, pr.column, pr.num_values, pr.lower_inclusive, pr.upper_inclusive};
    put(f, sizeof f);
    for (int j = 0; j < pr.num_values; ++j) {
      const char* sv = pr.values && pr.values[j] ? pr.values[j] : "";
      const uint32_t n = (uint32_t)strlen(sv);
      put(&n, 4);
      put(sv, n);
    }
  }
  put(&q->num_filter_ops, 4);
  if (q->num_filter_ops > 0) put(q->filter, sizeof(pgpu_filter_op) * (size_t)q->num_filter_ops);
  put(&q->num_group_by, 4);
  if (q->num_group_by > 0) put(q->group_by, sizeof(int32_t) * (size_t)q->num_group_by);
  put(&q->num_aggs, 4);
  if (q->num_aggs > 0) put(q->aggs, sizeof(pgpu_agg) * (size_t)q->num_aggs);
  put(&q->num_groups_limit, 4);
  put(&q->options, 4);
  return k;
}

// On a hit, *P becomes a copy of the cached image (not executed, no scratch).
bool plan_cache_get(pgpu_table_s* t, const std::string& key, pgpu_plan_s* P) {
  std::lock_guard<std::mutex> g(t->cache_mu);
  for (auto it = t->plan_cache.begin(); it != t->plan_cache.end(); ++it) {
    if (it->first != key) continue;
    pgpu_plan_s& src = *it->second;
    // Once its device image is built, a hit needs none of the host records: copy the plan without them (the
    // records of a 1000-segment plan are ~250 KB -- most of a hit's host time).  cache_mu is held: no other
    // thread reads the cached image meanwhile.
    const bool lean = src.image && src.image->uploaded.load() && !check_launch_on();
    std::vector<uint8_t> segrec;
    std::vector<uint32_t> set_words;
    std::vector<std::pair<int64_t, int64_t>> set_fix;
    std::vector<KeyLut> key_lut;
    if (lean) {
      segrec.swap(src.segrec);
      set_words.swap(src.set_words);
      set_fix.swap(src.set_fix);
      key_lut.swap(src.key_lut);
    }
    *P = src;
    if (lean) {
      src.segrec.swap(segrec);
      src.set_words.swap(set_words);
      src.set_fix.swap(set_fix);
      src.key_lut.swap(key_lut);
    }
    t->plan_cache.splice(t->plan_cache.begin(), t->plan_cache, it);
    P->scratch = nullptr;
    P->executed = false;
    P->launches_done = 0;
    P->d_table_used = nullptr;
    P->last_stream = nullptr;
    P->star_docs_read = 0;
    P->shard = nullptr;
    P->cancel = 0;
    // a hash table sized by the groups the last execution of this plan found (deterministic for a cached plan:
    // same query over the same pinned segments)
    if (P->hash && P->groups_seen && P->stage_end.empty() && P->merged_records < 0) {
      const int64_t g = P->groups_seen->load(std::memory_order_relaxed);
      if (g >= 0) P->num_keys = hash_capacity(std::min<int64_t>(g, P->group_bound));
      if (g >= 0 && P->part_hash) hash_part_resize(P, std::max<int64_t>(g, 1));
    }
    return true;
  }
  return false;
}

// Every change of pinned state (pin, unpin, index attach, dictionary growth) bumps the table version, which is part
// of every cache key: the cached plans of earlier versions can never hit again, and they hold segment and LUT
// references, so they are dropped right away.
void plan_cache_clear(pgpu_table_s* t) {
  std::list<std::pair<std::string, std::shared_ptr<pgpu_plan_s>>> old;
  {
    std::lock_guard<std::mutex> g(t->cache_mu);
    old.swap(t->plan_cache);
  }
}

void plan_cache_put(pgpu_table_s* t, const std::string& key, pgpu_plan_s& P) {
  if (P.chunks.size() == 1 && P.docbit_words == 0 && !P.set_words_bound && !P.tile_bound)
    P.image = std::make_shared<DeviceImage>();  // built by the first execution, shared by every later hit
  auto img = std::make_shared<pgpu_plan_s>(P);
  img->scratch = nullptr;
  std::lock_guard<std::mutex> g(t->cache_mu);
  // The key was taken before planning.  Every change of pinned state bumps the version before it clears the cache:
  // a plan built across such a change carries the old version in its key and may reference state of that time
  // (an unpinned segment, an old dictionary snapshot), so it is not stored.
  uint64_t v;
  memcpy(&v, key.data(), 8);
  if (v != t->version.load()) return;
  t->plan_cache.emplace_front(key, std::move(img));
  while (t->plan_cache.size() > kPlanCacheEntries) t->plan_cache.pop_back();
}

}  // namespace

// PGPU_TRACE=serialize (diagnostics): every entry point of this file runs under one process-wide lock, so
// concurrent callers are serialised (isolates host-side races from device-side ones).
namespace {
std::recursive_mutex g_abi_mu;
bool abi_serialize() {
  static const bool on = diag("serialize");
  return on;
}
struct AbiGuard {
  bool on;
  AbiGuard() : on(abi_serialize()) { if (on) g_abi_mu.lock(); }
  ~AbiGuard() { if (on) g_abi_mu.unlock(); }
};
}  // namespace
#define PGPU_ABI_GUARD AbiGuard _abi_guard

// ================================================================================================ C ABI
extern "C" {

int pgpu_abi_version(void) { return PGPU_ABI_VERSION; }

namespace {
std::mutex g_init_mu;
int g_init_devices = 0;
}  // namespace

int pgpu_init(int n_gpus) try {
  PGPU_ABI_GUARD;
  install_crash_trace();
  int count = 0;
  HIP_TRY(hipGetDeviceCount(&count));
  if (n_gpus > count) return fail(PGPU_ERR_INVALID_ARGUMENT, "%d devices requested, %d visible", n_gpus, count);
  const int n = n_gpus > 0 ? n_gpus : count;
  std::lock_guard<std::mutex> g(g_init_mu);
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  for (int d = g_init_devices; d < n; ++d) {
    HIP_TRY(hipSetDevice(d));
    HIP_TRY(hipFree(nullptr));  // creates the device's context now
  }
  HIP_TRY(hipSetDevice(prev));
  g_init_devices = std::max(g_init_devices, n);
  host_pool();  // the planning workers start here, not inside the first query
  return n;
} PGPU_ABI_CATCH

int pgpu_shutdown(void) try {
  PGPU_ABI_GUARD;
  std::lock_guard<std::mutex> g(g_init_mu);
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  for (int d = 0; d < g_init_devices; ++d) {
    HIP_TRY(hipSetDevice(d));
    HIP_TRY(hipDeviceSynchronize());
  }
  HIP_TRY(hipSetDevice(prev));
  return 0;
} PGPU_ABI_CATCH

int pgpu_last_error(char* buf, size_t len) try {
  if (buf && len) {
    size_t n = std::min(len - 1, g_err.size());
    memcpy(buf, g_err.data(), n);
    buf[n] = 0;
  }
  return (int)g_err.size();
} PGPU_ABI_CATCH

int pgpu_device_count(int* count) try {
  PGPU_ABI_GUARD;
  if (!count) return fail(PGPU_ERR_INVALID_ARGUMENT, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) { *count = 0; return fail(PGPU_ERR_DEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e)); }
  *count = n;
  return 0;
} PGPU_ABI_CATCH

int pgpu_table_create(int device, int num_columns, const char* const* names, const int32_t* types, pgpu_table* out) try {
  PGPU_ABI_GUARD;
  install_crash_trace();
  if (!out || num_columns <= 0 || !types) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad table arguments");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(PGPU_ERR_DEVICE, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(PGPU_ERR_INVALID_ARGUMENT, "device %d out of range", device);
  for (int i = 0; i < num_columns; ++i)
    if (types[i] < PGPU_INT || types[i] > PGPU_STRING) return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: bad type", i);
  auto t = std::make_unique<pgpu_table_s>();
  t->device = device;
  for (int i = 0; i < num_columns; ++i) {
    t->names.push_back(names && names[i] ? names[i] : ("col" + std::to_string(i)));
    t->types.push_back(types[i]);
    auto d = std::make_shared<Dict>();
    d->type = types[i];
    d->id = g_dict_ids.fetch_add(1);
    t->global.push_back(std::move(d));
    t->global_version.push_back(0);
    t->gvalues.emplace_back();
  }
  DeviceGuard g(device);
  HIP_TRY(hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking));
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
    t->num_cus = cus;
  *out = t.release();
  return 0;
} PGPU_ABI_CATCH

int pgpu_config_default(pgpu_config* out) try {
  PGPU_ABI_GUARD;
  if (!out) return fail(PGPU_ERR_INVALID_ARGUMENT, "null config");
  *out = default_config();
  return 0;
} PGPU_ABI_CATCH

int pgpu_table_set_config(pgpu_table t, const pgpu_config* c) try {
  PGPU_ABI_GUARD;
  if (!t || !c || c->struct_size <= (int32_t)offsetof(pgpu_config, plan_cache))
    return fail(PGPU_ERR_INVALID_ARGUMENT, "bad config arguments");
  // fields past the caller's struct keep their defaults
  pgpu_config v = default_config();
  memcpy(&v, c, std::min<size_t>((size_t)c->struct_size, sizeof v));
  v.struct_size = (int32_t)sizeof v;
  if (v.hash_partition_bits < 0 || v.hash_partition_bits > 14 || v.hash_partition_lds_kb < 0 ||
      v.hash_partition_lds_kb > 128 || v.lds_table_kb < 1 || v.lds_table_kb > 160 || v.plan_chunk_segments < 1 ||
      v.stream_chunks < 1 || v.star_tree_workgroups < 0 || !(v.dense_selectivity >= 0.0))
    return fail(PGPU_ERR_INVALID_ARGUMENT, "config value out of range");
  {
    std::lock_guard<std::mutex> g(t->cfg_mu);
    t->cfg = v;
  }
  t->version.fetch_add(1);  // compiled plans were made with the previous settings
  plan_cache_clear(t);
  return 0;
} PGPU_ABI_CATCH

int pgpu_table_get_config(pgpu_table t, pgpu_config* out) try {
  PGPU_ABI_GUARD;
  if (!t || !out) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  *out = table_config(t);
  return 0;
} PGPU_ABI_CATCH

int pgpu_table_destroy(pgpu_table t) try {
  PGPU_ABI_GUARD;
  if (!t) return 0;
  DeviceGuard g(t->device);
  hipStreamSynchronize(t->stream);
  plan_cache_clear(t);
  t->segments.clear();  // freed here unless a live plan still holds a segment (destroy plans first)
  t->by_handle.clear();
  for (auto& s : t->scratch_pool) if (s) s->release();
  t->gen.pos.release(); t->gen.presence.release(); t->gen.code_to_pos.release(); t->gen.cdf.release();
  t->gen.pos_to_id.release();
  if (t->d_docid_fwd) hipFree(t->d_docid_fwd);
  if (t->d_docid_key) hipFree(t->d_docid_key);
  for (void* p : t->retired) hipFree(p);
  if (t->clock_stream) hipStreamDestroy(t->clock_stream);
  if (t->clock_pinned) hipHostFree(t->clock_pinned);
  hipStreamDestroy(t->stream);
  delete t;
  return 0;
} PGPU_ABI_CATCH

int pgpu_pin_segment(pgpu_table t, const pgpu_segment_desc* d, int64_t* handle) try {
  PGPU_ABI_GUARD;
  if (!t || !d || !handle) return fail(PGPU_ERR_INVALID_ARGUMENT, "null argument");
  if (d->num_columns != (int)t->names.size())
    return fail(PGPU_ERR_INVALID_ARGUMENT, "segment has %d columns, table has %zu", d->num_columns, t->names.size());
  if (d->num_docs < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "negative numDocs");
  DeviceGuard g(t->device);
  auto seg = std::make_unique<Segment>();
  seg->num_docs = d->num_docs;
  seg->cols.resize(d->num_columns);
  int64_t total_words = 0;
  std::vector<std::vector<uint32_t>> sorted_expansion(d->num_columns);
  std::vector<RawValues> raw_values(d->num_columns);
  bool any_raw = false;
  for (int c = 0; c < d->num_columns; ++c) {
    const pgpu_column_buffers& cb = d->columns[c];
    Column& col = seg->cols[c];
    col.card = cb.cardinality;
    col.entry_width = cb.entry_width;
    col.padding = cb.padding_byte;
    TRY(parse_dictionary(t->types[c], cb, &col.dict));
    if (cb.dict && cb.cardinality > 0) col.raw_dict.assign(cb.dict, cb.dict + (int64_t)cb.cardinality * cb.entry_width);
    if (cb.fwd_format == PGPU_FWD_FIXED_BIT) {
      col.bits = cb.bits_per_element;
      if (col.bits < 1 || col.bits > 31) return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: bitsPerElement %d", c, col.bits);
      const int64_t need = ((int64_t)d->num_docs * col.bits + 7) / 8;
      if (d->num_docs > 0 && (!cb.fwd || cb.fwd_len < need))
        return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: forward index has %lld bytes, needs %lld", c,
                    (long long)cb.fwd_len, (long long)need);
      col.fwd_bytes = need;
    } else if (cb.fwd_format == PGPU_FWD_SORTED_PAIRS) {
      // SortedIndexReaderImpl (start, end) pairs -> the fixed-bit layout the kernels read.
      if (cb.fwd_len < (int64_t)cb.cardinality * 8) return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: sorted index too small", c);
      col.bits = num_bits_per_value(cb.cardinality - 1);
      col.fwd_bytes = ((int64_t)d->num_docs * col.bits + 7) / 8;
      std::vector<uint32_t>& w = sorted_expansion[c];
      w.assign(padded_fwd_words(d->num_docs, col.bits), 0u);
      col.sorted = true;
      col.sorted_start.assign((size_t)cb.cardinality + 1, d->num_docs);
      int32_t prev_end = -1;
      for (int32_t id = 0; id < cb.cardinality; ++id) {
        const int32_t s = (int32_t)rd_be32(cb.fwd + (int64_t)id * 8), e = (int32_t)rd_be32(cb.fwd + (int64_t)id * 8 + 4);
        if (s < 0 || e >= d->num_docs || (e < s && e != s - 1)) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad sorted pair");
        if (s != prev_end + 1) return fail(PGPU_ERR_INVALID_ARGUMENT, "sorted pairs are not contiguous");
        prev_end = e;
        col.sorted_start[id] = s;
        for (int32_t doc = s; doc <= e; ++doc) {  // PinotDataBitSet.writeInt into BE words
          const uint64_t bit = (uint64_t)doc * col.bits;
          for (int b = 0; b < col.bits; ++b)
            if ((id >> (col.bits - 1 - b)) & 1) {
              const uint64_t pos = bit + b;
              w[pos >> 5] |= 1u << (31 - (pos & 31));
            }
        }
      }
      if (d->num_docs > 0 && prev_end != d->num_docs - 1)
        return fail(PGPU_ERR_INVALID_ARGUMENT, "sorted pairs do not cover every doc");
      for (auto& x : w) x = __builtin_bswap32(x);  // the device reads the forward index as big-endian bytes
    } else if (cb.fwd_format == PGPU_FWD_RAW_FIXED) {
      TRY(parse_raw_column(t->types[c], cb, d->num_docs, c, &col, &raw_values[c]));
      any_raw = true;
      continue;  // no per-segment forward-index words: the values live in d_key / d_val
    } else {
      return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: bad forward-index format", c);
    }
    col.fwd_words = padded_fwd_words(d->num_docs, col.bits);
    total_words += (col.fwd_words + 63) & ~int64_t(63);  // 256-byte aligned columns
  }
  HIP_TRY(hipMalloc(&seg->d_block, (size_t)std::max<int64_t>(total_words, 64) * 4));
  t->device_bytes += std::max<int64_t>(total_words, 64) * 4;
  int64_t off = 0;
  for (int c = 0; c < d->num_columns; ++c) {
    Column& col = seg->cols[c];
    if (col.raw) {
      const size_t n = (size_t)raw_padded_docs(d->num_docs);
      raw_values[c].key.resize(n, 0);
      raw_values[c].val.resize(n, 0.0);
      HIP_TRY(hipMalloc(&col.d_key, n * 8));
      HIP_TRY(hipMalloc(&col.d_val, n * 8));
      t->device_bytes += 16 * (int64_t)n;
      HIP_TRY(hipMemcpyAsync(col.d_key, raw_values[c].key.data(), n * 8, hipMemcpyHostToDevice, t->stream));
      HIP_TRY(hipMemcpyAsync(col.d_val, raw_values[c].val.data(), n * 8, hipMemcpyHostToDevice, t->stream));
      continue;
    }
    col.d_fwd = reinterpret_cast<uint32_t*>(seg->d_block) + off;
    const pgpu_column_buffers& cb = d->columns[c];
    HIP_TRY(hipMemsetAsync(col.d_fwd, 0, (size_t)col.fwd_words * 4, t->stream));
    if (cb.fwd_format == PGPU_FWD_SORTED_PAIRS) {
      HIP_TRY(hipMemcpyAsync(col.d_fwd, sorted_expansion[c].data(), (size_t)col.fwd_words * 4, hipMemcpyHostToDevice,
                             t->stream));
    } else if (col.fwd_bytes > 0) {
      HIP_TRY(hipMemcpyAsync(col.d_fwd, cb.fwd, (size_t)col.fwd_bytes, hipMemcpyHostToDevice, t->stream));
    }
    off += (col.fwd_words + 63) & ~int64_t(63);
  }
  // dictIds within the dictionary (fwd_max_kernel): only columns whose bit width can hold values >= cardinality
  std::vector<int> check;
  for (int c = 0; c < d->num_columns; ++c) {
    const Column& col = seg->cols[c];
    if (!col.raw && !col.sorted && d->num_docs > 0 && (int64_t)col.card < (INT64_C(1) << col.bits)) check.push_back(c);
  }
  DevBuf dmax;
  struct Release { DevBuf& b; ~Release() { b.release(); } } release_dmax{dmax};
  std::vector<uint32_t> hmax(check.size(), 0);
  if (!check.empty()) {
    TRY(dmax.ensure(check.size() * 4));
    HIP_TRY(hipMemsetAsync(dmax.p, 0, check.size() * 4, t->stream));
    for (size_t i = 0; i < check.size(); ++i)
      if (launch_fwd_max(seg->cols[check[i]].d_fwd, d->num_docs, seg->cols[check[i]].bits,
                         dmax.as<unsigned int>() + i, t->stream))
        return fail(PGPU_ERR_DEVICE, "forward-index check launch failed: %s", hipGetErrorString(hipGetLastError()));
    HIP_TRY(hipMemcpyAsync(hmax.data(), dmax.p, check.size() * 4, hipMemcpyDeviceToHost, t->stream));
  }
  HIP_TRY(hipStreamSynchronize(t->stream));
  for (size_t i = 0; i < check.size(); ++i)
    if ((int64_t)hmax[i] >= seg->cols[check[i]].card) {
      account_unpin(t, seg.get());
      return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: forward index holds dictId %u, cardinality is %d", check[i],
                  hmax[i], seg->cols[check[i]].card);
    }
  std::lock_guard<std::mutex> lk(t->mu);
  if (any_raw) TRY(ensure_docid(t, d->num_docs, t->stream));
  *handle = register_segment(t, std::move(seg));
  return 0;
} PGPU_ABI_CATCH

int pgpu_unpin_segment(pgpu_table t, int64_t h) try {
  PGPU_ABI_GUARD;
  if (t) t->version++;
  if (!t) return fail(PGPU_ERR_INVALID_ARGUMENT, "null table");
  DeviceGuard g(t->device);
  std::shared_ptr<Segment> seg;  // released after the table mutex (the free may wait for the device)
  {
    std::lock_guard<std::mutex> lk(t->mu);
    auto it = t->segments.find(h);
    if (it == t->segments.end()) return fail(PGPU_ERR_NOT_FOUND, "unknown segment handle %lld", (long long)h);
    seg = std::move(it->second);
    account_unpin(t, seg.get());
    t->by_handle[h].reset();
    t->segments.erase(it);
  }
  plan_cache_clear(t);  // cached plans reference the segment set of their time
  hipStreamSynchronize(t->stream);  // work queued on the table's own stream (pins, reads) is done with it
  return 0;
} PGPU_ABI_CATCH

namespace {
// Portable RoaringBitmap deserialisation (RoaringBitmap 0.9.x RoaringArray.deserialize, little-endian): cookie
// 12346 (no run containers; u32 size follows) or 12347 | (size - 1) << 16 (with a run-container bitmap); per
// container (u16 key, u16 card - 1); offsets (u32, skipped) unless a run-cookie bitmap has < 4 containers; then
// ARRAY (card <= 4096: u16 values), BITMAP (1024 u64) or RUN (u16 count, (u16 start, u16 length - 1) pairs).
// Appends device-layout payload words and container entries; returns false on malformed input.
bool parse_roaring(const uint8_t* b, int64_t n, int32_t num_docs, std::vector<uint32_t>& words,
                   std::vector<InvIndex::Cont>& conts, int64_t* docs) {
  auto u16 = [&](int64_t o) { return (uint32_t)b[o] | ((uint32_t)b[o + 1] << 8); };
  auto u32 = [&](int64_t o) { return u16(o) | (u16(o + 2) << 16); };
  if (n < 4) return false;
  const uint32_t cookie = u32(0);
  int64_t pos, size;
  const uint8_t* runbits = nullptr;
  bool offsets;
  if ((cookie & 0xFFFF) == 12347) {
    size = (cookie >> 16) + 1;
    runbits = b + 4;
    pos = 4 + (size + 7) / 8;
    offsets = size >= 4;
  } else if (cookie == 12346) {
    if (n < 8) return false;
    size = u32(4);
    pos = 8;
    offsets = true;
  } else {
    return false;
  }
  if (size < 0 || size > 65536 || pos + size * 4 > n) return false;
  const int64_t desc = pos;
  pos += size * 4 + (offsets ? size * 4 : 0);
  *docs = 0;
  int32_t prev_key = -1;
  std::vector<uint32_t> vals;
  for (int64_t i = 0; i < size; ++i) {
    const int32_t key = (int32_t)u16(desc + 4 * i);
    const int32_t card = (int32_t)u16(desc + 4 * i + 2) + 1;
    if (key <= prev_key || ((int64_t)key << 16) >= num_docs) return false;
    prev_key = key;
    const bool run = runbits && ((runbits[i >> 3] >> (i & 7)) & 1);
    vals.clear();
    std::vector<uint32_t> bm;
    if (run) {
      if (pos + 2 > n) return false;
      const int64_t nruns = u16(pos);
      pos += 2;
      if (pos + nruns * 4 > n) return false;
      for (int64_t r = 0; r < nruns; ++r) {
        const uint32_t start = u16(pos + 4 * r), len = u16(pos + 4 * r + 2);
        if (start + len > 65535) return false;
        // the runs may not hold more values than the declared cardinality (bounds the expansion)
        if ((int64_t)vals.size() + len + 1 > card) return false;
        for (uint32_t v = start; v <= start + len; ++v) vals.push_back(v);
      }
      pos += nruns * 4;
    } else if (card <= 4096) {
      if (pos + (int64_t)card * 2 > n) return false;
      for (int32_t k = 0; k < card; ++k) vals.push_back(u16(pos + 2 * k));
      pos += (int64_t)card * 2;
    } else {
      if (pos + 8192 > n) return false;
      bm.resize(kContainerWords);
      for (int w = 0; w < kContainerWords; ++w) bm[w] = u32(pos + 4 * w);
      pos += 8192;
    }
    int64_t c = 0;
    if (bm.empty()) {
      if ((int64_t)vals.size() != card) return false;
      if (vals.size() > 4096) {  // long runs: bitmap form
        bm.assign(kContainerWords, 0);
        for (uint32_t v : vals) bm[v >> 5] |= 1u << (v & 31);
      }
    }
    if (!bm.empty()) {
      int32_t top = -1;
      for (int w = 0; w < kContainerWords; ++w)
        if (bm[w]) { c += __builtin_popcount(bm[w]); top = w * 32 + 31 - __builtin_clz(bm[w]); }
      if (((int64_t)key << 16) + top >= num_docs) return false;
      if (c != card) return false;  // overlapping runs / a bitmap whose popcount is not its cardinality
      conts.push_back({(int64_t)words.size(), CONT_BITMAP, (int32_t)c, key});
      words.insert(words.end(), bm.begin(), bm.end());
    } else {
      for (size_t k = 1; k < vals.size(); ++k)
        if (vals[k] <= vals[k - 1]) return false;
      if (!vals.empty() && ((int64_t)key << 16) + vals.back() >= num_docs) return false;
      c = (int64_t)vals.size();
      conts.push_back({(int64_t)words.size(), CONT_ARRAY, (int32_t)c, key});
      for (size_t k = 0; k < vals.size(); k += 2)
        words.push_back(vals[k] | (k + 1 < vals.size() ? vals[k + 1] << 16 : 0u));
    }
    *docs += c;
  }
  return pos <= n;
}

// A `<column>.bitmap.inv` file (BitmapInvertedIndexReader.java:40-70): (card + 1) big-endian int32 bitmap offsets,
// then one portable Roaring bitmap per dictId, parsed into `inv`'s per-dictId container lists and the device
// payload `words`.  Pure host code (pgpu_attach_inverted_index, pgpu_inverted_index_check).
int parse_inverted_index(const uint8_t* b, int64_t num_bytes, int64_t card, int32_t num_docs, int column,
                         InvIndex* inv, std::vector<uint32_t>& words) {
  if (card < 0 || num_docs < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad cardinality / document count");
  const int64_t hdr = (card + 1) * 4;
  if (!b || num_bytes < hdr) return fail(PGPU_ERR_INVALID_ARGUMENT, "inverted index shorter than its offset header");
  auto be32 = [&](int64_t o) {
    return (int64_t)(int32_t)(((uint32_t)b[o] << 24) | ((uint32_t)b[o + 1] << 16) | ((uint32_t)b[o + 2] << 8) | b[o + 3]);
  };
  inv->ids.assign(card, InvIndex::Entry{0, 0, 0});
  const int64_t first = be32(0);
  for (int64_t id = 0; id < card; ++id) {
    const int64_t off = be32(id * 4) - first, end = be32((id + 1) * 4) - first;
    inv->ids[id].begin = (int32_t)inv->conts.size();
    if (off < 0 || end < off || hdr + end > num_bytes)
      return fail(PGPU_ERR_INVALID_ARGUMENT, "bitmap %lld of column %d overruns the index", (long long)id, column);
    if (!parse_roaring(b + hdr + off, end - off, num_docs, words, inv->conts, &inv->ids[id].docs))
      return fail(PGPU_ERR_INVALID_ARGUMENT, "malformed Roaring bitmap for dictId %lld of column %d", (long long)id,
                  column);
  }
  for (int64_t id = 0; id < card; ++id)
    inv->ids[id].count = (int32_t)((id + 1 < card ? inv->ids[id + 1].begin : (int32_t)inv->conts.size()) -
                                   inv->ids[id].begin);
  return 0;
}
}  // namespace

}  // extern "C"
bool pgpu::roaring_cardinality(const uint8_t* b, int64_t n, int32_t num_docs, int64_t* docs) {
  std::vector<uint32_t> words;
  std::vector<InvIndex::Cont> conts;
  return parse_roaring(b, n, num_docs, words, conts, docs);
}
extern "C" {

namespace {
void put_le16(std::vector<uint8_t>& o, uint32_t v) { o.push_back((uint8_t)v); o.push_back((uint8_t)(v >> 8)); }
void put_le32(std::vector<uint8_t>& o, uint32_t v) { put_le16(o, v & 0xFFFF); put_le16(o, v >> 16); }

// RoaringBitmap.serialize of a sorted docId list without run containers (cookie 12346).
void serialize_roaring_plain(const int32_t* docs, int64_t n, std::vector<uint8_t>& o) {
  std::vector<std::pair<int64_t, int64_t>> conts;  // [begin, end) per key
  for (int64_t i = 0; i < n;) {
    int64_t j = i;
    while (j < n && (docs[j] >> 16) == (docs[i] >> 16)) ++j;
    conts.emplace_back(i, j);
    i = j;
  }
  const size_t base = o.size();
  put_le32(o, 12346);
  put_le32(o, (uint32_t)conts.size());
  for (auto& c : conts) {
    put_le16(o, (uint32_t)(docs[c.first] >> 16));
    put_le16(o, (uint32_t)(c.second - c.first - 1));
  }
  uint32_t off = (uint32_t)(o.size() - base + 4 * conts.size());
  for (auto& c : conts) {
    put_le32(o, off);
    const int64_t card = c.second - c.first;
    off += card <= 4096 ? (uint32_t)(2 * card) : 8192u;
  }
  for (auto& c : conts) {
    const int64_t card = c.second - c.first;
    if (card <= 4096) {
      for (int64_t k = c.first; k < c.second; ++k) put_le16(o, (uint32_t)(docs[k] & 0xFFFF));
    } else {
      std::vector<uint32_t> bm(kContainerWords, 0);
      for (int64_t k = c.first; k < c.second; ++k) bm[(docs[k] & 0xFFFF) >> 5] |= 1u << (docs[k] & 31);
      for (uint32_t w : bm) put_le32(o, w);
    }
  }
}
}  // namespace

// Host-side inverted-index creator (OffHeapBitmapInvertedIndexCreator + BitmapInvertedIndexWriter,
// seglocal/segment/creator/impl/inv/BitmapInvertedIndexWriter.java:60-78): dictIds of the MSB-first fixed-bit
// forward index -> per dictId the sorted docIds -> (card + 1) BE offsets + serialised bitmaps.
int pgpu_build_inverted_index(const void* fwd, int64_t fwd_len, int32_t bits, int32_t num_docs, int32_t cardinality,
                              void* out, int64_t out_cap, int64_t* out_len) try {
  PGPU_ABI_GUARD;
  if (!fwd || !out_len || bits < 1 || bits > 31 || num_docs < 0 || cardinality < 1 ||
      fwd_len < ((int64_t)num_docs * bits + 7) / 8)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "bad inverted-index build arguments");
  const uint8_t* b = reinterpret_cast<const uint8_t*>(fwd);
  std::vector<int32_t> ids(num_docs);
  for (int64_t d = 0; d < num_docs; ++d) {
    const int64_t bit = d * bits;
    uint64_t w = 0;
    for (int k = 0; k < 5; ++k) {
      const int64_t byte = (bit >> 3) + k;
      w = (w << 8) | (byte < fwd_len ? b[byte] : 0);
    }
    ids[d] = (int32_t)((w >> (40 - (bit & 7) - bits)) & ((1u << bits) - 1u));
    if (ids[d] >= cardinality) return fail(PGPU_ERR_INVALID_ARGUMENT, "dictId %d >= cardinality", ids[d]);
  }
  std::vector<int64_t> start(cardinality + 1, 0);
  for (int32_t id : ids) start[id + 1]++;
  for (int32_t i = 0; i < cardinality; ++i) start[i + 1] += start[i];
  std::vector<int32_t> docs(num_docs);
  {
    std::vector<int64_t> fill(start.begin(), start.end() - 1);
    for (int32_t d = 0; d < num_docs; ++d) docs[fill[ids[d]]++] = d;
  }
  std::vector<uint8_t> body;
  std::vector<uint32_t> offs(cardinality + 1);
  const uint32_t hdr = 4u * (uint32_t)(cardinality + 1);
  for (int32_t i = 0; i < cardinality; ++i) {
    offs[i] = hdr + (uint32_t)body.size();
    serialize_roaring_plain(docs.data() + start[i], start[i + 1] - start[i], body);
  }
  offs[cardinality] = hdr + (uint32_t)body.size();
  *out_len = (int64_t)hdr + (int64_t)body.size();
  if (!out) return 0;
  if (out_cap < *out_len) return fail(PGPU_ERR_INVALID_ARGUMENT, "output buffer too small");
  uint8_t* o = reinterpret_cast<uint8_t*>(out);
  for (int32_t i = 0; i <= cardinality; ++i) {
    o[4 * i] = (uint8_t)(offs[i] >> 24); o[4 * i + 1] = (uint8_t)(offs[i] >> 16);
    o[4 * i + 2] = (uint8_t)(offs[i] >> 8); o[4 * i + 3] = (uint8_t)offs[i];
  }
  memcpy(o + hdr, body.data(), body.size());
  return 0;
} PGPU_ABI_CATCH

int pgpu_raw_forward_index_values(const void* fwd, int64_t fwd_len, int32_t data_type, int32_t num_docs,
                                  int64_t* out_i64, double* out_f64) try {
  PGPU_ABI_GUARD;
  if (!fwd || num_docs < 0 || data_type < PGPU_INT || data_type > PGPU_STRING)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  RawValues v;
  TRY(decode_raw_forward_index(data_type, reinterpret_cast<const uint8_t*>(fwd), fwd_len, num_docs, 0, &v));
  for (int32_t i = 0; i < num_docs; ++i) {
    if (out_i64) out_i64[i] = is_int_type(data_type) ? v.key[i] : 0;
    if (out_f64) out_f64[i] = v.val[i];
  }
  return 0;
} PGPU_ABI_CATCH

int pgpu_inverted_index_check(const void* bytes, int64_t num_bytes, int32_t cardinality, int32_t num_docs,
                              int64_t* total_docs) try {
  PGPU_ABI_GUARD;
  if (!bytes && num_bytes) return fail(PGPU_ERR_INVALID_ARGUMENT, "null argument");
  InvIndex inv;
  std::vector<uint32_t> words;
  TRY(parse_inverted_index(reinterpret_cast<const uint8_t*>(bytes), num_bytes, cardinality, num_docs, -1, &inv,
                           words));
  if (total_docs) {
    *total_docs = 0;
    for (const auto& e : inv.ids) *total_docs += e.docs;
  }
  return 0;
} PGPU_ABI_CATCH

int pgpu_attach_inverted_index(pgpu_table t, int64_t h, int32_t column, const void* bytes, int64_t num_bytes) try {
  PGPU_ABI_GUARD;
  if (t) t->version++;
  if (t) plan_cache_clear(t);
  if (!t || (!bytes && num_bytes)) return fail(PGPU_ERR_INVALID_ARGUMENT, "null argument");
  DeviceGuard g(t->device);
  std::lock_guard<std::mutex> lk(t->mu);
  auto it = t->segments.find(h);
  if (it == t->segments.end()) return fail(PGPU_ERR_NOT_FOUND, "unknown segment handle %lld", (long long)h);
  Segment& seg = *it->second;
  if (column < 0 || column >= (int)seg.cols.size()) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad column %d", column);
  Column& col = seg.cols[column];
  auto inv = std::make_shared<InvIndex>();
  std::vector<uint32_t> words;
  TRY(parse_inverted_index(reinterpret_cast<const uint8_t*>(bytes), num_bytes, col.card, seg.num_docs, column,
                           inv.get(), words));
  inv->bytes = (int64_t)std::max<size_t>(words.size(), 1) * 4;
  HIP_TRY(hipMalloc(&inv->d_block, inv->bytes));
  if (!words.empty()) HIP_TRY(hipMemcpy(inv->d_block, words.data(), words.size() * 4, hipMemcpyHostToDevice));
  if (col.inv) t->device_bytes -= col.inv->bytes;  // freed when the last plan using it is destroyed
  t->device_bytes += inv->bytes;
  col.inv = inv;
  return 0;
} PGPU_ABI_CATCH

int pgpu_attach_range_index(pgpu_table t, int64_t h, int32_t column, const void* bytes, int64_t num_bytes) try {
  PGPU_ABI_GUARD;
  if (!t || (!bytes && num_bytes) || num_bytes < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  t->version++;
  plan_cache_clear(t);
  std::lock_guard<std::mutex> lk(t->mu);
  auto it = t->segments.find(h);
  if (it == t->segments.end()) return fail(PGPU_ERR_NOT_FOUND, "unknown segment handle %lld", (long long)h);
  Segment& seg = *it->second;
  if (column < 0 || column >= (int)seg.cols.size()) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad column %d", column);
  Column& col = seg.cols[column];
  if (num_bytes == 0) {
    col.rng.reset();
    return 0;
  }
  if (col.raw) return fail(PGPU_ERR_UNSUPPORTED, "range index on raw (no-dictionary) column %d", column);
  auto r = std::make_shared<RangeIdx>();
  TRY(parse_range_index(reinterpret_cast<const uint8_t*>(bytes), num_bytes, col.card, seg.num_docs, r.get()));
  if (r->version == 0) col.rng.reset();  // a version Pinot does not load: no range index
  else col.rng = r;
  return 0;
} PGPU_ABI_CATCH

}  // extern "C"

namespace {
// The device traversal (K5) and residual scan (K6) index node, child, document and dictionary arrays with the
// star-tree's own numbers, so a tree read from files is checked here as OffHeapStarTree + StarTreeBuilderUtils
// guarantee it (BFS order, children contiguous and sorted by value, documents and dictIds in range) instead of
// being read out of bounds on the device.
int validate_startree(const pgpu_startree_desc* d, const std::vector<int32_t>& dim_card,
                      const std::vector<int32_t>& dim_bits) {
  const int N = d->num_nodes, D = d->num_dims, docs = d->num_docs;
  auto f = [&](int i, int k) {
    int32_t v;
    memcpy(&v, d->nodes + (size_t)i * 28 + (size_t)k * 4, 4);  // little-endian records, as the file holds them
    return v;
  };
  int next_child = 1;
  for (int i = 0; i < N; ++i) {
    const int dim = f(i, 0), val = f(i, 1), sd = f(i, 2), ed = f(i, 3), ad = f(i, 4), fc = f(i, 5), lc = f(i, 6);
    if (i == 0 ? dim != -1 : (dim < 0 || dim >= D))
      return fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree node %d: dimension id %d", i, dim);
    if (i > 0 && (val < -1 || val >= dim_card[dim]))
      return fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree node %d: dimension value %d", i, val);
    // start / end stay StarTreeNode.ALL (-1) where the builder never sets them (the root: TreeNode defaults)
    if ((!(sd == -1 && ed == -1) && (sd < 0 || sd > ed || ed > docs)) || ad < 0 || ad >= docs)
      return fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree node %d: documents [%d, %d) / %d of %d", i, sd, ed, ad, docs);
    if ((fc < 0) != (lc < 0)) return fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree node %d: child range", i);
    if (fc < 0) continue;
    if (fc != next_child || lc < fc || lc >= N || fc <= i)
      return fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree node %d: children [%d, %d] out of BFS order", i, fc, lc);
    const int cd = f(fc, 0);
    for (int c = fc; c <= lc; ++c)
      if (f(c, 0) != cd || cd <= dim)
        return fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree node %d: child %d dimension %d", i, c, f(c, 0));
    next_child = lc + 1;
  }
  if (next_child != N) return fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree: %d nodes unreachable", N - next_child);
  for (int k = 0; k < D; ++k) {  // every document's dictId within the segment dictionary (PinotDataBitSet.readInt)
    const uint8_t* b = d->dim_fwd[k];
    const int bits = dim_bits[k];
    for (int64_t i = 0; i < docs; ++i) {
      const int64_t bit = i * bits;
      uint64_t w = 0;
      for (int j = 0; j < 5 && (bit >> 3) + j < d->dim_fwd_len[k]; ++j) w |= (uint64_t)b[(bit >> 3) + j] << (32 - 8 * j);
      const uint32_t v = (uint32_t)((w >> (40 - (bit & 7) - bits)) & ((1ull << bits) - 1));
      if ((int64_t)v >= dim_card[k])
        return fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree dimension %d: document %lld has dictId %u of %d", k,
                    (long long)i, v, dim_card[k]);
    }
  }
  return 0;
}
}  // namespace

extern "C" {

int pgpu_attach_startree(pgpu_table t, int64_t h, const pgpu_startree_desc* d) try {
  PGPU_ABI_GUARD;
  if (t) t->version++;
  if (t) plan_cache_clear(t);
  if (!t || !d) return fail(PGPU_ERR_INVALID_ARGUMENT, "null argument");
  if (d->num_dims < 1 || d->num_dims > kMaxStarDims || d->num_nodes < 1 || d->num_docs < 0 || d->num_metrics < 1)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "bad star-tree shape (dims %d, nodes %d, docs %d, metrics %d)",
                d->num_dims, d->num_nodes, d->num_docs, d->num_metrics);
  DeviceGuard g(t->device);
  std::lock_guard<std::mutex> lk(t->mu);
  auto it = t->segments.find(h);
  if (it == t->segments.end()) return fail(PGPU_ERR_NOT_FOUND, "unknown segment handle %lld", (long long)h);
  Segment& seg = *it->second;
  auto st = std::make_unique<StarTreeDev>();
  st->num_dims = d->num_dims;
  st->num_nodes = d->num_nodes;
  st->num_docs = d->num_docs;
  // layout: nodes | dim fwd (padded words) | metric doubles | metric counts
  std::vector<int64_t> fwd_words(d->num_dims);
  int64_t bytes = ((int64_t)d->num_nodes * 28 + 15) & ~int64_t(15);
  for (int k = 0; k < d->num_dims; ++k) {
    const int c = d->dim_columns[k];
    if (c < 0 || c >= (int)seg.cols.size()) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad star-tree dimension column");
    const int bits = seg.cols[c].bits;
    const int64_t need = ((int64_t)d->num_docs * bits + 7) / 8;
    if (!d->dim_fwd[k] || d->dim_fwd_len[k] < need)
      return fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree dimension %d forward index too short", k);
    st->dim_cols.push_back(c);
    st->dim_bits.push_back(bits);
    fwd_words[k] = ((int64_t)d->num_docs + 31) / 32 * bits + kFwdPadWords;  // whole 32-doc groups (K6 decode)
    bytes += ((fwd_words[k] * 4) + 15) & ~int64_t(15);
  }
  {
    std::vector<int32_t> card;
    for (int c : st->dim_cols) card.push_back(std::max(seg.cols[c].card, 1));
    TRY(validate_startree(d, card, st->dim_bits));
  }
  for (int m = 0; m < d->num_metrics; ++m) {
    const pgpu_agg a = d->metrics[m];
    if (a.fn < PGPU_AGG_COUNT || a.fn > PGPU_AGG_AVG) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad metric function");
    const bool needs_f = a.fn != PGPU_AGG_COUNT, needs_c = a.fn == PGPU_AGG_COUNT || a.fn == PGPU_AGG_AVG;
    if ((needs_f && !d->metric_f64[m]) || (needs_c && !d->metric_i64[m]))
      return fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree metric %d values missing", m);
    if (needs_f && (a.column < 0 || a.column >= (int)seg.cols.size()))
      return fail(PGPU_ERR_INVALID_ARGUMENT, "bad star-tree metric column");
    st->metrics.push_back(a);
    bytes += (needs_f ? (int64_t)d->num_docs * 8 : 0) + (needs_c ? (int64_t)d->num_docs * 8 : 0) + 32;
  }
  HIP_TRY(hipMalloc(&st->d_block, bytes));
  st->bytes = bytes;
  std::vector<uint8_t> host(bytes, 0);
  int64_t off = 0;
  memcpy(host.data(), d->nodes, (size_t)d->num_nodes * 28);  // little-endian, as the file holds it
  st->d_nodes = reinterpret_cast<const int32_t*>(st->d_block);
  off = ((int64_t)d->num_nodes * 28 + 15) & ~int64_t(15);
  for (int k = 0; k < d->num_dims; ++k) {
    const int64_t nb = ((int64_t)d->num_docs * st->dim_bits[k] + 7) / 8;
    memcpy(host.data() + off, d->dim_fwd[k], nb);
    st->d_dim_fwd.push_back(reinterpret_cast<const uint32_t*>((uint8_t*)st->d_block + off));
    off += ((fwd_words[k] * 4) + 15) & ~int64_t(15);
  }
  for (int m = 0; m < d->num_metrics; ++m) {
    const pgpu_agg a = d->metrics[m];
    const double* pf = nullptr;
    const int64_t* pc = nullptr;
    if (a.fn != PGPU_AGG_COUNT) {
      memcpy(host.data() + off, d->metric_f64[m], (size_t)d->num_docs * 8);
      pf = reinterpret_cast<const double*>((uint8_t*)st->d_block + off);
      off += (int64_t)d->num_docs * 8 + 16;
    }
    if (a.fn == PGPU_AGG_COUNT || a.fn == PGPU_AGG_AVG) {
      memcpy(host.data() + off, d->metric_i64[m], (size_t)d->num_docs * 8);
      pc = reinterpret_cast<const int64_t*>((uint8_t*)st->d_block + off);
      off += (int64_t)d->num_docs * 8 + 16;
    }
    st->d_mf.push_back(pf);
    st->d_mc.push_back(pc);
  }
  HIP_TRY(hipMemcpyAsync(st->d_block, host.data(), bytes, hipMemcpyHostToDevice, t->stream));
  HIP_TRY(hipStreamSynchronize(t->stream));
  if (seg.star && seg.star->d_block) {
    hipFree(seg.star->d_block);
    t->device_bytes -= seg.star->bytes;
  }
  t->device_bytes += bytes;
  seg.star = std::move(st);
  return 0;
} PGPU_ABI_CATCH

int pgpu_table_num_segments(pgpu_table t, int32_t* count) try {
  PGPU_ABI_GUARD;
  if (!t || !count) return fail(PGPU_ERR_INVALID_ARGUMENT, "null argument");
  std::lock_guard<std::mutex> lk(t->mu);
  *count = (int32_t)t->segments.size();
  return 0;
} PGPU_ABI_CATCH

int64_t pgpu_table_device_bytes(pgpu_table t) { return t ? t->device_bytes : 0; }

int pgpu_table_add_dictionary_values(pgpu_table t, int col, int64_t n, const int64_t* vi, const double* vd,
                                     const uint8_t* blob, const int64_t* offsets) try {
  PGPU_ABI_GUARD;
  if (t) t->version++;
  if (t) plan_cache_clear(t);
  if (!t || col < 0 || col >= (int)t->names.size() || n < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  Dict d;
  d.type = t->types[col];
  if (is_int_type(d.type)) {
    if (n && !vi) return fail(PGPU_ERR_INVALID_ARGUMENT, "values_i64 required");
    d.iv.assign(vi, vi + n);
    std::sort(d.iv.begin(), d.iv.end());
    d.iv.erase(std::unique(d.iv.begin(), d.iv.end()), d.iv.end());
  } else if (is_fp_type(d.type)) {
    if (n && !vd) return fail(PGPU_ERR_INVALID_ARGUMENT, "values_f64 required");
    d.dv.assign(vd, vd + n);
  } else {
    if (n && (!blob || !offsets)) return fail(PGPU_ERR_INVALID_ARGUMENT, "blob/offsets required");
    for (int64_t i = 0; i < n; ++i) d.sv.emplace_back(reinterpret_cast<const char*>(blob + offsets[i]), offsets[i + 1] - offsets[i]);
    std::sort(d.sv.begin(), d.sv.end());
    d.sv.erase(std::unique(d.sv.begin(), d.sv.end()), d.sv.end());
  }
  std::lock_guard<std::mutex> lk(t->mu);
  if (merge_dict(t->global[col], d)) t->global_version[col]++;
  return 0;
} PGPU_ABI_CATCH

int pgpu_table_dictionary_size(pgpu_table t, int col, int64_t* size) try {
  PGPU_ABI_GUARD;
  if (!t || !size || col < 0 || col >= (int)t->names.size()) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  std::lock_guard<std::mutex> lk(t->mu);
  *size = (int64_t)t->global[col]->size();
  return 0;
} PGPU_ABI_CATCH

int pgpu_table_dictionary_i64(pgpu_table t, int col, int64_t* out) try {
  PGPU_ABI_GUARD;
  if (!t || !out || col < 0 || col >= (int)t->names.size() || !is_int_type(t->types[col]))
    return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  std::lock_guard<std::mutex> lk(t->mu);
  std::copy(t->global[col]->iv.begin(), t->global[col]->iv.end(), out);
  return 0;
} PGPU_ABI_CATCH

int pgpu_table_dictionary_f64(pgpu_table t, int col, double* out) try {
  PGPU_ABI_GUARD;
  if (!t || !out || col < 0 || col >= (int)t->names.size() || !is_fp_type(t->types[col]))
    return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  std::lock_guard<std::mutex> lk(t->mu);
  std::copy(t->global[col]->dv.begin(), t->global[col]->dv.end(), out);
  return 0;
} PGPU_ABI_CATCH

int pgpu_table_dictionary_str(pgpu_table t, int col, uint8_t* blob, int64_t cap, int64_t* offsets) try {
  PGPU_ABI_GUARD;
  if (!t || !offsets || col < 0 || col >= (int)t->names.size() || t->types[col] != PGPU_STRING)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  std::lock_guard<std::mutex> lk(t->mu);
  int64_t off = 0;
  offsets[0] = 0;
  const auto& sv = t->global[col]->sv;
  for (size_t i = 0; i < sv.size(); ++i) {
    if (blob) {
      if (off + (int64_t)sv[i].size() > cap) return fail(PGPU_ERR_INVALID_ARGUMENT, "blob too small");
      memcpy(blob + off, sv[i].data(), sv[i].size());
    }
    off += (int64_t)sv[i].size();
    offsets[i + 1] = off;
  }
  return 0;
} PGPU_ABI_CATCH

int pgpu_read_dict_ids(pgpu_table t, int64_t h, int col, const int32_t* docs, int32_t n, int32_t* out) try {
  PGPU_ABI_GUARD;
  if (!t || (n > 0 && (!docs || !out))) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  DeviceGuard g(t->device);
  std::shared_ptr<Segment> s;
  {
    std::lock_guard<std::mutex> lk(t->mu);
    auto it = t->segments.find(h);
    if (it == t->segments.end()) return fail(PGPU_ERR_NOT_FOUND, "unknown segment handle");
    s = it->second;
  }
  if (col < 0 || col >= (int)s->cols.size()) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad column");
  if (n <= 0) return 0;
  for (int32_t i = 0; i < n; ++i)
    if (docs[i] < 0 || docs[i] >= s->num_docs) return fail(PGPU_ERR_INVALID_ARGUMENT, "docId %d out of range", docs[i]);
  int32_t *d_docs = nullptr, *d_out = nullptr;
  HIP_TRY(hipMallocAsync((void**)&d_docs, (size_t)n * 4, t->stream));
  HIP_TRY(hipMallocAsync((void**)&d_out, (size_t)n * 4, t->stream));
  HIP_TRY(hipMemcpyAsync(d_docs, docs, (size_t)n * 4, hipMemcpyHostToDevice, t->stream));
  if (launch_gather_ids(s->cols[col].d_fwd, s->cols[col].bits, d_docs, n, d_out, t->stream))
    return fail(PGPU_ERR_DEVICE, "gather launch failed");
  HIP_TRY(hipMemcpyAsync(out, d_out, (size_t)n * 4, hipMemcpyDeviceToHost, t->stream));
  HIP_TRY(hipFreeAsync(d_docs, t->stream));
  HIP_TRY(hipFreeAsync(d_out, t->stream));
  HIP_TRY(hipStreamSynchronize(t->stream));
  return 0;
} PGPU_ABI_CATCH

int pgpu_unpack_fixed_bit_device(const void* d_fwd, int64_t fwd_len, int32_t bits, int64_t start, int64_t n,
                                 int32_t* d_out, void* stream) try {
  PGPU_ABI_GUARD;
  if (bits < 1 || bits > 31 || start < 0 || n < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  // the two-word gather reads up to word ((start+n-1)*bits >> 5) + 1
  const int64_t last_word = n > 0 ? (((start + n - 1) * bits) >> 5) + 1 : 0;
  if (n > 0 && (last_word + 1) * 4 > fwd_len)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "device buffer must hold %lld bytes (2 words past the last value)",
                (long long)((last_word + 1) * 4));
  if (launch_unpack(reinterpret_cast<const uint32_t*>(d_fwd), bits, start, n, d_out, stream))
    return fail(PGPU_ERR_DEVICE, "unpack launch failed: %s", hipGetErrorString(hipGetLastError()));
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_create(pgpu_table t, const int64_t* handles, int32_t nsegs, const pgpu_query* q, pgpu_plan* out) try {
  PGPU_ABI_GUARD;
  if (!t || !out || (nsegs > 0 && !handles) || nsegs < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  DeviceGuard g(t->device);
  auto P = std::make_unique<pgpu_plan_s>();
  // A cached plan is never a numGroupsLimit split (composite plans are not cached) and the split decision is a
  // function of the cache key (query, segments, pinned-state version): a hit skips it.
  const bool cache = plan_cache_enabled(t, q);
  const std::string key = cache ? plan_cache_key(t, handles, nsegs, q) : std::string();
  if (!cache || !plan_cache_get(t, key, P.get())) {
    bool composite = false;
    TRY(split_for_groups_limit(t, handles, nsegs, q, P.get(), &composite));
    if (composite) {
      *out = P.release();
      return 0;
    }
    TRY(plan_create_impl(t, handles, nsegs, q, P.get()));
    if (cache) plan_cache_put(t, key, *P);
  }
  P->end_time_ms = q->end_time_ms;
  P->scratch = acquire_scratch(t);
  *out = P.release();
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_destroy(pgpu_plan P) try {
  PGPU_ABI_GUARD;
  if (!P) return 0;
  for (auto& part : P->parts) release_scratch(P->table, part.plan->scratch);
  release_scratch(P->table, P->scratch);
  delete P;
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_cancel(pgpu_plan P) try {
  // no ABI guard: the canceller must not wait behind the query thread's own entry points
  if (!P) return fail(PGPU_ERR_INVALID_ARGUMENT, "null plan");
  __atomic_store_n(&P->cancel, 1, __ATOMIC_RELEASE);
  for (auto& part : P->parts) __atomic_store_n(&part.plan->cancel, 1, __ATOMIC_RELEASE);
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_leaf_kinds(pgpu_plan P, int64_t* counts) try {
  PGPU_ABI_GUARD;
  if (!P || !counts) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  for (int k = 0; k < kLeafKinds; ++k) counts[k] = P->leaf_kinds[k];
  for (const auto& part : P->parts)
    for (int k = 0; k < kLeafKinds; ++k) counts[k] += part.plan->leaf_kinds[k];
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_group_path(pgpu_plan P, int32_t* path) try {
  PGPU_ABI_GUARD;
  if (!P || !path) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  const pgpu_plan_s* K = P->composite && !P->parts.empty() ? P->parts[0].plan.get() : P;
  *path = K->part_hash     ? PGPU_PATH_HASH_PARTITIONED
          : K->partitioned ? PGPU_PATH_PARTITIONED
          : K->mode == MODE_HASH ? PGPU_PATH_HASH
          : K->mode == MODE_GLOBAL ? PGPU_PATH_GLOBAL
                                   : PGPU_PATH_LDS;
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_layout(pgpu_plan P, int32_t* num_slots, int64_t* num_keys, int32_t* kinds) try {
  PGPU_ABI_GUARD;
  if (!P) return fail(PGPU_ERR_INVALID_ARGUMENT, "null plan");
  if (P->composite) return fail(PGPU_ERR_UNSUPPORTED, "numGroupsLimit plan: its parts have their own group tables");
  if (num_slots) *num_slots = (int32_t)P->slot_kind.size();
  if (num_keys) *num_keys = P->hash ? 0 : P->num_keys;
  if (kinds) for (size_t i = 0; i < P->slot_kind.size(); ++i) kinds[i] = P->slot_kind[i];
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_create_execute(pgpu_table t, const int64_t* handles, int32_t nsegs, const pgpu_query* q, void* stream,
                             void* d_table, pgpu_plan* out) try {
  PGPU_ABI_GUARD;
  if (!t || !out || (nsegs > 0 && !handles) || nsegs < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  const double tt0 = trace_on() ? now_us() : 0;
  DeviceGuard g(t->device);
  auto P = std::make_unique<pgpu_plan_s>();
  // a cache hit skips the numGroupsLimit split decision (pgpu_plan_create)
  const bool cache = plan_cache_enabled(t, q);
  const std::string key = cache ? plan_cache_key(t, handles, nsegs, q) : std::string();  // before planning
  const bool hit = cache && plan_cache_get(t, key, P.get());
  const double tt1 = trace_on() ? now_us() : 0;
  if (!hit) {
    bool composite = false;
    TRY(split_for_groups_limit(t, handles, nsegs, q, P.get(), &composite));
    if (composite) {  // executed part by part at finalize
      if (d_table) return fail(PGPU_ERR_UNSUPPORTED, "external table with a numGroupsLimit plan");
      P->executed = true;
      *out = P.release();
      return 0;
    }
  }
  StreamExec se;
  se.stream = stream ? reinterpret_cast<hipStream_t>(stream) : t->stream;
  se.d_table = d_table;
  const double tt2 = trace_on() ? now_us() : 0;
  P->end_time_ms = q->end_time_ms;
  P->scratch = acquire_scratch(t);  // before plan_create_impl takes the table lock (acquire_scratch locks it too)
  const double tt3 = trace_on() ? now_us() : 0;
  int rc = 0;
  if (!hit) {
    rc = plan_create_impl(t, handles, nsegs, q, P.get(), &se);
    if (!rc && cache && !P->executed) plan_cache_put(t, key, *P);
  }
  if (!rc && !P->executed) {
    if (P->hash && d_table) rc = fail(PGPU_ERR_UNSUPPORTED, "external table with a hash-mode plan");
    else rc = plan_execute_impl(P.get(), se.stream, d_table);
  }
  if (trace_on())
    fprintf(stderr, "[pgpu] create_execute%s: cache %.1f, groups-limit split %.1f, scratch %.1f, plan+execute %.1f us\n",
            hit ? " (hit)" : "", tt1 - tt0, tt2 - tt1, tt3 - tt2, now_us() - tt3);
  if (rc) {
    if (P->scratch) {
      // no launch of this plan may still use its scratch: wait, or (timeout) leave it to the queued work
      if (rc == PGPU_ERR_TIMEOUT || rc == PGPU_ERR_CANCELLED) abandon_scratch(P->scratch, se.stream);
      else hipStreamSynchronize(se.stream);
      release_scratch(t, P->scratch);
      P->scratch = nullptr;
    }
    return rc;
  }
  *out = P.release();
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_execute(pgpu_plan P, void* stream, void* d_table) try {
  PGPU_ABI_GUARD;
  if (!P) return fail(PGPU_ERR_INVALID_ARGUMENT, "null plan");
  if (P->composite) {
  PGPU_ABI_GUARD;
    if (d_table) return fail(PGPU_ERR_UNSUPPORTED, "external table with a numGroupsLimit plan");
    P->executed = true;
    return 0;
  }
  if (P->hash && d_table) return fail(PGPU_ERR_UNSUPPORTED, "external table with a hash-mode plan");
  DeviceGuard g(P->table->device);
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : P->table->stream;
  return plan_execute_impl(P, s, d_table);
} PGPU_ABI_CATCH

int pgpu_plan_finalize(pgpu_plan P, void* stream, const void* d_table, pgpu_result* out) try {
  PGPU_ABI_GUARD;
  if (!P || !out) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  DeviceGuard g(P->table->device);
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : P->table->stream;
  auto R = std::make_unique<pgpu_result_s>();
  if (P->composite) {
    if (!P->executed) return fail(PGPU_ERR_INVALID_ARGUMENT, "plan not executed");
    if (d_table) return fail(PGPU_ERR_UNSUPPORTED, "external table with a numGroupsLimit plan");
    TRY(composite_finalize(P, s, R.get()));
  } else if (P->shard) {  // reduce-scattered by pgpu_plan_combine: this rank's key range
    TRY(plan_finalize_impl(P, s, P->shard, P->shard_begin, P->shard_count, R.get()));
  } else {
    TRY(plan_finalize_impl(P, s, d_table, 0, P->num_keys, R.get()));
  }
  *out = R.release();
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_finalize_range(pgpu_plan P, void* stream, const void* d_table_shard, int64_t key_begin,
                             int64_t key_count, pgpu_result* out) try {
  PGPU_ABI_GUARD;
  if (!P || !out || !d_table_shard || key_begin < 0 || key_count < 0 || key_begin + key_count > P->num_keys)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  if (P->hash) return fail(PGPU_ERR_UNSUPPORTED, "hash-mode group tables are not key-range shardable");
  if (P->composite)
    return fail(PGPU_ERR_UNSUPPORTED, "numGroupsLimit below the key space: finalize the whole table");
  DeviceGuard g(P->table->device);
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : P->table->stream;
  auto R = std::make_unique<pgpu_result_s>();
  TRY(plan_finalize_impl(P, s, d_table_shard, key_begin, key_count, R.get()));
  *out = R.release();
  return 0;
} PGPU_ABI_CATCH

// ---- cross-GPU combine of hash-mode tables (device records) and of any finalized result (host rows)
namespace {
int exchangeable(pgpu_plan P) {
  if (!P) return fail(PGPU_ERR_INVALID_ARGUMENT, "null plan");
  if (P->composite) return fail(PGPU_ERR_UNSUPPORTED, "numGroupsLimit plan: exchange its finalized result rows");
  if (!P->hash) return fail(PGPU_ERR_UNSUPPORTED, "dense group tables merge element-wise (all-reduce / reduce-scatter)");
  if (!P->stage_end.empty())
    return fail(PGPU_ERR_UNSUPPORTED, "ARRAY_MAP key stages are rank-local: exchange the finalized result rows");
  if (!P->executed || !P->scratch) return fail(PGPU_ERR_INVALID_ARGUMENT, "plan not executed");
  return 0;
}
// The agreed kinds of the exchange: the plan's own, except that an int64 SUM may travel (and merge) as float64 when
// another rank's sum of the same slot is float64 (int_sum_fits differs by the ranks' segments).
int check_kinds(const std::vector<int32_t>& mine, const int32_t* kinds, uint32_t* conv) {
  *conv = 0;
  if (!kinds) return 0;
  for (size_t s = 0; s < mine.size(); ++s) {
    if (kinds[s] == mine[s]) continue;
    if (mine[s] == SLOT_SUM_I64 && kinds[s] == SLOT_SUM_F64) { *conv |= 1u << s; continue; }
    return fail(PGPU_ERR_INVALID_ARGUMENT, "slot %zu: kind %d cannot become %d", s, mine[s], kinds[s]);
  }
  return 0;
}
// Owner rank of a finalized group (its dictId tuple): the same on every rank.
int32_t row_owner(const int64_t* ids, int nk, int32_t nparts) {
  uint64_t h = 0x9E3779B97F4A7C15ull;
  for (int j = 0; j < nk; ++j) h = (h ^ (uint64_t)ids[j]) * 0xD6E8FEB86659FD93ull;
  h ^= h >> 32;
  return (int32_t)(h % (uint64_t)nparts);
}
}  // namespace

}  // extern "C"

namespace {
// A fresh hash table of >= 2n slots holding n (key, slot words) records (merged per slot kind): the owner's merge of
// an exchange, and the materialised table of a K8h plan.
int build_hash_table(pgpu_plan_s* P, hipStream_t s, const uint64_t* d_records, int64_t n) {
  Scratch* sc = P->scratch;
  const int nslots = (int)P->slot_kind.size();
  int64_t G = 1024;
  while (G < 2 * n) G <<= 1;
  // DevBuf growth frees the old buffer with hipFree, which waits for the device: nothing queued still reads it
  TRY(sc->table.ensure((size_t)nslots * G * 8 + 64));
  TRY(sc->hash_keys.ensure((size_t)G * 8));
  P->num_keys = G;
  P->d_table_used = sc->table.p;
  if (launch_table_init(sc->table.as<uint64_t>(), P->slot_kind.data(), nslots, G, sc->hash_keys.as<unsigned long long>(), s))
    return fail(PGPU_ERR_DEVICE, "table init launch failed: %s", hipGetErrorString(hipGetLastError()));
  if (launch_merge_records(d_records, n, nslots, P->slot_kind.data(), sc->table.as<uint64_t>(),
                           sc->hash_keys.as<unsigned long long>(), G, s))
    return fail(PGPU_ERR_DEVICE, "merge launch failed: %s", hipGetErrorString(hipGetLastError()));
  return 0;
}

// A K8h plan's groups as the hash table the exchange entries read (pgpu_plan_exchange_counts / _export): the
// statistics words move out of the (record-less) table buffer first, then the records are inserted.
int part_hash_materialize(pgpu_plan_s* P, hipStream_t s) {
  if (!P->part_hash_live) return 0;
  Scratch* sc = P->scratch;
  TRY(sc->stats.ensure(64));
  if (P->d_stats != sc->stats.as<unsigned long long>()) {
    HIP_TRY(hipMemcpyAsync(sc->stats.p, P->d_stats, 64, hipMemcpyDeviceToDevice, s));
    P->d_stats = sc->stats.as<unsigned long long>();
  }
  TRY(sc->xstage.ensure(64));
  uint64_t* st = reinterpret_cast<uint64_t*>(sc->xstage.p);
  HIP_TRY(hipMemcpyAsync(st, sc->counter.p, 8, hipMemcpyDeviceToHost, s));
  TRY(wait_plan(P, s));
  if (st[0] > (uint64_t)part_hash_out_cap(P)) return part_hash_overflow(P, st[0]);
  const int64_t n = (int64_t)st[0];
  TRY(build_hash_table(P, s, sc->ckeys.as<uint64_t>(), n));
  P->part_hash_live = false;
  return 0;
}
}  // namespace

extern "C" {

int pgpu_plan_exchange_counts(pgpu_plan P, void* stream, int32_t nparts, int64_t* counts) try {
  PGPU_ABI_GUARD;
  TRY(exchangeable(P));
  if (nparts < 1 || nparts > 64 || !counts) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  if (P->merged_records >= 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "the table already holds merged records");
  DeviceGuard g(P->table->device);
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : P->table->stream;
  TRY(part_hash_materialize(P, s));
  Scratch* sc = P->scratch;
  TRY(sc->counter.ensure((size_t)nparts * 8 + 64));
  HIP_TRY(hipMemsetAsync(sc->counter.p, 0, (size_t)nparts * 8, s));
  if (launch_exchange_count(reinterpret_cast<const uint64_t*>(P->d_table_used), sc->hash_keys.as<unsigned long long>(),
                            P->num_keys, nparts, sc->counter.as<unsigned long long>(), s))
    return fail(PGPU_ERR_DEVICE, "exchange count launch failed: %s", hipGetErrorString(hipGetLastError()));
  TRY(sc->xstage.ensure((size_t)nparts * 8 + 64));
  uint64_t* st = reinterpret_cast<uint64_t*>(sc->xstage.p);
  HIP_TRY(hipMemcpyAsync(st, sc->counter.p, (size_t)nparts * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(st + nparts, P->d_stats, 48, hipMemcpyDeviceToHost, s));
  TRY(wait_plan(P, s));
  if (st[nparts + 5]) return timeout_fail(P);
  P->xchg_counts.assign(nparts, 0);
  for (int p = 0; p < nparts; ++p) counts[p] = P->xchg_counts[p] = (int64_t)st[p];
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_exchange_export(pgpu_plan P, void* stream, int32_t nparts, const int32_t* kinds, void* d_out,
                              int64_t cap) try {
  PGPU_ABI_GUARD;
  TRY(exchangeable(P));
  if ((int32_t)P->xchg_counts.size() != nparts || nparts < 1)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "pgpu_plan_exchange_counts with %d parts first", nparts);
  int64_t total = 0;
  for (int64_t c : P->xchg_counts) total += c;
  if (total > 0 && (!d_out || cap < total))
    return fail(PGPU_ERR_INVALID_ARGUMENT, "the records need %lld rows", (long long)total);
  uint32_t conv = 0;
  TRY(check_kinds(P->slot_kind, kinds, &conv));
  if (total == 0) return 0;
  DeviceGuard g(P->table->device);
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : P->table->stream;
  Scratch* sc = P->scratch;
  TRY(sc->xcursor.ensure((size_t)nparts * 8));
  TRY(sc->xstage.ensure((size_t)nparts * 8 + 64));
  uint64_t* st = reinterpret_cast<uint64_t*>(sc->xstage.p);
  uint64_t off = 0;
  for (int p = 0; p < nparts; ++p) { st[p] = off; off += (uint64_t)P->xchg_counts[p]; }
  HIP_TRY(hipMemcpyAsync(sc->xcursor.p, st, (size_t)nparts * 8, hipMemcpyHostToDevice, s));
  if (launch_exchange_scatter(reinterpret_cast<const uint64_t*>(P->d_table_used), sc->hash_keys.as<unsigned long long>(),
                              P->num_keys, (int32_t)P->slot_kind.size(), nparts, conv,
                              sc->xcursor.as<unsigned long long>(), reinterpret_cast<uint64_t*>(d_out), s))
    return fail(PGPU_ERR_DEVICE, "exchange scatter launch failed: %s", hipGetErrorString(hipGetLastError()));
  // the staged cursors must stay put until the upload ran: the next use of xstage waits for this stream
  HIP_TRY(hipStreamSynchronize(s));
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_exchange_merge(pgpu_plan P, void* stream, const int32_t* kinds, const void* d_records, int64_t n) try {
  PGPU_ABI_GUARD;
  TRY(exchangeable(P));
  if (n < 0 || (n > 0 && !d_records) || n > (INT64_C(1) << 40))  // the table below holds >= 2n slots
    return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  uint32_t conv = 0;
  TRY(check_kinds(P->slot_kind, kinds, &conv));
  DeviceGuard g(P->table->device);
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : P->table->stream;
  Scratch* sc = P->scratch;
  const int nslots = (int)P->slot_kind.size();
  if (kinds && !std::equal(P->slot_kind.begin(), P->slot_kind.end(), kinds)) {
    if (P->slot_kind_planned.empty()) P->slot_kind_planned = P->slot_kind;  // restored by the next execution
    P->slot_kind.assign(kinds, kinds + nslots);
  }
  // the statistics words leave the table buffer (it is resized below)
  TRY(sc->stats.ensure(64));
  if (P->d_stats != sc->stats.as<unsigned long long>()) {
    HIP_TRY(hipMemcpyAsync(sc->stats.p, P->d_stats, 64, hipMemcpyDeviceToDevice, s));
    P->d_stats = sc->stats.as<unsigned long long>();
  }
  TRY(build_hash_table(P, s, reinterpret_cast<const uint64_t*>(d_records), n));
  P->merged_records = n;
  P->part_hash_live = false;  // the merged table replaces this rank's K8h records
  return 0;
} PGPU_ABI_CATCH

int pgpu_result_slot_kinds(pgpu_result r, int32_t* num_slots, int32_t* kinds) try {
  PGPU_ABI_GUARD;
  if (!r) return fail(PGPU_ERR_INVALID_ARGUMENT, "null result");
  if ((int)r->slot_kind.size() != r->num_slots) return fail(PGPU_ERR_UNSUPPORTED, "result without slot kinds");
  if (num_slots) *num_slots = r->num_slots;
  if (kinds) for (int i = 0; i < r->num_slots; ++i) kinds[i] = r->slot_kind[i];
  return 0;
} PGPU_ABI_CATCH

int pgpu_result_exchange_rows(pgpu_result r, int32_t nparts, const int32_t* kinds, int64_t* rows, int64_t* counts) try {
  PGPU_ABI_GUARD;
  if (!r || nparts < 1 || nparts > (1 << 20) || !counts || (r->n > 0 && !rows))
    return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  if ((int)r->slot_kind.size() != r->num_slots) return fail(PGPU_ERR_UNSUPPORTED, "result without slot kinds");
  uint32_t conv = 0;
  TRY(check_kinds(r->slot_kind, kinds, &conv));
  if (r->compact.load(std::memory_order_acquire)) TRY(pgpu::result_expand(r));
  const int nk = r->num_keys, ns = r->num_slots, w = nk + ns;
  std::vector<int32_t> owner((size_t)r->n);
  std::vector<int64_t> off(nparts + 1, 0), ids(std::max(nk, 1));
  for (int64_t i = 0; i < r->n; ++i) {
    for (int j = 0; j < nk; ++j) ids[j] = r->gid(j)[i];
    owner[i] = row_owner(ids.data(), nk, nparts);
    ++off[owner[i] + 1];
  }
  for (int p = 0; p < nparts; ++p) { counts[p] = off[p + 1]; off[p + 1] += off[p]; }
  for (int64_t i = 0; i < r->n; ++i) {
    int64_t* o = rows + off[owner[i]]++ * w;
    for (int j = 0; j < nk; ++j) o[j] = r->gid(j)[i];
    for (int k = 0; k < ns; ++k) {
      uint64_t v = r->slot(k)[i];
      if ((conv >> k) & 1u) {
        const double d = (double)(int64_t)v;
        memcpy(&v, &d, 8);
      }
      o[nk + k] = (int64_t)v;
    }
  }
  return 0;
} PGPU_ABI_CATCH

int pgpu_result_merge_rows(pgpu_result tmpl, const int64_t* rows, int64_t n, const int32_t* kinds, pgpu_result* out) try {
  PGPU_ABI_GUARD;
  if (!tmpl || !out || n < 0 || (n > 0 && !rows)) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  if ((int)tmpl->slot_kind.size() != tmpl->num_slots) return fail(PGPU_ERR_UNSUPPORTED, "result without slot kinds");
  uint32_t conv = 0;
  TRY(check_kinds(tmpl->slot_kind, kinds, &conv));
  const int nk = tmpl->num_keys, ns = tmpl->num_slots, w = nk + ns;
  std::vector<int32_t> kind(tmpl->slot_kind);
  if (kinds) kind.assign(kinds, kinds + ns);
  // GroupByDataTableReducer / IndexedTable.upsert across servers: rows of one group merge by AggregationFunction.merge
  using Key = std::array<int64_t, kMaxKeys>;
  struct KeyHash {
    size_t operator()(const Key& k) const {
      uint64_t h = 0;
      for (int64_t v : k) h = (h ^ (uint64_t)v) * 0x9E3779B97F4A7C15ull;
      return (size_t)(h ^ (h >> 29));
    }
  };
  std::unordered_map<Key, int64_t, KeyHash> index;
  index.reserve((size_t)n);
  std::vector<int64_t> first;  // per merged group: its first row, then the folded words
  std::vector<uint64_t> vals;
  for (int64_t r = 0; r < n; ++r) {
    const int64_t* e = rows + r * w;
    Key key{};
    for (int j = 0; j < nk; ++j) {
      if (e[j] < 0 || e[j] > INT32_MAX) return fail(PGPU_ERR_INVALID_ARGUMENT, "row %lld: bad dictId", (long long)r);
      key[j] = e[j];
    }
    auto it = index.find(key);
    if (it == index.end()) {
      index.emplace(key, (int64_t)first.size());
      first.push_back(r);
      for (int s = 0; s < ns; ++s) vals.push_back((uint64_t)e[nk + s]);
      continue;
    }
    uint64_t* dst = vals.data() + it->second * ns;
    for (int s = 0; s < ns; ++s) {
      const uint64_t v = (uint64_t)e[nk + s];
      switch (kind[s]) {
        case SLOT_COUNT: case SLOT_SUM_I64: dst[s] += v; break;
        case SLOT_SUM_F64: {
          double a, b;
          memcpy(&a, &dst[s], 8);
          memcpy(&b, &v, 8);
          a += b;
          memcpy(&dst[s], &a, 8);
          break;
        }
        case SLOT_MIN_KEY: if ((int64_t)v < (int64_t)dst[s]) dst[s] = v; break;
        default: if ((int64_t)v > (int64_t)dst[s]) dst[s] = v; break;
      }
    }
  }
  const int64_t m = (int64_t)first.size();
  std::vector<int64_t> order(m);
  std::iota(order.begin(), order.end(), 0);
  std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {  // ascending, last group-by column most significant
    const int64_t* x = rows + first[a] * w;
    const int64_t* y = rows + first[b] * w;
    for (int j = nk - 1; j >= 0; --j)
      if (x[j] != y[j]) return x[j] < y[j];
    return false;
  });
  auto R = std::make_unique<pgpu_result_s>();
  R->pool = tmpl->pool;
  TRY(R->alloc(nk, ns, m));
  for (int64_t i = 0; i < m; ++i) {
    const int64_t* e = rows + first[order[i]] * w;
    for (int j = 0; j < nk; ++j) R->gid(j)[i] = (int32_t)e[j];
    for (int s = 0; s < ns; ++s) R->slot(s)[i] = vals[order[i] * ns + s];
  }
  R->num_aggs = tmpl->num_aggs;
  R->agg_slot = tmpl->agg_slot;
  R->slot_kind = kind;
  R->agg_conv = tmpl->agg_conv;
  for (int a = 0; a < R->num_aggs; ++a)
    if ((tmpl->agg_fn[a] == PGPU_AGG_SUM || tmpl->agg_fn[a] == PGPU_AGG_AVG) && kind[R->agg_slot[a]] == SLOT_SUM_F64)
      R->agg_conv[a] = RCONV_F64;
  R->key_cols = tmpl->key_cols;
  R->key_types = tmpl->key_types;
  R->key_dicts = tmpl->key_dicts;
  R->agg_fn = tmpl->agg_fn;
  R->agg_col = tmpl->agg_col;
  memcpy(R->stats, tmpl->stats, sizeof R->stats);
  R->groups_limit_reached = tmpl->groups_limit_reached;
  *out = R.release();
  return 0;
} PGPU_ABI_CATCH

// ---- communicator and the one-call cross-GPU combine (comm.h / comm.cpp)
int pgpu_comm_unique_id(int32_t kind, void* id) try {
  PGPU_ABI_GUARD;
  if (!id) return fail(PGPU_ERR_INVALID_ARGUMENT, "null id");
  return pgpu::comm_unique_id(kind, id);
} PGPU_ABI_CATCH

int pgpu_comm_create(int32_t kind, const void* id, int32_t nranks, int32_t rank, int32_t device, pgpu_comm* out) try {
  PGPU_ABI_GUARD;
  if (!out) return fail(PGPU_ERR_INVALID_ARGUMENT, "null out");
  pgpu::Comm* c = nullptr;
  TRY(pgpu::comm_create(kind, id, nranks, rank, device, &c));
  auto h = new pgpu_comm_s();
  h->impl.reset(c);
  h->kind = kind;
  *out = h;
  return 0;
} PGPU_ABI_CATCH

int pgpu_comm_destroy(pgpu_comm c) try {
  PGPU_ABI_GUARD;
  if (!c) return 0;
  delete c;  // the communicator itself goes with its last reference (plans combined on it hold one)
  return 0;
} PGPU_ABI_CATCH

int pgpu_comm_recreate(pgpu_comm c, const void* id) try {
  PGPU_ABI_GUARD;
  if (!c || !id) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  pgpu::Comm* fresh = nullptr;
  const pgpu::Comm& old = *c->impl;
  TRY(pgpu::comm_create(c->kind, id, old.nranks, old.rank, old.device, &fresh));
  fresh->timeout_ms.store(old.timeout_ms.load(std::memory_order_relaxed), std::memory_order_relaxed);
  // plans combined on the old communicator keep it (pgpu_plan_s::comm_used) until they are finalized or destroyed
  c->impl.reset(fresh);
  return 0;
} PGPU_ABI_CATCH

int pgpu_comm_status(pgpu_comm c, int32_t* aborted) try {
  PGPU_ABI_GUARD;
  if (!c || !aborted) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  *aborted = c->impl->aborted.load() ? 1 : 0;
  return 0;
} PGPU_ABI_CATCH

int pgpu_comm_rank(pgpu_comm c, int32_t* rank, int32_t* nranks) try {
  PGPU_ABI_GUARD;
  if (!c) return fail(PGPU_ERR_INVALID_ARGUMENT, "null communicator");
  if (rank) *rank = c->impl->rank;
  if (nranks) *nranks = c->impl->nranks;
  return 0;
} PGPU_ABI_CATCH

int pgpu_comm_set_timeout(pgpu_comm c, int64_t timeout_ms) try {
  PGPU_ABI_GUARD;
  if (!c) return fail(PGPU_ERR_INVALID_ARGUMENT, "null communicator");
  c->impl->timeout_ms.store(timeout_ms, std::memory_order_relaxed);
  return 0;
} PGPU_ABI_CATCH

int pgpu_comm_abort(pgpu_comm c) try {
  PGPU_ABI_GUARD;
  if (!c) return fail(PGPU_ERR_INVALID_ARGUMENT, "null communicator");
  c->impl->abort();
  return 0;
} PGPU_ABI_CATCH

int pgpu_comm_allgather(pgpu_comm c, const void* send, int64_t bytes, void* recv) try {
  PGPU_ABI_GUARD;
  if (!c || bytes < 0 || (bytes > 0 && (!send || !recv))) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  DeviceGuard g(c->impl->device);
  return c->impl->allgather_host(send, (size_t)bytes, recv);
} PGPU_ABI_CATCH

namespace {
// Content hash of a dictionary snapshot (computed once per snapshot): ranks compare their key spaces with it.
uint64_t dict_digest(const Dict& d) {
  uint64_t h = __atomic_load_n(&d.digest, __ATOMIC_RELAXED);
  if (h) return h;
  h = 0xcbf29ce484222325ull ^ (uint64_t)d.type;
  auto mix = [&h](uint64_t v) {
    h = (h ^ v) * 0x100000001b3ull;
    h ^= h >> 31;
  };
  mix(d.size());
  if (is_int_type(d.type)) {
    for (int64_t v : d.iv) mix((uint64_t)v);
  } else if (is_fp_type(d.type)) {
    for (double v : d.dv) {
      uint64_t u;
      memcpy(&u, &v, 8);
      mix(u);
    }
  } else {
    for (const std::string& v : d.sv) {
      mix(v.size());
      for (size_t i = 0; i < v.size(); i += 8) {
        uint64_t u = 0;
        memcpy(&u, v.data() + i, std::min<size_t>(8, v.size() - i));
        mix(u);
      }
    }
  }
  if (!h) h = 1;
  __atomic_store_n(const_cast<uint64_t*>(&d.digest), h, __ATOMIC_RELAXED);
  return h;
}

// The group-key space of a plan: dictionaries of the group-by columns and, for table-keyed modes, the composite key
// layout.  Equal on every rank after a dictionary union.
uint64_t key_space_digest(const pgpu_plan_s* P, bool layout) {
  uint64_t h = 0x84222325cbf29ce4ull;
  auto mix = [&h](uint64_t v) { h = (h ^ v) * 0x9E3779B97F4A7C15ull; h ^= h >> 29; };
  mix(P->key_dicts.size());
  for (const auto& d : P->key_dicts) mix(d ? dict_digest(*d) : 0);
  if (layout) {
    for (int64_t v : P->key_card) mix((uint64_t)v);
    for (int64_t v : P->key_off) mix((uint64_t)v);
    for (int64_t v : P->key_stride) mix((uint64_t)v);
  }
  return h;
}

// One rank's part of the mode agreement (int64 words).
enum { CI_MODE = 0, CI_KEYS, CI_SLOTS, CI_DIGEST, CI_KINDS, CI_WORDS = CI_KINDS + kMaxSlots };

// Agreed kinds of ranks' slots: equal, or int64 / float64 sums of one slot meeting as float64.
int agree_kinds(const std::vector<int64_t>& all, int nranks, int ns, int32_t* kinds) {
  for (int s = 0; s < ns; ++s) {
    bool i64 = false, f64 = false, other = false;
    int32_t k0 = (int32_t)all[CI_KINDS + s];
    for (int r = 0; r < nranks; ++r) {
      const int32_t k = (int32_t)all[(size_t)r * CI_WORDS + CI_KINDS + s];
      i64 |= k == SLOT_SUM_I64;
      f64 |= k == SLOT_SUM_F64;
      if (k != SLOT_SUM_I64 && k != SLOT_SUM_F64) other = true;
      if (other && k != k0) return fail(PGPU_ERR_INVALID_ARGUMENT, "ranks disagree on slot %d (kinds %d, %d)", s, k0, k);
    }
    kinds[s] = other ? k0 : f64 ? SLOT_SUM_F64 : SLOT_SUM_I64;
    (void)i64;
  }
  return 0;
}
}  // namespace

namespace {
// Every rank's status before a collective phase, exchanged with `bytes` of payload whose first int64 word is the
// status (all = nranks x bytes): a rank whose own part failed still takes part in this exchange, so the ranks fail
// together instead of some waiting in a collective the failed one never enters.  Returns this rank's own failure
// (its message kept), or one naming the first peer that failed.
int agree_status_with(pgpu::Comm* C, int rc, const void* payload, size_t bytes, void* all) {
  const std::string keep = rc ? g_err : std::string();
  TRY(C->allgather_host(payload, bytes, all));
  if (rc) {
    g_err = keep;
    return rc;
  }
  for (int p = 0; p < C->nranks; ++p) {
    int64_t st;
    memcpy(&st, static_cast<const uint8_t*>(all) + (size_t)p * bytes, 8);
    if (st) return fail((int)st, "rank %d of %d failed its part of the cross-GPU combine (error %lld)", p, C->nranks,
                        (long long)st);
  }
  return 0;
}
int agree_status(pgpu::Comm* C, int rc) {
  std::vector<int64_t> all(C->nranks);
  const int64_t mine = rc;
  return agree_status_with(C, rc, &mine, 8, all.data());
}
}  // namespace

int pgpu_plan_combine_mode(pgpu_plan P, pgpu_comm c, int64_t shard_bytes, int32_t* mode, int32_t* kinds) try {
  PGPU_ABI_GUARD;
  if (!P || !c || !mode) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  pgpu::CommWaitScope wait_limits(P->end_time_ms, &P->cancel);
  const int N = c->impl->nranks;
  int local;
  const pgpu_plan_s* K = P;  // the plan whose key space and slots describe the query on this rank
  if (P->composite) {
    local = PGPU_COMBINE_ROWS;
    if (!P->parts.empty()) K = P->parts[0].plan.get();
  } else if (P->hash) {
    local = P->stage_end.empty() ? PGPU_COMBINE_HASH : PGPU_COMBINE_ROWS;  // ARRAY_MAP stages: rank-local keys
  } else {
    local = (int64_t)P->slot_kind.size() * P->num_keys * 8 >= shard_bytes ? PGPU_COMBINE_REDUCE_SCATTER
                                                                           : PGPU_COMBINE_ALL_REDUCE;
  }
  std::vector<int64_t> mine(CI_WORDS, 0), all((size_t)N * CI_WORDS, 0);
  mine[CI_MODE] = local;
  mine[CI_KEYS] = local == PGPU_COMBINE_ALL_REDUCE || local == PGPU_COMBINE_REDUCE_SCATTER ? P->num_keys : 0;
  mine[CI_SLOTS] = (int64_t)K->slot_kind.size();
  mine[CI_DIGEST] = (int64_t)key_space_digest(K, local != PGPU_COMBINE_ROWS);
  for (size_t s = 0; s < K->slot_kind.size() && s < (size_t)kMaxSlots; ++s) mine[CI_KINDS + s] = K->slot_kind[s];
  {
    DeviceGuard g(c->impl->device);
    TRY(c->impl->allgather_host(mine.data(), mine.size() * 8, all.data()));
  }
  bool same = true, any_rows = false;
  for (int r = 0; r < N; ++r) {
    const int64_t* w = all.data() + (size_t)r * CI_WORDS;
    same &= w[CI_MODE] == local && w[CI_KEYS] == mine[CI_KEYS];
    any_rows |= w[CI_MODE] == PGPU_COMBINE_ROWS;
  }
  const int agreed = same ? local : PGPU_COMBINE_ROWS;  // rows merge any plan kind
  // the key spaces must match: the row and table digests both carry the group-by dictionaries
  for (int r = 0; r < N; ++r) {
    const int64_t* w = all.data() + (size_t)r * CI_WORDS;
    if (w[CI_SLOTS] != mine[CI_SLOTS])
      return fail(PGPU_ERR_INVALID_ARGUMENT, "ranks disagree on the number of accumulators (%lld, %lld)",
                  (long long)w[CI_SLOTS], (long long)mine[CI_SLOTS]);
    if (same && w[CI_DIGEST] != mine[CI_DIGEST])
      return fail(PGPU_ERR_INVALID_ARGUMENT, "rank %d's group-key space differs from rank %d's: union the group-by "
                  "dictionaries (pgpu_table_add_dictionary_values) before the query", r, c->impl->rank);
  }
  (void)any_rows;
  if (!same) {
    // plans of different kinds meet as rows; their dictionaries must still agree
    std::vector<int64_t> d(1, (int64_t)key_space_digest(K, false)), alld(N);
    DeviceGuard g(c->impl->device);
    TRY(c->impl->allgather_host(d.data(), 8, alld.data()));
    for (int r = 0; r < N; ++r)
      if (alld[r] != d[0])
        return fail(PGPU_ERR_INVALID_ARGUMENT, "rank %d's group-by dictionaries differ from rank %d's: union them "
                    "(pgpu_table_add_dictionary_values) before the query", r, c->impl->rank);
  }
  if (kinds) TRY(agree_kinds(all, N, (int)mine[CI_SLOTS], kinds));
  *mode = agreed;
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_combine(pgpu_plan P, pgpu_comm c, void* stream, void* d_table, int32_t mode, const int32_t* kinds,
                      void* d_shard, int64_t* key_begin, int64_t* key_count) try {
  PGPU_ABI_GUARD;
  if (!P || !c) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  if (mode == PGPU_COMBINE_LOCAL) {
    if (key_begin) *key_begin = 0;
    if (key_count) *key_count = P->num_keys;
    return 0;
  }
  if (mode == PGPU_COMBINE_ROWS)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "PGPU_COMBINE_ROWS: finalize the plan, then pgpu_result_combine_rows");
  if (mode != PGPU_COMBINE_ALL_REDUCE && mode != PGPU_COMBINE_REDUCE_SCATTER && mode != PGPU_COMBINE_HASH)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "combine mode %d", mode);
  pgpu::Comm* C = c->impl.get();
  const int N = C->nranks, me = C->rank;
  // the query's deadline and cancel flag bound every wait on the peers below (and finalize's, via comm_used)
  pgpu::CommWaitScope wait_limits(P->end_time_ms, &P->cancel);
  TRY(C->usable());
  // This rank's own checks.  In HASH mode their outcome travels with the per-owner counts (the first host exchange),
  // so a rank that fails here still meets its peers there and every rank fails together.  The dense modes have no
  // host exchange (one would cost every query a round trip): a failed rank issues no collective, its peers' ones stay
  // pending on their streams, and their finalize waits end at the query deadline or the communicator's timeout,
  // which aborts the communicator.
  uint32_t conv = 0;
  int pre = 0;
  if (P->composite) pre = fail(PGPU_ERR_UNSUPPORTED, "numGroupsLimit plan: combine its finalized rows (ROWS)");
  else if (!P->executed || !P->scratch) pre = fail(PGPU_ERR_INVALID_ARGUMENT, "plan not executed");
  else if (P->shard) pre = fail(PGPU_ERR_INVALID_ARGUMENT, "plan already combined");
  else if (C->device != P->table->device)
    pre = fail(PGPU_ERR_INVALID_ARGUMENT, "communicator on device %d, table on %d", C->device, P->table->device);
  else if (mode == PGPU_COMBINE_HASH && !P->hash)
    pre = fail(PGPU_ERR_UNSUPPORTED, "dense group tables merge element-wise (ALL_REDUCE / REDUCE_SCATTER)");
  else if (mode != PGPU_COMBINE_HASH && P->hash)
    pre = fail(PGPU_ERR_UNSUPPORTED, "hash-mode tables merge with PGPU_COMBINE_HASH");
  if (!pre) pre = check_kinds(P->slot_kind, kinds, &conv);
  if (mode != PGPU_COMBINE_HASH && pre) return pre;
  DeviceGuard g(P->table->device);
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : P->table->stream;
  Scratch* sc = P->scratch;
  const int ns = (int)P->slot_kind.size();
  if (mode == PGPU_COMBINE_HASH) {
    // per rank: [status, count for owner 0, ..., count for owner N-1]
    std::vector<int64_t> counts(N + 1, 0), all((size_t)N * (N + 1)), rcount(N);
    if (!pre) pre = pgpu_plan_exchange_counts(P, s, N, counts.data() + 1);
    counts[0] = pre;
    TRY(agree_status_with(C, pre, counts.data(), (size_t)(N + 1) * 8, all.data()));
    int64_t total = 0, nrecv = 0;
    for (int p = 0; p < N; ++p) {
      total += counts[1 + p];
      rcount[p] = all[(size_t)p * (N + 1) + 1 + me];
      nrecv += rcount[p];
    }
    const size_t rec = (size_t)(1 + ns) * 8;
    int rc = sc->xsend.ensure((size_t)std::max<int64_t>(total, 1) * rec);
    if (!rc) rc = pgpu_plan_exchange_export(P, s, N, kinds, sc->xsend.p, total);
    if (!rc) rc = sc->xrecv.ensure((size_t)std::max<int64_t>(nrecv, 1) * rec);
    TRY(agree_status(C, rc));  // before the all-to-all: every rank has its records and room for its peers'
    P->comm_used = c->impl;
    TRY(C->alltoallv(sc->xsend.p, counts.data() + 1, sc->xrecv.p, rcount.data(), rec, s));
    TRY(pgpu_plan_exchange_merge(P, s, kinds, nrecv ? sc->xrecv.p : nullptr, nrecv));
    if (key_begin) *key_begin = 0;
    if (key_count) *key_count = P->num_keys;
    return 0;
  }
  uint64_t* table = reinterpret_cast<uint64_t*>(d_table ? d_table : const_cast<void*>(P->d_table_used));
  if (!table) return fail(PGPU_ERR_INVALID_ARGUMENT, "no group table");
  const int64_t G = P->num_keys;
  for (int k = 0; k < ns; ++k)
    if ((conv >> k) & 1u)
      if (launch_i64_to_f64(table + (size_t)k * G, G, s))
        return fail(PGPU_ERR_DEVICE, "slot conversion launch failed: %s", hipGetErrorString(hipGetLastError()));
  if (kinds && !std::equal(P->slot_kind.begin(), P->slot_kind.end(), kinds)) {
    if (P->slot_kind_planned.empty()) P->slot_kind_planned = P->slot_kind;  // restored when executed again
    P->slot_kind.assign(kinds, kinds + ns);
  }
  P->comm_used = c->impl;
  auto dtype = [&](int k) { return P->slot_kind[k] == SLOT_SUM_F64 ? pgpu::CDT_F64 : pgpu::CDT_I64; };
  auto op = [&](int k) {
    return P->slot_kind[k] == SLOT_MIN_KEY ? pgpu::COP_MIN : P->slot_kind[k] == SLOT_MAX_KEY ? pgpu::COP_MAX : pgpu::COP_SUM;
  };
  if (mode == PGPU_COMBINE_ALL_REDUCE) {
    // consecutive rows of one element type and op in one collective
    for (int k0 = 0; k0 < ns;) {
      int k1 = k0 + 1;
      while (k1 < ns && dtype(k1) == dtype(k0) && op(k1) == op(k0)) ++k1;
      TRY(C->allreduce(table + (size_t)k0 * G, (size_t)(k1 - k0) * G, dtype(k0), op(k0), s));
      k0 = k1;
    }
    if (key_begin) *key_begin = 0;
    if (key_count) *key_count = G;
    return 0;
  }
  // REDUCE_SCATTER: rank r keeps keys [r*chunk, (r+1)*chunk) -- half an all-reduce's link bytes, 1/N of the finalize
  const int64_t chunk = (G + N - 1) / N;
  const int64_t begin = std::min<int64_t>(G, (int64_t)me * chunk);
  const int64_t count = std::min<int64_t>(G, begin + chunk) - begin;
  uint64_t* shard = reinterpret_cast<uint64_t*>(d_shard);
  if (!shard) {
    TRY(sc->xshard.ensure((size_t)ns * std::max<int64_t>(chunk, 1) * 8 + 64));
    shard = sc->xshard.as<uint64_t>();
  }
  if (G % N == 0) {
    for (int k = 0; k < ns; ++k)
      TRY(C->reduce_scatter(table + (size_t)k * G, shard + (size_t)k * chunk, (size_t)chunk, dtype(k), op(k), s));
  } else {
    // rows padded to N x chunk (the padded keys have COUNT 0 and are never finalized), then the rank's rows moved
    // to a count-word stride
    TRY(sc->xsend.ensure((size_t)ns * N * chunk * 8));
    TRY(sc->xrecv.ensure((size_t)ns * chunk * 8));
    uint64_t* pad = sc->xsend.as<uint64_t>();
    uint64_t* part = sc->xrecv.as<uint64_t>();
    HIP_TRY(hipMemsetAsync(pad, 0, (size_t)ns * N * chunk * 8, s));
    HIP_TRY(hipMemcpy2DAsync(pad, (size_t)N * chunk * 8, table, (size_t)G * 8, (size_t)G * 8, (size_t)ns,
                             hipMemcpyDeviceToDevice, s));
    for (int k = 0; k < ns; ++k)
      TRY(C->reduce_scatter(pad + (size_t)k * N * chunk, part + (size_t)k * chunk, (size_t)chunk, dtype(k), op(k), s));
    if (count > 0)
      HIP_TRY(hipMemcpy2DAsync(shard, (size_t)count * 8, part, (size_t)chunk * 8, (size_t)count * 8, (size_t)ns,
                               hipMemcpyDeviceToDevice, s));
  }
  P->shard = shard;
  P->shard_begin = begin;
  P->shard_count = count;
  if (key_begin) *key_begin = begin;
  if (key_count) *key_count = count;
  return 0;
} PGPU_ABI_CATCH

int pgpu_result_combine_rows(pgpu_result r, pgpu_comm c, pgpu_result* out) try {
  PGPU_ABI_GUARD;
  if (!r || !c || !out) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  pgpu::Comm* C = c->impl.get();
  const int N = C->nranks, me = C->rank;
  TRY(C->usable());
  // a rank whose own steps fail still meets its peers in the next exchange (its status word first), so every rank
  // fails together
  int pre = 0;
  if ((int)r->slot_kind.size() != r->num_slots) pre = fail(PGPU_ERR_UNSUPPORTED, "result without slot kinds");
  else if (r->compact.load(std::memory_order_acquire)) pre = pgpu::result_expand(r);
  // agree on the slot kinds; the group ids index the ranks' dictionary snapshots, which must be the same
  std::vector<int64_t> mine(CI_WORDS, 0), all((size_t)N * CI_WORDS, 0);
  uint64_t h = 0x84222325cbf29ce4ull;
  auto mix = [&h](uint64_t v) { h = (h ^ v) * 0x9E3779B97F4A7C15ull; h ^= h >> 29; };
  mix(r->key_dicts.size());
  for (const auto& d : r->key_dicts) mix(d ? dict_digest(*static_cast<const Dict*>(d.get())) : 0);
  mine[CI_KEYS] = r->num_keys;
  mine[CI_SLOTS] = r->num_slots;
  mine[CI_DIGEST] = (int64_t)h;
  for (int s = 0; s < r->num_slots && s < kMaxSlots && s < (int)r->slot_kind.size(); ++s)
    mine[CI_KINDS + s] = r->slot_kind[s];
  mine[CI_MODE] = pre;  // the status word
  DeviceGuard g(C->device);
  TRY(agree_status_with(C, pre, mine.data(), mine.size() * 8, all.data()));
  for (int p = 0; p < N; ++p) {
    const int64_t* w = all.data() + (size_t)p * CI_WORDS;
    if (w[CI_KEYS] != mine[CI_KEYS] || w[CI_SLOTS] != mine[CI_SLOTS])
      return fail(PGPU_ERR_INVALID_ARGUMENT, "rank %d's result has another shape", p);
    if (w[CI_DIGEST] != mine[CI_DIGEST])
      return fail(PGPU_ERR_INVALID_ARGUMENT, "rank %d's group-by dictionaries differ from rank %d's: union them "
                  "(pgpu_table_add_dictionary_values) before the query", p, me);
  }
  std::vector<int32_t> kinds(std::max(r->num_slots, 1));
  TRY(agree_kinds(all, N, r->num_slots, kinds.data()));
  const int w = r->num_keys + r->num_slots;
  // per rank: [status, rows for owner 0, ..., rows for owner N-1]
  std::vector<int64_t> rows((size_t)std::max<int64_t>(r->n, 1) * w), counts(N + 1, 0), cm((size_t)N * (N + 1)),
      rcount(N);
  const int rc = pgpu_result_exchange_rows(r, N, kinds.data(), rows.data(), counts.data() + 1);
  counts[0] = rc;
  TRY(agree_status_with(C, rc, counts.data(), (size_t)(N + 1) * 8, cm.data()));
  int64_t nrecv = 0;
  for (int p = 0; p < N; ++p) nrecv += rcount[p] = cm[(size_t)p * (N + 1) + 1 + me];
  std::vector<int64_t> recv((size_t)std::max<int64_t>(nrecv, 1) * w);
  TRY(C->alltoallv_host(rows.data(), counts.data() + 1, recv.data(), rcount.data(), (size_t)w * 8));
  return pgpu_result_merge_rows(r, nrecv ? recv.data() : nullptr, nrecv, kinds.data(), out);
} PGPU_ABI_CATCH

int pgpu_execute_groupby(pgpu_table t, const int64_t* handles, int32_t nsegs, const pgpu_query* q, void* stream,
                         pgpu_result* out) try {
  PGPU_ABI_GUARD;
  pgpu_plan P = nullptr;
  TRY(pgpu_plan_create_execute(t, handles, nsegs, q, stream, nullptr, &P));
  int rc = pgpu_plan_finalize(P, stream, nullptr, out);
  std::string keep = g_err;
  pgpu_plan_destroy(P);
  g_err = keep;
  return rc;
} PGPU_ABI_CATCH

int pgpu_plan_scanned_segments(pgpu_plan P, uint8_t* out) try {
  PGPU_ABI_GUARD;
  if (!P || !out) return fail(PGPU_ERR_INVALID_ARGUMENT, "null argument");
  if (!P->seg_scanned.empty()) memcpy(out, P->seg_scanned.data(), P->seg_scanned.size());
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_star_work(pgpu_plan P, int64_t* out3) try {
  PGPU_ABI_GUARD;
  if (!P || !out3) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  int64_t nodes = 0;
  for (const KStarSeg& k : P->star) nodes += k.num_nodes;
  out3[0] = (int64_t)P->star.size();
  out3[1] = nodes;
  out3[2] = P->star_docs_read;
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_timing(pgpu_plan P, double* out3) try {
  PGPU_ABI_GUARD;
  if (!P || !out3 || !P->executed) return fail(PGPU_ERR_INVALID_ARGUMENT, "plan not executed");
  if (P->composite) return fail(PGPU_ERR_UNSUPPORTED, "numGroupsLimit plan: timing is per part");
  Scratch* sc = P->scratch;
#ifdef PGPU_NO_TIMING_EVENTS
  for (int i = 0; i < 4; ++i) out3[i] = i == 2 ? (double)P->launches_done : 0.0;
  return 0;
#endif
  HIP_TRY(hipEventSynchronize(sc->ev[3]));
  float a = 0;
  HIP_TRY(hipEventElapsedTime(&a, sc->ev[0], sc->ev[3]));
  double k = 0;
  for (int c = 0; c < P->launches_done; ++c) {  // scan launches only (no host gaps between streamed launches)
    float b = 0;
    HIP_TRY(hipEventElapsedTime(&b, sc->cev[2 * c], sc->cev[2 * c + 1]));
    k += b;
  }
  float st = 0;
  if (!P->star.empty()) HIP_TRY(hipEventElapsedTime(&st, sc->ev[1], sc->ev[2]));
  out3[0] = a * 1000.0;
  out3[1] = k * 1000.0;
  out3[2] = P->num_tiles > 0 ? (double)P->launches_done : 0.0;
  out3[3] = st * 1000.0;
  return 0;
} PGPU_ABI_CATCH

int pgpu_result_num_groups(pgpu_result r, int64_t* n) try {
  PGPU_ABI_GUARD;
  if (!r || !n) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  *n = r->n;
  return 0;
} PGPU_ABI_CATCH
static const Dict* result_dict(pgpu_result r, int key) {
  if (!r || key < 0 || key >= r->num_keys || key >= (int)r->key_dicts.size() || !r->key_dicts[key]) return nullptr;
  return static_cast<const Dict*>(r->key_dicts[key].get());
}
int pgpu_result_key_dictionary(pgpu_result r, int key, uint64_t* snapshot_id, int64_t* size) try {
  PGPU_ABI_GUARD;
  const Dict* d = result_dict(r, key);
  if (!d) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad group-by key %d", key);
  if (snapshot_id) *snapshot_id = d->id;
  if (size) *size = (int64_t)d->size();
  return 0;
} PGPU_ABI_CATCH
int pgpu_result_key_dictionary_i64(pgpu_result r, int key, int64_t* out) try {
  PGPU_ABI_GUARD;
  const Dict* d = result_dict(r, key);
  if (!d || !out || !is_int_type(d->type)) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  std::copy(d->iv.begin(), d->iv.end(), out);
  return 0;
} PGPU_ABI_CATCH
int pgpu_result_key_dictionary_f64(pgpu_result r, int key, double* out) try {
  PGPU_ABI_GUARD;
  const Dict* d = result_dict(r, key);
  if (!d || !out || !is_fp_type(d->type)) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  std::copy(d->dv.begin(), d->dv.end(), out);
  return 0;
} PGPU_ABI_CATCH
int pgpu_result_key_dictionary_str(pgpu_result r, int key, uint8_t* blob, int64_t cap, int64_t* offsets) try {
  PGPU_ABI_GUARD;
  const Dict* d = result_dict(r, key);
  if (!d || !offsets || d->type != PGPU_STRING) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  int64_t off = 0;
  offsets[0] = 0;
  for (size_t i = 0; i < d->sv.size(); ++i) {
    if (blob) {
      if (off + (int64_t)d->sv[i].size() > cap) return fail(PGPU_ERR_INVALID_ARGUMENT, "blob too small");
      memcpy(blob + off, d->sv[i].data(), d->sv[i].size());
    }
    off += (int64_t)d->sv[i].size();
    offsets[i + 1] = off;
  }
  return 0;
} PGPU_ABI_CATCH
int pgpu_result_group_ids(pgpu_result r, int32_t* out) try {
  PGPU_ABI_GUARD;
  if (!r || (!out && r->n)) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  if (r->compact.load(std::memory_order_acquire)) TRY(pgpu::result_expand(r));  // compact: columnar form first
  const int nk = r->num_keys;
  for (int j = 0; j < nk; ++j) {
    const int32_t* g = r->gid(j);
    for (int64_t i = 0; i < r->n; ++i) out[i * nk + j] = g[i];
  }
  return 0;
} PGPU_ABI_CATCH
int pgpu_result_group_ids_column(pgpu_result r, int key, int32_t* out) try {
  PGPU_ABI_GUARD;
  if (!r || key < 0 || key >= r->num_keys || (!out && r->n)) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  if (r->compact.load(std::memory_order_acquire)) TRY(pgpu::result_expand(r));  // compact: columnar form first
  if (r->n) memcpy(out, r->gid(key), (size_t)r->n * 4);
  return 0;
} PGPU_ABI_CATCH
int pgpu_result_group_ids_view(pgpu_result r, int key, const int32_t** out) try {
  PGPU_ABI_GUARD;
  if (!r || key < 0 || key >= r->num_keys || !out) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  if (r->compact.load(std::memory_order_acquire)) TRY(pgpu::result_expand(r));  // compact: columnar form first
  *out = r->gid(key);
  return 0;
} PGPU_ABI_CATCH
int pgpu_result_words_view(pgpu_result r, int agg, const uint64_t** out, int32_t* form) try {
  PGPU_ABI_GUARD;
  if (!r || agg < -1 || agg >= r->num_aggs || !out || !form) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  if (r->compact.load(std::memory_order_acquire)) TRY(pgpu::result_expand(r));  // compact: columnar form first
  if (agg == -1) {  // the COUNT slot (AvgPair.count of every AVG)
    *out = r->slot(0);
    *form = RCONV_I64;
    return 0;
  }
  *out = r->slot(r->agg_slot[agg]);
  *form = r->agg_conv[agg];
  return 0;
} PGPU_ABI_CATCH
int pgpu_result_values(pgpu_result r, int agg, double* out) try {
  PGPU_ABI_GUARD;
  if (!r || agg < 0 || agg >= r->num_aggs || (!out && r->n)) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  if (r->compact.load(std::memory_order_acquire)) TRY(pgpu::result_expand(r));  // compact: columnar form first
  const uint64_t* w = r->slot(r->agg_slot[agg]);
  switch (r->agg_conv[agg]) {
    case RCONV_I64: for (int64_t i = 0; i < r->n; ++i) out[i] = (double)(int64_t)w[i]; break;
    case RCONV_F64: if (r->n) memcpy(out, w, (size_t)r->n * 8); break;
    default: for (int64_t i = 0; i < r->n; ++i) out[i] = key_double((int64_t)w[i]); break;
  }
  return 0;
} PGPU_ABI_CATCH
int pgpu_result_avg_counts(pgpu_result r, int agg, int64_t* out) try {
  PGPU_ABI_GUARD;
  if (!r || agg < 0 || agg >= r->num_aggs || (!out && r->n)) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  if (r->compact.load(std::memory_order_acquire)) TRY(pgpu::result_expand(r));  // compact: columnar form first
  if (r->n) memcpy(out, r->slot(0), (size_t)r->n * 8);  // slot 0 = COUNT = AvgPair.count
  return 0;
} PGPU_ABI_CATCH
int pgpu_result_values_i64(pgpu_result r, int agg, int64_t* out) try {
  PGPU_ABI_GUARD;
  if (!r || agg < 0 || agg >= r->num_aggs || (!out && r->n)) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  if (r->compact.load(std::memory_order_acquire)) TRY(pgpu::result_expand(r));  // compact: columnar form first
  if (r->agg_conv[agg] != RCONV_I64) return fail(PGPU_ERR_INVALID_ARGUMENT, "aggregation %d is floating point", agg);
  if (r->n) memcpy(out, r->slot(r->agg_slot[agg]), (size_t)r->n * 8);
  return 0;
} PGPU_ABI_CATCH
int pgpu_result_stats(pgpu_result r, int64_t* out6) try {
  PGPU_ABI_GUARD;
  if (!r || !out6) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  memcpy(out6, r->stats, sizeof r->stats);
  return 0;
} PGPU_ABI_CATCH
int pgpu_result_groups_limit_reached(pgpu_result r, int32_t* out) try {
  PGPU_ABI_GUARD;
  if (!r || !out) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  *out = r->groups_limit_reached ? 1 : 0;
  return 0;
} PGPU_ABI_CATCH
int pgpu_result_destroy(pgpu_result r) try {
  PGPU_ABI_GUARD;
  delete r;
  return 0;
} PGPU_ABI_CATCH
int pgpu_free_result(pgpu_result r) { return pgpu_result_destroy(r); }

int pgpu_filter_bitmap(pgpu_table t, int64_t h, const pgpu_query* q, uint64_t* out_words) try {
  PGPU_ABI_GUARD;
  if (!t || !q || !out_words) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  DeviceGuard g(t->device);
  // A plan over the one segment with a COUNT-by-first-column shape; only its filter part is used.
  pgpu_query fq = *q;
  int32_t gb = q->num_group_by > 0 ? q->group_by[0] : 0;
  fq.num_group_by = 1;
  fq.group_by = &gb;
  fq.num_aggs = 0;
  fq.aggs = nullptr;
  auto P = std::make_unique<pgpu_plan_s>();
  P->no_inverted = true;  // the standalone filter kernel reads scan / sorted / raw-value leaves only
  TRY(plan_create_impl(t, &h, 1, &fq, P.get()));
  Segment* s = P->segs[0];
  const int64_t ngroups = ((int64_t)s->num_docs + 31) / 32;
  const int64_t nwords = ((int64_t)s->num_docs + 63) / 64;
  if (P->segrec.empty()) {  // filter folded to EmptyFilterOperator
    memset(out_words, 0, (size_t)nwords * 8);
    return 0;
  }
  Scratch* sc = acquire_scratch(t);
  int rc = 0;
  do {
    if ((rc = sc->segrec.ensure(P->segrec.size()))) break;
    if ((rc = sc->sets.ensure(std::max<size_t>(P->set_words.size() * 4, 16)))) break;
    for (auto& f : P->set_fix) {
      const uint32_t* p = sc->sets.as<uint32_t>() + f.second;
      memcpy(P->segrec.data() + f.first, &p, sizeof p);
    }
    if (!P->raw_tasks.empty()) {  // raw-value leaves: their docbits regions first (inverted leaves are off here)
      if ((rc = sc->docbits.ensure((size_t)P->docbit_words * 4))) break;
      for (auto& f : P->bit_fix) {
        const uint32_t* p = sc->docbits.as<uint32_t>() + f.second;
        memcpy(P->segrec.data() + f.first, &p, sizeof p);
      }
      if ((rc = launch_raw_leaves(P.get(), sc, t->stream))) break;
    }
    if ((rc = sc->bitmap.ensure((size_t)nwords * 8))) break;
    hipMemsetAsync(sc->bitmap.p, 0, (size_t)nwords * 8, t->stream);
    hipMemcpyAsync(sc->segrec.p, P->segrec.data(), P->segrec.size(), hipMemcpyHostToDevice, t->stream);
    if (!P->set_words.empty())
      hipMemcpyAsync(sc->sets.p, P->set_words.data(), P->set_words.size() * 4, hipMemcpyHostToDevice, t->stream);
    KParams kp;
    memset(&kp, 0, sizeof kp);
    kp.pack_slot = -1;
    kp.segs = sc->segrec.as<uint8_t>();
    kp.seg_stride = P->seg_stride;
    kp.num_cols = (int)P->query_cols.size();
    kp.num_segs = 1;
    kp.num_tiles = (int32_t)((ngroups + kBlock - 1) / kBlock);
    kp.num_ops = (int)P->ops.size();
    kp.pure_and = P->pure_and;
    for (size_t i = 0; i < P->ops.size(); ++i) kp.ops[i] = P->ops[i];
    kp.num_leaves = P->num_leaves;
    for (int i = 0; i < P->num_leaves; ++i) kp.leaf_col[i] = P->leaf_slot[i];
    if (launch_filter_bitmap(kp, sc->bitmap.as<uint32_t>(), t->stream)) {
      rc = fail(PGPU_ERR_DEVICE, "filter bitmap launch failed");
      break;
    }
    hipError_t e = hipMemcpyAsync(out_words, sc->bitmap.p, (size_t)nwords * 8, hipMemcpyDeviceToHost, t->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(t->stream);
    if (e != hipSuccess) rc = fail(PGPU_ERR_DEVICE, "filter bitmap: %s", hipGetErrorString(e));
  } while (0);
  release_scratch(t, sc);
  return rc;
} PGPU_ABI_CATCH

int pgpu_generate_segment(pgpu_table t, const pgpu_gen_column* gc, int32_t ncols, int64_t row0, int32_t num_docs,
                          int64_t* handle) try {
  PGPU_ABI_GUARD;
  if (!t || !gc || !handle || ncols != (int)t->names.size() || num_docs < 0)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  DeviceGuard g(t->device);
  hipStream_t st = t->stream;
  auto seg = std::make_unique<Segment>();
  seg->num_docs = num_docs;
  seg->cols.resize(ncols);
  // Domain of each column in value order: positions; the dictionary is the set of positions present.
  struct Domain {
    std::vector<int32_t> code_to_pos;
    std::vector<int64_t> pos_i64;
    std::vector<double> pos_f64;
    int64_t npos = 0;
  };
  std::vector<Domain> dom(ncols);
  int64_t total_words = 0;
  for (int c = 0; c < ncols; ++c) {
    const pgpu_gen_column& g0 = gc[c];
    const int type = t->types[c];
    Domain& D = dom[c];
    if (g0.kind == PGPU_GEN_UNIFORM) {
      if (!is_int_type(type) || g0.hi <= g0.lo || g0.hi - g0.lo > (int64_t(1) << 28))
        return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: bad UNIFORM spec", c);
      D.npos = g0.hi - g0.lo;
    } else if (g0.kind == PGPU_GEN_ZIPF) {
      if (!is_int_type(type) || g0.n <= 0 || !g0.cdf || !g0.ids) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad ZIPF spec");
      std::vector<int32_t> order(g0.n);
      for (int i = 0; i < g0.n; ++i) order[i] = i;
      std::sort(order.begin(), order.end(), [&](int a, int b) { return g0.ids[a] < g0.ids[b]; });
      D.code_to_pos.assign(g0.n, 0);
      for (int i = 0; i < g0.n; ++i) {
        if (i > 0 && g0.ids[order[i]] == g0.ids[order[i - 1]]) return fail(PGPU_ERR_INVALID_ARGUMENT, "duplicate ZIPF ids");
        D.code_to_pos[order[i]] = i;
        D.pos_i64.push_back(g0.ids[order[i]]);
      }
      D.npos = g0.n;
    } else if (g0.kind == PGPU_GEN_TABLE) {
      if (!is_fp_type(type) || g0.n <= 0 || !g0.table) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad TABLE spec");
      std::vector<double> vals(g0.table, g0.table + g0.n);
      if (type == PGPU_FLOAT) for (double& v : vals) v = (double)(float)v;
      std::vector<double> sorted = vals;
      std::sort(sorted.begin(), sorted.end(), dbl_less);
      sorted.erase(std::unique(sorted.begin(), sorted.end(),
                               [](double a, double b) { return !dbl_less(a, b) && !dbl_less(b, a); }),
                   sorted.end());
      D.code_to_pos.resize(g0.n);
      for (int i = 0; i < g0.n; ++i)
        D.code_to_pos[i] = (int32_t)(std::lower_bound(sorted.begin(), sorted.end(), vals[i], dbl_less) - sorted.begin());
      D.pos_f64 = sorted;
      D.npos = (int64_t)sorted.size();
    } else {
      return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: bad generator kind", c);
    }
  }
  // pass 1 per column: positions + presence bitmap
  GenScratch& G = t->gen;
  std::vector<std::vector<int32_t>> pos_to_id(ncols);
  TRY(G.pos.ensure((size_t)std::max(num_docs, 1) * 4 * ncols));
  for (int c = 0; c < ncols; ++c) {
    const pgpu_gen_column& g0 = gc[c];
    Domain& D = dom[c];
    const int64_t pres_words = (D.npos + 31) / 32;
    TRY(G.presence.ensure((size_t)pres_words * 4));
    HIP_TRY(hipMemsetAsync(G.presence.p, 0, (size_t)pres_words * 4, st));
    if (!D.code_to_pos.empty()) {
      TRY(G.code_to_pos.ensure(D.code_to_pos.size() * 4));
      HIP_TRY(hipMemcpyAsync(G.code_to_pos.p, D.code_to_pos.data(), D.code_to_pos.size() * 4, hipMemcpyHostToDevice, st));
    }
    if (g0.kind == PGPU_GEN_ZIPF) {
      TRY(G.cdf.ensure((size_t)g0.n * 8));
      HIP_TRY(hipMemcpyAsync(G.cdf.p, g0.cdf, (size_t)g0.n * 8, hipMemcpyHostToDevice, st));
    }
    const uint64_t seed = (uint64_t)(0x5EED0000u + (uint32_t)g0.column_index) << 32;
    const int32_t ncodes = g0.kind == PGPU_GEN_UNIFORM ? 0 : g0.n;
    if (launch_gen_positions(g0.kind, seed, g0.lo, g0.hi - g0.lo, G.cdf.as<double>(), G.code_to_pos.as<int32_t>(),
                             ncodes, row0, num_docs, G.pos.as<int32_t>() + (size_t)c * std::max(num_docs, 1),
                             G.presence.as<uint32_t>(), st))
      return fail(PGPU_ERR_DEVICE, "gen positions launch failed");
    std::vector<uint32_t> pres(pres_words);
    HIP_TRY(hipMemcpyAsync(pres.data(), G.presence.p, (size_t)pres_words * 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    // dictionary = present positions in value order (SegmentDictionaryCreator: sorted distinct values)
    Column& col = seg->cols[c];
    col.dict.type = t->types[c];
    std::vector<int32_t>& p2i = pos_to_id[c];
    p2i.assign(std::max<int64_t>(D.npos, 1), 0);
    int32_t card = 0;
    for (int64_t p = 0; p < D.npos; ++p)
      if ((pres[p >> 5] >> (p & 31)) & 1u) {
        p2i[p] = card++;
        if (g0.kind == PGPU_GEN_UNIFORM) col.dict.iv.push_back(g0.lo + p);
        else if (g0.kind == PGPU_GEN_ZIPF) col.dict.iv.push_back(D.pos_i64[p]);
        else col.dict.dv.push_back(D.pos_f64[p]);
      }
    col.card = card;
    col.bits = num_bits_per_value(card - 1);
    const int type = t->types[c];
    col.entry_width = (type == PGPU_INT || type == PGPU_FLOAT) ? 4 : 8;
    col.raw_dict.assign((size_t)card * col.entry_width, 0);
    for (int32_t i = 0; i < card; ++i) {
      uint8_t* o = col.raw_dict.data() + (size_t)i * col.entry_width;
      if (type == PGPU_INT) wr_be32(o, (uint32_t)(int32_t)col.dict.iv[i]);
      else if (type == PGPU_LONG) wr_be64(o, (uint64_t)col.dict.iv[i]);
      else if (type == PGPU_FLOAT) { float f = (float)col.dict.dv[i]; uint32_t u; memcpy(&u, &f, 4); wr_be32(o, u); }
      else { uint64_t u; memcpy(&u, &col.dict.dv[i], 8); wr_be64(o, u); }
    }
    col.fwd_bytes = ((int64_t)num_docs * col.bits + 7) / 8;
    col.fwd_words = padded_fwd_words(num_docs, col.bits);
    total_words += (col.fwd_words + 63) & ~int64_t(63);
  }
  HIP_TRY(hipMalloc(&seg->d_block, (size_t)std::max<int64_t>(total_words, 64) * 4));
  t->device_bytes += std::max<int64_t>(total_words, 64) * 4;
  HIP_TRY(hipMemsetAsync(seg->d_block, 0, (size_t)std::max<int64_t>(total_words, 64) * 4, st));
  int64_t off = 0;
  for (int c = 0; c < ncols; ++c) {
    Column& col = seg->cols[c];
    col.d_fwd = reinterpret_cast<uint32_t*>(seg->d_block) + off;
    off += (col.fwd_words + 63) & ~int64_t(63);
    TRY(G.pos_to_id.ensure(pos_to_id[c].size() * 4));
    HIP_TRY(hipMemcpyAsync(G.pos_to_id.p, pos_to_id[c].data(), pos_to_id[c].size() * 4, hipMemcpyHostToDevice, st));
    if (launch_gen_pack(G.pos.as<int32_t>() + (size_t)c * std::max(num_docs, 1), G.pos_to_id.as<int32_t>(), num_docs,
                        col.bits, col.d_fwd, st))
      return fail(PGPU_ERR_DEVICE, "gen pack launch failed");
    HIP_TRY(hipStreamSynchronize(st));  // pos_to_id is reused by the next column
  }
  std::lock_guard<std::mutex> lk(t->mu);
  *handle = register_segment(t, std::move(seg));
  return 0;
} PGPU_ABI_CATCH

int pgpu_segment_column_info(pgpu_table t, int64_t h, int col, int32_t* card, int32_t* bits, int64_t* dict_len,
                             int64_t* fwd_len) try {
  PGPU_ABI_GUARD;
  if (!t) return fail(PGPU_ERR_INVALID_ARGUMENT, "null table");
  std::lock_guard<std::mutex> lk(t->mu);
  auto it = t->segments.find(h);
  if (it == t->segments.end()) return fail(PGPU_ERR_NOT_FOUND, "unknown segment handle");
  if (col < 0 || col >= (int)it->second->cols.size()) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad column");
  const Column& c = it->second->cols[col];
  if (card) *card = c.card;
  if (bits) *bits = c.bits;
  if (dict_len) *dict_len = (int64_t)c.raw_dict.size();
  if (fwd_len) *fwd_len = c.fwd_bytes;
  return 0;
} PGPU_ABI_CATCH

int pgpu_segment_column_bytes(pgpu_table t, int64_t h, int col, uint8_t* dict_out, uint8_t* fwd_out) try {
  PGPU_ABI_GUARD;
  if (!t) return fail(PGPU_ERR_INVALID_ARGUMENT, "null table");
  DeviceGuard g(t->device);
  std::shared_ptr<Segment> s;
  {
    std::lock_guard<std::mutex> lk(t->mu);
    auto it = t->segments.find(h);
    if (it == t->segments.end()) return fail(PGPU_ERR_NOT_FOUND, "unknown segment handle");
    s = it->second;
  }
  if (col < 0 || col >= (int)s->cols.size()) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad column");
  const Column& c = s->cols[col];
  if (dict_out && !c.raw_dict.empty()) memcpy(dict_out, c.raw_dict.data(), c.raw_dict.size());
  if (fwd_out && c.fwd_bytes > 0) {
    HIP_TRY(hipMemcpyAsync(fwd_out, c.d_fwd, (size_t)c.fwd_bytes, hipMemcpyDeviceToHost, t->stream));
    HIP_TRY(hipStreamSynchronize(t->stream));
  }
  return 0;
} PGPU_ABI_CATCH

}  // extern "C"
