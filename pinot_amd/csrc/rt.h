// rt.h -- the host runtime's model (tables, pinned segments, dictionaries, plans, scratch) and the functions
// its sources share: rt_core.cpp (errors, diagnostics), rt_dict.cpp (dictionaries), rt_plan.cpp (planning),
// rt_exec.cpp (execution, finalize), rt_groups.cpp (numGroupsLimit split, plan cache) and the C ABI in
// abi_table.cpp / abi_plan.cpp / abi_combine.cpp / abi_result.cpp.  Not part of the ABI.
#pragma once
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



namespace pgpu {

// ---- errors and diagnostics (rt_core.cpp)
bool diag(const char* word);
void install_crash_trace();
extern thread_local std::string g_err;
bool trace_on();
double now_us();
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));


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

// The execution's timing events (pgpu_plan_timing), recorded only when the query asked for them (PGPU_OPT_TIMING):
// each event is a marker packet between two dependent dispatches of the stream.
#define PGPU_TIMING_RECORD(P, ev, stream)                   \
  do {                                                      \
    if ((P)->timed) HIP_TRY(hipEventRecord(ev, stream));    \
  } while (0)

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

inline HostPool& host_pool() {
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
inline int stream_chunk_count(const pgpu_config& cfg, size_t nseg) {
  if (cfg.stream_chunks > 1) return std::min<int>(cfg.stream_chunks, (int)std::max<size_t>(nseg, 1));
  return 1;
}

inline size_t plan_chunk_segs(const pgpu_config& cfg) {
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
inline const double kCanonicalNaN = [] {
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
// A dense-mode combine has no status exchange: a peer that failed its own checks never joins the collectives.  The
// finalize of a query without a deadline waits at most this long for them (then aborts the communicator), instead of
// the communicator's whole timeout.
constexpr int64_t kDenseCombineWaitMs = 30 * 1000;
constexpr int64_t kExportBytes = 64 * 1024;  // LDS-table plans up to this size: the epilogue writes them to host memory
constexpr int64_t kPartMinBytes = 32ll << 20;        // dense tables this large use the partitioned group-by
#ifndef PGPU_PART_LDS_KB
#define PGPU_PART_LDS_KB 64
#endif
constexpr int64_t kPartLds = PGPU_PART_LDS_KB * 1024;  // K8d accumulators per partition (LDS)
constexpr int64_t kMaxParts = 16384;                 // K8a/K8c LDS histogram entries
constexpr int64_t kHashPartLdsMax = 64 * 1024;       // K8h LDS hash table per partition, at most
constexpr int64_t kPartMaxRecordBytes = 32ll << 30;  // scratch for the partitioned records
constexpr int kDocIdColumn = -2;                     // query column of the virtual $docId (hidden first-doc slot)

inline bool is_int_type(int t) { return t == PGPU_INT || t == PGPU_LONG; }
inline bool is_fp_type(int t) { return t == PGPU_FLOAT || t == PGPU_DOUBLE; }

// PinotDataBitSet.getNumBitsPerValue (seglocal/io/util/PinotDataBitSet.java:59-70): bit length, at least 1.
inline int num_bits_per_value(int max_value) {
  if (max_value <= 1) return 1;
  int n = 0;
  while (max_value) { n++; max_value >>= 1; }
  return n;
}

// Strict decimal conversion of Integer.parseInt / Long.parseLong.
inline bool parse_long(const char* s, int64_t lo, int64_t hi, int64_t* out) {
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
inline bool parse_double(const char* s, double* out) {
  char* end = nullptr;
  errno = 0;
  double d = strtod(s, &end);
  if (end == s) return false;
  while (*end == 'd' || *end == 'D' || *end == 'f' || *end == 'F' || *end == ' ') ++end;
  if (*end) return false;
  *out = d;
  return true;
}

inline int cmp_bytes(const uint8_t* a, size_t na, const uint8_t* b, size_t nb) {
  int c = memcmp(a, b, std::min(na, nb));
  if (c) return c;
  return na < nb ? -1 : (na > nb ? 1 : 0);
}

// ================================================================================================ model
// Host copy of one dictionary (segment-local or table-global), sorted ascending.  A table-global dictionary is an
// immutable snapshot (copy on growth, `id` unique per snapshot): plans and their results keep the snapshot their
// group ids index, so a pin that grows the dictionary while a query runs never re-labels that query's groups.
inline std::atomic<uint64_t> g_dict_ids{1};
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
  // per metric: its device array holds int32 values (every pre-aggregated value an integer of int32 range; the
  // kernel widens them exactly) -- half the bytes per star-tree document
  std::vector<uint8_t> mf_narrow, mc_narrow;
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
  // small LDS-table plans: the epilogue's copy of table + statistics (pinned host) and its block counter
  HostPinned exported;
  DevBuf export_done;
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
                            &mid_key, &mid_val, &leap_maps, &mask_jobs, &leaf_masks, &hsort, &part_mm,
                            &export_done})
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
    exported.release(); export_done.release();
    for (auto& e : ev) if (e) { hipEventDestroy(e); e = nullptr; }
  }
};

struct GenScratch {
  DevBuf pos, presence, code_to_pos, cdf, pos_to_id;
};


}  // namespace pgpu

using namespace pgpu;

// pgpu_config_default: the library's settings (include/pinotgpu.h documents each field).
inline pgpu_config default_config() {
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
  c.slot_weight_step = 0.11;
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
    int64_t n = 0;  // entries of the current arrays (device_bytes holds 16 n for them)
  };
  std::vector<GlobalValues> gvalues;
  hipStream_t stream = nullptr;
  std::vector<std::unique_ptr<Scratch>> scratch_pool;
  GenScratch gen;
  std::shared_ptr<ResultPool> result_pool = std::make_shared<ResultPool>();
  int64_t device_bytes = 0;
  int num_cus = 256;
  // executions launched and not yet seen complete (wait_plan) or destroyed: a launch with none beside it has the CUs
  // to itself (set_slot_weights)
  std::atomic<int> scans_inflight{0};
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


namespace pgpu {
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

}  // namespace pgpu

pgpu_config table_config(const pgpu_table_s* t);

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
  bool timed = false;  // PGPU_OPT_TIMING: the executions record their timing events
  bool inflight_counted = false;  // counted in table->scans_inflight (inflight_begin / inflight_end)
  bool alone = false;             // no other execution of the table was in flight when this one launched
  bool exported = false;          // the last execution's epilogue copied table + statistics to scratch->exported
  bool comm_dense = false;        // combined element-wise (ALL_REDUCE / REDUCE_SCATTER): no host exchange of status
  bool k8d_counts = false;        // K8d wrote the compaction's chunk counts / ranges (KPartParams.chunk_cnt)
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
  int64_t star_metric_bytes = -1;  // K6's metric-array sectors (64 B) holding a matched doc, x 64 (small tables)
  int64_t star_docs_read = 0;                                // star-tree documents K6 read (after finalize)
};

namespace pgpu {

// Dictionaries of at least this many entries are read through the table-global value arrays when their segment's
// dictionary lacks at most kMaxValueGaps of the global values (smaller ones stay L2-resident on their own).
#ifndef PGPU_NO_GLOBAL_VALUES  // (defined only by an A/B build of the library: every segment's own arrays)
constexpr int32_t kGlobalValuesMinCard = 8192;
#else
constexpr int32_t kGlobalValuesMinCard = INT32_MAX;
#endif

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
  bool external = false;  // the caller's device table (pgpu_plan_execute's d_table)
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

constexpr size_t kPlanCacheEntries = 16;

}  // namespace pgpu

namespace pgpu {
// PGPU_TRACE=serialize (diagnostics): every entry point of this file runs under one process-wide lock, so
// concurrent callers are serialised (isolates host-side races from device-side ones).
inline std::recursive_mutex g_abi_mu;
inline bool abi_serialize() {
  static const bool on = diag("serialize");
  return on;
}
struct AbiGuard {
  bool on;
  AbiGuard() : on(abi_serialize()) { if (on) g_abi_mu.lock(); }
  ~AbiGuard() { if (on) g_abi_mu.unlock(); }
};
}  // namespace pgpu
#define PGPU_ABI_GUARD AbiGuard _abi_guard

