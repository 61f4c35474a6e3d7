// comm.cpp — pgpu_comm: RCCL over xGMI (one rank per GPU) and the host shared-memory rehearsal transport (comm.h).
//
// What this replaces: the cross-server half of GroupByCombineOperator / GroupByOrderByCombineOperator
// (pinot-core/.../operator/combine/GroupByCombineOperator.java:113-160, GroupByOrderByCombineOperator.java:170-181)
// runs per GPU of one node here; the per-GPU group tables meet through these collectives (abi_combine.cpp's
// pgpu_plan_combine / pgpu_result_combine_rows).
#include "comm.h"

#include <dlfcn.h>
#include <fcntl.h>
#include <rccl/rccl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "host_common.h"

namespace pgpu {
namespace {

#define CTRY(x)                  \
  do {                           \
    const int _rc = (x);         \
    if (_rc) return _rc;         \
  } while (0)
#define CHIP(x)                                                                                             \
  do {                                                                                                      \
    const hipError_t _e = (x);                                                                              \
    if (_e != hipSuccess) return host_fail(PGPU_ERR_DEVICE, "%s: %s", #x, hipGetErrorString(_e));           \
  } while (0)

// ------------------------------------------------------------------------------------------------- RCCL
// librccl is opened on first use, not linked: the library loads (and its CPU tests run) where RCCL is absent, and a
// process that already holds an RCCL (torch links one, soname librccl.so.1) shares that copy instead of mapping a
// second one.
struct RcclApi {
  bool ok = false;
  std::string err;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*ReduceScatter)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

RcclApi load_rccl() {
  RcclApi a;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    a.err = std::string("librccl.so.1 not found: ") + (dlerror() ? dlerror() : "?");
    return a;
  }
  bool all = true;
  auto sym = [&](auto& fn, const char* name) {
    fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
    if (!fn) {
      all = false;
      a.err += std::string(a.err.empty() ? "" : ", ") + name;
    }
  };
  sym(a.GetUniqueId, "ncclGetUniqueId");
  sym(a.CommInitRank, "ncclCommInitRank");
  sym(a.CommDestroy, "ncclCommDestroy");
  sym(a.CommAbort, "ncclCommAbort");
  sym(a.AllReduce, "ncclAllReduce");
  sym(a.ReduceScatter, "ncclReduceScatter");
  sym(a.AllGather, "ncclAllGather");
  sym(a.Send, "ncclSend");
  sym(a.Recv, "ncclRecv");
  sym(a.GroupStart, "ncclGroupStart");
  sym(a.GroupEnd, "ncclGroupEnd");
  sym(a.GetErrorString, "ncclGetErrorString");
  if (!all) a.err = "librccl lacks " + a.err;
  a.ok = all;
  return a;
}

const RcclApi& rccl() {
  static const RcclApi api = load_rccl();
  return api;
}

#define NTRY(x)                                                                                             \
  do {                                                                                                      \
    const ncclResult_t _r = (x);                                                                            \
    if (_r != ncclSuccess) return host_fail(PGPU_ERR_DEVICE, "%s: %s", #x, rccl().GetErrorString(_r));      \
  } while (0)

ncclDataType_t nccl_type(CommDtype t) { return t == CDT_F64 ? ncclFloat64 : ncclInt64; }
ncclRedOp_t nccl_op(CommOp op) { return op == COP_MIN ? ncclMin : op == COP_MAX ? ncclMax : ncclSum; }

// Polls a stream until its work is done, within the calling thread's wait limits (Comm::wait_expired): a collective
// whose peer never joins it must not block the caller forever.  Spins ~2 ms, then sleeps 20 us between polls.
int poll_stream(const Comm& comm, hipStream_t s) {
  const double t0 = comm_now_us();
  for (int spin = 0;; ++spin) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return 0;
    if (e != hipErrorNotReady) return host_fail(PGPU_ERR_DEVICE, "collective wait failed: %s", hipGetErrorString(e));
    CTRY(comm.wait_expired(t0));
    if ((spin & 63) == 63 && comm_now_us() - t0 > 2000.0) {
      struct timespec ts = {0, 20000};
      nanosleep(&ts, nullptr);
    }
  }
}

struct RcclComm : Comm {
  ncclComm_t c = nullptr;
  std::atomic<bool> c_aborted{false};
  std::mutex mu;
  hipStream_t hs = nullptr;  // host-buffer collectives
  void* stage = nullptr;
  size_t stage_cap = 0;
  // The collectives of one communicator run on the device in the order they were issued, whatever streams the
  // callers use (queries in flight on their own streams): each waits for the previous one's completion event.
  // Issue order is the same on every rank, so no rank can start collective k+1 while a peer is still in k.
  hipEvent_t last = nullptr;
  bool issued = false;
  ~RcclComm() override {
    if (c && !c_aborted.load()) rccl().CommDestroy(c);
    if (stage) hipFree(stage);
    if (last) hipEventDestroy(last);
    if (hs) hipStreamDestroy(hs);
  }
  // Not under `mu`: the thread that gives up may be another query's (wait_plan), while this one is parked in a wait.
  // ncclCommAbort makes the kernels of collectives still waiting on a peer exit; the communicator is unusable after.
  void abort() override {
    if (aborted.exchange(true)) return;
    if (c && rccl().CommAbort && !c_aborted.exchange(true)) rccl().CommAbort(c);
  }
  int before(hipStream_t s) {
    CTRY(usable());
    if (issued) CHIP(hipStreamWaitEvent(s, last, 0));
    return 0;
  }
  // The host-buffer collectives' stream, waited for within the caller's limits; an expired wait aborts.
  int sync_hs() {
    const int rc = poll_stream(*this, hs);
    if (rc == PGPU_ERR_TIMEOUT || rc == PGPU_ERR_CANCELLED) abort();
    return rc;
  }
  int after(hipStream_t s) {
    CHIP(hipEventRecord(last, s));
    issued = true;
    return 0;
  }
  int allreduce(void* d, size_t count, CommDtype t, CommOp op, hipStream_t s) override {
    std::lock_guard<std::mutex> g(mu);
    if (count == 0) return 0;
    CTRY(before(s));
    NTRY(rccl().AllReduce(d, d, count, nccl_type(t), nccl_op(op), c, s));
    return after(s);
  }
  int reduce_scatter(const void* dsend, void* drecv, size_t count, CommDtype t, CommOp op, hipStream_t s) override {
    std::lock_guard<std::mutex> g(mu);
    if (count == 0) return 0;
    CTRY(before(s));
    NTRY(rccl().ReduceScatter(dsend, drecv, count, nccl_type(t), nccl_op(op), c, s));
    return after(s);
  }
  int alltoallv(const void* dsend, const int64_t* scount, void* drecv, const int64_t* rcount, size_t rec,
                hipStream_t s) override {
    std::lock_guard<std::mutex> g(mu);
    CTRY(before(s));
    CTRY(alltoallv_impl(dsend, scount, drecv, rcount, rec, s));
    return after(s);
  }
  int alltoallv_host(const void* send, const int64_t* scount, void* recv, const int64_t* rcount, size_t rec) override {
    std::lock_guard<std::mutex> g(mu);
    CTRY(usable());
    size_t st = 0, rt = 0;
    for (int p = 0; p < nranks; ++p) {
      st += (size_t)scount[p] * rec;
      rt += (size_t)rcount[p] * rec;
    }
    void* d = nullptr;
    CHIP(hipMalloc(&d, std::max<size_t>(st + rt, 64)));
    int rc = 0;
    if (st && hipMemcpyAsync(d, send, st, hipMemcpyHostToDevice, hs) != hipSuccess)
      rc = host_fail(PGPU_ERR_DEVICE, "all-to-all staging upload failed");
    if (!rc) rc = before(hs);
    if (!rc) rc = alltoallv_impl(d, scount, (uint8_t*)d + st, rcount, rec, hs);
    if (!rc) rc = after(hs);
    if (!rc && rt && hipMemcpyAsync(recv, (uint8_t*)d + st, rt, hipMemcpyDeviceToHost, hs) != hipSuccess)
      rc = host_fail(PGPU_ERR_DEVICE, "all-to-all staging download failed");
    if (!rc) rc = sync_hs();
    else if (!aborted.load()) hipStreamSynchronize(hs);  // staging freed below: nothing may still read it
    if (!aborted.load()) hipFree(d);  // (after an abort, queued work may still hold it: leaked, not freed under it)
    return rc;
  }
  int alltoallv_impl(const void* dsend, const int64_t* scount, void* drecv, const int64_t* rcount, size_t rec,
                     hipStream_t s) {
    const size_t words = rec / 8;
    std::vector<size_t> soff(nranks + 1, 0), roff(nranks + 1, 0);
    for (int p = 0; p < nranks; ++p) {
      soff[p + 1] = soff[p] + (size_t)scount[p] * rec;
      roff[p + 1] = roff[p] + (size_t)rcount[p] * rec;
    }
    if (scount[rank] != rcount[rank]) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "self counts differ");
    if (scount[rank] > 0)
      CHIP(hipMemcpyAsync((uint8_t*)drecv + roff[rank], (const uint8_t*)dsend + soff[rank], (size_t)scount[rank] * rec,
                          hipMemcpyDeviceToDevice, s));
    if (nranks == 1) return 0;
    NTRY(rccl().GroupStart());
    int rc = 0;
    for (int p = 0; p < nranks && !rc; ++p) {
      if (p == rank) continue;
      if (scount[p] > 0) {
        const ncclResult_t r = rccl().Send((const uint8_t*)dsend + soff[p], (size_t)scount[p] * words, ncclInt64, p, c, s);
        if (r != ncclSuccess) rc = host_fail(PGPU_ERR_DEVICE, "ncclSend to %d: %s", p, rccl().GetErrorString(r));
      }
      if (!rc && rcount[p] > 0) {
        const ncclResult_t r = rccl().Recv((uint8_t*)drecv + roff[p], (size_t)rcount[p] * words, ncclInt64, p, c, s);
        if (r != ncclSuccess) rc = host_fail(PGPU_ERR_DEVICE, "ncclRecv from %d: %s", p, rccl().GetErrorString(r));
      }
    }
    const ncclResult_t r = rccl().GroupEnd();  // always closes the group, even after a failed enqueue
    if (rc) return rc;
    if (r != ncclSuccess) return host_fail(PGPU_ERR_DEVICE, "ncclGroupEnd: %s", rccl().GetErrorString(r));
    return 0;
  }
  int allgather_host(const void* send, size_t bytes, void* recv) override {
    std::lock_guard<std::mutex> g(mu);
    CTRY(usable());
    if (bytes == 0) return 0;
    const size_t need = bytes * (size_t)nranks;
    if (need > stage_cap) {
      if (stage) CHIP(hipFree(stage));
      stage = nullptr;
      stage_cap = 0;
      CHIP(hipMalloc(&stage, std::max<size_t>(need, 4096)));
      stage_cap = std::max<size_t>(need, 4096);
    }
    uint8_t* mine = (uint8_t*)stage + bytes * (size_t)rank;
    CHIP(hipMemcpyAsync(mine, send, bytes, hipMemcpyHostToDevice, hs));
    CTRY(before(hs));
    NTRY(rccl().AllGather(mine, stage, bytes, ncclInt8, c, hs));  // in place
    CTRY(after(hs));
    CHIP(hipMemcpyAsync(recv, stage, need, hipMemcpyDeviceToHost, hs));
    return sync_hs();
  }
};

// ------------------------------------------------------------------------------------------ host transport
constexpr int kHostMaxRanks = 64;
struct HostCtl {
  struct alignas(64) Slot {
    std::atomic<uint64_t> gen;
  } slot[kHostMaxRanks];
  alignas(64) std::atomic<int32_t> live;  // ranks that joined and have not left: the last one out removes the file
};

struct HostComm : Comm {
  std::string name;  // /dev/shm/<name>.ctl, /dev/shm/<name>.<seq>.<rank>
  HostCtl* ctl = nullptr;
  uint64_t gen = 0, seq = 0;
  std::mutex mu;
  // No barrier on the way out: a peer that already exited (or crashed) must not hold this rank's teardown.  Each rank
  // removes its own files; the last rank out removes the control file.
  ~HostComm() override {
    if (ctl) {
      if (ctl->live.fetch_sub(1) == 1) unlink(("/dev/shm/" + name + ".ctl").c_str());
      munmap(ctl, sizeof(HostCtl));
    }
  }
  int barrier() {
    CTRY(usable());
    ++gen;
    ctl->slot[rank].gen.store(gen, std::memory_order_release);
    const double t0 = comm_now_us();
    for (int r = 0; r < nranks; ++r) {
      int spins = 0;
      while (ctl->slot[r].gen.load(std::memory_order_acquire) < gen) {
        if (++spins > 256) {
          struct timespec ts = {0, 20000};
          nanosleep(&ts, nullptr);
          if (const int rc = wait_expired(t0)) {
            abort();  // this rank's generation is ahead of its peers': later barriers would not pair up
            return rc;
          }
        } else {
          sched_yield();
        }
      }
    }
    return 0;
  }
  // Every rank's bytes, in rank order.
  int exchange(const void* data, size_t bytes, std::vector<std::vector<uint8_t>>* all) {
    ++seq;
    auto path = [&](int r) { return "/dev/shm/" + name + "." + std::to_string(seq) + "." + std::to_string(r); };
    {
      const std::string p = path(rank);
      FILE* f = fopen(p.c_str(), "wb");
      if (!f) return host_fail(PGPU_ERR_DEVICE, "host communicator: cannot write %s", p.c_str());
      const size_t w = bytes ? fwrite(data, 1, bytes, f) : 0;
      if (fclose(f) != 0 || w != bytes) return host_fail(PGPU_ERR_DEVICE, "host communicator: short write %s", p.c_str());
    }
    CTRY(barrier());
    all->assign(nranks, {});
    for (int r = 0; r < nranks; ++r) {
      const std::string p = path(r);
      FILE* f = fopen(p.c_str(), "rb");
      if (!f) return host_fail(PGPU_ERR_DEVICE, "host communicator: cannot read %s", p.c_str());
      fseek(f, 0, SEEK_END);
      const long n = ftell(f);
      fseek(f, 0, SEEK_SET);
      (*all)[r].resize((size_t)std::max<long>(n, 0));
      const size_t got = n > 0 ? fread((*all)[r].data(), 1, (size_t)n, f) : 0;
      fclose(f);
      if ((long)got != std::max<long>(n, 0)) return host_fail(PGPU_ERR_DEVICE, "host communicator: short read %s", p.c_str());
    }
    CTRY(barrier());
    unlink(path(rank).c_str());
    return 0;
  }
  template <class T>
  static void fold(T* acc, const T* v, size_t n, CommOp op) {
    for (size_t i = 0; i < n; ++i) {
      if (op == COP_SUM) acc[i] += v[i];
      else if (op == COP_MIN) acc[i] = std::min(acc[i], v[i]);
      else acc[i] = std::max(acc[i], v[i]);
    }
  }
  // acc (n elements) = reduction over ranks of their block at element offset `off`.
  static void reduce_blocks(const std::vector<std::vector<uint8_t>>& all, size_t off, size_t n, CommDtype t, CommOp op,
                            void* acc) {
    memcpy(acc, all[0].data() + off * 8, n * 8);
    for (size_t r = 1; r < all.size(); ++r) {
      if (t == CDT_F64) fold((double*)acc, (const double*)(all[r].data() + off * 8), n, op);
      else fold((int64_t*)acc, (const int64_t*)(all[r].data() + off * 8), n, op);
    }
  }
  int allreduce(void* d, size_t count, CommDtype t, CommOp op, hipStream_t s) override {
    std::lock_guard<std::mutex> g(mu);
    std::vector<uint8_t> h(count * 8);
    CHIP(hipMemcpyAsync(h.data(), d, count * 8, hipMemcpyDeviceToHost, s));
    CHIP(hipStreamSynchronize(s));
    std::vector<std::vector<uint8_t>> all;
    CTRY(exchange(h.data(), h.size(), &all));
    for (auto& a : all)
      if (a.size() != h.size()) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "all-reduce: ranks' sizes differ");
    reduce_blocks(all, 0, count, t, op, h.data());
    CHIP(hipMemcpyAsync(d, h.data(), count * 8, hipMemcpyHostToDevice, s));
    CHIP(hipStreamSynchronize(s));
    return 0;
  }
  int reduce_scatter(const void* dsend, void* drecv, size_t count, CommDtype t, CommOp op, hipStream_t s) override {
    std::lock_guard<std::mutex> g(mu);
    std::vector<uint8_t> h(count * 8 * (size_t)nranks);
    CHIP(hipMemcpyAsync(h.data(), dsend, h.size(), hipMemcpyDeviceToHost, s));
    CHIP(hipStreamSynchronize(s));
    std::vector<std::vector<uint8_t>> all;
    CTRY(exchange(h.data(), h.size(), &all));
    for (auto& a : all)
      if (a.size() != h.size()) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "reduce-scatter: ranks' sizes differ");
    std::vector<uint8_t> out(count * 8);
    reduce_blocks(all, count * (size_t)rank, count, t, op, out.data());
    CHIP(hipMemcpyAsync(drecv, out.data(), out.size(), hipMemcpyHostToDevice, s));
    CHIP(hipStreamSynchronize(s));
    return 0;
  }
  // rcount[p] records of rank p, back to back in rank order, appended to *out
  int alltoallv_bytes(const uint8_t* send, const int64_t* scount, const int64_t* rcount, size_t rec,
                      std::vector<uint8_t>* out) {
    size_t total = 0;
    for (int p = 0; p < nranks; ++p) total += (size_t)scount[p] * rec;
    // this rank's file: its send counts, then its records
    std::vector<uint8_t> h(sizeof(int64_t) * nranks + total);
    memcpy(h.data(), scount, sizeof(int64_t) * nranks);
    if (total) memcpy(h.data() + sizeof(int64_t) * nranks, send, total);
    std::vector<std::vector<uint8_t>> all;
    CTRY(exchange(h.data(), h.size(), &all));
    for (int p = 0; p < nranks; ++p) {
      const int64_t* pc = reinterpret_cast<const int64_t*>(all[p].data());
      if (all[p].size() < sizeof(int64_t) * nranks || pc[rank] != rcount[p])
        return host_fail(PGPU_ERR_INVALID_ARGUMENT, "all-to-all: rank %d sends %lld records, %lld expected", p,
                         all[p].size() < sizeof(int64_t) * nranks ? -1LL : (long long)pc[rank], (long long)rcount[p]);
      size_t off = sizeof(int64_t) * nranks;
      for (int q = 0; q < rank; ++q) off += (size_t)pc[q] * rec;
      if (off + (size_t)pc[rank] * rec > all[p].size())
        return host_fail(PGPU_ERR_INVALID_ARGUMENT, "all-to-all: rank %d sent a short buffer", p);
      out->insert(out->end(), all[p].begin() + off, all[p].begin() + off + (size_t)pc[rank] * rec);
    }
    return 0;
  }
  int alltoallv(const void* dsend, const int64_t* scount, void* drecv, const int64_t* rcount, size_t rec,
                hipStream_t s) override {
    std::lock_guard<std::mutex> g(mu);
    size_t total = 0;
    for (int p = 0; p < nranks; ++p) total += (size_t)scount[p] * rec;
    std::vector<uint8_t> h(total);
    if (total) CHIP(hipMemcpyAsync(h.data(), dsend, total, hipMemcpyDeviceToHost, s));
    CHIP(hipStreamSynchronize(s));
    std::vector<uint8_t> out;
    CTRY(alltoallv_bytes(h.data(), scount, rcount, rec, &out));
    if (!out.empty()) {
      CHIP(hipMemcpyAsync(drecv, out.data(), out.size(), hipMemcpyHostToDevice, s));
      CHIP(hipStreamSynchronize(s));
    }
    return 0;
  }
  int alltoallv_host(const void* send, const int64_t* scount, void* recv, const int64_t* rcount, size_t rec) override {
    std::lock_guard<std::mutex> g(mu);
    std::vector<uint8_t> out;
    CTRY(alltoallv_bytes(static_cast<const uint8_t*>(send), scount, rcount, rec, &out));
    if (!out.empty()) memcpy(recv, out.data(), out.size());
    return 0;
  }
  int allgather_host(const void* send, size_t bytes, void* recv) override {
    std::lock_guard<std::mutex> g(mu);
    std::vector<std::vector<uint8_t>> all;
    CTRY(exchange(send, bytes, &all));
    for (int r = 0; r < nranks; ++r) {
      if (all[r].size() != bytes) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "all-gather: ranks' sizes differ");
      memcpy((uint8_t*)recv + bytes * (size_t)r, all[r].data(), bytes);
    }
    return 0;
  }
};

}  // namespace

CommWait& comm_wait() {
  static thread_local CommWait w;
  return w;
}

double comm_now_us() {
  return (double)std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

int Comm::usable() const {
  if (aborted.load(std::memory_order_acquire))
    return host_fail(PGPU_ERR_DEVICE, "communicator aborted: a collective's wait on its peers expired earlier "
                     "(create a new communicator)");
  return 0;
}

int Comm::wait_expired(double t0_us) const {
  const CommWait& w = comm_wait();
  if (w.cancel && __atomic_load_n(w.cancel, __ATOMIC_ACQUIRE))
    return host_fail(PGPU_ERR_CANCELLED, "QueryException 503 (QUERY_CANCELLATION_ERROR): Query was cancelled while "
                     "waiting on the other GPUs' combine");
  if (w.end_time_ms > 0) {
    const double now_ms = (double)std::chrono::duration_cast<std::chrono::microseconds>(
                              std::chrono::system_clock::now().time_since_epoch()).count() / 1000.0;
    if (now_ms >= (double)w.end_time_ms)
      return host_fail(PGPU_ERR_TIMEOUT, "QueryException 200 (QUERY_EXECUTION_ERROR): Timed out while combining "
                       "group-by results across GPUs");
  }
  const int64_t lim = timeout_ms.load(std::memory_order_relaxed);
  if (lim > 0 && comm_now_us() - t0_us > (double)lim * 1000.0)
    return host_fail(PGPU_ERR_TIMEOUT, "communicator: rank peers did not join a collective within %lld ms "
                     "(rank %d of %d)", (long long)lim, rank, nranks);
  return 0;
}

int comm_unique_id(int32_t kind, void* id) {
  memset(id, 0, PGPU_COMM_ID_BYTES);
  if (kind == PGPU_COMM_RCCL) {
    static_assert(sizeof(ncclUniqueId) <= PGPU_COMM_ID_BYTES, "ncclUniqueId does not fit");
    if (!rccl().ok) return host_fail(PGPU_ERR_UNSUPPORTED, "RCCL unavailable: %s", rccl().err.c_str());
    ncclUniqueId u;
    NTRY(rccl().GetUniqueId(&u));
    memcpy(id, &u, sizeof u);
    return 0;
  }
  if (kind == PGPU_COMM_HOST) {
    uint64_t r = 0;
    int fd = open("/dev/urandom", O_RDONLY);
    if (fd < 0 || read(fd, &r, sizeof r) != (ssize_t)sizeof r) r = (uint64_t)time(nullptr) * 0x9E3779B97F4A7C15ull;
    if (fd >= 0) close(fd);
    r ^= (uint64_t)getpid() << 32;
    snprintf((char*)id, PGPU_COMM_ID_BYTES, "pgpu-comm-%d-%016llx", (int)getpid(), (unsigned long long)r);
    return 0;
  }
  return host_fail(PGPU_ERR_INVALID_ARGUMENT, "communicator kind %d", kind);
}

int comm_create(int32_t kind, const void* id, int32_t nranks, int32_t rank, int32_t device, Comm** out) {
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks)
    return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad communicator arguments (nranks %d, rank %d)", nranks, rank);
  if (kind == PGPU_COMM_RCCL) {
    CHIP(hipSetDevice(device));
    if (!rccl().ok) return host_fail(PGPU_ERR_UNSUPPORTED, "RCCL unavailable: %s", rccl().err.c_str());
    auto c = std::make_unique<RcclComm>();
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    NTRY(rccl().CommInitRank(&c->c, nranks, u, rank));
    CHIP(hipStreamCreateWithFlags(&c->hs, hipStreamNonBlocking));
    CHIP(hipEventCreateWithFlags(&c->last, hipEventDisableTiming));
    *out = c.release();
    return 0;
  }
  if (kind == PGPU_COMM_HOST) {
    if (nranks > kHostMaxRanks) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "host communicator: at most %d ranks", kHostMaxRanks);
    const char* s = (const char*)id;
    if (memchr(s, 0, PGPU_COMM_ID_BYTES) == nullptr || strncmp(s, "pgpu-comm-", 10) != 0 || strchr(s, '/'))
      return host_fail(PGPU_ERR_INVALID_ARGUMENT, "not a host communicator id");
    auto c = std::make_unique<HostComm>();
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    c->name = s;
    const std::string p = "/dev/shm/" + c->name + ".ctl";
    const int fd = open(p.c_str(), O_RDWR | O_CREAT, 0600);
    if (fd < 0) return host_fail(PGPU_ERR_DEVICE, "host communicator: cannot open %s", p.c_str());
    // every rank sizes the file the same way; a fresh file reads as zeros, which is every generation's start
    if (ftruncate(fd, sizeof(HostCtl)) != 0) {
      close(fd);
      return host_fail(PGPU_ERR_DEVICE, "host communicator: cannot size %s", p.c_str());
    }
    void* m = mmap(nullptr, sizeof(HostCtl), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return host_fail(PGPU_ERR_DEVICE, "host communicator: cannot map %s", p.c_str());
    c->ctl = static_cast<HostCtl*>(m);
    c->ctl->live.fetch_add(1);
    CTRY(c->barrier());  // every rank joined
    *out = c.release();
    return 0;
  }
  return host_fail(PGPU_ERR_INVALID_ARGUMENT, "communicator kind %d", kind);
}

}  // namespace pgpu
