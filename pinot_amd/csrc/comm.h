// comm.h — the communicator behind pgpu_comm (comm.cpp): the collectives the cross-GPU combine issues.  Not part of
// the ABI.
//
// Two transports, one interface:
//   RCCL  one rank per GPU, collectives over xGMI on the caller's stream (librccl is opened at the first
//         pgpu_comm_unique_id / pgpu_comm_create, preferring the copy already in the process, e.g. torch's);
//   HOST  processes of one machine exchange through files in /dev/shm with a shared-memory barrier: the same combine
//         code with several ranks on one GPU, where RCCL refuses two ranks per device.  Every call synchronises the
//         stream and stages through host memory -- a rehearsal transport, never the measured one.
// Collectives must be issued in the same order on every rank (as with RCCL); a communicator serialises its callers.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <memory>

#include "../../include/pinotgpu.h"

namespace pgpu {

enum CommDtype { CDT_I64 = 0, CDT_F64 = 1 };
enum CommOp { COP_SUM = 0, COP_MIN = 1, COP_MAX = 2 };

// Blocking waits on peers give up after this unless the communicator or the calling query sets another limit
// (pgpu_comm_set_timeout; a query's end_time_ms).
constexpr int64_t kDefaultCommTimeoutMs = 600 * 1000;

// The wait limits of the calling thread's collectives: the query's deadline and cancel flag, set by the combine entry
// points for the duration of the call (CommWaitScope).  A collective that waits on a peer past them fails instead of
// blocking forever (a peer that failed before the collective never enters it); RCCL's communicator is aborted then.
struct CommWait {
  int64_t end_time_ms = 0;     // epoch ms; 0 = none
  const int* cancel = nullptr;  // the plan's cancel flag (__atomic_* reads)
};
CommWait& comm_wait();
struct CommWaitScope {
  CommWait saved;
  CommWaitScope(int64_t end_time_ms, const int* cancel) : saved(comm_wait()) {
    comm_wait().end_time_ms = end_time_ms;
    comm_wait().cancel = cancel;
  }
  ~CommWaitScope() { comm_wait() = saved; }
};

struct Comm {
  virtual ~Comm() {}
  int nranks = 1, rank = 0, device = 0;
  std::atomic<int64_t> timeout_ms{kDefaultCommTimeoutMs};  // <= 0: no limit of the communicator's own
  std::atomic<bool> aborted{false};  // a wait expired: collectives of the peers may never complete; unusable
  // Gives the communicator up (RCCL: ncclCommAbort, so kernels of collectives a peer never joined exit).
  virtual void abort() { aborted.store(true); }
  // While waiting on peers since t0 (steady-clock us): 0, or fails with PGPU_ERR_CANCELLED / PGPU_ERR_TIMEOUT.
  int wait_expired(double t0_us) const;
  // PGPU_ERR_DEVICE once aborted.
  int usable() const;
  // In place on the device, ordered on `s`.
  virtual int allreduce(void* d, size_t count, CommDtype t, CommOp op, hipStream_t s) = 0;
  // send: nranks x count elements; rank r receives the reduction of block r into recv (count elements).
  virtual int reduce_scatter(const void* dsend, void* drecv, size_t count, CommDtype t, CommOp op, hipStream_t s) = 0;
  // send holds scount[p] records of `rec` bytes for rank p back to back (rank order); recv gets rcount[p] records from
  // rank p back to back.  rec is a multiple of 8.
  virtual int alltoallv(const void* dsend, const int64_t* scount, void* drecv, const int64_t* rcount, size_t rec,
                        hipStream_t s) = 0;
  // alltoallv over host buffers, blocking (finalized result rows).
  virtual int alltoallv_host(const void* send, const int64_t* scount, void* recv, const int64_t* rcount, size_t rec) = 0;
  // Host memory, blocking: recv = every rank's `bytes` bytes, in rank order.
  virtual int allgather_host(const void* send, size_t bytes, void* recv) = 0;
};

double comm_now_us();  // steady clock
int comm_unique_id(int32_t kind, void* id);
int comm_create(int32_t kind, const void* id, int32_t nranks, int32_t rank, int32_t device, Comm** out);

}  // namespace pgpu

// Shared ownership: a plan combined on the communicator keeps it alive (pgpu_plan_s::comm_used: finalize reads its
// timeout and may abort it) after pgpu_comm_destroy has dropped the caller's handle -- e.g. a server that replaces an
// aborted communicator while other plans combined on it are still unfinalized.
struct pgpu_comm_s {
  std::shared_ptr<pgpu::Comm> impl;
  int32_t kind = PGPU_COMM_RCCL;  // the transport pgpu_comm_recreate builds the replacement on
};
