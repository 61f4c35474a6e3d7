// host_result.h — the host-side result of a plan (pgpu_result) and the pinned buffers behind it, shared by the
// runtime (rt_*.cpp, abi_*.cpp) and the server-response / broker-reduce code (server_response.cpp).  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/pinotgpu.h"
#include "host_common.h"

namespace pgpu {

struct HostPinned {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t n) {
    if (n <= cap) return 0;
    if (p) hipHostFree(p);
    p = nullptr;
    size_t c = std::max<size_t>(n + n / 4, 4096);
    if (hipHostMalloc(&p, c, hipHostMallocDefault) != hipSuccess) {
      p = nullptr;
      return host_fail(PGPU_ERR_OUT_OF_MEMORY, "hipHostMalloc of %zu bytes failed", c);
    }
    cap = c;
    return 0;
  }
  void release() {
    if (p) hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Pinned host buffers that hold finalized results, reused across queries (a result of ~10M groups is hundreds of
// MB: pinning it per query would cost more than the scan).  Shared by a table and the results it produced, so a
// result may outlive its table.
struct ResultPool {
  std::mutex mu;
  std::vector<HostPinned> free;
  ~ResultPool() {
    for (auto& h : free) h.release();
  }
  HostPinned take() {
    std::lock_guard<std::mutex> g(mu);
    if (free.empty()) return HostPinned();
    HostPinned h = free.back();
    free.pop_back();
    return h;
  }
  void give(HostPinned h) {
    if (!h.p) return;
    std::lock_guard<std::mutex> g(mu);
    free.push_back(h);
    if (free.size() > 4) {  // keep the largest few
      auto it = std::min_element(free.begin(), free.end(), [](const HostPinned& a, const HostPinned& b) { return a.cap < b.cap; });
      it->release();
      free.erase(it);
    }
  }
};

}  // namespace pgpu

struct pgpu_result_s;
namespace pgpu {
// Builds the columnar form of a result held in compact form (rt_exec.cpp); 0 or a PGPU_ERR_* status.
int result_expand(pgpu_result_s* r);
}  // namespace pgpu

struct pgpu_result_s {
  int64_t n = 0;
  int num_keys = 0;
  int num_aggs = 0;
  int num_slots = 0;
  // Groups columnar in one pinned buffer (ascending composite key, except hash-mode results of >= 4096 groups: their
  // partition order -- order-dependent consumers compare keys, server_response.cpp KeyOrder): int32 group-by dictIds
  // [num_keys][n], then (8-aligned) u64 accumulator words [num_slots][n]; slot 0 = COUNT.
  pgpu::HostPinned buf;
  std::shared_ptr<pgpu::ResultPool> pool;
  std::vector<int32_t> agg_slot;          // per aggregation: its slot
  std::vector<int32_t> slot_kind;         // per slot: how its words accumulate (internal.h SLOT_*)
  std::vector<uint8_t> agg_conv;          // per aggregation: how the slot word reads (RCONV_*)
  int64_t stats[6] = {0, 0, 0, 0, 0, 0};
  // what the rows are (DataTable / trimming): table columns and types of the group-by keys, per aggregation its
  // function and table column (-1: COUNT(*)), and numGroupsLimitReached
  std::vector<int32_t> key_cols, key_types, agg_fn, agg_col;
  // per group-by key: the table-global dictionary snapshot its group ids index (rt.h's Dict)
  std::vector<std::shared_ptr<const void>> key_dicts;
  bool groups_limit_reached = false;
  // Compact form (large tables, e.g. C5's 10M groups): the groups are the set bits of the bitmap at the start
  // of `cbuf` over the composite keys [ckey_base, ckey_base + cbits), and slot s holds their words in key order,
  // cwidth[s] bytes each (two's complement, sign-extended) at cbuf + cslot_off[s].  The columnar form above is built
  // from it on first access to gid() / slot() (pgpu::result_expand), as Pinot's group-key iterator decodes raw keys.
  pgpu::HostPinned cbuf;
  std::atomic<bool> compact{false};
  std::mutex expand_mu;
  int64_t ckey_base = 0, cbits = 0;
  // ckey_width 4 / 8 (hash-mode results): instead of the bitmap, cbuf starts with the n groups' composite keys in
  // ascending order at that width (8-aligned area); the slots follow as above.
  int32_t ckey_width = 0;
  std::vector<int64_t> cstride, ccard, coff;
  std::vector<int32_t> cwidth;
  std::vector<size_t> cslot_off;
  ~pgpu_result_s() {
    if (pool) {
      pool->give(buf);
      pool->give(cbuf);
    } else {
      buf.release();
      cbuf.release();
    }
  }
  static size_t slot_offset(int nk, int64_t n) { return ((size_t)nk * n * 4 + 7) & ~size_t(7); }
  int alloc(int nk, int ns, int64_t rows) {
    num_keys = nk;
    num_slots = ns;
    n = rows;
    if (pool && !buf.p) buf = pool->take();
    return buf.ensure(std::max<size_t>(slot_offset(nk, rows) + (size_t)ns * rows * 8, 64));
  }
  int32_t* gid_raw(int j) { return reinterpret_cast<int32_t*>(buf.p) + (size_t)j * n; }
  uint64_t* slot_raw(int s) { return reinterpret_cast<uint64_t*>((uint8_t*)buf.p + slot_offset(num_keys, n)) + (size_t)s * n; }
  int32_t* gid(int j) {
    if (compact.load(std::memory_order_acquire)) pgpu::result_expand(this);
    return gid_raw(j);
  }
  uint64_t* slot(int s) {
    if (compact.load(std::memory_order_acquire)) pgpu::result_expand(this);
    return slot_raw(s);
  }
};
enum { RCONV_I64 = 0, RCONV_F64 = 1, RCONV_KEY_F64 = 2 };

namespace pgpu {

// Read-only view of a table-global dictionary (group ids of results index it), for the response code.
struct DictView {
  std::shared_ptr<const void> keep;  // the snapshot the pointers below point into
  int type = PGPU_INT;
  const std::vector<int64_t>* iv = nullptr;
  const std::vector<double>* dv = nullptr;
  const std::vector<std::string>* sv = nullptr;
  std::string name;
};
int table_dict_view(pgpu_table t, int col, DictView* out);
// The dictionary snapshot group-by key `key` of result r indexes (the table's current one for results without).
int result_key_dict_view(const pgpu_result_s* r, pgpu_table t, int key, DictView* out);

}  // namespace pgpu
