// abi_combine.cpp -- C ABI: the cross-GPU exchange, row merges, communicator, combine.
#include "rt_decls.h"

extern "C" {

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

namespace pgpu {
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
}  // namespace pgpu

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
  P->exported = false;
  P->k8d_counts = false;
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
  P->exported = false;  // the table changes: finalize reads it from the device
  P->k8d_counts = false;
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
  // which aborts the communicator -- for a query without a deadline at most kDenseCombineWaitMs (wait_plan), not the
  // communicator's whole timeout.
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
  P->comm_dense = true;
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

}  // extern "C"
