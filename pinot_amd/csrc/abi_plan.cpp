// abi_plan.cpp -- C ABI: star-trees, dictionaries, plans (create / execute / finalize).
#include "rt_decls.h"

namespace pgpu {
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
}  // namespace pgpu

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
  // PGPU_STAR_NARROW (an A/B build of the library only): metric arrays whose values are all integers of int32 range
  // are pinned as int32 (the kernel widens them exactly) -- half the metric bytes per star-tree document.  Measured
  // and not the default (r06 sessions k, m): K6 on C4 175 -> 268 us although its traffic fell 505 -> 417 MB.
  auto ints32_f = [](const double* v, int64_t n) {
#ifndef PGPU_STAR_NARROW
    return false;
#endif
    for (int64_t i = 0; i < n; ++i)
      if (!(v[i] >= -2147483648.0 && v[i] <= 2147483647.0) || v[i] != (double)(int32_t)v[i]) return false;
    return true;
  };
  auto ints32_c = [](const int64_t* v, int64_t n) {
#ifndef PGPU_STAR_NARROW
    return false;
#endif
    for (int64_t i = 0; i < n; ++i)
      if (v[i] < INT32_MIN || v[i] > INT32_MAX) return false;
    return true;
  };
  for (int m = 0; m < d->num_metrics; ++m) {
    const pgpu_agg a = d->metrics[m];
    if (a.fn < PGPU_AGG_COUNT || a.fn > PGPU_AGG_AVG) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad metric function");
    const bool needs_f = a.fn != PGPU_AGG_COUNT, needs_c = a.fn == PGPU_AGG_COUNT || a.fn == PGPU_AGG_AVG;
    if ((needs_f && !d->metric_f64[m]) || (needs_c && !d->metric_i64[m]))
      return fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree metric %d values missing", m);
    if (needs_f && (a.column < 0 || a.column >= (int)seg.cols.size()))
      return fail(PGPU_ERR_INVALID_ARGUMENT, "bad star-tree metric column");
    st->metrics.push_back(a);
    st->mf_narrow.push_back(needs_f && ints32_f(d->metric_f64[m], d->num_docs));
    st->mc_narrow.push_back(needs_c && ints32_c(d->metric_i64[m], d->num_docs));
    bytes += (needs_f ? (int64_t)d->num_docs * (st->mf_narrow.back() ? 4 : 8) : 0) +
             (needs_c ? (int64_t)d->num_docs * (st->mc_narrow.back() ? 4 : 8) : 0) + 32;
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
      if (st->mf_narrow[m]) {
        int32_t* o = reinterpret_cast<int32_t*>(host.data() + off);
        for (int64_t i = 0; i < d->num_docs; ++i) o[i] = (int32_t)d->metric_f64[m][i];
      } else {
        memcpy(host.data() + off, d->metric_f64[m], (size_t)d->num_docs * 8);
      }
      pf = reinterpret_cast<const double*>((uint8_t*)st->d_block + off);
      off += (int64_t)d->num_docs * (st->mf_narrow[m] ? 4 : 8) + 16;
    }
    if (a.fn == PGPU_AGG_COUNT || a.fn == PGPU_AGG_AVG) {
      if (st->mc_narrow[m]) {
        int32_t* o = reinterpret_cast<int32_t*>(host.data() + off);
        for (int64_t i = 0; i < d->num_docs; ++i) o[i] = (int32_t)d->metric_i64[m][i];
      } else {
        memcpy(host.data() + off, d->metric_i64[m], (size_t)d->num_docs * 8);
      }
      pc = reinterpret_cast<const int64_t*>((uint8_t*)st->d_block + off);
      off += (int64_t)d->num_docs * (st->mc_narrow[m] ? 4 : 8) + 16;
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
  P->timed = (q->options & PGPU_OPT_TIMING) != 0;
  P->scratch = acquire_scratch(t);
  *out = P.release();
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_destroy(pgpu_plan P) try {
  PGPU_ABI_GUARD;
  if (!P) return 0;
  for (auto& part : P->parts) {
    inflight_end(part.plan.get());
    release_scratch(P->table, part.plan->scratch);
  }
  inflight_end(P);
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
  P->timed = (q->options & PGPU_OPT_TIMING) != 0;
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
}  // extern "C"
