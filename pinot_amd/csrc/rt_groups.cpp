// rt_groups.cpp -- the numGroupsLimit split and the compiled-plan cache (rt.h).
#include "rt_decls.h"

namespace pgpu {

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
  const int32_t opts = q->options & ~PGPU_OPT_TIMING;  // timing events are per execution, not compiled in
  put(&opts, 4);
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
    P->inflight_counted = false;
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
  img->inflight_counted = false;
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

}  // namespace pgpu

