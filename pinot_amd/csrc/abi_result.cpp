// abi_result.cpp -- C ABI: one-call execution, plan statistics, results, generator.
#include "rt_decls.h"

extern "C" {

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

int pgpu_plan_star_metric_bytes(pgpu_plan P, int64_t* bytes) try {
  PGPU_ABI_GUARD;
  if (!P || !bytes) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  *bytes = P->star_metric_bytes;
  return 0;
} PGPU_ABI_CATCH

int pgpu_plan_timing(pgpu_plan P, double* out3) try {
  PGPU_ABI_GUARD;
  if (!P || !out3 || !P->executed) return fail(PGPU_ERR_INVALID_ARGUMENT, "plan not executed");
  if (P->composite) return fail(PGPU_ERR_UNSUPPORTED, "numGroupsLimit plan: timing is per part");
  if (!P->timed) return fail(PGPU_ERR_INVALID_ARGUMENT, "execution not timed (query option PGPU_OPT_TIMING)");
  Scratch* sc = P->scratch;
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

