// rt_plan.cpp -- query planning: predicate translation, filter folding, group-key layout, launch configuration (rt.h).
#include "rt_decls.h"

namespace pgpu {

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
  const int cnt_m = cnt_pair >= 0 ? cnt_pair : has_avg ? st->pair(PGPU_AGG_AVG, avg_col) : -1;
  if (cnt_m >= 0) {
    k.src_c[0] = st->d_mc[cnt_m];
    if (st->mc_narrow[cnt_m]) k.narrow |= 1u << 31;
  }
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
    if (st->mf_narrow[m]) k.narrow |= 1u << sl;
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
                     const StreamExec* se) {
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

}  // namespace pgpu
