// filter_stats.cpp — numEntriesScannedInFilter of one segment (see filter_stats.h).
#include "filter_stats.h"

#include <algorithm>
#include <climits>
#include <memory>

#include "../../include/pinotgpu.h"
#include "host_common.h"
#include "internal.h"

namespace pgpu {

namespace {

bool is_primitive(int type) {
  return type == SN_SCAN || type == SN_SORTED || type == SN_BITMAP || type == SN_RANGEIDX || type == SN_NOT;
}
// Index-based leaves: their docIdSet is a sorted range or a bitmap, no iterator scans for them.
bool is_index(int type) { return type == SN_SORTED || type == SN_BITMAP || type == SN_RANGEIDX; }

// reorderAndFilterChildOperators priorities (FilterOperatorUtils.java:143-178); NOT ranks with the scans.
int and_priority(int type) {
  switch (type) {
    case SN_SORTED: return 0;
    case SN_BITMAP: return 1;
    case SN_RANGEIDX: return 2;
    case SN_AND: return 3;
    case SN_OR: return 4;
    default: return 5;
  }
}

}  // namespace

StatTree build_stat_tree(const std::vector<int32_t>& ops, const std::vector<int32_t>& leaf) {
  StatTree t;
  auto add = [&](int type, int lf = -1) {
    StatNode n;
    n.type = type;
    n.leaf = lf;
    t.nodes.push_back(n);
    return (int32_t)t.nodes.size() - 1;
  };
  if (ops.empty()) {
    t.root = add(SN_ALL);
    return t;
  }
  std::vector<int32_t> st;
  for (int32_t e : ops) {
    const int op = e >> 16, arg = e & 0xFFFF;
    if (op == OP_LEAF) {
      static const int kType[] = {SN_EMPTY, SN_ALL, SN_SCAN, SN_SORTED, SN_BITMAP, SN_RANGEIDX};
      st.push_back(add(kType[leaf[arg]], arg));
    } else if (op == OP_NOT) {
      const int32_t c = st.back();
      st.pop_back();
      if (t.nodes[c].type == SN_EMPTY) st.push_back(add(SN_ALL));
      else if (t.nodes[c].type == SN_ALL) st.push_back(add(SN_EMPTY));
      else {
        const int32_t n = add(SN_NOT);
        t.nodes[n].kids.push_back(c);
        st.push_back(n);
      }
    } else {
      const bool is_and = op == OP_AND;
      std::vector<int32_t> kids(st.end() - arg, st.end());
      st.resize(st.size() - arg);
      int32_t result = -1;
      std::vector<int32_t> keep;
      for (int32_t c : kids) {  // getAndFilterOperator :90-95 / getOrFilterOperator :115-120
        const int ty = t.nodes[c].type;
        if (is_and ? ty == SN_EMPTY : ty == SN_ALL) { result = c; break; }
        if (is_and ? ty == SN_ALL : ty == SN_EMPTY) continue;
        keep.push_back(c);
      }
      if (result < 0) {
        if (keep.empty()) result = add(is_and ? SN_ALL : SN_EMPTY);
        else if (keep.size() == 1) result = keep[0];
        else {
          if (is_and)
            std::stable_sort(keep.begin(), keep.end(), [&](int32_t x, int32_t y) {
              return and_priority(t.nodes[x].type) < and_priority(t.nodes[y].type);
            });
          result = add(is_and ? SN_AND : SN_OR);
          t.nodes[result].kids = keep;
        }
      }
      st.push_back(result);
    }
  }
  t.root = st.back();
  return t;
}

StatsPlan classify_stat_tree(const StatTree& t, int64_t num_docs) {
  StatsPlan p;
  const StatNode& r = t.nodes[t.root];
  switch (r.type) {
    case SN_EMPTY: case SN_ALL: case SN_SORTED: case SN_BITMAP: case SN_RANGEIDX: return p;  // no scan-based iterator
    case SN_SCAN: case SN_NOT: p.constant = num_docs; return p;          // iterated over every doc
    default: break;
  }
  for (int32_t c : r.kids)
    if (!is_primitive(t.nodes[c].type)) { p.kind = STATS_GENERIC; return p; }
  if (r.type == SN_OR) {
    // OrDocIdIterator.next: every scan child runs through the whole segment (index children merged or not)
    for (int32_t c : r.kids)
      if (t.nodes[c].type == SN_SCAN || t.nodes[c].type == SN_NOT) p.constant += num_docs;
    return p;
  }
  int nidx = 0, nscan = 0, nnot = 0;
  for (int32_t c : r.kids) {
    const int ty = t.nodes[c].type;
    if (is_index(ty)) { ++nidx; p.index_leaves.push_back(t.nodes[c].leaf); }
    else if (ty == SN_SCAN) { ++nscan; p.scan_leaves.push_back(t.nodes[c].leaf); }
    else ++nnot;
  }
  if (nnot > 0) { p.kind = STATS_GENERIC; return p; }
  if ((nidx > 0 && nscan > 0) || nidx > 1) {  // AndDocIdSet: index bitmap, then each scan's applyAnd
    p.kind = nscan > 0 ? STATS_CHAIN : STATS_CONST;
    return p;
  }
  p.kind = nscan == 2 ? STATS_LEAP2 : STATS_GENERIC;  // AndDocIdIterator over the children
  return p;
}

std::vector<int32_t> range_index_leaves(const StatTree& t) {
  std::vector<int32_t> out;
  if (t.root < 0) return out;
  std::vector<int32_t> st{t.root};
  while (!st.empty()) {
    const StatNode& n = t.nodes[st.back()];
    st.pop_back();
    if (n.type == SN_RANGEIDX) out.push_back(n.leaf);
    if (n.type == SN_AND || n.type == SN_OR)
      for (int32_t k : n.kids) st.push_back(k);
  }
  std::sort(out.begin(), out.end());
  return out;
}

// ------------------------------------------------------------------------------------------------ replay
namespace {

constexpr int kEof = INT_MIN;  // Constants.EOF

struct Bits {
  std::vector<uint32_t> w;
  int32_t n = 0;
  // First set bit >= from (docs < n), or -1.
  int next(int32_t from) const {
    if (from >= n) return -1;
    size_t g = (size_t)from >> 5;
    uint32_t m = w[g] & (~0u << (from & 31));
    while (!m) {
      if (++g >= w.size()) return -1;
      m = w[g];
    }
    const int d = (int)(g * 32 + __builtin_ctz(m));
    return d < n ? d : -1;
  }
  int64_t count() const {
    int64_t c = 0;
    for (uint32_t x : w) c += __builtin_popcount(x);
    return c;
  }
};

enum ItType { IT_EMPTY, IT_ALL, IT_SCAN, IT_IDX, IT_AND, IT_OR };
struct It {
  int type = IT_EMPTY;
  int next_doc = 0;
  int64_t scanned = 0;
  Bits bits;                   // IT_SCAN: the predicate's matches; IT_IDX: the doc set
  bool sorted = false;
  std::vector<It*> kids;
  std::vector<int> next_ids;   // IT_OR
  int num_not_exhausted = 0, prev_doc = -1;
};

int it_next(It* it);
int it_advance(It* it, int target);

int it_next(It* it) {
  switch (it->type) {
    case IT_EMPTY: return kEof;
    case IT_ALL: return it->next_doc < it->bits.n ? it->next_doc++ : kEof;
    case IT_IDX: {
      const int d = it->bits.next(it->next_doc);
      if (d < 0) { it->next_doc = it->bits.n; return kEof; }
      it->next_doc = d + 1;
      return d;
    }
    case IT_SCAN: {  // SVScanDocIdIterator.next: every doc from the cursor up to the match is an entry
      if (it->next_doc >= it->bits.n) return kEof;
      const int d = it->bits.next(it->next_doc);
      if (d < 0) {
        it->scanned += it->bits.n - it->next_doc;
        it->next_doc = it->bits.n;
        return kEof;
      }
      it->scanned += d - it->next_doc + 1;
      it->next_doc = d + 1;
      return d;
    }
    case IT_AND: {  // AndDocIdIterator.next
      int max_doc = it->next_doc, max_idx = -1, index = 0;
      const int k = (int)it->kids.size();
      while (index < k) {
        if (index == max_idx) { ++index; continue; }
        const int d = it_advance(it->kids[index], max_doc);
        if (d == kEof) return kEof;
        if (d == max_doc) ++index;
        else { max_doc = d; max_idx = index; index = 0; }
      }
      it->next_doc = max_doc;
      return it->next_doc++;
    }
    default: {  // OrDocIdIterator.next
      int next = INT_MAX;
      bool exhausted = false;
      for (int i = 0; i < it->num_not_exhausted; ++i) {
        int d = it->next_ids[i];
        if (d == it->prev_doc) {
          d = it_next(it->kids[i]);
          it->next_ids[i] = d;
          if (d == kEof) { exhausted = true; continue; }
        }
        next = std::min(next, d);
      }
      if (exhausted) {
        int w = 0;
        for (int i = 0; i < it->num_not_exhausted; ++i)
          if (it->next_ids[i] != kEof) { it->kids[w] = it->kids[i]; it->next_ids[w] = it->next_ids[i]; ++w; }
        it->num_not_exhausted = w;
      }
      if (next != INT_MAX) { it->prev_doc = next; return next; }
      return kEof;
    }
  }
}

int it_advance(It* it, int target) {
  if (it->type != IT_OR) {
    if (it->type == IT_EMPTY) return kEof;
    it->next_doc = target;
    return it_next(it);
  }
  int next = INT_MAX;  // OrDocIdIterator.advance
  bool exhausted = false;
  for (int i = 0; i < it->num_not_exhausted; ++i) {
    int d = it->next_ids[i];
    if (d < target) {
      d = it_advance(it->kids[i], target);
      it->next_ids[i] = d;
      if (d == kEof) { exhausted = true; continue; }
    }
    next = std::min(next, d);
  }
  if (exhausted) {
    int w = 0;
    for (int i = 0; i < it->num_not_exhausted; ++i)
      if (it->next_ids[i] != kEof) { it->kids[w] = it->kids[i]; it->next_ids[w] = it->next_ids[i]; ++w; }
    it->num_not_exhausted = w;
  }
  if (next != INT_MAX) { it->prev_doc = next; return next; }
  return kEof;
}

struct Replay {
  const StatTree& t;
  const std::vector<const uint32_t*>& masks;
  int32_t n;
  size_t nw;
  std::vector<std::unique_ptr<It>> pool;

  Bits leaf_bits(int leaf) const {
    Bits b;
    b.n = n;
    b.w.assign(masks[leaf], masks[leaf] + nw);
    return b;
  }
  // Documents a (sub)tree matches (NOT's operand: evaluated per document, no iterator runs).
  Bits match(int32_t node) const {
    const StatNode& s = t.nodes[node];
    Bits b;
    b.n = n;
    switch (s.type) {
      case SN_EMPTY: b.w.assign(nw, 0u); break;
      case SN_ALL: b.w.assign(nw, ~0u); break;
      case SN_SCAN: case SN_SORTED: case SN_BITMAP: case SN_RANGEIDX: b = leaf_bits(s.leaf); break;
      case SN_NOT: b = match(s.kids[0]); for (auto& x : b.w) x = ~x; break;
      case SN_AND:
        b.w.assign(nw, ~0u);
        for (int32_t c : s.kids) { Bits k = match(c); for (size_t i = 0; i < nw; ++i) b.w[i] &= k.w[i]; }
        break;
      default:
        b.w.assign(nw, 0u);
        for (int32_t c : s.kids) { Bits k = match(c); for (size_t i = 0; i < nw; ++i) b.w[i] |= k.w[i]; }
        break;
    }
    if (nw && (n & 31)) b.w[nw - 1] &= (1u << (n & 31)) - 1u;
    return b;
  }
  It* make(int type) {
    pool.emplace_back(new It());
    It* it = pool.back().get();
    it->type = type;
    it->bits.n = n;
    return it;
  }
  It* make_multi(int type, std::vector<It*> kids) {
    It* it = make(type);
    it->kids = std::move(kids);
    if (type == IT_OR) {
      it->next_ids.assign(it->kids.size(), -1);
      it->num_not_exhausted = (int)it->kids.size();
    }
    return it;
  }
  // FilterBlockDocIdSet.iterator() (AndDocIdSet.java:60-146, OrDocIdSet.java:57-110).
  It* build(int32_t node) {
    const StatNode& s = t.nodes[node];
    switch (s.type) {
      case SN_EMPTY: return make(IT_EMPTY);
      case SN_ALL: return make(IT_ALL);
      case SN_SCAN: case SN_NOT: { It* it = make(IT_SCAN); it->bits = match(node); return it; }
      case SN_SORTED: case SN_BITMAP: case SN_RANGEIDX: {
        It* it = make(IT_IDX);
        it->bits = match(node);
        it->sorted = s.type == SN_SORTED;
        return it;
      }
      default: break;
    }
    std::vector<It*> kids;
    for (int32_t c : s.kids) kids.push_back(build(c));
    int nidx = 0, nscan = 0;
    for (It* k : kids) { nidx += k->type == IT_IDX; nscan += k->type == IT_SCAN; }
    const int nrem = (int)kids.size() - nidx - nscan;
    if (s.type == SN_AND) {
      if (!((nidx > 0 && nscan > 0) || nidx > 1)) return make_multi(IT_AND, kids);
      It* rangeless = make(IT_IDX);
      rangeless->bits.w.assign(nw, ~0u);
      if (nw && (n & 31)) rangeless->bits.w[nw - 1] &= (1u << (n & 31)) - 1u;
      for (It* k : kids)
        if (k->type == IT_IDX) for (size_t i = 0; i < nw; ++i) rangeless->bits.w[i] &= k->bits.w[i];
      for (It* k : kids) {  // ScanBasedDocIdIterator.applyAnd (SVScanDocIdIterator.java:75-94)
        if (k->type != IT_SCAN) continue;
        k->scanned += rangeless->bits.count();
        for (size_t i = 0; i < nw; ++i) rangeless->bits.w[i] &= k->bits.w[i];
      }
      if (nrem == 0) return rangeless;
      std::vector<It*> ks{rangeless};
      for (It* k : kids) if (k->type != IT_IDX && k->type != IT_SCAN) ks.push_back(k);
      return make_multi(IT_AND, ks);
    }
    if (nidx <= 1) return make_multi(IT_OR, kids);
    It* merged = make(IT_IDX);
    merged->bits.w.assign(nw, 0u);
    for (It* k : kids)
      if (k->type == IT_IDX) for (size_t i = 0; i < nw; ++i) merged->bits.w[i] |= k->bits.w[i];
    if (nidx == (int)kids.size()) return merged;
    std::vector<It*> ks{merged};
    for (It* k : kids) if (k->type != IT_IDX) ks.push_back(k);
    return make_multi(IT_OR, ks);
  }
};

}  // namespace

int64_t simulate_entries_scanned(const StatTree& t, const std::vector<const uint32_t*>& leaf_masks, int32_t num_docs) {
  if (num_docs <= 0) return 0;
  Replay r{t, leaf_masks, num_docs, ((size_t)num_docs + 31) / 32, {}};
  It* root = r.build(t.root);
  if (root->type != IT_IDX && root->type != IT_ALL && root->type != IT_EMPTY)
    while (it_next(root) != kEof) {}  // DocIdSetOperator pulls every matching doc
  int64_t s = 0;
  for (auto& it : r.pool) if (it->type == IT_SCAN) s += it->scanned;
  return s;
}

}  // namespace pgpu

// ================================================================================================ C ABI
extern "C" int pgpu_filter_entries_scanned(const pgpu_filter_op* filter, int32_t num_filter_ops,
                                           const int32_t* leaf_types, const uint32_t* const* leaf_masks,
                                           int32_t num_leaves, int32_t num_docs, int64_t* out) try {
  using namespace pgpu;
  if (!out || num_leaves < 0 || num_filter_ops < 0 || num_docs < 0 || (num_filter_ops && !filter) ||
      (num_leaves && !leaf_types))
    return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  std::vector<int32_t> ops, types(leaf_types, leaf_types + num_leaves);
  int depth = 0;
  for (int i = 0; i < num_filter_ops; ++i) {
    const pgpu_filter_op& o = filter[i];
    if (o.op == PGPU_OP_PRED) {
      if (o.arg < 0 || o.arg >= num_leaves) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad predicate index");
      ops.push_back((OP_LEAF << 16) | o.arg);
      ++depth;
    } else if (o.op == PGPU_OP_NOT) {
      if (depth < 1) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "malformed filter program");
      ops.push_back(OP_NOT << 16);
    } else if (o.op == PGPU_OP_AND || o.op == PGPU_OP_OR) {
      if (o.arg < 1 || o.arg > depth) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "malformed filter program");
      depth -= o.arg - 1;
      ops.push_back(((o.op == PGPU_OP_AND ? OP_AND : OP_OR) << 16) | o.arg);
    } else {
      return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad filter opcode %d", o.op);
    }
  }
  if (num_filter_ops && depth != 1) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "malformed filter program");
  std::vector<const uint32_t*> masks(num_leaves, nullptr);
  for (int i = 0; i < num_leaves; ++i) {
    if (types[i] < SL_EMPTY || types[i] > SL_RANGEIDX) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad leaf type");
    if (types[i] >= SL_SCAN) {
      if (!leaf_masks || !leaf_masks[i]) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "leaf %d has no doc set", i);
      masks[i] = leaf_masks[i];
    }
  }
  *out = simulate_entries_scanned(build_stat_tree(ops, types), masks, num_docs);
  return 0;
} PGPU_ABI_CATCH
