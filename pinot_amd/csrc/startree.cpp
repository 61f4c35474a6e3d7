// startree.cpp — star-tree index builder (host): the pre-aggregated tree a star-tree query traverses on the GPU.
//
// Restates Pinot's on-heap builder so pinned segments can carry a star-tree for the star-tree query path
// (SURVEY.md §8 a29-a32):
//   BaseSingleTreeBuilder.build / constructStarTree / constructNonStarNodes / constructStarNode /
//   createAggregatedDocs (seglocal/startree/v2/builder/BaseSingleTreeBuilder.java:298-453),
//   OnHeapSingleTreeBuilder.sortAndAggregateSegmentRecords / generateRecordsForStarNode
//   (seglocal/startree/v2/builder/OnHeapSingleTreeBuilder.java:57-160),
//   StarTreeBuilderUtils.serializeTree (BFS node order, children sorted by dimension value, :91-230),
//   Sum/Count/Min/Max/AvgValueAggregator (seglocal/aggregator/).
// Children of a node are visited in java.util.HashMap<Integer, TreeNode> iteration order (bucket of the key, then
// insertion order), which fixes the star-tree document order exactly as the reference builder lays it out.
// Pure host code: no HIP call (the CPU tests build star-trees without a GPU).
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/pinotgpu.h"
#include "host_common.h"

namespace {

constexpr int kAll = -1;           // StarTreeNode.ALL (segspi/index/startree/StarTreeNode.java:29)
constexpr int kStarInFwd = 0;      // StarTreeV2Constants.STAR_IN_FORWARD_INDEX (:38)
constexpr int kInvalid = -1;       // StarTreeBuilderUtils.INVALID_ID (:53)

inline uint32_t rd_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
inline uint64_t rd_be64(const uint8_t* p) { return ((uint64_t)rd_be32(p) << 32) | rd_be32(p + 4); }

// PinotDataBitSet.readInt (seglocal/io/util/PinotDataBitSet.java:78-100).
int32_t read_bits(const uint8_t* buf, int64_t index, int bits) {
  const int64_t bit = index * bits;
  int64_t byte = bit >> 3;
  int off = (int)(bit & 7);
  uint32_t v = 0;
  int need = bits;
  while (need > 0) {
    const int avail = 8 - off;
    const int take = avail < need ? avail : need;
    const uint32_t b = (buf[byte] >> (avail - take)) & ((1u << take) - 1u);
    v = (v << take) | b;
    need -= take;
    off = 0;
    ++byte;
  }
  return (int32_t)v;
}

// PinotDataBitSet.writeInt (:138-165), into a zeroed buffer.
void write_bits(uint8_t* buf, int64_t index, int bits, uint32_t value) {
  int64_t bit = index * bits;
  for (int i = bits - 1; i >= 0; --i, ++bit)
    if ((value >> i) & 1u) buf[bit >> 3] |= (uint8_t)(0x80u >> (bit & 7));
}

int bits_for(int32_t card) {  // PinotDataBitSet.getNumBitsPerValue(card - 1) (:59-70)
  int32_t m = card - 1;
  if (m <= 1) return 1;
  int n = 0;
  while (m) { ++n; m >>= 1; }
  return n;
}

struct Node {
  int dim_id = kInvalid, dim_value = kInvalid, start = kInvalid, end = kInvalid, agg_doc = kInvalid;
  int child_dim_id = kInvalid;
  bool has_children = false;
  std::vector<int> children;   // node indices in HashMap iteration order
  int star_child = -1;
};

struct Builder {
  int D = 0, M = 0;
  std::vector<int> fn;                       // per metric: PGPU_AGG_*
  std::vector<int> skip_star;                // per dimension
  int max_leaf = 10000;
  // records (structure of arrays)
  std::vector<int32_t> dims;                 // [doc][D]
  std::vector<double> mf;                    // [doc][M] SUM/MIN/MAX value, AVG sum
  std::vector<int64_t> mc;                   // [doc][M] COUNT, AVG count
  int num_docs = 0;
  std::vector<Node> nodes;

  int new_node() {
    nodes.emplace_back();
    return (int)nodes.size() - 1;
  }
  void append(const int32_t* d, const double* f, const int64_t* c) {
    dims.insert(dims.end(), d, d + D);
    mf.insert(mf.end(), f, f + M);
    mc.insert(mc.end(), c, c + M);
    ++num_docs;
  }
  int dim_value(int doc, int d) const { return dims[(size_t)doc * D + d]; }

  // ValueAggregator.applyAggregatedValue on record (f, c) <- (f2, c2)
  void merge_into(double* f, int64_t* c, const double* f2, const int64_t* c2) const {
    for (int m = 0; m < M; ++m) {
      switch (fn[m]) {
        case PGPU_AGG_COUNT: c[m] += c2[m]; break;
        case PGPU_AGG_SUM: f[m] += f2[m]; break;
        case PGPU_AGG_MIN: f[m] = std::min(f[m], f2[m]); break;
        case PGPU_AGG_MAX: f[m] = std::max(f[m], f2[m]); break;
        default: f[m] += f2[m]; c[m] += c2[m]; break;  // AVG: AvgPair.apply
      }
    }
  }

  // java.util.HashMap<Integer, TreeNode> iteration order for keys inserted in `keys` order (ascending dictIds,
  // then StarTreeNode.ALL last): table length is the smallest power of two >= 16 holding size <= 0.75 * length;
  // bucket = (h ^ (h >>> 16)) & (length - 1); ties keep insertion order (HashMap.resize preserves it).
  static void hashmap_order(std::vector<int>& idx, const std::vector<int>& keys) {
    size_t cap = 16;
    while ((double)keys.size() > 0.75 * (double)cap) cap <<= 1;
    std::vector<std::pair<uint32_t, int>> order(idx.size());
    for (size_t i = 0; i < idx.size(); ++i) {
      const uint32_t h = (uint32_t)keys[i];
      order[i] = {(h ^ (h >> 16)) & (uint32_t)(cap - 1), (int)i};
    }
    std::stable_sort(order.begin(), order.end(),
                     [](const std::pair<uint32_t, int>& a, const std::pair<uint32_t, int>& b) { return a.first < b.first; });
    std::vector<int> out(idx.size());
    for (size_t i = 0; i < idx.size(); ++i) out[i] = idx[order[i].second];
    idx.swap(out);
  }

  // constructNonStarNodes (:369-394)
  void non_star_nodes(int start, int end, int d, std::vector<int>& kids, std::vector<int>& keys) {
    int node_start = start;
    int value = dim_value(start, d);
    for (int i = start + 1; i < end; ++i) {
      const int v = dim_value(i, d);
      if (v != value) {
        const int n = new_node();
        nodes[n].dim_id = d;
        nodes[n].dim_value = value;
        nodes[n].start = node_start;
        nodes[n].end = i;
        kids.push_back(n);
        keys.push_back(value);
        node_start = i;
        value = v;
      }
    }
    const int n = new_node();
    nodes[n].dim_id = d;
    nodes[n].dim_value = value;
    nodes[n].start = node_start;
    nodes[n].end = end;
    kids.push_back(n);
    keys.push_back(value);
  }

  // OnHeapSingleTreeBuilder.generateRecordsForStarNode (:120-160) + constructStarNode (:396-408)
  int star_node(int start, int end, int d) {
    const int n = new_node();
    nodes[n].dim_id = d;
    nodes[n].dim_value = kAll;
    nodes[n].start = num_docs;
    std::vector<int> recs(end - start);
    for (int i = 0; i < end - start; ++i) recs[i] = start + i;
    std::stable_sort(recs.begin(), recs.end(), [&](int a, int b) {  // Arrays.sort(Object[]) is stable
      for (int k = d + 1; k < D; ++k) {
        const int x = dim_value(a, k), y = dim_value(b, k);
        if (x != y) return x < y;
      }
      return false;
    });
    std::vector<int32_t> dd(D);
    std::vector<double> f(M);
    std::vector<int64_t> c(M);
    size_t i = 0;
    while (i < recs.size()) {
      const int first = recs[i];
      // records appended below may reallocate `dims`: copy the group's first record before appending
      for (int k = 0; k < D; ++k) dd[k] = dim_value(first, k);
      dd[d] = kStarInFwd;
      for (int m = 0; m < M; ++m) { f[m] = mf[(size_t)first * M + m]; c[m] = mc[(size_t)first * M + m]; }
      size_t j = i + 1;
      for (; j < recs.size(); ++j) {
        bool same = true;
        for (int k = d + 1; k < D && same; ++k) same = dim_value(recs[j], k) == dim_value(first, k);
        if (!same) break;
        merge_into(f.data(), c.data(), &mf[(size_t)recs[j] * M], &mc[(size_t)recs[j] * M]);
      }
      append(dd.data(), f.data(), c.data());
      i = j;
    }
    nodes[n].end = num_docs;
    return n;
  }

  // constructStarTree (:344-367)
  void construct(int node, int start, int end) {
    const int child_dim = nodes[node].dim_id + 1;
    if (child_dim == D) return;
    nodes[node].child_dim_id = child_dim;
    std::vector<int> kids, keys;
    non_star_nodes(start, end, child_dim, kids, keys);
    if (!skip_star[child_dim] && kids.size() > 1) {
      const int s = star_node(start, end, child_dim);
      kids.push_back(s);
      keys.push_back(kAll);
      nodes[node].star_child = s;
    }
    hashmap_order(kids, keys);
    nodes[node].children = kids;
    nodes[node].has_children = true;
    for (int k : kids)
      if (nodes[k].end - nodes[k].start > max_leaf) construct(k, nodes[k].start, nodes[k].end);
  }

  // createAggregatedDocs (:410-453); returns the record as (dims, f, c) in the out vectors.
  void aggregated(int node, std::vector<int32_t>& od, std::vector<double>& of, std::vector<int64_t>& oc) {
    Node& N = nodes[node];
    if (!N.has_children) {
      od.assign(&dims[(size_t)N.start * D], &dims[(size_t)N.start * D] + D);
      of.assign(&mf[(size_t)N.start * M], &mf[(size_t)N.start * M] + M);
      oc.assign(&mc[(size_t)N.start * M], &mc[(size_t)N.start * M] + M);
      for (int i = N.start + 1; i < N.end; ++i) merge_into(of.data(), oc.data(), &mf[(size_t)i * M], &mc[(size_t)i * M]);
      for (int k = N.dim_id + 1; k < D; ++k) od[k] = kStarInFwd;
      nodes[node].agg_doc = num_docs;
      append(od.data(), of.data(), oc.data());
      return;
    }
    const std::vector<int> kids = N.children;
    if (N.star_child >= 0) {
      std::vector<int32_t> d2;
      std::vector<double> f2;
      std::vector<int64_t> c2;
      for (int k : kids) {
        if (k == nodes[node].star_child) {
          aggregated(k, od, of, oc);
          nodes[node].agg_doc = nodes[k].agg_doc;
        } else {
          aggregated(k, d2, f2, c2);
        }
      }
      return;
    }
    bool first = true;
    std::vector<int32_t> d2;
    std::vector<double> f2;
    std::vector<int64_t> c2;
    for (int k : kids) {
      aggregated(k, d2, f2, c2);
      if (first) { od = d2; of = f2; oc = c2; first = false; }
      else merge_into(of.data(), oc.data(), f2.data(), c2.data());
    }
    for (int k = nodes[node].dim_id + 1; k < D; ++k) od[k] = kStarInFwd;
    nodes[node].agg_doc = num_docs;
    append(od.data(), of.data(), oc.data());
  }
};

}  // namespace

struct pgpu_startree_s {
  std::vector<int32_t> dim_columns;
  std::vector<pgpu_agg> metrics;
  std::vector<uint8_t> nodes;                 // LE OffHeapStarTreeNode records
  std::vector<std::vector<uint8_t>> dim_fwd;  // BE fixed-bit
  std::vector<int64_t> dim_fwd_len;
  std::vector<int32_t> dim_bits;
  std::vector<std::vector<double>> mf;
  std::vector<std::vector<int64_t>> mc;
  std::vector<const uint8_t*> fwd_ptrs;
  std::vector<const double*> f_ptrs;
  std::vector<const int64_t*> c_ptrs;
  int32_t num_docs = 0;
  int32_t num_raw_records = 0;                // star-tree records before star-node / aggregated documents
};

extern "C" {

int pgpu_startree_build(const pgpu_segment_desc* seg, const int32_t* column_types, const int32_t* split_order,
                        int32_t num_dims, const int32_t* skip_star_dims, int32_t num_skip, const pgpu_agg* pairs,
                        int32_t num_pairs, int32_t max_leaf_records, pgpu_startree* out) {
  if (!seg || !column_types || !split_order || num_dims < 1 || num_pairs < 1 || !pairs || !out)
    return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad star-tree build arguments");
  const int N = seg->num_docs;
  if (N < 1) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree over an empty segment");
  Builder b;
  b.D = num_dims;
  b.M = num_pairs;
  b.max_leaf = max_leaf_records > 0 ? max_leaf_records : 10000;  // StarTreeV2BuilderConfig.DEFAULT_MAX_LEAF_RECORDS
  b.skip_star.assign(num_dims, 0);
  for (int i = 0; i < num_skip; ++i)
    if (skip_star_dims[i] >= 0 && skip_star_dims[i] < num_dims) b.skip_star[skip_star_dims[i]] = 1;
  auto st = std::make_unique<pgpu_startree_s>();
  // dimension dictIds per doc
  std::vector<int32_t> raw_dims((size_t)N * num_dims);
  for (int d = 0; d < num_dims; ++d) {
    const int c = split_order[d];
    if (c < 0 || c >= seg->num_columns) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad dimension column");
    const pgpu_column_buffers& cb = seg->columns[c];
    if (cb.fwd_format != PGPU_FWD_FIXED_BIT)
      return pgpu::host_fail(PGPU_ERR_UNSUPPORTED, "star-tree dimension must be a fixed-bit column");
    if ((int64_t)(((int64_t)N * cb.bits_per_element + 7) / 8) > cb.fwd_len)
      return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "forward index too short");
    for (int i = 0; i < N; ++i) raw_dims[(size_t)i * num_dims + d] = read_bits(cb.fwd, i, cb.bits_per_element);
    st->dim_columns.push_back(c);
    st->dim_bits.push_back(bits_for(cb.cardinality));
  }
  // raw metric values (PinotSegmentColumnReader.getValue -> Number)
  std::vector<std::vector<double>> raw(num_pairs);
  for (int m = 0; m < num_pairs; ++m) {
    b.fn.push_back(pairs[m].fn);
    st->metrics.push_back(pairs[m]);
    if (pairs[m].fn == PGPU_AGG_COUNT) continue;
    const int c = pairs[m].column;
    if (c < 0 || c >= seg->num_columns) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad metric column");
    const pgpu_column_buffers& cb = seg->columns[c];
    const int t = column_types[c];
    if (t == PGPU_STRING) return pgpu::host_fail(PGPU_ERR_UNSUPPORTED, "numeric star-tree metric required");
    std::vector<double> dv(cb.cardinality);
    for (int i = 0; i < cb.cardinality; ++i) {
      const uint8_t* p = cb.dict + (int64_t)i * cb.entry_width;
      if (t == PGPU_INT) dv[i] = (double)(int32_t)rd_be32(p);
      else if (t == PGPU_LONG) dv[i] = (double)(int64_t)rd_be64(p);
      else if (t == PGPU_FLOAT) { uint32_t u = rd_be32(p); float f; memcpy(&f, &u, 4); dv[i] = f; }
      else { uint64_t u = rd_be64(p); memcpy(&dv[i], &u, 8); }
    }
    raw[m].resize(N);
    if (cb.fwd_format != PGPU_FWD_FIXED_BIT)
      return pgpu::host_fail(PGPU_ERR_UNSUPPORTED, "star-tree metric must be a fixed-bit column");
    for (int i = 0; i < N; ++i) raw[m][i] = dv[read_bits(cb.fwd, i, cb.bits_per_element)];
  }
  // sortAndAggregateSegmentRecords: stable sort by dimensions in split order, merge equal rows in doc order
  std::vector<int> order(N);
  for (int i = 0; i < N; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
    const int32_t* a = &raw_dims[(size_t)x * num_dims];
    const int32_t* c = &raw_dims[(size_t)y * num_dims];
    for (int d = 0; d < num_dims; ++d)
      if (a[d] != c[d]) return a[d] < c[d];
    return false;
  });
  std::vector<double> f(num_pairs);
  std::vector<int64_t> cnt(num_pairs);
  for (size_t i = 0; i < order.size();) {
    const int first = order[i];
    const int32_t* fd = &raw_dims[(size_t)first * num_dims];
    for (int m = 0; m < num_pairs; ++m) {  // ValueAggregator.getInitialAggregatedValue
      f[m] = pairs[m].fn == PGPU_AGG_COUNT ? 0.0 : raw[m][first];
      cnt[m] = (pairs[m].fn == PGPU_AGG_COUNT || pairs[m].fn == PGPU_AGG_AVG) ? 1 : 0;
    }
    size_t j = i + 1;
    for (; j < order.size(); ++j) {
      const int r = order[j];
      if (memcmp(&raw_dims[(size_t)r * num_dims], fd, sizeof(int32_t) * num_dims) != 0) break;
      for (int m = 0; m < num_pairs; ++m) {  // applyRawValue
        switch (pairs[m].fn) {
          case PGPU_AGG_COUNT: cnt[m] += 1; break;
          case PGPU_AGG_SUM: f[m] += raw[m][r]; break;
          case PGPU_AGG_MIN: f[m] = std::min(f[m], raw[m][r]); break;
          case PGPU_AGG_MAX: f[m] = std::max(f[m], raw[m][r]); break;
          default: f[m] += raw[m][r]; cnt[m] += 1; break;
        }
      }
    }
    b.append(fd, f.data(), cnt.data());
    i = j;
  }
  st->num_raw_records = b.num_docs;
  const int root = b.new_node();
  b.construct(root, 0, b.num_docs);
  {
    std::vector<int32_t> od;
    std::vector<double> of;
    std::vector<int64_t> oc;
    b.aggregated(root, od, of, oc);
  }
  // serializeTree: BFS, children sorted by dimension value (ALL = -1 first)
  const int num_nodes = (int)b.nodes.size();
  st->nodes.assign((size_t)num_nodes * 28, 0);
  std::vector<int> queue;
  queue.reserve(num_nodes);
  queue.push_back(root);
  auto put = [&](int64_t off, int32_t v) { memcpy(&st->nodes[off], &v, 4); };  // little-endian host
  for (size_t head = 0; head < queue.size(); ++head) {
    const Node& n = b.nodes[queue[head]];
    int first = kInvalid, last = kInvalid;
    if (n.has_children) {
      std::vector<int> kids = n.children;
      std::sort(kids.begin(), kids.end(), [&](int x, int y) { return b.nodes[x].dim_value < b.nodes[y].dim_value; });
      first = (int)queue.size();
      last = first + (int)kids.size() - 1;
      queue.insert(queue.end(), kids.begin(), kids.end());
    }
    const int64_t off = (int64_t)head * 28;
    put(off + 0, n.dim_id);
    put(off + 4, n.dim_value);
    put(off + 8, n.start);
    put(off + 12, n.end);
    put(off + 16, n.agg_doc);
    put(off + 20, first);
    put(off + 24, last);
  }
  // forward indexes of the star-tree documents
  st->num_docs = b.num_docs;
  for (int d = 0; d < num_dims; ++d) {
    const int bits = st->dim_bits[d];
    const int64_t len = ((int64_t)b.num_docs * bits + 7) / 8;
    std::vector<uint8_t> buf(len + 16, 0);  // tail padding for readers that load past the last value
    for (int i = 0; i < b.num_docs; ++i) write_bits(buf.data(), i, bits, (uint32_t)b.dim_value(i, d));
    st->dim_fwd_len.push_back(len);
    st->dim_fwd.push_back(std::move(buf));
  }
  st->mf.resize(num_pairs);
  st->mc.resize(num_pairs);
  for (int m = 0; m < num_pairs; ++m) {
    const int fnm = pairs[m].fn;
    if (fnm != PGPU_AGG_COUNT) {
      st->mf[m].resize(b.num_docs);
      for (int i = 0; i < b.num_docs; ++i) st->mf[m][i] = b.mf[(size_t)i * num_pairs + m];
    }
    if (fnm == PGPU_AGG_COUNT || fnm == PGPU_AGG_AVG) {
      st->mc[m].resize(b.num_docs);
      for (int i = 0; i < b.num_docs; ++i) st->mc[m][i] = b.mc[(size_t)i * num_pairs + m];
    }
  }
  for (auto& v : st->dim_fwd) st->fwd_ptrs.push_back(v.data());
  for (int m = 0; m < num_pairs; ++m) {
    st->f_ptrs.push_back(st->mf[m].empty() ? nullptr : st->mf[m].data());
    st->c_ptrs.push_back(st->mc[m].empty() ? nullptr : st->mc[m].data());
  }
  *out = st.release();
  return PGPU_OK;
}

int pgpu_startree_get_desc(pgpu_startree st, pgpu_startree_desc* d) {
  if (!st || !d) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "null star-tree");
  d->num_dims = (int32_t)st->dim_columns.size();
  d->num_metrics = (int32_t)st->metrics.size();
  d->num_nodes = (int32_t)(st->nodes.size() / 28);
  d->num_docs = st->num_docs;
  d->dim_columns = st->dim_columns.data();
  d->nodes = st->nodes.data();
  d->dim_fwd = st->fwd_ptrs.data();
  d->dim_fwd_len = st->dim_fwd_len.data();
  d->metrics = st->metrics.data();
  d->metric_f64 = st->f_ptrs.data();
  d->metric_i64 = st->c_ptrs.data();
  return PGPU_OK;
}

int pgpu_startree_num_raw_records(pgpu_startree st, int32_t* n) {
  if (!st || !n) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "null star-tree");
  *n = st->num_raw_records;
  return PGPU_OK;
}

int pgpu_startree_destroy(pgpu_startree st) {
  delete st;
  return PGPU_OK;
}

}  // extern "C"
