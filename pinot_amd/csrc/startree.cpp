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
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>
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

// A fixed-bit forward index of N docs that read_bits may read: 1..31 bits per value, the bytes present, a dictionary.
bool fixed_bit_ok(const pgpu_column_buffers& cb, int64_t N) {
  return cb.bits_per_element >= 1 && cb.bits_per_element <= 31 && cb.cardinality >= 1 && cb.fwd != nullptr &&
         (N * cb.bits_per_element + 7) / 8 <= cb.fwd_len;
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

// ---------------------------------------------------------------------------------------- Pinot's star-tree files
// The star_tree_index file of a segment (StarTreeIndexCombiner.java:55-76: per star-tree the OffHeapStarTree buffer,
// then each split-order dimension's forward index, then each function-column pair's raw forward index) and its
// star_tree_index_map properties (StarTreeIndexMapUtils.java:150-190), read as StarTreeLoaderUtils.loadStarTreeV2
// does (seglocal/startree/v2/store/StarTreeLoaderUtils.java:57-107).
namespace {

inline uint32_t rd_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
inline uint64_t rd_le64(const uint8_t* p) { return (uint64_t)rd_le32(p) | ((uint64_t)rd_le32(p + 4) << 32); }

struct Span {
  int64_t off = -1, size = -1;
};

std::string trim(const std::string& x) {
  size_t a = 0, b = x.size();
  while (a < b && (x[a] == ' ' || x[a] == '\t' || x[a] == '\r')) ++a;
  while (b > a && (x[b - 1] == ' ' || x[b - 1] == '\t' || x[b - 1] == '\r')) --b;
  return x.substr(a, b - a);
}

// "<id>.<column>.<STAR_TREE|FORWARD_INDEX>.<OFFSET|SIZE> = <value>" lines of star-tree `id`; the column may hold
// '.' (StarTreeIndexMapUtils.loadFromFile joins the middle tokens).  Forward indexes come back in file order.
int parse_index_map(const char* text, int64_t len, int id, Span* tree, std::vector<std::pair<std::string, Span>>* fwd) {
  std::vector<std::pair<std::string, Span>> cols;
  const std::string all(text, (size_t)len);
  size_t pos = 0;
  while (pos < all.size()) {
    size_t nl = all.find('\n', pos);
    if (nl == std::string::npos) nl = all.size();
    const std::string line = trim(all.substr(pos, nl - pos));
    pos = nl + 1;
    if (line.empty() || line[0] == '#' || line[0] == '!') continue;
    const size_t eq = line.find_first_of("=:");
    if (eq == std::string::npos) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree index map: bad line '%s'", line.c_str());
    const std::string key = trim(line.substr(0, eq)), val = trim(line.substr(eq + 1));
    const size_t d1 = key.find('.'), d3 = key.rfind('.');
    const size_t d2 = d3 == std::string::npos || d3 == 0 ? std::string::npos : key.rfind('.', d3 - 1);
    if (d1 == std::string::npos || d2 == std::string::npos || d2 <= d1)
      return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree index map: bad key '%s'", key.c_str());
    char* end = nullptr;
    const long tid = strtol(key.c_str(), &end, 10);
    if (end != key.c_str() + d1) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree index map: bad id in '%s'", key.c_str());
    if (tid != id) continue;
    const std::string column = key.substr(d1 + 1, d2 - d1 - 1), type = key.substr(d2 + 1, d3 - d2 - 1);
    const std::string suffix = key.substr(d3 + 1);
    errno = 0;
    const long long v = strtoll(val.c_str(), &end, 10);
    if (errno || end == val.c_str() || *end || v < 0)
      return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree index map: bad value of '%s'", key.c_str());
    Span* sp;
    if (type == "STAR_TREE") {
      sp = tree;
    } else if (type == "FORWARD_INDEX") {
      auto it = std::find_if(cols.begin(), cols.end(), [&](const std::pair<std::string, Span>& e) { return e.first == column; });
      if (it == cols.end()) {
        cols.emplace_back(column, Span());
        it = cols.end() - 1;
      }
      sp = &it->second;
    } else {
      return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree index map: index type '%s'", type.c_str());
    }
    if (suffix == "OFFSET") sp->off = v;
    else if (suffix == "SIZE") sp->size = v;
    else return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree index map: suffix '%s'", suffix.c_str());
  }
  std::sort(cols.begin(), cols.end(), [](const std::pair<std::string, Span>& a, const std::pair<std::string, Span>& b) {
    return a.second.off < b.second.off;
  });
  *fwd = std::move(cols);
  return PGPU_OK;
}

// Header of the chunk forward index (BaseChunkSVForwardIndexReader.java:56-100, versions 2 / 3, PASS_THROUGH):
// returns the start of the chunk-offset table's end (the data) and the entry size / docs per chunk.
struct ChunkHeader {
  int32_t version, num_chunks, per_chunk, entry, total, compression, header_start;
};
int read_chunk_header(const uint8_t* b, int64_t n, const std::string& name, ChunkHeader* h) {
  if (n < 28) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree metric %s: forward index too short", name.c_str());
  h->version = (int32_t)rd_be32(b);
  h->num_chunks = (int32_t)rd_be32(b + 4);
  h->per_chunk = (int32_t)rd_be32(b + 8);
  h->entry = (int32_t)rd_be32(b + 12);
  h->total = (int32_t)rd_be32(b + 16);
  h->compression = (int32_t)rd_be32(b + 20);
  h->header_start = (int32_t)rd_be32(b + 24);
  if (h->version != 2 && h->version != 3)
    return pgpu::host_fail(PGPU_ERR_UNSUPPORTED, "star-tree metric %s: raw forward index version %d", name.c_str(), h->version);
  if (h->compression != 0)
    return pgpu::host_fail(PGPU_ERR_UNSUPPORTED, "star-tree metric %s: compressed chunks (type %d)", name.c_str(), h->compression);
  if (h->num_chunks < 0 || h->per_chunk <= 0 || h->header_start < 28 ||
      h->header_start + (int64_t)h->num_chunks * (h->version == 2 ? 4 : 8) > n)
    return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree metric %s: bad raw forward index header", name.c_str());
  return PGPU_OK;
}

int64_t chunk_position(const uint8_t* b, const ChunkHeader& h, int c) {
  const uint8_t* e = b + h.header_start + (int64_t)c * (h.version == 2 ? 4 : 8);
  return h.version == 2 ? (int64_t)(int32_t)rd_be32(e) : (int64_t)rd_be64(e);
}

// FixedByteChunkSVForwardIndexReader over PASS_THROUGH chunks: value i at data + i * entry (:30-110).
int read_fixed_metric(const uint8_t* b, int64_t n, int32_t num_docs, int32_t entry, const std::string& name,
                      std::vector<uint64_t>* out) {
  ChunkHeader h;
  if (int rc = read_chunk_header(b, n, name, &h)) return rc;
  if (h.entry != entry)
    return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree metric %s: entry size %d, expected %d", name.c_str(), h.entry, entry);
  const int64_t data = h.header_start + (int64_t)h.num_chunks * (h.version == 2 ? 4 : 8);
  if (h.total < num_docs || (int64_t)h.num_chunks * h.per_chunk < num_docs || data + (int64_t)num_docs * entry > n)
    return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree metric %s: covers fewer than %d documents", name.c_str(), num_docs);
  out->resize(num_docs);
  for (int32_t i = 0; i < num_docs; ++i) (*out)[i] = rd_be64(b + data + (int64_t)i * 8);
  return PGPU_OK;
}

// VarByteChunkSVForwardIndexReader over PASS_THROUGH chunks (:104-190): per chunk numDocsPerChunk int offsets of
// its rows, then the bytes; AVG's values are AvgPair.toBytes (double sum, long count; AvgPair.java:53-68).
int read_avg_metric(const uint8_t* b, int64_t n, int32_t num_docs, const std::string& name, std::vector<double>* sum,
                    std::vector<int64_t>* cnt) {
  ChunkHeader h;
  if (int rc = read_chunk_header(b, n, name, &h)) return rc;
  if ((int64_t)h.num_chunks * h.per_chunk < num_docs)
    return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree metric %s: covers fewer than %d documents", name.c_str(), num_docs);
  sum->resize(num_docs);
  cnt->resize(num_docs);
  for (int32_t i = 0; i < num_docs; ++i) {
    const int c = i / h.per_chunk, r = i % h.per_chunk;
    const int64_t cs = chunk_position(b, h, c);
    if (cs < 0 || cs + (int64_t)(r + 1) * 4 > n) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree metric %s: chunk overrun", name.c_str());
    const int64_t vs = cs + (int32_t)rd_be32(b + cs + (int64_t)r * 4);
    if (vs < cs || vs + 16 > n)
      return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree metric %s: value of document %d out of range", name.c_str(), i);
    const uint64_t u = rd_be64(b + vs);
    double d;
    memcpy(&d, &u, 8);
    (*sum)[i] = d;
    (*cnt)[i] = (int64_t)rd_be64(b + vs + 8);
  }
  return PGPU_OK;
}

}  // namespace

extern "C" {

int pgpu_startree_load(const void* index, int64_t index_len, const char* index_map, int64_t index_map_len,
                       int32_t star_tree_id, int32_t num_docs, int32_t num_columns, const char* const* column_names,
                       const int32_t* bits_per_element, pgpu_startree* out) try {
  if (!index || index_len < 0 || !index_map || index_map_len < 0 || num_docs < 0 || num_columns < 1 || !column_names ||
      !bits_per_element || !out)
    return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad star-tree load arguments");
  const uint8_t* base = static_cast<const uint8_t*>(index);
  Span tree;
  std::vector<std::pair<std::string, Span>> fwd;
  if (int rc = parse_index_map(index_map, index_map_len, star_tree_id, &tree, &fwd)) return rc;
  // offsets and sizes come from the text of the index map (up to LLONG_MAX each): compared without an add that
  // could overflow
  auto in_file = [&](const Span& sp) {
    return sp.off >= 0 && sp.size >= 0 && index_len >= 0 && sp.off <= index_len && sp.size <= index_len - sp.off;
  };
  if (!in_file(tree))
    return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree %d: no STAR_TREE entry inside the index file", star_tree_id);
  // OffHeapStarTree header, little-endian (OffHeapStarTree.java:45-80; StarTreeBuilderUtils.java:118-171)
  const uint8_t* tb = base + tree.off;
  const int64_t tn = tree.size;
  if (tn < 24 || rd_le64(tb) != 0xBADDA55B00DAD00DULL)
    return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "Invalid magic marker in star-tree data buffer");
  if (rd_le32(tb + 8) != 1) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "Invalid version in star-tree data buffer");
  const int64_t root = (int32_t)rd_le32(tb + 12);
  const int32_t nd = (int32_t)rd_le32(tb + 16);
  if (nd < 1 || nd > 16) return pgpu::host_fail(PGPU_ERR_UNSUPPORTED, "star-tree with %d dimensions (1..16)", nd);
  int64_t off = 20;
  std::vector<std::string> dims(nd);
  std::vector<int> seen(nd, 0);
  for (int i = 0; i < nd; ++i) {
    if (off + 8 > tn) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree header truncated");
    const int32_t id = (int32_t)rd_le32(tb + off), nb = (int32_t)rd_le32(tb + off + 4);
    off += 8;
    if (id < 0 || id >= nd || seen[id] || nb < 0 || off + nb > tn)
      return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree header: bad dimension entry %d", i);
    seen[id] = 1;
    dims[id].assign(reinterpret_cast<const char*>(tb + off), (size_t)nb);
    off += nb;
  }
  if (off + 4 > tn) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree header truncated");
  const int32_t num_nodes = (int32_t)rd_le32(tb + off);
  off += 4;
  if (off != root) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "Error loading star-tree, header length mis-match");
  if (num_nodes < 1 || off + (int64_t)num_nodes * 28 != tn)
    return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "Error loading star-tree, buffer size mis-match");
  auto st = std::make_unique<pgpu_startree_s>();
  st->num_docs = num_docs;
  st->nodes.assign(tb + off, tb + tn);
  // dimensions: split order = header order; forward indexes BIG_ENDIAN fixed-bit with the segment column's bits
  for (int i = 0; i < nd; ++i) {
    int col = -1;
    for (int c = 0; c < num_columns; ++c)
      if (column_names[c] && dims[i] == column_names[c]) col = c;
    if (col < 0) return pgpu::host_fail(PGPU_ERR_NOT_FOUND, "star-tree dimension '%s' is not a table column", dims[i].c_str());
    auto it = std::find_if(fwd.begin(), fwd.end(), [&](const std::pair<std::string, Span>& e) { return e.first == dims[i]; });
    if (it == fwd.end() || !in_file(it->second))
      return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree dimension '%s': no forward index", dims[i].c_str());
    const int bits = bits_per_element[col];
    const int64_t need = ((int64_t)num_docs * bits + 7) / 8;
    if (bits < 1 || bits > 31 || it->second.size < need)
      return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree dimension '%s': forward index too short", dims[i].c_str());
    std::vector<uint8_t> buf(base + it->second.off, base + it->second.off + need);
    buf.resize(need + 16, 0);
    st->dim_columns.push_back(col);
    st->dim_bits.push_back(bits);
    st->dim_fwd_len.push_back(need);
    st->dim_fwd.push_back(std::move(buf));
  }
  // function-column pairs "<fn>__<col>" (AggregationFunctionColumnPair.java:50-66); value types per
  // ValueAggregatorFactory.getAggregatedValueType: COUNT LONG, SUM / MIN / MAX DOUBLE, AVG BYTES (AvgPair)
  for (const auto& e : fwd) {
    if (std::find(dims.begin(), dims.end(), e.first) != dims.end()) continue;
    const size_t sep = e.first.find("__");
    if (sep == std::string::npos) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree metric '%s'", e.first.c_str());
    const std::string fn = e.first.substr(0, sep), colname = e.first.substr(sep + 2);
    int f = -1;
    if (fn == "count") f = PGPU_AGG_COUNT;
    else if (fn == "sum") f = PGPU_AGG_SUM;
    else if (fn == "min") f = PGPU_AGG_MIN;
    else if (fn == "max") f = PGPU_AGG_MAX;
    else if (fn == "avg") f = PGPU_AGG_AVG;
    if (f < 0) continue;  // pairs of other functions (distinctCountHLL, percentileEst, ...): never fit a GPU query
    int col = -1;
    if (f != PGPU_AGG_COUNT) {
      for (int c = 0; c < num_columns; ++c)
        if (column_names[c] && colname == column_names[c]) col = c;
      if (col < 0) return pgpu::host_fail(PGPU_ERR_NOT_FOUND, "star-tree metric '%s': no such column", e.first.c_str());
    }
    if (!in_file(e.second)) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "star-tree metric '%s' outside the file", e.first.c_str());
    const uint8_t* mb = base + e.second.off;
    std::vector<double> mf;
    std::vector<int64_t> mc;
    if (f == PGPU_AGG_AVG) {
      if (int rc = read_avg_metric(mb, e.second.size, num_docs, e.first, &mf, &mc)) return rc;
    } else {
      std::vector<uint64_t> w;
      if (int rc = read_fixed_metric(mb, e.second.size, num_docs, 8, e.first, &w)) return rc;
      if (f == PGPU_AGG_COUNT) {
        mc.resize(num_docs);
        for (int32_t i = 0; i < num_docs; ++i) mc[i] = (int64_t)w[i];
      } else {
        mf.resize(num_docs);
        for (int32_t i = 0; i < num_docs; ++i) memcpy(&mf[i], &w[i], 8);
      }
    }
    st->metrics.push_back(pgpu_agg{f, col});
    st->mf.push_back(std::move(mf));
    st->mc.push_back(std::move(mc));
  }
  if (st->metrics.empty())
    return pgpu::host_fail(PGPU_ERR_UNSUPPORTED, "star-tree %d has no COUNT / SUM / MIN / MAX / AVG pair", star_tree_id);
  for (auto& v : st->dim_fwd) st->fwd_ptrs.push_back(v.data());
  for (size_t m = 0; m < st->metrics.size(); ++m) {
    st->f_ptrs.push_back(st->mf[m].empty() ? nullptr : st->mf[m].data());
    st->c_ptrs.push_back(st->mc[m].empty() ? nullptr : st->mc[m].data());
  }
  st->num_raw_records = -1;  // not recorded in the files
  *out = st.release();
  return PGPU_OK;
} PGPU_ABI_CATCH

int pgpu_startree_build(const pgpu_segment_desc* seg, const int32_t* column_types, const int32_t* split_order,
                        int32_t num_dims, const int32_t* skip_star_dims, int32_t num_skip, const pgpu_agg* pairs,
                        int32_t num_pairs, int32_t max_leaf_records, pgpu_startree* out) try {
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
    if (!fixed_bit_ok(cb, N)) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad dimension forward index");
    for (int i = 0; i < N; ++i) {
      const int32_t id = read_bits(cb.fwd, i, cb.bits_per_element);
      if (id < 0 || id >= cb.cardinality) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "dictId past the dictionary");
      raw_dims[(size_t)i * num_dims + d] = id;
    }
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
    if (cb.fwd_format != PGPU_FWD_FIXED_BIT)
      return pgpu::host_fail(PGPU_ERR_UNSUPPORTED, "star-tree metric must be a fixed-bit column");
    const int width = t == PGPU_INT || t == PGPU_FLOAT ? 4 : 8;
    if (!fixed_bit_ok(cb, N) || cb.entry_width < width || !cb.dict ||
        (int64_t)cb.cardinality * cb.entry_width > cb.dict_len)
      return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad metric column buffers");
    std::vector<double> dv(cb.cardinality);
    for (int i = 0; i < cb.cardinality; ++i) {
      const uint8_t* p = cb.dict + (int64_t)i * cb.entry_width;
      if (t == PGPU_INT) dv[i] = (double)(int32_t)rd_be32(p);
      else if (t == PGPU_LONG) dv[i] = (double)(int64_t)rd_be64(p);
      else if (t == PGPU_FLOAT) { uint32_t u = rd_be32(p); float f; memcpy(&f, &u, 4); dv[i] = f; }
      else { uint64_t u = rd_be64(p); memcpy(&dv[i], &u, 8); }
    }
    raw[m].resize(N);
    for (int i = 0; i < N; ++i) {
      const int32_t id = read_bits(cb.fwd, i, cb.bits_per_element);
      if (id < 0 || id >= cb.cardinality) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "dictId past the dictionary");
      raw[m][i] = dv[id];
    }
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
} PGPU_ABI_CATCH

int pgpu_startree_get_desc(pgpu_startree st, pgpu_startree_desc* d) try {
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
} PGPU_ABI_CATCH

int pgpu_startree_num_raw_records(pgpu_startree st, int32_t* n) try {
  if (!st || !n) return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "null star-tree");
  *n = st->num_raw_records;
  return PGPU_OK;
} PGPU_ABI_CATCH

int pgpu_startree_destroy(pgpu_startree st) try {
  delete st;
  return PGPU_OK;
} PGPU_ABI_CATCH

}  // extern "C"
