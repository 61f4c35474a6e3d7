// server_response.cpp — what a Pinot server does with a combined group-by result after the GPU path, and the
// broker's reduce of the servers' responses:
//   - SQL-mode server trim (GroupByOrderByCombineOperator + IndexedTable.finish, core/operator/combine/
//     GroupByOrderByCombineOperator.java:82-97, core/data/table/IndexedTable.java:62-89, TableResizer.java:224-260);
//   - PQL-mode trim (AggregationGroupByTrimmingService.java:54-120, also the broker's trimFinalResults);
//   - the server response bytes (IntermediateResultsBlock.getResultDataTable, core/operator/blocks/
//     IntermediateResultsBlock.java:329-345, DataTableBuilder.java:55-103, DataTableImplV3.toBytes :183-290);
//   - the broker's GroupByDataTableReducer for SQL (core/query/reduce/GroupByDataTableReducer.java:290-330): merge
//     the servers' tables by key, ORDER BY, LIMIT, final results.
// All of it runs on the host over the compacted result (hundreds of rows to millions): it is the step after the
// device path, in the same native library.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <limits>
#include <map>
#include <numeric>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/pinotgpu.h"
#include "host_common.h"
#include "host_result.h"

using namespace pgpu;

namespace {

enum { RC_I64 = 0, RC_F64 = 1, RC_KEY_F64 = 2 };

double key_to_double(uint64_t w) {
  int64_t k = (int64_t)w;
  int64_t b = k >= 0 ? k : (k ^ INT64_MAX);
  double d;
  memcpy(&d, &b, 8);
  return d;
}

// Intermediate value of aggregation a at row i as Pinot's holders keep it (COUNT: long; SUM / MIN / MAX: double;
// AVG: AvgPair.sum -- its count is the COUNT row).
double agg_double(const pgpu_result_s* R, int a, int64_t i) {
  if (R->agg_fn[a] == PGPU_AGG_COUNT) return (double)(int64_t)const_cast<pgpu_result_s*>(R)->slot(0)[i];
  const uint64_t w = const_cast<pgpu_result_s*>(R)->slot(R->agg_slot[a])[i];
  switch (R->agg_conv[a]) {
    case RC_I64: return (double)(int64_t)w;
    case RC_F64: { double d; memcpy(&d, &w, 8); return d; }
    default: return key_to_double(w);
  }
}
int64_t row_count(const pgpu_result_s* R, int64_t i) { return (int64_t)const_cast<pgpu_result_s*>(R)->slot(0)[i]; }

// AggregationFunction.extractFinalResult: AVG = sum / count (-inf for no docs, AvgAggregationFunction.java:185-192).
double agg_final(const pgpu_result_s* R, int a, int64_t i) {
  const double v = agg_double(R, a, i);
  if (R->agg_fn[a] != PGPU_AGG_AVG) return v;
  const int64_t c = row_count(R, i);
  return c ? v / (double)c : -INFINITY;
}

// Double.compare order (NaN last; -0.0 < 0.0).
int dcmp(double a, double b) {
  if (a < b) return -1;
  if (a > b) return 1;
  int64_t x, y;
  memcpy(&x, &a, 8);
  memcpy(&y, &b, 8);
  return x == y ? 0 : (x < y ? -1 : 1);
}

// Ascending composite-key order of two rows (group-by column 0 least significant, the mixed-radix key of
// DictionaryBasedGroupKeyGenerator.java:276-323 over table-global dictIds).  Dense results come back in that order
// already, but hash-mode results of 4096 groups and more come in partition / hash order (the LONG_MAP holder's
// iteration order), so every consumer that depends on an order compares the keys, not the row indexes.
struct KeyOrder {
  std::vector<const int32_t*> g;
  explicit KeyOrder(const pgpu_result_s* R) {
    pgpu_result_s* S = const_cast<pgpu_result_s*>(R);
    for (int j = 0; j < R->num_keys; ++j) g.push_back(S->gid(j));
  }
  bool less(int64_t x, int64_t y) const {
    for (int j = (int)g.size() - 1; j >= 0; --j)
      if (g[j][x] != g[j][y]) return g[j][x] < g[j][y];
    return x < y;
  }
};

// TableResizer's comparator over ORDER BY expressions (group-by column: dictId order = value order of the sorted
// global dictionary; aggregation: its final result).  Ties fall back to the composite-key order, so the choice among
// equal records -- thread-order dependent in Pinot -- is deterministic here.
struct RowOrder {
  const pgpu_result_s* R;
  std::vector<pgpu_order_by> ob;
  KeyOrder key{R};
  bool less(int64_t x, int64_t y) const {
    for (const pgpu_order_by& o : ob) {
      int c;
      if (o.kind == PGPU_ORDER_GROUP_BY) {
        const int32_t* g = const_cast<pgpu_result_s*>(R)->gid(o.index);
        c = g[x] < g[y] ? -1 : (g[x] > g[y] ? 1 : 0);
      } else {
        c = dcmp(agg_final(R, o.index, x), agg_final(R, o.index, y));
      }
      if (c) return o.ascending ? c < 0 : c > 0;
    }
    return key.less(x, y);
  }
};

// Top `k` rows of [0, n) in comparator order (sorted).
std::vector<int64_t> top_rows(int64_t n, int64_t k, const std::function<bool(int64_t, int64_t)>& less) {
  std::vector<int64_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  if (k < n) {
    std::nth_element(idx.begin(), idx.begin() + k, idx.end(), less);
    idx.resize(k);
  }
  std::sort(idx.begin(), idx.end(), less);
  return idx;
}

int copy_rows(const pgpu_result_s* R, const std::vector<int64_t>& rows, pgpu_result* out) {
  auto* O = new pgpu_result_s();
  O->pool = R->pool;
  const int64_t m = (int64_t)rows.size();
  int rc = O->alloc(R->num_keys, R->num_slots, m);
  if (rc) { delete O; return rc; }
  pgpu_result_s* S = const_cast<pgpu_result_s*>(R);
  for (int j = 0; j < R->num_keys; ++j)
    for (int64_t r = 0; r < m; ++r) O->gid(j)[r] = S->gid(j)[rows[r]];
  for (int s = 0; s < R->num_slots; ++s)
    for (int64_t r = 0; r < m; ++r) O->slot(s)[r] = S->slot(s)[rows[r]];
  O->num_aggs = R->num_aggs;
  O->agg_slot = R->agg_slot;
  O->agg_conv = R->agg_conv;
  memcpy(O->stats, R->stats, sizeof O->stats);
  O->key_cols = R->key_cols;
  O->key_types = R->key_types;
  O->agg_fn = R->agg_fn;
  O->agg_col = R->agg_col;
  O->groups_limit_reached = R->groups_limit_reached;
  O->key_dicts = R->key_dicts;
  *out = O;
  return 0;
}

// ------------------------------------------------------------------------------------------------ bytes
struct Out {
  std::vector<uint8_t> b;
  void i32(int32_t v) { for (int k = 3; k >= 0; --k) b.push_back((uint8_t)((uint32_t)v >> (8 * k))); }
  void i64(int64_t v) { for (int k = 7; k >= 0; --k) b.push_back((uint8_t)((uint64_t)v >> (8 * k))); }
  void f64(double d) { int64_t v; memcpy(&v, &d, 8); i64(v); }
  void str(const std::string& s) { i32((int32_t)s.size()); b.insert(b.end(), s.begin(), s.end()); }
  void raw(const std::vector<uint8_t>& x) { b.insert(b.end(), x.begin(), x.end()); }
};
struct In {
  const uint8_t* p;
  int64_t n, pos = 0;
  bool ok = true;
  bool need(int64_t k) { if (pos < 0 || k < 0 || pos > n || k > n - pos) ok = false; return ok; }
  int32_t i32() { if (!need(4)) return 0; uint32_t v = 0; for (int k = 0; k < 4; ++k) v = v << 8 | p[pos++]; return (int32_t)v; }
  int64_t i64() { if (!need(8)) return 0; uint64_t v = 0; for (int k = 0; k < 8; ++k) v = v << 8 | p[pos++]; return (int64_t)v; }
  double f64() { int64_t v = i64(); double d; memcpy(&d, &v, 8); return d; }
  std::string str() { int32_t l = i32(); if (!need(l)) return std::string(); std::string s((const char*)p + pos, l); pos += l; return s; }
  // a wire count of entries of at least `each` bytes: no larger than what is left (a corrupt count must not size an
  // allocation before the reads behind it fail)
  bool count(int32_t c, int64_t each) { if (c < 0 || (int64_t)c * each > n - pos) ok = false; return ok; }
};

// Java long addition (two's complement wrap-around): CountAggregationFunction.merge and the broker's statistics sums.
inline int64_t java_add(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }

// java.lang.String.hashCode over UTF-16 units (the names here are ASCII) and java.util.HashMap's iteration order
// (bucket (h ^ h >>> 16) & (capacity - 1), insertion order within a bucket, capacity 16 doubling past 0.75 load):
// the metadata and dictionary-map sections are serialized in that order, so the bytes match the reference's.
uint32_t java_hash(const std::string& s) {
  uint32_t h = 0;  // int arithmetic mod 2^32
  for (unsigned char c : s) h = 31u * h + (uint32_t)c;
  return h;
}
std::vector<size_t> java_hashmap_order(const std::vector<std::string>& keys) {
  size_t cap = 16;
  while ((double)keys.size() > 0.75 * (double)cap) cap <<= 1;
  std::vector<std::pair<uint32_t, size_t>> v;
  for (size_t i = 0; i < keys.size(); ++i) {
    const uint32_t h = java_hash(keys[i]);
    v.push_back({(h ^ (h >> 16)) & (uint32_t)(cap - 1), i});
  }
  std::stable_sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  std::vector<size_t> out;
  for (auto& e : v) out.push_back(e.second);
  return out;
}

// DataSchema.ColumnDataType names (pinot-common/.../DataSchema.java:247-265).
const char* column_type_name(int t) {
  switch (t) {
    case PGPU_INT: return "INT";
    case PGPU_LONG: return "LONG";
    case PGPU_FLOAT: return "FLOAT";
    case PGPU_DOUBLE: return "DOUBLE";
    default: return "STRING";
  }
}
const char* fn_name(int fn) {
  switch (fn) {
    case PGPU_AGG_COUNT: return "count";
    case PGPU_AGG_SUM: return "sum";
    case PGPU_AGG_MIN: return "min";
    case PGPU_AGG_MAX: return "max";
    default: return "avg";
  }
}
constexpr int kObjectTypeAvgPair = 4;  // ObjectSerDeUtils.ObjectType.AvgPair

// DataTable.MetadataKey ordinals and value types (pinot-common/.../common/utils/DataTable.java:90-110; every key a
// reference server may attach, e.g. requestId from InstanceRequestHandler / QueryScheduler, is decoded).
struct MetaKey { const char* name; int ordinal; int kind; };  // kind 0 string, 1 int, 2 long
const MetaKey kMetaKeys[] = {
    {"unknown", 0, 0}, {"table", 1, 0}, {"numDocsScanned", 2, 2}, {"numEntriesScannedInFilter", 3, 2},
    {"numEntriesScannedPostFilter", 4, 2}, {"numSegmentsQueried", 5, 1}, {"numSegmentsProcessed", 6, 1},
    {"numSegmentsMatched", 7, 1}, {"numConsumingSegmentsProcessed", 8, 1}, {"minConsumingFreshnessTimeMs", 9, 2},
    {"totalDocs", 10, 2}, {"numGroupsLimitReached", 11, 0}, {"timeUsedMs", 12, 2}, {"traceInfo", 13, 0},
    {"requestId", 14, 2}, {"numResizes", 15, 1}, {"resizeTimeMs", 16, 2}, {"threadCpuTimeNs", 17, 2},
    {"systemActivitiesCpuTimeNs", 18, 2}, {"responseSerializationCpuTimeNs", 19, 2}};
const MetaKey* meta_by_name(const std::string& n) {
  for (const MetaKey& k : kMetaKeys) if (n == k.name) return &k;
  return nullptr;
}
const MetaKey* meta_by_ordinal(int o) {
  for (const MetaKey& k : kMetaKeys) if (o == k.ordinal) return &k;
  return nullptr;
}

// One server table as the broker reads it.
struct Table {
  std::vector<std::string> names, types;
  int64_t rows = 0;
  std::vector<std::vector<uint8_t>> cells;  // per row: fixed-size bytes
  std::vector<int> offsets;
  int row_size = 0;
  std::map<std::string, std::unordered_map<int32_t, std::string>> dict;
  std::vector<uint8_t> var;
  std::map<std::string, std::string> meta;
};

int type_size(const std::string& t) {
  if (t == "INT" || t == "STRING") return 4;
  return 8;  // LONG, FLOAT (8 for backward compatibility, DataTableUtils.java:74-78), DOUBLE, OBJECT
}

bool parse_table(const uint8_t* p, int64_t n, Table* T, std::string* err) {
  In in{p, n};
  const int32_t version = in.i32();
  if (version != 3) { *err = "not a DataTable V3 (version " + std::to_string(version) + ")"; return false; }
  T->rows = in.i32();
  const int32_t ncols = in.i32();
  int32_t sec[10];
  for (int k = 0; k < 10; ++k) sec[k] = in.i32();
  if (!in.ok) { *err = "truncated header"; return false; }
  if (T->rows < 0 || ncols < 0) { *err = "negative row / column count"; return false; }
  // every section lies inside the bytes (offsets and lengths come from the wire: negative ones are rejected)
  for (int k = 0; k < 5; ++k)
    if (sec[2 * k] < 0 || sec[2 * k + 1] < 0 || (int64_t)sec[2 * k] + sec[2 * k + 1] > n) {
      *err = "section " + std::to_string(k) + " outside the DataTable bytes";
      return false;
    }
  auto section = [&](int k) { return In{p + sec[2 * k], sec[2 * k + 1]}; };
  In ex = section(0);
  if (sec[1]) {
    const int32_t ne = ex.i32();
    if (ne) { *err = "server exceptions present"; return false; }
  }
  if (sec[3]) {
    In d = section(1);
    const int32_t nd = d.i32();
    d.count(nd, 8);
    for (int i = 0; i < nd && d.ok; ++i) {
      const std::string col = d.str();
      const int32_t sz = d.i32();
      if (!d.count(sz, 8)) break;
      auto& m = T->dict[col];
      for (int j = 0; j < sz && d.ok; ++j) { const int32_t key = d.i32(); m[key] = d.str(); }
    }
    if (!d.ok) { *err = "bad dictionary section"; return false; }
  }
  if (sec[5]) {
    In s = section(2);
    const int32_t nc = s.i32();
    s.count(nc, 8);
    for (int i = 0; i < nc && s.ok; ++i) T->names.push_back(s.str());
    for (int i = 0; i < nc && s.ok; ++i) T->types.push_back(s.str());
    if (!s.ok || nc != ncols) { *err = "bad data schema"; return false; }
  }
  for (const auto& t : T->types) { T->offsets.push_back(T->row_size); T->row_size += type_size(t); }
  if (sec[7]) {
    if ((int64_t)sec[7] != T->rows * T->row_size || sec[6] + (int64_t)sec[7] > n) { *err = "bad fixed-size section"; return false; }
    for (int64_t r = 0; r < T->rows; ++r)
      T->cells.emplace_back(p + sec[6] + r * T->row_size, p + sec[6] + (r + 1) * T->row_size);
  }
  if ((int64_t)T->cells.size() != T->rows) { *err = "rows without a fixed-size section"; return false; }
  if (sec[9]) T->var.assign(p + sec[8], p + sec[8] + sec[9]);
  // metadata follows the sections
  In m{p, n};
  m.pos = std::max<int64_t>({(int64_t)13 * 4, (int64_t)sec[0] + sec[1], (int64_t)sec[2] + sec[3], (int64_t)sec[4] + sec[5],
                             (int64_t)sec[6] + sec[7], (int64_t)sec[8] + sec[9]});
  const int32_t ml = m.i32();
  if (!m.ok || ml < 0 || m.pos + (int64_t)ml > n) { *err = "bad metadata"; return false; }
  In md{p + m.pos, ml};
  const int32_t ne = md.i32();
  md.count(ne, 8);
  for (int i = 0; i < ne && md.ok; ++i) {
    const int32_t ord = md.i32();
    const MetaKey* k = meta_by_ordinal(ord);
    if (!k) continue;  // DataTableImplV3.deserializeMetadata ignores keys it does not know (:361-365)
    if (k->kind == 1) T->meta[k->name] = std::to_string(md.i32());
    else if (k->kind == 2) T->meta[k->name] = std::to_string(md.i64());
    else T->meta[k->name] = md.str();
  }
  if (!md.ok) { *err = "bad metadata"; return false; }
  return true;
}

// A typed cell value (keys compare by value; aggregations merge per function).
struct Cell {
  int kind = 0;  // 0 int64, 1 double, 2 string, 3 AvgPair
  int64_t i = 0;
  double d = 0, c = 0;
  std::string s;
};

void json_double(std::string& o, double d) {
  char buf[64];
  // Jackson writes non-finite doubles as strings ("NaN", "Infinity", "-Infinity"); bare nan / inf is not JSON
  if (std::isnan(d)) { o += "\"NaN\""; return; }
  if (std::isinf(d)) { o += d < 0 ? "\"-Infinity\"" : "\"Infinity\""; return; }
  snprintf(buf, sizeof buf, "%.17g", d);
  o += buf;
}
void json_str(std::string& o, const std::string& s) {
  o += '"';
  for (unsigned char ch : s) {
    if (ch == '"' || ch == '\\') { o += '\\'; o += (char)ch; }
    else if (ch < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", ch); o += b; }
    else o += (char)ch;
  }
  o += '"';
}

}  // namespace

// ================================================================================================ C ABI
extern "C" {

int pgpu_result_trim_sql(pgpu_result r, const pgpu_sql_trim* spec, pgpu_result* out) try {
  if (!r || !spec || !out || spec->num_order_by < 0 || (spec->num_order_by && !spec->order_by) || spec->limit < 0)
    return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  if (r->compact.load(std::memory_order_acquire))
    if (const int rc = pgpu::result_expand(r)) return rc;  // compact results: columnar form first
  for (int i = 0; i < spec->num_order_by; ++i) {
    const pgpu_order_by& o = spec->order_by[i];
    const int lim = o.kind == PGPU_ORDER_GROUP_BY ? r->num_keys : r->num_aggs;
    if ((o.kind != PGPU_ORDER_GROUP_BY && o.kind != PGPU_ORDER_AGGREGATION) || o.index < 0 || o.index >= lim)
      return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad ORDER BY expression %d", i);
  }
  const int64_t n = r->n;
  std::vector<int64_t> rows;
  if (spec->min_server_group_trim_size <= 0) {
    // server trim disabled (UnboundedConcurrentIndexedTable): every group, sorted when there is an ORDER BY
    RowOrder ord{r, std::vector<pgpu_order_by>(spec->order_by, spec->order_by + spec->num_order_by)};
    rows = top_rows(n, n, [&](int64_t x, int64_t y) { return ord.less(x, y); });
  } else if (spec->num_order_by > 0) {
    // ConcurrentIndexedTable(resultSize = trimSize): the top max(limit * 5, minServerGroupTrimSize) records
    const int64_t trim = std::max<int64_t>((int64_t)spec->limit * 5, spec->min_server_group_trim_size);
    RowOrder ord{r, std::vector<pgpu_order_by>(spec->order_by, spec->order_by + spec->num_order_by)};
    rows = top_rows(n, std::min(trim, n), [&](int64_t x, int64_t y) { return ord.less(x, y); });
  } else {
    // no ORDER BY: the table stops taking new keys at `limit` groups (which ones is thread-order dependent in
    // Pinot; here the smallest composite keys, whatever order the result holds its rows in)
    const KeyOrder key(r);
    rows = top_rows(n, std::min<int64_t>(spec->limit, n), [&](int64_t x, int64_t y) { return key.less(x, y); });
  }
  return copy_rows(r, rows, out);
} PGPU_ABI_CATCH

int pgpu_result_trim_pql(pgpu_result r, int32_t limit, int32_t final_results, int64_t* rows, int64_t cap,
                         int64_t* counts) try {
  if (!r || !counts || limit <= 0) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  if (r->compact.load(std::memory_order_acquire))
    if (const int rc = pgpu::result_expand(r)) return rc;  // compact results: columnar form first
  // AggregationGroupByTrimmingService: trimSize = max(limit * 5, 5000), applied past 4 x trimSize groups;
  // trimFinalResults (broker): the top `limit` of each function
  const int64_t trim = final_results ? limit : std::max<int64_t>((int64_t)limit * 5, 5000);
  const bool apply = final_results || r->n > 4 * trim;
  const int64_t k = apply ? std::min<int64_t>(trim, r->n) : r->n;
  for (int a = 0; a < r->num_aggs; ++a) {
    counts[a] = k;
    if (!rows) continue;
    if (cap < k) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "row buffer too small (%lld < %lld)", (long long)cap,
                                  (long long)k);
    // MIN keeps the smallest values, every other function the largest (getSorter, :162-181); ties by key
    const bool min_order = r->agg_fn[a] == PGPU_AGG_MIN;
    const KeyOrder key(r);
    std::vector<int64_t> top = top_rows(r->n, k, [&](int64_t x, int64_t y) {
      const int c = dcmp(agg_final(r, a, x), agg_final(r, a, y));
      if (c) return min_order ? c < 0 : c > 0;
      return key.less(x, y);
    });
    std::copy(top.begin(), top.end(), rows + (int64_t)a * cap);
  }
  return 0;
} PGPU_ABI_CATCH

int pgpu_result_datatable(pgpu_result r, pgpu_table t, void* out, int64_t cap, int64_t* len) try {
  if (!r || !t || !len) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  if (r->compact.load(std::memory_order_acquire))
    if (const int rc = pgpu::result_expand(r)) return rc;  // compact results: columnar form first
  const int nk = r->num_keys, na = r->num_aggs, nc = nk + na;
  std::vector<DictView> dv(nk);
  std::vector<std::string> names, types;
  std::vector<int> tsz;
  for (int j = 0; j < nk; ++j) {
    if (result_key_dict_view(r, t, j, &dv[j])) return PGPU_ERR_INVALID_ARGUMENT;
    names.push_back(dv[j].name);  // ExpressionContext.toString of an identifier
    types.push_back(column_type_name(r->key_types[j]));
  }
  for (int a = 0; a < na; ++a) {  // AggregationFunction.getResultColumnName / getIntermediateResultColumnType
    std::string arg = "*";
    if (r->agg_col[a] >= 0) {
      DictView v;
      if (table_dict_view(t, r->agg_col[a], &v)) return PGPU_ERR_INVALID_ARGUMENT;
      arg = v.name;
    }
    names.push_back(std::string(fn_name(r->agg_fn[a])) + "(" + arg + ")");
    types.push_back(r->agg_fn[a] == PGPU_AGG_COUNT ? "LONG" : r->agg_fn[a] == PGPU_AGG_AVG ? "OBJECT" : "DOUBLE");
  }
  for (const auto& ty : types) tsz.push_back(type_size(ty));
  // fixed-size rows, string dictionaries (ids in first-use order, DataTableBuilder.setColumn(String)), objects
  Out fixed, var;
  std::vector<std::unordered_map<int32_t, int32_t>> sid(nk);  // global dictId -> table dictId
  std::vector<std::vector<int32_t>> sorder(nk);
  for (int64_t i = 0; i < r->n; ++i) {
    for (int j = 0; j < nk; ++j) {
      const int32_t g = r->gid(j)[i];
      switch (r->key_types[j]) {
        case PGPU_INT: fixed.i32((int32_t)(*dv[j].iv)[g]); break;
        case PGPU_LONG: fixed.i64((*dv[j].iv)[g]); break;
        case PGPU_FLOAT: {  // putFloat: 4 bytes, then the slot's 4 unused (zero) bytes (DataTableUtils.java:74-78)
          const float f = (float)(*dv[j].dv)[g];
          int32_t bits;
          memcpy(&bits, &f, 4);
          fixed.i32(bits);
          fixed.i32(0);
          break;
        }
        case PGPU_DOUBLE: fixed.f64((*dv[j].dv)[g]); break;
        default: {
          auto it = sid[j].find(g);
          if (it == sid[j].end()) {
            it = sid[j].emplace(g, (int32_t)sorder[j].size()).first;
            sorder[j].push_back(g);
          }
          fixed.i32(it->second);
        }
      }
    }
    for (int a = 0; a < na; ++a) {
      if (r->agg_fn[a] == PGPU_AGG_COUNT) { fixed.i64(row_count(r, i)); continue; }
      if (r->agg_fn[a] != PGPU_AGG_AVG) { fixed.f64(agg_double(r, a, i)); continue; }
      fixed.i32((int32_t)var.b.size());  // OBJECT: (offset, length) into the variable-size data
      fixed.i32(16);
      var.i32(kObjectTypeAvgPair);       // then the object type and AvgPair.toBytes (sum, count)
      var.f64(agg_double(r, a, i));
      var.i64(row_count(r, i));
    }
  }
  // sections
  Out exc;
  exc.i32(0);
  Out dict;
  std::vector<std::string> dcols;
  std::vector<int> dcol_j;
  for (int j = 0; j < nk; ++j)
    if (r->key_types[j] == PGPU_STRING && !sorder[j].empty()) { dcols.push_back(names[j]); dcol_j.push_back(j); }
  dict.i32((int32_t)dcols.size());
  for (size_t k : java_hashmap_order(dcols)) {
    const int j = dcol_j[k];
    dict.str(dcols[k]);
    dict.i32((int32_t)sorder[j].size());
    for (size_t id = 0; id < sorder[j].size(); ++id) {  // Integer keys 0..n-1: HashMap order is ascending
      dict.i32((int32_t)id);
      dict.str((*dv[j].sv)[sorder[j][id]]);
    }
  }
  Out schema;
  schema.i32(nc);
  for (const auto& nm : names) schema.str(nm);
  for (const auto& ty : types) schema.str(ty);
  // metadata (IntermediateResultsBlock.attachMetadataToDataTable, :456-478)
  std::vector<std::string> mk = {"numDocsScanned", "numEntriesScannedInFilter", "numEntriesScannedPostFilter",
                                 "numSegmentsProcessed", "numSegmentsMatched", "numResizes", "resizeTimeMs",
                                 "totalDocs"};
  std::vector<int64_t> mv = {r->stats[0], r->stats[1], r->stats[2], r->stats[4], r->stats[5], 0, 0, r->stats[3]};
  if (r->groups_limit_reached) { mk.push_back("numGroupsLimitReached"); mv.push_back(1); }
  Out meta;
  meta.i32((int32_t)mk.size());
  for (size_t k : java_hashmap_order(mk)) {
    const MetaKey* key = meta_by_name(mk[k]);
    meta.i32(key->ordinal);
    if (key->kind == 1) meta.i32((int32_t)mv[k]);
    else if (key->kind == 2) meta.i64(mv[k]);
    else meta.str("true");
  }
  Out o;
  constexpr int32_t kHeader = 13 * 4;
  int32_t off = kHeader;
  o.i32(3);
  o.i32((int32_t)r->n);
  o.i32(nc);
  o.i32(off); o.i32((int32_t)exc.b.size()); off += (int32_t)exc.b.size();
  o.i32(off); o.i32((int32_t)dict.b.size()); off += (int32_t)dict.b.size();
  o.i32(off); o.i32((int32_t)schema.b.size()); off += (int32_t)schema.b.size();
  o.i32(off); o.i32((int32_t)fixed.b.size()); off += (int32_t)fixed.b.size();
  o.i32(off); o.i32((int32_t)var.b.size());
  o.raw(exc.b); o.raw(dict.b); o.raw(schema.b); o.raw(fixed.b); o.raw(var.b);
  o.i32((int32_t)meta.b.size());
  o.raw(meta.b);
  *len = (int64_t)o.b.size();
  if (!out) return 0;
  if (cap < *len) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "output buffer too small");
  memcpy(out, o.b.data(), o.b.size());
  return 0;
} PGPU_ABI_CATCH

int pgpu_broker_reduce_sql(const void* const* tables, const int64_t* lens, int32_t num_tables,
                           const pgpu_sql_trim* spec, char* json, int64_t cap, int64_t* len) try {
  if (!tables || !lens || num_tables < 0 || !spec || !len) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  std::vector<Table> T(num_tables);
  std::string err;
  for (int i = 0; i < num_tables; ++i)
    if (!parse_table(reinterpret_cast<const uint8_t*>(tables[i]), lens[i], &T[i], &err))
      return host_fail(PGPU_ERR_INVALID_ARGUMENT, "server %d: %s", i, err.c_str());
  // schema: group-by columns, then "fn(col)" aggregation columns (GroupByDataTableReducer.java:290-330)
  const Table* S = nullptr;
  for (const Table& t : T) if (!t.names.empty()) { S = &t; break; }
  std::vector<std::string> names, types;
  int nk = 0;
  std::vector<int> fn;
  if (S) {
    names = S->names;
    types = S->types;
    for (size_t c = 0; c < names.size(); ++c) {
      int f = -1;
      for (int k = 0; k <= PGPU_AGG_AVG; ++k) {
        const std::string pre = std::string(fn_name(k)) + "(";
        if (names[c].compare(0, pre.size(), pre) == 0 && names[c].back() == ')') f = k;
      }
      if (f < 0) { if ((int)c != nk) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "group-by columns must lead"); ++nk; }
      fn.push_back(f);
    }
  }
  const int nc = (int)names.size();
  for (const Table& t : T)
    if (!t.names.empty() && (t.names != names || t.types != types))
      return host_fail(PGPU_ERR_INVALID_ARGUMENT, "servers returned different data schemas");
  // merge the rows by key (AggregationFunction.merge per column)
  std::map<std::string, size_t> index;  // encoded key -> row
  std::vector<std::vector<Cell>> rows;
  for (const Table& t : T) {
    for (int64_t r = 0; r < t.rows; ++r) {
      In in{t.cells[r].data(), (int64_t)t.cells[r].size()};
      std::vector<Cell> cells(nc);
      std::string key;
      for (int c = 0; c < nc; ++c) {
        Cell& x = cells[c];
        const std::string& ty = types[c];
        if (ty == "INT") { x.kind = 0; x.i = in.i32(); }
        else if (ty == "LONG") { x.kind = 0; x.i = in.i64(); }
        else if (ty == "FLOAT") { x.kind = 1; int32_t b = in.i32(); in.i32(); float f; memcpy(&f, &b, 4); x.d = f; }
        else if (ty == "DOUBLE") { x.kind = 1; x.d = in.f64(); }
        else if (ty == "STRING") {
          x.kind = 2;
          const int32_t id = in.i32();
          auto dit = t.dict.find(names[c]);
          if (dit == t.dict.end() || !dit->second.count(id))
            return host_fail(PGPU_ERR_INVALID_ARGUMENT, "string id %d missing from the dictionary of %s", id,
                             names[c].c_str());
          x.s = dit->second.at(id);
        } else {  // OBJECT: AvgPair
          const int32_t off = in.i32(), ln = in.i32();
          In v{t.var.data(), (int64_t)t.var.size()};
          v.pos = off;
          const int32_t obj_type = v.i32();
          if (!v.ok) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "object offset %d outside the variable-size data", off);
          if (obj_type != kObjectTypeAvgPair || ln != 16)
            return host_fail(PGPU_ERR_UNSUPPORTED, "object column %s is not an AvgPair", names[c].c_str());
          x.kind = 3;
          x.d = v.f64();
          x.c = (double)v.i64();
          if (!v.ok) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad object bytes");
        }
        if (c < nk) {
          // exact encoding: the string bytes (length-prefixed), or the 8 bytes of the integer / IEEE double (a
          // decimal rendering such as %f would merge keys that differ past its precision)
          const char tag = x.kind == 2 ? 's' : x.kind == 0 ? 'i' : 'd';
          key += tag;
          if (x.kind == 2) {
            const uint32_t ln = (uint32_t)x.s.size();
            key.append(reinterpret_cast<const char*>(&ln), 4);
            key += x.s;
          } else if (x.kind == 0) {
            key.append(reinterpret_cast<const char*>(&x.i), 8);
          } else {
            // Double.equals: doubleToLongBits -- -0.0 and 0.0 are distinct keys, every NaN is one key
            const double d = std::isnan(x.d) ? std::numeric_limits<double>::quiet_NaN() : x.d;
            key.append(reinterpret_cast<const char*>(&d), 8);
          }
        }
      }
      if (!in.ok) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad row bytes");
      auto it = index.find(key);
      if (it == index.end()) { index.emplace(key, rows.size()); rows.push_back(std::move(cells)); continue; }
      std::vector<Cell>& dst = rows[it->second];
      for (int c = nk; c < nc; ++c) {
        switch (fn[c]) {
          case PGPU_AGG_COUNT: dst[c].i = java_add(dst[c].i, cells[c].i); break;
          case PGPU_AGG_SUM: dst[c].d += cells[c].d; break;
          case PGPU_AGG_MIN: dst[c].d = std::min(dst[c].d, cells[c].d); break;
          case PGPU_AGG_MAX: dst[c].d = std::max(dst[c].d, cells[c].d); break;
          default: dst[c].d += cells[c].d; dst[c].c += cells[c].c; break;
        }
      }
    }
  }
  // final results, ORDER BY, LIMIT (IndexedTable.finish on the broker: the top `limit` records)
  auto final_value = [&](const Cell& x) {
    if (x.kind == 3) return x.c ? x.d / x.c : -INFINITY;
    return x.kind == 0 ? (double)x.i : x.d;
  };
  std::vector<size_t> order(rows.size());
  std::iota(order.begin(), order.end(), 0);
  auto cmp_cell = [&](const Cell& a, const Cell& b) {
    if (a.kind == 2) return a.s < b.s ? -1 : (a.s > b.s ? 1 : 0);
    if (a.kind == 0 && b.kind == 0) return a.i < b.i ? -1 : (a.i > b.i ? 1 : 0);
    return dcmp(final_value(a), final_value(b));
  };
  std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) {  // ties: composite key order
    for (int i = 0; i < spec->num_order_by; ++i) {
      const pgpu_order_by& o = spec->order_by[i];
      const int c = o.kind == PGPU_ORDER_GROUP_BY ? o.index : nk + o.index;
      if (c < 0 || c >= nc) continue;
      const int r = cmp_cell(rows[x][c], rows[y][c]);
      if (r) return o.ascending ? r < 0 : r > 0;
    }
    for (int c = 0; c < nk; ++c) {
      const int r = cmp_cell(rows[x][c], rows[y][c]);
      if (r) return r < 0;
    }
    return false;
  });
  if ((int64_t)order.size() > spec->limit) order.resize(spec->limit);
  // the SELECT list (group-by columns and aggregations in query order; ORDER BY-only aggregations are not shown)
  std::vector<int> sel;
  for (int i = 0; i < spec->num_select; ++i) {
    const pgpu_order_by& e = spec->select[i];
    const int c = e.kind == PGPU_ORDER_GROUP_BY ? e.index : nk + e.index;
    if (c < 0 || c >= nc) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad SELECT expression %d", i);
    sel.push_back(c);
  }
  if (spec->num_select == 0)
    for (int c = 0; c < nc; ++c) sel.push_back(c);
  // BrokerResponseNative JSON: resultTable (final column types: COUNT LONG, the others DOUBLE) + statistics
  std::string o = "{\"resultTable\":{\"dataSchema\":{\"columnNames\":[";
  for (size_t k = 0; k < sel.size(); ++k) { if (k) o += ","; json_str(o, names[sel[k]]); }
  o += "],\"columnDataTypes\":[";
  for (size_t k = 0; k < sel.size(); ++k) {
    const int c = sel[k];
    if (k) o += ",";
    json_str(o, c < nk ? types[c] : (fn[c] == PGPU_AGG_COUNT ? "LONG" : "DOUBLE"));
  }
  o += "]},\"rows\":[";
  for (size_t k = 0; k < order.size(); ++k) {
    if (k) o += ",";
    o += "[";
    const std::vector<Cell>& row = rows[order[k]];
    for (size_t q = 0; q < sel.size(); ++q) {
      const int c = sel[q];
      if (q) o += ",";
      const Cell& x = row[c];
      if (c < nk) {
        if (x.kind == 2) json_str(o, x.s);
        else if (x.kind == 0) o += std::to_string(x.i);
        else json_double(o, x.d);
      } else if (fn[c] == PGPU_AGG_COUNT) {
        o += std::to_string(x.i);
      } else {
        json_double(o, final_value(x));
      }
    }
    o += "]";
  }
  o += "]}";
  int64_t sums[6] = {0, 0, 0, 0, 0, 0};
  const char* stat_names[6] = {"numDocsScanned", "numEntriesScannedInFilter", "numEntriesScannedPostFilter",
                               "numSegmentsProcessed", "numSegmentsMatched", "totalDocs"};
  bool limit_reached = false;
  for (const Table& t : T) {
    for (int k = 0; k < 6; ++k) {
      auto it = t.meta.find(stat_names[k]);
      if (it != t.meta.end()) sums[k] = java_add(sums[k], std::stoll(it->second));
    }
    limit_reached |= t.meta.count("numGroupsLimitReached") > 0;
  }
  o += ",\"exceptions\":[],\"numServersQueried\":" + std::to_string(num_tables) +
       ",\"numServersResponded\":" + std::to_string(num_tables);
  for (int k = 0; k < 6; ++k) o += ",\"" + std::string(stat_names[k]) + "\":" + std::to_string(sums[k]);
  o += std::string(",\"numGroupsLimitReached\":") + (limit_reached ? "true" : "false") + "}";
  *len = (int64_t)o.size();
  if (!json) return 0;
  if (cap < *len + 1) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "output buffer too small");
  memcpy(json, o.c_str(), o.size() + 1);
  return 0;
} PGPU_ABI_CATCH

}  // extern "C"
