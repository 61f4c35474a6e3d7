// host_fuzz: the host-side parsers and builders of libpinotgpu under AddressSanitizer + UndefinedBehaviorSanitizer.
//
// Built by pinot_amd/build.py:build_host_fuzz() from the library's own sources with host-only sanitizer flags
// (-Xarch_host -fsanitize=...; the device code is compiled as usual and never runs: no GPU is touched) and driven by
// tests/test_host_sanitizers_cpu.py.  Every entry point exercised here is pure host code that reads bytes a server
// takes from outside the process:
//   raw   pgpu_raw_forward_index_values  FixedByteChunkSVForwardIndexReader chunks, PASS_THROUGH / LZ4 / LZ4_LENGTH
//   dt    pgpu_broker_reduce_sql         DataTable V3 bytes from servers (DataTableImplV3(ByteBuffer))
//   st    pgpu_startree_load             star_tree_index + star_tree_index_map files (StarTreeLoaderUtils)
//   invf  pgpu_inverted_index_check      bitmap.inv files (BitmapInvertedIndexReader + portable RoaringBitmap)
//   inv   pgpu_build_inverted_index      fixed-bit forward index -> bitmap.inv bytes
//   stb   pgpu_startree_build            segment buffers -> star-tree (OnHeapSingleTreeBuilder)
//   flt   pgpu_filter_entries_scanned    postfix filter programs + per-leaf doc sets
// Seeds (valid inputs written by the product's Python writers) come from <corpus>; each iteration applies 1-4 byte
// mutations (bit flips, random bytes, boundary int32 / int64 values, truncation, splices) and hands the result to the
// entry point in a buffer of exactly its size, so any read past it is reported.  The return codes are not checked
// (most mutants must be rejected); the sanitizers are the oracle, and exit status 0 means no report.
//
// usage: host_fuzz <corpus_dir> <iterations per target> <seed>
#include <dirent.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "pinotgpu.h"

namespace {

struct Rng {
  uint64_t s;
  uint64_t next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  }
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

using Bytes = std::vector<uint8_t>;

Bytes read_file(const std::string& path) {
  Bytes b;
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return b;
  uint8_t buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + n);
  fclose(f);
  return b;
}

void put_be(Bytes& v, size_t pos, uint64_t x, int width) {
  for (int i = 0; i < width; ++i) v[pos + i] = (uint8_t)(x >> (8 * (width - 1 - i)));
}

Bytes mutate(const Bytes& in, Rng& r) {
  Bytes v = in;
  const int n = 1 + (int)r.below(4);
  static const int64_t interesting[] = {0, -1, 1, 2, 0x7f, 0xff, 0x7fff, 0xffff, 0x10000, INT32_MAX, INT32_MIN,
                                        (int64_t)INT32_MAX + 1, INT64_MAX, INT64_MIN};
  for (int i = 0; i < n; ++i) {
    switch (r.below(7)) {
      case 0:
        if (!v.empty()) v[r.below(v.size())] ^= (uint8_t)(1u << r.below(8));
        break;
      case 1:
        if (!v.empty()) v[r.below(v.size())] = (uint8_t)r.next();
        break;
      case 2:
        if (v.size() >= 4) {
          const int64_t x = r.below(3) == 0 ? (int64_t)v.size() + (int64_t)r.below(3) - 1
                                            : interesting[r.below(sizeof interesting / sizeof *interesting)];
          put_be(v, r.below(v.size() - 3), (uint64_t)x, 4);
        }
        break;
      case 3:
        if (v.size() >= 8) put_be(v, r.below(v.size() - 7), (uint64_t)interesting[r.below(14)], 8);
        break;
      case 4:
        v.resize(r.below(v.size() + 1));
        break;
      case 5:
        if (!v.empty() && !in.empty()) {  // splice: a range of the input copied over another position
          const size_t a = r.below(in.size());
          const size_t len = 1 + r.below(std::min<size_t>({64, in.size() - a, v.size()}));
          memcpy(v.data() + r.below(v.size() - len + 1), in.data() + a, len);
        }
        break;
      default:  // a little-endian int32 (LZ4_LENGTH_PREFIXED lengths, roaring fields)
        if (v.size() >= 4) {
          const uint32_t x = (uint32_t)interesting[r.below(11)];
          const size_t p = r.below(v.size() - 3);
          for (int k = 0; k < 4; ++k) v[p + k] = (uint8_t)(x >> (8 * k));
        }
    }
  }
  return v;
}

// Exactly-sized heap copy: a read one byte past `v` lands in ASan's redzone.
struct Exact {
  uint8_t* p;
  size_t n;
  explicit Exact(const Bytes& v) : p((uint8_t*)malloc(v.size() ? v.size() : 1)), n(v.size()) {
    if (!v.empty()) memcpy(p, v.data(), v.size());
  }
  ~Exact() { free(p); }
};

std::vector<std::string> list_dir(const std::string& dir) {
  std::vector<std::string> out;
  if (DIR* d = opendir(dir.c_str())) {
    while (dirent* e = readdir(d)) out.push_back(e->d_name);
    closedir(d);
  }
  std::sort(out.begin(), out.end());
  return out;
}

// ---- raw.<type>.<num_docs>.<k>.bin
long fuzz_raw(const std::string& dir, long iters, Rng& r) {
  long calls = 0;
  for (const std::string& name : list_dir(dir)) {
    int type = 0, docs = 0, k = 0;
    if (sscanf(name.c_str(), "raw.%d.%d.%d.bin", &type, &docs, &k) != 3) continue;
    const Bytes seed = read_file(dir + "/" + name);
    for (long it = 0; it < iters; ++it) {
      Exact b(it == 0 ? seed : mutate(seed, r));
      const int n = r.below(8) == 0 ? docs + (int)r.below(3) - 1 : docs;
      if (n < 0) continue;
      std::vector<int64_t> oi((size_t)n + 1);
      std::vector<double> of((size_t)n + 1);
      pgpu_raw_forward_index_values(b.p, (int64_t)b.n, type, n, r.below(2) ? oi.data() : nullptr, of.data());
      ++calls;
    }
  }
  return calls;
}

// ---- inv.<cardinality>.<num_docs>.<k>.bin
long fuzz_invfile(const std::string& dir, long iters, Rng& r) {
  long calls = 0;
  for (const std::string& name : list_dir(dir)) {
    int card = 0, docs = 0, k = 0;
    if (sscanf(name.c_str(), "inv.%d.%d.%d.bin", &card, &docs, &k) != 3) continue;
    const Bytes seed = read_file(dir + "/" + name);
    for (long it = 0; it < iters; ++it) {
      Exact b(it == 0 ? seed : mutate(seed, r));
      int64_t total = 0;
      const int c = it > 0 && r.below(10) == 0 ? card + (int)r.below(3) - 1 : card;
      const int n = it > 0 && r.below(10) == 0 ? docs - (int)r.below(70000) : docs;
      const int rc = pgpu_inverted_index_check(b.p, (int64_t)b.n, c, n, &total);
      if (it == 0 && (rc != 0 || total != docs)) {
        fprintf(stderr, "seed %s rejected (rc %d, %lld docs)\n", name.c_str(), rc, (long long)total);
        exit(4);
      }
      ++calls;
    }
  }
  return calls;
}

// ---- dt.<k>.bin: one mutated DataTable, alone or beside a valid one
long fuzz_dt(const std::string& dir, long iters, Rng& r) {
  std::vector<Bytes> seeds;
  for (const std::string& name : list_dir(dir))
    if (name.rfind("dt.", 0) == 0) seeds.push_back(read_file(dir + "/" + name));
  if (seeds.empty()) return 0;
  long calls = 0;
  for (long it = 0; it < iters * (long)seeds.size(); ++it) {
    const Bytes& s = seeds[r.below(seeds.size())];
    Exact a(it < (long)seeds.size() ? seeds[it] : mutate(s, r));
    Exact b(seeds[r.below(seeds.size())]);
    const void* tabs[2] = {a.p, b.p};
    const int64_t lens[2] = {(int64_t)a.n, (int64_t)b.n};
    pgpu_order_by ob[2] = {{PGPU_ORDER_AGGREGATION, (int32_t)r.below(3), (int32_t)r.below(2)},
                           {PGPU_ORDER_GROUP_BY, (int32_t)r.below(3), 1}};
    pgpu_sql_trim spec;
    memset(&spec, 0, sizeof spec);
    spec.num_order_by = (int32_t)r.below(3);
    spec.order_by = ob;
    spec.limit = 1 + (int32_t)r.below(20);
    spec.min_server_group_trim_size = 5000;
    spec.group_trim_threshold = 1000000;
    int64_t len = 0;
    const int nt = 1 + (int)r.below(2);
    if (pgpu_broker_reduce_sql(tabs, lens, nt, &spec, nullptr, 0, &len) == 0 && len >= 0 && len < (1 << 26)) {
      std::vector<char> json((size_t)len + 1);
      pgpu_broker_reduce_sql(tabs, lens, nt, &spec, json.data(), len + 1, &len);
    }
    ++calls;
  }
  return calls;
}

// ---- st.idx + st.map + st.args ("num_docs num_columns" then "name bits" per column)
long fuzz_st(const std::string& dir, long iters, Rng& r) {
  const Bytes idx = read_file(dir + "/st.idx"), map = read_file(dir + "/st.map"), args = read_file(dir + "/st.args");
  if (idx.empty() || map.empty() || args.empty()) return 0;
  std::string a(args.begin(), args.end());
  int num_docs = 0, ncols = 0, off = 0;
  if (sscanf(a.c_str(), "%d %d%n", &num_docs, &ncols, &off) != 2 || ncols <= 0 || ncols > 64) return 0;
  std::vector<std::string> names((size_t)ncols);
  std::vector<int32_t> bits((size_t)ncols);
  const char* p = a.c_str() + off;
  for (int c = 0; c < ncols; ++c) {
    char nm[128];
    int b = 0, used = 0;
    if (sscanf(p, "%127s %d%n", nm, &b, &used) != 2) return 0;
    names[c] = nm;
    bits[c] = b;
    p += used;
  }
  std::vector<const char*> cn;
  for (auto& s : names) cn.push_back(s.c_str());
  long calls = 0;
  for (long it = 0; it < iters; ++it) {
    const int which = it == 0 ? -1 : (int)r.below(3);
    Exact bi(which == 0 || which == 2 ? mutate(idx, r) : idx);
    Exact bm(which == 1 || which == 2 ? mutate(map, r) : map);
    const int nd = r.below(8) == 0 ? num_docs + (int)r.below(5) - 2 : num_docs;
    pgpu_startree st = nullptr;
    if (pgpu_startree_load(bi.p, (int64_t)bi.n, (const char*)bm.p, (int64_t)bm.n, (int32_t)r.below(8) == 0 ? 1 : 0,
                           nd, ncols, cn.data(), bits.data(), &st) == 0) {
      pgpu_startree_desc d;
      pgpu_startree_get_desc(st, &d);
      pgpu_startree_destroy(st);
    }
    ++calls;
  }
  return calls;
}

// MSB-first fixed-bit packing (FixedBitSVForwardIndexWriter / PinotDataBitSet layout), padded to whole int32 words.
Bytes pack_bits(const std::vector<uint32_t>& ids, int bits) {
  Bytes out(((ids.size() * (size_t)bits + 31) / 32) * 4, 0);
  size_t bit = 0;
  for (uint32_t v : ids)
    for (int k = bits - 1; k >= 0; --k, ++bit)
      if ((v >> k) & 1) out[bit / 8] |= (uint8_t)(0x80u >> (bit % 8));
  return out;
}

int bits_for(int card) {
  int b = 1;
  while (b < 31 && (1 << b) < card) ++b;
  return b;
}

long fuzz_inv(long iters, Rng& r) {
  long calls = 0;
  for (long it = 0; it < iters; ++it) {
    const int card = 1 + (int)r.below(r.below(4) == 0 ? 70000 : 300);
    const int bits = r.below(10) == 0 ? 1 + (int)r.below(31) : bits_for(card);
    const int docs = (int)r.below(r.below(8) == 0 ? 200000 : 3000);
    std::vector<uint32_t> ids((size_t)docs);
    const uint32_t lim = bits >= 31 ? 0x7fffffffu : (1u << bits);
    for (auto& x : ids) x = (uint32_t)r.below(r.below(16) == 0 ? lim : (uint64_t)card);
    Bytes fwd = pack_bits(ids, bits);
    if (r.below(6) == 0) fwd.resize(r.below(fwd.size() + 1));
    Exact f(fwd);
    int64_t len = 0;
    if (pgpu_build_inverted_index(f.p, (int64_t)f.n, bits, docs, card, nullptr, 0, &len) == 0 && len > 0 &&
        len < (1 << 28)) {
      const int64_t cap = r.below(4) == 0 ? len - 1 - (int64_t)r.below(8) : len;
      if (cap > 0) {
        uint8_t* out = (uint8_t*)malloc((size_t)cap);
        pgpu_build_inverted_index(f.p, (int64_t)f.n, bits, docs, card, out, cap, &len);
        free(out);
      }
    }
    ++calls;
  }
  return calls;
}

long fuzz_startree_build(long iters, Rng& r) {
  long calls = 0;
  for (long it = 0; it < iters; ++it) {
    const int ndims = 1 + (int)r.below(4);
    const int ncols = ndims + 1;  // dims, then one INT metric
    const int docs = (int)r.below(4000);
    std::vector<Bytes> fwd((size_t)ncols), dict((size_t)ncols);
    std::vector<pgpu_column_buffers> cols((size_t)ncols);
    std::vector<int32_t> types((size_t)ncols, PGPU_INT);
    for (int c = 0; c < ncols; ++c) {
      const int card = 1 + (int)r.below(c < ndims ? 40 : 500);
      const int bits = bits_for(card);
      std::vector<uint32_t> ids((size_t)docs);
      for (auto& x : ids) x = (uint32_t)r.below((uint64_t)card);
      fwd[c] = pack_bits(ids, bits);
      dict[c].resize((size_t)card * 4);
      for (int v = 0; v < card; ++v) put_be(dict[c], (size_t)v * 4, (uint64_t)(int64_t)(v * 3 - 7), 4);
      pgpu_column_buffers& b = cols[c];
      memset(&b, 0, sizeof b);
      b.cardinality = card;
      b.bits_per_element = bits;
      b.entry_width = 4;
      b.fwd_format = PGPU_FWD_FIXED_BIT;
      if (r.below(12) == 0) {  // a malformed column: short forward index, short dictionary or wrong width
        switch (r.below(3)) {
          case 0: fwd[c].resize(r.below(fwd[c].size() + 1)); break;
          case 1: dict[c].resize(r.below(dict[c].size() + 1)); break;
          default: b.bits_per_element = 1 + (int)r.below(31);
        }
      }
    }
    std::vector<Exact*> keep;
    for (int c = 0; c < ncols; ++c) {
      keep.push_back(new Exact(fwd[c]));
      keep.push_back(new Exact(dict[c]));
      cols[c].fwd = keep[keep.size() - 2]->p;
      cols[c].fwd_len = (int64_t)fwd[c].size();
      cols[c].dict = keep.back()->p;
      cols[c].dict_len = (int64_t)dict[c].size();
    }
    pgpu_segment_desc seg{docs, ncols, cols.data()};
    std::vector<int32_t> split((size_t)ndims);
    for (int d = 0; d < ndims; ++d) split[d] = d;
    if (r.below(10) == 0) split[r.below(ndims)] = (int32_t)r.below(ncols + 2) - 1;  // bad / duplicate dimension
    std::vector<int32_t> skip;
    for (int d = 0; d < ndims; ++d)
      if (r.below(3) == 0) skip.push_back(d);
    const pgpu_agg pairs[3] = {{PGPU_AGG_SUM, ndims}, {PGPU_AGG_COUNT, -1}, {PGPU_AGG_MAX, ndims}};
    pgpu_startree st = nullptr;
    if (pgpu_startree_build(&seg, types.data(), split.data(), ndims, skip.data(), (int32_t)skip.size(), pairs,
                            1 + (int32_t)r.below(3), 1 + (int32_t)r.below(200), &st) == 0) {
      pgpu_startree_desc d;
      int32_t n = 0;
      pgpu_startree_get_desc(st, &d);
      pgpu_startree_num_raw_records(st, &n);
      pgpu_startree_destroy(st);
    }
    for (Exact* e : keep) delete e;
    ++calls;
  }
  return calls;
}

long fuzz_filter(long iters, Rng& r) {
  long calls = 0;
  for (long it = 0; it < iters; ++it) {
    const int leaves = 1 + (int)r.below(6);
    const int docs = (int)r.below(5000);
    const size_t words = ((size_t)docs + 31) / 32;
    std::vector<int32_t> types((size_t)leaves);
    std::vector<std::vector<uint32_t>> masks((size_t)leaves);
    std::vector<const uint32_t*> mp((size_t)leaves);
    for (int i = 0; i < leaves; ++i) {
      types[i] = (int32_t)r.below(r.below(20) == 0 ? 9 : 5);
      masks[i].resize(words + 1);
      for (auto& w : masks[i]) w = (uint32_t)r.next() & (uint32_t)r.next();
      mp[i] = (types[i] <= PGPU_LEAF_MATCH_ALL && r.below(2)) ? nullptr : masks[i].data();
    }
    // a well-formed postfix program most of the time; otherwise random ops
    std::vector<pgpu_filter_op> ops;
    if (r.below(5)) {
      int depth = 0;
      for (int i = 0; i < leaves; ++i) {
        ops.push_back({PGPU_OP_PRED, i});
        ++depth;
        if (depth >= 2 && r.below(2)) {
          const int k = 2 + (int)r.below(depth - 1);
          ops.push_back({1 + (int32_t)r.below(2), k});
          depth -= k - 1;
        }
        if (r.below(6) == 0) ops.push_back({PGPU_OP_NOT, 0});
      }
      if (depth > 1) ops.push_back({PGPU_OP_AND, depth});
    } else {
      const int n = (int)r.below(12);
      for (int i = 0; i < n; ++i) ops.push_back({(int32_t)r.below(5) - (r.below(9) == 0), (int32_t)r.below(9) - 2});
    }
    int64_t out = 0;
    pgpu_filter_entries_scanned(ops.data(), (int32_t)ops.size(), types.data(), mp.data(), leaves, docs, &out);
    ++calls;
  }
  return calls;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s <corpus_dir> <iterations> <seed>\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const long iters = atol(argv[2]);
  Rng r{(uint64_t)strtoull(argv[3], nullptr, 10) * 0x9E3779B97F4A7C15ull + 1};
  auto timed = [](const char* name, auto&& f) {
    const auto t0 = std::chrono::steady_clock::now();
    const long calls = f();
    printf("%-4s %7ld calls %8.2f s\n", name, calls,
           std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    fflush(stdout);
    return calls;
  };
  const long raw = timed("raw", [&] { return fuzz_raw(dir, iters, r); });
  const long dt = timed("dt", [&] { return fuzz_dt(dir, iters, r); });
  const long st = timed("st", [&] { return fuzz_st(dir, iters, r); });
  const long invf = timed("invf", [&] { return fuzz_invfile(dir, iters, r); });
  const long inv = timed("inv", [&] { return fuzz_inv(iters, r); });
  const long stb = timed("stb", [&] { return fuzz_startree_build(iters / 4 + 1, r); });
  const long flt = timed("flt", [&] { return fuzz_filter(iters, r); });
  printf("host_fuzz calls: raw %ld dt %ld st %ld invf %ld inv %ld stb %ld flt %ld\n", raw, dt, st, invf, inv, stb,
         flt);
  return (raw > 0 && dt > 0 && st > 0 && invf > 0) ? 0 : 3;  // 3: a seed family is missing from the corpus
}
