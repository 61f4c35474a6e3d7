// rt_dict.cpp -- segment and table-global dictionaries, LUTs, value arrays (rt.h).
#include "rt_decls.h"

namespace pgpu {

// ------------------------------------------------------------------------------------------------ dictionaries
int parse_dictionary(int type, const pgpu_column_buffers& cb, Dict* d) {
  d->type = type;
  const int64_t card = cb.cardinality;
  if (card < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "negative cardinality");
  const int w = cb.entry_width;
  if (card > 0 && (!cb.dict || cb.dict_len < card * (int64_t)w))
    return fail(PGPU_ERR_INVALID_ARGUMENT, "dictionary buffer too small (%lld < %lld x %d)", (long long)cb.dict_len,
                (long long)card, w);
  switch (type) {
    case PGPU_INT:
      if (w != 4) return fail(PGPU_ERR_INVALID_ARGUMENT, "INT dictionary entry width %d", w);
      d->iv.resize(card);
      for (int64_t i = 0; i < card; ++i) d->iv[i] = (int32_t)rd_be32(cb.dict + i * 4);
      break;
    case PGPU_LONG:
      if (w != 8) return fail(PGPU_ERR_INVALID_ARGUMENT, "LONG dictionary entry width %d", w);
      d->iv.resize(card);
      for (int64_t i = 0; i < card; ++i) d->iv[i] = (int64_t)rd_be64(cb.dict + i * 8);
      break;
    case PGPU_FLOAT:
      if (w != 4) return fail(PGPU_ERR_INVALID_ARGUMENT, "FLOAT dictionary entry width %d", w);
      d->dv.resize(card);
      for (int64_t i = 0; i < card; ++i) {
        uint32_t u = rd_be32(cb.dict + i * 4);
        float f;
        memcpy(&f, &u, 4);
        d->dv[i] = f;
      }
      break;
    case PGPU_DOUBLE:
      if (w != 8) return fail(PGPU_ERR_INVALID_ARGUMENT, "DOUBLE dictionary entry width %d", w);
      d->dv.resize(card);
      for (int64_t i = 0; i < card; ++i) {
        uint64_t u = rd_be64(cb.dict + i * 8);
        memcpy(&d->dv[i], &u, 8);
      }
      break;
    case PGPU_STRING:
      d->sv.resize(card);
      for (int64_t i = 0; i < card; ++i) {  // FixedByteValueReaderWriter.getUnpaddedString (:57-95)
        const uint8_t* s = cb.dict + i * w;
        int n = 0;
        while (n < w && s[n] != (uint8_t)cb.padding_byte) ++n;
        d->sv[i].assign(reinterpret_cast<const char*>(s), n);
      }
      break;
    default:
      return fail(PGPU_ERR_INVALID_ARGUMENT, "unsupported data type %d", type);
  }
  return 0;
}

bool dbl_less(double a, double b) {  // Double.compare order for the sorted global dictionary
  if (a < b) return true;
  if (a > b) return false;
  int64_t x, y;
  memcpy(&x, &a, 8);
  memcpy(&y, &b, 8);
  return x < y;
}

// Merges sorted `src` into the global dictionary snapshot `g`: a new snapshot replaces it when the union grew.
// Returns true if it grew.
bool merge_dict(std::shared_ptr<const Dict>& g, const Dict& src) {
  const Dict& dst = *g;
  auto out = std::make_shared<Dict>();
  out->type = dst.type;
  if (is_int_type(dst.type)) {
    out->iv.reserve(dst.iv.size() + src.iv.size());
    std::set_union(dst.iv.begin(), dst.iv.end(), src.iv.begin(), src.iv.end(), std::back_inserter(out->iv));
  } else if (is_fp_type(dst.type)) {
    std::vector<double> s = src.dv;
    std::sort(s.begin(), s.end(), dbl_less);
    out->dv.reserve(dst.dv.size() + s.size());
    std::set_union(dst.dv.begin(), dst.dv.end(), s.begin(), s.end(), std::back_inserter(out->dv), dbl_less);
  } else {
    std::vector<std::string> s = src.sv;
    std::sort(s.begin(), s.end());
    out->sv.reserve(dst.sv.size() + s.size());
    std::set_union(dst.sv.begin(), dst.sv.end(), s.begin(), s.end(), std::back_inserter(out->sv));
  }
  if (out->size() == dst.size()) return false;
  out->id = g_dict_ids.fetch_add(1);
  g = std::move(out);
  return true;
}

// BaseImmutableDictionary.insertionIndexOf behind PredicateUtils.getStoredValue (Dictionary.java:49-100,
// BaseImmutableDictionary.java:97-230).  Returns false when the literal does not convert (BadQueryRequest).
int64_t global_index_of(const Dict& g, const Dict& local, size_t i) {
  if (is_int_type(g.type)) {
    auto it = std::lower_bound(g.iv.begin(), g.iv.end(), local.iv[i]);
    return (it != g.iv.end() && *it == local.iv[i]) ? it - g.iv.begin() : -1;
  }
  if (is_fp_type(g.type)) {
    auto it = std::lower_bound(g.dv.begin(), g.dv.end(), local.dv[i], dbl_less);
    return (it != g.dv.end() && !dbl_less(local.dv[i], *it)) ? it - g.dv.begin() : -1;
  }
  auto it = std::lower_bound(g.sv.begin(), g.sv.end(), local.sv[i]);
  return (it != g.sv.end() && *it == local.sv[i]) ? it - g.sv.begin() : -1;
}

// Makes the local->global LUT of (seg, col) current.
int ensure_lut(pgpu_table_s* t, Segment& s, int col, hipStream_t stream) {
  Column& c = s.cols[col];
  if (c.lut_version == t->global_version[col] && c.lut) return 0;
  std::vector<int32_t> lut(std::max<int32_t>(c.card, 1));
  for (int32_t i = 0; i < c.card; ++i) {
    int64_t g = global_index_of(*t->global[col], c.dict, i);
    if (g < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "value missing from the global dictionary (column %d)", col);
    lut[i] = (int32_t)g;
  }
  auto m = std::make_shared<DevMem>();
  HIP_TRY(hipMalloc(&m->p, sizeof(int32_t) * lut.size()));
  if (!c.lut) t->device_bytes += sizeof(int32_t) * lut.size();
  HIP_TRY(hipMemcpyAsync(m->p, lut.data(), sizeof(int32_t) * lut.size(), hipMemcpyHostToDevice, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  c.lut = std::move(m);  // the previous version lives on in the plans that reference it
  c.lut_version = t->global_version[col];
  // strictly increasing (both dictionaries sorted), so the ends decide whether it is a contiguous run
  c.lut_off = c.card > 0 && lut[c.card - 1] - lut[0] == c.card - 1 ? lut[0] : -1;
  return 0;
}

// Dictionary values for aggregation (Dictionary.readDoubleValues, DataFetcher.java:469-478).
int ensure_values(pgpu_table_s* t, Segment& s, int col, hipStream_t stream) {
  Column& c = s.cols[col];
  if (c.d_key) return 0;
  const size_t n = std::max<int32_t>(c.card, 1);
  std::vector<int64_t> key(n, 0);
  std::vector<double> val(n, 0.0);
  for (int32_t i = 0; i < c.card; ++i) {
    if (is_int_type(c.dict.type)) {
      key[i] = c.dict.iv[i];
      val[i] = (double)c.dict.iv[i];
    } else {
      key[i] = double_key(c.dict.dv[i]);
      val[i] = c.dict.dv[i];
    }
  }
  HIP_TRY(hipMalloc(&c.d_key, sizeof(int64_t) * n));
  HIP_TRY(hipMalloc(&c.d_val, sizeof(double) * n));
  t->device_bytes += 16 * n;
  HIP_TRY(hipMemcpyAsync(c.d_key, key.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipMemcpyAsync(c.d_val, val.data(), sizeof(double) * n, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  if (is_int_type(c.dict.type) && c.card > 0) {  // sorted distinct integers: consecutive iff the ends span card
    const __int128 span = (__int128)c.dict.iv[c.card - 1] - (__int128)c.dict.iv[0];
    c.key_affine = span == (__int128)(c.card - 1);
    c.key_base = c.dict.iv[0];
  }
  return 0;
}


// The table-global value arrays of `col` for its current global dictionary (under the table mutex).
int ensure_global_values(pgpu_table_s* t, int col, hipStream_t stream) {
  auto& gv = t->gvalues[col];
  if (gv.version == t->global_version[col] && gv.keys) return 0;
  const Dict& g = *t->global[col];
  const size_t n = std::max<size_t>(g.size(), 1);
  std::vector<int64_t> key(n, 0);
  std::vector<double> val(n, 0.0);
  for (size_t i = 0; i < g.size(); ++i) {
    if (is_int_type(g.type)) {
      key[i] = g.iv[i];
      val[i] = (double)g.iv[i];
    } else {
      key[i] = double_key(g.dv[i]);
      val[i] = g.dv[i];
    }
  }
  auto k = std::make_shared<DevMem>(), v = std::make_shared<DevMem>();
  HIP_TRY(hipMalloc(&k->p, sizeof(int64_t) * n));
  HIP_TRY(hipMalloc(&v->p, sizeof(double) * n));
  HIP_TRY(hipMemcpyAsync(k->p, key.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipMemcpyAsync(v->p, val.data(), sizeof(double) * n, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  // the current arrays' bytes (a rebuild after the dictionary grew replaces the previous arrays in the account; those
  // live on only in the plans that still reference them)
  t->device_bytes += 16 * ((int64_t)n - gv.n);
  gv.n = (int64_t)n;
  gv.keys = std::move(k);
  gv.vals = std::move(v);
  gv.version = t->global_version[col];
  return 0;
}

// How (seg, col)'s local dictIds index the table-global value arrays (under the table mutex): from the global id of
// local id 0 on, skipping the global values the segment's dictionary lacks -- at most kMaxValueGaps of them, as
// thresholds (KCol.gaps, vidx) -- or not at all (dictionaries below kGlobalValuesMinCard, or more missing values: the
// segment's own arrays).
int ensure_value_map(pgpu_table_s* t, Segment& s, int col) {
  Column& c = s.cols[col];
  if (c.vmap_version == t->global_version[col]) return 0;
  c.vgap_first = -1;
  c.vgaps.clear();
  c.vmap_version = t->global_version[col];
  if (c.raw || c.card < kGlobalValuesMinCard) return 0;
  const Dict& g = *t->global[col];
  int64_t prev = -1, first = -1;
  std::vector<uint32_t> gaps;
  for (int32_t i = 0; i < c.card; ++i) {
    const int64_t gi = global_index_of(g, c.dict, i);
    if (gi < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "value missing from the global dictionary (column %d)", col);
    if (i == 0) first = gi;
    // each global id skipped before local id i: a threshold at i, in mapped space (+ the thresholds before it)
    for (int64_t d = i == 0 ? 0 : gi - prev - 1; d > 0; --d) {
      if ((int)gaps.size() == kMaxValueGaps) return 0;
      gaps.push_back((uint32_t)(i + (int64_t)gaps.size()));
    }
    prev = gi;
  }
  c.vgap_first = (int32_t)first;
  c.vgaps = std::move(gaps);
  return 0;
}

int64_t padded_fwd_words(int64_t num_docs, int bits);
int scan_variant(const pgpu_plan_s* P);

// Identity forward index of the virtual $docId column over docs [0, n): Pinot's MSB-first fixed-bit layout of the
// values 0..n-1 (a sorted "dictionary" of docIds), and the values as int64 (the MIN slot's keys).
int ensure_docid(pgpu_table_s* t, int64_t n, hipStream_t stream) {
  if (n <= t->docid_n) return 0;
  int bits = 1;
  while (bits < 31 && (int64_t(1) << bits) < n) ++bits;
  const int64_t words = padded_fwd_words(n, bits);
  std::vector<uint8_t> fwd((size_t)words * 4, 0);
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t bit = (uint64_t)i * bits;
    for (int b = 0; b < bits; ++b)
      if ((i >> (bits - 1 - b)) & 1) fwd[(bit + b) >> 3] |= (uint8_t)(0x80u >> ((bit + b) & 7));
  }
  std::vector<int64_t> key(n);
  for (int64_t i = 0; i < n; ++i) key[i] = i;
  if (t->d_docid_fwd) t->retired.push_back(t->d_docid_fwd);
  if (t->d_docid_key) t->retired.push_back(t->d_docid_key);
  t->d_docid_fwd = nullptr;
  t->d_docid_key = nullptr;
  t->docid_n = 0;
  HIP_TRY(hipMalloc(&t->d_docid_fwd, fwd.size()));
  HIP_TRY(hipMalloc(&t->d_docid_key, (size_t)n * 8));
  HIP_TRY(hipMemcpyAsync(t->d_docid_fwd, fwd.data(), fwd.size(), hipMemcpyHostToDevice, stream));
  HIP_TRY(hipMemcpyAsync(t->d_docid_key, key.data(), (size_t)n * 8, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  t->docid_bits = bits;
  t->docid_n = n;
  t->device_bytes += (int64_t)fwd.size() + n * 8;
  return 0;
}

// Unpin accounting: the segment's device bytes leave the table's total now; the memory itself goes with the last
// reference (~Segment).
void account_unpin(pgpu_table_s* t, const Segment* s) {
  int64_t fwd_words = 0;
  for (const auto& c : s->cols) {
    if (c.inv) t->device_bytes -= c.inv->bytes;
    t->device_bytes -= (c.lut ? 4 * std::max(c.card, 1) : 0) +
                       (c.d_key ? 16 * (c.raw ? raw_padded_docs(s->num_docs) : std::max(c.card, 1)) : 0);
    if (!c.raw) fwd_words += (c.fwd_words + 63) & ~int64_t(63);
  }
  if (s->d_block) t->device_bytes -= std::max<int64_t>(fwd_words, 64) * 4;
  if (s->star) t->device_bytes -= s->star->bytes;
}

int64_t padded_fwd_words(int64_t num_docs, int bits) {
  return ((num_docs + kTileDocs - 1) / kTileDocs) * (int64_t)kBlock * bits + kFwdPadWords;
}

// LZ4 block decoder (the LZ4 block format of lz4-java's LZ4SafeDecompressor, behind Pinot's LZ4Decompressor /
// LZ4WithLengthDecompressor, seglocal/io/compression/LZ4Decompressor.java:40-50).  Every length and offset is
// checked against both buffers; returns the decoded length or -1.
int64_t lz4_decode_block(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap) {
  const uint8_t* ip = src;
  const uint8_t* const iend = src + n;
  uint8_t* op = dst;
  uint8_t* const oend = dst + cap;
  auto ext_len = [&](int64_t& len) -> bool {  // 255-continued length bytes
    uint32_t b;
    do {
      if (ip >= iend) return false;
      b = *ip++;
      len += b;
    } while (b == 255);
    return true;
  };
  while (ip < iend) {
    const uint32_t token = *ip++;
    int64_t lit = token >> 4;
    if (lit == 15 && !ext_len(lit)) return -1;
    if (lit > iend - ip || lit > oend - op) return -1;
    memcpy(op, ip, (size_t)lit);
    ip += lit;
    op += lit;
    if (ip == iend) return op - dst;  // last sequence: literals only
    if (iend - ip < 2) return -1;
    const int64_t off = (int64_t)ip[0] | ((int64_t)ip[1] << 8);
    ip += 2;
    int64_t ml = token & 15;
    if (ml == 15 && !ext_len(ml)) return -1;
    ml += 4;
    if (off == 0 || off > op - dst || ml > oend - op) return -1;
    const uint8_t* m = op - off;
    if (off >= ml) {
      memcpy(op, m, (size_t)ml);
      op += ml;
    } else {  // overlapping: the last `off` bytes repeat
      for (int64_t k = 0; k < ml; ++k) op[k] = m[k];
      op += ml;
    }
  }
  return -1;  // an empty block has no token
}

int decode_raw_forward_index(int type, const uint8_t* b, int64_t n, int32_t num_docs, int c, RawValues* out) {
  if (type == PGPU_STRING) return fail(PGPU_ERR_UNSUPPORTED, "column %d: raw STRING columns are not on the GPU path", c);
  if (!b || n < 16) return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: raw forward index too short", c);
  const int32_t version = (int32_t)rd_be32(b), num_chunks = (int32_t)rd_be32(b + 4);
  const int32_t per_chunk = (int32_t)rd_be32(b + 8), size = (int32_t)rd_be32(b + 12);
  if (version != 2 && version != 3)
    return fail(PGPU_ERR_UNSUPPORTED, "column %d: raw forward index version %d (2 and 3 are read)", c, version);
  if (n < 28) return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: raw forward index header truncated", c);
  const int32_t total = (int32_t)rd_be32(b + 16), compression = (int32_t)rd_be32(b + 20);
  const int32_t header_start = (int32_t)rd_be32(b + 24);
  // ChunkCompressionType: PASS_THROUGH 0, SNAPPY 1, ZSTANDARD 2, LZ4 3, LZ4_LENGTH_PREFIXED 4
  if (compression != 0 && compression != 3 && compression != 4)
    return fail(PGPU_ERR_UNSUPPORTED, "column %d: raw chunk compression type %d (PASS_THROUGH, LZ4 and "
                "LZ4_LENGTH_PREFIXED are read)", c, compression);
  const int want = (type == PGPU_INT || type == PGPU_FLOAT) ? 4 : 8;
  if (size != want) return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: raw entry size %d, type needs %d", c, size, want);
  if (num_chunks < 0 || per_chunk <= 0 || total < num_docs || (int64_t)num_chunks * per_chunk < num_docs)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: raw forward index covers %d docs, segment has %d", c, total,
                num_docs);
  const int entry = version == 2 ? 4 : 8;
  const int64_t data = (int64_t)header_start + (int64_t)num_chunks * entry;
  if (header_start < 28 || data > n || (compression == 0 && data + (int64_t)num_docs * size > n))
    return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: raw forward index too short for %d docs", c, num_docs);
  // A chunk decodes to at most min(numDocsPerChunk, totalDocs) entries, and an LZ4 block expands at most ~255x
  // (each sequence byte of a match length stands for <= 255 output bytes): a header claiming more is rejected
  // before anything is allocated.
  const int64_t chunk_bytes = compression ? std::min<int64_t>(per_chunk, total) * size : 0;
  if (compression && chunk_bytes > (n - data) * 256 + 64)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: raw chunk of %d docs cannot come from a %lld-byte index", c,
                per_chunk, (long long)n);
  std::vector<uint8_t> chunk;
  try {
    out->key.assign(std::max<int32_t>(num_docs, 1), 0);
    out->val.assign(std::max<int32_t>(num_docs, 1), 0.0);
    chunk.resize((size_t)chunk_bytes);
  } catch (const std::bad_alloc&) {
    return fail(PGPU_ERR_OUT_OF_MEMORY, "column %d: host memory for %d raw values", c, num_docs);
  }
  int64_t lo = INT64_MAX, hi = INT64_MIN;
  for (int64_t k = 0, d0 = 0; d0 < num_docs; ++k, d0 += per_chunk) {
    const int64_t nd = std::min<int64_t>(per_chunk, num_docs - d0);
    const uint8_t* v = b + data + d0 * size;
    if (compression) {
      auto chunk_pos = [&](int64_t i) {
        const uint8_t* e = b + header_start + i * entry;
        return entry == 4 ? (int64_t)rd_be32(e) : (int64_t)rd_be64(e);
      };
      const int64_t pos = chunk_pos(k), end = k + 1 < num_chunks ? chunk_pos(k + 1) : n;
      if (pos < data || end < pos || end > n)
        return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: chunk %lld outside the forward index", c, (long long)k);
      int64_t skip = compression == 4 ? 4 : 0;  // LZ4WithLength: little-endian decompressed length first
      if (end - pos < skip) return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: chunk %lld truncated", c, (long long)k);
      const int64_t got = lz4_decode_block(b + pos + skip, end - pos - skip, chunk.data(), (int64_t)chunk.size());
      if (got < nd * size)
        return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: LZ4 chunk %lld is malformed or short", c, (long long)k);
      v = chunk.data();
    }
    for (int64_t i = 0; i < nd; ++i, v += size) {
      const int64_t d = d0 + i;
      switch (type) {
        case PGPU_INT: { const int64_t x = (int32_t)rd_be32(v); out->key[d] = x; out->val[d] = (double)x; lo = std::min(lo, x); hi = std::max(hi, x); break; }
        case PGPU_LONG: { const int64_t x = (int64_t)rd_be64(v); out->key[d] = x; out->val[d] = (double)x; lo = std::min(lo, x); hi = std::max(hi, x); break; }
        case PGPU_FLOAT: {
          const uint32_t u = rd_be32(v);
          float f;
          memcpy(&f, &u, 4);
          out->val[d] = (double)f;
          out->key[d] = double_key(std::isnan(out->val[d]) ? kCanonicalNaN : out->val[d]);
          break;
        }
        default: {
          const uint64_t u = rd_be64(v);
          double x;
          memcpy(&x, &u, 8);
          out->val[d] = x;
          out->key[d] = double_key(std::isnan(x) ? kCanonicalNaN : x);
        }
      }
    }
  }
  out->lo = num_docs > 0 && lo <= hi ? lo : 0;
  out->hi = num_docs > 0 && lo <= hi ? hi : 0;
  return 0;
}

int parse_raw_column(int type, const pgpu_column_buffers& cb, int32_t num_docs, int c, Column* col, RawValues* out) {
  TRY(decode_raw_forward_index(type, cb.fwd, cb.fwd_len, num_docs, c, out));
  col->raw = true;
  col->card = 0;
  col->bits = 0;
  col->fwd_bytes = cb.fwd_len;
  col->raw_min = out->lo;
  col->raw_max = out->hi;
  return 0;
}

// Registers a segment whose columns have parsed dictionaries and device forward indexes.
void plan_cache_clear(pgpu_table_s* t);

int64_t register_segment(pgpu_table_s* t, std::unique_ptr<Segment> seg_in) {
  std::shared_ptr<Segment> seg(std::move(seg_in));
  t->version++;
  for (size_t c = 0; c < seg->cols.size(); ++c)
    if (merge_dict(t->global[c], seg->cols[c].dict)) t->global_version[c]++;
  int64_t h = t->next_handle++;
  seg->handle = h;
  if ((int64_t)t->by_handle.size() <= h) t->by_handle.resize(h + 1);
  t->by_handle[h] = seg;
  t->segments[h] = std::move(seg);
  plan_cache_clear(t);
  return h;
}

}  // namespace pgpu
