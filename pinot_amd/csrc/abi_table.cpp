// abi_table.cpp -- C ABI: library, tables, segments, inverted / range indexes.
#include "rt_decls.h"

// ================================================================================================ C ABI
extern "C" {

int pgpu_abi_version(void) { return PGPU_ABI_VERSION; }

namespace {
std::mutex g_init_mu;
int g_init_devices = 0;
}  // namespace

int pgpu_init(int n_gpus) try {
  PGPU_ABI_GUARD;
  install_crash_trace();
  int count = 0;
  HIP_TRY(hipGetDeviceCount(&count));
  if (n_gpus > count) return fail(PGPU_ERR_INVALID_ARGUMENT, "%d devices requested, %d visible", n_gpus, count);
  const int n = n_gpus > 0 ? n_gpus : count;
  std::lock_guard<std::mutex> g(g_init_mu);
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  for (int d = g_init_devices; d < n; ++d) {
    HIP_TRY(hipSetDevice(d));
    HIP_TRY(hipFree(nullptr));  // creates the device's context now
  }
  HIP_TRY(hipSetDevice(prev));
  g_init_devices = std::max(g_init_devices, n);
  host_pool();  // the planning workers start here, not inside the first query
  return n;
} PGPU_ABI_CATCH

int pgpu_shutdown(void) try {
  PGPU_ABI_GUARD;
  std::lock_guard<std::mutex> g(g_init_mu);
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  for (int d = 0; d < g_init_devices; ++d) {
    HIP_TRY(hipSetDevice(d));
    HIP_TRY(hipDeviceSynchronize());
  }
  HIP_TRY(hipSetDevice(prev));
  return 0;
} PGPU_ABI_CATCH

int pgpu_last_error(char* buf, size_t len) try {
  if (buf && len) {
    size_t n = std::min(len - 1, g_err.size());
    memcpy(buf, g_err.data(), n);
    buf[n] = 0;
  }
  return (int)g_err.size();
} PGPU_ABI_CATCH

int pgpu_device_count(int* count) try {
  PGPU_ABI_GUARD;
  if (!count) return fail(PGPU_ERR_INVALID_ARGUMENT, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) { *count = 0; return fail(PGPU_ERR_DEVICE, "hipGetDeviceCount: %s", hipGetErrorString(e)); }
  *count = n;
  return 0;
} PGPU_ABI_CATCH

int pgpu_table_create(int device, int num_columns, const char* const* names, const int32_t* types, pgpu_table* out) try {
  PGPU_ABI_GUARD;
  install_crash_trace();
  if (!out || num_columns <= 0 || !types) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad table arguments");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(PGPU_ERR_DEVICE, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(PGPU_ERR_INVALID_ARGUMENT, "device %d out of range", device);
  for (int i = 0; i < num_columns; ++i)
    if (types[i] < PGPU_INT || types[i] > PGPU_STRING) return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: bad type", i);
  auto t = std::make_unique<pgpu_table_s>();
  t->device = device;
  for (int i = 0; i < num_columns; ++i) {
    t->names.push_back(names && names[i] ? names[i] : ("col" + std::to_string(i)));
    t->types.push_back(types[i]);
    auto d = std::make_shared<Dict>();
    d->type = types[i];
    d->id = g_dict_ids.fetch_add(1);
    t->global.push_back(std::move(d));
    t->global_version.push_back(0);
    t->gvalues.emplace_back();
  }
  DeviceGuard g(device);
  HIP_TRY(hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking));
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
    t->num_cus = cus;
  *out = t.release();
  return 0;
} PGPU_ABI_CATCH

int pgpu_config_default(pgpu_config* out) try {
  PGPU_ABI_GUARD;
  if (!out) return fail(PGPU_ERR_INVALID_ARGUMENT, "null config");
  *out = default_config();
  return 0;
} PGPU_ABI_CATCH

int pgpu_table_set_config(pgpu_table t, const pgpu_config* c) try {
  PGPU_ABI_GUARD;
  if (!t || !c || c->struct_size <= (int32_t)offsetof(pgpu_config, plan_cache))
    return fail(PGPU_ERR_INVALID_ARGUMENT, "bad config arguments");
  // fields past the caller's struct keep their defaults
  pgpu_config v = default_config();
  memcpy(&v, c, std::min<size_t>((size_t)c->struct_size, sizeof v));
  v.struct_size = (int32_t)sizeof v;
  if (v.hash_partition_bits < 0 || v.hash_partition_bits > 14 || v.hash_partition_lds_kb < 0 ||
      v.hash_partition_lds_kb > 128 || v.lds_table_kb < 1 || v.lds_table_kb > 160 || v.plan_chunk_segments < 1 ||
      v.stream_chunks < 1 || v.star_tree_workgroups < 0 || !(v.dense_selectivity >= 0.0) ||
      !(v.slot_weight_step >= 0.0 && v.slot_weight_step <= 4.0))
    return fail(PGPU_ERR_INVALID_ARGUMENT, "config value out of range");
  {
    std::lock_guard<std::mutex> g(t->cfg_mu);
    t->cfg = v;
  }
  t->version.fetch_add(1);  // compiled plans were made with the previous settings
  plan_cache_clear(t);
  return 0;
} PGPU_ABI_CATCH

int pgpu_table_get_config(pgpu_table t, pgpu_config* out) try {
  PGPU_ABI_GUARD;
  if (!t || !out) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  *out = table_config(t);
  return 0;
} PGPU_ABI_CATCH

int pgpu_table_destroy(pgpu_table t) try {
  PGPU_ABI_GUARD;
  if (!t) return 0;
  DeviceGuard g(t->device);
  hipStreamSynchronize(t->stream);
  plan_cache_clear(t);
  t->segments.clear();  // freed here unless a live plan still holds a segment (destroy plans first)
  t->by_handle.clear();
  for (auto& s : t->scratch_pool) if (s) s->release();
  t->gen.pos.release(); t->gen.presence.release(); t->gen.code_to_pos.release(); t->gen.cdf.release();
  t->gen.pos_to_id.release();
  if (t->d_docid_fwd) hipFree(t->d_docid_fwd);
  if (t->d_docid_key) hipFree(t->d_docid_key);
  for (void* p : t->retired) hipFree(p);
  if (t->clock_stream) hipStreamDestroy(t->clock_stream);
  if (t->clock_pinned) hipHostFree(t->clock_pinned);
  hipStreamDestroy(t->stream);
  delete t;
  return 0;
} PGPU_ABI_CATCH

int pgpu_pin_segment(pgpu_table t, const pgpu_segment_desc* d, int64_t* handle) try {
  PGPU_ABI_GUARD;
  if (!t || !d || !handle) return fail(PGPU_ERR_INVALID_ARGUMENT, "null argument");
  if (d->num_columns != (int)t->names.size())
    return fail(PGPU_ERR_INVALID_ARGUMENT, "segment has %d columns, table has %zu", d->num_columns, t->names.size());
  if (d->num_docs < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "negative numDocs");
  DeviceGuard g(t->device);
  auto seg = std::make_unique<Segment>();
  seg->num_docs = d->num_docs;
  seg->cols.resize(d->num_columns);
  int64_t total_words = 0;
  std::vector<std::vector<uint32_t>> sorted_expansion(d->num_columns);
  std::vector<RawValues> raw_values(d->num_columns);
  bool any_raw = false;
  for (int c = 0; c < d->num_columns; ++c) {
    const pgpu_column_buffers& cb = d->columns[c];
    Column& col = seg->cols[c];
    col.card = cb.cardinality;
    col.entry_width = cb.entry_width;
    col.padding = cb.padding_byte;
    TRY(parse_dictionary(t->types[c], cb, &col.dict));
    if (cb.dict && cb.cardinality > 0) col.raw_dict.assign(cb.dict, cb.dict + (int64_t)cb.cardinality * cb.entry_width);
    if (cb.fwd_format == PGPU_FWD_FIXED_BIT) {
      col.bits = cb.bits_per_element;
      if (col.bits < 1 || col.bits > 31) return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: bitsPerElement %d", c, col.bits);
      const int64_t need = ((int64_t)d->num_docs * col.bits + 7) / 8;
      if (d->num_docs > 0 && (!cb.fwd || cb.fwd_len < need))
        return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: forward index has %lld bytes, needs %lld", c,
                    (long long)cb.fwd_len, (long long)need);
      col.fwd_bytes = need;
    } else if (cb.fwd_format == PGPU_FWD_SORTED_PAIRS) {
      // SortedIndexReaderImpl (start, end) pairs -> the fixed-bit layout the kernels read.
      if (cb.fwd_len < (int64_t)cb.cardinality * 8) return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: sorted index too small", c);
      col.bits = num_bits_per_value(cb.cardinality - 1);
      col.fwd_bytes = ((int64_t)d->num_docs * col.bits + 7) / 8;
      std::vector<uint32_t>& w = sorted_expansion[c];
      w.assign(padded_fwd_words(d->num_docs, col.bits), 0u);
      col.sorted = true;
      col.sorted_start.assign((size_t)cb.cardinality + 1, d->num_docs);
      int32_t prev_end = -1;
      for (int32_t id = 0; id < cb.cardinality; ++id) {
        const int32_t s = (int32_t)rd_be32(cb.fwd + (int64_t)id * 8), e = (int32_t)rd_be32(cb.fwd + (int64_t)id * 8 + 4);
        if (s < 0 || e >= d->num_docs || (e < s && e != s - 1)) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad sorted pair");
        if (s != prev_end + 1) return fail(PGPU_ERR_INVALID_ARGUMENT, "sorted pairs are not contiguous");
        prev_end = e;
        col.sorted_start[id] = s;
        for (int32_t doc = s; doc <= e; ++doc) {  // PinotDataBitSet.writeInt into BE words
          const uint64_t bit = (uint64_t)doc * col.bits;
          for (int b = 0; b < col.bits; ++b)
            if ((id >> (col.bits - 1 - b)) & 1) {
              const uint64_t pos = bit + b;
              w[pos >> 5] |= 1u << (31 - (pos & 31));
            }
        }
      }
      if (d->num_docs > 0 && prev_end != d->num_docs - 1)
        return fail(PGPU_ERR_INVALID_ARGUMENT, "sorted pairs do not cover every doc");
      for (auto& x : w) x = __builtin_bswap32(x);  // the device reads the forward index as big-endian bytes
    } else if (cb.fwd_format == PGPU_FWD_RAW_FIXED) {
      TRY(parse_raw_column(t->types[c], cb, d->num_docs, c, &col, &raw_values[c]));
      any_raw = true;
      continue;  // no per-segment forward-index words: the values live in d_key / d_val
    } else {
      return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: bad forward-index format", c);
    }
    col.fwd_words = padded_fwd_words(d->num_docs, col.bits);
    total_words += (col.fwd_words + 63) & ~int64_t(63);  // 256-byte aligned columns
  }
  HIP_TRY(hipMalloc(&seg->d_block, (size_t)std::max<int64_t>(total_words, 64) * 4));
  t->device_bytes += std::max<int64_t>(total_words, 64) * 4;
  int64_t off = 0;
  for (int c = 0; c < d->num_columns; ++c) {
    Column& col = seg->cols[c];
    if (col.raw) {
      const size_t n = (size_t)raw_padded_docs(d->num_docs);
      raw_values[c].key.resize(n, 0);
      raw_values[c].val.resize(n, 0.0);
      HIP_TRY(hipMalloc(&col.d_key, n * 8));
      HIP_TRY(hipMalloc(&col.d_val, n * 8));
      t->device_bytes += 16 * (int64_t)n;
      HIP_TRY(hipMemcpyAsync(col.d_key, raw_values[c].key.data(), n * 8, hipMemcpyHostToDevice, t->stream));
      HIP_TRY(hipMemcpyAsync(col.d_val, raw_values[c].val.data(), n * 8, hipMemcpyHostToDevice, t->stream));
      continue;
    }
    col.d_fwd = reinterpret_cast<uint32_t*>(seg->d_block) + off;
    const pgpu_column_buffers& cb = d->columns[c];
    HIP_TRY(hipMemsetAsync(col.d_fwd, 0, (size_t)col.fwd_words * 4, t->stream));
    if (cb.fwd_format == PGPU_FWD_SORTED_PAIRS) {
      HIP_TRY(hipMemcpyAsync(col.d_fwd, sorted_expansion[c].data(), (size_t)col.fwd_words * 4, hipMemcpyHostToDevice,
                             t->stream));
    } else if (col.fwd_bytes > 0) {
      HIP_TRY(hipMemcpyAsync(col.d_fwd, cb.fwd, (size_t)col.fwd_bytes, hipMemcpyHostToDevice, t->stream));
    }
    off += (col.fwd_words + 63) & ~int64_t(63);
  }
  // dictIds within the dictionary (fwd_max_kernel): only columns whose bit width can hold values >= cardinality
  std::vector<int> check;
  for (int c = 0; c < d->num_columns; ++c) {
    const Column& col = seg->cols[c];
    if (!col.raw && !col.sorted && d->num_docs > 0 && (int64_t)col.card < (INT64_C(1) << col.bits)) check.push_back(c);
  }
  DevBuf dmax;
  struct Release { DevBuf& b; ~Release() { b.release(); } } release_dmax{dmax};
  std::vector<uint32_t> hmax(check.size(), 0);
  if (!check.empty()) {
    TRY(dmax.ensure(check.size() * 4));
    HIP_TRY(hipMemsetAsync(dmax.p, 0, check.size() * 4, t->stream));
    for (size_t i = 0; i < check.size(); ++i)
      if (launch_fwd_max(seg->cols[check[i]].d_fwd, d->num_docs, seg->cols[check[i]].bits,
                         dmax.as<unsigned int>() + i, t->stream))
        return fail(PGPU_ERR_DEVICE, "forward-index check launch failed: %s", hipGetErrorString(hipGetLastError()));
    HIP_TRY(hipMemcpyAsync(hmax.data(), dmax.p, check.size() * 4, hipMemcpyDeviceToHost, t->stream));
  }
  HIP_TRY(hipStreamSynchronize(t->stream));
  for (size_t i = 0; i < check.size(); ++i)
    if ((int64_t)hmax[i] >= seg->cols[check[i]].card) {
      account_unpin(t, seg.get());
      return fail(PGPU_ERR_INVALID_ARGUMENT, "column %d: forward index holds dictId %u, cardinality is %d", check[i],
                  hmax[i], seg->cols[check[i]].card);
    }
  std::lock_guard<std::mutex> lk(t->mu);
  if (any_raw) TRY(ensure_docid(t, d->num_docs, t->stream));
  *handle = register_segment(t, std::move(seg));
  return 0;
} PGPU_ABI_CATCH

int pgpu_unpin_segment(pgpu_table t, int64_t h) try {
  PGPU_ABI_GUARD;
  if (t) t->version++;
  if (!t) return fail(PGPU_ERR_INVALID_ARGUMENT, "null table");
  DeviceGuard g(t->device);
  std::shared_ptr<Segment> seg;  // released after the table mutex (the free may wait for the device)
  {
    std::lock_guard<std::mutex> lk(t->mu);
    auto it = t->segments.find(h);
    if (it == t->segments.end()) return fail(PGPU_ERR_NOT_FOUND, "unknown segment handle %lld", (long long)h);
    seg = std::move(it->second);
    account_unpin(t, seg.get());
    t->by_handle[h].reset();
    t->segments.erase(it);
  }
  plan_cache_clear(t);  // cached plans reference the segment set of their time
  hipStreamSynchronize(t->stream);  // work queued on the table's own stream (pins, reads) is done with it
  return 0;
} PGPU_ABI_CATCH

namespace {
// Portable RoaringBitmap deserialisation (RoaringBitmap 0.9.x RoaringArray.deserialize, little-endian): cookie
// 12346 (no run containers; u32 size follows) or 12347 | (size - 1) << 16 (with a run-container bitmap); per
// container (u16 key, u16 card - 1); offsets (u32, skipped) unless a run-cookie bitmap has < 4 containers; then
// ARRAY (card <= 4096: u16 values), BITMAP (1024 u64) or RUN (u16 count, (u16 start, u16 length - 1) pairs).
// Appends device-layout payload words and container entries; returns false on malformed input.
bool parse_roaring(const uint8_t* b, int64_t n, int32_t num_docs, std::vector<uint32_t>& words,
                   std::vector<InvIndex::Cont>& conts, int64_t* docs) {
  auto u16 = [&](int64_t o) { return (uint32_t)b[o] | ((uint32_t)b[o + 1] << 8); };
  auto u32 = [&](int64_t o) { return u16(o) | (u16(o + 2) << 16); };
  if (n < 4) return false;
  const uint32_t cookie = u32(0);
  int64_t pos, size;
  const uint8_t* runbits = nullptr;
  bool offsets;
  if ((cookie & 0xFFFF) == 12347) {
    size = (cookie >> 16) + 1;
    runbits = b + 4;
    pos = 4 + (size + 7) / 8;
    offsets = size >= 4;
  } else if (cookie == 12346) {
    if (n < 8) return false;
    size = u32(4);
    pos = 8;
    offsets = true;
  } else {
    return false;
  }
  if (size < 0 || size > 65536 || pos + size * 4 > n) return false;
  const int64_t desc = pos;
  pos += size * 4 + (offsets ? size * 4 : 0);
  *docs = 0;
  int32_t prev_key = -1;
  std::vector<uint32_t> vals;
  for (int64_t i = 0; i < size; ++i) {
    const int32_t key = (int32_t)u16(desc + 4 * i);
    const int32_t card = (int32_t)u16(desc + 4 * i + 2) + 1;
    if (key <= prev_key || ((int64_t)key << 16) >= num_docs) return false;
    prev_key = key;
    const bool run = runbits && ((runbits[i >> 3] >> (i & 7)) & 1);
    vals.clear();
    std::vector<uint32_t> bm;
    if (run) {
      if (pos + 2 > n) return false;
      const int64_t nruns = u16(pos);
      pos += 2;
      if (pos + nruns * 4 > n) return false;
      for (int64_t r = 0; r < nruns; ++r) {
        const uint32_t start = u16(pos + 4 * r), len = u16(pos + 4 * r + 2);
        if (start + len > 65535) return false;
        // the runs may not hold more values than the declared cardinality (bounds the expansion)
        if ((int64_t)vals.size() + len + 1 > card) return false;
        for (uint32_t v = start; v <= start + len; ++v) vals.push_back(v);
      }
      pos += nruns * 4;
    } else if (card <= 4096) {
      if (pos + (int64_t)card * 2 > n) return false;
      for (int32_t k = 0; k < card; ++k) vals.push_back(u16(pos + 2 * k));
      pos += (int64_t)card * 2;
    } else {
      if (pos + 8192 > n) return false;
      bm.resize(kContainerWords);
      for (int w = 0; w < kContainerWords; ++w) bm[w] = u32(pos + 4 * w);
      pos += 8192;
    }
    int64_t c = 0;
    if (bm.empty()) {
      if ((int64_t)vals.size() != card) return false;
      if (vals.size() > 4096) {  // long runs: bitmap form
        bm.assign(kContainerWords, 0);
        for (uint32_t v : vals) bm[v >> 5] |= 1u << (v & 31);
      }
    }
    if (!bm.empty()) {
      int32_t top = -1;
      for (int w = 0; w < kContainerWords; ++w)
        if (bm[w]) { c += __builtin_popcount(bm[w]); top = w * 32 + 31 - __builtin_clz(bm[w]); }
      if (((int64_t)key << 16) + top >= num_docs) return false;
      if (c != card) return false;  // overlapping runs / a bitmap whose popcount is not its cardinality
      conts.push_back({(int64_t)words.size(), CONT_BITMAP, (int32_t)c, key});
      words.insert(words.end(), bm.begin(), bm.end());
    } else {
      for (size_t k = 1; k < vals.size(); ++k)
        if (vals[k] <= vals[k - 1]) return false;
      if (!vals.empty() && ((int64_t)key << 16) + vals.back() >= num_docs) return false;
      c = (int64_t)vals.size();
      conts.push_back({(int64_t)words.size(), CONT_ARRAY, (int32_t)c, key});
      for (size_t k = 0; k < vals.size(); k += 2)
        words.push_back(vals[k] | (k + 1 < vals.size() ? vals[k + 1] << 16 : 0u));
    }
    *docs += c;
  }
  return pos <= n;
}

// A `<column>.bitmap.inv` file (BitmapInvertedIndexReader.java:40-70): (card + 1) big-endian int32 bitmap offsets,
// then one portable Roaring bitmap per dictId, parsed into `inv`'s per-dictId container lists and the device
// payload `words`.  Pure host code (pgpu_attach_inverted_index, pgpu_inverted_index_check).
int parse_inverted_index(const uint8_t* b, int64_t num_bytes, int64_t card, int32_t num_docs, int column,
                         InvIndex* inv, std::vector<uint32_t>& words) {
  if (card < 0 || num_docs < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad cardinality / document count");
  const int64_t hdr = (card + 1) * 4;
  if (!b || num_bytes < hdr) return fail(PGPU_ERR_INVALID_ARGUMENT, "inverted index shorter than its offset header");
  auto be32 = [&](int64_t o) {
    return (int64_t)(int32_t)(((uint32_t)b[o] << 24) | ((uint32_t)b[o + 1] << 16) | ((uint32_t)b[o + 2] << 8) | b[o + 3]);
  };
  inv->ids.assign(card, InvIndex::Entry{0, 0, 0});
  const int64_t first = be32(0);
  for (int64_t id = 0; id < card; ++id) {
    const int64_t off = be32(id * 4) - first, end = be32((id + 1) * 4) - first;
    inv->ids[id].begin = (int32_t)inv->conts.size();
    if (off < 0 || end < off || hdr + end > num_bytes)
      return fail(PGPU_ERR_INVALID_ARGUMENT, "bitmap %lld of column %d overruns the index", (long long)id, column);
    if (!parse_roaring(b + hdr + off, end - off, num_docs, words, inv->conts, &inv->ids[id].docs))
      return fail(PGPU_ERR_INVALID_ARGUMENT, "malformed Roaring bitmap for dictId %lld of column %d", (long long)id,
                  column);
  }
  for (int64_t id = 0; id < card; ++id)
    inv->ids[id].count = (int32_t)((id + 1 < card ? inv->ids[id + 1].begin : (int32_t)inv->conts.size()) -
                                   inv->ids[id].begin);
  return 0;
}
}  // namespace

}  // extern "C"
bool pgpu::roaring_cardinality(const uint8_t* b, int64_t n, int32_t num_docs, int64_t* docs) {
  std::vector<uint32_t> words;
  std::vector<InvIndex::Cont> conts;
  return parse_roaring(b, n, num_docs, words, conts, docs);
}
extern "C" {

namespace {
void put_le16(std::vector<uint8_t>& o, uint32_t v) { o.push_back((uint8_t)v); o.push_back((uint8_t)(v >> 8)); }
void put_le32(std::vector<uint8_t>& o, uint32_t v) { put_le16(o, v & 0xFFFF); put_le16(o, v >> 16); }

// RoaringBitmap.serialize of a sorted docId list without run containers (cookie 12346).
void serialize_roaring_plain(const int32_t* docs, int64_t n, std::vector<uint8_t>& o) {
  std::vector<std::pair<int64_t, int64_t>> conts;  // [begin, end) per key
  for (int64_t i = 0; i < n;) {
    int64_t j = i;
    while (j < n && (docs[j] >> 16) == (docs[i] >> 16)) ++j;
    conts.emplace_back(i, j);
    i = j;
  }
  const size_t base = o.size();
  put_le32(o, 12346);
  put_le32(o, (uint32_t)conts.size());
  for (auto& c : conts) {
    put_le16(o, (uint32_t)(docs[c.first] >> 16));
    put_le16(o, (uint32_t)(c.second - c.first - 1));
  }
  uint32_t off = (uint32_t)(o.size() - base + 4 * conts.size());
  for (auto& c : conts) {
    put_le32(o, off);
    const int64_t card = c.second - c.first;
    off += card <= 4096 ? (uint32_t)(2 * card) : 8192u;
  }
  for (auto& c : conts) {
    const int64_t card = c.second - c.first;
    if (card <= 4096) {
      for (int64_t k = c.first; k < c.second; ++k) put_le16(o, (uint32_t)(docs[k] & 0xFFFF));
    } else {
      std::vector<uint32_t> bm(kContainerWords, 0);
      for (int64_t k = c.first; k < c.second; ++k) bm[(docs[k] & 0xFFFF) >> 5] |= 1u << (docs[k] & 31);
      for (uint32_t w : bm) put_le32(o, w);
    }
  }
}
}  // namespace

// Host-side inverted-index creator (OffHeapBitmapInvertedIndexCreator + BitmapInvertedIndexWriter,
// seglocal/segment/creator/impl/inv/BitmapInvertedIndexWriter.java:60-78): dictIds of the MSB-first fixed-bit
// forward index -> per dictId the sorted docIds -> (card + 1) BE offsets + serialised bitmaps.
int pgpu_build_inverted_index(const void* fwd, int64_t fwd_len, int32_t bits, int32_t num_docs, int32_t cardinality,
                              void* out, int64_t out_cap, int64_t* out_len) try {
  PGPU_ABI_GUARD;
  if (!fwd || !out_len || bits < 1 || bits > 31 || num_docs < 0 || cardinality < 1 ||
      fwd_len < ((int64_t)num_docs * bits + 7) / 8)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "bad inverted-index build arguments");
  const uint8_t* b = reinterpret_cast<const uint8_t*>(fwd);
  std::vector<int32_t> ids(num_docs);
  for (int64_t d = 0; d < num_docs; ++d) {
    const int64_t bit = d * bits;
    uint64_t w = 0;
    for (int k = 0; k < 5; ++k) {
      const int64_t byte = (bit >> 3) + k;
      w = (w << 8) | (byte < fwd_len ? b[byte] : 0);
    }
    ids[d] = (int32_t)((w >> (40 - (bit & 7) - bits)) & ((1u << bits) - 1u));
    if (ids[d] >= cardinality) return fail(PGPU_ERR_INVALID_ARGUMENT, "dictId %d >= cardinality", ids[d]);
  }
  std::vector<int64_t> start(cardinality + 1, 0);
  for (int32_t id : ids) start[id + 1]++;
  for (int32_t i = 0; i < cardinality; ++i) start[i + 1] += start[i];
  std::vector<int32_t> docs(num_docs);
  {
    std::vector<int64_t> fill(start.begin(), start.end() - 1);
    for (int32_t d = 0; d < num_docs; ++d) docs[fill[ids[d]]++] = d;
  }
  std::vector<uint8_t> body;
  std::vector<uint32_t> offs(cardinality + 1);
  const uint32_t hdr = 4u * (uint32_t)(cardinality + 1);
  for (int32_t i = 0; i < cardinality; ++i) {
    offs[i] = hdr + (uint32_t)body.size();
    serialize_roaring_plain(docs.data() + start[i], start[i + 1] - start[i], body);
  }
  offs[cardinality] = hdr + (uint32_t)body.size();
  *out_len = (int64_t)hdr + (int64_t)body.size();
  if (!out) return 0;
  if (out_cap < *out_len) return fail(PGPU_ERR_INVALID_ARGUMENT, "output buffer too small");
  uint8_t* o = reinterpret_cast<uint8_t*>(out);
  for (int32_t i = 0; i <= cardinality; ++i) {
    o[4 * i] = (uint8_t)(offs[i] >> 24); o[4 * i + 1] = (uint8_t)(offs[i] >> 16);
    o[4 * i + 2] = (uint8_t)(offs[i] >> 8); o[4 * i + 3] = (uint8_t)offs[i];
  }
  memcpy(o + hdr, body.data(), body.size());
  return 0;
} PGPU_ABI_CATCH

int pgpu_raw_forward_index_values(const void* fwd, int64_t fwd_len, int32_t data_type, int32_t num_docs,
                                  int64_t* out_i64, double* out_f64) try {
  PGPU_ABI_GUARD;
  if (!fwd || num_docs < 0 || data_type < PGPU_INT || data_type > PGPU_STRING)
    return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  RawValues v;
  TRY(decode_raw_forward_index(data_type, reinterpret_cast<const uint8_t*>(fwd), fwd_len, num_docs, 0, &v));
  for (int32_t i = 0; i < num_docs; ++i) {
    if (out_i64) out_i64[i] = is_int_type(data_type) ? v.key[i] : 0;
    if (out_f64) out_f64[i] = v.val[i];
  }
  return 0;
} PGPU_ABI_CATCH

int pgpu_inverted_index_check(const void* bytes, int64_t num_bytes, int32_t cardinality, int32_t num_docs,
                              int64_t* total_docs) try {
  PGPU_ABI_GUARD;
  if (!bytes && num_bytes) return fail(PGPU_ERR_INVALID_ARGUMENT, "null argument");
  InvIndex inv;
  std::vector<uint32_t> words;
  TRY(parse_inverted_index(reinterpret_cast<const uint8_t*>(bytes), num_bytes, cardinality, num_docs, -1, &inv,
                           words));
  if (total_docs) {
    *total_docs = 0;
    for (const auto& e : inv.ids) *total_docs += e.docs;
  }
  return 0;
} PGPU_ABI_CATCH

int pgpu_attach_inverted_index(pgpu_table t, int64_t h, int32_t column, const void* bytes, int64_t num_bytes) try {
  PGPU_ABI_GUARD;
  if (t) t->version++;
  if (t) plan_cache_clear(t);
  if (!t || (!bytes && num_bytes)) return fail(PGPU_ERR_INVALID_ARGUMENT, "null argument");
  DeviceGuard g(t->device);
  std::lock_guard<std::mutex> lk(t->mu);
  auto it = t->segments.find(h);
  if (it == t->segments.end()) return fail(PGPU_ERR_NOT_FOUND, "unknown segment handle %lld", (long long)h);
  Segment& seg = *it->second;
  if (column < 0 || column >= (int)seg.cols.size()) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad column %d", column);
  Column& col = seg.cols[column];
  auto inv = std::make_shared<InvIndex>();
  std::vector<uint32_t> words;
  TRY(parse_inverted_index(reinterpret_cast<const uint8_t*>(bytes), num_bytes, col.card, seg.num_docs, column,
                           inv.get(), words));
  inv->bytes = (int64_t)std::max<size_t>(words.size(), 1) * 4;
  HIP_TRY(hipMalloc(&inv->d_block, inv->bytes));
  if (!words.empty()) HIP_TRY(hipMemcpy(inv->d_block, words.data(), words.size() * 4, hipMemcpyHostToDevice));
  if (col.inv) t->device_bytes -= col.inv->bytes;  // freed when the last plan using it is destroyed
  t->device_bytes += inv->bytes;
  col.inv = inv;
  return 0;
} PGPU_ABI_CATCH

int pgpu_attach_range_index(pgpu_table t, int64_t h, int32_t column, const void* bytes, int64_t num_bytes) try {
  PGPU_ABI_GUARD;
  if (!t || (!bytes && num_bytes) || num_bytes < 0) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  t->version++;
  plan_cache_clear(t);
  std::lock_guard<std::mutex> lk(t->mu);
  auto it = t->segments.find(h);
  if (it == t->segments.end()) return fail(PGPU_ERR_NOT_FOUND, "unknown segment handle %lld", (long long)h);
  Segment& seg = *it->second;
  if (column < 0 || column >= (int)seg.cols.size()) return fail(PGPU_ERR_INVALID_ARGUMENT, "bad column %d", column);
  Column& col = seg.cols[column];
  if (num_bytes == 0) {
    col.rng.reset();
    return 0;
  }
  if (col.raw) return fail(PGPU_ERR_UNSUPPORTED, "range index on raw (no-dictionary) column %d", column);
  auto r = std::make_shared<RangeIdx>();
  TRY(parse_range_index(reinterpret_cast<const uint8_t*>(bytes), num_bytes, col.card, seg.num_docs, r.get()));
  if (r->version == 0) col.rng.reset();  // a version Pinot does not load: no range index
  else col.rng = r;
  return 0;
} PGPU_ABI_CATCH

}  // extern "C"

