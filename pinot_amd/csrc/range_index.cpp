// range_index.cpp — range index files of dictionary-encoded columns (range_index.h) and their C ABI.
#include "range_index.h"

#include <string.h>

#include <string>

#include "../../include/pinotgpu.h"
#include "host_common.h"

namespace pgpu {

namespace {
constexpr int32_t kRangeV1 = 1;  // RangeIndexCreator.VERSION
constexpr int32_t kRangeV2 = 2;  // BitSlicedRangeIndexCreator.VERSION

int64_t be32(const uint8_t* b) {
  return (int64_t)(int32_t)(((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3]);
}
int64_t be64(const uint8_t* b) { return (int64_t)(((uint64_t)(uint32_t)be32(b) << 32) | (uint32_t)be32(b + 4)); }
}  // namespace

// RangeIndexReaderImpl.findRangeId (:198-205): the range the value falls in; -1 below the first range, num_ranges
// above the last one.
static int64_t find_range_id(const RangeIdx& r, int64_t v) {
  for (size_t i = 0; i < r.start.size(); ++i)
    if (v < r.start[i]) return (int64_t)i - 1;
  return v <= r.last_end ? (int64_t)r.start.size() - 1 : (int64_t)r.start.size();
}

int64_t RangeIdx::partial_entries(int64_t lo, int64_t hi) const {
  if (version != kRangeV1) return 0;  // BitSlicedRangeIndexReader.getPartiallyMatchingDocIds: null
  const int64_t first = find_range_id(*this, lo), last = find_range_id(*this, hi), n = (int64_t)start.size();
  auto out = [&](int64_t id) { return id < 0 || id >= n; };
  // getPartialMatchesInRange (:252-260); the ranges' bitmaps are disjoint, so the OR of two is the sum of their
  // sizes, and of one range with itself that range
  if (out(first)) return out(last) ? 0 : docs[last];
  if (out(last)) return docs[first];
  return first == last ? docs[first] : docs[first] + docs[last];
}

// RangeIndexReaderImpl's constructor (:46-104) over the file RangeIndexCreator.seal writes (RangeIndexCreator.java
// "RANGE INDEX FILE LAYOUT", big-endian): version, value type (length-prefixed name; "INT" for a dictionary-encoded
// column, whose values are dictIds), range count R, R range starts + the last range's end, R + 1 bitmap offsets
// (the last = the file size), then R portable Roaring bitmaps.  Every bitmap is read: the docs of each range, and
// all of them together must be the column's docs (a complete single-value index).
int parse_range_index(const uint8_t* b, int64_t n, int64_t card, int32_t num_docs, RangeIdx* out) {
  *out = RangeIdx();
  if (!b || n < 4) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "range index shorter than its version");
  const int32_t version = (int32_t)be32(b);
  if (version == kRangeV2) {
    // BitSlicedRangeIndexReader: version, min value (long), then a RangeBitmap -- exact answers, no partial scan; the
    // matches are the forward index's, so only the header is checked
    if (n < 12) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "bit-sliced range index shorter than its header");
    out->version = kRangeV2;
    return 0;
  }
  if (version != kRangeV1) return 0;  // DefaultIndexReaderProvider.newRangeIndexReader: unknown version, skipped
  int64_t off = 4;
  if (n < off + 4) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "range index header truncated");
  const int64_t tlen = be32(b + off);
  off += 4;
  if (tlen < 0 || tlen > 16 || off + tlen + 4 > n) return host_fail(PGPU_ERR_INVALID_ARGUMENT, "range index value type");
  const std::string type((const char*)b + off, (size_t)tlen);
  off += tlen;
  if (type != "INT")
    return host_fail(PGPU_ERR_INVALID_ARGUMENT, "range index of value type %s on a dictionary-encoded column",
                     type.c_str());
  const int64_t R = be32(b + off);
  off += 4;
  if (R < 1 || R > (int64_t)num_docs + 1 || off + (R + 1) * 4 + (R + 1) * 8 > n)
    return host_fail(PGPU_ERR_INVALID_ARGUMENT, "range index with %lld ranges", (long long)R);
  out->start.resize(R);
  for (int64_t i = 0; i < R; ++i) {
    out->start[i] = be32(b + off + 4 * i);
    if (out->start[i] < 0 || out->start[i] >= card || (i && out->start[i] <= out->start[i - 1]))
      return host_fail(PGPU_ERR_INVALID_ARGUMENT, "range index: range %lld starts at dictId %lld", (long long)i,
                       (long long)out->start[i]);
  }
  out->last_end = be32(b + off + 4 * R);
  if (out->last_end < out->start[R - 1] || out->last_end >= card)
    return host_fail(PGPU_ERR_INVALID_ARGUMENT, "range index: last range ends at dictId %lld", (long long)out->last_end);
  off += (R + 1) * 4;
  const int64_t bitmap_index = off;
  if (be64(b + bitmap_index + 8 * R) != n)  // Preconditions.checkState(lastOffset == dataBuffer.size())
    return host_fail(PGPU_ERR_INVALID_ARGUMENT, "range index: last offset %lld, file size %lld",
                     (long long)be64(b + bitmap_index + 8 * R), (long long)n);
  out->docs.resize(R);
  int64_t total = 0;
  for (int64_t i = 0; i < R; ++i) {
    const int64_t s = be64(b + bitmap_index + 8 * i), e = be64(b + bitmap_index + 8 * (i + 1));
    if (s < bitmap_index + 8 * (R + 1) || e < s || e > n)
      return host_fail(PGPU_ERR_INVALID_ARGUMENT, "range index: bitmap %lld at [%lld, %lld)", (long long)i,
                       (long long)s, (long long)e);
    if (!roaring_cardinality(b + s, e - s, num_docs, &out->docs[i]))
      return host_fail(PGPU_ERR_INVALID_ARGUMENT, "range index: malformed Roaring bitmap of range %lld", (long long)i);
    total += out->docs[i];
  }
  if (total != num_docs)
    return host_fail(PGPU_ERR_INVALID_ARGUMENT, "range index covers %lld of %d documents", (long long)total, num_docs);
  out->version = kRangeV1;
  return 0;
}

}  // namespace pgpu

extern "C" {

int pgpu_range_index_check(const void* bytes, int64_t num_bytes, int32_t cardinality, int32_t num_docs,
                           int32_t* version, int32_t* num_ranges, int64_t* total_docs) try {
  if ((!bytes && num_bytes) || num_bytes < 0 || cardinality < 0 || num_docs < 0)
    return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  pgpu::RangeIdx r;
  if (const int rc = pgpu::parse_range_index((const uint8_t*)bytes, num_bytes, cardinality, num_docs, &r)) return rc;
  if (version) *version = r.version;
  if (num_ranges) *num_ranges = (int32_t)r.start.size();
  if (total_docs) {
    *total_docs = 0;
    for (int64_t d : r.docs) *total_docs += d;
  }
  return 0;
} PGPU_ABI_CATCH

int pgpu_range_index_partial_entries(const void* bytes, int64_t num_bytes, int32_t cardinality, int32_t num_docs,
                                     int32_t lo, int32_t hi, int64_t* entries) try {
  if (!entries || (!bytes && num_bytes) || num_bytes < 0 || cardinality < 0 || num_docs < 0 || lo > hi)
    return pgpu::host_fail(PGPU_ERR_INVALID_ARGUMENT, "bad arguments");
  pgpu::RangeIdx r;
  if (const int rc = pgpu::parse_range_index((const uint8_t*)bytes, num_bytes, cardinality, num_docs, &r)) return rc;
  *entries = r.partial_entries(lo, hi);
  return 0;
} PGPU_ABI_CATCH

}  // extern "C"
