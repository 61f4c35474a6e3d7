/*
 * oracle.c — CPU restatement of Pinot's server filter -> group-by -> aggregation path.
 * TEST INFRASTRUCTURE ONLY (see oracle.h): the checker and the CPU baseline, never the product.
 *
 * Path abbreviations: seglocal/ = pinot-segment-local/src/main/java/org/apache/pinot/segment/local/,
 * core/ = pinot-core/src/main/java/org/apache/pinot/core/.
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <errno.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define EOF_DOC INT32_MIN /* segspi Constants.EOF = Integer.MIN_VALUE */
#define MAX_DOC_PER_CALL 10000 /* core/plan/DocIdSetPlanNode.java:29 */
#define INVALID_ID (-1)        /* GroupKeyGenerator.INVALID_ID */

/* ======================================================================================= codec */

/* PinotDataBitSet.getNumBitsPerValue (seglocal/io/util/PinotDataBitSet.java:59-70). */
int or_num_bits_per_value(int max_value) {
  if (max_value <= 1) return 1;
  int nbits = 8;
  unsigned v = (unsigned)max_value;
  while (v > 0xFF) {
    v >>= 8;
    nbits += 8;
  }
  int first_bit_set = 0; /* FIRST_BIT_SET[v]: index of the highest set bit counted from the MSB of the byte */
  while (!(v & (0x80u >> first_bit_set))) first_bit_set++;
  return nbits - first_bit_set;
}

/* PinotDataBitSet.readInt(index, numBitsPerValue) (:78-100). */
int32_t or_bitset_read_int(const uint8_t* buf, int64_t index, int nbits) {
  int64_t bit_offset = index * nbits;
  int64_t byte_offset = bit_offset / 8;
  int bit_in_first = (int)(bit_offset % 8);
  uint32_t cur = buf[byte_offset] & (0xFFu >> bit_in_first);
  int left = nbits - (8 - bit_in_first);
  if (left <= 0) return (int32_t)(cur >> -left);
  while (left > 8) {
    byte_offset++;
    cur = (cur << 8) | buf[byte_offset];
    left -= 8;
  }
  return (int32_t)((cur << left) | ((uint32_t)buf[byte_offset + 1] >> (8 - left)));
}

/* PinotDataBitSet.readInt(startIndex, numBitsPerValue, length, buffer) (:102-136). */
void or_bitset_read_ints(const uint8_t* buf, int64_t start, int nbits, int len, int32_t* out) {
  int64_t bit_offset = start * nbits;
  int64_t byte_offset = bit_offset / 8;
  int bit_in_first = (int)(bit_offset % 8);
  uint32_t cur = buf[byte_offset] & (0xFFu >> bit_in_first);
  for (int i = 0; i < len; i++) {
    if (bit_in_first == 8) {
      bit_in_first = 0;
      byte_offset++;
      cur = buf[byte_offset];
    }
    int left = nbits - (8 - bit_in_first);
    if (left <= 0) {
      out[i] = (int32_t)(cur >> -left);
      bit_in_first = 8 + left;
      cur = cur & (0xFFu >> bit_in_first);
    } else {
      while (left > 8) {
        byte_offset++;
        cur = (cur << 8) | buf[byte_offset];
        left -= 8;
      }
      byte_offset++;
      uint32_t next = buf[byte_offset];
      out[i] = (int32_t)((cur << left) | (next >> (8 - left)));
      bit_in_first = left;
      cur = next & (0xFFu >> bit_in_first);
    }
  }
}

/* PinotDataBitSet.writeInt(index, numBitsPerValue, value) (:138-165). */
void or_bitset_write_int(uint8_t* buf, int64_t index, int nbits, int32_t value) {
  int64_t bit_offset = index * nbits;
  int64_t byte_offset = bit_offset / 8;
  int bit_in_first = (int)(bit_offset % 8);
  uint32_t v = (uint32_t)value;
  uint32_t first = buf[byte_offset];
  uint32_t first_mask = 0xFFu >> bit_in_first;
  int left = nbits - (8 - bit_in_first);
  if (left <= 0) {
    first_mask &= 0xFFu << -left;
    buf[byte_offset] = (uint8_t)((first & ~first_mask) | (v << -left));
  } else {
    buf[byte_offset] = (uint8_t)((first & ~first_mask) | ((v >> left) & first_mask));
    while (left > 8) {
      left -= 8;
      byte_offset++;
      buf[byte_offset] = (uint8_t)(v >> left);
    }
    byte_offset++;
    uint32_t last = buf[byte_offset];
    buf[byte_offset] = (uint8_t)((last & (0xFFu >> left)) | (v << (8 - left)));
  }
}

/* PinotDataBitSet.writeInt(startIndex, numBitsPerValue, length, values) (:167-205); per-value form is equivalent. */
void or_bitset_write_ints(uint8_t* buf, int64_t start, int nbits, int len, const int32_t* values) {
  for (int i = 0; i < len; i++) or_bitset_write_int(buf, start + i, nbits, values[i]);
}

int64_t or_fwd_num_bytes(int64_t num_values, int nbits) { return (num_values * nbits + 7) / 8; }

/* FixedBitIntReader.read/readUnchecked for every width (seglocal/io/reader/impl/FixedBitIntReader.java:37-119,
 * e.g. Bit9Reader :656-725) return the same value as PinotDataBitSet.readInt; read32 decodes 32 values from
 * 4*b bytes at byte offset (index/8)*b.  Restated as one generic BE/MSB-first extraction. */
static inline int32_t fixedbit_read(const uint8_t* fwd, int64_t index, int nbits) {
  return or_bitset_read_int(fwd, index, nbits);
}

/* FixedBitSVForwardIndexReaderV2.readDictIds (:62-96): bulk read32 when docIds are contiguous and >= 64 long,
 * per-doc reads otherwise.  The bulk and per-doc paths decode identical values, so the restatement keeps the
 * control flow (which docs go through which path) and one decoder. */
void or_read_dict_ids(const uint8_t* fwd, int nbits, int num_docs, const int32_t* doc_ids, int len, int32_t* out) {
  (void)num_docs;
  if (len <= 0) return;
  int first = doc_ids[0], last = doc_ids[len - 1];
  int index = 0;
  if (last - first + 1 == len && len >= 64) {
    int bulk_start = (first + 31) & ~31;
    int bulk_end = last & ~31;
    for (int i = first; i < bulk_start; i++) out[index++] = fixedbit_read(fwd, i, nbits);
    for (int i = bulk_start; i < bulk_end; i += 32) {
      or_bitset_read_ints(fwd, i, nbits, 32, out + index); /* read32 */
      index += 32;
    }
  }
  for (int i = index; i < len; i++) out[i] = fixedbit_read(fwd, doc_ids[i], nbits);
}

/* ======================================================================================= dictionaries */

static inline uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
static inline uint64_t be64(const uint8_t* p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); }
static inline void put_be32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}
static inline void put_be64(uint8_t* p, uint64_t v) { put_be32(p, (uint32_t)(v >> 32)); put_be32(p + 4, (uint32_t)v); }

static inline int32_t dict_int(const or_column* c, int id) { return (int32_t)be32(c->dict + (int64_t)id * 4); }
static inline int64_t dict_long(const or_column* c, int id) { return (int64_t)be64(c->dict + (int64_t)id * 8); }
static inline float dict_float(const or_column* c, int id) {
  uint32_t u = be32(c->dict + (int64_t)id * 4); float f; memcpy(&f, &u, 4); return f;
}
static inline double dict_double(const or_column* c, int id) {
  uint64_t u = be64(c->dict + (int64_t)id * 8); double d; memcpy(&d, &u, 8); return d;
}
/* FixedByteValueReaderWriter.getUnpaddedString (seglocal/io/util/FixedByteValueReaderWriter.java:57-95):
 * bytes up to the first padding byte. */
static inline int dict_str(const or_column* c, int id, const uint8_t** p) {
  const uint8_t* s = c->dict + (int64_t)id * c->entry_width;
  int n = 0;
  while (n < c->entry_width && s[n] != (uint8_t)c->padding_byte) n++;
  *p = s;
  return n;
}

/* LZ4 block decompression (the published LZ4 block format, as lz4-java's LZ4SafeDecompressor implements it for
 * LZ4Decompressor / LZ4WithLengthDecompressor, seglocal/io/compression/LZ4Decompressor.java:40-50; lz4-java is a
 * Maven dependency absent from /root/reference): a block is a sequence of (token, literal length extension bytes,
 * literals, 2-byte little-endian match offset, match length extension bytes); token = literal length (high nibble)
 * | match length - 4 (low nibble), 15 = extended by 255-continued bytes; the last sequence has literals only.
 * Returns the decoded length, or -1 on malformed input or output overflow. */
int64_t or_lz4_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap) {
  int64_t ip = 0, op = 0;
  for (;;) {
    if (ip >= n) return -1;
    const int token = src[ip++];
    int64_t lit = token >> 4;
    if (lit == 15) {
      int b;
      do { if (ip >= n) return -1; b = src[ip++]; lit += b; } while (b == 255);
    }
    if (lit > n - ip || lit > cap - op) return -1;
    memcpy(dst + op, src + ip, (size_t)lit);
    ip += lit;
    op += lit;
    if (ip == n) return op;  /* the last sequence: literals only */
    if (n - ip < 2) return -1;
    const int64_t off = (int64_t)src[ip] | ((int64_t)src[ip + 1] << 8);
    ip += 2;
    if (off == 0 || off > op) return -1;
    int64_t ml = (token & 15);
    if (ml == 15) {
      int b;
      do { if (ip >= n) return -1; b = src[ip++]; ml += b; } while (b == 255);
    }
    ml += 4;
    if (ml > cap - op) return -1;
    for (int64_t k = 0; k < ml; k++, op++) dst[op] = dst[op - off]; /* overlapping copies repeat the pattern */
  }
}

/* FixedByteChunkSVForwardIndexReader over every chunk (BaseChunkSVForwardIndexReader.java:56-154): header (version,
 * numChunks, numDocsPerChunk, sizeOfEntry; version >= 2: totalDocs, compression type, dataHeaderStart), chunk
 * offsets (int for versions 1-2, long for 3), each chunk decompressed on its own (getChunkPosition; the last chunk
 * runs to the end of the buffer).  Compression: PASS_THROUGH (0), LZ4 (3), LZ4_LENGTH_PREFIXED (4).  Values are the
 * big-endian entries: ival gets INT / LONG values, dval every value as a double.  Returns 0, -1 on malformed bytes,
 * -2 on an unsupported codec. */
int or_raw_decode(const or_column* c, const uint8_t* b, int64_t len, int num_docs, int64_t* ival, double* dval) {
  if (len < 16) return -1;
  const int version = (int)be32(b), num_chunks = (int)be32(b + 4), per_chunk = (int)be32(b + 8);
  const int size = (int)be32(b + 12);
  int compression = 1, header_start = 16;
  if (version > 1) {
    if (len < 28) return -1;
    compression = (int)be32(b + 20);
    header_start = (int)be32(b + 24);
  }
  if (compression != 0 && compression != 3 && compression != 4) return -2;
  const int entry = version <= 2 ? 4 : 8;
  if (per_chunk <= 0 || num_chunks < 0 || (int64_t)num_chunks * per_chunk < num_docs || header_start < 0 ||
      (size != 4 && size != 8))
    return -1;
  const int64_t raw_start = (int64_t)header_start + (int64_t)num_chunks * entry;
  if (raw_start > len) return -1;
  uint8_t* chunk = compression ? malloc((size_t)per_chunk * size) : NULL;
  for (int k = 0; k < num_chunks && (int64_t)k * per_chunk < num_docs; k++) {
    const uint8_t* vals;
    const int d0 = k * per_chunk;
    const int nd = num_docs - d0 < per_chunk ? num_docs - d0 : per_chunk;
    if (compression == 0) {
      /* PASS_THROUGH: FixedByteChunkSVForwardIndexReader reads docId * size from rawDataStart */
      if (raw_start + (int64_t)(d0 + nd) * size > len) { free(chunk); return -1; }
      vals = b + raw_start + (int64_t)d0 * size;
    } else {
      const uint8_t* hp = b + header_start + (int64_t)k * entry;
      const int64_t pos = entry == 4 ? (int64_t)be32(hp) : (int64_t)be64(hp);
      const int64_t end = k == num_chunks - 1 ? len : (entry == 4 ? (int64_t)be32(hp + 4) : (int64_t)be64(hp + 8));
      if (pos < raw_start || end < pos || end > len) { free(chunk); return -1; }
      const uint8_t* src = b + pos;
      int64_t sn = end - pos;
      if (compression == 4) { /* LZ4DecompressorWithLength: little-endian decompressed length first */
        if (sn < 4) { free(chunk); return -1; }
        src += 4;
        sn -= 4;
      }
      const int64_t got = or_lz4_decompress(src, sn, chunk, (int64_t)per_chunk * size);
      if (got < (int64_t)nd * size) { free(chunk); return -1; }
      vals = chunk;
    }
    for (int i = 0; i < nd; i++) {
      const uint8_t* v = vals + (int64_t)i * size;
      const uint64_t hi = be32(v), lo = size == 8 ? be32(v + 4) : 0;
      double d;
      int64_t x = 0;
      switch (c->data_type) {
        case OR_INT: x = (int32_t)hi; d = (double)x; break;
        case OR_LONG: x = (int64_t)((hi << 32) | lo); d = (double)x; break;
        case OR_FLOAT: { uint32_t u = (uint32_t)hi; float f; memcpy(&f, &u, 4); d = (double)f; break; }
        default: { uint64_t u = (hi << 32) | lo; memcpy(&d, &u, 8); break; }
      }
      if (ival) ival[d0 + i] = x;
      if (dval) dval[d0 + i] = d;
    }
  }
  free(chunk);
  return 0;
}

/* Dictionary.readDoubleValues -> getDoubleValue per type (IntDictionary.java:62-64 etc.). */
double or_raw_get_double(const or_column* c, int doc) {
  const uint8_t* b = c->fwd;
  const int version = (int)be32(b), num_chunks = (int)be32(b + 4), size = (int)be32(b + 12);
  int data_header_start = 16;
  if (version > 1) data_header_start = (int)be32(b + 24);
  const int entry = version <= 2 ? 4 : 8; /* BaseChunkSVForwardIndexWriter.getHeaderEntryChunkOffsetSize */
  const uint8_t* v = b + data_header_start + (int64_t)num_chunks * entry + (int64_t)doc * size;
  const uint64_t hi = be32(v), lo = size == 8 ? be32(v + 4) : 0;
  switch (c->data_type) {
    case OR_INT: return (double)(int32_t)hi;
    case OR_LONG: return (double)(int64_t)((hi << 32) | lo);
    case OR_FLOAT: { uint32_t u = (uint32_t)hi; float f; memcpy(&f, &u, 4); return (double)f; }
    default: { uint64_t u = (hi << 32) | lo; double d; memcpy(&d, &u, 8); return d; }
  }
}

double or_dict_get_double(const or_column* c, int id) {
  switch (c->data_type) {
    case OR_INT: return (double)dict_int(c, id);
    case OR_LONG: return (double)dict_long(c, id);
    case OR_FLOAT: return (double)dict_float(c, id);
    case OR_DOUBLE: return dict_double(c, id);
    default: {
      const uint8_t* p; int n = dict_str(c, id, &p);
      char tmp[256]; if (n > 255) n = 255; memcpy(tmp, p, n); tmp[n] = 0;
      return strtod(tmp, NULL); /* StringDictionary.getDoubleValue: Double.parseDouble */
    }
  }
}

/* Java Integer.parseInt / Long.parseLong: optional sign, decimal digits only, range-checked. */
static int parse_java_long(const char* s, int64_t lo, int64_t hi, int64_t* out) {
  const char* p = s;
  int neg = 0;
  if (*p == '-' || *p == '+') { neg = (*p == '-'); p++; }
  if (!*p) return -1;
  __int128 v = 0;
  for (; *p; p++) {
    if (*p < '0' || *p > '9') return -1;
    v = v * 10 + (*p - '0');
    if (v > (__int128)hi + 1) return -1;
  }
  if (neg) v = -v;
  if (v < lo || v > hi) return -1;
  *out = (int64_t)v;
  return 0;
}
static int parse_java_double(const char* s, double* out) {
  char* end; errno = 0;
  double d = strtod(s, &end);
  while (*end == ' ' || *end == 'd' || *end == 'D' || *end == 'f' || *end == 'F') end++;
  if (end == s || *end) return -1;
  *out = d;
  return 0;
}

static int cmp_bytes(const uint8_t* a, int na, const uint8_t* b, int nb) {
  int n = na < nb ? na : nb;
  int c = memcmp(a, b, (size_t)n);
  if (c) return c;
  return na - nb;
}

/* BaseImmutableDictionary.binarySearch(int/long/float/double/String) (:97-230) behind
 * {Int,Long,Float,Double,String}Dictionary.insertionIndexOf(String) (IntDictionary.java:32-34 etc.).
 * *err = 1 when the literal does not parse for the column type (PredicateEvaluatorProvider.java:85-88 turns
 * that into BadQueryRequestException). */
int or_dict_insertion_index_of(const or_column* c, const char* lit, int* err) {
  int low = 0, high = c->cardinality - 1;
  *err = 0;
  switch (c->data_type) {
    case OR_INT: case OR_LONG: {
      int64_t v;
      if (parse_java_long(lit, c->data_type == OR_INT ? INT32_MIN : INT64_MIN,
                          c->data_type == OR_INT ? INT32_MAX : INT64_MAX, &v)) { *err = 1; return 0; }
      while (low <= high) {
        int mid = (int)(((unsigned)low + (unsigned)high) >> 1);
        int64_t m = c->data_type == OR_INT ? dict_int(c, mid) : dict_long(c, mid);
        if (m < v) low = mid + 1; else if (m > v) high = mid - 1; else return mid;
      }
      return -(low + 1);
    }
    case OR_FLOAT: case OR_DOUBLE: {
      double v;
      if (parse_java_double(lit, &v)) { *err = 1; return 0; }
      if (c->data_type == OR_FLOAT) v = (double)(float)v; /* Float.parseFloat */
      while (low <= high) {
        int mid = (int)(((unsigned)low + (unsigned)high) >> 1);
        double m = c->data_type == OR_FLOAT ? (double)dict_float(c, mid) : dict_double(c, mid);
        if (m < v) low = mid + 1; else if (m > v) high = mid - 1; else return mid;
      }
      return -(low + 1);
    }
    default: {
      const uint8_t* lv = (const uint8_t*)lit;
      int ln = (int)strlen(lit);
      if (c->padding_byte == 0) {
        while (low <= high) {
          int mid = (int)(((unsigned)low + (unsigned)high) >> 1);
          const uint8_t* p; int n = dict_str(c, mid, &p);
          int r = cmp_bytes(p, n, lv, ln);
          if (r < 0) low = mid + 1; else if (r > 0) high = mid - 1; else return mid;
        }
      } else { /* legacy non-zero padding: compare padded strings (BaseImmutableDictionary.java:215-228) */
        uint8_t padded[4096];
        int pn = ln;
        if (ln < c->entry_width && c->entry_width <= (int)sizeof padded) {
          memcpy(padded, lv, ln);
          memset(padded + ln, c->padding_byte, c->entry_width - ln);
          pn = c->entry_width;
          lv = padded;
        }
        while (low <= high) {
          int mid = (int)(((unsigned)low + (unsigned)high) >> 1);
          const uint8_t* p = c->dict + (int64_t)mid * c->entry_width;
          int r = cmp_bytes(p, c->entry_width, lv, pn);
          if (r < 0) low = mid + 1; else if (r > 0) high = mid - 1; else return mid;
        }
      }
      return -(low + 1);
    }
  }
}

/* ---- dictionary creation (SegmentDictionaryCreator: sorted distinct values; dictId = rank) */

/* Java Double.compare total order (used by Arrays.sort for the dictionary). */
static int java_double_compare(double a, double b) {
  if (a < b) return -1;
  if (a > b) return 1;
  uint64_t ua, ub;
  if (a != a) a = NAN; if (b != b) b = NAN; /* canonical NaN */
  memcpy(&ua, &a, 8); memcpy(&ub, &b, 8);
  int64_t sa = (int64_t)ua, sb = (int64_t)ub;
  return sa == sb ? 0 : (sa < sb ? -1 : 1);
}

typedef struct { int64_t iv; double dv; int64_t row; } sort_rec;
static int cmp_i64_rec(const void* a, const void* b) {
  const sort_rec* x = a; const sort_rec* y = b;
  if (x->iv != y->iv) return x->iv < y->iv ? -1 : 1;
  return x->row < y->row ? -1 : (x->row > y->row);
}
static int cmp_f64_rec(const void* a, const void* b) {
  const sort_rec* x = a; const sort_rec* y = b;
  int c = java_double_compare(x->dv, y->dv);
  if (c) return c;
  return x->row < y->row ? -1 : (x->row > y->row);
}

static void pack_ids(const int32_t* ids, int64_t n, int bits, uint8_t* fwd) {
  for (int64_t i = 0; i < n; i++) or_bitset_write_int(fwd, i, bits, ids[i]);
}

int or_build_column_i64(int data_type, const int64_t* values, int64_t n, uint8_t* dict_out, uint8_t* fwd_out,
                        int* bits_out, int* width_out) {
  sort_rec* r = malloc(sizeof(sort_rec) * (size_t)(n ? n : 1));
  int32_t* ids = malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  for (int64_t i = 0; i < n; i++) { r[i].iv = values[i]; r[i].row = i; }
  qsort(r, (size_t)n, sizeof(sort_rec), cmp_i64_rec);
  int width = data_type == OR_INT ? 4 : 8;
  int card = 0;
  for (int64_t i = 0; i < n; i++) {
    if (i == 0 || r[i].iv != r[i - 1].iv) {
      if (width == 4) put_be32(dict_out + (int64_t)card * 4, (uint32_t)(int32_t)r[i].iv);
      else put_be64(dict_out + (int64_t)card * 8, (uint64_t)r[i].iv);
      card++;
    }
    ids[r[i].row] = card - 1;
  }
  int bits = or_num_bits_per_value(card - 1);
  pack_ids(ids, n, bits, fwd_out);
  *bits_out = bits; *width_out = width;
  free(r); free(ids);
  return card;
}

int or_build_column_f64(int data_type, const double* values, int64_t n, uint8_t* dict_out, uint8_t* fwd_out,
                        int* bits_out, int* width_out) {
  sort_rec* r = malloc(sizeof(sort_rec) * (size_t)(n ? n : 1));
  int32_t* ids = malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  for (int64_t i = 0; i < n; i++) {
    r[i].dv = data_type == OR_FLOAT ? (double)(float)values[i] : values[i];
    r[i].row = i;
  }
  qsort(r, (size_t)n, sizeof(sort_rec), cmp_f64_rec);
  int width = data_type == OR_FLOAT ? 4 : 8;
  int card = 0;
  for (int64_t i = 0; i < n; i++) {
    if (i == 0 || java_double_compare(r[i].dv, r[i - 1].dv) != 0) {
      if (width == 4) { float f = (float)r[i].dv; uint32_t u; memcpy(&u, &f, 4); put_be32(dict_out + (int64_t)card * 4, u); }
      else { uint64_t u; memcpy(&u, &r[i].dv, 8); put_be64(dict_out + (int64_t)card * 8, u); }
      card++;
    }
    ids[r[i].row] = card - 1;
  }
  int bits = or_num_bits_per_value(card - 1);
  pack_ids(ids, n, bits, fwd_out);
  *bits_out = bits; *width_out = width;
  free(r); free(ids);
  return card;
}

typedef struct { const uint8_t* p; int n; int64_t row; } str_rec;
static int cmp_str_rec(const void* a, const void* b) {
  const str_rec* x = a; const str_rec* y = b;
  int c = cmp_bytes(x->p, x->n, y->p, y->n);
  if (c) return c;
  return x->row < y->row ? -1 : (x->row > y->row);
}

int or_build_column_str(const uint8_t* blob, const int64_t* offsets, int64_t n, uint8_t* dict_out,
                        uint8_t* fwd_out, int* bits_out, int* width_out) {
  str_rec* r = malloc(sizeof(str_rec) * (size_t)(n ? n : 1));
  int32_t* ids = malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
  int width = 0;
  for (int64_t i = 0; i < n; i++) {
    r[i].p = blob + offsets[i]; r[i].n = (int)(offsets[i + 1] - offsets[i]); r[i].row = i;
    if (r[i].n > width) width = r[i].n;
  }
  if (width == 0) width = 1;
  qsort(r, (size_t)n, sizeof(str_rec), cmp_str_rec);
  int card = 0;
  for (int64_t i = 0; i < n; i++) {
    if (i == 0 || cmp_bytes(r[i].p, r[i].n, r[i - 1].p, r[i - 1].n) != 0) {
      uint8_t* d = dict_out + (int64_t)card * width;
      memset(d, 0, (size_t)width);
      memcpy(d, r[i].p, (size_t)r[i].n);
      card++;
    }
    ids[r[i].row] = card - 1;
  }
  int bits = or_num_bits_per_value(card - 1);
  pack_ids(ids, n, bits, fwd_out);
  *bits_out = bits; *width_out = width;
  free(r); free(ids);
  return card;
}

/* ======================================================================================= predicates */

/* One dictionary-based PredicateEvaluator for one segment (core/operator/filter/predicate/). */
typedef struct {
  int always_true, always_false;
  int kind;         /* 0 = range [start,end), 1 = dictId set, 2 = single id, 3 = not single id, 4 = not in set,
                       5 = raw-value evaluator (no-dictionary column) */
  int start, end;
  int id;
  uint8_t* set;     /* card flags for kinds 1 / 4 */
  int num_matching;
  /* kind 5 (BaseRawValueBasedPredicateEvaluator subclasses): the column's values per doc, decoded from its chunks */
  int ptype, dtype;                 /* predicate type, column data type */
  int64_t* rival;                   /* INT / LONG values */
  double* rdval;                    /* FLOAT / DOUBLE values (widened) */
  int64_t ilo, ihi;                 /* RANGE / EQ / NOT_EQ bounds (integers) */
  double dlo, dhi;                  /* RANGE / EQ / NOT_EQ bounds (FLOAT: float values) */
  int lo_inc, hi_inc;
  int64_t* vset;                    /* IN / NOT_IN: Integer/Long values, or doubleToLongBits / floatToIntBits */
  int nvset;
} pred_eval;

static void pred_eval_free(pred_eval* e) {
  free(e->set); free(e->rival); free(e->rdval); free(e->vset);
  e->set = NULL; e->rival = NULL; e->rdval = NULL; e->vset = NULL;
}

/* Double.doubleToLongBits / Float.floatToIntBits (canonical NaN): the equality of fastutil's Double / Float
 * OpenHashSets (fastutil 8.2.3, absent here) behind InPredicateEvaluatorFactory's raw IN evaluators. */
static int64_t java_double_bits(double d) {
  if (d != d) return 0x7ff8000000000000LL;
  int64_t b; memcpy(&b, &d, 8); return b;
}
static int64_t java_float_bits(float f) {
  if (f != f) return 0x7fc00000;
  int32_t b; memcpy(&b, &f, 4); return b;
}

/* Literal conversion of the raw evaluators: Integer.parseInt / Long.parseLong / Float.parseFloat /
 * Double.parseDouble (RangePredicateEvaluatorFactory.java:65-102, EqualsPredicateEvaluatorFactory.java:60-70,
 * InPredicateEvaluatorFactory.java:69-126). */
static int parse_java_long(const char* s, int64_t lo, int64_t hi, int64_t* out);
static int raw_literal(int dtype, const char* s, int64_t* iv, double* dv) {
  if (dtype == OR_INT) return parse_java_long(s, INT32_MIN, INT32_MAX, iv);
  if (dtype == OR_LONG) return parse_java_long(s, INT64_MIN, INT64_MAX, iv);
  char* end = NULL;
  double d = strtod(s, &end);
  if (end == s) return -1;
  while (*end == 'd' || *end == 'D' || *end == 'f' || *end == 'F') end++;
  if (*end) return -1;
  *dv = dtype == OR_FLOAT ? (double)(float)d : d;
  return 0;
}

static int build_raw_eval(const or_segment* seg, const or_column* c, const or_predicate* p, pred_eval* e) {
  e->kind = 5;
  e->ptype = p->type;
  e->dtype = c->data_type;
  const int fp = c->data_type == OR_FLOAT || c->data_type == OR_DOUBLE;
  const int nd = seg->num_docs > 0 ? seg->num_docs : 1;
  if (fp) e->rdval = malloc(sizeof(double) * (size_t)nd);
  else e->rival = malloc(sizeof(int64_t) * (size_t)nd);
  if (c->data_type == OR_STRING || or_raw_decode(c, c->fwd, c->fwd_len, seg->num_docs, e->rival, e->rdval))
    return -3;
  switch (p->type) {
    case OR_PRED_EQ: case OR_PRED_NOT_EQ:
      if (raw_literal(c->data_type, p->values[0], &e->ilo, &e->dlo)) return -2;
      return 0;
    case OR_PRED_IN: case OR_PRED_NOT_IN:
      e->vset = malloc(sizeof(int64_t) * (size_t)(p->num_values ? p->num_values : 1));
      for (int i = 0; i < p->num_values; i++) {
        int64_t iv = 0; double dv = 0;
        if (raw_literal(c->data_type, p->values[i], &iv, &dv)) return -2;
        e->vset[e->nvset++] = !fp ? iv : c->data_type == OR_FLOAT ? java_float_bits((float)dv) : java_double_bits(dv);
      }
      return 0;
    default: { /* RANGE: unbounded = inclusive MIN / MAX (-inf / +inf) of the type */
      const char* lo = p->values[0];
      const char* hi = p->values[1];
      const int lu = strcmp(lo, "*") == 0, hu = strcmp(hi, "*") == 0;
      e->lo_inc = lu || p->lower_inclusive;
      e->hi_inc = hu || p->upper_inclusive;
      if (lu) { e->ilo = c->data_type == OR_INT ? INT32_MIN : INT64_MIN; e->dlo = -INFINITY; }
      else if (raw_literal(c->data_type, lo, &e->ilo, &e->dlo)) return -2;
      if (hu) { e->ihi = c->data_type == OR_INT ? INT32_MAX : INT64_MAX; e->dhi = INFINITY; }
      else if (raw_literal(c->data_type, hi, &e->ihi, &e->dhi)) return -2;
      return 0;
    }
  }
}

/* applySV of the raw evaluators (RangePredicateEvaluatorFactory.java:268-448 Int/Long/Float/Double...Range, Equals
 * :113-187 `==`, NotEquals `!=`, In / NotIn: set contains). */
static int raw_apply(const pred_eval* e, int doc) {
  const int fp = e->rdval != NULL;
  switch (e->ptype) {
    case OR_PRED_EQ: return fp ? e->rdval[doc] == e->dlo : e->rival[doc] == e->ilo;
    case OR_PRED_NOT_EQ: return fp ? e->rdval[doc] != e->dlo : e->rival[doc] != e->ilo;
    case OR_PRED_IN: case OR_PRED_NOT_IN: {
      const int64_t k = !fp ? e->rival[doc] : e->dtype == OR_FLOAT ? java_float_bits((float)e->rdval[doc])
                                                                   : java_double_bits(e->rdval[doc]);
      int hit = 0;
      for (int i = 0; i < e->nvset && !hit; i++) hit = e->vset[i] == k;
      return e->ptype == OR_PRED_IN ? hit : !hit;
    }
    default:
      if (fp) {
        const double v = e->rdval[doc];
        return (e->lo_inc ? e->dlo <= v : e->dlo < v) && (e->hi_inc ? e->dhi >= v : e->dhi > v);
      } else {
        const int64_t v = e->rival[doc];
        return (e->lo_inc ? e->ilo <= v : e->ilo < v) && (e->hi_inc ? e->ihi >= v : e->ihi > v);
      }
  }
}

static int dict_index_of(const or_column* c, const char* lit, int* err) {
  int idx = or_dict_insertion_index_of(c, lit, err);
  return idx >= 0 ? idx : -1; /* BaseImmutableDictionary.indexOf :81-84 */
}

static int build_pred_eval(const or_segment* seg, const or_predicate* p, pred_eval* e, char* msg, int ml) {
  memset(e, 0, sizeof *e);
  if (p->column < 0 || p->column >= seg->num_columns) { snprintf(msg, ml, "bad predicate column"); return -1; }
  const or_column* c = &seg->columns[p->column];
  int err = 0;
  if (c->raw) { /* no dictionary: a raw-value evaluator, never always-true / always-false (FilterPlanNode) */
    const int st = build_raw_eval(seg, c, p, e);
    if (st == -2) goto bad;
    if (st) { snprintf(msg, ml, "raw forward index of column %d is unreadable", p->column); pred_eval_free(e); return -1; }
    return 0;
  }
  switch (p->type) {
    case OR_PRED_EQ: { /* EqualsPredicateEvaluatorFactory.java:86-99 */
      int id = dict_index_of(c, p->values[0], &err);
      if (err) goto bad;
      e->kind = 2; e->id = id;
      if (id >= 0) { if (c->cardinality == 1) e->always_true = 1; }
      else e->always_false = 1;
      return 0;
    }
    case OR_PRED_NOT_EQ: { /* NotEqualsPredicateEvaluatorFactory.java:88-102 */
      int id = dict_index_of(c, p->values[0], &err);
      if (err) goto bad;
      e->kind = 3; e->id = id;
      if (id >= 0) { if (c->cardinality == 1) e->always_false = 1; }
      else e->always_true = 1;
      return 0;
    }
    case OR_PRED_IN: case OR_PRED_NOT_IN: { /* InPredicateEvaluatorFactory.java:138-154, NotIn...:140-160 */
      e->kind = p->type == OR_PRED_IN ? 1 : 4;
      e->set = calloc((size_t)(c->cardinality ? c->cardinality : 1), 1);
      int n = 0;
      for (int i = 0; i < p->num_values; i++) {
        int id = dict_index_of(c, p->values[i], &err);
        if (err) goto bad;
        if (id >= 0 && !e->set[id]) { e->set[id] = 1; n++; }
      }
      e->num_matching = n;
      if (p->type == OR_PRED_IN) {
        if (n == 0) e->always_false = 1; else if (n == c->cardinality) e->always_true = 1;
      } else {
        if (n == 0) e->always_true = 1; else if (n == c->cardinality) e->always_false = 1;
      }
      return 0;
    }
    case OR_PRED_RANGE: { /* SortedDictionaryBasedRangePredicateEvaluator (RangePredicateEvaluatorFactory.java:115-159) */
      const char* lo = p->values[0];
      const char* hi = p->values[1];
      int start, end;
      if (strcmp(lo, "*") == 0) start = 0;
      else {
        int ins = or_dict_insertion_index_of(c, lo, &err);
        if (err) goto bad;
        if (ins < 0) start = -(ins + 1); else start = p->lower_inclusive ? ins : ins + 1;
      }
      if (strcmp(hi, "*") == 0) end = c->cardinality;
      else {
        int ins = or_dict_insertion_index_of(c, hi, &err);
        if (err) goto bad;
        if (ins < 0) end = -(ins + 1); else end = p->upper_inclusive ? ins + 1 : ins;
      }
      e->kind = 0; e->start = start; e->end = end;
      int nm = end - start;
      if (nm <= 0) e->always_false = 1; else if (c->cardinality == nm) e->always_true = 1;
      return 0;
    }
    default:
      snprintf(msg, ml, "unsupported predicate type %d", p->type);
      return -1;
  }
bad:
  snprintf(msg, ml, "BadQueryRequestException: cannot convert literal for column %d", p->column);
  pred_eval_free(e);
  return -2;
}

static inline int pred_apply(const pred_eval* e, int id) {
  switch (e->kind) {
    case 0: return e->start <= id && e->end > id;
    case 1: return e->set[id];
    case 2: return e->id == id;
    case 3: return e->id != id;
    default: return !e->set[id];
  }
}

/* ======================================================================================= filter operators */

/* Operator tree after FilterPlanNode.constructPhysicalOperator (core/plan/FilterPlanNode.java:146-247) and
 * FilterOperatorUtils (:42-135): EMPTY, MATCH_ALL, leaf operators (scan / sorted-index / bitmap-index), AND, OR,
 * NOT.  Leaf choice = FilterOperatorUtils.getLeafFilterOperator (:42-82): RANGE on a sorted column ->
 * SortedIndexBasedFilterOperator, on a column with a range index -> RangeIndexBasedFilterOperator, else scan;
 * EQ / NOT_EQ / IN / NOT_IN on a sorted column
 * -> sorted, else on a column with an inverted index -> BitmapBasedFilterOperator, else scan.  NOT is not part of
 * the 0.10 FilterContext; it is modelled as a scan-based iterator over its child (match = child does not match). */
enum { FN_EMPTY = 0, FN_ALL = 1, FN_SCAN = 2, FN_AND = 3, FN_OR = 4, FN_NOT = 5, FN_SORTED = 6, FN_BITMAP = 7,
       FN_RANGEIDX = 8 };
typedef struct fnode {
  int type;
  int pred;              /* leaves: predicate index */
  int nchild;
  struct fnode** child;
} fnode;

static fnode* fn_new(int type) { fnode* n = calloc(1, sizeof(fnode)); n->type = type; return n; }
static void fn_free(fnode* n) {
  if (!n) return;
  for (int i = 0; i < n->nchild; i++) fn_free(n->child[i]);
  free(n->child); free(n);
}

/* ---- range index (RangeIndexReaderImpl / BitSlicedRangeIndexReader, seglocal/segment/index/readers/): the reader a
 * column's `.bitmap.range` bytes give (DefaultIndexReaderProvider.newRangeIndexReader :128-139: version 1 or 2, any
 * other version is skipped -- no range index). */
static int32_t be_i32(const uint8_t* b) {
  return (int32_t)(((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3]);
}
static int64_t be_i64(const uint8_t* b) { return (int64_t)(((uint64_t)(uint32_t)be_i32(b) << 32) | (uint32_t)be_i32(b + 4)); }
static int range_index_version(const or_column* c) {
  if (!c->range_index || c->range_index_len < 4 || c->raw) return 0;
  int v = be_i32(c->range_index);
  return v == 1 || v == 2 ? v : 0;
}
/* ImmutableRoaringBitmap.getCardinality of a portable serialisation: the sum of the containers' cardinalities, read
 * from the descriptive header (cookie 12346: u32 size; 12347 | (size - 1) << 16: run-container bitmap) -- each
 * container's (u16 key, u16 cardinality - 1). */
static int64_t roaring_card(const uint8_t* b, int64_t n) {
  if (n < 4) return -1;
  uint32_t cookie = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
  int64_t size, pos;
  if ((cookie & 0xFFFF) == 12347) { size = (cookie >> 16) + 1; pos = 4 + (size + 7) / 8; }
  else if (cookie == 12346) {
    if (n < 8) return -1;
    size = (int64_t)((uint32_t)b[4] | ((uint32_t)b[5] << 8) | ((uint32_t)b[6] << 16) | ((uint32_t)b[7] << 24));
    pos = 8;
  } else return -1;
  if (pos + size * 4 > n) return -1;
  int64_t card = 0;
  for (int64_t i = 0; i < size; i++) card += (int64_t)((uint32_t)b[pos + 4 * i + 2] | ((uint32_t)b[pos + 4 * i + 3] << 8)) + 1;
  return card;
}
/* RangeIndexBasedFilterOperator.getNextBlock (:57-129) entries for the dictIds [start, end): the size of
 * getPartiallyMatchingDocIds(startDictId, endDictId - 1), which its ScanBasedFilterOperator's applyAnd scans; 0 for a
 * bit-sliced (exact) index.  Version 1 layout (RangeIndexCreator.seal, big-endian): version, value type name, range
 * count R, R range starts + the last range's end (INT: dictIds), R + 1 bitmap offsets, the bitmaps. */
static int64_t range_partial_entries(const or_column* c, int start, int end) {
  if (range_index_version(c) != 1) return 0;
  const uint8_t* b = c->range_index;
  int64_t off = 4;
  int32_t tlen = be_i32(b + off);
  off += 4 + tlen;
  int32_t R = be_i32(b + off);
  off += 4;
  const uint8_t* starts = b + off;          /* _rangeStartArray, then _lastRangeEnd */
  const uint8_t* offs = b + off + 4 * ((int64_t)R + 1); /* _bitmapIndexOffset */
  int first = -2, last = -2;
  int vals[2] = {start, end - 1};
  for (int k = 0; k < 2; k++) { /* findRangeId (RangeIndexReaderImpl.java:198-205) */
    int id = -2;
    for (int i = 0; i < R; i++)
      if (vals[k] < be_i32(starts + 4 * i)) { id = i - 1; break; }
    if (id == -2) id = vals[k] <= be_i32(starts + 4 * R) ? R - 1 : R;
    if (k == 0) first = id; else last = id;
  }
  int out_first = first < 0 || first >= R, out_last = last < 0 || last >= R;
#define RANGE_DOCS(i) roaring_card(b + be_i64(offs + 8 * (int64_t)(i)), be_i64(offs + 8 * ((int64_t)(i) + 1)) - be_i64(offs + 8 * (int64_t)(i)))
  /* getPartialMatchesInRange (:252-260): the first and last ranges (disjoint docs; OR of a range with itself is it) */
  if (out_first) return out_last ? 0 : RANGE_DOCS(last);
  if (out_last) return RANGE_DOCS(first);
  return first == last ? RANGE_DOCS(first) : RANGE_DOCS(first) + RANGE_DOCS(last);
#undef RANGE_DOCS
}

/* reorderAndFilterChildOperators priorities (FilterOperatorUtils.java:143-178). */
static int and_priority(const fnode* n) {
  switch (n->type) {
    case FN_SORTED: return 0;
    case FN_BITMAP: return 1;
    case FN_RANGEIDX: return 2; /* RangeIndexBasedFilterOperator */
    case FN_AND: return 3;
    case FN_OR: return 4;
    default: return 5; /* scan (single-value columns), NOT */
  }
}

/* Build from the postfix program, simplifying always-true/false leaves exactly as FilterPlanNode does. */
static fnode* build_filter_tree(const or_segment* seg, const or_query* q, const pred_eval* evals, char* msg, int ml) {
  if (q->num_filter_ops == 0) return fn_new(FN_ALL);
  fnode** stack = calloc((size_t)q->num_filter_ops + 1, sizeof(fnode*));
  int sp = 0;
  for (int i = 0; i < q->num_filter_ops; i++) {
    const or_filter_op* op = &q->filter[i];
    if (op->op == OR_OP_PRED) {
      const pred_eval* e = &evals[op->arg];
      const or_predicate* pr = &q->predicates[op->arg];
      const or_column* c = &seg->columns[pr->column];
      fnode* n;
      if (e->always_false) n = fn_new(FN_EMPTY);          /* FilterOperatorUtils.java:44-46 */
      else if (e->always_true) n = fn_new(FN_ALL);        /* :47-48 */
      else {
        int type = FN_SCAN;
        if (c->is_sorted) type = FN_SORTED;                                    /* :57-58, :73-74 */
        else if (pr->type == OR_PRED_RANGE && range_index_version(c)) type = FN_RANGEIDX; /* :60-62 */
        else if (pr->type != OR_PRED_RANGE && c->has_inverted) type = FN_BITMAP; /* :76-77 */
        n = fn_new(type);
        n->pred = op->arg;
      }
      stack[sp++] = n;
    } else if (op->op == OR_OP_NOT) {
      if (sp < 1) goto bad;
      fnode* c = stack[--sp];
      fnode* n;
      if (c->type == FN_EMPTY) { fn_free(c); n = fn_new(FN_ALL); }
      else if (c->type == FN_ALL) { fn_free(c); n = fn_new(FN_EMPTY); }
      else { n = fn_new(FN_NOT); n->nchild = 1; n->child = malloc(sizeof(fnode*)); n->child[0] = c; }
      stack[sp++] = n;
    } else {
      int k = op->arg;
      if (k < 1 || sp < k) goto bad;
      fnode** kids = stack + sp - k;
      int is_and = op->op == OR_OP_AND;
      fnode* result = NULL;
      fnode** keep = malloc(sizeof(fnode*) * (size_t)k);
      int nk = 0;
      for (int j = 0; j < k; j++) {
        fnode* c = kids[j];
        if (result) { fn_free(c); continue; }
        if (is_and) {
          if (c->type == FN_EMPTY) { result = c; continue; }      /* getAndFilterOperator :90-95 */
          if (c->type == FN_ALL) { fn_free(c); continue; }
        } else {
          if (c->type == FN_ALL) { result = c; continue; }        /* getOrFilterOperator :115-120 */
          if (c->type == FN_EMPTY) { fn_free(c); continue; }
        }
        keep[nk++] = c;
      }
      if (result) { for (int j = 0; j < nk; j++) fn_free(keep[j]); free(keep); }
      else if (nk == 0) { free(keep); result = fn_new(is_and ? FN_ALL : FN_EMPTY); }
      else if (nk == 1) { result = keep[0]; free(keep); }
      else {
        result = fn_new(is_and ? FN_AND : FN_OR);
        if (is_and) { /* stable sort by priority */
          fnode** sorted = malloc(sizeof(fnode*) * (size_t)nk);
          int ns = 0;
          for (int pr = 0; pr <= 5; pr++)
            for (int j = 0; j < nk; j++)
              if (and_priority(keep[j]) == pr) sorted[ns++] = keep[j];
          free(keep);
          keep = sorted;
        }
        result->nchild = nk; result->child = keep;
      }
      sp -= k;
      stack[sp++] = result;
    }
  }
  if (sp != 1) goto bad;
  fnode* root = stack[0];
  free(stack);
  return root;
bad:
  for (int i = 0; i < sp; i++) fn_free(stack[i]);
  free(stack);
  snprintf(msg, ml, "malformed filter program");
  return NULL;
}

static int node_match(const fnode* n, const or_segment* seg, const pred_eval* evals, const or_query* q, int doc) {
  switch (n->type) {
    case FN_EMPTY: return 0;
    case FN_ALL: return 1;
    case FN_SCAN: case FN_SORTED: case FN_BITMAP: case FN_RANGEIDX: {
      const or_column* c = &seg->columns[q->predicates[n->pred].column];
      if (evals[n->pred].kind == 5) return raw_apply(&evals[n->pred], doc);
      return pred_apply(&evals[n->pred], fixedbit_read(c->fwd, doc, c->bits));
    }
    case FN_AND: for (int i = 0; i < n->nchild; i++) if (!node_match(n->child[i], seg, evals, q, doc)) return 0; return 1;
    case FN_OR: for (int i = 0; i < n->nchild; i++) if (node_match(n->child[i], seg, evals, q, doc)) return 1; return 0;
    default: return !node_match(n->child[0], seg, evals, q, doc);
  }
}

/* ---- DocId iterators (core/operator/dociditerators/, docidsets/):
 *   IT_SCAN  SVScanDocIdIterator (:56-94): next / advance / applyAnd, counting _numEntriesScanned (NOT: same, over
 *            the negated child);
 *   IT_IDX   SortedDocIdIterator / BitmapDocIdIterator / RangelessBitmapDocIdIterator: a docId set, no entries
 *            scanned (`sorted` tells SortedDocIdIterator apart for AndDocIdSet's classification);
 *   IT_AND   AndDocIdIterator leap-frog (:40-67);  IT_OR  OrDocIdIterator (:25-130).
 * Sorted-index and bitmap-index doc sets are built from the forward index (the docs a sorted / inverted index
 * returns are exactly the predicate's matches) without counting entries. */
enum { IT_EMPTY = 0, IT_ALL = 1, IT_SCAN = 2, IT_IDX = 3, IT_AND = 4, IT_OR = 5 };
typedef struct iter {
  int type;
  int next_doc;            /* scan / idx / and / all */
  int64_t scanned;         /* scan: _numEntriesScanned */
  int64_t partial;         /* idx of a RangeIndexBasedFilterOperator: its partial-match scan's entries */
  const fnode* node;       /* scan: the leaf (or NOT) node */
  uint64_t* bits;          /* idx: docId set */
  int sorted;              /* idx: a SortedDocIdIterator */
  int num_docs;
  int n;                   /* children */
  struct iter** kids;
  int* next_ids;           /* or: _nextDocIds */
  int num_not_exhausted;   /* or */
  int prev_doc;            /* or */
  const or_segment* seg;
  const pred_eval* evals;
  const or_query* q;
} iter;

static int it_next(iter* it);
static int it_advance(iter* it, int target);

static inline int scan_match(iter* it, int doc) {
  if (it->node->type == FN_NOT) return !node_match(it->node->child[0], it->seg, it->evals, it->q, doc);
  return node_match(it->node, it->seg, it->evals, it->q, doc);
}

static int idx_next(iter* it) {
  int nw = (it->num_docs + 63) / 64;
  if (it->next_doc >= it->num_docs) return EOF_DOC;
  int w = it->next_doc >> 6;
  uint64_t m = it->bits[w] & (~0ull << (it->next_doc & 63));
  while (!m) {
    if (++w >= nw) return EOF_DOC;
    m = it->bits[w];
  }
  int d = w * 64 + __builtin_ctzll(m);
  if (d >= it->num_docs) return EOF_DOC;
  it->next_doc = d + 1;
  return d;
}

static int it_next(iter* it) {
  switch (it->type) {
    case IT_EMPTY: return EOF_DOC;
    case IT_ALL: return it->next_doc < it->num_docs ? it->next_doc++ : EOF_DOC;
    case IT_IDX: return idx_next(it);
    case IT_SCAN: /* SVScanDocIdIterator.next :56-66 */
      while (it->next_doc < it->num_docs) {
        int d = it->next_doc++;
        it->scanned++;
        if (scan_match(it, d)) return d;
      }
      return EOF_DOC;
    case IT_AND: { /* AndDocIdIterator.next :40-67 */
      int max_doc = it->next_doc, max_idx = -1, index = 0;
      while (index < it->n) {
        if (index == max_idx) { index++; continue; }
        int d = it_advance(it->kids[index], max_doc);
        if (d != EOF_DOC) {
          if (d == max_doc) index++;
          else { max_doc = d; max_idx = index; index = 0; }
        } else return EOF_DOC;
      }
      it->next_doc = max_doc;
      return it->next_doc++;
    }
    default: { /* IT_OR: OrDocIdIterator.next */
      int next = INT32_MAX;
      int exhausted = 0;
      for (int i = 0; i < it->num_not_exhausted; i++) {
        int d = it->next_ids[i];
        if (d == it->prev_doc) {
          d = it_next(it->kids[i]);
          it->next_ids[i] = d;
          if (d == EOF_DOC) { exhausted = 1; continue; }
        }
        if (d < next) next = d;
      }
      if (exhausted) { /* removeExhaustedIterators */
        int w = 0;
        for (int i = 0; i < it->num_not_exhausted; i++)
          if (it->next_ids[i] != EOF_DOC) { it->kids[w] = it->kids[i]; it->next_ids[w] = it->next_ids[i]; w++; }
        it->num_not_exhausted = w;
      }
      if (next != INT32_MAX) { it->prev_doc = next; return next; }
      return EOF_DOC;
    }
  }
}

static int it_advance(iter* it, int target) {
  switch (it->type) {
    case IT_EMPTY: return EOF_DOC;
    case IT_ALL: case IT_IDX: case IT_SCAN: case IT_AND: /* SVScanDocIdIterator.advance :69-72, ... */
      it->next_doc = target;
      return it_next(it);
    default: { /* OrDocIdIterator.advance */
      int next = INT32_MAX;
      int exhausted = 0;
      for (int i = 0; i < it->num_not_exhausted; i++) {
        int d = it->next_ids[i];
        if (d < target) {
          d = it_advance(it->kids[i], target);
          it->next_ids[i] = d;
          if (d == EOF_DOC) { exhausted = 1; continue; }
        }
        if (d < next) next = d;
      }
      if (exhausted) {
        int w = 0;
        for (int i = 0; i < it->num_not_exhausted; i++)
          if (it->next_ids[i] != EOF_DOC) { it->kids[w] = it->kids[i]; it->next_ids[w] = it->next_ids[i]; w++; }
        it->num_not_exhausted = w;
      }
      if (next != INT32_MAX) { it->prev_doc = next; return next; }
      return EOF_DOC;
    }
  }
}

typedef struct { iter** all; int n, cap; } iter_pool;
static iter* it_new(int type, const or_segment* seg, const pred_eval* evals, const or_query* q, iter_pool* pool) {
  iter* it = calloc(1, sizeof(iter));
  if (pool->n == pool->cap) { pool->cap = pool->cap ? pool->cap * 2 : 16; pool->all = realloc(pool->all, sizeof(iter*) * pool->cap); }
  pool->all[pool->n++] = it;
  it->type = type;
  it->num_docs = seg->num_docs;
  it->seg = seg;
  it->evals = evals;
  it->q = q;
  return it;
}
static iter* it_new_idx(uint64_t* bits, int sorted, const or_segment* seg, const pred_eval* evals, const or_query* q,
                        iter_pool* pool) {
  iter* it = it_new(IT_IDX, seg, evals, q, pool);
  it->bits = bits;
  it->sorted = sorted;
  return it;
}
static iter* it_new_multi(int type, iter** kids, int n, const or_segment* seg, const pred_eval* evals,
                          const or_query* q, iter_pool* pool) {
  iter* it = it_new(type, seg, evals, q, pool);
  it->n = n;
  it->kids = kids;
  if (type == IT_OR) {
    it->next_ids = malloc(sizeof(int) * (size_t)(n ? n : 1));
    for (int i = 0; i < n; i++) it->next_ids[i] = -1;
    it->num_not_exhausted = n;
    it->prev_doc = -1;
  }
  return it;
}

/* FilterBlockDocIdSet.iterator() of node n: AndDocIdSet.iterator (:60-146) / OrDocIdSet.iterator (:57-110) build
 * their children's iterators first, then merge index-based ones (sorted ranges, bitmaps) into one bitmap; an AND
 * with index-based and scan-based children runs the scans' applyAnd over it (numEntriesScanned += its size). */
static iter* it_build(const fnode* n, const or_segment* seg, const pred_eval* evals, const or_query* q,
                      iter_pool* pool) {
  const int nd = seg->num_docs, nw = (nd + 63) / 64;
  switch (n->type) {
    case FN_EMPTY: return it_new(IT_EMPTY, seg, evals, q, pool);
    case FN_ALL: return it_new(IT_ALL, seg, evals, q, pool);
    case FN_SCAN: case FN_NOT: {
      iter* it = it_new(IT_SCAN, seg, evals, q, pool);
      it->node = n;
      return it;
    }
    case FN_SORTED: case FN_BITMAP: case FN_RANGEIDX: {
      uint64_t* bits = calloc((size_t)(nw ? nw : 1), 8);
      for (int d = 0; d < nd; d++) if (node_match(n, seg, evals, q, d)) bits[d >> 6] |= 1ull << (d & 63);
      iter* it = it_new_idx(bits, n->type == FN_SORTED, seg, evals, q, pool);
      if (n->type == FN_RANGEIDX) /* matches | scan(partial matches): the predicate's docs, BitmapDocIdSet */
        it->partial = range_partial_entries(&seg->columns[q->predicates[n->pred].column], evals[n->pred].start,
                                            evals[n->pred].end);
      return it;
    }
    default: break;
  }
  const int k = n->nchild;
  iter** kids = calloc((size_t)k, sizeof(iter*));
  for (int i = 0; i < k; i++) kids[i] = it_build(n->child[i], seg, evals, q, pool);
  int nsorted = 0, nbitmap = 0, nscan = 0, nrem = 0;
  for (int i = 0; i < k; i++) {
    if (kids[i]->type == IT_IDX) { if (kids[i]->sorted) nsorted++; else nbitmap++; }
    else if (kids[i]->type == IT_SCAN) nscan++;
    else nrem++;
  }
  const int nidx = nsorted + nbitmap;
  if (n->type == FN_AND) {
    if (!((nidx > 0 && nscan > 0) || nidx > 1)) return it_new_multi(IT_AND, kids, k, seg, evals, q, pool);
    uint64_t* bits = malloc(sizeof(uint64_t) * (size_t)(nw ? nw : 1));
    for (int w = 0; w < nw; w++) bits[w] = ~0ull;
    for (int i = 0; i < k; i++)
      if (kids[i]->type == IT_IDX) for (int w = 0; w < nw; w++) bits[w] &= kids[i]->bits[w];
    for (int i = 0; i < k; i++) { /* ScanBasedDocIdIterator.applyAnd (SVScanDocIdIterator.java:75-94) */
      iter* sc = kids[i];
      if (sc->type != IT_SCAN) continue;
      for (int w = 0; w < nw; w++) {
        uint64_t m = bits[w];
        while (m) {
          int b = __builtin_ctzll(m);
          m &= m - 1;
          int d = w * 64 + b;
          if (d >= nd) { bits[w] &= ~(1ull << b); continue; }
          sc->scanned++;
          if (!scan_match(sc, d)) bits[w] &= ~(1ull << b);
        }
      }
    }
    iter* rangeless = it_new_idx(bits, 0, seg, evals, q, pool);
    if (nrem == 0) { free(kids); return rangeless; }
    iter** ks = calloc((size_t)nrem + 1, sizeof(iter*));
    int j = 0;
    ks[j++] = rangeless;
    for (int i = 0; i < k; i++) if (kids[i]->type != IT_IDX && kids[i]->type != IT_SCAN) ks[j++] = kids[i];
    free(kids);
    return it_new_multi(IT_AND, ks, j, seg, evals, q, pool);
  }
  /* OR */
  if (nidx <= 1) return it_new_multi(IT_OR, kids, k, seg, evals, q, pool);
  uint64_t* bits = calloc((size_t)(nw ? nw : 1), 8);
  for (int i = 0; i < k; i++)
    if (kids[i]->type == IT_IDX) for (int w = 0; w < nw; w++) bits[w] |= kids[i]->bits[w];
  iter* merged = it_new_idx(bits, 0, seg, evals, q, pool);
  if (nidx == k) { free(kids); return merged; }
  iter** ks = calloc((size_t)(k - nidx) + 1, sizeof(iter*));
  int j = 0;
  ks[j++] = merged;
  for (int i = 0; i < k; i++) if (kids[i]->type != IT_IDX) ks[j++] = kids[i];
  free(kids);
  return it_new_multi(IT_OR, ks, j, seg, evals, q, pool);
}
static int64_t pool_scanned(iter_pool* p) {
  int64_t s = 0;
  for (int i = 0; i < p->n; i++) s += (p->all[i]->type == IT_SCAN ? p->all[i]->scanned : 0) + p->all[i]->partial;
  return s;
}
static void pool_free(iter_pool* p) {
  for (int i = 0; i < p->n; i++) { free(p->all[i]->kids); free(p->all[i]->next_ids); free(p->all[i]->bits); free(p->all[i]); }
  free(p->all);
}

/* ======================================================================================= group-by */

/* fastutil 8.2.3 it.unimi.dsi.fastutil.HashCommon.mix(int) — published: h = x * 0x9E3779B9; h ^ (h >>> 16). */
static inline int32_t or_mix32(int32_t x) {
  uint32_t h = (uint32_t)x * 0x9E3779B9u;
  return (int32_t)(h ^ (h >> 16));
}

/* IntGroupIdMap (DictionaryBasedGroupKeyGenerator.java:1061-1152). */
typedef struct { int32_t* kv; int capacity, mask, max_entries, size; } int_gid_map;
static void igm_init(int_gid_map* m) {
  m->capacity = 1 << 9;
  int holder = m->capacity << 1;
  m->kv = calloc((size_t)holder, sizeof(int32_t));
  m->mask = holder - 1;
  m->max_entries = (int)(m->capacity * 0.75f);
  m->size = 0;
}
static void igm_expand(int_gid_map* m) {
  m->capacity <<= 1;
  int holder = m->capacity << 1;
  int32_t* old = m->kv;
  m->kv = calloc((size_t)holder, sizeof(int32_t));
  m->mask = holder - 1;
  m->max_entries <<= 1;
  int oi = 0;
  for (int i = 0; i < m->size; i++) {
    while (old[oi] == 0) oi += 2;
    int32_t key = old[oi], val = old[oi + 1];
    int ni = (or_mix32(key) << 1) & m->mask;
    while (m->kv[ni] != 0) ni = (ni + 2) & m->mask;
    m->kv[ni] = key; m->kv[ni + 1] = val;
    oi += 2;
  }
  free(old);
}
static int igm_get_group_id(int_gid_map* m, int32_t raw_key, int upper_bound) {
  int32_t ik = raw_key + 1;
  int idx = (or_mix32(ik) << 1) & m->mask;
  for (;;) {
    int32_t k = m->kv[idx];
    if (k == ik) return m->kv[idx + 1];
    if (k == 0) {
      if (m->size >= upper_bound) return INVALID_ID;
      int gid = m->size++;
      m->kv[idx] = ik; m->kv[idx + 1] = gid;
      if (m->size > m->max_entries) igm_expand(m);
      return gid;
    }
    idx = (idx + 2) & m->mask;
  }
}

/* Generic first-seen id map for LONG_MAP (fastutil Long2IntOpenHashMap.putIfAbsent, :675-683) and ARRAY_MAP
 * (Object2IntOpenHashMap<IntArray>.computeIntIfAbsent, :886-893).  Only first-seen id assignment and the
 * upper-bound cut are observable; slot order is not. */
typedef struct { uint64_t* keys; int32_t* keylen_or_ids; int32_t* ids; int nkeyw; int64_t cap; int64_t size; } gen_map;
static uint64_t hash_words(const uint64_t* w, int n) {
  uint64_t h = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < n; i++) { h ^= w[i]; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 31; }
  return h;
}
static void gm_init(gen_map* m, int nkeyw) {
  m->nkeyw = nkeyw; m->cap = 1024; m->size = 0;
  m->keys = malloc(sizeof(uint64_t) * (size_t)m->cap * nkeyw);
  m->ids = malloc(sizeof(int32_t) * (size_t)m->cap);
  for (int64_t i = 0; i < m->cap; i++) m->ids[i] = -1;
  m->keylen_or_ids = NULL;
}
static void gm_grow(gen_map* m) {
  int64_t oc = m->cap;
  uint64_t* ok = m->keys; int32_t* oid = m->ids;
  m->cap *= 2;
  m->keys = malloc(sizeof(uint64_t) * (size_t)m->cap * m->nkeyw);
  m->ids = malloc(sizeof(int32_t) * (size_t)m->cap);
  for (int64_t i = 0; i < m->cap; i++) m->ids[i] = -1;
  for (int64_t i = 0; i < oc; i++) {
    if (oid[i] < 0) continue;
    int64_t s = (int64_t)(hash_words(ok + i * m->nkeyw, m->nkeyw) & (uint64_t)(m->cap - 1));
    while (m->ids[s] >= 0) s = (s + 1) & (m->cap - 1);
    memcpy(m->keys + s * m->nkeyw, ok + i * m->nkeyw, sizeof(uint64_t) * m->nkeyw);
    m->ids[s] = oid[i];
  }
  free(ok); free(oid);
}
static int gm_get_group_id(gen_map* m, const uint64_t* key, int upper_bound) {
  int64_t s = (int64_t)(hash_words(key, m->nkeyw) & (uint64_t)(m->cap - 1));
  for (;;) {
    if (m->ids[s] < 0) {
      if (m->size >= upper_bound) return INVALID_ID;
      memcpy(m->keys + s * m->nkeyw, key, sizeof(uint64_t) * m->nkeyw);
      int id = (int)m->size++;
      m->ids[s] = id;
      if (m->size * 2 > m->cap) gm_grow(m);
      return id;
    }
    if (memcmp(m->keys + s * m->nkeyw, key, sizeof(uint64_t) * m->nkeyw) == 0) return m->ids[s];
    s = (s + 1) & (m->cap - 1);
  }
}
static void gm_free(gen_map* m) { free(m->keys); free(m->ids); }

/* Per-segment group-by state: DictionaryBasedGroupKeyGenerator + DoubleGroupByResultHolder per function. */
typedef struct {
  int holder;
  int nk;                    /* group-by columns */
  int card[16];
  int64_t upper_bound;       /* _globalGroupIdUpperBound */
  uint8_t* flags;            /* ARRAY */
  int64_t num_keys;          /* ARRAY */
  int_gid_map imap;
  gen_map gmap;              /* LONG_MAP (1 word) and ARRAY_MAP (nk words) */
  int64_t* raw_of_gid;       /* gid -> raw key (INT/LONG map) */
  int32_t* dictids_of_gid;   /* gid -> dictIds (ARRAY_MAP) */
  int64_t ngid_cap;
  double** vals;             /* per agg */
  int64_t** avg_cnt;
  int64_t vcap;
} seg_groupby;

static void sg_ensure(seg_groupby* g, const or_query* q, int64_t need) {
  if (need <= g->vcap) return;
  int64_t nc = g->vcap ? g->vcap : 1024;
  while (nc < need) nc *= 2;
  for (int a = 0; a < q->num_aggs; a++) {
    g->vals[a] = realloc(g->vals[a], sizeof(double) * (size_t)nc);
    g->avg_cnt[a] = realloc(g->avg_cnt[a], sizeof(int64_t) * (size_t)nc);
    double dv = q->aggs[a].fn == OR_AGG_MIN ? INFINITY : q->aggs[a].fn == OR_AGG_MAX ? -INFINITY : 0.0;
    for (int64_t i = g->vcap; i < nc; i++) { g->vals[a][i] = dv; g->avg_cnt[a][i] = 0; }
  }
  if (g->holder == OR_HOLDER_INT_MAP || g->holder == OR_HOLDER_LONG_MAP) {
    g->raw_of_gid = realloc(g->raw_of_gid, sizeof(int64_t) * (size_t)nc);
  } else if (g->holder == OR_HOLDER_ARRAY_MAP) {
    g->dictids_of_gid = realloc(g->dictids_of_gid, sizeof(int32_t) * (size_t)nc * g->nk);
  }
  g->vcap = nc;
}

/* ---- result blobs */
typedef struct { uint8_t* b; int64_t n, cap; } bbuf;
static void bb_put(bbuf* b, const void* p, int64_t n) {
  if (b->n + n > b->cap) { b->cap = (b->cap + n) * 2; b->b = realloc(b->b, (size_t)b->cap); }
  memcpy(b->b + b->n, p, (size_t)n); b->n += n;
}
static void key_append_value(bbuf* b, const or_column* c, int id) {
  if (c->data_type == OR_INT || c->data_type == OR_LONG) {
    int64_t v = c->data_type == OR_INT ? dict_int(c, id) : dict_long(c, id);
    bb_put(b, &v, 8);
  } else if (c->data_type == OR_FLOAT || c->data_type == OR_DOUBLE) {
    double v = c->data_type == OR_FLOAT ? (double)dict_float(c, id) : dict_double(c, id);
    bb_put(b, &v, 8);
  } else {
    const uint8_t* p; int n = dict_str(c, id, &p);
    uint32_t len = (uint32_t)n;
    bb_put(b, &len, 4); bb_put(b, p, n);
  }
}

typedef struct {
  int64_t ngroups;
  bbuf keys;
  int64_t* koff; int64_t kcap;
  double* vals;      /* [ngroups][naggs] */
  int64_t* cnts;
  int64_t vcap;
  int64_t docs_scanned, in_filter, post_filter, total_docs;
  int holder;
  int limit_reached;
  int status;
  char msg[256];
} seg_result;

static void sr_add_group(seg_result* r, int naggs) {
  if (r->ngroups + 2 > r->kcap) { r->kcap = (r->kcap + 2) * 2; r->koff = realloc(r->koff, sizeof(int64_t) * (size_t)r->kcap); }
  if (r->ngroups + 1 > r->vcap) {
    r->vcap = (r->vcap + 1) * 2;
    r->vals = realloc(r->vals, sizeof(double) * (size_t)r->vcap * (naggs ? naggs : 1));
    r->cnts = realloc(r->cnts, sizeof(int64_t) * (size_t)r->vcap * (naggs ? naggs : 1));
  }
}

/* Columns projected by the operator (TransformOperator.getNumColumnsProjected): distinct columns referenced by
 * group-by expressions and aggregation arguments. */
static int num_projected(const or_query* q) {
  int seen[256] = {0};
  int n = 0;
  for (int i = 0; i < q->num_group_by; i++) if (!seen[q->group_by[i]]) { seen[q->group_by[i]] = 1; n++; }
  for (int i = 0; i < q->num_aggs; i++)
    if (q->aggs[i].column >= 0 && !seen[q->aggs[i].column]) { seen[q->aggs[i].column] = 1; n++; }
  return n;
}

/* AggregationGroupByOperator.getNextBlock (core/operator/query/AggregationGroupByOperator.java:62-79) on one
 * segment: DocIdSetOperator blocks of <= 10000 docIds, DefaultGroupByExecutor.process (:117-147). */
static int run_star_segment(const or_segment* seg, const or_query* q, const pred_eval* evals, seg_result* r);

static void run_segment(const or_segment* seg, const or_query* q, seg_result* r) {
  memset(r, 0, sizeof *r);
  r->total_docs = seg->num_docs;
  int np = q->num_predicates;
  pred_eval* evals = calloc((size_t)(np ? np : 1), sizeof(pred_eval));
  for (int i = 0; i < np; i++) {
    int st = build_pred_eval(seg, &q->predicates[i], &evals[i], r->msg, sizeof r->msg);
    if (st) { r->status = st; for (int j = 0; j < i; j++) pred_eval_free(&evals[j]); free(evals); return; }
  }
  if (q->use_star_tree && seg->star_tree && run_star_segment(seg, q, evals, r)) {
    for (int j = 0; j < np; j++) pred_eval_free(&evals[j]);
    free(evals);
    return;
  }
  fnode* root = build_filter_tree(seg, q, evals, r->msg, sizeof r->msg);
  if (!root) { r->status = -1; for (int j = 0; j < np; j++) pred_eval_free(&evals[j]); free(evals); return; }
  iter_pool pool = {0};
  iter* it = it_build(root, seg, evals, q, &pool);

  /* DictionaryBasedGroupKeyGenerator ctor (:97-161): holder choice. */
  seg_groupby g;
  memset(&g, 0, sizeof g);
  g.nk = q->num_group_by;
  g.vals = calloc((size_t)q->num_aggs + 1, sizeof(double*));
  g.avg_cnt = calloc((size_t)q->num_aggs + 1, sizeof(int64_t*));
  long long card_product = 1;
  int long_overflow = 0;
  for (int i = 0; i < g.nk; i++) {
    int card = seg->columns[q->group_by[i]].cardinality;
    if (card < 1) card = 1; /* empty segment: Pinot never builds one; keep the key math defined */
    g.card[i] = card;
    if (!long_overflow) {
      if (card_product > INT64_MAX / card) long_overflow = 1;
      else card_product *= card;
    }
  }
  if (long_overflow) {
    g.holder = OR_HOLDER_ARRAY_MAP; g.upper_bound = q->num_groups_limit;
    gm_init(&g.gmap, g.nk);
  } else if (card_product > INT32_MAX) {
    g.holder = OR_HOLDER_LONG_MAP; g.upper_bound = q->num_groups_limit;
    gm_init(&g.gmap, 1);
  } else {
    g.upper_bound = card_product < q->num_groups_limit ? card_product : q->num_groups_limit;
    if (card_product > q->max_initial_result_holder_capacity) { g.holder = OR_HOLDER_INT_MAP; igm_init(&g.imap); }
    else { g.holder = OR_HOLDER_ARRAY; g.flags = calloc((size_t)g.upper_bound + 1, 1); }
  }
  r->holder = g.holder;
  if (g.holder == OR_HOLDER_ARRAY) sg_ensure(&g, q, g.upper_bound);

  int32_t* docs = malloc(sizeof(int32_t) * MAX_DOC_PER_CALL);
  int32_t* gids = malloc(sizeof(int32_t) * MAX_DOC_PER_CALL);
  int32_t* dids[16];
  for (int i = 0; i < g.nk; i++) dids[i] = malloc(sizeof(int32_t) * MAX_DOC_PER_CALL);
  int32_t* mids = malloc(sizeof(int32_t) * MAX_DOC_PER_CALL);
  double* dvals = malloc(sizeof(double) * MAX_DOC_PER_CALL);
  int nproj = num_projected(q);
  /* raw aggregation operands: the column's chunks decoded once per segment (ChunkReaderContext caches the chunk in
   * use; the values read are the same) */
  double** raw_vals = calloc((size_t)q->num_aggs + 1, sizeof(double*));
  for (int a = 0; a < q->num_aggs; a++) {
    const or_column* c = q->aggs[a].column >= 0 ? &seg->columns[q->aggs[a].column] : NULL;
    if (!c || !c->raw) continue;
    raw_vals[a] = malloc(sizeof(double) * (size_t)(seg->num_docs > 0 ? seg->num_docs : 1));
    if (or_raw_decode(c, c->fwd, c->fwd_len, seg->num_docs, NULL, raw_vals[a])) {
      snprintf(r->msg, sizeof r->msg, "raw forward index of column %d is unreadable", q->aggs[a].column);
      r->status = -1;
    }
  }

  int eof = 0;
  while (!eof) {
    /* DocIdSetOperator.getNextBlock (core/operator/DocIdSetOperator.java:59-84) */
    int pos = 0;
    for (int i = 0; i < MAX_DOC_PER_CALL; i++) {
      int d = it_next(it);
      if (d == EOF_DOC) { eof = 1; break; }
      docs[pos++] = d;
    }
    if (pos == 0) break;
    r->docs_scanned += pos;
    /* generateKeysForBlock: DataFetcher.readDictIds -> FixedBitSVForwardIndexReaderV2.readDictIds */
    for (int i = 0; i < g.nk; i++) {
      const or_column* c = &seg->columns[q->group_by[i]];
      or_read_dict_ids(c->fwd, c->bits, seg->num_docs, docs, pos, dids[i]);
    }
    switch (g.holder) {
      case OR_HOLDER_ARRAY: /* ArrayBasedHolder.processSingleValue (:259-323) */
        for (int d = 0; d < pos; d++) {
          int gid = 0;
          for (int j = g.nk - 1; j >= 0; j--) gid = gid * g.card[j] + dids[j][d];
          gids[d] = gid;
        }
        if (g.num_keys < g.upper_bound) /* markGroups (:296-308) */
          for (int d = 0; d < pos; d++)
            if (!g.flags[gids[d]]) { g.num_keys++; g.flags[gids[d]] = 1; if (g.num_keys == g.upper_bound) break; }
        break;
      case OR_HOLDER_INT_MAP: /* IntMapBasedHolder (:420-450) */
        for (int d = 0; d < pos; d++) {
          int raw = 0;
          for (int j = g.nk - 1; j >= 0; j--) raw = raw * g.card[j] + dids[j][d];
          int gid = igm_get_group_id(&g.imap, raw, (int)g.upper_bound);
          if (gid >= 0) { sg_ensure(&g, q, gid + 1); g.raw_of_gid[gid] = raw; }
          gids[d] = gid;
        }
        break;
      case OR_HOLDER_LONG_MAP: /* LongMapBasedHolder (:644-683) */
        for (int d = 0; d < pos; d++) {
          uint64_t raw = 0;
          for (int j = g.nk - 1; j >= 0; j--) raw = raw * (uint64_t)g.card[j] + (uint64_t)dids[j][d];
          int gid = gm_get_group_id(&g.gmap, &raw, (int)g.upper_bound);
          if (gid >= 0) { sg_ensure(&g, q, gid + 1); g.raw_of_gid[gid] = (int64_t)raw; }
          gids[d] = gid;
        }
        break;
      default: /* ArrayMapBasedHolder (:850-893) */
        for (int d = 0; d < pos; d++) {
          uint64_t key[16];
          for (int j = 0; j < g.nk; j++) key[j] = (uint64_t)dids[j][d];
          int gid = gm_get_group_id(&g.gmap, key, (int)g.upper_bound);
          if (gid >= 0) {
            sg_ensure(&g, q, gid + 1);
            for (int j = 0; j < g.nk; j++) g.dictids_of_gid[(int64_t)gid * g.nk + j] = dids[j][d];
          }
          gids[d] = gid;
        }
        break;
    }
    /* aggregateGroupBySV per function, in query order, docs in block order. */
    for (int a = 0; a < q->num_aggs; a++) {
      const or_agg* ag = &q->aggs[a];
      double* h = g.vals[a];
      if (ag->fn == OR_AGG_COUNT) { /* CountAggregationFunction.java:90-96 */
        for (int d = 0; d < pos; d++) if (gids[d] != INVALID_ID) h[gids[d]] = h[gids[d]] + 1;
        continue;
      }
      const or_column* c = &seg->columns[ag->column];
      if (c->raw) { /* DataFetcher.readDoubleValues on a raw column: ForwardIndexReader.readValuesSV */
        for (int d = 0; d < pos; d++) dvals[d] = raw_vals[a][docs[d]];
      } else {
        or_read_dict_ids(c->fwd, c->bits, seg->num_docs, docs, pos, mids);   /* DataFetcher.readDoubleValues */
        for (int d = 0; d < pos; d++) dvals[d] = or_dict_get_double(c, mids[d]);
      }
      switch (ag->fn) {
        case OR_AGG_SUM: /* SumAggregationFunction.java:66-73 */
          for (int d = 0; d < pos; d++) if (gids[d] != INVALID_ID) h[gids[d]] = h[gids[d]] + dvals[d];
          break;
        case OR_AGG_MIN: /* MinAggregationFunction.java:69-79 */
          for (int d = 0; d < pos; d++) if (gids[d] != INVALID_ID && dvals[d] < h[gids[d]]) h[gids[d]] = dvals[d];
          break;
        case OR_AGG_MAX:
          for (int d = 0; d < pos; d++) if (gids[d] != INVALID_ID && dvals[d] > h[gids[d]]) h[gids[d]] = dvals[d];
          break;
        default: /* AVG: AvgPair(sum, count) (AvgAggregationFunction.java:93-146) */
          for (int d = 0; d < pos; d++)
            if (gids[d] != INVALID_ID) { h[gids[d]] += dvals[d]; g.avg_cnt[a][gids[d]] += 1; }
          break;
      }
    }
  }
  r->in_filter = pool_scanned(&pool);
  r->post_filter = r->docs_scanned * nproj; /* AggregationGroupByOperator.java:94 */
  if (g.nk == 0 && root->type == FN_ALL) {
    /* Aggregation-only over a match-all filter (AggregationPlanNode.java:165-183): COUNT-only queries are answered
     * from segment metadata (MetadataBasedAggregationOperator.java:89-92), MIN/MAX-only from the dictionaries
     * (DictionaryBasedAggregationOperator.java:171-173) -- same values as the scan, statistics
     * (numTotalDocs, 0, 0, numTotalDocs). */
    int all_count = 1, all_minmax = 1;
    for (int a = 0; a < q->num_aggs; a++) {
      all_count &= q->aggs[a].fn == OR_AGG_COUNT;
      /* isFitForDictionaryBasedPlan needs a dictionary (AggregationPlanNode.java:196-213) */
      all_minmax &= (q->aggs[a].fn == OR_AGG_MIN || q->aggs[a].fn == OR_AGG_MAX) &&
                    !seg->columns[q->aggs[a].column].raw;
    }
    if (all_count || all_minmax) r->post_filter = 0;
  }

  /* Emit groups through getStringGroupKeys order: ARRAY ascending raw key; maps in id order (iteration order of
   * hash maps is not observable after the combine). */
  bbuf* kb = &r->keys;
  int64_t ngid = 0;
  if (g.holder == OR_HOLDER_ARRAY) ngid = g.upper_bound;
  else if (g.holder == OR_HOLDER_INT_MAP) ngid = g.imap.size;
  else ngid = g.gmap.size;
  if (g.holder != OR_HOLDER_ARRAY && (ngid >= g.upper_bound)) r->limit_reached = 1;
  for (int64_t gid = 0; gid < ngid; gid++) {
    if (g.holder == OR_HOLDER_ARRAY && !g.flags[gid]) continue;
    sr_add_group(r, q->num_aggs);
    r->koff[r->ngroups] = kb->n;
    int64_t raw = 0;
    if (g.holder == OR_HOLDER_ARRAY) raw = gid;
    else if (g.holder != OR_HOLDER_ARRAY_MAP) raw = g.raw_of_gid[gid];
    for (int j = 0; j < g.nk; j++) {
      int id;
      if (g.holder == OR_HOLDER_ARRAY_MAP) id = g.dictids_of_gid[gid * g.nk + j];
      else { id = (int)(raw % g.card[j]); raw /= g.card[j]; } /* getKeys (:608-624) */
      key_append_value(kb, &seg->columns[q->group_by[j]], id);
    }
    for (int a = 0; a < q->num_aggs; a++) {
      r->vals[r->ngroups * q->num_aggs + a] = g.vals[a][gid];
      r->cnts[r->ngroups * q->num_aggs + a] = g.avg_cnt[a][gid];
    }
    r->ngroups++;
  }
  if (r->koff) r->koff[r->ngroups] = kb->n;

  for (int a = 0; a < q->num_aggs; a++) { free(g.vals[a]); free(g.avg_cnt[a]); }
  free(g.vals); free(g.avg_cnt); free(g.flags); free(g.raw_of_gid); free(g.dictids_of_gid);
  if (g.holder == OR_HOLDER_INT_MAP) free(g.imap.kv);
  if (g.holder == OR_HOLDER_LONG_MAP || g.holder == OR_HOLDER_ARRAY_MAP) gm_free(&g.gmap);
  free(docs); free(gids); free(mids); free(dvals);
  for (int a = 0; a < q->num_aggs; a++) free(raw_vals[a]);
  free(raw_vals);
  for (int i = 0; i < g.nk; i++) free(dids[i]);
  pool_free(&pool);
  fn_free(root);
  for (int j = 0; j < np; j++) pred_eval_free(&evals[j]);
  free(evals);
}

/* ======================================================================================= star-tree */

/* The filter program as a tree (FilterContext): AND / OR / PREDICATE / NOT nodes over predicate indexes. */
typedef struct qnode { int op; int pred; int n; struct qnode** kid; } qnode;
static void qn_free(qnode* n) {
  if (!n) return;
  for (int i = 0; i < n->n; i++) qn_free(n->kid[i]);
  free(n->kid); free(n);
}
static qnode* qn_build(const or_query* q) {
  qnode** st = calloc((size_t)q->num_filter_ops + 1, sizeof(qnode*));
  int sp = 0;
  for (int i = 0; i < q->num_filter_ops; i++) {
    const or_filter_op* o = &q->filter[i];
    qnode* n = calloc(1, sizeof(qnode));
    n->op = o->op;
    if (o->op == OR_OP_PRED) n->pred = o->arg;
    else {
      n->n = o->op == OR_OP_NOT ? 1 : o->arg;
      n->kid = calloc((size_t)n->n, sizeof(qnode*));
      for (int k = n->n - 1; k >= 0; k--) n->kid[k] = st[--sp];
    }
    st[sp++] = n;
  }
  qnode* root = sp ? st[0] : NULL;
  free(st);
  return root;
}

/* Per star-tree dimension: the composite predicate evaluators on it (StarTreeUtils.extractPredicateEvaluatorsMap,
 * core/startree/StarTreeUtils.java:95-138): a list, ANDed, of predicate-index lists, ORed. */
typedef struct { int ncomp; int* comp_off; int* preds; int npreds; } dim_preds;

static void dp_add(dim_preds* d, const int* p, int n) {
  d->comp_off = realloc(d->comp_off, sizeof(int) * (size_t)(d->ncomp + 2));
  if (d->ncomp == 0) d->comp_off[0] = 0;
  d->preds = realloc(d->preds, sizeof(int) * (size_t)(d->npreds + n + 1));
  memcpy(d->preds + d->npreds, p, sizeof(int) * (size_t)n);
  d->npreds += n;
  d->ncomp++;
  d->comp_off[d->ncomp] = d->npreds;
}

static int star_dim_of(const or_star_tree* st, int column) {
  for (int k = 0; k < st->num_dims; k++) if (st->dim_columns[k] == column) return k;
  return -1;
}

/* isOrClauseValidForStarTree (:180-219) over extractOrClausePredicates (:222-244): the predicates under an OR; returns
 * 0 when the clause cannot be solved with the star-tree. */
static int or_preds(const qnode* n, int* out, int* nout) {
  for (int i = 0; i < n->n; i++) {
    const qnode* c = n->kid[i];
    if (c->op == OR_OP_PRED) out[(*nout)++] = c->pred;
    else if (c->op == OR_OP_OR) { if (!or_preds(c, out, nout)) return 0; }
    else return 0; /* AND / NOT under OR */
  }
  return 1;
}

/* extractPredicateEvaluatorsMap + isFitForStarTree: fills dp[dim]; returns 0 when the filter does not fit. */
static int star_filter_fit(const or_segment* seg, const or_query* q, const pred_eval* ev, const qnode* root,
                           dim_preds* dp) {
  const or_star_tree* st = seg->star_tree;
  if (!root) return 1;
  const qnode** queue = malloc(sizeof(qnode*) * (size_t)(q->num_filter_ops + 1));
  int head = 0, tail = 0, ok = 1;
  int* buf = malloc(sizeof(int) * (size_t)(q->num_predicates + 1));
  queue[tail++] = root;
  while (ok && head < tail) {
    const qnode* n = queue[head++];
    if (n->op == OR_OP_AND) {
      for (int i = 0; i < n->n; i++) queue[tail++] = n->kid[i];
    } else if (n->op == OR_OP_PRED) {
      const int col = q->predicates[n->pred].column, d = star_dim_of(st, col);
      if (d < 0 || seg->columns[col].raw) { ok = 0; break; }        /* not a star-tree dimension */
      if (!ev[n->pred].always_true) dp_add(&dp[d], &n->pred, 1);
    } else if (n->op == OR_OP_OR) {
      int np = 0;
      if (!or_preds(n, buf, &np)) { ok = 0; break; }
      int col = -1, keep = 0, always_true = 0;
      for (int i = 0; i < np && ok; i++) {
        const int c = q->predicates[buf[i]].column;
        if (star_dim_of(st, c) < 0 || seg->columns[c].raw) { ok = 0; break; }
        if (ev[buf[i]].always_true) { always_true = 1; break; }     /* the whole clause is always true */
        if (ev[buf[i]].always_false) continue;
        if (col >= 0 && col != c) { ok = 0; break; }                /* predicates on several columns */
        col = c;
        buf[keep++] = buf[i];
      }
      if (ok && !always_true && keep > 0) dp_add(&dp[star_dim_of(st, col)], buf, keep);
      /* NOTE (reference): an OR whose predicates are all always-false yields an empty list, read as always-true */
    } else {
      ok = 0; /* NOT */
    }
  }
  free(queue); free(buf);
  return ok;
}

/* StarTreeFilterOperator.getMatchingDictIds (:353-423) as flags over the dimension's dictIds: the AND of the
 * composites, each the OR of its predicates. */
static uint8_t* dim_match(const dim_preds* d, const pred_eval* ev, int card, int* any) {
  uint8_t* m = malloc((size_t)(card ? card : 1));
  *any = 0;
  for (int id = 0; id < card; id++) {
    int v = 1;
    for (int c = 0; c < d->ncomp && v; c++) {
      int o = 0;
      for (int i = d->comp_off[c]; i < d->comp_off[c + 1] && !o; i++) o = pred_apply(&ev[d->preds[i]], id);
      v = o;
    }
    m[id] = (uint8_t)v;
    *any |= v;
  }
  return m;
}

static int composite_apply(const dim_preds* d, const pred_eval* ev, int c, int id) {
  for (int i = d->comp_off[c]; i < d->comp_off[c + 1]; i++) if (pred_apply(&ev[d->preds[i]], id)) return 1;
  return 0;
}

/* StarTreeFilterOperator + StarTreeGroupByExecutor over one segment's star-tree (core/startree/operator/
 * StarTreeFilterOperator.java:185-338, core/startree/executor/StarTreeGroupByExecutor.java:60-71).  Returns 0 when
 * the query does not fit the tree (StarTreeUtils.isFitForStarTree, :151-176): the caller then scans. */
static int run_star_segment(const or_segment* seg, const or_query* q, const pred_eval* ev, seg_result* r) {
  const or_star_tree* st = seg->star_tree;
  const int nd = st->num_dims, na = q->num_aggs, nk = q->num_group_by;
  if (nd > 30 || nk > 16) return 0;
  /* function-column pairs (extractAggregationFunctionPairs + containsFunctionColumnPair) */
  int* metric_of = malloc(sizeof(int) * (size_t)(na ? na : 1));
  for (int a = 0; a < na; a++) {
    metric_of[a] = -1;
    for (int m = 0; m < st->num_metrics; m++)
      if (st->metric_fn[m] == q->aggs[a].fn && st->metric_column[m] == q->aggs[a].column) { metric_of[a] = m; break; }
    if (metric_of[a] < 0) { free(metric_of); return 0; }
  }
  int gdim[16];
  uint32_t group_mask = 0;
  for (int j = 0; j < nk; j++) {
    gdim[j] = star_dim_of(st, q->group_by[j]);
    if (gdim[j] < 0) { free(metric_of); return 0; }
  }
  qnode* root = qn_build(q);
  dim_preds* dp = calloc((size_t)nd, sizeof(dim_preds));
  if (!star_filter_fit(seg, q, ev, root, dp)) {
    for (int k = 0; k < nd; k++) { free(dp[k].comp_off); free(dp[k].preds); }
    free(dp); qn_free(root); free(metric_of);
    return 0;
  }
  uint32_t pred_mask = 0;
  for (int k = 0; k < nd; k++) if (dp[k].ncomp) pred_mask |= 1u << k;
  for (int j = 0; j < nk; j++) if (!((pred_mask >> gdim[j]) & 1u)) group_mask |= 1u << gdim[j];
  /* _groupByColumns are the group-by columns without a predicate (StarTreeFilterOperator ctor, :150-160) */

  /* traverseStarTree (:234-338): BFS; matching dictIds computed on first use, an empty set empties the result */
  uint8_t** match = calloc((size_t)nd, sizeof(uint8_t*));
  const int32_t* N = st->nodes;
  uint8_t* docs = calloc((size_t)(st->num_docs ? st->num_docs : 1), 1);
  uint32_t remaining = 0;
  int empty = 0;
  typedef struct { int node; uint32_t rp, rg; } entry;
  int64_t qcap = 1024, qh = 0, qt = 0;
  entry* queue = malloc(sizeof(entry) * (size_t)qcap);
  queue[qt++] = (entry){0, pred_mask, group_mask};
  while (qh < qt && !empty) {
    const entry e = queue[qh++];
    const int32_t* n = N + (int64_t)e.node * 7;
    const int first = n[5], last = n[6];
#define PUSH(nd_, rp_, rg_)                                                              \
    do {                                                                                 \
      if (qt == qcap) { qcap *= 2; queue = realloc(queue, sizeof(entry) * (size_t)qcap); } \
      queue[qt++] = (entry){(nd_), (rp_), (rg_)};                                        \
    } while (0)
    if (!e.rp && !e.rg) { docs[n[4]] = 1; continue; }              /* the node's aggregated document */
    if (first < 0) {                                               /* leaf: its documents, predicates remain */
      for (int d = n[2]; d < n[3]; d++) docs[d] = 1;
      remaining |= e.rp;
      continue;
    }
    const int cd = N[(int64_t)first * 7];                          /* the children's dimension */
    if ((e.rp >> cd) & 1u) {
      if (!match[cd]) {
        int any = 0;
        match[cd] = dim_match(&dp[cd], ev, seg->columns[st->dim_columns[cd]].cardinality, &any);
        if (!any) { empty = 1; break; }
      }
      for (int c = first; c <= last; c++) {
        const int v = N[(int64_t)c * 7 + 1];
        if (v != -1 && match[cd][v]) PUSH(c, e.rp & ~(1u << cd), e.rg);
      }
    } else {
      uint32_t rg = e.rg;
      if (!((e.rg >> cd) & 1u)) {
        if (N[(int64_t)first * 7 + 1] == -1) { PUSH(first, e.rp, e.rg); continue; } /* the star node */
      } else {
        rg &= ~(1u << cd);
      }
      for (int c = first; c <= last; c++) if (N[(int64_t)c * 7 + 1] != -1) PUSH(c, e.rp, rg);
    }
#undef PUSH
  }
  free(queue);

  /* residual filter (:185-226): the remaining predicate columns' composites ANDed with the traversal's documents */
  int64_t bitmap_docs = 0, matched = 0;
  int nrem = 0;
  for (int k = 0; k < nd; k++) nrem += (remaining >> k) & 1u;
  int32_t** dimids = calloc((size_t)nd, sizeof(int32_t*));
  /* a remaining composite that can match nothing is an EmptyFilterOperator leaf, which empties the AND
   * (FilterOperatorUtils.getLeafFilterOperator / getAndFilterOperator): no document is read */
  for (int k = 0; k < nd && !empty; k++)
    if ((remaining >> k) & 1u)
      for (int c = 0; c < dp[k].ncomp && !empty; c++) {
        int all_false = 1;
        for (int i = dp[k].comp_off[c]; i < dp[k].comp_off[c + 1]; i++) all_false &= ev[dp[k].preds[i]].always_false;
        empty = all_false;
      }
  if (!empty) {
    for (int k = 0; k < nd; k++) {
      const int used = ((remaining >> k) & 1u) != 0;
      int grouped = 0;
      for (int j = 0; j < nk; j++) grouped |= gdim[j] == k;
      if (!used && !grouped) continue;
      dimids[k] = malloc(sizeof(int32_t) * (size_t)(st->num_docs ? st->num_docs : 1));
      const int bits = seg->columns[st->dim_columns[k]].bits;
      for (int d = 0; d < st->num_docs; d++) dimids[k][d] = fixedbit_read(st->dim_fwd[k], d, bits);
    }
    for (int d = 0; d < st->num_docs; d++) {
      if (!docs[d]) continue;
      bitmap_docs++;
      int keep = 1;
      for (int k = 0; k < nd && keep; k++)
        if ((remaining >> k) & 1u)
          for (int c = 0; c < dp[k].ncomp && keep; c++) keep = composite_apply(&dp[k], ev, c, dimids[k][d]);
      docs[d] = (uint8_t)keep;
      matched += keep;
    }
  }

  /* StarTreeGroupByExecutor: DictionaryBasedGroupKeyGenerator over the star-tree's dimensions (mixed radix of the
   * segment dictionaries' cardinalities, first column fastest) and the function-column pairs' pre-aggregated values
   * (COUNT adds count__*, CountAggregationFunction.java:97-104; SUM / MIN / MAX / AVG their pairs), in ascending
   * star-tree docId order. */
  int64_t card[16], stride[16], space = 1;
  for (int j = 0; j < nk; j++) {
    card[j] = seg->columns[q->group_by[j]].cardinality > 0 ? seg->columns[q->group_by[j]].cardinality : 1;
    stride[j] = space;
    space = space > INT64_MAX / card[j] ? INT64_MAX : space * card[j];
  }
  gen_map gm;
  gm_init(&gm, 1);
  int64_t ng = 0, vcap = 0;
  double* vals = NULL;
  int64_t* cnts = NULL;
  int64_t* raw_of = NULL;
  if (!empty && matched) {
    for (int d = 0; d < st->num_docs; d++) {
      if (!docs[d]) continue;
      uint64_t raw = 0;
      for (int j = 0; j < nk; j++) raw += (uint64_t)dimids[gdim[j]][d] * (uint64_t)stride[j];
      const int gid = gm_get_group_id(&gm, &raw, INT32_MAX);
      if (gid >= ng) {
        if (gid >= vcap) {
          vcap = vcap ? vcap * 2 : 1024;
          vals = realloc(vals, sizeof(double) * (size_t)(vcap * (na ? na : 1)));
          cnts = realloc(cnts, sizeof(int64_t) * (size_t)(vcap * (na ? na : 1)));
          raw_of = realloc(raw_of, sizeof(int64_t) * (size_t)vcap);
        }
        for (; ng <= gid; ng++) {
          raw_of[ng] = (int64_t)raw;
          for (int a = 0; a < na; a++) {
            vals[ng * na + a] = q->aggs[a].fn == OR_AGG_MIN ? INFINITY : q->aggs[a].fn == OR_AGG_MAX ? -INFINITY : 0.0;
            cnts[ng * na + a] = 0;
          }
        }
      }
      for (int a = 0; a < na; a++) {
        const int m = metric_of[a];
        double* v = &vals[(int64_t)gid * na + a];
        switch (q->aggs[a].fn) {
          case OR_AGG_COUNT: *v += (double)st->metric_i64[m][d]; break;
          case OR_AGG_SUM: *v += st->metric_f64[m][d]; break;
          case OR_AGG_MIN: if (st->metric_f64[m][d] < *v) *v = st->metric_f64[m][d]; break;
          case OR_AGG_MAX: if (st->metric_f64[m][d] > *v) *v = st->metric_f64[m][d]; break;
          default: *v += st->metric_f64[m][d]; cnts[(int64_t)gid * na + a] += st->metric_i64[m][d]; break;
        }
      }
    }
  }
  r->holder = OR_HOLDER_LONG_MAP;
  r->docs_scanned = matched;
  r->in_filter = bitmap_docs * nrem;  /* the residual scan leaves read each traversal document once per column */
  r->post_filter = matched * num_projected(q);
  bbuf* kb = &r->keys;
  for (int64_t g = 0; g < ng; g++) {
    sr_add_group(r, na);
    r->koff[r->ngroups] = kb->n;
    for (int j = 0; j < nk; j++)
      key_append_value(kb, &seg->columns[q->group_by[j]], (int)((raw_of[g] / stride[j]) % card[j]));
    for (int a = 0; a < na; a++) {
      r->vals[r->ngroups * na + a] = vals[g * na + a];
      r->cnts[r->ngroups * na + a] = cnts[g * na + a];
    }
    r->ngroups++;
  }
  if (r->koff) r->koff[r->ngroups] = kb->n;
  gm_free(&gm);
  free(vals); free(cnts); free(raw_of);
  for (int k = 0; k < nd; k++) { free(dimids[k]); free(match[k]); free(dp[k].comp_off); free(dp[k].preds); }
  free(dimids); free(match); free(dp); free(docs);
  qn_free(root); free(metric_of);
  return 1;
}

/* ======================================================================================= combine */

typedef struct { const or_segment* segs; int nsegs; const or_query* q; seg_result* res; atomic_int next; } task_ctx;
static void* worker(void* arg) {
  task_ctx* t = arg;
  for (;;) {
    int i = atomic_fetch_add(&t->next, 1);
    if (i >= t->nsegs) break;
    run_segment(&t->segs[i], t->q, &t->res[i]);
  }
  return NULL;
}

/* blob-keyed map for GroupByCombineOperator._resultsMap */
typedef struct { int64_t* slot; int64_t cap; } blob_map;
static uint64_t hash_bytes(const uint8_t* p, int64_t n) {
  uint64_t h = 1469598103934665603ull;
  for (int64_t i = 0; i < n; i++) { h ^= p[i]; h *= 1099511628211ull; }
  return h;
}

/* One hash shard of the combine's merged map (keys with (hash >> 40) % nshards == shard), in segment order. */
typedef struct { bbuf kb; int64_t* koff; double* vals; int64_t* cnts; int64_t ng; } merge_shard;
typedef struct {
  seg_result* res; int nsegs; const or_query* q; int64_t limit; int nshards; merge_shard* shard; atomic_int next;
} merge_ctx;
static void merge_one(merge_ctx* mc, int sh) {
  const int na = mc->q->num_aggs;
  merge_shard* m = &mc->shard[sh];
  int64_t counter = 0;
  blob_map bm; bm.cap = 1024; bm.slot = malloc(sizeof(int64_t) * (size_t)bm.cap);
  for (int64_t i = 0; i < bm.cap; i++) bm.slot[i] = -1;
  bbuf kb = {0};
  int64_t* koff = malloc(sizeof(int64_t) * 2); int64_t kcap = 2;
  double* vals = NULL; int64_t* cnts = NULL; int64_t ng = 0, vcap = 0;
  koff[0] = 0;
  for (int s = 0; s < mc->nsegs; s++) {
    seg_result* r = &mc->res[s];
    for (int64_t gi = 0; gi < r->ngroups; gi++) {
      const uint8_t* k = r->keys.b + r->koff[gi];
      int64_t kn = r->koff[gi + 1] - r->koff[gi];
      uint64_t h = hash_bytes(k, kn);
      if (mc->nshards > 1 && (int)((h >> 40) % (uint64_t)mc->nshards) != sh) continue;
      int64_t sidx = (int64_t)(h & (uint64_t)(bm.cap - 1));
      int64_t found = -1;
      while (bm.slot[sidx] >= 0) {
        int64_t cand = bm.slot[sidx];
        if (koff[cand + 1] - koff[cand] == kn && memcmp(kb.b + koff[cand], k, (size_t)kn) == 0) { found = cand; break; }
        sidx = (sidx + 1) & (bm.cap - 1);
      }
      const double* v = r->vals + gi * na;
      const int64_t* c = r->cnts + gi * na;
      if (found < 0) {
        if (counter++ >= mc->limit) continue; /* _numGroups.getAndIncrement() < _interSegmentNumGroupsLimit */
        if (ng + 2 > kcap) { kcap *= 2; koff = realloc(koff, sizeof(int64_t) * (size_t)kcap); }
        if (ng + 1 > vcap) { vcap = vcap ? vcap * 2 : 64; vals = realloc(vals, sizeof(double) * vcap * (na ? na : 1)); cnts = realloc(cnts, sizeof(int64_t) * vcap * (na ? na : 1)); }
        bb_put(&kb, k, kn);
        koff[ng + 1] = kb.n;
        for (int a = 0; a < na; a++) { vals[ng * na + a] = v[a]; cnts[ng * na + a] = c[a]; }
        bm.slot[sidx] = ng;
        ng++;
        if (ng * 2 > bm.cap) {
          int64_t nc = bm.cap * 2;
          int64_t* ns = malloc(sizeof(int64_t) * (size_t)nc);
          for (int64_t i = 0; i < nc; i++) ns[i] = -1;
          for (int64_t e = 0; e < ng; e++) {
            uint64_t hh = hash_bytes(kb.b + koff[e], koff[e + 1] - koff[e]);
            int64_t p = (int64_t)(hh & (uint64_t)(nc - 1));
            while (ns[p] >= 0) p = (p + 1) & (nc - 1);
            ns[p] = e;
          }
          free(bm.slot); bm.slot = ns; bm.cap = nc;
        }
      } else {
        for (int a = 0; a < na; a++) { /* AggregationFunction.merge */
          double* dst = &vals[found * na + a];
          switch (mc->q->aggs[a].fn) {
            case OR_AGG_MIN: if (!(*dst < v[a])) *dst = v[a]; break; /* MinAggregationFunction.merge */
            case OR_AGG_MAX: if (!(*dst > v[a])) *dst = v[a]; break;
            case OR_AGG_COUNT: *dst = (double)((int64_t)*dst + (int64_t)v[a]); break; /* Long merge */
            default: *dst += v[a]; cnts[found * na + a] += c[a]; break;        /* SUM / AvgPair.apply */
          }
        }
      }
    }
  }
  free(bm.slot);
  m->kb = kb; m->koff = koff; m->vals = vals; m->cnts = cnts; m->ng = ng;
}
static void* merge_worker(void* arg) {
  merge_ctx* mc = arg;
  for (;;) {
    int sh = atomic_fetch_add(&mc->next, 1);
    if (sh >= mc->nshards) break;
    merge_one(mc, sh);
  }
  return NULL;
}

int or_execute_groupby(const or_segment* segs, int nsegs, const or_query* q, int nthreads, or_result* out,
                       char* msg, int msg_len) {
  memset(out, 0, sizeof *out);
  /* num_group_by == 0: aggregation-only (AggregationOperator / DefaultAggregationExecutor): one group with the empty
   * key, emitted when a doc matched; the caller supplies the functions' defaults for an empty result. */
  if (q->num_group_by < 0 || q->num_group_by > 16) { snprintf(msg, msg_len, "need 0..16 group-by columns"); return -1; }
  /* DictionaryBasedGroupKeyGenerator ctor: assert numGroupsLimit >= arrayBasedThreshold (:99) */
  if (q->num_groups_limit < q->max_initial_result_holder_capacity) {
    snprintf(msg, msg_len, "numGroupsLimit must be >= maxInitialResultHolderCapacity");
    return -1;
  }
  seg_result* res = calloc((size_t)(nsegs ? nsegs : 1), sizeof(seg_result));
  task_ctx t = {segs, nsegs, q, res, 0};
  if (nthreads < 1) nthreads = 1;
  if (nthreads > nsegs) nthreads = nsegs > 0 ? nsegs : 1;
  pthread_t* th = malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, worker, &t);
  for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
  free(th);
  for (int i = 0; i < nsegs; i++)
    if (res[i].status) {
      snprintf(msg, msg_len, "%s", res[i].msg);
      int st = res[i].status;
      for (int j = 0; j < nsegs; j++) { free(res[j].keys.b); free(res[j].koff); free(res[j].vals); free(res[j].cnts); }
      free(res);
      return st;
    }

  /* GroupByCombineOperator.processSegments merge (:113-160).  Pinot's worker threads merge their segments into one
   * ConcurrentHashMap (compute per key, :136); when the 2 x numGroupsLimit admission cap cannot bind (the segments
   * hold no more groups than it admits) the merge here runs on `nthreads` threads too, each owning the keys of one
   * hash shard -- the same merged map.  Otherwise segments are merged in order (one of the admission orders Pinot's
   * threads can produce). */
  int na = q->num_aggs;
  int64_t limit = q->combine ? (int64_t)q->num_groups_limit * 2 : INT64_MAX; /* INTER_SEGMENT_NUM_GROUPS_LIMIT_FACTOR */
  if (limit > INT32_MAX) limit = INT32_MAX;
  int64_t total_groups = 0;
  for (int s = 0; s < nsegs; s++) {
    seg_result* r = &res[s];
    out->num_docs_scanned += r->docs_scanned;
    out->num_entries_scanned_in_filter += r->in_filter;
    out->num_entries_scanned_post_filter += r->post_filter;
    out->num_total_docs += r->total_docs;
    out->holder_kind = r->holder;
    out->num_groups_limit_reached |= r->limit_reached;
    total_groups += r->ngroups;
  }
  int nshards = total_groups <= limit && total_groups >= 65536 ? nthreads : 1;
  merge_ctx mc = {res, nsegs, q, limit, nshards, NULL, 0};
  mc.shard = calloc((size_t)nshards, sizeof(merge_shard));
  if (nshards > 1) {
    pthread_t* mt = malloc(sizeof(pthread_t) * (size_t)nshards);
    for (int i = 0; i < nshards; i++) pthread_create(&mt[i], NULL, merge_worker, &mc);
    for (int i = 0; i < nshards; i++) pthread_join(mt[i], NULL);
    free(mt);
  } else {
    merge_worker(&mc);
  }
  /* the shards' maps back to back (keys are disjoint across shards) */
  int64_t ng = 0, kbytes = 0;
  for (int i = 0; i < nshards; i++) { ng += mc.shard[i].ng; kbytes += mc.shard[i].kb.n; }
  bbuf kb = {0};
  kb.b = malloc((size_t)(kbytes ? kbytes : 1));
  kb.cap = kbytes ? kbytes : 1;
  int64_t* koff = malloc(sizeof(int64_t) * (size_t)(ng + 2));
  double* vals = malloc(sizeof(double) * (size_t)(ng * na + 1));
  int64_t* cnts = malloc(sizeof(int64_t) * (size_t)(ng * na + 1));
  koff[0] = 0;
  int64_t g0 = 0;
  for (int i = 0; i < nshards; i++) {
    merge_shard* m = &mc.shard[i];
    if (m->kb.n) memcpy(kb.b + kb.n, m->kb.b, (size_t)m->kb.n);
    for (int64_t e = 0; e < m->ng; e++) koff[g0 + e + 1] = kb.n + m->koff[e + 1];
    kb.n += m->kb.n;
    if (m->ng && na) {
      memcpy(vals + g0 * na, m->vals, sizeof(double) * (size_t)(m->ng * na));
      memcpy(cnts + g0 * na, m->cnts, sizeof(int64_t) * (size_t)(m->ng * na));
    }
    g0 += m->ng;
    free(m->kb.b); free(m->koff); free(m->vals); free(m->cnts);
  }
  free(mc.shard);
  out->num_groups = ng;
  /* GroupByCombineOperator.mergeResults (:215-219): the merged map holds >= numGroupsLimit groups (PQL combine);
   * without the combine, a segment's holder reached its bound. */
  if (q->combine) out->num_groups_limit_reached = q->num_group_by > 0 && ng >= q->num_groups_limit;
  out->key_blob = kb.b;
  out->key_offsets = koff;
  out->values = malloc(sizeof(double) * (size_t)(ng * na + 1));
  out->avg_counts = malloc(sizeof(int64_t) * (size_t)(ng * na + 1));
  for (int64_t gi = 0; gi < ng; gi++)
    for (int a = 0; a < na; a++) {
      out->values[a * ng + gi] = vals[gi * na + a];
      out->avg_counts[a * ng + gi] = cnts[gi * na + a];
    }
  free(vals); free(cnts);
  for (int j = 0; j < nsegs; j++) { free(res[j].keys.b); free(res[j].koff); free(res[j].vals); free(res[j].cnts); }
  free(res);
  return 0;
}

void or_free_result(or_result* r) {
  free(r->key_blob); free(r->key_offsets); free(r->values); free(r->avg_counts);
  memset(r, 0, sizeof *r);
}

int or_filter_bitmap(const or_segment* seg, const or_query* q, uint64_t* bits, char* msg, int ml) {
  int np = q->num_predicates;
  pred_eval* evals = calloc((size_t)(np ? np : 1), sizeof(pred_eval));
  for (int i = 0; i < np; i++) {
    int st = build_pred_eval(seg, &q->predicates[i], &evals[i], msg, ml);
    if (st) { for (int j = 0; j < i; j++) pred_eval_free(&evals[j]); free(evals); return st; }
  }
  fnode* root = build_filter_tree(seg, q, evals, msg, ml);
  if (!root) { for (int j = 0; j < np; j++) pred_eval_free(&evals[j]); free(evals); return -1; }
  memset(bits, 0, sizeof(uint64_t) * (size_t)((seg->num_docs + 63) / 64));
  for (int d = 0; d < seg->num_docs; d++)
    if (node_match(root, seg, evals, q, d)) bits[d >> 6] |= 1ull << (d & 63);
  fn_free(root);
  for (int j = 0; j < np; j++) pred_eval_free(&evals[j]);
  free(evals);
  return 0;
}

int64_t or_bytes_alg(const or_segment* seg, const or_query* q, const uint64_t* match) {
  int is_filter[256] = {0}, is_other[256] = {0};
  for (int i = 0; i < q->num_predicates; i++) is_filter[q->predicates[i].column] = 1;
  for (int i = 0; i < q->num_group_by; i++) is_other[q->group_by[i]] = 1;
  for (int i = 0; i < q->num_aggs; i++) if (q->aggs[i].column >= 0) is_other[q->aggs[i].column] = 1;
  int64_t bytes = 0;
  for (int c = 0; c < seg->num_columns && c < 256; c++) {
    const or_column* col = &seg->columns[c];
    if (!is_filter[c] && !is_other[c]) continue;
    bytes += (int64_t)col->cardinality * col->entry_width; /* dictionary once per segment */
    if (is_filter[c]) { bytes += or_fwd_num_bytes(seg->num_docs, col->bits); continue; }
    int64_t nbytes = or_fwd_num_bytes(seg->num_docs, col->bits);
    int64_t nlines = (nbytes + 127) / 128;
    int64_t last_line = -1, lines = 0;
    for (int64_t w = 0; w < (seg->num_docs + 63) / 64; w++) {
      uint64_t m = match[w];
      while (m) {
        int b = __builtin_ctzll(m); m &= m - 1;
        int64_t d = w * 64 + b;
        int64_t bit0 = d * col->bits, bit1 = bit0 + col->bits - 1;
        for (int64_t l = (bit0 >> 3) / 128; l <= (bit1 >> 3) / 128; l++)
          if (l > last_line) { last_line = l; lines++; }
      }
    }
    (void)nlines;
    bytes += lines * 128;
  }
  return bytes;
}

/* ======================================================================================= synthetic data */

uint64_t or_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
uint64_t or_seed(int column_index) { return (uint64_t)(0x5EED0000u + (uint32_t)column_index) << 32; }

void or_zipf_cdf(int n, double s, double* cdf) {
  double acc = 0.0;
  for (int k = 0; k < n; k++) { acc += 1.0 / pow((double)(k + 1), s); cdf[k] = acc; }
  for (int k = 0; k < n; k++) cdf[k] /= acc;
  cdf[n - 1] = 1.0;
}
static inline double unit_double(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }
void or_double_table(int n, int column_index, double lo, double hi, double* out) {
  for (int i = 0; i < n; i++) out[i] = lo + (hi - lo) * unit_double(or_splitmix64(or_seed(column_index) ^ (uint64_t)(0xDB1E000000ull + i)));
}
static inline int zipf_rank(const double* cdf, int n, double u) {
  int lo = 0, hi = n - 1; /* first k with cdf[k] > u */
  while (lo < hi) { int mid = (lo + hi) >> 1; if (cdf[mid] > u) hi = mid; else lo = mid + 1; }
  return lo;
}
void or_gen_i64(const or_gen_spec* sp, int64_t row0, int64_t n, int64_t* out) {
  uint64_t seed = or_seed(sp->column_index);
  for (int64_t i = 0; i < n; i++) {
    uint64_t h = or_splitmix64(seed ^ (uint64_t)(row0 + i));
    if (sp->kind == OR_GEN_UNIFORM) out[i] = sp->lo + (int64_t)(h % (uint64_t)(sp->hi - sp->lo));
    else out[i] = sp->ids[zipf_rank(sp->cdf, sp->n, unit_double(h))];
  }
}
void or_gen_f64(const or_gen_spec* sp, int64_t row0, int64_t n, double* out) {
  uint64_t seed = or_seed(sp->column_index);
  for (int64_t i = 0; i < n; i++) {
    uint64_t h = or_splitmix64(seed ^ (uint64_t)(row0 + i));
    out[i] = sp->table[h % (uint64_t)sp->n];
  }
}
