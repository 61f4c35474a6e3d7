/*
 * oracle.h — CPU restatement of Apache Pinot's server-side filter -> group-by -> aggregation path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so, and only as the checker / CPU baseline.  The product (pinot_amd/libpinotgpu.so) never
 * links, loads or calls anything in this directory.
 *
 * Parity anchor: the reference is Java (kbastani/pinot 0.10.0-SNAPSHOT) and cannot be built or run in this
 * image (no JDK, no Maven cache).  Every function below restates one reference routine and cites
 * it (file:line, paths abbreviated as in SURVEY.md: seglocal/, core/, segspi/).  The restatement is pinned by:
 *   - the reference's own known-answer tests on pinot-core/src/test/resources/data/test_data-sv.avro
 *     (InnerSegmentAggregationSingleValueQueriesTest.java:52-219, InterSegment*SingleValueQueriesTest.java),
 *     decoded to tests/golden/ by tests/golden/make_golden.py;
 *   - real Pinot-written segment bytes (padding{Old,Null,Percent}.tar.gz) for the codec and dictionaries;
 *   - the bit layout spelled out in FixedBitIntReader.java (e.g. Bit9Reader :656-725).
 * Third-party arithmetic that is absent from /root/reference: fastutil 8.2.3 HashCommon.mix (published
 * algorithm, restated in or_mix32) only orders IntGroupIdMap slots; it never changes result values.
 */
#ifndef PINOT_ORACLE_H
#define PINOT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* FieldSpec.DataType subset used by dictionary-encoded SV columns. */
enum { OR_INT = 0, OR_LONG = 1, OR_FLOAT = 2, OR_DOUBLE = 3, OR_STRING = 4 };

/* ---------------- codec: seglocal/io/util/PinotDataBitSet.java, seglocal/io/reader/impl/FixedBitIntReader.java */
int or_num_bits_per_value(int max_value);                                       /* PinotDataBitSet.java:59-70 */
int32_t or_bitset_read_int(const uint8_t* buf, int64_t index, int nbits);       /* :78-100 */
void or_bitset_read_ints(const uint8_t* buf, int64_t start, int nbits, int len, int32_t* out); /* :102-136 */
void or_bitset_write_int(uint8_t* buf, int64_t index, int nbits, int32_t value); /* :138-165 */
void or_bitset_write_ints(uint8_t* buf, int64_t start, int nbits, int len, const int32_t* values); /* :167-205 */
int64_t or_fwd_num_bytes(int64_t num_values, int nbits);                        /* FixedBitSVForwardIndexWriter */
/* FixedBitSVForwardIndexReaderV2.readDictIds (seglocal/segment/index/readers/forward/...V2.java:62-96). */
void or_read_dict_ids(const uint8_t* fwd, int nbits, int num_docs, const int32_t* doc_ids, int len, int32_t* out);

/* ---------------- segment (on-disk bytes exactly as Pinot writes them) */
typedef struct {
  int32_t data_type;    /* OR_INT .. OR_STRING */
  int32_t cardinality;  /* dictionary length */
  int32_t bits;         /* bitsPerElement = getNumBitsPerValue(cardinality - 1) */
  int32_t entry_width;  /* bytes per dictionary entry: 4 / 8 / numBytesPerValue for strings */
  int32_t padding_byte; /* string dictionary padding byte (0 for segments built since 0.3) */
  int32_t is_sorted;    /* column.X.isSorted: predicates run as SortedIndexBasedFilterOperator (the forward index
                           here is always fixed-bit; the sorted docId ranges are read from it) */
  int32_t has_inverted; /* a bitmap inverted index is loaded: EQ / NOT_EQ / IN / NOT_IN run as
                           BitmapBasedFilterOperator (docIds read from the forward index) */
  const uint8_t* dict;  /* BIG_ENDIAN fixed-width sorted values (BaseImmutableDictionary.java:45-60) */
  const uint8_t* fwd;   /* MSB-first packed dictIds (FixedBitSVForwardIndexWriter.java:39-50), or for a raw column the
                           FixedByteChunkSVForwardIndexWriter bytes (PASS_THROUGH chunks) */
  int32_t raw;          /* 1: no-dictionary column (cardinality 0), values read by FixedByteChunkSVForwardIndexReader */
  int64_t fwd_len;      /* bytes of fwd (raw columns: the chunk file, whose last chunk runs to its end) */
  const uint8_t* range_index; /* `<column>.bitmap.range` bytes (NULL: none): a RANGE predicate on the unsorted column
                                 runs as RangeIndexBasedFilterOperator (FilterOperatorUtils.java:57-62) -- version 1
                                 (RangeIndexReaderImpl) or 2 (BitSlicedRangeIndexReader); other versions are skipped */
  int64_t range_index_len;
} or_column;

/* FixedByteChunkSVForwardIndexReader.getInt / getLong / getFloat / getDouble on an uncompressed (PASS_THROUGH)
 * file (BaseChunkSVForwardIndexReader.java:57-98: header, chunk offsets, raw data from rawDataStart). */
double or_raw_get_double(const or_column* c, int doc);
/* LZ4 block decompression (LZ4Decompressor / LZ4WithLengthDecompressor, seglocal/io/compression/): decoded length, or
 * -1 on malformed input / output overflow. */
int64_t or_lz4_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap);
/* Every value of a raw column's forward index (BaseChunkSVForwardIndexReader.java:56-154, PASS_THROUGH / LZ4 /
 * LZ4_LENGTH_PREFIXED chunks): INT / LONG into ival, all types as double into dval (either may be NULL).
 * 0, -1 malformed, -2 unsupported codec. */
int or_raw_decode(const or_column* c, const uint8_t* fwd, int64_t len, int num_docs, int64_t* ival, double* dval);

/* A star-tree of a segment (StarTreeV2: OffHeapStarTree + its documents; seglocal/startree/OffHeapStarTree.java:45-80,
 * seglocal/startree/v2/store/StarTreeDataSource): nodes as OffHeapStarTreeNode records, the star-tree documents'
 * dimension dictIds (the segment's dictionaries, the segment column's bitsPerElement, MSB-first) and the
 * pre-aggregated function-column pairs. */
typedef struct {
  int32_t num_nodes;
  const int32_t* nodes;           /* [num_nodes][7]: dimension id, value (-1 = ALL), start doc, end doc, aggregated doc,
                                     first child, last child (-1: leaf) */
  int32_t num_docs;               /* star-tree documents */
  int32_t num_dims;
  const int32_t* dim_columns;     /* split order: segment column of each dimension */
  const uint8_t* const* dim_fwd;  /* per dimension: packed dictIds of the star-tree documents */
  int32_t num_metrics;
  const int32_t* metric_fn;       /* per function-column pair: OR_AGG_* */
  const int32_t* metric_column;   /* -1 for COUNT(*) */
  const double* const* metric_f64;  /* SUM / MIN / MAX values, AVG sums (NULL for COUNT) */
  const int64_t* const* metric_i64; /* COUNT counts, AVG counts (NULL otherwise) */
} or_star_tree;

typedef struct {
  int32_t num_docs;
  int32_t num_columns;
  const or_column* columns;
  const or_star_tree* star_tree;  /* NULL: none (queries use_star_tree run on it when they fit, see or_query) */
} or_segment;

/* Dictionary + forward index creation, as SegmentDictionaryCreator / SegmentColumnarIndexCreator produce them
 * (seglocal/segment/creator/impl/SegmentDictionaryCreator.java, SegmentColumnarIndexCreator.java:632-635):
 * dictionary = sorted distinct values, dictId = rank, bitsPerElement = getNumBitsPerValue(card-1).
 * Numeric values come in as int64 (INT/LONG) or double (FLOAT/DOUBLE; FLOAT values must be float-representable).
 * String values come in as a blob + (n+1) offsets; entries are padded with 0 to the longest value.
 * Caller supplies dict_out (>= n * width bytes) and fwd_out (>= or_fwd_num_bytes(n, 31) bytes, zeroed).
 * Returns cardinality; *bits_out and *width_out receive bitsPerElement and entry width. */
int or_build_column_i64(int data_type, const int64_t* values, int64_t n, uint8_t* dict_out, uint8_t* fwd_out,
                        int* bits_out, int* width_out);
int or_build_column_f64(int data_type, const double* values, int64_t n, uint8_t* dict_out, uint8_t* fwd_out,
                        int* bits_out, int* width_out);
int or_build_column_str(const uint8_t* blob, const int64_t* offsets, int64_t n, uint8_t* dict_out,
                        uint8_t* fwd_out, int* bits_out, int* width_out);

/* Dictionary lookups: BaseImmutableDictionary.binarySearch (:97-230) via insertionIndexOf(String). */
int or_dict_insertion_index_of(const or_column* col, const char* literal, int* err);
double or_dict_get_double(const or_column* col, int dict_id);                   /* Dictionary.readDoubleValues */

/* ---------------- query (QueryContext subset on the path) */
enum { OR_PRED_EQ = 0, OR_PRED_NOT_EQ = 1, OR_PRED_IN = 2, OR_PRED_NOT_IN = 3, OR_PRED_RANGE = 4 };
typedef struct {
  int32_t type;
  int32_t column;
  int32_t num_values;           /* EQ/NOT_EQ: 1; IN/NOT_IN: k; RANGE: 2 = (lower, upper), "*" = unbounded */
  const char* const* values;    /* string literals, parsed per column type as PredicateUtils.getStoredValue */
  int32_t lower_inclusive;
  int32_t upper_inclusive;
} or_predicate;

enum { OR_OP_PRED = 0, OR_OP_AND = 1, OR_OP_OR = 2, OR_OP_NOT = 3 };
typedef struct {
  int32_t op;   /* PRED: arg = predicate index; AND/OR: arg = number of children popped; NOT: arg unused */
  int32_t arg;
} or_filter_op;

enum { OR_AGG_COUNT = 0, OR_AGG_SUM = 1, OR_AGG_MIN = 2, OR_AGG_MAX = 3, OR_AGG_AVG = 4 };
typedef struct {
  int32_t fn;
  int32_t column; /* -1 for COUNT(*) */
} or_agg;

typedef struct {
  int32_t num_predicates;
  const or_predicate* predicates;
  int32_t num_filter_ops;        /* postfix program; 0 = no filter (MatchAll) */
  const or_filter_op* filter;
  int32_t num_group_by;          /* 0 = aggregation-only (AggregationOperator): one group with the empty key */
  const int32_t* group_by;
  int32_t num_aggs;
  const or_agg* aggs;
  int32_t num_groups_limit;      /* InstancePlanMakerImplV2.DEFAULT_NUM_GROUPS_LIMIT = 100000 (:70) */
  int32_t max_initial_result_holder_capacity; /* DEFAULT_MAX_INITIAL_RESULT_HOLDER_CAPACITY = 10000 (:66) */
  int32_t combine;               /* 1: GroupByCombineOperator merge (PQL) across segments; 0: single segment */
  int32_t use_star_tree;         /* 1: segments with a star-tree the query fits run StarTreeFilterOperator +
                                    StarTreeGroupByExecutor (AggregationGroupByPlanNode.java:67-92) */
} or_query;

/* Holder kinds chosen by DictionaryBasedGroupKeyGenerator (:110-160). */
enum { OR_HOLDER_ARRAY = 0, OR_HOLDER_INT_MAP = 1, OR_HOLDER_LONG_MAP = 2, OR_HOLDER_ARRAY_MAP = 3 };

typedef struct {
  int64_t num_groups;
  /* Group keys, one record per group: for each group-by column, numeric -> 8 bytes (int64 for INT/LONG,
   * IEEE double bits for FLOAT/DOUBLE, little-endian), string -> uint32 length + unpadded bytes. */
  uint8_t* key_blob;
  int64_t* key_offsets;      /* num_groups + 1 */
  double* values;            /* [num_aggs][num_groups]: COUNT/SUM/MIN/MAX value, AVG sum */
  int64_t* avg_counts;       /* [num_aggs][num_groups]: AVG count (0 for other fns) */
  int64_t num_docs_scanned;
  int64_t num_entries_scanned_in_filter;   /* scan-only model, see or_execute_groupby */
  int64_t num_entries_scanned_post_filter;
  int64_t num_total_docs;
  int32_t holder_kind;       /* of the last segment processed */
  int32_t num_groups_limit_reached;
} or_result;

/* Runs the per-segment operator (AggregationGroupByOperator.getNextBlock, core/operator/query/
 * AggregationGroupByOperator.java:62-79) on every segment on `nthreads` workers (one task per segment,
 * GroupByCombineOperator.java:91-97), then merges per-segment results in segment order the way
 * GroupByCombineOperator.processSegments does (:113-160).  Returns 0, or <0 on bad query (err in msg). */
int or_execute_groupby(const or_segment* segs, int nsegs, const or_query* q, int nthreads, or_result* out,
                       char* msg, int msg_len);
void or_free_result(or_result* r);

/* Per-segment docId match bitmap (bit d of word d>>6 set iff doc d passes the filter): the FilterOperator's
 * doc set.  Used to cross-check the GPU filter stage and to compute bytes_alg. */
int or_filter_bitmap(const or_segment* seg, const or_query* q, uint64_t* bits_out, char* msg, int msg_len);

/* bytes_alg of SURVEY.md §8d for one segment: full filter-column bytes + 128-B lines of the other referenced
 * columns holding >= 1 matched doc + referenced dictionaries. */
int64_t or_bytes_alg(const or_segment* seg, const or_query* q, const uint64_t* match_bits);

/* ---------------- synthetic data: value = f(splitmix64(seed_c ^ global_row)) */
uint64_t or_splitmix64(uint64_t x);
uint64_t or_seed(int column_index);    /* (0x5EED0000 + column_index) << 32 */
/* Column generator kinds. */
enum { OR_GEN_UNIFORM = 0, OR_GEN_ZIPF = 1, OR_GEN_TABLE = 2 };
typedef struct {
  int32_t kind;
  int32_t column_index;  /* seed index */
  int64_t lo, hi;        /* UNIFORM: values in [lo, hi) */
  int32_t n;             /* ZIPF: number of ranks; TABLE: table size */
  const double* cdf;     /* ZIPF: cumulative table (or_zipf_cdf) */
  const int64_t* ids;    /* ZIPF: rank -> value */
  const double* table;   /* TABLE: values */
} or_gen_spec;
void or_zipf_cdf(int n, double s, double* cdf_out);
void or_double_table(int n, int column_index, double lo, double hi, double* out);
void or_gen_i64(const or_gen_spec* spec, int64_t row0, int64_t n, int64_t* out);
void or_gen_f64(const or_gen_spec* spec, int64_t row0, int64_t n, double* out);

#ifdef __cplusplus
}
#endif
#endif
