/*
 * pinotgpu.h — C ABI of libpinotgpu.so, the MI355X (gfx950) executor for Apache Pinot's server-side
 * filter -> group-by -> aggregation path over dictionary-encoded immutable segments.
 *
 * Plain C: pointers, sizes and status codes; no C++ or torch types cross this boundary and no C++ exception
 * escapes it.  Every call returns PGPU_OK (0) or a negative status; the message of the last failure on the
 * calling thread is available from pgpu_last_error().
 *
 * Each entry point names the reference interface it stands in for.  Citations use SURVEY.md's abbreviations:
 *   core/     = pinot-core/src/main/java/org/apache/pinot/core/
 *   seglocal/ = pinot-segment-local/src/main/java/org/apache/pinot/segment/local/
 *   segspi/   = pinot-segment-spi/src/main/java/org/apache/pinot/segment/spi/
 * The Java-side bindings a maintainer adds (JNI, and the ctypes binding used by this repo's tests) are in
 * INTEGRATION.md.
 *
 * Threading: every entry point is thread-safe, and any number of queries may run concurrently on one table
 * (Pinot runs many queries at once over the same segments, BaseCombineOperator.java:85-115).  Each plan owns a
 * per-query device arena (scratch buffers, statistics, group table) taken from the table's pool; plan creation holds
 * the table's mutex only to take its segment references and build lazily made per-segment arrays, so concurrent
 * cache-miss plans translate their predicates in parallel.  Give concurrent queries their own streams for their
 * device work to overlap (stream NULL = the table's stream: correct, but those queries' kernels run one after
 * another).  Pinned segments are immutable and reference-counted like Pinot's SegmentDataManager: unpinning a
 * segment that a live plan references frees its device memory when that plan is destroyed.  Global dictionaries
 * are snapshots: a pin that grows one never changes the ids of plans and results made before it.  Attach inverted
 * indexes and star-trees at segment load, before queries reference the segment.
 */
#ifndef PINOTGPU_H
#define PINOTGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PGPU_ABI_VERSION 3  /* 2: pgpu_query.end_time_ms, PGPU_ERR_TIMEOUT; 3: pgpu_comm, pgpu_plan_combine */

/* ---- status codes (BaseCombineOperator.java:101-107 maps failures to ProcessingException; the Java shim maps
 * these codes the same way and keeps Pinot's CPU operator for PGPU_ERR_UNSUPPORTED). */
#define PGPU_OK 0
#define PGPU_ERR_INVALID_ARGUMENT (-1)
#define PGPU_ERR_BAD_QUERY (-2)      /* literal does not convert to the column type: BadQueryRequestException
                                        (core/operator/filter/predicate/PredicateEvaluatorProvider.java:85-88) */
#define PGPU_ERR_UNSUPPORTED (-3)    /* query shape outside the GPU path (caller runs Pinot's own operator) */
#define PGPU_ERR_DEVICE (-4)         /* HIP runtime / kernel failure */
#define PGPU_ERR_OUT_OF_MEMORY (-5)
#define PGPU_ERR_NOT_FOUND (-6)      /* unknown segment handle / column */
#define PGPU_ERR_TIMEOUT (-7)        /* the query's end time passed before its device work completed: the combine's
                                        timeout (BaseCombineOperator.java:193-203 EXECUTION_TIMEOUT_ERROR for
                                        aggregation-only, GroupByCombineOperator.java:193-203 QUERY_EXECUTION_ERROR
                                        wrapping a TimeoutException for group-by); no partial result is returned */
#define PGPU_ERR_CANCELLED (-8)      /* pgpu_plan_cancel: the caller abandoned the query (BaseOperator.nextBlock's
                                        EarlyTerminationException after Future.cancel(true), BaseOperator.java:37-39,
                                        BaseCombineOperator.java:124-130); no partial result is returned */

/* FieldSpec.DataType subset of dictionary-encoded single-value columns. */
enum pgpu_data_type { PGPU_INT = 0, PGPU_LONG = 1, PGPU_FLOAT = 2, PGPU_DOUBLE = 3, PGPU_STRING = 4 };

/* Forward-index formats:
 *   PGPU_FWD_FIXED_BIT    FixedBitSVForwardIndexReaderV2 bytes (seglocal/segment/index/readers/forward/
 *                         FixedBitSVForwardIndexReaderV2.java:33-96: MSB-first big-endian bit packing, PinotDataBitSet);
 *   PGPU_FWD_SORTED_PAIRS SortedIndexReaderImpl (seglocal/segment/index/readers/sorted/SortedIndexReaderImpl.java:
 *                         37-116: BIG_ENDIAN (startDocId, endDocId) int pairs per dictId);
 *   PGPU_FWD_RAW_FIXED    a raw (no-dictionary) INT / LONG / FLOAT / DOUBLE column as FixedByteChunkSVForwardIndexWriter
 *                         writes it, versions 2 / 3, chunks PASS_THROUGH, LZ4 or LZ4_LENGTH_PREFIXED
 *                         (BaseChunkSVForwardIndexWriter.java:130-193; BaseChunkSVForwardIndexReader.java:56-154) --
 *                         cardinality 0, no dictionary; decoded once at pin into per-doc values: an aggregation
 *                         operand (SUM / MIN / MAX / AVG) and a raw-value predicate column (EQ / NOT_EQ / IN / NOT_IN /
 *                         RANGE, RangePredicateEvaluatorFactory.java:60-102,268-448).  SNAPPY / ZSTANDARD chunks:
 *                         PGPU_ERR_UNSUPPORTED. */
enum pgpu_fwd_format { PGPU_FWD_FIXED_BIT = 0, PGPU_FWD_SORTED_PAIRS = 1, PGPU_FWD_RAW_FIXED = 2 };

int pgpu_abi_version(void);
/* Process start-up / shut-down of the executor (the server's lifecycle around PlanMaker, ServerInstance.java:86-90):
 * pgpu_init brings up the HIP runtime on devices 0..n_gpus-1 (n_gpus <= 0: every visible device) so the first query
 * pays no context creation, and returns the number of devices initialised (or a negative status); pgpu_shutdown
 * waits for every initialised device's queued work.  Tables, plans and results own their memory and are released by
 * their destroy calls (segments on unpin / table destroy, as ImmutableSegmentImpl.destroy frees them). */
int pgpu_init(int n_gpus);
int pgpu_shutdown(void);
/* Copies the calling thread's last error message (NUL-terminated, truncated to len). Returns its full length. */
int pgpu_last_error(char* buf, size_t len);
int pgpu_device_count(int* count);

/* ============================================================================ tables and pinned segments */

typedef struct pgpu_table_s* pgpu_table;

/* A table owns the per-column global dictionaries: the key space shared by all of its segments, replacing the
 * by-value merge of GroupByCombineOperator (core/operator/combine/GroupByCombineOperator.java:132-151). */
int pgpu_table_create(int device, int num_columns, const char* const* column_names, const int32_t* data_types,
                      pgpu_table* out);
int pgpu_table_destroy(pgpu_table table);

/* Executor settings of a table: what a Pinot server's configuration sets.  The JNI shim maps its
 * pinot.server.query.executor.gpu.* keys (PinotConfiguration, as InstancePlanMakerImplV2 reads its
 * max.execution.threads / num.groups.limit / min.segment.group.trim.size keys, InstancePlanMakerImplV2.java:75-110)
 * onto these fields; INTEGRATION.md lists the mapping.  pgpu_config_default fills every field with the library's
 * default, which a new table starts with.  Settings apply to plans made after pgpu_table_set_config (the table's
 * compiled-plan cache is cleared); a plan already made keeps the settings it was planned with. */
typedef struct {
  int32_t struct_size;            /* sizeof(pgpu_config) as the caller compiled it: later fields keep their defaults */
  int32_t plan_cache;             /* 1 (default): a repeated query (same bytes, same segments) reuses its compiled
                                     plan; 0: every query is planned afresh (pgpu_query.options can opt out per query) */
  int32_t partitioned_group_by;   /* 1 (default): dense key spaces whose table is >= 32 MB are radix-partitioned and
                                     aggregated per partition in LDS (K8a-K8d); 0: global atomics into the table */
  int32_t hash_partitions;        /* 1 (default): key spaces past every dense table and below 2^31 are aggregated by
                                     hashed partitions (K8h, LDS hash tables); 0: the global hash table */
  int32_t hash_partition_bits;    /* most partition bits of hashed partitions, 0..14 (default 14) */
  int32_t hash_partition_lds_kb;  /* LDS of one hashed partition's table, KB, 1..128 (default 0: 20 KB-class tables) */
  int32_t lds_table_kb;           /* largest group table privatised in LDS per workgroup, KB (default 112) */
  int32_t plan_chunk_segments;    /* segments per host planning task (default 4096) */
  int32_t stream_chunks;          /* scan launches of pgpu_plan_create_execute's streamed plan (default 1) */
  int32_t compact_results;        /* 1 (default): large results cross PCIe in the compact form (presence bitmap /
                                     keys + narrowed slot words) and are decoded on first access; 0: columnar */
  int32_t star_tree_workgroups;   /* workgroups of the star-tree document scan (default 0: the library's choice) */
  double dense_selectivity;       /* estimated selectivity from which plans take the dense scan instance
                                     (default 0.25; > 1 = never) */
  double slot_weight_step;        /* chunked scans launched with no other query's scan in flight: the workgroup
                                     dispatched to CU slot s of S takes a share of tiles weighted 1 + step (S-1-s)
                                     (the SIMDs issue the oldest wave first; default 0.11; 0 = equal shares) */
} pgpu_config;
int pgpu_config_default(pgpu_config* out);
int pgpu_table_set_config(pgpu_table table, const pgpu_config* config);
int pgpu_table_get_config(pgpu_table table, pgpu_config* out);

/* One column of an ImmutableSegment as Pinot holds it in memory (PinotDataBuffer views; the JNI shim takes the
 * addresses from PinotDataBuffer.toDirectByteBuffer, segspi/memory/PinotDataBuffer.java:382). */
typedef struct {
  int32_t cardinality;        /* Dictionary.length() (segspi/index/reader/Dictionary.java:49) */
  int32_t bits_per_element;   /* column.X.bitsPerElement = PinotDataBitSet.getNumBitsPerValue(card - 1) */
  int32_t entry_width;        /* bytes per dictionary entry (numBytesPerValue) */
  int32_t padding_byte;       /* string dictionaries: segment.padding.character (0 for current segments) */
  int32_t fwd_format;         /* enum pgpu_fwd_format */
  int32_t reserved;
  const uint8_t* dict;        /* BIG_ENDIAN fixed-width sorted values (BaseImmutableDictionary.java:45-60) */
  int64_t dict_len;
  const uint8_t* fwd;         /* forward index bytes */
  int64_t fwd_len;
} pgpu_column_buffers;

typedef struct {
  int32_t num_docs;
  int32_t num_columns;        /* must equal the table's column count; entries follow the table's column order */
  const pgpu_column_buffers* columns;
} pgpu_segment_desc;

/* Pins one ImmutableSegment into HBM (the H2D copy happens here, once; ImmutableSegmentLoader.load,
 * seglocal/indexsegment/immutable/ImmutableSegmentLoader.java:67-201, is where the shim calls it). */
int pgpu_pin_segment(pgpu_table table, const pgpu_segment_desc* desc, int64_t* segment_handle);
/* Frees the device copy (ImmutableSegmentImpl.destroy, seglocal/indexsegment/immutable/ImmutableSegmentImpl.java:147). */
int pgpu_unpin_segment(pgpu_table table, int64_t segment_handle);
int pgpu_table_num_segments(pgpu_table table, int32_t* count);
int64_t pgpu_table_device_bytes(pgpu_table table);

/* Adds values to a column's global dictionary (multi-GPU: every rank merges the union of all ranks' values so
 * per-GPU group tables share one key space before the RCCL reduce).  Numeric columns read `values_i64` (INT/LONG)
 * or `values_f64` (FLOAT/DOUBLE); STRING columns read blob + offsets[n+1]. */
int pgpu_table_add_dictionary_values(pgpu_table table, int column, int64_t n, const int64_t* values_i64,
                                     const double* values_f64, const uint8_t* blob, const int64_t* offsets);
/* Global dictionary of a column (sorted, ascending); gid = index. */
int pgpu_table_dictionary_size(pgpu_table table, int column, int64_t* size);
int pgpu_table_dictionary_i64(pgpu_table table, int column, int64_t* out);       /* INT / LONG */
int pgpu_table_dictionary_f64(pgpu_table table, int column, double* out);        /* FLOAT / DOUBLE */
/* STRING: writes all values as blob + offsets (offsets has size+1 entries); blob_cap in bytes. */
int pgpu_table_dictionary_str(pgpu_table table, int column, uint8_t* blob, int64_t blob_cap, int64_t* offsets);

/* ============================================================================ single-segment readers */

/* ForwardIndexReader.readDictIds (segspi/index/reader/ForwardIndexReader.java:83; implemented by
 * FixedBitSVForwardIndexReaderV2.readDictIds :62-96): host docIds in, host dictIds out, decoded on the GPU
 * from the pinned copy by the unpack kernel (K1). */
int pgpu_read_dict_ids(pgpu_table table, int64_t segment_handle, int column, const int32_t* doc_ids, int32_t n,
                       int32_t* dict_ids_out);

/* Device-level K1: unpack n values starting at `start` from a packed MSB-first buffer already in device memory
 * into int32 (all pointers are device pointers; stream may be NULL). */
int pgpu_unpack_fixed_bit_device(const void* d_fwd, int64_t fwd_len, int32_t bits, int64_t start, int64_t n,
                                 int32_t* d_out, void* stream);

/* ============================================================================ queries */

/* Predicate types (segspi Predicate.Type subset on dictionary columns). RANGE literal pair uses "*" for
 * unbounded (RangePredicate.UNBOUNDED). Literals are strings, converted per column type exactly as
 * PredicateUtils.getStoredValue + Dictionary.insertionIndexOf do. */
enum pgpu_predicate_type { PGPU_PRED_EQ = 0, PGPU_PRED_NOT_EQ = 1, PGPU_PRED_IN = 2, PGPU_PRED_NOT_IN = 3,
                           PGPU_PRED_RANGE = 4 };
typedef struct {
  int32_t type;
  int32_t column;
  int32_t num_values;         /* EQ/NOT_EQ 1, IN/NOT_IN k, RANGE 2 (lower, upper) */
  int32_t lower_inclusive;
  const char* const* values;
  int32_t upper_inclusive;
  int32_t reserved;
} pgpu_predicate;

/* Filter tree (FilterContext AND / OR / PREDICATE, plus NOT) as a postfix program. */
enum pgpu_filter_opcode { PGPU_OP_PRED = 0, PGPU_OP_AND = 1, PGPU_OP_OR = 2, PGPU_OP_NOT = 3 };
typedef struct {
  int32_t op;   /* PRED: arg = predicate index; AND / OR: arg = number of operands popped; NOT: unused */
  int32_t arg;
} pgpu_filter_op;

/* AggregationFunctionType subset (core/query/aggregation/function/{Count,Sum,Min,Max,Avg}AggregationFunction). */
enum pgpu_agg_fn { PGPU_AGG_COUNT = 0, PGPU_AGG_SUM = 1, PGPU_AGG_MIN = 2, PGPU_AGG_MAX = 3, PGPU_AGG_AVG = 4 };
typedef struct {
  int32_t fn;
  int32_t column;   /* -1 for COUNT(*) */
} pgpu_agg;

typedef struct {
  int32_t num_predicates;
  int32_t num_filter_ops;     /* 0 = no filter (MatchAllFilterOperator) */
  const pgpu_predicate* predicates;
  const pgpu_filter_op* filter;
  int32_t num_group_by;       /* >= 1 (the group-by path) */
  int32_t num_aggs;
  const int32_t* group_by;    /* table column indices */
  const pgpu_agg* aggs;
  int32_t num_groups_limit;   /* InstancePlanMakerImplV2.DEFAULT_NUM_GROUPS_LIMIT = 100000 (:70); <= 0 = unlimited */
  int32_t options;            /* PGPU_OPT_* bits */
  int64_t end_time_ms;        /* QueryContext.getEndTimeMs(): absolute deadline in ms since the Unix epoch (the
                                 broker's arrival time + timeoutMs); 0 = none.  Checked before launch and on the
                                 device (the persistent scans stop taking tiles past it): PGPU_ERR_TIMEOUT.  Not part
                                 of the compiled-plan cache key. */
} pgpu_query;

/* Query options: debug option useStarTree=false (StarTreeUtils.isStarTreeDisabled, core/startree/StarTreeUtils.java:
 * 51-59) keeps the scan path on segments that carry a star-tree. */
#define PGPU_OPT_NO_STAR_TREE 1
/* Group-by combine of SQL mode (queryOptions groupByMode=sql: GroupByOrderByCombineOperator) instead of the default
 * PQL GroupByCombineOperator: no inter-segment cap of 2 x numGroupsLimit (GroupByCombineOperator.java:61,78-80,138)
 * and no numGroupsLimitReached flag (GroupByOrderByCombineOperator.java:246).  Either way a segment whose group-key
 * space exceeds numGroupsLimit keeps its first numGroupsLimit groups in first-seen docId order
 * (DictionaryBasedGroupKeyGenerator.java:1101-1113), as Pinot's map-based holders do. */
#define PGPU_OPT_SQL_GROUP_BY 2
/* Compile the plan afresh instead of reusing the table's cached compilation of the same query over the same
 * segments (the cache is dropped whenever pinned state changes; PGPU_PLAN_CACHE=0 disables it process-wide). */
#define PGPU_OPT_NO_PLAN_CACHE 4
/* Record HIP timing events around the execution's kernels for pgpu_plan_timing.  Off by default: each event is a
 * marker packet between two dependent dispatches of the stream (about 10 us per query of gaps at 125 segments,
 * measured), so a serving query carries none.  Not part of the plan-cache key. */
#define PGPU_OPT_TIMING 8

/* A query compiled against a list of pinned segments (InstancePlanMakerImplV2.makeInstancePlan +
 * per-segment AggregationGroupByPlanNode: predicate evaluators per segment, group-key layout, accumulators). */
typedef struct pgpu_plan_s* pgpu_plan;
typedef struct pgpu_result_s* pgpu_result;

int pgpu_plan_create(pgpu_table table, const int64_t* segment_handles, int32_t num_segments, const pgpu_query* q,
                     pgpu_plan* out);
int pgpu_plan_destroy(pgpu_plan plan);

/* Dense group table layout of a plan: num_slots rows of num_keys 8-byte words (row s holds accumulator s of
 * every group key; row 0 is the COUNT row).  slot_kinds[s] (enum pgpu_slot_kind) gives the element type and the
 * RCCL reduce op that merges two ranks' tables: COUNT/SUM_I64 -> int64 sum, SUM_F64 -> float64 sum,
 * MIN_KEY -> int64 min, MAX_KEY -> int64 max.  num_keys = 0 when the plan uses the hash table (high cardinality). */
enum pgpu_slot_kind { PGPU_SLOT_COUNT = 0, PGPU_SLOT_SUM_I64 = 1, PGPU_SLOT_SUM_F64 = 2, PGPU_SLOT_MIN_KEY = 3,
                      PGPU_SLOT_MAX_KEY = 4 };
int pgpu_plan_layout(pgpu_plan plan, int32_t* num_slots, int64_t* num_keys, int32_t* slot_kinds /* >= 32 */);

/* Cancels the plan's query from any thread (the broker abandoned it; Pinot's BaseCombineOperator cancels the
 * segment tasks' futures, whose operators stop at the next block, BaseOperator.java:37-39).  A finalize waiting for
 * the plan's device work -- or any later one -- returns PGPU_ERR_CANCELLED at once; launches the plan has not
 * issued yet are not issued, and the device work already queued runs out while the plan's scratch stays out of the
 * pool until it has (as for a timeout).  The table and its other queries are unaffected.  Idempotent. */
int pgpu_plan_cancel(pgpu_plan plan);

/* Diagnostics: how the plan's leaves run in the kernels, as (segment, leaf) pairs of the scanned segments per kernel
 * leaf kind (counts[9]: NONE, ALL, RANGE, SET, DOCRANGE, BITMAP (a docId bitmap materialised per query),
 * RAW_RANGE, RAW_IN, BITDIR (inverted-index containers read in place)). */
int pgpu_plan_leaf_kinds(pgpu_plan plan, int64_t* counts);

/* Diagnostics: the group-by path the plan's scan takes (a numGroupsLimit plan: its first part's).  LDS: tables
 * privatised per workgroup in LDS; GLOBAL: a dense table with global atomics; HASH: the global open-addressing hash
 * table (sparse key spaces); PARTITIONED: radix-partitioned dense keys aggregated per partition in LDS; HASH_PARTITIONED:
 * hash-partitioned sparse keys aggregated per partition in LDS hash tables. */
enum pgpu_group_path { PGPU_PATH_LDS = 0, PGPU_PATH_GLOBAL = 1, PGPU_PATH_HASH = 2, PGPU_PATH_PARTITIONED = 3,
                       PGPU_PATH_HASH_PARTITIONED = 4 };
int pgpu_plan_group_path(pgpu_plan plan, int32_t* path);

/* Runs the plan on `stream` (hipStream_t; NULL = the table's stream): predicate translation results are
 * uploaded, the fused filter/group/aggregate kernel runs over every segment, and the dense group table is
 * written to d_table (device pointer, num_slots * num_keys * 8 bytes, caller-owned; may be NULL to use an
 * internal buffer).  Asynchronous: nothing is copied back.  Replaces the per-segment operator loop
 * (AggregationGroupByOperator.getNextBlock, core/operator/query/AggregationGroupByOperator.java:62-79) and the
 * combine (GroupByCombineOperator.processSegments, :113-160) for the segments of the plan. */
int pgpu_plan_execute(pgpu_plan plan, void* stream, void* d_table);

/* Compacts the (possibly RCCL-reduced) dense group table into a result: groups with COUNT > 0, their global
 * dictionary ids and finished aggregation values.  Synchronises `stream`. */
int pgpu_plan_finalize(pgpu_plan plan, void* stream, const void* d_table, pgpu_result* out);

/* Finalize of one key-range shard of a dense group table: d_table_shard is [num_slots][key_count] words holding
 * the composite keys [key_begin, key_begin + key_count) -- a rank's part after a reduce-scatter of the per-GPU
 * tables (the multi-GPU combine of large key spaces; every rank then returns its own disjoint groups, as Pinot
 * servers return partial tables).  PGPU_ERR_UNSUPPORTED for hash-mode tables and for queries whose
 * numGroupsLimit is below the key space (those finalize the whole table). */
int pgpu_plan_finalize_range(pgpu_plan plan, void* stream, const void* d_table_shard, int64_t key_begin,
                             int64_t key_count, pgpu_result* out);

/* ---- cross-GPU combine of hash-mode tables (key spaces past 2^26): a hash-partitioned all-to-all instead of the
 * element-wise merge of dense tables.  Replaces GroupByOrderByCombineOperator's IndexedTable.upsert loop
 * (core/operator/combine/GroupByOrderByCombineOperator.java:170-181) across GPUs: every rank splits its executed
 * table's groups by owner rank (a hash of the global composite key, the same on every rank), the records travel over
 * RCCL (all_to_all), and each owner merges what it receives into a fresh table and finalizes its own disjoint groups.
 * A record is 1 + num_slots int64 words: the composite key, then the slot words.  `kinds` (num_slots entries, or
 * NULL = the plan's own) are the kinds every rank agreed on: an int64 SUM may travel as float64 when another rank's
 * sum of that slot is float64.  Plans with ARRAY_MAP key stages (rank-local keys) and numGroupsLimit plans exchange
 * their finalized result rows instead (pgpu_result_exchange_rows). */
/* Per-owner group counts of the executed table (counts[nparts], nparts <= 64); waits for the plan's work. */
int pgpu_plan_exchange_counts(pgpu_plan plan, void* stream, int32_t nparts, int64_t* counts);
/* The records, grouped by owner in rank order, into d_out (device, cap records). */
int pgpu_plan_exchange_export(pgpu_plan plan, void* stream, int32_t nparts, const int32_t* kinds, void* d_out,
                              int64_t cap);
/* Replaces the plan's table by the merge of n received records (device); pgpu_plan_finalize then returns them. */
int pgpu_plan_exchange_merge(pgpu_plan plan, void* stream, const int32_t* kinds, const void* d_records, int64_t n);

/* ---- communicator and the one-call cross-GPU combine (what a Pinot server calls instead of the combine merge when
 * its segments are spread over the GPUs of a node; GroupByCombineOperator.java:113-160 /
 * GroupByOrderByCombineOperator.java:170-181).  One process (or thread) per GPU; every rank issues the same
 * combine calls in the same order, as with any RCCL communicator.
 *   PGPU_COMM_RCCL  RCCL over xGMI, one rank per GPU; collectives run on the caller's stream.  librccl.so.1 is opened
 *                   on first use (the copy already in the process if there is one).
 *   PGPU_COMM_HOST  processes of one machine exchanging through /dev/shm: the same combine with several ranks on one
 *                   GPU (RCCL refuses two ranks per device).  Synchronous, staged through host memory; for
 *                   rehearsals and tests, never the measured path.
 * The unique id (PGPU_COMM_ID_BYTES) is made by one rank and handed to the others out of band (the JVM's own
 * cluster channel, torch's TCPStore, ...), as ncclUniqueId is. */
typedef struct pgpu_comm_s* pgpu_comm;
#define PGPU_COMM_RCCL 0
#define PGPU_COMM_HOST 1
#define PGPU_COMM_ID_BYTES 128
int pgpu_comm_unique_id(int32_t kind, void* id /* PGPU_COMM_ID_BYTES */);
int pgpu_comm_create(int32_t kind, const void* id, int32_t nranks, int32_t rank, int32_t device, pgpu_comm* out);
/* Drops the handle; the communicator goes with the last plan combined on it (pgpu_plan_finalize / _destroy). */
int pgpu_comm_destroy(pgpu_comm comm);
int pgpu_comm_rank(pgpu_comm comm, int32_t* rank, int32_t* nranks);
/* Host memory, blocking: recv[nranks * bytes] = every rank's `bytes` bytes in rank order (dictionary unions, the
 * mode agreement, timing barriers -- the small control exchanges of a multi-GPU query). */
int pgpu_comm_allgather(pgpu_comm comm, const void* send, int64_t bytes, void* recv);
/* Waits on peers -- the host exchanges above and in the combine, and a combined plan's finalize waiting for its
 * stream-ordered collectives -- end with PGPU_ERR_TIMEOUT after timeout_ms (<= 0: no limit of the communicator's
 * own; default 600 000), or earlier at the query's end_time_ms / pgpu_plan_cancel.  An expired wait aborts the
 * communicator (RCCL: ncclCommAbort, so collectives a peer never joined stop waiting on the device); every later call
 * on it fails with PGPU_ERR_DEVICE and the caller creates a new one (BaseCombineOperator's timeout,
 * BaseCombineOperator.java:193-203: the combine always ends by the query deadline). */
int pgpu_comm_set_timeout(pgpu_comm comm, int64_t timeout_ms);
/* Gives the communicator up from any thread (a server shutting a query down); see pgpu_comm_set_timeout. */
int pgpu_comm_abort(pgpu_comm comm);
/* *aborted = 1 once the communicator was given up (a wait on peers expired, or pgpu_comm_abort): every collective on
 * it fails with PGPU_ERR_DEVICE until pgpu_comm_recreate. */
int pgpu_comm_status(pgpu_comm comm, int32_t* aborted);
/* Collective over the handle's ranks: a fresh communicator of the same transport, ranks and device from a new id
 * (made by one rank with pgpu_comm_unique_id and handed to the others out of band, as for pgpu_comm_create -- the
 * aborted one cannot carry it), replacing the handle's; the timeout carries over.  The recovery after one rank's
 * failure aborted the communicator (BaseCombineOperator.java:101-107, 193-203: a failed or timed-out combine fails
 * that query only, the server keeps serving): every rank calls it, then the next query combines as before.  Plans
 * combined on the old communicator keep it alive until they are finalized or destroyed.  No other call may use the
 * handle while it runs. */
int pgpu_comm_recreate(pgpu_comm comm, const void* id);

/* How the ranks' partial results of one query merge. */
#define PGPU_COMBINE_LOCAL 0          /* one rank: nothing to merge */
#define PGPU_COMBINE_ALL_REDUCE 1     /* dense tables, element-wise, every rank ends with the merged table */
#define PGPU_COMBINE_REDUCE_SCATTER 2 /* dense tables >= shard_bytes: rank r ends with keys [r*chunk, (r+1)*chunk) */
#define PGPU_COMBINE_HASH 3           /* hash-mode tables: groups hashed to an owner rank, all-to-all, owner merges */
#define PGPU_COMBINE_ROWS 4           /* numGroupsLimit plans / ARRAY_MAP key stages: finalized rows, by owner */
/* Collective: the mode every rank agrees on for this query (a plan, executed or not, of the query over the rank's
 * segments), and in kinds[num_slots] the slot kinds the merge runs in (an int64 SUM travels as float64 when another
 * rank's sum of the slot is float64).  Modes that differ between ranks fall back to ROWS, which merges any plan
 * kind.  PGPU_ERR_INVALID_ARGUMENT when the ranks' group-by dictionaries differ (pgpu_table_add_dictionary_values
 * with the union first).  The caller may reuse the answer for every later query of the same shape. */
int pgpu_plan_combine_mode(pgpu_plan plan, pgpu_comm comm, int64_t shard_bytes, int32_t* mode, int32_t* kinds);
/* Collective, ordered on `stream`: merges the executed plan's table (d_table as given to execute, NULL = the plan's
 * own) with the other ranks' in `mode` (ALL_REDUCE, REDUCE_SCATTER or HASH).  For REDUCE_SCATTER, d_shard (NULL = the
 * plan's scratch) receives [num_slots][key_count] words, key_begin / key_count say which keys; they are 0 / num_keys
 * otherwise.  pgpu_plan_finalize(plan, stream, d_table) then returns this rank's share of the merged groups (all of
 * them for ALL_REDUCE; disjoint shares otherwise). */
int pgpu_plan_combine(pgpu_plan plan, pgpu_comm comm, void* stream, void* d_table, int32_t mode, const int32_t* kinds,
                      void* d_shard, int64_t* key_begin, int64_t* key_count);
/* Collective, ROWS mode: the finalized result's rows split by owner, exchanged, merged by the owner as the broker
 * merges server responses.  *out = this rank's disjoint share. */
int pgpu_result_combine_rows(pgpu_result r, pgpu_comm comm, pgpu_result* out);

/* One-call form: plan + execute + finalize (the whole per-server query path). */
int pgpu_execute_groupby(pgpu_table table, const int64_t* segment_handles, int32_t num_segments, const pgpu_query* q,
                         void* stream, pgpu_result* out);

/* Plan + execute in one call, streamed: the segment list is planned in equal chunks and each chunk's scan is
 * launched as soon as it is planned, so the GPU scans while the host still translates predicates for the next
 * chunk (one launch per chunk; plans with star-tree segments, partitioned or staged scans run as one launch).
 * The plan is returned executed: finalize (or merge across GPUs, then finalize) as after pgpu_plan_execute. */
int pgpu_plan_create_execute(pgpu_table table, const int64_t* segment_handles, int32_t num_segments,
                             const pgpu_query* q, void* stream, void* d_table, pgpu_plan* out);

/* Timing of the last execution of this plan (HIP events on the execution stream; the query carried PGPU_OPT_TIMING,
 * else PGPU_ERR_INVALID_ARGUMENT), microseconds:
 * [0] whole execute, [1] the scan kernel launches (summed), [2] number of scan launches, [3] the star-tree kernels
 * (traversal + pre-aggregated document scan; 0 without star-tree segments).  out holds 4 doubles. */
int pgpu_plan_timing(pgpu_plan plan, double* out4);

/* Star-tree work of the last execution (after finalize): [0] segments answered from their star-tree, [1] their
 * tree nodes (28 bytes each, OffHeapStarTreeNode), [2] star-tree documents the residual scan read. */
int pgpu_plan_star_work(pgpu_plan plan, int64_t* out3);
/* Bytes of the star-tree metric arrays the last execution's document scan read (after finalize): the 64-byte
 * sectors holding at least one matched document, summed over the arrays read; -1 where finalize did not read the
 * counter back (tables past 512 KB).  The star path's line-granular bytes model (bench.py). */
int pgpu_plan_star_metric_bytes(pgpu_plan plan, int64_t* bytes);

/* Per plan segment (plan order): 1 if the segment is scanned, 0 if its filter folds to always-false against the
 * segment's dictionaries (EmptyFilterOperator, core/plan/FilterPlanNode.java:146-176).  out holds num_segments. */
int pgpu_plan_scanned_segments(pgpu_plan plan, uint8_t* out);

/* numEntriesScannedInFilter of one segment (ExecutionStatistics, AndDocIdSet.getNumEntriesScannedInFilter,
 * core/operator/docidsets/AndDocIdSet.java:148-155) from the doc sets of its predicates: `filter` is the query's
 * postfix program; leaf_types[i] is predicate i's leaf operator in this segment (enum pgpu_leaf_type, the outcome
 * of FilterOperatorUtils.getLeafFilterOperator, core/operator/filter/FilterOperatorUtils.java:42-82) and
 * leaf_masks[i] its matching docs (bit d % 32 of word d / 32; may be NULL for EMPTY / ALL leaves).  Pinot's
 * iterators (AndDocIdSet / OrDocIdSet merging, SVScanDocIdIterator.applyAnd, AndDocIdIterator leap-frog,
 * OrDocIdIterator) are replayed over the sets.  The plans compute the same statistic on the device; this entry is
 * the host form (a caller holding the doc sets, tests).  PGPU_LEAF_RANGE_INDEX (RangeIndexBasedFilterOperator) is an
 * index-based leaf ranked after the bitmap leaves; the entries of its own partial-match scan are not included (the
 * caller adds them: pgpu_range_index_partial_entries). */
enum pgpu_leaf_type { PGPU_LEAF_EMPTY = 0, PGPU_LEAF_MATCH_ALL = 1, PGPU_LEAF_SCAN = 2, PGPU_LEAF_SORTED = 3,
                      PGPU_LEAF_BITMAP = 4, PGPU_LEAF_RANGE_INDEX = 5 };
int pgpu_filter_entries_scanned(const pgpu_filter_op* filter, int32_t num_filter_ops, const int32_t* leaf_types,
                                const uint32_t* const* leaf_masks, int32_t num_leaves, int32_t num_docs,
                                int64_t* out);

/* ---- after the combine: server trim, server response, broker reduce (the step after the device path) */
/* ORDER BY expression over the result: a group-by column (index = its position in the GROUP BY) or an aggregation
 * (index = its position in the query; compared by its final result, as TableResizer's extractors do). */
enum pgpu_order_kind { PGPU_ORDER_GROUP_BY = 0, PGPU_ORDER_AGGREGATION = 1 };
typedef struct {
  int32_t kind;
  int32_t index;
  int32_t ascending;
} pgpu_order_by;
/* SQL-mode query options of the combine (QueryContext / InstancePlanMakerImplV2.java:64-84). */
typedef struct {
  int32_t num_order_by;
  const pgpu_order_by* order_by;
  int32_t limit;                       /* LIMIT (SQL default 10) */
  int32_t min_server_group_trim_size;  /* min.server.group.trim.size (default 5000); <= 0 disables server trim */
  int32_t group_trim_threshold;        /* groupby.trim.threshold (default 1000000) */
  int32_t num_select;                  /* broker reduce: the SELECT list in order (kind / index as for ORDER BY; */
  const pgpu_order_by* select;         /* ascending unused); 0 = every group-by column, then every aggregation */
} pgpu_sql_trim;

/* The server's SQL-mode combined table (GroupByOrderByCombineOperator.java:82-97 + IndexedTable.finish,
 * core/data/table/IndexedTable.java:62-89): with ORDER BY the top max(limit * 5, minServerGroupTrimSize) groups in
 * ORDER BY order; without it `limit` groups (Pinot keeps the first keys its threads insert -- thread-order
 * dependent; here the smallest composite keys); trim disabled: every group (sorted if ORDER BY).  Ties order by
 * composite key.  Pinot resizes lossily past groupby.trim.threshold groups; the device combine is exact, so the
 * result is the exact top records.  `out` is a new result (destroy both). */
int pgpu_result_trim_sql(pgpu_result r, const pgpu_sql_trim* spec, pgpu_result* out);

/* PQL-mode trim (AggregationGroupByTrimmingService.trimIntermediateResultsMap, :54-120): per aggregation the rows of
 * its top max(limit * 5, 5000) groups (MIN: smallest values, the others largest; by final result), applied only past
 * 4 x that many groups; final_results != 0 gives the broker's trimFinalResults (:126-150): the top `limit`.
 * rows is [num_aggs][cap] (may be NULL to get counts[num_aggs] only). */
int pgpu_result_trim_pql(pgpu_result r, int32_t limit, int32_t final_results, int64_t* rows, int64_t cap,
                         int64_t* counts);

/* Server response of a SQL-mode group-by (IntermediateResultsBlock.getResultDataTable, core/operator/blocks/
 * IntermediateResultsBlock.java:329-345; DataTableBuilder.java:55-103; DataTableImplV3.toBytes :183-290): DataTable V3
 * bytes with the group-by columns and the aggregations' intermediate results (COUNT LONG, SUM / MIN / MAX DOUBLE,
 * AVG an AvgPair OBJECT) of every row of `r`, and the block's execution statistics as metadata.  `table` supplies
 * the group keys' values and column names.  out == NULL: *len = the size needed. */
int pgpu_result_datatable(pgpu_result r, pgpu_table table, void* out, int64_t cap, int64_t* len);

/* Broker reduce of SQL-mode group-by responses (GroupByDataTableReducer.java:290-330): the servers' DataTable V3
 * bytes merged by key (AggregationFunction.merge), final results, ORDER BY (ties by key), LIMIT, and summed
 * statistics, written as the BrokerResponseNative JSON (resultTable + statistics) into json (NUL-terminated;
 * json == NULL: *len = the length needed without the NUL). */
int pgpu_broker_reduce_sql(const void* const* tables, const int64_t* lens, int32_t num_tables,
                           const pgpu_sql_trim* spec, char* json, int64_t cap, int64_t* len);

/* ---- results: AggregationGroupByResult (core/query/aggregation/groupby/AggregationGroupByResult.java:31-81) */
int pgpu_result_num_groups(pgpu_result r, int64_t* n);
/* The table-global dictionary that group-by column `key`'s ids index, as the result's plan saw it: a pin that grows
 * the table's dictionary while the query runs does not re-label this result (GroupKeyGenerator.getKeys reads the
 * segment dictionaries the operator was built on).  *snapshot_id identifies the snapshot (callers cache the values
 * by it); *size its entries.  Values as for pgpu_table_dictionary_{i64,f64,str}. */
int pgpu_result_key_dictionary(pgpu_result r, int key, uint64_t* snapshot_id, int64_t* size);
int pgpu_result_key_dictionary_i64(pgpu_result r, int key, int64_t* out);
int pgpu_result_key_dictionary_f64(pgpu_result r, int key, double* out);
int pgpu_result_key_dictionary_str(pgpu_result r, int key, uint8_t* blob, int64_t blob_cap, int64_t* offsets);
/* [n][num_group_by] global dictionary ids, in the result's group order: ascending composite key for dense tables
 * (Pinot's ARRAY / INT_MAP holders) and hash-mode results below 4096 groups; larger hash-mode results (the LONG_MAP
 * holder, whose iterator runs in fastutil hash order) come in partition order, which may differ between runs.  The
 * trims (pgpu_result_trim_sql / _trim_pql) compare composite keys themselves, so their output never depends on it. */
int pgpu_result_group_ids(pgpu_result r, int32_t* out);
/* Column `key` of the above ([n] dictIds of group-by column `key`): a plain copy, the layout the result holds. */
int pgpu_result_group_ids_column(pgpu_result r, int key, int32_t* out);
/* Zero-copy views valid until pgpu_result_destroy (a JNI caller wraps them in direct ByteBuffers):
 * the [n] dictIds of group-by column `key`, and the [n] accumulator words of aggregation `agg` (agg = -1: the
 * COUNT words, i.e. AvgPair.count) with their form: 0 = exact int64, 1 = IEEE double bits, 2 = order-preserving
 * int64 key of a double (MIN/MAX over FLOAT/DOUBLE; pgpu_result_values converts it). */
int pgpu_result_group_ids_view(pgpu_result r, int key, const int32_t** out);
int pgpu_result_words_view(pgpu_result r, int agg, const uint64_t** out, int32_t* form);
/* Per aggregation i (query order): value per group as Pinot's intermediate result holds it (double) — COUNT,
 * SUM, MIN, MAX, and AVG's AvgPair.sum; AVG's AvgPair.count via pgpu_result_avg_counts. */
int pgpu_result_values(pgpu_result r, int agg, double* out);
int pgpu_result_avg_counts(pgpu_result r, int agg, int64_t* out);
/* Exact integer accumulators where the aggregation is integer-valued (COUNT, AVG count, SUM over INT/LONG):
 * returns PGPU_ERR_INVALID_ARGUMENT for floating-point sums. */
int pgpu_result_values_i64(pgpu_result r, int agg, int64_t* out);
/* ExecutionStatistics (core/operator/ExecutionStatistics.java:42): numDocsScanned, numEntriesScannedInFilter,
 * numEntriesScannedPostFilter, numTotalDocs, plus [4] numSegmentsProcessed, [5] numSegmentsMatched. */
int pgpu_result_stats(pgpu_result r, int64_t* out6);
/* numGroupsLimitReached (GroupByCombineOperator.java:215-219, PQL mode): 1 when the combined groups reach
 * numGroupsLimit. */
int pgpu_result_groups_limit_reached(pgpu_result r, int32_t* out);
/* Accumulator slots of a result (num_slots, and kinds[num_slots], enum pgpu_slot_kind; slot 0 = COUNT). */
int pgpu_result_slot_kinds(pgpu_result r, int32_t* num_slots, int32_t* kinds);
/* Cross-rank merge of finalized results (any plan kind; each GPU as one Pinot server): the result's rows as int64
 * records [num_keys dictIds, num_slots words] grouped by owner rank (a hash of the dictIds), into rows (n records),
 * counts[nparts] per owner; `kinds` as for pgpu_plan_exchange_export.  The ranks' dictionaries must agree (union). */
int pgpu_result_exchange_rows(pgpu_result r, int32_t nparts, const int32_t* kinds, int64_t* rows, int64_t* counts);
/* The owner's merge of n received records (GroupByDataTableReducer's merge across servers, AggregationFunction.merge)
 * into a new result in ascending key order, with tmpl's aggregations, dictionaries and statistics. */
int pgpu_result_merge_rows(pgpu_result tmpl, const int64_t* rows, int64_t n, const int32_t* kinds, pgpu_result* out);
int pgpu_result_destroy(pgpu_result r);
/* The same as pgpu_result_destroy (the name SURVEY.md §8b lists). */
int pgpu_free_result(pgpu_result r);

/* Docid match bitmap of one segment's filter (the FilterOperator's doc set, K2): bit d of 64-bit word d/64.
 * out_words must hold ceil(num_docs / 64) words. */
int pgpu_filter_bitmap(pgpu_table table, int64_t segment_handle, const pgpu_query* q, uint64_t* out_words);

/* ============================================================================ star-tree index */

/* A star-tree of one segment (StarTreeV2: seglocal/startree/OffHeapStarTree.java:38-80 + the star-tree's own
 * documents).  Dimension / metric columns are indexes into the segment's (= the table's) columns.
 *   nodes      : num_nodes records of 7 little-endian int32 {dimensionId, dimensionValue, startDocId, endDocId,
 *                aggregatedDocId, firstChildId, lastChildId} in BFS order (OffHeapStarTreeNode.java:28-64; the
 *                node array of the star-tree file, after its header);
 *   dim_fwd[d] : the star-tree documents' dictIds of dimension d, BIG_ENDIAN fixed-bit with the segment column's
 *                bitsPerElement (StarTreeLoaderUtils.java:73-92); STAR = dictId 0 (StarTreeV2Constants.java:38);
 *   metrics    : the function-column pairs (AggregationFunctionColumnPair, segspi/index/startree/
 *                AggregationFunctionColumnPair.java:25-50); COUNT's column is -1;
 *   metric_f64 : per pair, the pre-aggregated double per star-tree document (SUM / MIN / MAX, AVG's sum), NULL for
 *                COUNT — the values of the PASS_THROUGH raw chunk column "fn__col" (BaseSingleTreeBuilder.java:
 *                471-475), decoded by the caller;
 *   metric_i64 : per pair, COUNT's long (and AVG's count) per star-tree document, NULL otherwise. */
typedef struct {
  int32_t num_dims;
  int32_t num_metrics;
  int32_t num_nodes;
  int32_t num_docs;
  const int32_t* dim_columns;
  const uint8_t* nodes;
  const uint8_t* const* dim_fwd;
  const int64_t* dim_fwd_len;
  const pgpu_agg* metrics;
  const double* const* metric_f64;
  const int64_t* const* metric_i64;
} pgpu_startree_desc;

/* Pins a star-tree for a pinned segment (StarTreeIndexContainer at ImmutableSegmentLoader.java:198-201).  Queries
 * that fit it (StarTreeUtils.isFitForStarTree, core/startree/StarTreeUtils.java:151-176) then traverse it on the
 * GPU (StarTreeFilterOperator, core/startree/operator/StarTreeFilterOperator.java:234-338) and aggregate the
 * pre-aggregated documents (StarTreeGroupByExecutor, core/startree/executor/StarTreeGroupByExecutor.java:60-71). */
int pgpu_attach_startree(pgpu_table table, int64_t segment_handle, const pgpu_startree_desc* desc);

/* Pins the bitmap inverted index of one column of a pinned segment: `bytes` is the `<column>.bitmap.inv` file
 * (v1) or the column's `inverted_index` buffer of columns.psf (v3) verbatim -- (cardinality + 1) big-endian int32
 * bitmap offsets, then one portable-format RoaringBitmap per dictId (BitmapInvertedIndexWriter /
 * BitmapInvertedIndexReader, seglocal/segment/index/readers/BitmapInvertedIndexReader.java:40-70; the reader the
 * DefaultIndexReaderProvider hands to the DataSource).  From then on EQ / NOT_EQ / IN / NOT_IN predicates on an
 * unsorted column of that segment are BitmapBasedFilterOperator leaves (FilterOperatorUtils.java:72-79): the
 * matching dictIds' containers are ORed into a docId bitmap on the device per query, and the leaf scans no
 * forward-index entries.  Malformed bitmaps (bad cookie, overruns, docIds >= numDocs) return
 * PGPU_ERR_INVALID_ARGUMENT.  Attach at segment load, before queries reference the segment (as Pinot builds its
 * DataSource readers): re-attaching replaces the column's index and must not race plan creation on that segment;
 * plans created before a re-attach (or an unpin) keep the index they were planned on alive until destroyed. */
int pgpu_attach_inverted_index(pgpu_table table, int64_t segment_handle, int32_t column, const void* bytes,
                               int64_t num_bytes);
/* The same file checked on the host without a device or a table (a loader can reject a bad index before it pins
 * the segment): the offsets and every Roaring bitmap are validated exactly as pgpu_attach_inverted_index does for a
 * column of `cardinality` values in a segment of num_docs documents; *total_docs (may be NULL) = the summed bitmap
 * cardinalities (num_docs for a single-value column's complete index). */
int pgpu_inverted_index_check(const void* bytes, int64_t num_bytes, int32_t cardinality, int32_t num_docs,
                              int64_t* total_docs);

/* A range index (`<column>.bitmap.range`, DefaultIndexReaderProvider.newRangeIndexReader,
 * seglocal/segment/index/readers/DefaultIndexReaderProvider.java:128-139) of a dictionary-encoded column of a pinned
 * segment.  A RANGE predicate on the column (unless it is sorted) then runs as RangeIndexBasedFilterOperator
 * (FilterOperatorUtils.java:57-62): an index-based leaf, ordered after the bitmap leaves in an AND (:143-178), whose
 * docs are exactly the predicate's matches (read here from the forward index) and whose numEntriesScannedInFilter is
 * its partial-match scan (RangeIndexBasedFilterOperator.java:110-126):
 *   version 1 (RangeIndexCreator / RangeIndexReaderImpl): header (version, value type "INT", range count, the ranges'
 *             first dictIds + the last range's end, bitmap offsets) and one Roaring bitmap per range, all read and
 *             validated; the partial matches are the first and last ranges the predicate touches
 *             (RangeIndexReaderImpl.java:198-264);
 *   version 2 (BitSlicedRangeIndexCreator / BitSlicedRangeIndexReader): exact, no partial matches (0 entries); only
 *             the header is read.
 * Another version is skipped as Pinot skips it (no range index, PGPU_OK); a malformed version-1 file fails with
 * PGPU_ERR_INVALID_ARGUMENT; raw (no-dictionary) columns: PGPU_ERR_UNSUPPORTED.  Re-attaching replaces the index;
 * num_bytes = 0 detaches it.  Plans created before keep what they planned with. */
int pgpu_attach_range_index(pgpu_table table, int64_t segment_handle, int32_t column, const void* bytes,
                            int64_t num_bytes);
/* Host check of a range index file without a table: *version (0 = not a range index Pinot loads), *num_ranges and
 * the documents of its ranges (total_docs, the column's docs for a complete index). */
int pgpu_range_index_check(const void* bytes, int64_t num_bytes, int32_t cardinality, int32_t num_docs,
                           int32_t* version, int32_t* num_ranges, int64_t* total_docs);
/* numEntriesScannedInFilter of RangeIndexBasedFilterOperator for the dictId range [lo, hi] (inclusive) over a range
 * index file: the documents of its partial-match bitmap (0 for version 2). */
int pgpu_range_index_partial_entries(const void* bytes, int64_t num_bytes, int32_t cardinality, int32_t num_docs,
                                     int32_t lo, int32_t hi, int64_t* entries);

/* Host-side reader of a raw forward index (PGPU_FWD_RAW_FIXED bytes; FixedByteChunkSVForwardIndexReader.readValuesSV
 * over every chunk, LZ4 chunks decompressed as LZ4Decompressor / LZ4WithLengthDecompressor do): num_docs values of a
 * column of `data_type` -- INT / LONG into out_i64, every type as double into out_f64 (either may be NULL).  The
 * decoder pgpu_pin_segment uses; pure host code. */
int pgpu_raw_forward_index_values(const void* fwd, int64_t fwd_len, int32_t data_type, int32_t num_docs,
                                  int64_t* out_i64, double* out_f64);

/* Host-side bitmap inverted-index creator (OffHeapBitmapInvertedIndexCreator + BitmapInvertedIndexWriter,
 * seglocal/segment/creator/impl/inv/BitmapInvertedIndexWriter.java:60-78) over a fixed-bit forward index: writes
 * the `<column>.bitmap.inv` bytes (portable Roaring without run containers) into `out` (capacity out_cap) and their
 * length into *out_len; out == NULL only reports the length.  Pure host code, for segment fixtures and benches. */
int pgpu_build_inverted_index(const void* fwd, int64_t fwd_len, int32_t bits, int32_t num_docs, int32_t cardinality,
                              void* out, int64_t out_cap, int64_t* out_len);

/* Host-side star-tree builder (BaseSingleTreeBuilder + OnHeapSingleTreeBuilder, seglocal/startree/v2/builder/):
 * builds the star-tree of a segment given in Pinot's byte format (the pgpu_segment_desc of pgpu_pin_segment;
 * column_types per column), split order (column indexes), dimensions without star nodes (indexes into the split
 * order), function-column pairs and maxLeafRecords (<= 0: StarTreeV2BuilderConfig default 10000).  Pure host code:
 * no device is needed.  The result is read with pgpu_startree_get_desc and released with pgpu_startree_destroy. */
typedef struct pgpu_startree_s* pgpu_startree;
int pgpu_startree_build(const pgpu_segment_desc* segment, const int32_t* column_types, const int32_t* split_order,
                        int32_t num_dims, const int32_t* skip_star_dims, int32_t num_skip, const pgpu_agg* pairs,
                        int32_t num_pairs, int32_t max_leaf_records, pgpu_startree* out);
int pgpu_startree_get_desc(pgpu_startree st, pgpu_startree_desc* out);
/* Star-tree `star_tree_id` of a segment from Pinot's own files, as StarTreeLoaderUtils.loadStarTreeV2 reads them
 * (seglocal/startree/v2/store/StarTreeLoaderUtils.java:57-107): `index` is the segment's star_tree_index file (v1;
 * in a v3 segment the star-tree buffer of columns.psf), `index_map` the text of star_tree_index_map
 * (StarTreeIndexMapUtils.java:150-190: "<id>.<column>.<STAR_TREE|FORWARD_INDEX>.<OFFSET|SIZE> = n").  The
 * OffHeapStarTree buffer is validated as its constructor does (magic 0xBADDA55B00DAD00D, version 1, header length,
 * buffer size; OffHeapStarTree.java:45-80); its dimension names (the split order) are matched against
 * column_names (the table's columns); dimension forward indexes are FixedBitSVForwardIndexReaderV2 bytes with the
 * segment column's bits_per_element[column]; each "<fn>__<col>" pair's raw PASS_THROUGH chunk forward index
 * (versions 2 / 3) is decoded -- COUNT as LONG, SUM / MIN / MAX as DOUBLE (FixedByteChunkSVForwardIndexReader),
 * AVG as AvgPair bytes (VarByteChunkSVForwardIndexReader) -- and pairs of other functions are skipped.  num_docs is
 * the star-tree's total docs (metadata startree.v2.<id>.total.docs).  Pure host code; attach the result with
 * pgpu_startree_get_desc + pgpu_attach_startree, release it with pgpu_startree_destroy. */
int pgpu_startree_load(const void* index, int64_t index_len, const char* index_map, int64_t index_map_len,
                       int32_t star_tree_id, int32_t num_docs, int32_t num_columns, const char* const* column_names,
                       const int32_t* bits_per_element, pgpu_startree* out);
/* Number of star-tree records that come straight from the segment (sorted + aggregated rows), before the star-node
 * and aggregated documents (-1 for star-trees read by pgpu_startree_load: the files do not record it). */
int pgpu_startree_num_raw_records(pgpu_startree st, int32_t* n);
int pgpu_startree_destroy(pgpu_startree st);

/* ============================================================================ synthetic segments (bench) */

/* Column generators of BASELINE.md §3: value = f(splitmix64(seed_c ^ global_row)),
 * seed_c = (0x5EED0000 + column_index) << 32.  UNIFORM: lo + h % (hi - lo); ZIPF: ids[first k with cdf[k] > u];
 * TABLE: table[h % n].  The segment (dictionary = sorted distinct values present, fixed-bit forward index) is
 * built on the device and pinned directly; bytes are identical to Pinot's segment creator on the same values. */
enum pgpu_gen_kind { PGPU_GEN_UNIFORM = 0, PGPU_GEN_ZIPF = 1, PGPU_GEN_TABLE = 2 };
typedef struct {
  int32_t kind;
  int32_t column_index;
  int64_t lo, hi;             /* UNIFORM */
  int32_t n;                  /* ZIPF ranks / TABLE size */
  int32_t reserved;
  const double* cdf;          /* ZIPF cumulative distribution (host) */
  const int64_t* ids;         /* ZIPF rank -> value (host), ascending-id order not required */
  const double* table;        /* TABLE values (host) */
} pgpu_gen_column;
int pgpu_generate_segment(pgpu_table table, const pgpu_gen_column* columns, int32_t num_columns, int64_t row0,
                          int32_t num_docs, int64_t* segment_handle);
/* Copies a pinned segment column's bytes back to the host (parity checks of the generator). */
int pgpu_segment_column_info(pgpu_table table, int64_t segment_handle, int column, int32_t* cardinality,
                             int32_t* bits, int64_t* dict_len, int64_t* fwd_len);
int pgpu_segment_column_bytes(pgpu_table table, int64_t segment_handle, int column, uint8_t* dict_out,
                              uint8_t* fwd_out);

#ifdef __cplusplus
}
#endif
#endif
