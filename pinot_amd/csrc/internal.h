// internal.h — device-side data layout shared by the gfx950 kernels (kernels.hip) and the host runtime
// (rt_*.cpp, abi_*.cpp).  Not part of the ABI.
//
// HBM layout of a pinned segment column (one hipMalloc per segment, columns packed back to back):
//   fwd   : Pinot's forward-index bytes verbatim (MSB-first, big-endian bit packing of
//           FixedBitSVForwardIndexReaderV2), read as big-endian u32 words, zero-padded to a whole number of
//           8192-doc tiles (ceil(numDocs/8192) * 256 * bits words) + 4 spare words, so that a tile's LDS-DMA and a
//           two-word gather never leave the allocation;
//   lut   : int32 local dictId -> table-global dictId (group-by columns; built lazily, rebuilt when the
//           table's global dictionary grows);
//   dkey  : int64 per dictId: the value (INT/LONG) or an order-preserving key of the IEEE double
//           (FLOAT/DOUBLE) — the operand of SUM over integers and of MIN/MAX;
//   dval  : double per dictId — the operand of SUM/AVG over FLOAT/DOUBLE.
#pragma once
#include <stdint.h>

namespace pgpu {

constexpr int kBlock = 256;                 // threads per workgroup (4 waves of 64)
constexpr int kDocsPerLane = 32;            // one lane owns a 32-doc group = `bits` u32 words
constexpr int kTileDocs = kBlock * kDocsPerLane;  // 8192 docs per tile
constexpr int kLdsPackShift = 40;           // KParams.pack_shift of an LDS table (COUNT < 2^24, SUM < 2^40)
constexpr int kMaxQueryCols = 16;           // distinct columns referenced by one query
constexpr int kMaxLeaves = 16;              // predicate leaves
constexpr int kMaxOps = 48;                 // postfix filter program length
constexpr int kMaxKeys = 16;                // group-by columns handled on the GPU
constexpr int kMaxSlots = 24;               // accumulator rows of the group table
constexpr int kMaxStack = 8;                // filter evaluation stack depth
constexpr int kFwdPadWords = 4;
constexpr int kWaveQ = 256;                 // direct kernel: per-wave queue of sparse matched docs (LDS, u32)
constexpr int kFlushAt = 128;               // ... aggregated in 2-per-lane batches once it holds this many
constexpr int kDenseGroupMin = 256;        // matches per wave-tile (of 2048 docs) above which whole groups are decoded
constexpr int kFastLeaves = 4;              // pure-AND programs up to this many leaves keep them in registers

// LEAF_DOCRANGE: a predicate on a sorted column (SortedIndexBasedFilterOperator, core/operator/filter/
// SortedIndexBasedFilterOperator.java:51-125): docIds [lo, lo + span), evaluated without reading any column.
// LEAF_BITMAP: a predicate on a column with a bitmap inverted index (BitmapBasedFilterOperator, core/operator/filter/
// BitmapBasedFilterOperator.java:63-100): `set` is the segment's materialised docId bitmap (bit i of word g = doc
// 32g + i), the OR of the matching dictIds' Roaring bitmaps, built per query by inv_materialize_kernel.
// LEAF_RAW_RANGE / LEAF_RAW_IN: host-side kinds of a raw-value predicate on a no-dictionary column
// (RangePredicateEvaluatorFactory / InPredicateEvaluatorFactory raw evaluators).  raw_leaf_bitmap_kernel evaluates
// them per query into a docId bitmap (KRawTask), which the scans read as a LEAF_BITMAP leaf.
// LEAF_BITDIR: a LEAF_BITMAP of one dictId -- its Roaring containers read in place, as BitmapBasedFilterOperator
// uses a single bitmap without an OR (BitmapBasedFilterOperator.java:77-79): `set` is a directory of one 64-bit entry
// per 65536-doc block: 0 = no docs in the block; a BITMAP container's address (its 2048 words); an ARRAY container's
// address | 1 with its entry count in bits 48..63 (array_group_mask, device.h).
enum LeafKind : int32_t { LEAF_NONE = 0, LEAF_ALL = 1, LEAF_RANGE = 2, LEAF_SET = 3, LEAF_DOCRANGE = 4, LEAF_BITMAP = 5,
                          LEAF_RAW_RANGE = 6, LEAF_RAW_IN = 7, LEAF_BITDIR = 8 };
constexpr int kLeafKinds = 9;
enum OpCode : int32_t { OP_LEAF = 0, OP_AND = 1, OP_OR = 2, OP_NOT = 3 };
enum SlotKind : int32_t { SLOT_COUNT = 0, SLOT_SUM_I64 = 1, SLOT_SUM_F64 = 2, SLOT_MIN_KEY = 3, SLOT_MAX_KEY = 4 };
enum Mode : int32_t { MODE_LDS = 0, MODE_GLOBAL = 1, MODE_HASH = 2 };

// One predicate leaf evaluated against one segment: dictId in [lo, lo + span) (RANGE), bit set in `set`
// (SET), docId in [lo, lo + span) (DOCRANGE), constant (ALL / NONE); `negate` flips the result (NOT_EQ / NOT_IN).
struct KLeaf {
  int32_t kind;
  int32_t negate;
  uint32_t lo;
  uint32_t span;
  const uint32_t* set;
};

// One query column of one segment.  Dictionaries of consecutive values need no lookup: `lut` null = the segment's
// dictionary is a contiguous run of the table-global one (global dictId = dictId + lut_off); `dkey` null = an
// INT / LONG dictionary of consecutive values (value = key_base + dictId).  Typical of bounded integer columns
// (C1, C2, C5's metrics and keys), it saves a dependent gather per matched doc.
// Missing global values a segment's accumulator dictionary may have and still be read through the table-global
// value arrays (KCol.gaps).
constexpr int kMaxValueGaps = 16;

struct KCol {
  const uint32_t* fwd;
  const int32_t* lut;
  const int64_t* dkey;
  const double* dval;
  int64_t key_base;
  int32_t bits;
  int32_t lut_off;
  // Accumulator operands with table-global value arrays (rt_dict.cpp ensure_value_map): dkey / dval are the table's
  // arrays from the global dictId of the segment's first value on, and local dictId i is at i + the number of global
  // ids missing from the segment's dictionary below it -- ngaps thresholds in mapped space, applied in order as
  // i += (i >= gaps[k]) (vidx); 0 for the segment's own arrays or a contiguous run of the global dictionary.
  int32_t ngaps;
  uint32_t gaps[kMaxValueGaps];
};

// Per-plan, per-segment record (uploaded once per plan): a KSegHdr followed by num_cols KCol and num_leaves
// KLeaf; records are seg_stride bytes apart.
struct KSegHdr {
  int32_t num_docs;
  int32_t tile_base;  // first tile of this segment in the plan's tile space
  int32_t num_tiles;
  int32_t stats;      // numEntriesScannedInFilter counted in the scan kernel (filter_stats.h): STATS_* kind in bits
                      // 0-1; STATS_CHAIN: bit 4 + k = leaf k (evaluation order) is a scan whose applyAnd input is
                      // counted; STATS_LEAP2: leaves of scans A / B in bits 8-9 / 10-11
};
enum KStats : int32_t { KSTATS_NONE = 0, KSTATS_CHAIN = 1, KSTATS_LEAP2 = 2 };

struct KParams {
  const uint8_t* segs;     // num_segs records of seg_stride bytes
  const int32_t* tile_seg; // tile -> segment record (expand_tiles_kernel)
  int32_t seg_stride;
  int32_t num_cols;
  int32_t num_segs;
  int32_t num_tiles;
  int32_t tile_shift;      // small plans: each 8192-doc tile is split into 1 << tile_shift tiles (16 / 8 docs per lane)
  int32_t tile_chunks;     // 1: each workgroup takes a contiguous run of tiles (else XCD-interleaved tiles)
  // chunked runs weighted by the CU slot a workgroup is dispatched to: with slot_n resident workgroups per CU, workgroup
  // b (b / (grid / slot_n) = its slot, dispatch order) takes a share of its XCD's tiles proportional to slot_w[slot].
  // The SIMDs issue oldest wave first, so equal shares end slot by slot (C3: 1 : 1.08 : 1.17 : 1.27 loop-end times,
  // the same at 125 and 1000 segments).  slot_n = 0: equal shares.
  int32_t slot_n;
  uint16_t slot_w[4];
  int32_t pair_leaves;     // 1: an index leaf + a range scan are evaluated together (bitdir_range; 0 = A/B off)
  int32_t num_ops;         // 0 = match all
  int32_t pure_and;        // program is LEAF... AND(n): evaluate leaves with early exit, no stack
  int32_t ops[kMaxOps];    // (opcode << 16) | arg
  int32_t num_leaves;
  int32_t leaf_col[kMaxLeaves];
  int32_t num_keys;
  int32_t key_col[kMaxKeys];
  int64_t key_stride[kMaxKeys];
  int64_t num_keys_total;  // dense table width G, or hash capacity
  int64_t key_bias;        // subtracted from every composite key (filter-restricted key spaces; 0 otherwise)
  int32_t num_slots;
  int32_t slot_kind[kMaxSlots];
  int32_t slot_col[kMaxSlots];
  // Dense LDS tables (MODE_LDS, dense instance), set at plan time where the plan's value ranges allow:
  // pack_slot >= 0: an integer SUM slot whose whole-group adds carry the COUNT too -- (1 << 40) | value in one LDS
  //   atomic (values >= 0, a workgroup's docs < 2^24 and their sum < 2^40); the kernel splits the word into the COUNT
  //   row (slot 0) and the sum before it stores its slab.  MODE_HASH: the same add, (1 << pack_shift) | value, into the
  //   global table word (pack_shift = 64 - bits(plan docs)); hash_unpack_kernel splits the occupied words afterwards.
  // narrow (bit s): MIN / MAX slot s of an integer column with values in [0, 2^32 - 1): the whole-group path takes
  //   32-bit LDS min / max on the word's low half (the word starts at 2^32 - 1 / 0, so the 64-bit atomics of the
  //   per-doc path see the same order).
  int32_t pack_slot;
  int32_t pack_shift;      // the COUNT's low bit in the pack slot's word (kLdsPackShift for MODE_LDS)
  uint32_t narrow;
  uint64_t* table;         // [num_slots][num_keys_total] (MODE_GLOBAL / MODE_HASH), init by table_init_kernel
  uint64_t* slab;          // [gridDim][num_slots][num_keys_total] (MODE_LDS)
  unsigned long long* hash_keys;  // [num_keys_total] (MODE_HASH), empty = ~0
  // Key spaces beyond 64 bits (ArrayMapBasedHolder): the key columns split into consecutive groups; the key of group
  // s (previous group's slot x stage_mult[s - 1] + the mixed-radix key of its columns, which end at stage_end[s]) is
  // mapped to its slot in hash table s (stage_cap[s] slots at stage_keys + stage_off[s]); the last group's key is the
  // group key of the plan's own hash table.  num_stages = 0: one mixed-radix key over all columns.
  int32_t num_stages;
  int32_t stage_end[kMaxKeys];
  int64_t stage_cap[kMaxKeys];
  int64_t stage_off[kMaxKeys];
  int64_t stage_mult[kMaxKeys];
  unsigned long long* stage_keys;
  unsigned long long* stats;      // [0] docs matched, [2] entries scanned in filter (STATS_CHAIN / LEAP2 segments)
  // STATS_LEAP2 segments: per (tile, wave) one byte of AndDocIdIterator state over scans A, B: bit 0 = a doc
  // matches, bit 1 = scanner after the wave's docs (1 = B), bits 2-3 = entry difference at its first match + 1
  uint8_t* leap_maps;
  // QueryContext.getEndTimeMs as a wall_clock64() reading of this device (0 = no deadline): past it the persistent
  // scans stop taking tiles and set stats[5] (BaseCombineOperator.java:79-132 / GroupByCombineOperator.java:193-203
  // give up at the same point; the host then reports the timeout instead of a partial result)
  uint64_t deadline;
  // diagnostics build only (PGPU_DIAG_WG_TIMES, PGPU_TRACE=wgtimes): per workgroup {start, tile loop end, end, tiles | first tile << 32, HW_ID, XCC_ID, 0, 0}
  unsigned long long* diag_times;
  // Run-time balance of chunked plans (tile_chunks = 1): the static runs cover tiles [0, claim_base); the rest is
  // claimed claim_tiles at a time through *claim (zeroed with the statistics per execution) by whichever workgroup
  // finishes its work first.  claim = null: the static runs cover every tile.
  unsigned int* claim;
  int32_t claim_base;
  int32_t claim_tiles;
};

// leaf_masks_kernel work item: groups [group0, group0 + 256) of plan record `rec`; its leaves' masks go to
// out + out_word + leaf * ceil(numDocs / 32) (STATS_GENERIC segments, replayed on the host).
struct KMaskJob {
  int32_t rec;
  int32_t group0;
  int64_t out_word;
};

// ---------------------------------------------------------------------------------------------- star-tree
constexpr int kMaxStarDims = 16;

// One star-tree segment of a plan (uploaded per query).  Dimension indexes are split-order positions.
struct KStarSeg {
  const int32_t* nodes;                   // num_nodes x 7 int32 (OffHeapStarTreeNode layout)
  int32_t num_nodes;
  int32_t num_docs;                       // star-tree documents
  int32_t pred_mask;                      // dims with predicates (traversal's remaining predicate columns)
  int32_t group_mask;                     // group-by dims without predicates
  int32_t num_dims;
  // bit s: src_f[s] holds int32 values (a metric whose pre-aggregated doubles are all integers of int32 range,
  // narrowed at pin time; s < kMaxSlots = 24); bit 31: src_c[0] holds int32 counts
  uint32_t narrow;
  const uint32_t* dim_fwd[kMaxStarDims];  // star-tree documents' dictIds (MSB-first, padded)
  int32_t dim_bits[kMaxStarDims];
  int32_t dim_card[kMaxStarDims];         // the segment's dictionary size of each group-by / predicate dim
  const uint32_t* match[kMaxStarDims];    // matching-dictId bitset of each predicate dim
  const int32_t* key_lut[kMaxKeys];       // local -> global dictId of each group-by key
  int32_t key_dim[kMaxKeys];              // dim of each group-by key
  const double* src_f[kMaxSlots];         // per slot: pre-aggregated double per document (int32 if narrow)
  const int64_t* src_c[kMaxSlots];        // per slot: pre-aggregated count per document (slot 0; null = 1; int32 if narrow)
  int32_t* ranges;                        // scratch: 2 x num_nodes (startDocId, endDocId)
  int64_t* prefix;                        // scratch: num_nodes + 1 prefix sums of range lengths
  int32_t* frontier;                      // scratch: 2 x 3 x num_nodes
  int32_t* out;                           // [0] ranges emitted, [1] remaining predicate dims (residual filter)
};

struct KStarParams {
  const KStarSeg* segs;
  int32_t num_segs;                       // <= kStarMaxSegs per launch
  int32_t range_cache;                    // ranges per segment cached in LDS (0: binary search in global memory)
  const int64_t* seg_total;               // K5: 32-doc groups of each segment's emitted ranges
  int32_t num_wgs;                        // K6 workgroups (persistent: each takes a contiguous run of groups)
  int32_t pad0;
  int32_t num_keys;
  int32_t num_slots;
  int64_t key_stride[kMaxKeys];
  int64_t num_keys_total;
  int64_t key_bias;                       // as KParams.key_bias
  int32_t slot_kind[kMaxSlots];
  int32_t slot_int[kMaxSlots];            // 1: the slot's column is INT/LONG (MIN/MAX keys are the value)
  int32_t lds_table_words;
  int32_t cache_ints;                     // LDS ints for a segment's key LUTs + residual match sets (0: read global)
  uint64_t* table;                        // MODE_GLOBAL / MODE_HASH
  uint64_t* slab;                         // MODE_LDS: this kernel's first slab
  unsigned long long* hash_keys;
  unsigned long long* stats;              // [0] docs matched, [1] entries scanned in filter, [3] star-tree
                                          // documents read (positions of the emitted ranges), [5] timed out
  uint64_t deadline;                      // as KParams.deadline
};

// ---------------------------------------------------------------------------------------------- partitioned
// Parameters of the partitioned group-by of large dense key spaces (partition.h, k_partition.hip).
struct KPartParams {
  KParams base;                     // segments, filter program, key layout (num_keys_total = G), slots
  int32_t pshift;                   // keys per partition = 1 << pshift (<= 65536: u16 record keys)
  int32_t num_parts;
  int32_t num_streams;              // 8-byte operand streams of a record
  int32_t stream_col[kMaxSlots];    // query column slot of each stream
  int32_t stream_f64[kMaxSlots];    // 1: the column's dval (double), 0: its dkey (int64 value / ordered key)
  int32_t slot_stream[kMaxSlots];   // per slot: its operand stream (-1: COUNT)
  uint32_t* part_start;             // [num_parts + 1]: K8a totals, scanned in place into run starts by K8b
  uint32_t* block_off;              // [gridDim][num_coarse]: a workgroup's offset inside each coarse run
  uint16_t* rec_key;                // [rec_cap] final layout: key within its partition
  uint64_t* rec_val;                // [num_streams][rec_cap]
  int64_t rec_cap;
  // Two-level scatter (num_parts > 64): K8c writes runs of 2^cshift partitions ("coarse" partitions, few enough
  // that every workgroup's open output lines stay in L2), K8e splits each coarse run into its partitions.
  int32_t cshift;                   // 0: single level (K8c writes the final layout)
  int32_t num_coarse;               // ceil(num_parts / 2^cshift)
  int32_t chunks_per_coarse;        // K8e workgroups per coarse run
  int32_t split_batch;              // K8e records sorted in LDS per batch (multiple of kBlock)
  uint32_t* coarse_fill;            // [num_coarse] K8a reservation counters
  uint32_t* fine_fill;              // [num_parts] K8e reservation counters
  uint32_t* mid_key;                // [rec_cap] coarse layout: key within its coarse range
  uint64_t* mid_val;                // [num_streams][rec_cap]
  // 1: every stream is an integer whose values fit int32 (checked over the plan's dictionaries): rec_val / mid_val
  // hold u32 words ([num_streams][rec_cap] u32, sign-extended on read) -- 4 bytes less per record and stream in
  // each of the four record passes
  int32_t val32;
  // > 0 (two-level, one integer stream): K8c packs (value - pack_min) into the mid_key bits above the key's
  // cshift + pshift bits (pack_bits of them) and writes no mid_val; K8e unpacks -- 4 bytes per record instead of 8
  int32_t pack_bits;
  int64_t pack_min;
  // 1 (pack_bits > 0 and pshift + pack_bits <= 32): K8e writes the final records packed the same way -- the key
  // within its partition in the low pshift bits, (value - pack_min) above -- as u32 words at rec_val, and K8d
  // unpacks them: 4 bytes per record instead of 6 (u16 key + u32 value) in K8e's write and K8d's read
  int32_t fine_pack;
  // 1 (fine_pack, slots exactly COUNT + integer SUM of the stream): K8d adds (1 << 40) | (value - pack_min) into one
  // LDS word per key instead of two atomics, where the partition's records bound both halves (count < 2^24, the
  // sum of offsets < 2^40: pack_range x records); the word is split when the slice is stored
  int32_t cs_pack;
  int64_t pack_range;
  // Hashed partitions (MODE_HASH key spaces < 2^31, partition.h K8h): a record's partition is the top pbits of
  // part_hash(key), its key is stored whole (mid_key / rec_key32), and K8h aggregates each partition in an LDS hash
  // table of 2^sbits entries, appending (key, slot words) records at out_rec / out_count (the compacted form of a
  // hash table, finalized as one).  pshift is 0 and pack_bits / fine_pack / cs_pack are off.
  int32_t hashed;
  int32_t pbits;
  int32_t sbits;
  uint32_t* rec_key32;                // [rec_cap] final layout: the whole key
  // 1 (hashed, two-level, one u32 value stream): K8c writes each record as one u64 (hk | value << 32) at mid_val
  // instead of a u32 key and a u32 value in two arrays; K8e reads it so
  int32_t mid_pair;
  // K8c staging (part_pass_kernel STAGE 1 / 2): 0 = off; else the records' form (1: pack_bits u32, 2: mid_pair u64),
  // and the u32 word of K8c's LDS where the waves' staging regions start (set by launch_partitioned)
  int32_t staged;
  int32_t stage_off;
  uint64_t* out_rec;                  // [out_cap][1 + num_slots]
  unsigned long long* out_count;      // groups appended (counts past out_cap too: the host reports the overflow)
  int64_t out_cap;                    // records out_rec holds (part_hash_out_cap)
  // [num_parts][2][num_slots]: each partition's range of every slot's words (order-preserving u64, min then max) --
  // the compact result form's widths without a pass over the records (launch_hash_minmax_parts folds them)
  unsigned long long* out_mm;
  // K8d with cs_pack and 2^pshift == kCompactChunk keys per partition (C5): partition b is the ordered compaction's
  // chunk b, and K8d writes what compact_count_kernel would -- the chunk's present keys (chunk_cnt[b]) and the
  // [min COUNT, min SUM, max COUNT, max SUM] row of its present keys (chunk_mm + 4 b) -- so finalize skips that
  // pass over the 10 M-key table (null: not written)
  uint32_t* chunk_cnt;
  long long* chunk_mm;
};
// K8h: value streams a record carries in registers (plans with more use the global hash table).
constexpr int kHashPartStreams = 4;
// K8h: linear probes of the LDS hash table before a record is left for the partition's next round.
constexpr int kHashPartProbes = 128;

// K8e batch: records sorted by partition in LDS per step (at most kSplitBatch; fewer with many value streams).
constexpr int kSplitBatch = 2048;
// LDS bytes of part_split_kernel: 2^cshift partitions per coarse run, `streams` value streams, `batch` records.
constexpr size_t part_split_lds(int cshift, int streams, int batch, int key_bytes = 2) {
  return (size_t)3 * ((size_t)1 << cshift) * 4 + 8 + (size_t)streams * batch * 8 + (size_t)batch * (4 + key_bytes) + 16;
}
// LDS bytes of part_hash_aggregate_kernel: 2^sbits entries of a u32 key and num_slots u64 words.
constexpr size_t part_hash_lds(int sbits, int num_slots) {
  return ((size_t)1 << sbits) * ((size_t)num_slots * 8 + 4);
}

// ---------------------------------------------------------------------------------------------- inverted index
// One Roaring container of a pinned inverted index ORed into a query's docId bitmap.  Containers are kept on the
// device as ARRAY (n sorted u16 low halves, two per u32 word, little-endian) or BITMAP (2048 u32 words: bit v of
// the container = bit (v & 31) of word v >> 5, Roaring's long[1024] read as u32); run containers are converted at
// attach time.  dst = word of the container's first doc (key << 16) in the plan's docbits buffer.
enum ContainerType : int32_t { CONT_ARRAY = 0, CONT_BITMAP = 1 };
constexpr int kContainerWords = 2048;
struct KBitTask {
  const uint32_t* payload;
  int32_t type;
  int32_t n;
  int64_t dst;
};
// One 2048-word (65536-doc) block of a docbits region: the OR of its tasks [task_begin, task_begin + num_tasks),
// zero when it has none.  Every block of every region is listed, so the kernel writes the whole buffer.
struct KBitBlock {
  int64_t dst;
  int32_t task_begin;
  int32_t num_tasks;
};

// One raw-value leaf of one segment (ScanBasedFilterOperator over a raw forward index with a raw-value
// PredicateEvaluator): the column's per-doc int64 keys (integer value, or order-preserving key of the double; padded
// to whole 32-doc groups) tested against [lo, hi] (LEAF_RAW_RANGE) or the hi sorted keys raw_vals[lo, lo + hi)
// (LEAF_RAW_IN), negated for NOT_EQ / NOT_IN, into ceil(num_docs / 32) docbits words from `dst` (bits past numDocs
// clear).
struct KRawTask {
  const int64_t* keys;
  int64_t dst;
  int64_t lo, hi;
  int32_t num_docs;
  int32_t kind;
  int32_t negate;
  int32_t pad;
};
// raw_leaf_bitmap_kernel work item: groups [group0, group0 + 256) of task `task`.
struct KRawJob {
  int32_t task;
  int32_t group0;
};

// Host-callable launchers (kernels.hip).
int launch_unpack(const uint32_t* fwd, int32_t bits, int64_t start, int64_t n, int32_t* out, void* stream);
int launch_gather_ids(const uint32_t* fwd, int32_t bits, const int32_t* docs, int32_t n, int32_t* out, void* stream);
int launch_fwd_max(const void* d_fwd, int64_t n, int32_t bits, unsigned int* d_out, void* stream);
int launch_hash_unpack(uint64_t* table, const unsigned long long* hash_keys, int64_t cap, int32_t pack_slot,
                       int32_t shift, void* stream);
int launch_table_init(uint64_t* table, const int32_t* slot_kind, int32_t num_slots, int64_t num_keys,
                      unsigned long long* hash_keys, void* stream);
// Also the deadline gate of the scan launch that follows it: sets stats[5] when `deadline` (wall_clock64 ticks,
// 0 = none) has passed.
int launch_expand_tiles(const uint8_t* segs, int32_t seg_stride, int32_t num_segs, int32_t* tile_seg,
                        uint64_t deadline, unsigned long long* stats, void* stream);
// variant: 0 sparse instance, 1 dense, 2 dense "simple" (no LUT / dictionary gathers, no double sums)
int launch_filter_groupby(const KParams& p, int mode, int variant, int grid, size_t lds_bytes, void* stream);
// Resident workgroups per CU of the direct kernel instance (< 0: query failed).
int occupancy_filter_groupby(int mode, int variant, size_t lds_bytes);
int launch_reduce_slabs(const uint64_t* slab, const int32_t* slot_kind_dev, int32_t num_slots, int64_t num_keys,
                        int32_t num_blocks, uint64_t* out, void* stream);
int launch_compact(const uint64_t* table, const unsigned long long* hash_keys, int32_t num_slots, int64_t num_keys,
                   unsigned long long* counter, uint64_t* out, int64_t out_cap, void* stream);
// Dense tables: groups with COUNT > 0 in ascending key order, columnar with row stride cap (even): int32 group-by
// dictIds [num_key_cols][cap], then u64 slot words [num_slots][cap]; chunk_scratch holds
// compact_ordered_chunks(num_keys) u32.
int64_t compact_ordered_chunks(int64_t num_keys);
int launch_compact_ordered(const uint64_t* table, int32_t num_slots, int64_t num_keys, int64_t key_base,
                           const int64_t* key_stride, const int64_t* key_card, const int64_t* key_off,
                           int32_t num_key_cols,
                           uint32_t* chunk_scratch,
                           unsigned long long* total, void* out, int64_t cap, void* stream);
// Cross-GPU exchange of hash-mode tables: per-owner group counts (counts[nparts], zeroed by the caller), records
// [key, num_slots words] grouped by owner (cursor[p] = owner p's first record; conv bit s: int64 word -> double), and
// the owner's merge of n records into an initialised hash table.
int launch_exchange_count(const uint64_t* table, const unsigned long long* hash_keys, int64_t num_keys, int32_t nparts,
                          unsigned long long* counts, void* stream);
int launch_exchange_scatter(const uint64_t* table, const unsigned long long* hash_keys, int64_t num_keys,
                            int32_t num_slots, int32_t nparts, uint32_t conv, unsigned long long* cursor, uint64_t* out,
                            void* stream);
int launch_i64_to_f64(uint64_t* p, int64_t n, void* stream);
// k_hashsort.hip: hash-mode finalize on the device (radix sort of the compacted records by key, decode to columns).
int launch_hash_minmax(const uint64_t* rec, const unsigned long long* count, int64_t cap, int32_t num_slots,
                       unsigned long long* mm, void* stream);
int launch_hash_minmax_parts(const unsigned long long* part_mm, int32_t num_parts, int32_t num_slots,
                             unsigned long long* mm, void* stream);
int launch_hash_compact(const uint64_t* rec, int64_t n, int32_t num_slots, int32_t key_width, const int32_t* width,
                        const int64_t* slot_off, uint8_t* out, void* stream);
int launch_hash_decode(const uint64_t* rec, int64_t n, int32_t num_slots, int32_t num_keys, const int64_t* stride,
                       const int64_t* card, const int64_t* off, uint8_t* out, size_t slot_off, void* stream);
int launch_merge_records(const uint64_t* rec, int64_t n, int32_t num_slots, const int32_t* slot_kind, uint64_t* table,
                         unsigned long long* hash_keys, int64_t num_keys, void* stream);
// Compact form of a large dense table: counts per chunk + exclusive scan (total into *total) + each slot's range over
// the present groups (minmax [2][num_slots]); then the presence bitmap (ceil(num_keys / 64) words) and the slots'
// words of the present groups in key order at compact_slot_width bytes, slot s from out_slots + s * cap * 8.
// chunk_scratch bytes launch_compact_dense_count needs (chunk counts, then per-chunk slot ranges).
size_t compact_scratch_bytes(int64_t num_keys, int32_t num_slots);
// counted: chunk_scratch already holds the chunk counts and ranges (K8d's KPartParams.chunk_cnt / chunk_mm), only the
// ranges' fold and the scan run.
int launch_compact_dense_count(const uint64_t* table, int32_t num_slots, int64_t num_keys, uint32_t* chunk_scratch,
                               unsigned long long* total, long long* minmax, void* stream, bool counted = false);
// Keys per chunk of the ordered compaction (kernels.hip kCompactChunk).
constexpr int kCompactChunkKeys = 4096;
int launch_compact_dense_scatter(const uint64_t* table, int32_t num_slots, int64_t num_keys, const int32_t* slot_kind,
                                 const uint32_t* chunk_scratch, const long long* minmax, uint64_t* bitmap,
                                 void* out_slots, int64_t cap, void* stream);
int compact_slot_width(long long lo, long long hi, int kind);
// The ordered scatter alone (chunk offsets from launch_compact_dense_count): the columnar explicit form.
int launch_compact_ordered_scatter(const uint64_t* table, int32_t num_slots, int64_t num_keys, int64_t key_base,
                                   const int64_t* key_stride, const int64_t* key_card, const int64_t* key_off,
                                   int32_t num_key_cols, const uint32_t* chunk_scratch, void* out, int64_t cap,
                                   void* stream);
// Partitioned group-by (k_partition.hip): K8a count, scan, K8c scatter, K8d aggregate into p.base.table.
int occupancy_part_pass(size_t pass_lds, int num_parts, int num_coarse, int staged);
int launch_partitioned(const KPartParams& pp, int grid, size_t pass_lds, void* stream);
// In-place exclusive prefix sum of n u32 (one workgroup; n up to a few 10^4).
int launch_exclusive_scan_u32(uint32_t* data, int32_t n, void* stream);
int launch_filter_bitmap(const KParams& p, uint32_t* out_words, void* stream);
// Per STATS_LEAP2 record of a launch: composes its (tile, wave) maps in doc order into the segment's count
// (stats[2] += ...).
// reduce_slabs + leap2_compose of a one-launch plan as one launch; host_out (pinned, num_slots x num_keys + 6 words;
// null = none): the table and the statistics words copied there by the last block (done: a zeroed u32 counter).
int launch_epilogue(const uint64_t* slab, const int32_t* slot_kind, int32_t num_slots, int64_t num_keys,
                    int32_t num_blocks, uint64_t* out, const uint8_t* segs, int32_t seg_stride, int32_t num_segs,
                    const uint8_t* maps, unsigned long long* stats, uint64_t* host_out, unsigned int* done,
                    void* stream);
int launch_leap2_compose(const uint8_t* segs, int32_t seg_stride, int32_t num_segs, const uint8_t* maps,
                         unsigned long long* stats, void* stream);
int launch_leaf_masks(const KParams& p, const KMaskJob* jobs, int32_t num_jobs, uint32_t* out, void* stream);
int launch_inv_materialize(const KBitBlock* blocks, int64_t num_blocks, const KBitTask* tasks, uint32_t* docbits,
                           void* stream);
int launch_raw_leaf_bitmaps(const KRawJob* jobs, int64_t num_jobs, const KRawTask* tasks, const int64_t* raw_vals,
                            uint32_t* docbits, void* stream);
constexpr int kStarMaxSegs = 4096;  // star-tree segments per K6 launch (their group prefix lives in LDS)
int launch_deadline_gate(uint64_t deadline, unsigned long long* stats, void* stream);
int launch_startree_traverse(const KStarSeg* segs, int32_t num_segs, int64_t* seg_total, uint64_t deadline,
                             unsigned long long* stats, void* stream);
int launch_startree_scan(const KStarParams& p, int mode, size_t lds_bytes, void* stream);
// Synthetic generator (bench): positions of generated values in the sorted domain + presence bitmap, then pack.
int launch_gen_positions(int32_t kind, uint64_t seed, int64_t lo, int64_t span, const double* cdf,
                         const int32_t* code_to_pos, int32_t n_codes, int64_t row0, int32_t num_docs,
                         int32_t* pos_out, uint32_t* presence, void* stream);
// One wall_clock64() reading into `out` (host-visible memory): deadline calibration.
int launch_read_clock(uint64_t* out, void* stream);
int launch_gen_pack(const int32_t* pos, const int32_t* pos_to_id, int32_t num_docs, int32_t bits, uint32_t* fwd_out,
                    void* stream);

}  // namespace pgpu
