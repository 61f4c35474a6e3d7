// filter_stats.h — numEntriesScannedInFilter of one segment, as Pinot's filter operators count it.
//
// The statistic depends on the physical operator tree Pinot builds for the segment (FilterPlanNode.java:146-247,
// FilterOperatorUtils.java:42-178: leaf operator choice, constant folding, AND child order) and on how its
// docId iterators run (AndDocIdSet.java:60-146, OrDocIdSet.java:57-110, AndDocIdIterator.java:40-67,
// OrDocIdIterator.java:25-130, SVScanDocIdIterator.java:56-94).  The GPU computes the document sets; this module
// turns them into the count:
//   - shapes whose count needs no document data (a single leaf, an OR of leaves) are counted on the host;
//   - an AND of index leaves and scans without other children (applyAnd chain) and an AND of exactly two scans
//     (leap-frog) are counted inside the scan kernel (STATS_CHAIN / STATS_LEAP2, scan_direct.h);
//   - every other shape replays the iterators over the leaves' match bitmaps produced by leaf_masks_kernel
//     (simulate_entries_scanned), with scan lengths counted arithmetically from the bitmaps.
#pragma once
#include <stdint.h>

#include <vector>

namespace pgpu {

// Pinot leaf operator of a predicate in one segment (FilterOperatorUtils.getLeafFilterOperator).  SL_RANGEIDX:
// RangeIndexBasedFilterOperator (a RANGE predicate on an unsorted column with a range index, :57-62) -- its docIdSet
// is a BitmapDocIdSet like an inverted leaf's; the entries of its own partial-match scan
// (RangeIndexBasedFilterOperator.java:110-126) do not depend on the rest of the tree and are added by the caller.
enum StatLeaf : int32_t { SL_EMPTY = 0, SL_ALL = 1, SL_SCAN = 2, SL_SORTED = 3, SL_BITMAP = 4, SL_RANGEIDX = 5 };
constexpr int kStatLeafKinds = 6;

// Physical filter tree of one segment after folding (EmptyFilterOperator / MatchAllFilterOperator removed as
// FilterPlanNode and getAnd/OrFilterOperator do), AND children in reorderAndFilterChildOperators order.  NOT is not
// part of the reference's 0.10 FilterContext; it is a scan-based iterator over its child (the oracle's model).
enum StatNodeType : int32_t { SN_EMPTY = 0, SN_ALL = 1, SN_SCAN = 2, SN_SORTED = 3, SN_BITMAP = 4, SN_NOT = 5,
                              SN_AND = 6, SN_OR = 7, SN_RANGEIDX = 8 };
struct StatNode {
  int32_t type = SN_ALL;
  int32_t leaf = -1;           // leaves: predicate index
  std::vector<int32_t> kids;   // AND / OR / NOT: node indexes
};
struct StatTree {
  std::vector<StatNode> nodes;
  int32_t root = -1;
};

// ops: the plan's encoded postfix program ((opcode << 16) | arg, internal.h OpCode); leaf: per predicate index.
StatTree build_stat_tree(const std::vector<int32_t>& ops, const std::vector<int32_t>& leaf);

// How a segment's count is obtained.
enum StatsKind : int32_t { STATS_CONST = 0, STATS_CHAIN = 1, STATS_LEAP2 = 2, STATS_GENERIC = 3 };
struct StatsPlan {
  int32_t kind = STATS_CONST;
  int64_t constant = 0;              // STATS_CONST: the count
  std::vector<int32_t> index_leaves; // STATS_CHAIN: index leaves (ANDed first), then
  std::vector<int32_t> scan_leaves;  //   scan leaves in Pinot's order; STATS_LEAP2: the two scans (A, B)
};
StatsPlan classify_stat_tree(const StatTree& t, int64_t num_docs);
// Predicate indexes of the range-index leaves whose operator runs (SN_RANGEIDX nodes not under a NOT, which
// evaluates its child per document): each adds its partial-match scan's entries.
std::vector<int32_t> range_index_leaves(const StatTree& t);

// Replays Pinot's iterators over the leaves' match bitmaps (leaf_masks[leaf]: word g bit i = doc 32g + i, the
// predicate's own match, negation included) and returns numEntriesScannedInFilter of the segment.
int64_t simulate_entries_scanned(const StatTree& t, const std::vector<const uint32_t*>& leaf_masks, int32_t num_docs);

}  // namespace pgpu
