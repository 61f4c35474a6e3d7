// range_index.h — a pinned column's range index (`<column>.bitmap.range`) as RangeIndexBasedFilterOperator uses it
// (core/operator/filter/RangeIndexBasedFilterOperator.java:57-129).  Not part of the ABI.
//
// The docs a RANGE leaf on such a column selects are exactly the predicate's matches (matches ∪ the scanned partial
// matches), which the scans evaluate from the forward index; what the index adds is the leaf's place in the filter
// tree (an index-based leaf, AND priority 2: FilterOperatorUtils.java:57-62, :143-178) and the entries of its
// partial-match scan.  Version 1 (RangeIndexCreator / RangeIndexReaderImpl) keeps the ranges' bounds and each range's
// document count for that; version 2 (BitSlicedRangeIndexReader) is exact and scans nothing.
#pragma once
#include <stdint.h>

#include <vector>

namespace pgpu {

struct RangeIdx {
  int32_t version = 0;         // 1: RangeIndexReaderImpl, 2: BitSlicedRangeIndexReader; 0: none
  std::vector<int64_t> start;  // version 1: the first value (dictId) of each range (_rangeStartArray)
  int64_t last_end = 0;        // version 1: the last range's last value (_lastRangeEnd)
  std::vector<int64_t> docs;   // version 1: documents of each range (cardinality of its bitmap)
  // numEntriesScannedInFilter of the operator for dictIds [lo, hi] (inclusive: SortedDictionaryBasedRangePredicate-
  // Evaluator's [startDictId, endDictId - 1]): the size of getPartiallyMatchingDocIds, which the operator's
  // ScanBasedDocIdIterator.applyAnd scans (RangeIndexReaderImpl.java:147-264).
  int64_t partial_entries(int64_t lo, int64_t hi) const;
};

// Parses a range index file of a dictionary-encoded column of `card` values over num_docs documents.  0 and
// out->version set (0: a version Pinot does not load -- DefaultIndexReaderProvider.newRangeIndexReader skips it), or
// PGPU_ERR_INVALID_ARGUMENT with the thread's last error set.  Pure host code.
int parse_range_index(const uint8_t* b, int64_t n, int64_t card, int32_t num_docs, RangeIdx* out);

// Cardinality of a portable Roaring bitmap whose docs are below num_docs (abi_table.cpp parse_roaring); false on
// malformed input.
bool roaring_cardinality(const uint8_t* b, int64_t n, int32_t num_docs, int64_t* docs);

}  // namespace pgpu
