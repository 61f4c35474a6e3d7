"""startree_oracle.py — CPU restatement of Pinot's star-tree query path.

TEST INFRASTRUCTURE ONLY: tests/ use it as the checker of the GPU star-tree kernels; the product never imports it.

Restated semantics (SURVEY.md abbreviations):
  traverse()  StarTreeFilterOperator.traverseStarTree (core/startree/operator/StarTreeFilterOperator.java:234-338):
              BFS from the root; an entry with no remaining predicate / group-by dims adds the node's aggregated doc;
              a leaf adds [startDocId, endDocId) and its remaining predicate dims; a predicate dim expands the
              children whose dictId matches; a group-by dim expands all non-star children; otherwise the star child
              (OffHeapStarTreeNode.getChildForDimensionValue(ALL), :115-148) if any, else all non-star children.
  groupby()   the residual filter (remaining predicate columns ANDed with the traversal bitmap, :185-226) and
              StarTreeGroupByExecutor.aggregate (core/startree/executor/StarTreeGroupByExecutor.java:60-71) with the
              function-column pair columns: SUM/MIN/MAX/AVG read the pre-aggregated values, COUNT adds count__*
              (CountAggregationFunction.java:97-104), in ascending star-tree docId order (bitmap iteration), double
              accumulation as SumAggregationFunction.aggregateGroupBySV (:66-73).
Parity is pinned by the self-consistency rule of BaseStarTreeV2Test (core-test/core/startree/v2/
BaseStarTreeV2Test.java:219-295): the star-tree answer equals the scan answer over the raw segment (the C oracle).
"""
import numpy as np

ALL = -1
COUNT, SUM, MIN, MAX, AVG = 0, 1, 2, 3, 4


def unpack_bits(buf, n, bits):
    """PinotDataBitSet.readInt for docs 0..n-1 of an MSB-first big-endian packed buffer."""
    if n == 0:
        return np.zeros(0, dtype=np.int64)
    raw = np.unpackbits(np.frombuffer(buf, dtype=np.uint8))[:n * bits].reshape(n, bits).astype(np.int64)
    w = (1 << np.arange(bits - 1, -1, -1, dtype=np.int64))
    return raw @ w


def traverse(nodes, pred_match, group_dims):
    """nodes: [n,7] int32; pred_match: {dim: bool array over dictIds}; group_dims: set of dims (without predicate
    dims).  Returns (list of (start, end) doc ranges, set of remaining predicate dims) or None when a predicate
    matches no dictId."""
    for m in pred_match.values():
        if not m.any():
            return None
    ranges, remaining = [], set()
    queue = [(0, frozenset(pred_match), frozenset(group_dims))]
    head = 0
    while head < len(queue):
        node, rp, rg = queue[head]
        head += 1
        dim_id, value, start, end, agg, first, last = (int(x) for x in nodes[node])
        if not rp and not rg:
            ranges.append((agg, agg + 1))
            continue
        if first < 0:
            ranges.append((start, end))
            remaining |= set(rp)
            continue
        cd = int(nodes[first][0])
        children = range(first, last + 1)
        if cd in rp:
            m = pred_match[cd]
            for c in children:
                v = int(nodes[c][1])
                if v != ALL and m[v]:
                    queue.append((c, rp - {cd}, rg))
        else:
            if cd not in rg:
                if int(nodes[first][1]) == ALL:
                    queue.append((first, rp, rg))
                    continue
                nrg = rg
            else:
                nrg = rg - {cd}
            for c in children:
                if int(nodes[c][1]) != ALL:
                    queue.append((c, rp, nrg))
    return ranges, remaining


def groupby(star, dim_bits, pred_match, group_dims_in_order, aggs):
    """star: StarTree.arrays(); dim_bits: bits per split-order dim; pred_match: {dim: bool array};
    group_dims_in_order: split-order dim of each group-by column (query order); aggs: [(fn code, metric index)].
    Returns ({dictId tuple: [values]}, docs matched, entries scanned in filter)."""
    nodes = star["nodes"]
    nd = star["num_docs"]
    gset = set(group_dims_in_order) - set(pred_match)
    t = traverse(nodes, pred_match, gset)
    if t is None:
        return {}, 0, 0
    ranges, remaining = t
    bitmap = np.zeros(nd, dtype=bool)
    for s, e in ranges:
        bitmap[s:e] = True
    docs = np.nonzero(bitmap)[0]
    scanned = len(docs) * len(remaining)
    dims = {d: unpack_bits(star["dim_fwd"][d], nd, dim_bits[d]) for d in set(remaining) | set(group_dims_in_order)}
    keep = np.ones(len(docs), dtype=bool)
    for d in remaining:
        keep &= pred_match[d][dims[d][docs]]
    docs = docs[keep]
    if len(docs) == 0:
        return {}, 0, scanned
    keys = np.stack([dims[d][docs] for d in group_dims_in_order], axis=1)
    uniq, inv = np.unique(keys, axis=0, return_inverse=True)
    inv = inv.reshape(-1)
    out = {}
    cols = []
    for fn, m in aggs:
        f = star["metric_f64"][m]
        c = star["metric_i64"][m]
        if fn == COUNT:
            acc = np.zeros(len(uniq), dtype=np.int64)
            np.add.at(acc, inv, c[docs])
            cols.append([int(x) for x in acc])
        elif fn == SUM:
            acc = np.zeros(len(uniq), dtype=np.float64)
            np.add.at(acc, inv, f[docs])  # ascending docId order
            cols.append([float(x) for x in acc])
        elif fn == MIN:
            acc = np.full(len(uniq), np.inf)
            np.minimum.at(acc, inv, f[docs])
            cols.append([float(x) for x in acc])
        elif fn == MAX:
            acc = np.full(len(uniq), -np.inf)
            np.maximum.at(acc, inv, f[docs])
            cols.append([float(x) for x in acc])
        else:
            s = np.zeros(len(uniq), dtype=np.float64)
            n = np.zeros(len(uniq), dtype=np.int64)
            np.add.at(s, inv, f[docs])
            np.add.at(n, inv, c[docs])
            cols.append([(float(a), int(b)) for a, b in zip(s, n)])
    for g in range(len(uniq)):
        out[tuple(int(x) for x in uniq[g])] = [col[g] for col in cols]
    return out, len(docs), scanned
