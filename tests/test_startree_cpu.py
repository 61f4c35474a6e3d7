"""Star-tree on the CPU (no device): the product's host builder (pgpu_startree_build) and the star-tree oracle.

Pinned by BaseStarTreeV2Test's rule (core-test/core/startree/v2/BaseStarTreeV2Test.java:219-295): the answer read
off the star-tree equals the scan answer over the raw segment (here the C oracle, exactly for integer metrics and
counts, 1e-9 relative for double sums).  Structural invariants of the builder follow BaseSingleTreeBuilder
(seglocal/startree/v2/builder/BaseSingleTreeBuilder.java:298-453) and StarTreeBuilderUtils.serializeTree (:91-230).
"""
import numpy as np
import pytest

import startree_common as SC
from pinot_amd.query import parse_query
from pinot_amd.startree import StarTree


@pytest.fixture(scope="module")
def c4(oracle):
    rng = np.random.default_rng(44)
    cols = SC.c4_columns(rng, 60000, cards=(30, 12, 8, 5))
    seg = oracle.make_segment(SC.C4_SCHEMA, cols)
    st = StarTree.build(SC.C4_SCHEMA, seg, SC.C4_SPLIT, SC.C4_PAIRS, max_leaf_records=500)
    return seg, st, st.arrays(), cols


def test_builder_structure(c4):
    seg, st, a, cols = c4
    nodes = a["nodes"]
    n = len(nodes)
    assert nodes[0][0] == -1 and nodes[0][5] == 1  # root: dimensionId ALL, first child right after it (BFS)
    raw = st.num_raw_records()
    keys = np.stack([cols[c] for c in SC.C4_SPLIT], axis=1)
    assert raw == len(np.unique(keys, axis=0))  # sortAndAggregateSegmentRecords merges equal dimension tuples
    cnt = a["metric_i64"][1]
    assert int(cnt[:raw].sum()) == seg.num_docs
    assert a["metric_f64"][0][:raw].sum() == float(cols["m"].sum())
    for i in range(n):
        dim, val, start, end, agg, first, last = (int(x) for x in nodes[i])
        if first >= 0:
            kids = nodes[first:last + 1]
            assert list(kids[:, 1]) == sorted(kids[:, 1])          # children sorted, star (-1) first
            assert all(int(k[0]) == int(nodes[first][0]) for k in kids)
            assert (kids[:, 1] == -1).sum() <= 1
        else:
            assert end - start <= 500 or dim == len(SC.C4_SPLIT) - 1  # split until <= maxLeafRecords
        # the aggregated document holds the node's totals
        if start >= 0 and agg >= 0:
            assert cnt[agg] == cnt[start:end].sum()


@pytest.mark.parametrize("sql", SC.C4_QUERIES)
def test_startree_oracle_equals_scan(oracle, c4, sql):
    seg, st, a, cols = c4
    q = parse_query(sql, num_groups_limit=10 ** 9)
    got, docs, _ = SC.startree_answer(oracle, seg, SC.C4_SCHEMA, a, q, SC.C4_SPLIT, SC.C4_PAIRS)
    exp = oracle.run_groupby(SC.C4_SCHEMA, [seg], q).groups
    assert set(got) == set(exp)
    for k, ev in exp.items():
        for (fn, col), g, e in zip(q.aggregations, got[k], ev):
            if fn == "AVG":
                assert g.count == e.count and g.sum == pytest.approx(e.sum, rel=1e-12)
            elif col == "md":
                assert g == pytest.approx(e, rel=1e-9, abs=1e-6)
            else:
                assert g == e, (k, fn)
    assert docs < seg.num_docs  # pre-aggregation reads fewer documents than the scan


def test_skip_star_node_dimension(oracle):
    rng = np.random.default_rng(3)
    cols = SC.c4_columns(rng, 20000, cards=(6, 5, 4, 3))
    seg = oracle.make_segment(SC.C4_SCHEMA, cols)
    st = StarTree.build(SC.C4_SCHEMA, seg, SC.C4_SPLIT, SC.C4_PAIRS, max_leaf_records=50, skip_star_dims=["d2"])
    a = st.arrays()
    nodes = a["nodes"]
    assert not any(int(r[0]) == 1 and int(r[1]) == -1 for r in nodes)  # no star node on d2
    q = parse_query("SELECT SUM(m), COUNT(*) FROM t WHERE d3 = 2 GROUP BY d1", num_groups_limit=10 ** 9)
    got, _, _ = SC.startree_answer(oracle, seg, SC.C4_SCHEMA, a, q, SC.C4_SPLIT, SC.C4_PAIRS)
    assert got == oracle.run_groupby(SC.C4_SCHEMA, [seg], q).groups


@pytest.mark.parametrize("sql", SC.C4_QUERIES)
def test_c_startree_operator_matches(oracle, c4, sql):
    """The C oracle's StarTreeFilterOperator + StarTreeGroupByExecutor restatement (run_star_segment, the CPU
    baseline of bench.py's C4 line) against the Python restatement (same documents read) and the scan."""
    from dataclasses import replace
    seg, st, a, cols = c4
    q = parse_query(sql, num_groups_limit=10 ** 9)
    star_seg = replace(seg)
    star_seg.star_arrays = a
    got = oracle.run_groupby(SC.C4_SCHEMA, [star_seg], q, use_star_tree=True)
    exp_star, docs, scanned = SC.startree_answer(oracle, seg, SC.C4_SCHEMA, a, q, SC.C4_SPLIT, SC.C4_PAIRS)
    scan = oracle.run_groupby(SC.C4_SCHEMA, [seg], q)
    assert got.stats[0] == docs and got.stats[1] == scanned  # same documents and residual entries
    assert got.stats[3] == seg.num_docs
    for exp in (exp_star, scan.groups):
        assert set(got.groups) == set(exp)
        for k, ev in exp.items():
            for (fn, col), g, e in zip(q.aggregations, got.groups[k], ev):
                if fn == "AVG":
                    assert g.count == e.count and g.sum == pytest.approx(e.sum, rel=1e-12)
                elif col == "md" or fn == "SUM":
                    assert g == pytest.approx(e, rel=1e-9, abs=1e-6)
                else:
                    assert g == e, (k, fn)
    # a query the tree does not fit (no min__md pair) runs the scan
    q2 = parse_query("SELECT MIN(md) FROM t GROUP BY d1", num_groups_limit=10 ** 9)
    assert oracle.run_groupby(SC.C4_SCHEMA, [star_seg], q2, use_star_tree=True).stats == \
        oracle.run_groupby(SC.C4_SCHEMA, [seg], q2).stats
