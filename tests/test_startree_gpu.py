"""GPU star-tree parity: K5 traversal + K6 pre-aggregated scan through the C ABI against the star-tree oracle
(oracle/startree_oracle.py) and the scan oracle (BaseStarTreeV2Test's self-consistency rule,
core-test/core/startree/v2/BaseStarTreeV2Test.java:219-295): exact for counts and integer SUM/MIN/MAX, 1e-9
relative for double sums."""
import numpy as np
import pytest

import startree_common as SC
from pinot_amd.executor import GpuTable
from pinot_amd.query import parse_query
from pinot_amd.startree import StarTree

pytestmark = pytest.mark.gpu


def _check(got, exp, q):
    g = got.as_dict()
    assert set(g) == set(exp), sorted(set(g) ^ set(exp))[:5]
    for k, ev in exp.items():
        for (fn, col), x, y in zip(q.aggregations, g[k], ev):
            if fn == "AVG":
                assert x.count == y.count and x.sum == pytest.approx(y.sum, rel=1e-12), k
            elif col == "md":
                assert x == pytest.approx(y, rel=1e-9, abs=1e-6), k
            else:
                assert x == y, (k, fn, x, y)


@pytest.fixture(scope="module")
def c4_gpu(oracle, gpu_lib):
    rng = np.random.default_rng(404)
    segs, stars = [], []
    for i in range(3):
        seg = oracle.make_segment(SC.C4_SCHEMA, SC.c4_columns(rng, 40000 + 7919 * i, cards=(40, 15, 8, 6)))
        segs.append(seg)
        stars.append(StarTree.build(SC.C4_SCHEMA, seg, SC.C4_SPLIT, SC.C4_PAIRS, max_leaf_records=300))
    t = GpuTable(SC.C4_SCHEMA)
    hs = [t.pin_segment(s) for s in segs]
    for h, st in zip(hs, stars):
        t.attach_startree(h, st)
    yield segs, stars, t, hs
    t.close()


@pytest.mark.parametrize("sql", SC.C4_QUERIES)
def test_startree_matches_oracles(oracle, c4_gpu, sql):
    segs, stars, t, hs = c4_gpu
    q = parse_query(sql, num_groups_limit=10 ** 9)
    got = t.execute_groupby(hs, q)
    # star-tree oracle, segment by segment: documents read off the star-tree
    docs = 0
    for seg, st in zip(segs, stars):
        _, d, _ = SC.startree_answer(oracle, seg, SC.C4_SCHEMA, st.arrays(), q, SC.C4_SPLIT, SC.C4_PAIRS)
        docs += d
    assert got.stats.num_docs_scanned == docs
    exp = oracle.run_groupby(SC.C4_SCHEMA, segs, q).groups
    _check(got, exp, q)
    # useStarTree=false: the scan path over the raw documents gives the same answer
    q.use_star_tree = False
    scan = t.execute_groupby(hs, q)
    _check(scan, exp, q)
    assert scan.stats.num_docs_scanned >= got.stats.num_docs_scanned


def test_startree_mixed_with_scan_segments(oracle, c4_gpu):
    """Segments without a star-tree run the scan path in the same plan (per-segment choice, as
    AggregationGroupByPlanNode.run makes it, core/plan/AggregationGroupByPlanNode.java:66-67)."""
    segs, stars, t, hs = c4_gpu
    rng = np.random.default_rng(9)
    plain = oracle.make_segment(SC.C4_SCHEMA, SC.c4_columns(rng, 25000, cards=(40, 15, 8, 6)))
    h = t.pin_segment(plain)
    try:
        q = parse_query(SC.C4_QUERIES[0], num_groups_limit=10 ** 9)
        got = t.execute_groupby(hs + [h], q)
        _check(got, oracle.run_groupby(SC.C4_SCHEMA, segs + [plain], q).groups, q)
    finally:
        t.unpin_segment(h)


def test_startree_large_key_space(oracle, c4_gpu):
    """Group by every dimension: a key space past the LDS table (global table mode)."""
    segs, stars, t, hs = c4_gpu
    q = parse_query("SELECT SUM(m), COUNT(*) FROM t WHERE d2 < 6 GROUP BY d1, d2, d3, d4", num_groups_limit=10 ** 9)
    got = t.execute_groupby(hs, q)
    _check(got, oracle.run_groupby(SC.C4_SCHEMA, segs, q).groups, q)


def test_startree_empty_match(oracle, c4_gpu):
    segs, stars, t, hs = c4_gpu
    q = parse_query("SELECT COUNT(*) FROM t WHERE d3 = 2 AND d3 = 3 GROUP BY d1", num_groups_limit=10 ** 9)
    got = t.execute_groupby(hs, q)
    assert len(got) == 0 and got.stats.num_docs_scanned == 0


def test_startree_from_pinot_files(oracle, c4_gpu, tmp_path):
    """A segment directory with Pinot's star-tree files (v1 -> v3), pinned and its star-tree loaded from the files
    alone (pgpu_startree_load + pgpu_attach_startree): same answers as the oracle's scan of the raw segment."""
    from pinot_amd import segment_files as SF
    from pinot_amd.startree import load_star_trees, write_star_tree_files
    segs, stars, _, _ = c4_gpu
    rng = np.random.default_rng(77)
    cols = SC.c4_columns(rng, 33333, cards=(40, 15, 8, 6))
    path = str(tmp_path / "seg")
    seg = SF.write_v1_segment_dir(path, SC.C4_SCHEMA, cols)
    bits = {n: seg.columns[n].bits_per_element for n, _ in SC.C4_SCHEMA}
    write_star_tree_files(path, [StarTree.build(SC.C4_SCHEMA, seg, SC.C4_SPLIT, SC.C4_PAIRS, max_leaf_records=250)],
                          bits, 250)
    v3 = SF.convert_v1_to_v3(path)
    loaded = SF.load_segment_dir(path)
    trees = load_star_trees(v3, SC.C4_SCHEMA, bits)
    t = GpuTable(SC.C4_SCHEMA)
    try:
        h = t.pin_segment(loaded)
        t.attach_startree(h, trees[0])
        for sql in SC.C4_QUERIES:
            q = parse_query(sql, num_groups_limit=10 ** 9)
            got = t.execute_groupby([h], q)
            _check(got, oracle.run_groupby(SC.C4_SCHEMA, [loaded], q).groups, q)
    finally:
        t.close()


def test_startree_malformed_nodes_rejected(c4_gpu):
    """The attach validates the node array and the documents' dictIds before anything reaches the device."""
    import ctypes
    from pinot_amd import _lib as L
    segs, stars, t, hs = c4_gpu
    a = stars[0].arrays()
    for field, value in ((5, 10 ** 6), (0, 99), (3, a["num_docs"] + 5), (4, -1)):
        d = stars[0].desc()
        nodes = a["nodes"].copy()
        nodes[min(1, len(nodes) - 1), field] = value
        buf = np.ascontiguousarray(nodes, dtype="<i4")
        d.nodes = buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        with pytest.raises(L.PinotGpuError) as e:
            L.check(t.lib.pgpu_attach_startree(t.handle, hs[0], ctypes.byref(d)))
        assert e.value.code == L.PGPU_ERR_INVALID_ARGUMENT
    # the segment's original star-tree is still attached and answers
    q = parse_query(SC.C4_QUERIES[0], num_groups_limit=10 ** 9)
    assert len(t.execute_groupby(hs[:1], q)) > 0


def test_star_metric_bytes_counted(c4_gpu):
    """K6 counts the 64-B sectors of the metric arrays that hold a matched document (the star path's line-granular
    bytes model, bench.py): 8-byte metric arrays (an int32 form is an A/B build option, PGPU_STAR_NARROW)."""
    segs, stars, t, hs = c4_gpu
    q = parse_query("SELECT SUM(m), COUNT(*), SUM(md) FROM t WHERE d3 IN (1, 5) GROUP BY d1, d2",
                    num_groups_limit=10 ** 9)
    with t.plan_execute(hs, q) as p:
        p.finalize()
        nseg, nodes, docs = p.star_work()
        mb = p.star_metric_bytes()
    assert nseg == len(hs) and docs > 0
    # per 16 star documents read, at most two 64-B sectors of each of the three arrays read
    assert 0 < mb <= (docs // 16 + 2 * len(hs) * 1000) * 64 * 6, (mb, docs)
    assert mb % 64 == 0
