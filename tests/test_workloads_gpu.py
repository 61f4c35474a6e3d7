"""GPU parity on the benchmarked data: every BASELINE.json configuration (pinot_amd/workloads.py: C1, C2, C3
AdAnalytics, C4 star-tree, C5 high-cardinality) built by the device generator (pgpu_generate_segment) exactly as
bench.py builds it, at the bench's segment size (1M docs) and a reduced segment count.

Each test checks, per segment and column, that the device-built dictionary and forward-index bytes equal the
oracle's generator (or_gen_i64 / or_gen_f64) followed by Pinot segment creation (or_build_column_*: sorted
dictionary + MSB-first fixed-bit forward index), and that the HIP query result equals the oracle's operator +
combine over the oracle-built bytes: bit-exact for COUNT / integer SUM / MIN / MAX, 1e-9 relative for the double
SUM (C2's md).  C4 (star-tree) is checked by the reference's star-tree == scan rule (BaseStarTreeV2Test.java:219-295).
"""
import numpy as np
import pytest

from pinot_amd import _lib as L
from pinot_amd.executor import GpuTable
from pinot_amd.query import parse_query
from pinot_amd.workloads import SEGMENT_DOCS, WORKLOADS

pytestmark = pytest.mark.gpu
REL = 1e-9

# workload -> segments (1M docs each) in the test
SIZES = {"c1": 1, "c2": 4, "adanalytics": 8, "adanalytics_inv": 4, "c5": 2, "c4": 3, "c5_hash": 2}


def _oracle_segments(oracle, w, nseg, docs, table=None, handles=None):
    """Oracle-built segments from the oracle's generator; when a table is given, also checks that the device-built
    bytes of every column equal them."""
    from pinot_amd.segment import SegmentBuffers
    segs = []
    for i in range(nseg):
        cols = {}
        for (name, typ), g in zip(w.schema, w.gen):
            vals = oracle.gen_values(g, i * docs, docs)
            cols[name] = oracle.build_column(L.TYPE_NAMES[typ], vals)
            if table is not None:
                card, bits, d, f = table.segment_column_bytes(handles[i], name)
                c = cols[name]
                assert (card, bits) == (c.cardinality, c.bits_per_element), (name, i)
                assert d == c.dict_bytes, "dictionary bytes of %s, segment %d" % (name, i)
                assert f == c.fwd_bytes, "forward-index bytes of %s, segment %d" % (name, i)
        segs.append(SegmentBuffers(docs, cols))
    return segs


def assert_same_arrays(table, r, orc, q, schema):
    """Same groups, bit-exact integer work, 1e-9 relative FP sums (_oracle.compare_result_arrays, which bench.py's
    full-size parity leg reports too)."""
    import _oracle
    res = _oracle.compare_result_arrays(table, r, orc, q, schema, rel=REL, check_stats=False)
    assert res["ok"], res


@pytest.mark.parametrize("name", ["c1", "c2", "adanalytics", "c5", "c5_hash"])
def test_workload_generator_and_query(oracle, gpu_lib, name):
    w = WORKLOADS[name]()
    nseg, docs = SIZES[name], SEGMENT_DOCS
    q = parse_query(w.sql, num_groups_limit=w.num_groups_limit)
    t = GpuTable(w.schema)
    try:
        hs = [t.generate_segment(w.gen, row0=i * docs, num_docs=docs) for i in range(nseg)]
        segs = _oracle_segments(oracle, w, nseg, docs, t, hs)
        if name == "c5_hash":  # the global hash table (a 10^9-key space), sized from the segments' group bound
            with t.plan(hs, q) as p:
                assert p.layout()[1] == 0
        r = t.execute_groupby(hs, q)
        o = oracle.run_groupby_arrays(w.schema, segs, q)
        assert len(r) == len(o[0]) > 0
        if name == "c5_hash":  # again from the plan cache: the table re-sized by the groups found
            r2 = t.execute_groupby(hs, q)
            assert_same_arrays(t, r2, o, q, w.schema)
        assert_same_arrays(t, r, o, q, w.schema)
        assert r.stats.as_tuple() == o[3]  # numEntriesScannedInFilter included (C3: AndDocIdIterator leap-frog)
    finally:
        t.close()


def test_workload_adanalytics_inverted_index(oracle, gpu_lib):
    """C3 over the production-style layout of bench.py --workload adanalytics_inv: bitmap inverted indexes on
    accountId built by the host creator from the device-built forward index; same answer as the oracle's scan."""
    from bench import attach_inverted_indexes
    w = WORKLOADS["adanalytics_inv"]()
    nseg, docs = SIZES["adanalytics_inv"], SEGMENT_DOCS
    q = parse_query(w.sql, num_groups_limit=w.num_groups_limit)
    t = GpuTable(w.schema)
    try:
        hs = [t.generate_segment(w.gen, row0=i * docs, num_docs=docs) for i in range(nseg)]
        attach_inverted_indexes(t, hs, w, docs)
        from dataclasses import replace
        from pinot_amd.segment import SegmentBuffers
        segs = [SegmentBuffers(docs, {**s.columns, "accountId": replace(s.columns["accountId"], inv_bytes=b"x")})
                for s in _oracle_segments(oracle, w, nseg, docs)]  # the oracle: BitmapBasedFilterOperator leaf
        r = t.execute_groupby(hs, q)
        o = oracle.run_groupby_arrays(w.schema, segs, q)
        assert_same_arrays(t, r, o, q, w.schema)
        assert r.stats.as_tuple() == o[3]
        # accountId = one dictId: its containers (BITMAP blocks and the ARRAY container of each segment's partial last
        # block) are read in place by the scan -- no per-query docId bitmap (inv_materialize_kernel)
        with t.plan(hs, q) as p:
            assert p.leaf_kinds().get("bitdir") == nseg and "bitmap" not in p.leaf_kinds(), p.leaf_kinds()
    finally:
        t.close()


def test_workload_c4_star_tree(oracle, gpu_lib):
    """C4: the star-tree path (per-segment star-trees built by the host builder from the device-built bytes, as
    bench.py does) gives the oracle's scan answer on the same data, and so does the scan path (useStarTree=false)."""
    from bench import attach_star_trees
    w = WORKLOADS["c4"]()
    nseg, docs = SIZES["c4"], SEGMENT_DOCS
    q = parse_query(w.sql, num_groups_limit=w.num_groups_limit)
    t = GpuTable(w.schema)
    try:
        hs = [t.generate_segment(w.gen, row0=i * docs, num_docs=docs) for i in range(nseg)]
        segs = _oracle_segments(oracle, w, nseg, docs, t, hs)
        attach_star_trees(t, hs, w, docs)
        o = oracle.run_groupby_arrays(w.schema, segs, q)
        r = t.execute_groupby(hs, q)
        assert_same_arrays(t, r, o, q, w.schema)
        # ... and the C star-tree operator's answer over the same trees, statistics included (numDocsScanned = star-tree
        # documents read, entries scanned in / post filter): StarTreeFilterOperator.java:185-226 +
        # StarTreeGroupByExecutor restated in oracle.c (run_star_segment)
        from pinot_amd.startree import StarTree
        spec = w.star_tree
        for seg in segs:
            st = StarTree.build(w.schema, seg, spec["split_order"], spec["pairs"], spec["max_leaf_records"])
            seg.star_arrays = st.arrays()
            st.close()
        o_star = oracle.run_groupby_arrays(w.schema, segs, q, use_star_tree=True)
        res = oracle.compare_result_arrays(t, r, o_star, q, w.schema, rel=REL, check_stats=True)
        assert res["ok"], res
        q.use_star_tree = False
        rs = t.execute_groupby(hs, q)
        assert_same_arrays(t, rs, o, q, w.schema)
        # the scan path reads every doc; the star-tree path reads pre-aggregated documents only
        assert rs.stats.num_docs_scanned == o[3][0]
        assert r.stats.num_docs_scanned < rs.stats.num_docs_scanned
    finally:
        t.close()
