"""Raw (no-dictionary) metric columns on the GPU: segments whose metric columns are FixedByteChunk PASS_THROUGH
forward indexes (FixedByteChunkSVForwardIndexReader.java:30-110) aggregate exactly as the oracle's operator reads
them (DataFetcher over ForwardIndexReader.readValuesSV); predicates and group-by on a raw column, and compressed
chunks, are declined (PGPU_ERR_UNSUPPORTED: Pinot's own operator runs them)."""
import numpy as np
import pytest

from pinot_amd import _lib as L
from pinot_amd.executor import GpuTable
from pinot_amd.query import parse_query
from pinot_amd.segment import SegmentBuffers, build_raw_column
from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

SCHEMA = [("d", "INT"), ("f", "INT"), ("m", "INT"), ("l", "LONG"), ("x", "DOUBLE"), ("y", "FLOAT")]


def _segments(oracle, sizes, version=2, seed=3):
    rng = np.random.default_rng(seed)
    segs = []
    for n in sizes:
        cols = {"d": rng.integers(0, 40, n).tolist(), "f": rng.integers(0, 1000, n).tolist()}
        base = oracle.make_segment([("d", "INT"), ("f", "INT")], cols)
        raw = {"m": build_raw_column("INT", rng.integers(-10 ** 6, 10 ** 6, n).tolist(), version),
               "l": build_raw_column("LONG", rng.integers(-2 ** 40, 2 ** 40, n).tolist(), version),
               "x": build_raw_column("DOUBLE", rng.normal(0, 1e3, n).tolist(), version),
               "y": build_raw_column("FLOAT", np.float32(rng.normal(0, 10, n)).astype(np.float64).tolist(), version)}
        segs.append(SegmentBuffers(n, {**base.columns, **raw}))
    return segs


@pytest.mark.parametrize("version", [2, 3])
def test_raw_metric_aggregations(oracle, gpu_lib, version):
    segs = _segments(oracle, [7001, 1, 33, 20000], version)
    t = GpuTable(SCHEMA)
    try:
        hs = [t.pin_segment(s) for s in segs]
        for sql in ["SELECT COUNT(*), SUM(m), MIN(m), MAX(m), SUM(l), MIN(l), AVG(x), MAX(x), MIN(y), SUM(y) "
                    "FROM t WHERE f < 300 GROUP BY d",
                    "SELECT SUM(m), MAX(l), MIN(x) FROM t GROUP BY d"]:
            q = parse_query(sql)
            o = oracle.run_groupby(SCHEMA, segs, q)
            r = t.execute_groupby(hs, q)
            assert_same(r, o, q, SCHEMA)
            assert r.stats.as_tuple() == o.stats
    finally:
        t.close()


def test_raw_minmax_only_is_a_scan(oracle, gpu_lib):
    """MIN / MAX over a match-all filter is answered from the dictionary only when there is one
    (AggregationPlanNode.java:196-213): over raw columns it is a scan, numEntriesScannedPostFilter > 0."""
    segs = _segments(oracle, [5000, 3000])
    t = GpuTable(SCHEMA)
    try:
        hs = [t.pin_segment(s) for s in segs]
        q = parse_query("SELECT MIN(m), MAX(x) FROM t")
        o = oracle.run_groupby(SCHEMA, segs, q)
        r = t.execute_aggregation(hs, q)
        assert r.stats.as_tuple() == o.stats and o.stats[2] == 2 * 8000
        (ov,) = o.groups.values()
        assert list(r.values) == list(ov)
    finally:
        t.close()


def test_raw_columns_declined_where_pinot_scans_raw_values(oracle, gpu_lib):
    segs = _segments(oracle, [100])
    t = GpuTable(SCHEMA)
    try:
        h = t.pin_segment(segs[0])
        for sql in ["SELECT COUNT(*) FROM t WHERE m > 5 GROUP BY d", "SELECT SUM(f) FROM t GROUP BY m"]:
            with pytest.raises(L.UnsupportedQueryError):
                t.execute_groupby([h], parse_query(sql))
        from dataclasses import replace
        bad = bytearray(segs[0].columns["m"].fwd_bytes)
        bad[20:24] = (1).to_bytes(4, "big")  # SNAPPY chunks
        seg = SegmentBuffers(100, {**segs[0].columns, "m": replace(segs[0].columns["m"], fwd_bytes=bytes(bad))})
        with pytest.raises(L.UnsupportedQueryError):
            t.pin_segment(seg)
    finally:
        t.close()
