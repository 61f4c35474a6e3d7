"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the reference KATs.

Bar: bit-exact for COUNT, integer SUM/MIN/MAX, AVG counts, dictIds and filter bitmaps; 1e-9 relative error
for sums over FLOAT/DOUBLE columns (the reference sums doubles in a thread-order-dependent order).
"""
import ctypes

import numpy as np
import pytest

import kat_common as K
from pinot_amd import _lib as L
from pinot_amd.executor import AvgPair, GpuTable
from pinot_amd.query import FilterContext, Predicate, QueryContext, parse_query

pytestmark = pytest.mark.gpu
REL = 1e-9


def assert_same(gpu, orc, q, schema):
    types = dict(schema)
    g = gpu.as_dict()
    assert set(g) == set(orc.groups), (sorted(set(g) ^ set(orc.groups))[:5])
    for k, ov in orc.groups.items():
        gv = g[k]
        for a, (fn, col) in enumerate(q.aggregations):
            fp = col != "*" and types[col] in ("FLOAT", "DOUBLE")
            x, y = gv[a], ov[a]
            if isinstance(y, AvgPair):
                assert x.count == y.count, (k, fn)
                if fp:
                    assert x.sum == pytest.approx(y.sum, rel=REL, abs=1e-6), (k, fn)
                else:
                    assert x.sum == y.sum, (k, fn)
            elif fp and fn == "SUM":
                assert x == pytest.approx(y, rel=REL, abs=1e-6), (k, fn)
            else:
                assert x == y, (k, fn, x, y)


def gpu_table(schema, segments, config=None):
    t = GpuTable(schema, config=config)
    handles = [t.pin_segment(s) for s in segments]
    return t, handles


# ------------------------------------------------------------------------------------------------ KATs
@pytest.fixture(scope="module")
def sv(oracle, gpu_lib):
    """The KAT segment with the reference's index layout: the oracle reads its fixed-bit view with the sorted
    flags, the GPU pins column5 / daysSinceEpoch as SortedIndexReaderImpl pairs."""
    seg = K.kat_segment(oracle)
    t, hs = gpu_table(K.SCHEMA, [K.kat_segment(oracle, pairs=True)])
    yield seg, t, hs[0]
    t.close()


@pytest.mark.parametrize("case", K.KAT["inner_segment_group_by"][:3], ids=lambda c: c["holder"])
@pytest.mark.parametrize("with_filter", [False, True], ids=["no_filter", "filter"])
def test_kat_inner_segment(oracle, sv, case, with_filter):
    seg, t, h = sv
    q = K.inner_query(case["group_by"], with_filter)
    r = t.execute_groupby([h], q)
    exp = case["filter" if with_filter else "no_filter"]
    assert r.stats.as_tuple() == tuple(exp["stats"])  # numEntriesScannedInFilter 84134 with the filter
    key = K.key_tuple(case["group_by"], exp["key"])
    K.check_inner_values(r.as_dict()[key], exp["values"])
    assert_same(r, oracle.run_groupby(K.SCHEMA, [seg], q, combine=False), q, K.SCHEMA)


@pytest.mark.parametrize("with_filter", [False, True], ids=["no_filter", "filter"])
def test_kat_array_map_holder(oracle, sv, with_filter):
    """VERY_LARGE_GROUP_BY (InnerSegmentAggregationSingleValueQueriesTest.java:194-219): 9 group-by columns whose
    cardinality product overflows a long -- Pinot's ArrayMapBasedHolder.  The GPU maps consecutive column groups to
    dense slot ids through hash-table stages (KParams.num_stages) and must give the KAT's statistics and values and
    the oracle's every group."""
    seg, t, h = sv
    case = K.KAT["inner_segment_group_by"][3]
    q = K.inner_query(case["group_by"], with_filter)
    q.num_groups_limit = 10 ** 9
    r = t.execute_groupby([h], q)
    exp = case["filter" if with_filter else "no_filter"]
    assert r.stats.as_tuple() == tuple(exp["stats"])
    key = K.key_tuple(case["group_by"], exp["key"])
    K.check_inner_values(r.as_dict()[key], exp["values"])
    assert_same(r, oracle.run_groupby(K.SCHEMA, [seg], q, combine=False), q, K.SCHEMA)


def test_array_map_with_groups_limit(oracle, sv):
    """The ARRAY_MAP shape under the default numGroupsLimit (100000 > 30000 docs: nothing truncated) and a binding
    limit (first-seen truncation of the map holder, DictionaryBasedGroupKeyGenerator.java:1101-1113)."""
    seg, t, h = sv
    case = K.KAT["inner_segment_group_by"][3]
    for limit in (100_000, 1000):
        q = K.inner_query(case["group_by"], False)
        q.num_groups_limit = limit
        r = t.execute_groupby([h], q)
        o = oracle.run_groupby(K.SCHEMA, [seg], q, combine=False, max_initial_capacity=min(limit, 10_000))
        assert_same(r, o, q, K.SCHEMA)
        if limit < 26_993:  # the segment holds 26993 distinct 9-column groups
            assert len(r) == limit


@pytest.mark.parametrize("with_filter", [False, True])
def test_kat_aggregation_totals(sv, with_filter):
    seg, t, h = sv
    r = t.execute_groupby([h], K.inner_query(["column5"], with_filter))
    exp = K.KAT["inner_segment_aggregation_only"]["filter" if with_filter else "no_filter"]
    K.check_inner_values(r.as_dict()[("gFuH",)], exp["values"])


@pytest.mark.parametrize("case", K.KAT["inter_segment_group_by"], ids=lambda c: "_".join(c["group_by"]))
def test_kat_inter_segment(oracle, sv, case):
    seg, t, h = sv
    handles = [h] * K.KAT["inter_segment_num_segments"]
    q = QueryContext(case["group_by"], [tuple(a) for a in case["aggs"]])
    r = t.execute_groupby(handles, q)
    assert r.stats.as_tuple() == tuple(case["stats"])
    got = r.as_dict()
    rows = {K.key_tuple(case["group_by"], k): v for k, v in case["rows"]}
    if case["complete"]:
        assert set(got) == set(rows)
    for k, v in rows.items():
        assert [float(x) for x in got[k]] == [float(x) for x in v], k


def test_kat_sql_string_filter(oracle, sv):
    """The reference's filter string parsed by the PQL/SQL subset parser gives the same answer."""
    seg, t, h = sv
    sql = ("SELECT COUNT(*), SUM(column1), MAX(column3), MIN(column6), AVG(column7) FROM testTable "
           "WHERE column1 > 100000000 AND column3 BETWEEN 20000000 AND 1000000000 AND column5 = 'gFuH' "
           "AND (column6 < 500000000 OR column11 NOT IN ('t', 'P')) AND daysSinceEpoch = 126164076 GROUP BY column9")
    q = parse_query(sql)
    r = t.execute_groupby([h], q)
    exp = K.KAT["inner_segment_group_by"][0]["filter"]
    K.check_inner_values(r.as_dict()[(242920,)], exp["values"])
    assert r.stats.as_tuple() == tuple(exp["stats"])


def test_bad_literal_is_bad_query(sv):
    seg, t, h = sv
    q = QueryContext(["column9"], [("COUNT", "*")], FilterContext.pred(Predicate.eq("column1", "abc")))
    with pytest.raises(L.BadQueryRequestException):
        t.execute_groupby([h], q)


# ------------------------------------------------------------------------------------------------ randomized
def _random_segment(oracle, rng, schema, n):
    cols = {}
    for name, typ in schema:
        card = int(rng.integers(1, 3000))
        if typ == "INT":
            dom = rng.integers(-2 ** 31, 2 ** 31, size=card)
        elif typ == "LONG":
            dom = rng.integers(-2 ** 50, 2 ** 50, size=card)
        elif typ == "DOUBLE":
            dom = rng.uniform(-1e6, 1e6, size=card)
        elif typ == "FLOAT":
            dom = rng.uniform(-1e3, 1e3, size=card).astype(np.float32).astype(np.float64)
        else:
            dom = np.array(["s%05d" % i for i in rng.integers(0, 5000, size=card)])
        pick = rng.integers(0, card, size=n)
        cols[name] = [str(x) for x in dom[pick]] if typ == "STRING" else dom[pick]
    return oracle.make_segment(schema, cols)


SCHEMA_R = [("a", "INT"), ("b", "INT"), ("c", "LONG"), ("d", "DOUBLE"), ("e", "STRING"), ("f", "FLOAT")]


def _some_value(seg, col, rng):
    c = seg.columns[col]
    i = int(rng.integers(0, c.cardinality))
    w = c.entry_width
    raw = c.dict_bytes[i * w:(i + 1) * w]
    if c.data_type == L.INT:
        return str(int.from_bytes(raw, "big", signed=True))
    if c.data_type == L.LONG:
        return str(int.from_bytes(raw, "big", signed=True))
    if c.data_type == L.DOUBLE:
        return repr(float(np.frombuffer(raw, dtype=">f8")[0]))
    if c.data_type == L.FLOAT:
        return repr(float(np.frombuffer(raw, dtype=">f4")[0]))
    return raw.rstrip(b"\0").decode()


def _random_filter(rng, seg, depth=0):
    if depth < 2 and rng.random() < 0.4:
        kids = [_random_filter(rng, seg, depth + 1) for _ in range(int(rng.integers(2, 4)))]
        r = rng.random()
        f = FilterContext.and_(*kids) if r < 0.5 else FilterContext.or_(*kids)
        return FilterContext.not_(f) if rng.random() < 0.15 else f
    col = ["a", "b", "c", "d", "e", "f"][int(rng.integers(0, 6))]
    kind = int(rng.integers(0, 5))
    v1, v2 = _some_value(seg, col, rng), _some_value(seg, col, rng)
    if kind == 0:
        return FilterContext.pred(Predicate.eq(col, v1))
    if kind == 1:
        return FilterContext.pred(Predicate.not_eq(col, v1))
    if kind == 2:
        return FilterContext.pred(Predicate.in_(col, [v1, v2, _some_value(seg, col, rng)]))
    if kind == 3:
        return FilterContext.pred(Predicate.not_in(col, [v1, v2]))
    if col == "e":
        lo, hi = sorted([v1, v2])
    else:
        lo, hi = sorted([v1, v2], key=float)
    return FilterContext.pred(Predicate.range(col, lo if rng.random() < 0.8 else "*", hi if rng.random() < 0.8 else "*",
                                              bool(rng.random() < 0.5), bool(rng.random() < 0.5)))


@pytest.mark.parametrize("seed", list(range(12)))
def test_random_queries_vs_oracle(oracle, gpu_lib, seed):
    # odd seeds: streamed plans -- every segment its own launch, planned while the previous ones run
    cfg = {"stream_chunks": 4} if seed % 2 else None
    rng = np.random.default_rng(1000 + seed)
    nseg = int(rng.integers(1, 5))
    segs = [_random_segment(oracle, rng, SCHEMA_R, int(rng.integers(1, 40000))) for _ in range(nseg)]
    t, hs = gpu_table(SCHEMA_R, segs, cfg)
    try:
        for qi in range(4):
            gb = list(rng.choice(["a", "b", "e", "c"], size=int(rng.integers(1, 3)), replace=False))
            aggs = [("COUNT", "*"), ("SUM", "a"), ("MIN", "d"), ("MAX", "c"), ("AVG", "f"), ("SUM", "d"),
                    ("MAX", "f"), ("MIN", "b")]
            flt = _random_filter(rng, segs[0]) if qi % 3 != 0 else None
            q = QueryContext(gb, aggs, flt, num_groups_limit=10 ** 9)
            r = t.execute_groupby(hs, q)
            o = oracle.run_groupby(SCHEMA_R, segs, q, combine=False, max_initial_capacity=10000)
            assert_same(r, o, q, SCHEMA_R)
            assert r.stats.as_tuple() == o.stats, (q.filter, r.stats, o.stats)
    finally:
        t.close()


@pytest.mark.parametrize("n", [0, 1, 31, 32, 33, 8191, 8192, 8193, 70001])
def test_ragged_segment_sizes(oracle, gpu_lib, n):
    rng = np.random.default_rng(n)
    schema = [("g", "INT"), ("v", "INT")]
    seg = oracle.make_segment(schema, {"g": rng.integers(0, 7, size=n), "v": rng.integers(0, 1000, size=n)})
    t, hs = gpu_table(schema, [seg, seg])
    try:
        q = parse_query("SELECT COUNT(*), SUM(v) FROM t WHERE v >= 100 GROUP BY g")
        r = t.execute_groupby(hs, q)
        o = oracle.run_groupby(schema, [seg, seg], q)
        assert_same(r, o, q, schema)
        if n > 0:
            bm = t.filter_bitmap(hs[0], q, n)
            ob = oracle.filter_bitmap(schema, seg, q)
            np.testing.assert_array_equal(bm, ob)
    finally:
        t.close()


@pytest.mark.parametrize("nbits_card", [2, 3, 17, 255, 256, 5000, 70000, 2 ** 20 + 7])
def test_read_dict_ids_every_width(oracle, gpu_lib, nbits_card):
    rng = np.random.default_rng(nbits_card)
    n = 50000
    vals = rng.integers(0, nbits_card, size=n)
    m = min(nbits_card, n)
    vals[:m] = np.arange(m)
    seg = oracle.make_segment([("x", "INT")], {"x": vals})
    t, hs = gpu_table([("x", "INT")], [seg])
    try:
        docs = np.sort(rng.choice(n, 5000, replace=False)).astype(np.int32)
        got = t.read_dict_ids(hs[0], "x", docs)
        o = oracle.lib()
        c = seg.columns["x"]
        buf = np.frombuffer(c.fwd_bytes + b"\0" * 16, dtype=np.uint8).copy()
        exp = np.zeros(len(docs), dtype=np.int32)
        o.or_read_dict_ids(buf.ctypes.data, c.bits_per_element, n, docs.ctypes.data, len(docs), exp.ctypes.data)
        np.testing.assert_array_equal(got, exp)
    finally:
        t.close()


def test_unpack_device_with_torch(oracle, gpu_lib):
    import torch
    rng = np.random.default_rng(5)
    for bits in (1, 7, 9, 16, 17, 23, 31):
        n = 100003
        vals = rng.integers(0, 1 << bits, size=n).astype(np.int32)
        buf = np.zeros(oracle.lib().or_fwd_num_bytes(n, bits) + 16, dtype=np.uint8)
        oracle.lib().or_bitset_write_ints(buf.ctypes.data, 0, bits, n, vals.ctypes.data)
        d_fwd = torch.from_numpy(buf).cuda()
        d_out = torch.empty(n - 5, dtype=torch.int32, device="cuda")
        L.check(gpu_lib.pgpu_unpack_fixed_bit_device(ctypes.c_void_p(d_fwd.data_ptr()), len(buf), bits, 5, n - 5,
                                                     ctypes.c_void_p(d_out.data_ptr()), None))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d_out.cpu().numpy(), vals[5:])


def test_sorted_forward_index_format(oracle, gpu_lib):
    """SortedIndexReaderImpl pairs (sorted columns, e.g. daysSinceEpoch in the KAT segment) pin correctly."""
    from pinot_amd.segment import ColumnData, SegmentBuffers
    vals = np.repeat(np.arange(5), [3, 0, 4, 1, 2])[:10]
    seg = oracle.make_segment([("s", "INT"), ("v", "INT")], {"s": vals * 10, "v": np.arange(10)})
    c = seg.columns["s"]
    ids = np.unique(vals, return_inverse=True)[1]
    pairs = b"".join(int(np.where(ids == i)[0][0]).to_bytes(4, "big") + int(np.where(ids == i)[0][-1]).to_bytes(4, "big")
                     for i in range(c.cardinality))
    sorted_seg = SegmentBuffers(10, {"s": ColumnData(c.data_type, c.cardinality, c.bits_per_element, 4, c.dict_bytes,
                                                     pairs, fwd_format=L.FWD_SORTED_PAIRS),
                                     "v": seg.columns["v"]})
    t, hs = gpu_table([("s", "INT"), ("v", "INT")], [sorted_seg])
    try:
        r = t.execute_groupby(hs, parse_query("SELECT SUM(v), COUNT(*) FROM t GROUP BY s"))
        o = oracle.run_groupby([("s", "INT"), ("v", "INT")], [seg],
                               parse_query("SELECT SUM(v), COUNT(*) FROM t GROUP BY s"))
        assert r.as_dict() == o.groups
    finally:
        t.close()


def test_padding_segments_pin_and_query(gpu_lib, tmp_path):
    """Real Pinot-written v1 segments (padding*.tar.gz) pin and answer like the oracle reading the same bytes."""
    import json
    import os
    from pinot_amd.segment import ColumnData, SegmentBuffers
    segs = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "padding_segments.json")))
    for name, s in segs.items():
        pad = 0 if "u0000" in s["paddingCharacter"] else ord(s["paddingCharacter"][0])
        cols = {}
        schema = []
        for col, c in s["columns"].items():
            typ = c["dataType"]
            width = {"INT": 4, "FLOAT": 4, "LONG": 8, "DOUBLE": 8}.get(typ, c["lengthOfEachEntry"])
            cols[col] = ColumnData(L.TYPE_NAMES[typ], c["cardinality"], c["bitsPerElement"], width,
                                   bytes.fromhex(c["dict_hex"]), bytes.fromhex(c["fwd_hex"]),
                                   pad if typ == "STRING" else 0)
            schema.append((col, typ))
        t, hs = gpu_table(schema, [SegmentBuffers(s["totalDocs"], cols)])
        try:
            r = t.execute_groupby(hs, parse_query("SELECT SUM(age), COUNT(*) FROM t GROUP BY name"))
            got = {k[0]: v for k, v in r.as_dict().items()}
            assert sum(v[1] for v in got.values()) == 5
            assert got["lynda"][1] == 2 and got["lynda 2.0"][1] == 3
            ages = {617, 824, 837, 1209, 1228}
            assert sum(v[0] for v in got.values()) == float(sum(ages))
            r2 = t.execute_groupby(hs, parse_query("SELECT COUNT(*) FROM t WHERE name = 'lynda' GROUP BY age"))
            assert sum(v[0] for v in r2.as_dict().values()) == 2
        finally:
            t.close()


@pytest.mark.parametrize("nseg", [1, 4])
@pytest.mark.parametrize("sql", [False, True], ids=["pql", "sql"])
@pytest.mark.parametrize("with_filter", [False, True], ids=["no_filter", "filter"])
def test_num_groups_limit_first_seen(oracle, sv, nseg, sql, with_filter):
    """InterSegmentAggregationSingleValueQueriesTest.java:534-545: GROUP BY column1 with numGroupsLimit 1000 (and
    maxInitialResultHolderCapacity 1000).  column1's key space exceeds the limit, so each segment keeps the first
    1000 groups of its matching docs in docId order (IntGroupIdMap, DictionaryBasedGroupKeyGenerator.java:
    1101-1113) and drops the docs of later groups; numGroupsLimitReached is set in PQL mode."""
    seg, t, h = sv
    flt = K.inner_query(["column1"], True).filter if with_filter else None
    q = QueryContext(["column1"], [("COUNT", "*"), ("SUM", "column3"), ("MIN", "column6")], flt,
                     num_groups_limit=1000, sql_group_by=sql)
    o = oracle.run_groupby(K.SCHEMA, [seg] * nseg, q, combine=not sql, max_initial_capacity=1000)
    r = t.execute_groupby([h] * nseg, q)
    assert_same(r, o, q, K.SCHEMA)
    assert r.stats.as_tuple() == o.stats
    if not with_filter:
        assert len(r) == 1000
    assert r.num_groups_limit_reached == (not sql and len(r) >= 1000)
    if not sql:
        assert r.num_groups_limit_reached == o.limit_reached


@pytest.mark.parametrize("sql", [False, True], ids=["pql", "sql"])
def test_num_groups_limit_inter_segment_cap(oracle, sql):
    """Segments with disjoint keys: each keeps its first 1000 groups; the PQL combine admits 2 x 1000 groups in
    total (GroupByCombineOperator.java:61,78-80,138) -- segment by segment, as the oracle's single-threaded
    combine does -- while SQL mode keeps all 3 x 1000."""
    schema = [("k", "INT"), ("m", "INT")]
    rng = np.random.default_rng(7)
    segs = [oracle.make_segment(schema, {"k": (i * 100000 + rng.integers(0, 3000, 6000)).tolist(),
                                         "m": rng.integers(0, 1000, 6000).tolist()}) for i in range(3)]
    q = QueryContext(["k"], [("COUNT", "*"), ("SUM", "m"), ("MAX", "m")], None, num_groups_limit=1000,
                     sql_group_by=sql)
    o = oracle.run_groupby(schema, segs, q, combine=not sql, max_initial_capacity=1000)
    t, hs = gpu_table(schema, segs)
    try:
        r = t.execute_groupby(hs, q)
        assert_same(r, o, q, schema)
        assert len(r) == (3000 if sql else 2000)
        assert r.stats.as_tuple() == o.stats
    finally:
        t.close()


def test_num_groups_limit_not_reached_is_exact(oracle, sv):
    """A limit below the segment's key space but above the groups the filter leaves: no truncation happens in
    Pinot, and the GPU result equals the oracle's under the same limit."""
    seg, t, h = sv
    flt = K.inner_query(["column9"], True).filter
    q0 = QueryContext(["column9"], [("COUNT", "*"), ("SUM", "column1")], flt, num_groups_limit=10 ** 9)
    ngroups = len(oracle.run_groupby(K.SCHEMA, [seg], q0).groups)
    q = QueryContext(["column9"], [("COUNT", "*"), ("SUM", "column1")], flt, num_groups_limit=ngroups + 1)
    assert seg.columns["column9"].cardinality > ngroups
    o = oracle.run_groupby(K.SCHEMA, [seg], q, max_initial_capacity=min(10000, ngroups + 1))
    assert not o.limit_reached
    r = t.execute_groupby([h], q)
    assert_same(r, o, q, K.SCHEMA)


@pytest.mark.parametrize("partitioned", [True, False], ids=["partitioned", "atomics"])
@pytest.mark.parametrize("docs", [1, 4097, 150_000])
def test_high_cardinality_ordered_compaction(oracle, gpu_lib, docs, partitioned):
    """C5 shape (3-column composite key over a ~10^6 key space, INT_MAP holder in Pinot): the dense global table
    -- built by the partitioned group-by (partition.h) or by global atomics -- and its ordered device compaction
    (count / scan / scatter) give the oracle's groups in ascending key order, across chunk boundaries and with
    fewer docs than keys."""
    rng = np.random.default_rng(docs)
    schema = [("k1", "INT"), ("k2", "INT"), ("k3", "INT"), ("m", "INT"), ("x", "DOUBLE"), ("n", "INT"), ("l", "LONG"),
              ("q", "INT"), ("r", "INT")]
    segs = []
    for _ in range(2):
        segs.append(oracle.make_segment(schema, {"k1": rng.integers(0, 400, size=docs),
                                                 "k2": rng.integers(0, 60, size=docs),
                                                 "k3": rng.integers(0, 50, size=docs),
                                                 "m": rng.integers(0, 1000, size=docs),
                                                 "x": rng.uniform(-1e6, 1e6, size=docs),
                                                 "n": rng.integers(-2 ** 31, 2 ** 31, size=docs),
                                                 "l": rng.integers(-2 ** 40, 2 ** 40, size=docs),
                                                 "q": rng.integers(-500, 500, size=docs),
                                                 "r": rng.integers(-200000, 200000, size=docs)}))
    t, hs = gpu_table(schema, segs, None if partitioned else {"partitioned_group_by": 0})
    try:
        q = parse_query("SELECT SUM(m), COUNT(*), MIN(x), MAX(m), AVG(x) FROM t GROUP BY k1, k2, k3",
                        num_groups_limit=10 ** 7)
        r = t.execute_groupby(hs, q)
        rf = t.execute_groupby(hs, parse_query("SELECT COUNT(*), SUM(m), MIN(m), MAX(x), SUM(x) FROM t WHERE m < 500 OR x > 0 "
                                               "GROUP BY k1, k2, k3", num_groups_limit=10 ** 7))
        qf = parse_query("SELECT COUNT(*), SUM(m), MIN(m), MAX(x), SUM(x) FROM t WHERE m < 500 OR x > 0 GROUP BY k1, k2, k3",
                         num_groups_limit=10 ** 7)
        assert_same(rf, oracle.run_groupby(schema, segs, qf, combine=False, max_initial_capacity=10000), qf, schema)
        o = oracle.run_groupby(schema, segs, q, combine=False, max_initial_capacity=10000)
        assert_same(r, o, q, schema)
        g = r.gids.astype(np.int64)  # key = d0 + d1*c0 + d2*c0*c1 (DictionaryBasedGroupKeyGenerator.java:276-323)
        comp = (g[:, 2] * 10 ** 6 + g[:, 1]) * 10 ** 6 + g[:, 0]
        assert np.all(np.diff(comp) > 0)
        # integer streams only: int32 values (full range, negative included) ride in 4-byte records
        # (KPartParams.val32); a LONG stream beyond int32 keeps 8-byte records; a single stream of narrow range is
        # packed above the key bits of the coarse records (KPartParams.pack_bits), negative values included
        for sql in ("SELECT SUM(m), COUNT(*) FROM t GROUP BY k1, k2, k3",
                    "SELECT SUM(q), MIN(q), MAX(q), COUNT(*) FROM t GROUP BY k1, k2, k3",
                    "SELECT MIN(n), MAX(n), SUM(n) FROM t GROUP BY k1, k2, k3",
                    "SELECT SUM(n), MIN(n), MAX(m), COUNT(*) FROM t GROUP BY k1, k2, k3",
                    "SELECT SUM(l), MAX(l), MIN(n), COUNT(*) FROM t GROUP BY k1, k2, k3",
                    # packed records of filtered docs: K8c's staged write-out with partial lane masks
                    "SELECT SUM(m), COUNT(*) FROM t WHERE q < 0 OR m > 900 GROUP BY k1, k2, k3",
                    "SELECT COUNT(*) FROM t GROUP BY k1, k2, k3",  # no value stream at all
                    # sums past 16 bits and within 24, negative included: 3-byte words in the compact result form
                    "SELECT SUM(r), MIN(r), COUNT(*) FROM t GROUP BY k1, k2, k3"):
            qi = parse_query(sql, num_groups_limit=10 ** 7)
            assert_same(t.execute_groupby(hs, qi),
                        oracle.run_groupby(schema, segs, qi, combine=False, max_initial_capacity=10000), qi, schema)
    finally:
        t.close()


def test_finalize_key_range_shards(oracle, gpu_lib):
    """pgpu_plan_finalize_range over the key-range shards a reduce-scatter leaves on each rank: the union of the
    shards' groups is the whole table's result (the multi-GPU combine of large key spaces, combine.py)."""
    import torch
    from pinot_amd.combine import shard_range
    rng = np.random.default_rng(7)
    schema = [("a", "INT"), ("b", "INT"), ("m", "INT")]
    n = 120_000
    seg = oracle.make_segment(schema, {"a": rng.integers(0, 300, n), "b": rng.integers(0, 200, n),
                                       "m": rng.integers(0, 1000, n)})
    t, hs = gpu_table(schema, [seg])
    try:
        q = parse_query("SELECT COUNT(*), SUM(m) FROM t WHERE m < 900 GROUP BY a, b", num_groups_limit=10 ** 6)
        torch.cuda.set_stream(torch.cuda.Stream())  # a real stream (handle 0 is the table's own to the C ABI)
        stream = torch.cuda.current_stream().cuda_stream
        with t.plan(hs, q) as plan:
            nslots, nkeys, kinds = plan.layout()
            d = torch.empty((nslots, nkeys), dtype=torch.int64, device="cuda")
            plan.execute(stream, d.data_ptr())
            full = plan.finalize(stream, d.data_ptr())
            merged = {}
            for r in range(3):
                k0, kn, _ = shard_range(nkeys, 3, r)
                shard = d[:, k0:k0 + kn].contiguous()
                part = plan.finalize_range(stream, shard.data_ptr(), k0, kn)
                assert not (set(part.as_dict()) & set(merged))
                merged.update(part.as_dict())
        assert merged == full.as_dict()
        o = oracle.run_groupby(schema, [seg], q, combine=False, max_initial_capacity=10000)
        assert_same(full, o, q, schema)
    finally:
        t.close()


@pytest.mark.parametrize("chunk", [0, 64], ids=["one_thread", "chunks_of_64"])
@pytest.mark.parametrize("launches", [1, 4, 7])
def test_many_segments_chunked_planning(oracle, gpu_lib, chunk, launches):
    """Plans over hundreds of segments translate their predicates in parallel chunks (host worker pool); the
    concatenated records (tile offsets, IN-set bitsets) must give the oracle's combined result, including
    segments the filter prunes (EmptyFilterOperator) in the middle of a chunk."""
    cfg = {"stream_chunks": launches}
    if chunk:
        cfg["plan_chunk_segments"] = chunk
    rng = np.random.default_rng(11)
    schema = [("g", "INT"), ("f", "INT"), ("v", "LONG")]
    segs = []
    for i in range(300):
        n = int(rng.integers(1, 3000))
        lo = 0 if i % 7 else 5000  # every 7th segment has no f value below 5000: pruned by the range leaf
        segs.append(oracle.make_segment(schema, {"g": rng.integers(0, 40, n), "f": rng.integers(lo, lo + 200, n),
                                                 "v": rng.integers(-10 ** 9, 10 ** 9, n)}))
    t, hs = gpu_table(schema, segs, cfg)
    try:
        q = parse_query("SELECT COUNT(*), SUM(v), MIN(v) FROM t WHERE f < 150 AND g IN (1, 3, 5, 17, 39) GROUP BY g")
        r = t.execute_groupby(hs, q)
        o = oracle.run_groupby(schema, segs, q)
        assert_same(r, o, q, schema)
        assert r.stats.num_docs_scanned == o.stats[0]
        assert r.stats.num_segments_matched == sum(1 for i in range(300) if i % 7)
    finally:
        t.close()


@pytest.mark.parametrize("magnitude", [2 ** 60, 2 ** 44], ids=["past_int64", "past_2^53"])
def test_long_sum_overflow_guard(oracle, gpu_lib, magnitude):
    """SUM / AVG over a LONG column whose sum could leave int64 (values near 2^60 over 20k docs) accumulate the
    values' doubles instead of wrapping; sums between 2^53 and 2^62 stay exact int64.  Pinot sums doubles in doc
    order (SumAggregationFunction.java:66-73), so both match the oracle within the double-sum tolerance."""
    rng = np.random.default_rng(magnitude % 1000)
    schema = [("g", "INT"), ("x", "LONG")]
    n = 20_000
    segs = [oracle.make_segment(schema, {"g": rng.integers(0, 5, n),
                                         "x": rng.integers(magnitude // 2, magnitude, n)}) for _ in range(2)]
    t, hs = gpu_table(schema, segs)
    try:
        for sql in ("SELECT SUM(x), AVG(x), COUNT(*), MAX(x) FROM t GROUP BY g", "SELECT SUM(x), MIN(x) FROM t"):
            q = parse_query(sql)
            r = t.execute_groupby(hs, q)
            o = oracle.run_groupby(schema, segs, q)
            g = r.as_dict()
            assert set(g) == set(o.groups)
            for k, ov in o.groups.items():
                for (fn, _), x, y in zip(q.aggregations, g[k], ov):
                    if fn == "AVG":
                        assert x.count == y.count and x.sum == pytest.approx(y.sum, rel=REL)
                    elif fn == "SUM":
                        assert x == pytest.approx(y, rel=REL)
                        assert abs(x) > 2 ** 53
                    else:
                        assert x == y
    finally:
        t.close()


# ------------------------------------------------------------------------------------------------ aggregation-only
@pytest.mark.parametrize("case", K.KAT_AGG["cases"], ids=lambda c: "%s_%s" % (c["test"], c["variant"]))
def test_kat_inter_segment_aggregation(sv, case):
    """InterSegmentAggregationSingleValueQueriesTest SUM/COUNT/MIN/MAX/AVG (4 segments), aggregation-only and
    GROUP BY column9, values and statistics, through the GPU path."""
    seg, t, h = sv
    q = K.agg_case_query(case)
    if q.group_by:
        r = t.execute_groupby([h] * 4, q)
        values = K.top_group_values(q, r.values)
    else:
        r = t.execute_aggregation([h] * 4, q)
        values = r.values
    K.check_agg_case(case, q, r.stats.as_tuple(), values)


@pytest.mark.parametrize("seed", list(range(6)))
def test_random_aggregation_only_vs_oracle(oracle, gpu_lib, seed):
    """Aggregation-only queries (single-row table, wave-folded accumulation) against the oracle, dense and sparse
    filters, including filters that match nothing (the functions' defaults)."""
    from pinot_amd.executor import aggregation_defaults
    rng = np.random.default_rng(2000 + seed)
    segs = [_random_segment(oracle, rng, SCHEMA_R, int(rng.integers(1, 60000))) for _ in range(int(rng.integers(1, 4)))]
    t, hs = gpu_table(SCHEMA_R, segs)
    try:
        for qi in range(5):
            aggs = [("COUNT", "*"), ("SUM", "a"), ("MIN", "d"), ("MAX", "c"), ("AVG", "f"), ("SUM", "d"), ("MIN", "b")]
            flt = None if qi == 0 else _random_filter(rng, segs[0])
            if qi == 4:
                flt = FilterContext.and_(FilterContext.pred(Predicate.eq("a", "1")),
                                         FilterContext.pred(Predicate.not_eq("a", "1")))
            q = QueryContext([], aggs, flt)
            r = t.execute_aggregation(hs, q)
            o = oracle.run_groupby(SCHEMA_R, segs, q)
            exp = o.groups[()] if o.groups else aggregation_defaults(aggs)
            for (fn, col), x, y in zip(aggs, r.values, exp):
                fp = col != "*" and dict(SCHEMA_R)[col] in ("FLOAT", "DOUBLE")
                if fn == "AVG":
                    assert x.count == y.count
                    assert x.sum == pytest.approx(y.sum, rel=REL, abs=1e-6)
                elif fp and fn == "SUM":
                    assert x == pytest.approx(y, rel=REL, abs=1e-6)
                else:
                    assert x == y, (fn, col, x, y)
            assert r.stats.as_tuple() == o.stats, (q.filter, r.stats, o.stats)
    finally:
        t.close()


def test_aggregation_only_operators(sv):
    """GpuAggregationOperator / GpuAggregationOnlyCombineOperator return Pinot's aggregation result list."""
    from pinot_amd.operators import GpuAggregationOnlyCombineOperator, GpuAggregationOperator
    seg, t, h = sv
    op = GpuAggregationOperator(t, h, "SELECT COUNT(*), MAX(column3) FROM testTable")
    blk = op.next_block()
    assert blk.get_aggregation_result() == [30000, 2147419555.0]
    assert op.get_execution_statistics().as_tuple() == (30000, 0, 30000, 30000)
    comb = GpuAggregationOnlyCombineOperator(t, [h, h], "SELECT COUNT(*) FROM testTable")
    assert comb.next_block().get_aggregation_result() == [60000]
    assert comb.get_execution_statistics().as_tuple() == (60000, 0, 0, 60000)


# ------------------------------------------------------------------------------------------------ sorted columns
def _sorted_pair_segment(oracle, schema, cols, sorted_col):
    """The oracle's fixed-bit segment and the same segment with `sorted_col` in SortedIndexReaderImpl pair format."""
    from pinot_amd.segment import ColumnData, SegmentBuffers
    seg = oracle.make_segment(schema, cols)
    c = seg.columns[sorted_col]
    n = seg.num_docs
    ids = np.zeros(max(n, 1), dtype=np.int32)
    buf = ctypes.create_string_buffer(bytes(c.fwd_bytes), max(len(c.fwd_bytes), 1))
    oracle.lib().or_bitset_read_ints(buf, ctypes.c_int64(0), c.bits_per_element, n, ids.ctypes.data)
    ids = ids[:n]
    assert np.all(np.diff(ids) >= 0)
    pairs = b""
    for i in range(c.cardinality):
        w = np.nonzero(ids == i)[0]
        pairs += int(w[0]).to_bytes(4, "big") + int(w[-1]).to_bytes(4, "big")
    out = dict(seg.columns)
    out[sorted_col] = ColumnData(c.data_type, c.cardinality, c.bits_per_element, c.entry_width, c.dict_bytes, pairs,
                                 fwd_format=L.FWD_SORTED_PAIRS, is_sorted=True)
    from dataclasses import replace
    orc = dict(seg.columns)
    orc[sorted_col] = replace(c, is_sorted=True)  # the oracle: fixed-bit bytes, SortedIndexBasedFilterOperator leaves
    return SegmentBuffers(n, orc), SegmentBuffers(n, out)


SORTED_QUERIES = [
    "SELECT COUNT(*), SUM(v) FROM t WHERE s = 40 GROUP BY g",
    "SELECT COUNT(*), SUM(v), MIN(v) FROM t WHERE s BETWEEN 10 AND 70 AND v < 500 GROUP BY g",
    "SELECT COUNT(*), MAX(v) FROM t WHERE v < 500 AND s <> 30 GROUP BY g",
    "SELECT COUNT(*) FROM t WHERE s IN (10, 50, 90) OR v > 900 GROUP BY g",
    "SELECT COUNT(*), SUM(v) FROM t WHERE NOT (s < 55) GROUP BY s",
    "SELECT COUNT(*) FROM t WHERE s > 1000 GROUP BY g",
    "SELECT COUNT(*), SUM(v) FROM t WHERE s IN (20, 30, 40) AND g < 5 GROUP BY s, g",
]


@pytest.mark.parametrize("n", [1, 777, 50_000])
def test_sorted_column_docrange_leaves(oracle, gpu_lib, n):
    """Predicates on sorted columns become docId ranges (SortedIndexBasedFilterOperator: no column read, no
    entries scanned); results equal the oracle's scan over the same data; pure-AND programs evaluate them first."""
    rng = np.random.default_rng(n)
    schema = [("s", "INT"), ("v", "INT"), ("g", "INT")]
    cols = {"s": np.sort(rng.integers(0, 100, n)), "v": rng.integers(0, 1000, n), "g": rng.integers(0, 10, n)}
    seg, sseg = _sorted_pair_segment(oracle, schema, cols, "s")
    t, hs = gpu_table(schema, [sseg, sseg])
    try:
        for sql in SORTED_QUERIES:
            q = parse_query(sql)
            r = t.execute_groupby(hs, q)
            o = oracle.run_groupby(schema, [seg, seg], q)
            assert_same(r, o, q, schema)
            assert r.stats.as_tuple() == o.stats, (sql, r.stats, o.stats)
        # the sorted leaf scans no entries; the v leaf's applyAnd scans only the sorted leaf's docs
        # (AndDocIdSet.java:124-126)
        r = t.execute_groupby(hs, parse_query(SORTED_QUERIES[1]))
        in_range = int(np.count_nonzero((cols["s"] >= 10) & (cols["s"] <= 70)))
        if n > 1:  # one doc: every leaf folds to match-all or empty (cardinality 1)
            assert r.stats.num_entries_scanned_in_filter == 2 * in_range
        bm = t.filter_bitmap(hs[0], parse_query(SORTED_QUERIES[2]), n)
        np.testing.assert_array_equal(bm, oracle.filter_bitmap(schema, seg, parse_query(SORTED_QUERIES[2])))
    finally:
        t.close()


def _fixed_bit_view(seg):
    """The same segment with SortedIndexReaderImpl pair columns expanded to the fixed-bit forward index."""
    from dataclasses import replace
    from pinot_amd.segment import SegmentBuffers
    from pinot_amd.segment_files import pack_msb_first
    cols = {}
    for name, c in seg.columns.items():
        if c.fwd_format == L.FWD_SORTED_PAIRS:
            pairs = np.frombuffer(c.fwd_bytes, dtype=">i4").reshape(-1, 2).astype(np.int64)
            ids = np.repeat(np.arange(c.cardinality), np.maximum(pairs[:, 1] - pairs[:, 0] + 1, 0))
            c = replace(c, fwd_bytes=pack_msb_first(ids, c.bits_per_element), fwd_format=L.FWD_FIXED_BIT)
        cols[name] = c
    return SegmentBuffers(seg.num_docs, cols)


def test_v3_segment_files_pin_and_query(oracle, gpu_lib, tmp_path):
    """Segments written as Pinot v1 directories, converted to v3 (columns.psf + index_map) and loaded back pin and
    answer like the oracle over the same bytes (sorted time column, LONG and STRING group keys)."""
    from pinot_amd.segment_files import convert_v1_to_v3, load_segment_dir, write_v1_segment_dir
    schema = [("day", "INT"), ("acct", "LONG"), ("clicks", "INT"), ("name", "STRING")]
    segs = []
    for s in range(3):
        rng = np.random.default_rng(40 + s)
        n = [20000, 8193, 1][s]
        vals = {"day": np.sort(rng.integers(17000, 17030, n)).tolist(), "acct": rng.integers(0, 500, n).tolist(),
                "clicks": rng.integers(0, 1000, n).tolist(), "name": ["n%d" % v for v in rng.integers(0, 7, n)]}
        path = str(tmp_path / ("seg%d" % s))
        write_v1_segment_dir(path, schema, vals, sorted_columns=("day",))
        convert_v1_to_v3(path)
        segs.append(load_segment_dir(path))
    orc = [_fixed_bit_view(s) for s in segs]  # the oracle reads fixed-bit forward indexes only
    t, hs = gpu_table(schema, segs)
    try:
        for sql in ("SELECT SUM(clicks), COUNT(*), MAX(clicks) FROM t WHERE day BETWEEN 17005 AND 17020 "
                    "AND acct IN (3, 7, 11, 499) GROUP BY day",
                    "SELECT AVG(clicks), MIN(acct) FROM t WHERE clicks < 500 GROUP BY name, day",
                    "SELECT SUM(acct) FROM t WHERE name IN ('n1', 'n4') OR day = 17029 GROUP BY acct"):
            q = parse_query(sql)
            assert_same(t.execute_groupby(hs, q), oracle.run_groupby(schema, orc, q), q, schema)
    finally:
        t.close()


# ------------------------------------------------------------------------------------------------ inverted index
INV_QUERIES = [
    "SELECT COUNT(*), SUM(v) FROM t WHERE a = 3 GROUP BY g",
    "SELECT COUNT(*), SUM(v), MAX(v) FROM t WHERE b IN (7, 100, 2999, 4000) GROUP BY g",
    "SELECT COUNT(*), MIN(v) FROM t WHERE a NOT IN (1, 2) AND v < 500 GROUP BY g",
    "SELECT COUNT(*) FROM t WHERE a <> 4 OR b BETWEEN 10 AND 20 GROUP BY a",
    "SELECT COUNT(*), SUM(v) FROM t WHERE b = 5 AND a IN (0, 8) GROUP BY g, a",
    "SELECT SUM(v) FROM t WHERE NOT (b IN (1, 2, 3) OR a = 0) GROUP BY g",
    "SELECT COUNT(*) FROM t WHERE a = 12345 GROUP BY g",
    "SELECT COUNT(*), SUM(v) FROM t WHERE s BETWEEN 2 AND 5 AND a IN (3, 5) GROUP BY g",
    # one dictId: containers read in place (LEAF_BITDIR) -- ARRAY containers of the sparse column, negated too
    "SELECT COUNT(*), SUM(v), MIN(v) FROM t WHERE b = 2999 GROUP BY g",
    "SELECT COUNT(*), MAX(v) FROM t WHERE b <> 17 AND v < 300 GROUP BY g",
]


@pytest.mark.parametrize("run_optimize", [False, True], ids=["plain", "runs"])
def test_inverted_index_leaves(oracle, gpu_lib, tmp_path, run_optimize):
    """EQ / IN / NOT_EQ / NOT_IN on columns with a bitmap inverted index run as BitmapBasedFilterOperator leaves
    (Roaring containers ORed into a device docId bitmap); results identical to the oracle's scan, no entries
    scanned in the filter for those leaves.  Segments span several 65536-doc containers with ragged tails, ARRAY
    and BITMAP containers (dense `a`: card 9; sparse `b`: card 3000) and, with run_optimize, RUN containers."""
    from pinot_amd.segment_files import convert_v1_to_v3, load_segment_dir, write_v1_segment_dir
    schema = [("a", "INT"), ("b", "INT"), ("g", "INT"), ("v", "INT"), ("s", "INT")]
    segs, orc = [], []
    for k, n in enumerate([150001, 65536, 1, 70000]):
        rng = np.random.default_rng(70 + k)
        a = rng.integers(0, 9, n)
        if k == 3:
            a[:66000] = 3  # a full run container for a = 3
        vals = {"a": a.tolist(), "b": rng.integers(0, 3000, n).tolist(), "g": rng.integers(0, 12, n).tolist(),
                "v": rng.integers(0, 1000, n).tolist(), "s": np.sort(rng.integers(0, 10, n)).tolist()}
        path = str(tmp_path / ("inv%d" % k))
        write_v1_segment_dir(path, schema, vals, sorted_columns=("s",), inverted_columns=("a", "b", "s"),
                             run_optimize=run_optimize)
        if k % 2:
            convert_v1_to_v3(path)
        seg = load_segment_dir(path)
        assert seg.columns["a"].inv_bytes is not None
        segs.append(seg)
        orc.append(_fixed_bit_view(seg))
    from dataclasses import replace
    from pinot_amd.segment import SegmentBuffers
    t, hs = gpu_table(schema, segs)
    # a mixed table: the same data once more, this time with segment 1 lacking the indexes (bitmap leaves in some
    # segments, scan leaves in others, one plan)
    mixed = GpuTable(schema)
    hm = [mixed.pin_segment(s if k != 1 else
                            SegmentBuffers(s.num_docs, {c: replace(d, inv_bytes=None) for c, d in s.columns.items()}))
          for k, s in enumerate(segs)]
    orc_mixed = [o if k != 1 else SegmentBuffers(o.num_docs, {c: replace(d, inv_bytes=None) for c, d in o.columns.items()})
                 for k, o in enumerate(orc)]
    plain = GpuTable(schema)  # the same segments without inverted indexes: scan leaves
    hp = [plain.pin_segment(SegmentBuffers(s.num_docs, {c: replace(d, inv_bytes=None) for c, d in s.columns.items()}))
          for s in segs]
    try:
        for sql in INV_QUERIES:
            q = parse_query(sql)
            r = t.execute_groupby(hs, q)
            o = oracle.run_groupby(schema, orc, q)
            assert_same(r, o, q, schema)
            assert r.stats.as_tuple() == o.stats, (sql, r.stats, o.stats)
            rp = plain.execute_groupby(hp, q)
            assert r.stats.num_docs_scanned == rp.stats.num_docs_scanned, sql
            assert r.stats.num_entries_scanned_in_filter <= rp.stats.num_entries_scanned_in_filter, sql
            rm, om = mixed.execute_groupby(hm, q), oracle.run_groupby(schema, orc_mixed, q)
            assert_same(rm, om, q, schema)
            assert rm.stats.as_tuple() == om.stats, (sql, rm.stats, om.stats)
        r = t.execute_groupby(hs, parse_query("SELECT COUNT(*) FROM t WHERE a IN (2, 3) GROUP BY g"))
        assert r.stats.num_entries_scanned_in_filter == 0
        # single-dictId leaves are read in place whatever their container kinds (no docId bitmap materialised):
        # BITMAP containers of `a`, ARRAY containers of `b`, RUN containers (become ARRAY / BITMAP at attach)
        for sql in ("SELECT COUNT(*) FROM t WHERE a = 3 GROUP BY g", "SELECT COUNT(*) FROM t WHERE b = 2999 GROUP BY g",
                    "SELECT COUNT(*) FROM t WHERE b <> 17 GROUP BY g"):
            with t.plan(hs, parse_query(sql)) as p:
                kinds = p.leaf_kinds()
            assert kinds.get("bitdir", 0) >= 1 and "bitmap" not in kinds, (sql, kinds)
        with t.plan(hs, parse_query("SELECT COUNT(*) FROM t WHERE a IN (2, 3) GROUP BY g")) as p:
            assert "bitmap" in p.leaf_kinds()  # an OR of dictIds is materialised
        for sql in ("SELECT COUNT(*), SUM(v), MIN(v), MAX(g) FROM t WHERE a = 3",
                    "SELECT COUNT(*), SUM(v) FROM t WHERE b NOT IN (5, 6) AND a IN (1, 3, 7)",
                    "SELECT COUNT(*) FROM t WHERE a = 3 AND a <> 3"):
            q = parse_query(sql)
            o = oracle.run_groupby(schema, orc, q)
            from pinot_amd.executor import aggregation_defaults
            exp = o.groups[()] if o.groups else aggregation_defaults(q.aggregations)
            assert t.execute_aggregation(hs, q).values == list(exp), sql
            assert mixed.execute_aggregation(hm, q).values == list(exp), sql
    finally:
        t.close()
        mixed.close()
        plain.close()


def test_inverted_index_malformed(gpu_lib):
    from pinot_amd.segment_files import build_inverted_index, serialize_roaring
    schema = [("a", "INT")]
    t = GpuTable(schema)
    try:
        from pinot_amd.segment_files import build_column
        c = build_column(L.INT, [0, 1, 1, 0, 2], is_sorted=False)
        from pinot_amd.segment import SegmentBuffers
        h = t.pin_segment(SegmentBuffers(5, {"a": c}))
        good = build_inverted_index([0, 1, 1, 0, 2], 3)
        t.attach_inverted_index(h, "a", good)
        with pytest.raises(L.PinotGpuError):
            t.attach_inverted_index(h, "a", good[:-3])  # overrun
        bad = bytearray(good)
        bad[4 * 4] ^= 0x55  # first bitmap's cookie
        with pytest.raises(L.PinotGpuError):
            t.attach_inverted_index(h, "a", bytes(bad))
        out_of_range = serialize_roaring([7])  # docId 7 >= numDocs 5
        offs = np.cumsum([16, len(out_of_range), 0, 0]).astype(">i4").tobytes()
        with pytest.raises(L.PinotGpuError):
            t.attach_inverted_index(h, "a", offs + out_of_range)
        # a RUN container whose runs hold more values than its declared cardinality (0..3 declared as 2 values)
        run_bm = (np.array([12347], "<u4").tobytes() + b"\x01" + np.array([0, 1], "<u2").tobytes() +
                  np.array([1, 0, 3], "<u2").tobytes())
        offs = np.cumsum([16, len(run_bm), 0, 0]).astype(">i4").tobytes()
        with pytest.raises(L.PinotGpuError):
            t.attach_inverted_index(h, "a", offs + run_bm)
        r = t.execute_groupby([h], parse_query("SELECT COUNT(*) FROM t WHERE a IN (1, 2) GROUP BY a"))
        assert {k: v[0] for k, v in r.as_dict().items()} == {(1,): 2, (2,): 1}
    finally:
        t.close()


def test_pin_rejects_dict_ids_past_the_dictionary(gpu_lib):
    """A fixed-bit forward index holding a dictId >= cardinality (2 bits, cardinality 3, a stored 3) is refused at pin
    (fwd_max_kernel's pin-time check): every later scan would index past the column's dictionary arrays.  The table
    stays usable and its byte accounting unchanged."""
    from dataclasses import replace
    from pinot_amd.segment import SegmentBuffers
    from pinot_amd.segment_files import build_column, pack_msb_first
    t = GpuTable([("a", "INT")])
    try:
        c = build_column(L.INT, [0, 1, 2, 1, 0, 2], is_sorted=False)
        assert c.bits_per_element == 2 and c.cardinality == 3
        before = t.device_bytes()
        for ids in ([0, 1, 3, 1, 0, 2], [0] * 5 + [3]):
            bad = replace(c, fwd_bytes=pack_msb_first(ids, 2), fwd_format=L.FWD_FIXED_BIT)
            with pytest.raises(L.PinotGpuError) as e:
                t.pin_segment(SegmentBuffers(6, {"a": bad}))
            assert "dictId 3" in e.value.message
        assert t.device_bytes() == before
        h = t.pin_segment(SegmentBuffers(6, {"a": c}))
        r = t.execute_groupby([h], parse_query("SELECT COUNT(*) FROM t GROUP BY a"))
        assert {k: v[0] for k, v in r.as_dict().items()} == {(0,): 2, (1,): 2, (2,): 2}
    finally:
        t.close()


def test_long_literals_beyond_double_precision(oracle, gpu_lib):
    """Dictionary lookups of LONG literals that differ by less than one double ulp (values around 2^60, where
    interpolation in double precision degenerates) find the exact dictId (BaseImmutableDictionary.insertionIndexOf)."""
    base = 2 ** 60
    vals = np.array([base + (i % 7) for i in range(5000)] + [-(2 ** 62), 2 ** 62], dtype=np.int64)
    schema = [("x", "LONG"), ("g", "INT")]
    seg = oracle.make_segment(schema, {"x": vals, "g": np.arange(len(vals)) % 3})
    t, hs = gpu_table(schema, [seg])
    try:
        for sql in ("SELECT COUNT(*) FROM t WHERE x = %d GROUP BY g" % (base + 3),
                    "SELECT COUNT(*) FROM t WHERE x BETWEEN %d AND %d GROUP BY g" % (base + 1, base + 4),
                    "SELECT COUNT(*) FROM t WHERE x IN (%d, %d, 5) GROUP BY g" % (base + 2, base + 6),
                    "SELECT COUNT(*) FROM t WHERE x > %d GROUP BY g" % (base + 5)):
            q = parse_query(sql)
            assert_same(t.execute_groupby(hs, q), oracle.run_groupby(schema, [seg], q), q, schema)
    finally:
        t.close()


def test_plan_cache_reuse_and_invalidation(oracle):
    """A repeated query reuses the table's compiled plan (same result and statistics); growing a group-by
    column's global dictionary invalidates it (new key layout), and the answer is still the oracle's."""
    schema = [("d", "INT"), ("f", "INT"), ("m", "INT")]
    rng = np.random.default_rng(11)
    segs = [oracle.make_segment(schema, {"d": rng.integers(0, 50, 4000).tolist(), "f": rng.integers(0, 100, 4000).tolist(),
                                         "m": rng.integers(0, 1000, 4000).tolist()}) for _ in range(3)]
    q = parse_query("SELECT COUNT(*), SUM(m), MAX(m) FROM t WHERE f < 40 GROUP BY d")
    o = oracle.run_groupby(schema, segs, q)
    t, hs = gpu_table(schema, segs)
    try:
        r1 = t.execute_groupby(hs, q)
        r2 = t.execute_groupby(hs, q)
        assert_same(r1, o, q, schema)
        assert r1.as_dict() == r2.as_dict() and r1.stats.as_tuple() == r2.stats.as_tuple() == o.stats
        t.add_dictionary_values("d", [-5, 1000, 2000])  # the key space grows: cached plans are stale
        r3 = t.execute_groupby(hs, q)
        assert_same(r3, o, q, schema)
        assert r3.stats.as_tuple() == o.stats
    finally:
        t.close()


def test_table_config_roundtrip(gpu_lib):
    """pgpu_table_set_config / _get_config: fields set are kept, others keep their values, out-of-range values are
    refused, a caller's shorter struct leaves the later fields at their defaults."""
    import ctypes
    t = GpuTable([("a", "INT")], config={"stream_chunks": 3, "dense_selectivity": 0.5})
    try:
        c = t.config()
        assert c["stream_chunks"] == 3 and c["dense_selectivity"] == 0.5 and c["plan_cache"] == 1
        t.set_config(plan_cache=0)
        assert t.config()["plan_cache"] == 0 and t.config()["stream_chunks"] == 3
        for bad in ({"hash_partition_bits": 15}, {"lds_table_kb": 0}, {"stream_chunks": 0},
                    {"dense_selectivity": float("nan")}):
            with pytest.raises(L.PinotGpuError):
                t.set_config(**bad)
        short = L.ConfigC(8, 0)  # struct_size covers plan_cache only
        L.check(t.lib.pgpu_table_set_config(t.handle, ctypes.byref(short)))
        c = t.config()
        assert c["plan_cache"] == 0 and c["stream_chunks"] == 1 and c["dense_selectivity"] == 0.25
        t.reset_config()
        assert t.config()["plan_cache"] == 1
    finally:
        t.close()


def test_table_global_value_arrays(oracle, gpu_lib):
    """Accumulator columns with large dictionaries are gathered from the table-global value arrays (rt_dict.cpp
    ensure_value_map, KCol.gaps, device.h vidx): a segment whose dictionary lacks a few global values maps its dictIds
    past them with thresholds, a contiguous run by an offset alone; more than kMaxValueGaps (16) missing values keep the
    segment's own arrays.  Dense, sparse, partitioned and aggregation-only scans against the oracle, before and after a
    pin grows the global dictionary (new arrays, new maps)."""
    rng = np.random.default_rng(77)
    table_d = np.round(rng.uniform(-1e5, 1e5, 20000), 4)
    table_d = np.unique(table_d)
    table_i = np.unique(rng.integers(-10 ** 12, 10 ** 12, 20000))
    schema = [("g", "INT"), ("f", "INT"), ("x", "DOUBLE"), ("y", "LONG"), ("k", "INT")]

    def seg(n, xs, ys, seed):
        r = np.random.default_rng(seed)
        return oracle.make_segment(schema, {"g": r.integers(0, 50, n), "f": r.integers(0, 100, n),
                                            "x": r.choice(xs, n), "y": r.choice(ys, n),
                                            "k": r.integers(0, 40000, n)})

    # every value present (forced), except a few single values: single gaps
    def near_full(vals, drop, n, seed):
        keep = np.delete(vals, drop)
        r = np.random.default_rng(seed)
        return np.concatenate([keep, r.choice(keep, n - len(keep))])

    n = 60000
    segs = []
    # single missing values, none (a contiguous run), adjacent ones at both ends, 20 (the segment's own arrays)
    for i, drop in enumerate(([5, 900, 12345], [], [0, 1, 100, 101, 102, -1], list(range(7, 2000, 99)))):
        xs = near_full(table_d, drop, n, 10 + i)
        ys = near_full(table_i, drop, n, 20 + i)
        s = oracle.make_segment(schema, {"g": np.random.default_rng(i).integers(0, 50, n),
                                         "f": np.random.default_rng(i + 5).integers(0, 100, n),
                                         "x": np.random.default_rng(i + 9).permutation(xs),
                                         "y": np.random.default_rng(i + 7).permutation(ys),
                                         "k": np.random.default_rng(i + 3).integers(0, 40000, n)})
        segs.append(s)
    t, hs = gpu_table(schema, segs)
    try:
        queries = ["SELECT SUM(x), MIN(x), MAX(y), SUM(y), AVG(x), COUNT(*) FROM t WHERE f < 60 GROUP BY g",  # dense
                   "SELECT SUM(x), MAX(x), MIN(y) FROM t WHERE f = 7 GROUP BY g",                          # sparse
                   "SELECT SUM(y), COUNT(*) FROM t GROUP BY g, k",   # 2M keys: partitioned (one 8-B stream)
                   "SELECT SUM(x), MIN(y), COUNT(*) FROM t WHERE f < 50"]                                 # agg-only
        for sql in queries:
            q = parse_query(sql, num_groups_limit=10 ** 9)
            if q.group_by:
                assert_same(t.execute_groupby(hs, q), oracle.run_groupby(schema, segs, q), q, schema)
            else:
                r = t.execute_aggregation(hs, q)
                (exp,) = oracle.run_groupby(schema, segs, q).groups.values()
                assert r.values[0] == pytest.approx(exp[0], rel=REL)
                assert r.values[1:] == list(exp[1:])
        # a pin that adds values grows the global dictionaries: new arrays and maps for the next plans
        extra = seg(n, np.concatenate([table_d, [1e9, -1e9]]), np.concatenate([table_i, [7, 11]]), 99)
        hs2 = hs + [t.pin_segment(extra)]
        segs2 = segs + [extra]
        for sql in queries[:3]:
            q = parse_query(sql, num_groups_limit=10 ** 9)
            assert_same(t.execute_groupby(hs2, q), oracle.run_groupby(schema, segs2, q), q, schema)
    finally:
        t.close()
