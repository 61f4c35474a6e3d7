"""Hashed partitions (partition.h K8h): sparse group-key spaces (past every dense table, below 2^31) aggregated per
hash partition in LDS hash tables instead of the global hash table -- against the oracle's LONG_MAP restatement
(DictionaryBasedGroupKeyGenerator.java:644-746), including partitions that need several K8h rounds, the
global-hash-table path beside it, a filter, every accumulator kind and the exchange (materialised table)."""
import numpy as np
import pytest

from pinot_amd import _lib as L
from pinot_amd.query import parse_query
from test_gpu_parity import assert_same, gpu_table

pytestmark = pytest.mark.gpu

SCHEMA = [("a", "INT"), ("b", "INT"), ("c", "INT"), ("m", "INT"), ("x", "DOUBLE"), ("s", "INT")]
DOCS = 120000


def _columns(seed):
    rng = np.random.default_rng(seed)
    return {"a": rng.integers(0, 3000, DOCS).astype(np.int64), "b": rng.integers(0, 3000, DOCS).astype(np.int64),
            "c": rng.integers(0, 30, DOCS).astype(np.int64), "m": rng.integers(-400, 900, DOCS).astype(np.int64),
            "x": np.round(rng.uniform(-1e4, 1e4, DOCS), 3), "s": rng.integers(0, 100, DOCS).astype(np.int64)}


@pytest.fixture(scope="module")
def sparse(oracle, gpu_lib):
    segs = [oracle.make_segment(SCHEMA, _columns(41 + s)) for s in range(2)]
    t, hs = gpu_table(SCHEMA, segs)
    yield t, hs, segs
    t.close()


QUERIES = [
    "SELECT COUNT(*), SUM(m) FROM t GROUP BY a, b, c",
    "SELECT MIN(m), MAX(x), SUM(x), AVG(m), COUNT(*) FROM t WHERE c < 20 GROUP BY a, b, c",
    "SELECT SUM(m), MAX(m) FROM t WHERE m > 0 AND x < 5000 GROUP BY c, a, b",
    # one stream whose range (7 bits) fits under the partition bits: K8e / K8h records packed into a u32
    "SELECT COUNT(*), SUM(s), MAX(s) FROM t WHERE m >= 0 GROUP BY a, b, c",
    # ... and exactly COUNT + SUM of it: one LDS word per group (count in the high bits)
    "SELECT SUM(s), COUNT(*) FROM t GROUP BY b, c, a",
]


@pytest.mark.parametrize("sql", QUERIES)
def test_hash_partitions_match_oracle(oracle, sparse, sql):
    t, hs, segs = sparse
    q = parse_query(sql, num_groups_limit=10 ** 9)
    with t.plan(hs, q) as p:
        assert p.group_path() == "hash_partitioned"
    assert_same(t.execute_groupby(hs, q), oracle.run_groupby(SCHEMA, segs, q), q, SCHEMA)


def test_hash_partition_rounds(oracle, sparse):
    """One partition of 2^sbits LDS slots for ~2e5 groups: K8h loops over rounds, each placing the keys that find a
    slot and compacting the rest in place."""
    t, hs, segs = sparse
    t.set_config(hash_partition_bits=0)
    try:
        for sql in QUERIES[:2]:
            q = parse_query(sql, num_groups_limit=10 ** 9)
            with t.plan(hs, q) as p:
                assert p.group_path() == "hash_partitioned"
            assert_same(t.execute_groupby(hs, q), oracle.run_groupby(SCHEMA, segs, q), q, SCHEMA)
    finally:
        t.reset_config()


def test_hash_partition_rounds_packed(oracle, sparse):
    """Packed records (hashed key bits | value) left pending: 128 partitions of 256-entry LDS tables for ~1 800 groups
    each, so K8h writes packed words back and re-reads them over several rounds."""
    t, hs, segs = sparse
    # 256-entry tables (4 KB), 128 partitions: 7 bits, just room for the 7-bit values
    t.set_config(hash_partition_lds_kb=4, hash_partition_bits=7)
    try:
        q = parse_query(QUERIES[3], num_groups_limit=10 ** 9)
        assert_same(t.execute_groupby(hs, q), oracle.run_groupby(SCHEMA, segs, q), q, SCHEMA)
    finally:
        t.reset_config()


def test_hash_partitions_exchange_materialises_table(oracle, sparse):
    """pgpu_plan_exchange_counts / _export / _merge on a hashed-partition plan: its records become a hash table
    first; one part exported and merged back gives the plan's own groups."""
    import ctypes
    t, hs, segs = sparse
    q = parse_query(QUERIES[0], num_groups_limit=10 ** 9)
    plan = t.plan_execute(hs, q)
    try:
        lib = plan.lib
        counts = (ctypes.c_int64 * 1)()
        L.check(lib.pgpu_plan_exchange_counts(plan.handle, None, 1, counts))
        exp = oracle.run_groupby(SCHEMA, segs, q)
        assert counts[0] == len(exp.groups)
        import torch
        out = torch.empty((counts[0], 3), dtype=torch.int64, device="cuda")
        L.check(lib.pgpu_plan_exchange_export(plan.handle, None, 1, None, ctypes.c_void_p(out.data_ptr()),
                                              counts[0]))
        L.check(lib.pgpu_plan_exchange_merge(plan.handle, None, None, ctypes.c_void_p(out.data_ptr()), counts[0]))
        assert_same(plan.finalize(), exp, q, SCHEMA)
    finally:
        plan.close()


def test_group_paths(oracle, sparse):
    """pgpu_plan_group_path across the key-space sizes of one table: an LDS table (small dense), hashed partitions
    (sparse, < 2^31 keys), the global hash table (>= 2^31 keys) -- each against the oracle."""
    t, hs, segs = sparse
    for sql, path in (("SELECT COUNT(*), SUM(m) FROM t GROUP BY c", "lds"),
                      ("SELECT COUNT(*), SUM(m) FROM t GROUP BY a, b, c", "hash_partitioned"),
                      ("SELECT COUNT(*), SUM(m) FROM t GROUP BY a, b, c, s", "hash")):
        q = parse_query(sql, num_groups_limit=10 ** 9)
        with t.plan(hs, q) as p:
            assert p.group_path() == path, sql
        assert_same(t.execute_groupby(hs, q), oracle.run_groupby(SCHEMA, segs, q), q, SCHEMA)


def test_in_filter_narrows_the_key_space_to_a_dense_table(oracle, sparse):
    """The IN-filtered shape r04 dropped from QUERIES after its path assertion failed: the conjunct `c IN (1, 3, 5, 7)`
    bounds the group-by column c to the global ids of [1, 7], so the key space the planner sizes is 3000 x 3000 x 7 =
    6.3e7 < 2^26 -- a dense table, not hashed partitions (the filter-restricted key space, rt_plan.cpp "Key space
    restricted by the filter").  The path is asserted as the planner should pick it, and the values against the
    oracle."""
    t, hs, segs = sparse
    q = parse_query("SELECT SUM(m), MAX(m) FROM t WHERE m > 0 AND c IN (1, 3, 5, 7) GROUP BY c, a, b",
                    num_groups_limit=10 ** 9)
    with t.plan(hs, q) as p:
        assert p.group_path() in ("global", "partitioned"), p.group_path()
        assert p.layout()[1] == len(t.dictionary("a")) * len(t.dictionary("b")) * 7 < 2 ** 26
    assert_same(t.execute_groupby(hs, q), oracle.run_groupby(SCHEMA, segs, q), q, SCHEMA)


def _key_order(k):
    """Ascending composite key (DictionaryBasedGroupKeyGenerator mixed radix, column 0 least significant): the
    dictionaries are sorted, so value order is dictId order."""
    return tuple(reversed(k))


def test_hash_result_trims_order_by_key(oracle, sparse):
    """Hash-mode results of >= 4096 groups come back in partition order: the SQL trim without ORDER BY
    still keeps the smallest composite keys, and ORDER BY / PQL ties still fall back to the composite key."""
    t, hs, segs = sparse
    q = parse_query("SELECT COUNT(*), SUM(m) FROM t GROUP BY a, b, c LIMIT 100", num_groups_limit=10 ** 9)
    with t.plan(hs, q) as p:
        assert p.group_path() == "hash_partitioned"
    r = t.execute_groupby(hs, q)
    exp = oracle.run_groupby(SCHEMA, segs, q)
    exp_d = exp.groups
    assert len(r) == len(exp_d) >= 4096
    keys = sorted(exp_d, key=_key_order)
    assert r.keys != keys  # partition order: the trims below must not rely on row order
    trimmed = r.trim_sql(q)
    assert trimmed.keys == keys[:100]
    assert [v[0] for v in trimmed.values] == [exp_d[k][0] for k in keys[:100]]
    # ORDER BY COUNT(*) DESC: the top max(limit * 5, 5000) rows, count ties broken by composite key
    qo = parse_query("SELECT COUNT(*), SUM(m) FROM t GROUP BY a, b, c ORDER BY COUNT(*) DESC LIMIT 10",
                     num_groups_limit=10 ** 9)
    ordered = r.trim_sql(qo)
    want = sorted(exp_d, key=lambda k: (-exp_d[k][0], _key_order(k)))[:5000]
    assert ordered.keys == want
    # PQL: per function the top groups, ties by composite key
    top = r.trim_pql(50, final=True)
    assert [k for k, _ in top[0]] == sorted(exp_d, key=lambda k: (-exp_d[k][0], _key_order(k)))[:50]
