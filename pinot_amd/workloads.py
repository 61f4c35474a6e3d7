"""Synthetic workloads of BASELINE.json / BASELINE.md §3 (C1, C2, C3, C5): schemas, column generators and
queries.  Values follow f(splitmix64(seed_c ^ global_row)), seed_c = (0x5EED0000 + column index) << 32, so the
device generator (pgpu_generate_segment) and the CPU oracle produce identical segments.
"""
import numpy as np

SEGMENT_DOCS = 1_000_000


def zipf_cdf(n, s=1.0):
    """P(rank k) ~ 1 / (k + 1)^s, cumulative, last entry forced to 1 (same arithmetic as oracle or_zipf_cdf)."""
    w = 1.0 / np.power(np.arange(1, n + 1, dtype=np.float64), s)
    c = np.cumsum(w)
    out = c / c[-1]
    out[-1] = 1.0
    return out


def account_ids(n):
    """Rank -> accountId: rank 0 is 123456789 (the README query's account), the rest 1000000 + 37 * rank."""
    ids = 1_000_000 + 37 * np.arange(n, dtype=np.int64)
    ids[0] = 123456789
    return ids


def double_table(n, column_index, lo, hi):
    """Fixed table of n doubles U[lo, hi) (C2's `md` dictionary values)."""
    from ._splitmix import splitmix64_np
    seed = np.uint64((0x5EED0000 + column_index) << 32)
    h = splitmix64_np(seed ^ (np.uint64(0xDB1E000000) + np.arange(n, dtype=np.uint64)))
    u = (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return lo + (hi - lo) * u


class Workload:
    def __init__(self, name, schema, gen, sql, description, num_groups_limit=100_000, cpu_sample_segments=64,
                 star_tree=None, inverted_columns=()):
        self.name = name
        self.schema = schema          # [(column, type)]
        self.gen = gen                # generator spec per column (table column order)
        self.sql = sql
        self.description = description
        self.num_groups_limit = num_groups_limit  # query option numGroupsLimit of the config
        self.cpu_sample_segments = cpu_sample_segments  # bench CPU-baseline sample (~10-30 s of oracle work)
        self.star_tree = star_tree    # None, or {split_order, pairs, max_leaf_records}: built per segment at setup
        self.inverted_columns = tuple(inverted_columns)  # bitmap inverted indexes built per segment at setup


def adanalytics():
    """C3: the README AdAnalytics query (README.md:82-87) over daysSinceEpoch / accountId / clicks / impressions."""
    n = 100_000
    schema = [("daysSinceEpoch", "INT"), ("accountId", "INT"), ("clicks", "INT"), ("impressions", "INT")]
    gen = [
        {"kind": "UNIFORM", "column_index": 0, "lo": 17532, "hi": 17897},
        {"kind": "ZIPF", "column_index": 1, "cdf": zipf_cdf(n), "ids": account_ids(n)},
        {"kind": "UNIFORM", "column_index": 2, "lo": 0, "hi": 1000},
        {"kind": "UNIFORM", "column_index": 3, "lo": 0, "hi": 100_000},
    ]
    sql = ("SELECT sum(clicks), sum(impressions) FROM AdAnalyticsTable WHERE daysSinceEpoch BETWEEN 17849 AND 17856 "
           "AND accountId IN (123456789) GROUP BY daysSinceEpoch TOP 100")
    return Workload("adanalytics", schema, gen, sql, "C3 AdAnalytics filtered GROUP BY day")


def adanalytics_inv():
    """C3 over a production-style table: a bitmap inverted index on accountId (BitmapBasedFilterOperator leaf,
    evaluated before the daysSinceEpoch scan)."""
    w = adanalytics()
    w.name = "adanalytics_inv"
    w.description = "C3 AdAnalytics with an inverted index on accountId"
    w.inverted_columns = ("accountId",)
    return w


def c1():
    schema = [("dim", "INT"), ("filt", "INT"), ("metric", "INT")]
    gen = [
        {"kind": "UNIFORM", "column_index": 0, "lo": 0, "hi": 16},
        {"kind": "UNIFORM", "column_index": 1, "lo": 0, "hi": 1000},
        {"kind": "UNIFORM", "column_index": 2, "lo": 0, "hi": 10_000},
    ]
    sql = "SELECT SUM(metric) FROM t WHERE filt BETWEEN 250 AND 749 GROUP BY dim"
    return Workload("c1", schema, gen, sql, "C1 pinot-perf style range filter, SUM GROUP BY low-card dim")


def c2():
    schema = [("f", "INT"), ("d", "INT"), ("mi", "INT"), ("md", "DOUBLE")]
    gen = [
        {"kind": "UNIFORM", "column_index": 0, "lo": 0, "hi": 1000},
        {"kind": "UNIFORM", "column_index": 1, "lo": 0, "hi": 100},
        {"kind": "UNIFORM", "column_index": 2, "lo": 0, "hi": 65536},
        {"kind": "TABLE", "column_index": 3, "table": double_table(100_000, 3, -1e6, 1e6)},
    ]
    sql = "SELECT COUNT(*), SUM(mi), MIN(mi), MAX(mi), SUM(md) FROM t WHERE f < 500 GROUP BY d"
    return Workload("c2", schema, gen, sql, "C2 filtered SUM/COUNT/MIN/MAX GROUP BY")


def c5():
    schema = [("k1", "INT"), ("k2", "INT"), ("k3", "INT"), ("m", "INT")]
    gen = [
        {"kind": "UNIFORM", "column_index": 0, "lo": 0, "hi": 1000},
        {"kind": "UNIFORM", "column_index": 1, "lo": 0, "hi": 100},
        {"kind": "UNIFORM", "column_index": 2, "lo": 0, "hi": 100},
        {"kind": "UNIFORM", "column_index": 3, "lo": 0, "hi": 1000},
    ]
    sql = "SELECT SUM(m), COUNT(*) FROM t GROUP BY k1, k2, k3"
    # run with num.groups.limit = 10M and server trim off
    return Workload("c5", schema, gen, sql, "C5 high-cardinality 3-column GROUP BY", num_groups_limit=10_000_000,
                    cpu_sample_segments=16)


def c5_hash():
    """C5 through the global hash table (BASELINE configs[4] "with global-memory hash tables"): the same ~10M groups
    of a 3-column key as C5, but k3 has 10 000 values drawn from k2's hash stream (k3 % 100 == k2), so the key space
    is 1000 x 100 x 10 000 = 10^9 > 2^26 -- past every dense table -- while the data holds 10^7 combinations
    (DictionaryBasedGroupKeyGenerator's LONG_MAP holder, DictionaryBasedGroupKeyGenerator.java:644-746)."""
    schema = [("k1", "INT"), ("k2", "INT"), ("k3", "INT"), ("m", "INT")]
    gen = [
        {"kind": "UNIFORM", "column_index": 0, "lo": 0, "hi": 1000},
        {"kind": "UNIFORM", "column_index": 1, "lo": 0, "hi": 100},
        {"kind": "UNIFORM", "column_index": 1, "lo": 0, "hi": 10_000},
        {"kind": "UNIFORM", "column_index": 3, "lo": 0, "hi": 1000},
    ]
    sql = "SELECT SUM(m), COUNT(*) FROM t GROUP BY k1, k2, k3"
    return Workload("c5_hash", schema, gen, sql, "C5 ~10M groups in a 10^9-key space: global hash table",
                    num_groups_limit=1_000_000_000, cpu_sample_segments=16)


def c4():
    """C4: star-tree query: per segment d1 U[0,100), d2 U[0,50), d3 U[0,20), d4 U[0,10),
    m U[0,1000); star-tree split order [d1, d2, d3, d4], pairs SUM__m and COUNT__*, maxLeafRecords 10 000."""
    schema = [("d1", "INT"), ("d2", "INT"), ("d3", "INT"), ("d4", "INT"), ("m", "INT")]
    gen = [
        {"kind": "UNIFORM", "column_index": 0, "lo": 0, "hi": 100},
        {"kind": "UNIFORM", "column_index": 1, "lo": 0, "hi": 50},
        {"kind": "UNIFORM", "column_index": 2, "lo": 0, "hi": 20},
        {"kind": "UNIFORM", "column_index": 3, "lo": 0, "hi": 10},
        {"kind": "UNIFORM", "column_index": 4, "lo": 0, "hi": 1000},
    ]
    sql = "SELECT SUM(m), COUNT(*) FROM t WHERE d3 IN (1, 5, 7) GROUP BY d1, d2"
    star = {"split_order": ["d1", "d2", "d3", "d4"], "pairs": [("SUM", "m"), ("COUNT", "*")],
            "max_leaf_records": 10_000}
    return Workload("c4", schema, gen, sql, "C4 star-tree multi-dim GROUP BY", star_tree=star)


WORKLOADS = {"adanalytics": adanalytics, "adanalytics_inv": adanalytics_inv, "c1": c1, "c2": c2, "c4": c4, "c5": c5,
             "c5_hash": c5_hash}
