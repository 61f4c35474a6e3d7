"""world_size-2 CPU test (gloo) of the multi-GPU combine: the code bench.py runs between ranks
(pinot_amd/combine.py) merges per-rank dense group tables into the result of GroupByCombineOperator over the union
of the ranks' segments (core/operator/combine/GroupByCombineOperator.java:113-160).

Each rank owns a disjoint set of segments (weak scaling: segments shard).  The per-rank table is
the plan layout the GPU writes ([slot][key] int64 words: COUNT, integer SUM, float64 SUM bits, MIN/MAX keys) in the
table-global key space that union_dictionaries establishes; here it is filled from the oracle's per-rank result.
The merged table must equal the oracle run over all segments: bit-exact for integer slots, 1e-9 relative for the
float64 sum.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pinot_amd import _lib as L
from pinot_amd.combine import allreduce_group_table, reduce_scatter_group_table, shard_range, union_dictionaries
from pinot_amd.query import parse_query

SCHEMA = [("d", "INT"), ("f", "INT"), ("mi", "INT"), ("md", "DOUBLE")]
SQL = "SELECT COUNT(*), SUM(mi), MIN(mi), MAX(mi), SUM(md) FROM t WHERE f < 40 GROUP BY d"
KINDS = [L.SLOT_COUNT, L.SLOT_SUM_I64, L.SLOT_MIN_KEY, L.SLOT_MAX_KEY, L.SLOT_SUM_F64]
WORLD = 2
SEGS_PER_RANK = 2
DOCS = 3000


class _DictTable:
    """The two GpuTable methods union_dictionaries uses, over a host dictionary (no device needed)."""

    def __init__(self, dicts):
        self.dicts = {k: sorted(set(v)) for k, v in dicts.items()}

    def dictionary(self, column):
        return list(self.dicts[column])

    def add_dictionary_values(self, column, values):
        self.dicts[column] = sorted(set(self.dicts[column]) | set(values))


def _segment_columns(seg_index):
    rng = np.random.default_rng(1000 + seg_index)
    # every rank sees a different subset of group values, so the union of dictionaries matters
    d = rng.integers(0, 12, DOCS) + 3 * (seg_index % 3)
    return {"d": d.astype(np.int64), "f": rng.integers(0, 100, DOCS).astype(np.int64),
            "mi": rng.integers(-5000, 70000, DOCS).astype(np.int64),
            "md": rng.uniform(-1e6, 1e6, DOCS)}


def _dense_table(groups, gdict):
    """Oracle groups {(d,): [count, sum_mi, min_mi, max_mi, sum_md]} -> [5][G] int64 table in the global key space."""
    G = len(gdict)
    t = np.zeros((len(KINDS), G), dtype=np.int64)
    t[2, :] = np.iinfo(np.int64).max
    t[3, :] = np.iinfo(np.int64).min
    f64 = t[4].view(np.float64)
    f64[:] = 0.0
    pos = {v: i for i, v in enumerate(gdict)}
    for (d,), vals in groups.items():
        k = pos[d]
        t[0, k] = vals[0]
        t[1, k] = int(vals[1])
        t[2, k] = int(vals[2])
        t[3, k] = int(vals[3])
        f64[k] = vals[4]
    return torch.from_numpy(t)


def _worker(rank, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import _oracle
        q = parse_query(SQL)
        mine = [rank * SEGS_PER_RANK + i for i in range(SEGS_PER_RANK)]
        cols = [_segment_columns(s) for s in mine]
        segs = [_oracle.make_segment(SCHEMA, c) for c in cols]
        local = _oracle.run_groupby(SCHEMA, segs, q, nthreads=2)
        # global key space: union of the ranks' group-by dictionaries
        table = _DictTable({"d": np.concatenate([c["d"] for c in cols]).tolist()})
        union_dictionaries(table, ["d"])
        gdict = table.dictionary("d")
        dense = _dense_table(local.groups, gdict)
        shard, k0, kn = reduce_scatter_group_table(dense.clone(), KINDS)
        np.save(os.path.join(out_dir, "shard_%d.npy" % rank), shard.numpy())
        np.save(os.path.join(out_dir, "range_%d.npy" % rank), np.array([k0, kn], dtype=np.int64))
        allreduce_group_table(dense, KINDS)
        np.save(os.path.join(out_dir, "merged_%d.npy" % rank), dense.numpy())
        np.save(os.path.join(out_dir, "dict_%d.npy" % rank), np.array(gdict, dtype=np.int64))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_two_rank_combine_matches_oracle(oracle, tmp_path):
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    m0, m1 = np.load(tmp_path / "merged_0.npy"), np.load(tmp_path / "merged_1.npy")
    d0, d1 = np.load(tmp_path / "dict_0.npy"), np.load(tmp_path / "dict_1.npy")
    assert np.array_equal(d0, d1), "ranks disagree on the global key space"
    assert np.array_equal(m0, m1), "all-reduce left ranks with different tables"
    # reduce-scatter (the large-table combine): rank r holds exactly its key range of the merged table
    covered = 0
    for r in range(WORLD):
        shard, (k0, kn) = np.load(tmp_path / ("shard_%d.npy" % r)), np.load(tmp_path / ("range_%d.npy" % r))
        assert (k0, kn) == shard_range(m0.shape[1], WORLD, r)[:2]
        assert shard.shape == (m0.shape[0], kn)
        assert np.array_equal(shard, m0[:, k0:k0 + kn]), r
        covered += kn
    assert covered == m0.shape[1]
    # oracle over the union of all segments (GroupByCombineOperator semantics)
    q = parse_query(SQL)
    segs = [oracle.make_segment(SCHEMA, _segment_columns(s)) for s in range(WORLD * SEGS_PER_RANK)]
    exp = oracle.run_groupby(SCHEMA, segs, q, nthreads=2)
    got = {}
    f64 = m0[4].view(np.float64)
    for k, d in enumerate(d0):
        if m0[0, k] == 0:
            continue
        got[(int(d),)] = (int(m0[0, k]), int(m0[1, k]), int(m0[2, k]), int(m0[3, k]), float(f64[k]))
    assert set(got) == set(exp.groups)
    for key, vals in exp.groups.items():
        c, s, mn, mx, sd = got[key]
        assert c == vals[0] and s == int(vals[1]) and mn == int(vals[2]) and mx == int(vals[3]), key
        assert sd == pytest.approx(vals[4], rel=1e-9, abs=1e-6), key


def test_union_dictionaries_single_process_group(tmp_path):
    """union_dictionaries is a no-op on values already shared (world_size 1, gloo)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        t = _DictTable({"d": [5, 1, 3]})
        union_dictionaries(t, ["d"])
        assert t.dictionary("d") == [1, 3, 5]
    finally:
        dist.destroy_process_group()


def _exchange_worker(rank, port, out_dir):
    """The hash / row exchange's collectives (pinot_amd.combine): slot-kind agreement and the owner all-to-all."""
    from pinot_amd.combine import agreed_slot_kinds, all_to_all_rows
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        # rank 1's SUM could overflow int64 on its segments (float64 slot): every rank exchanges that slot as float64
        mine = [L.SLOT_COUNT, L.SLOT_SUM_I64 if rank == 0 else L.SLOT_SUM_F64, L.SLOT_MIN_KEY]
        agreed = agreed_slot_kinds(mine)
        # rows [key, rank, i] grouped by owner = key % WORLD; rank r sends 3 + r rows
        keys = np.arange(10 * rank, 10 * rank + 3 + rank, dtype=np.int64)
        owner = keys % WORLD
        order = np.argsort(owner, kind="stable")
        rows = np.stack([keys, np.full_like(keys, rank), np.arange(len(keys))], axis=1)[order]
        counts = np.bincount(owner, minlength=WORLD)
        recv = all_to_all_rows(torch.from_numpy(np.ascontiguousarray(rows)), counts).numpy()
        np.save(os.path.join(out_dir, "recv_%d.npy" % rank), recv)
        np.save(os.path.join(out_dir, "kinds_%d.npy" % rank), np.array(agreed, dtype=np.int64))
        bad = [L.SLOT_COUNT, L.SLOT_MIN_KEY if rank == 0 else L.SLOT_MAX_KEY, L.SLOT_MIN_KEY]
        try:
            agreed_slot_kinds(bad)
            np.save(os.path.join(out_dir, "bad_%d.npy" % rank), np.array([0]))
        except ValueError:
            np.save(os.path.join(out_dir, "bad_%d.npy" % rank), np.array([1]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_row_exchange(tmp_path):
    """Every row reaches its owner rank exactly once (rank order), and the ranks agree on the exchanged slot kinds:
    an int64 SUM travels as float64 when another rank's is float64; kinds that cannot be reconciled fail on every
    rank."""
    mp.spawn(_exchange_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    sent = []
    for r in range(WORLD):
        keys = np.arange(10 * r, 10 * r + 3 + r)
        sent += [(int(k), r) for k in keys]
    for r in range(WORLD):
        recv = np.load(tmp_path / ("recv_%d.npy" % r))
        assert all(int(k) % WORLD == r for k in recv[:, 0])
        assert list(recv[:, 1]) == sorted(recv[:, 1])  # rank order
        assert sorted((int(a), int(b)) for a, b, _ in recv) == sorted(x for x in sent if x[0] % WORLD == r)
        assert list(np.load(tmp_path / ("kinds_%d.npy" % r))) == [L.SLOT_COUNT, L.SLOT_SUM_F64, L.SLOT_MIN_KEY]
        assert int(np.load(tmp_path / ("bad_%d.npy" % r))[0]) == 1
