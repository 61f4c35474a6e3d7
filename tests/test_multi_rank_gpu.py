"""The multi-GPU query flow end to end on the device, world_size 2 (both ranks on the box's one GPU, gloo with
host-staged collectives; on a node the same code runs over RCCL): each rank pins its own segments, the ranks union
their group-by dictionaries (one key space), and every combine mode bench.py / a server uses is checked against the
oracle (GroupByCombineOperator semantics, core/operator/combine/GroupByCombineOperator.java:113-160):

- dense, small: plan + execute into a caller-owned device table (pgpu_plan_create_execute), all-reduce;
- dense, large: reduce-scatter by key range, pgpu_plan_finalize_range per rank (disjoint groups);
- C5 shape: 1M-doc segments, a 160 MB table built by the partitioned group-by, reduce-scattered;
- star-tree: segments answered from their star-trees, writing into the caller table, all-reduced;
- hash mode (key space past 2^26): device records hash-partitioned by owner rank, all_to_all, merged by the owner
  (GroupByOrderByCombineOperator's IndexedTable.upsert, :170-181);
- numGroupsLimit: each rank is one Pinot server (per-segment first-seen truncation and the PQL 2x cap per rank), the
  finalized rows are exchanged by owner and merged as the broker merges server responses.
This is bench.py's step for --gpus N."""
import datetime
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pinot_amd.combine import (allreduce_group_table, exchange_hash_table, exchange_result, plan_combine_mode,
                               reduce_scatter_group_table, union_dictionaries)
from pinot_amd.query import parse_query

pytestmark = pytest.mark.gpu

SCHEMA = [("d", "INT"), ("e", "INT"), ("f", "INT"), ("mi", "INT"), ("md", "DOUBLE")]
WORLD = 2
SEGS_PER_RANK = 3
DOCS = 20000
LIMIT = 5000
SHARDED = ("large", "odd")  # dense cases merged by reduce-scatter (disjoint key ranges per rank)
# name -> (sql, numGroupsLimit, expected combine mode)
CASES = {
    "small": ("SELECT COUNT(*), SUM(mi), MIN(mi), MAX(mi), SUM(md) FROM t WHERE f < 40 GROUP BY d", 10 ** 9, "dense"),
    "large": ("SELECT SUM(mi), COUNT(*) FROM t GROUP BY d, e", 10 ** 9, "dense"),
    # reduce-scattered over a key space of 41 x 27 = 1107 keys: not a multiple of the ranks (padded rows)
    "odd": ("SELECT COUNT(*), SUM(mi), MIN(mi), MAX(md), SUM(md) FROM t WHERE f BETWEEN 10 AND 50 AND d BETWEEN 3 AND 29 "
            "GROUP BY f, d", 10 ** 9, "dense"),
    "hash": ("SELECT COUNT(*), SUM(mi), MIN(md), MAX(mi) FROM t WHERE f >= 10 GROUP BY e, mi", 10 ** 9, "hash"),
    "limit": ("SELECT COUNT(*), SUM(mi), MAX(md) FROM t GROUP BY e, f", LIMIT, "rows"),
}
C5_DOCS = 1_000_000
C4_DOCS = 200_000


def _segment_columns(seg_index):
    rng = np.random.default_rng(5000 + seg_index)
    d = rng.integers(0, 40, DOCS) + 7 * (seg_index % 3)  # ranks see different group values
    return {"d": d.astype(np.int64), "e": rng.integers(0, 3000, DOCS).astype(np.int64),
            "f": rng.integers(0, 100, DOCS).astype(np.int64),
            "mi": rng.integers(-5000, 70000, DOCS).astype(np.int64), "md": rng.uniform(-1e6, 1e6, DOCS)}


def _dump(path, table, res, q):
    """A result as value-space key columns + aggregation values (the order of groups does not matter)."""
    cols = res.gid_columns
    keys = np.stack([np.asarray(table.dictionary(c))[g] for c, g in zip(q.group_by, cols)], axis=1) if len(res) else \
        np.zeros((0, len(q.group_by)))
    vals = [(v if v is not None else e.astype(np.float64)) for fn, v, e, c in res._col[2]]
    vals = np.array(vals).reshape(len(q.aggregations), len(res))
    np.savez(path, keys=keys.astype(np.float64), vals=vals)


def _run_dense(table, handles, q, stream, shard):
    probe = table.plan(handles, q)
    nslots, nkeys, kinds = probe.layout()
    probe.close()
    d_table = torch.empty((nslots, nkeys), dtype=torch.int64, device="cuda")
    plan = table.plan_execute(handles, q, stream, d_table.data_ptr())
    if shard:
        part, k0, kn = reduce_scatter_group_table(d_table, kinds)
        res = plan.finalize_range(stream, part.data_ptr(), k0, kn)
    else:
        allreduce_group_table(d_table, kinds)
        res = plan.finalize(stream, d_table.data_ptr())
    plan.close()
    return res


def _run_dense_comm(table, handles, q, stream, shard, comm):
    """The same merge through the C ABI (pgpu_plan_combine_mode / pgpu_plan_combine): all-reduce into a caller
    table, or reduce-scatter of the plan's own table (finalize then reads this rank's key range)."""
    from pinot_amd import _lib as L
    from pinot_amd.combine import combine_mode, combine_plan
    probe = table.plan(handles, q)
    nslots, nkeys, _ = probe.layout()
    mode, kinds = combine_mode(probe, comm, 0 if shard else 1 << 62)
    probe.close()
    assert mode == (L.COMBINE_REDUCE_SCATTER if shard else L.COMBINE_ALL_REDUCE), mode
    d_table = None if shard else torch.empty((nslots, nkeys), dtype=torch.int64, device="cuda")
    ptr = d_table.data_ptr() if d_table is not None else None
    plan = table.plan_execute(handles, q, stream, ptr)
    k0, kn = combine_plan(plan, comm, stream, mode, kinds, d_table=ptr)
    if shard:
        chunk = -(-nkeys // WORLD)
        assert (k0, kn) == (min(nkeys, comm.rank * chunk), min(nkeys, (comm.rank + 1) * chunk) - min(nkeys, comm.rank * chunk))
    res = plan.finalize(stream, ptr)
    plan.close()
    return res


class _TorchMerge:
    """Collectives through torch.distributed (gloo here, RCCL on a node): pinot_amd.combine's torch functions."""

    def __init__(self, rank, port):
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        # a rank that fails must not leave the other waiting in a collective forever
        dist.init_process_group("gloo", rank=rank, world_size=WORLD, timeout=datetime.timedelta(seconds=90))

    def union(self, table, cols):
        union_dictionaries(table, cols)

    def query(self, table, handles, q, stream, name):
        mode = plan_combine_mode(table, handles, q)
        if mode == "dense":
            res = _run_dense(table, handles, q, stream, shard=name in SHARDED)
        elif mode == "hash":
            plan = table.plan_execute(handles, q, stream)
            exchange_hash_table(plan)
            res = plan.finalize(stream)
            plan.close()
        else:
            res = exchange_result(table, table.execute_groupby(handles, q, stream))
        return mode, res

    def dense(self, table, handles, q, stream, shard):
        return _run_dense(table, handles, q, stream, shard)

    def close(self):
        dist.destroy_process_group()


class _CommMerge:
    """Collectives issued by libpinotgpu (pgpu_comm, host transport: two ranks on one GPU) -- the path a JNI server
    takes, with the combine in the C ABI."""

    def __init__(self, rank, uid):
        from pinot_amd import _lib as L
        from pinot_amd.combine import Communicator
        self.comm = Communicator(L.COMM_HOST, uid, WORLD, rank, 0)

    def union(self, table, cols):
        from pinot_amd.combine import union_dictionaries_comm
        union_dictionaries_comm(table, cols, self.comm)

    def query(self, table, handles, q, stream, name):
        from pinot_amd import _lib as L
        from pinot_amd.combine import combine_mode, combine_plan, combine_result_rows
        probe = table.plan(handles, q)
        mode, kinds = combine_mode(probe, self.comm, 0 if name in SHARDED else 1 << 62)
        probe.close()
        if mode in (L.COMBINE_ALL_REDUCE, L.COMBINE_REDUCE_SCATTER):
            return "dense", _run_dense_comm(table, handles, q, stream, mode == L.COMBINE_REDUCE_SCATTER, self.comm)
        if mode == L.COMBINE_HASH:
            plan = table.plan_execute(handles, q, stream)
            combine_plan(plan, self.comm, stream, mode, kinds)
            res = plan.finalize(stream)
            plan.close()
            return "hash", res
        assert mode == L.COMBINE_ROWS, mode
        return "rows", combine_result_rows(table, table.execute_groupby(handles, q, stream), self.comm)

    def dense(self, table, handles, q, stream, shard):
        return _run_dense_comm(table, handles, q, stream, shard, self.comm)

    def close(self):
        self.comm.close()


def _worker(rank, port, out_dir, transport="torch", uid=None):
    merge = _TorchMerge(rank, port) if transport == "torch" else _CommMerge(rank, uid)
    try:
        import _oracle
        from bench import attach_star_trees
        from pinot_amd.executor import GpuTable
        from pinot_amd.workloads import WORKLOADS
        torch.cuda.set_device(0)
        # a real stream: handle 0 (the default stream) means "the table's own stream" to the C ABI, and the
        # collectives' copies on torch's stream would not wait for the scan
        torch.cuda.set_stream(torch.cuda.Stream())
        stream = torch.cuda.current_stream().cuda_stream
        assert stream != 0
        table = GpuTable(SCHEMA, device=0)
        mine = [rank * SEGS_PER_RANK + i for i in range(SEGS_PER_RANK)]
        handles = [table.pin_segment(_oracle.make_segment(SCHEMA, _segment_columns(s))) for s in mine]
        merge.union(table, ["d", "e", "f", "mi"])
        modes = {}
        for name, (sql, limit, _) in CASES.items():
            q = parse_query(sql, num_groups_limit=limit)
            modes[name], res = merge.query(table, handles, q, stream, name)
            _dump(os.path.join(out_dir, "%s_%d.npz" % (name, rank)), table, res, q)
        table.close()
        with open(os.path.join(out_dir, "modes_%d.txt" % rank), "w") as f:
            f.write(" ".join("%s=%s" % kv for kv in sorted(modes.items())))

        # C5 shape: one 1M-doc segment per rank, 10M-key dense table (partitioned group-by), reduce-scattered
        w = WORKLOADS["c5"]()
        t5 = GpuTable(w.schema, device=0)
        h5 = [t5.generate_segment(w.gen, row0=rank * C5_DOCS, num_docs=C5_DOCS)]
        merge.union(t5, ["k1", "k2", "k3"])
        q5 = parse_query(w.sql, num_groups_limit=w.num_groups_limit)
        _dump(os.path.join(out_dir, "c5_%d.npz" % rank), t5, merge.dense(t5, h5, q5, stream, shard=True), q5)
        t5.close()

        # star-tree: one C4 segment per rank with its star-tree, into the caller table, all-reduced
        w = WORKLOADS["c4"]()
        t4 = GpuTable(w.schema, device=0)
        h4 = [t4.generate_segment(w.gen, row0=rank * C4_DOCS, num_docs=C4_DOCS)]
        attach_star_trees(t4, h4, w, C4_DOCS)
        merge.union(t4, ["d1", "d2"])
        q4 = parse_query(w.sql, num_groups_limit=w.num_groups_limit)
        probe = t4.plan(h4, q4)
        star_segments = probe.star_work()  # segments the plan answers from their star-trees
        probe.close()
        _dump(os.path.join(out_dir, "c4_%d.npz" % rank), t4, merge.dense(t4, h4, q4, stream, shard=False), q4)
        with open(os.path.join(out_dir, "c4_star_%d.txt" % rank), "w") as f:
            f.write(str(star_segments[0]))
        t4.close()
    finally:
        merge.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(tmp_path, limit_s=200, transport="torch"):
    uid = None
    if transport == "comm":
        from pinot_amd.combine import Communicator
        from pinot_amd import _lib as L
        uid = Communicator.unique_id(L.COMM_HOST)
    ctx = mp.spawn(_worker, args=(_free_port(), str(tmp_path), transport, uid), nprocs=WORLD, join=False)
    t0 = time.time()
    while not ctx.join(timeout=5):
        if time.time() - t0 > limit_s:
            for p in ctx.processes:
                if p.is_alive():
                    p.kill()
            pytest.fail("ranks did not finish within %d s" % limit_s)


def _load(path):
    z = np.load(path)
    return z["keys"], z["vals"]


def _as_map(keys, vals):
    return {tuple(k): vals[:, i] for i, k in enumerate(keys.tolist())}


def _broker_merge(parts, fns):
    """Server responses merged by key (AggregationFunction.merge): COUNT / SUM add, MIN / MAX fold."""
    out = {}
    for keys, vals in parts:
        for i, k in enumerate(keys.tolist()):
            k = tuple(k)
            v = vals[:, i]
            if k not in out:
                out[k] = v.copy()
                continue
            for a, fn in enumerate(fns):
                out[k][a] = min(out[k][a], v[a]) if fn == "MIN" else max(out[k][a], v[a]) if fn == "MAX" else \
                    out[k][a] + v[a]
    return out


def _oracle_arrays(oracle, schema, segs, q, **kw):
    keys, vals, _, _ = oracle.run_groupby_arrays(schema, segs, q, **kw)
    return keys.astype(np.float64), vals


def _compare(name, got, exp, q, fp_cols):
    missing, extra = set(exp) - set(got), set(got) - set(exp)
    assert not missing and not extra, (name, len(missing), len(extra), sorted(missing)[:3], sorted(extra)[:3])
    for key, ev in exp.items():
        gv = got[key]
        for a, (fn, col) in enumerate(q.aggregations):
            if col in fp_cols and fn in ("SUM", "AVG"):
                assert gv[a] == pytest.approx(ev[a], rel=1e-9, abs=1e-6), (name, key, fn, col)
            else:
                assert gv[a] == ev[a], (name, key, fn, col, gv[a], ev[a])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("transport", ["torch", "comm"])
def test_two_rank_query_flow_matches_oracle(oracle, gpu_lib, tmp_path, transport):
    """transport "torch": the collectives in pinot_amd.combine over torch.distributed (gloo); "comm": the combine
    inside the C ABI (pgpu_plan_combine / pgpu_result_combine_rows over the host transport)."""
    _run_ranks(tmp_path, transport=transport)
    for r in range(WORLD):
        modes = dict(kv.split("=") for kv in open(tmp_path / ("modes_%d.txt" % r)).read().split())
        assert modes == {name: c[2] for name, c in CASES.items()}, modes
    segs = [oracle.make_segment(SCHEMA, _segment_columns(s)) for s in range(WORLD * SEGS_PER_RANK)]
    for name, (sql, limit, mode) in CASES.items():
        q = parse_query(sql, num_groups_limit=limit)
        parts = [_load(tmp_path / ("%s_%d.npz" % (name, r))) for r in range(WORLD)]
        maps = [_as_map(*p) for p in parts]
        if name == "small":  # all-reduce: both ranks hold the whole answer
            assert maps[0].keys() == maps[1].keys() and all((maps[0][k] == maps[1][k]).all() for k in maps[0])
            got = maps[0]
        else:  # disjoint shares: together they are the answer
            assert not set(maps[0]) & set(maps[1]), name
            got = {**maps[0], **maps[1]}
        fns = [fn for fn, _ in q.aggregations]
        if name == "limit":  # each rank a server under numGroupsLimit, then the broker's merge
            per_rank = [_oracle_arrays(oracle, SCHEMA, segs[r * SEGS_PER_RANK:(r + 1) * SEGS_PER_RANK], q,
                                       max_initial_capacity=min(10000, LIMIT)) for r in range(WORLD)]
            assert all(len(k) <= 2 * LIMIT for k, _ in per_rank)  # the PQL cap bound on every rank
            exp = _broker_merge(per_rank, fns)
        else:
            exp = _as_map(*_oracle_arrays(oracle, SCHEMA, segs, q))
        _compare(name, got, exp, q, {"md"})

    from pinot_amd import _lib as L
    from pinot_amd.workloads import WORKLOADS
    for wname, docs in (("c5", C5_DOCS), ("c4", C4_DOCS)):
        w = WORKLOADS[wname]()
        q = parse_query(w.sql, num_groups_limit=w.num_groups_limit)
        wsegs = []
        for r in range(WORLD):
            from pinot_amd.segment import SegmentBuffers
            cols = {n: oracle.build_column(L.TYPE_NAMES[t], oracle.gen_values(g, r * docs, docs))
                    for (n, t), g in zip(w.schema, w.gen)}
            wsegs.append(SegmentBuffers(docs, cols))
        parts = [_load(tmp_path / ("%s_%d.npz" % (wname, r))) for r in range(WORLD)]
        if wname == "c5":
            assert not set(map(tuple, parts[0][0].tolist())) & set(map(tuple, parts[1][0].tolist()))
            keys = np.concatenate([p[0] for p in parts])
            vals = np.concatenate([p[1] for p in parts], axis=1)
        else:
            keys, vals = parts[0]
            assert np.array_equal(keys, parts[1][0]) and np.array_equal(vals, parts[1][1])
            assert all(int(open(tmp_path / ("c4_star_%d.txt" % r)).read()) == 1 for r in range(WORLD))
        ek, ev = _oracle_arrays(oracle, w.schema, wsegs, q)
        og, oe = np.lexsort(keys.T[::-1]), np.lexsort(ek.T[::-1])
        np.testing.assert_array_equal(keys[og], ek[oe], err_msg=wname)
        np.testing.assert_array_equal(vals[:, og], ev[:, oe], err_msg=wname)


def _failing_rank_worker(rank, uid, out_dir):
    """HASH-mode combine where rank 1 passes a plan it never executed (its own check fails): both ranks must return
    an error, quickly -- rank 0 from the status word of the counts exchange -- and neither may hang in a collective
    (a rank that failed alone left its peers blocked)."""
    import time
    from pinot_amd import _lib as L
    from pinot_amd.combine import Communicator, combine_mode, combine_plan, union_dictionaries_comm
    from pinot_amd.executor import GpuTable
    import _oracle
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    comm = Communicator(L.COMM_HOST, uid, WORLD, rank, 0)
    comm.set_timeout(60_000)
    table = GpuTable(SCHEMA, device=0)
    try:
        handles = [table.pin_segment(_oracle.make_segment(SCHEMA, _segment_columns(rank * SEGS_PER_RANK + i)))
                   for i in range(SEGS_PER_RANK)]
        union_dictionaries_comm(table, ["d", "e", "f", "mi"], comm)
        q = parse_query(CASES["hash"][0], num_groups_limit=CASES["hash"][1])
        probe = table.plan(handles, q)
        mode, kinds = combine_mode(probe, comm, 0)
        probe.close()
        assert mode == L.COMBINE_HASH, mode
        plan = table.plan(handles, q) if rank == 1 else table.plan_execute(handles, q, stream.cuda_stream)
        t0 = time.monotonic()
        try:
            combine_plan(plan, comm, stream.cuda_stream, mode, kinds)
            outcome = "ok"
        except L.PinotGpuError as e:
            outcome = "%d %s" % (e.code, e.message)
        waited = time.monotonic() - t0
        stream.synchronize()
        plan.close()
        with open(os.path.join(out_dir, "fail_%d.txt" % rank), "w") as f:
            f.write("%.3f\n%s" % (waited, outcome))
    finally:
        table.close()
        comm.close()


@pytest.mark.timeout(200)
def test_combine_rank_failure_fails_every_rank(gpu_lib, tmp_path):
    from pinot_amd import _lib as L
    from pinot_amd.combine import Communicator
    uid = Communicator.unique_id(L.COMM_HOST)
    ctx = mp.spawn(_failing_rank_worker, args=(uid, str(tmp_path)), nprocs=WORLD, join=False)
    t0 = time.time()
    while not ctx.join(timeout=5):
        if time.time() - t0 > 150:
            for p in ctx.processes:
                if p.is_alive():
                    p.kill()
            pytest.fail("ranks did not finish")
    res = {}
    for r in range(WORLD):
        waited, outcome = open(tmp_path / ("fail_%d.txt" % r)).read().split("\n", 1)
        res[r] = (float(waited), outcome)
    assert res[1][1].startswith(str(L.PGPU_ERR_INVALID_ARGUMENT)) and "not executed" in res[1][1], res
    assert res[0][1].startswith(str(L.PGPU_ERR_INVALID_ARGUMENT)) and "rank 1 of 2 failed" in res[0][1], res
    assert res[0][0] < 30 and res[1][0] < 30, res


def _recovery_worker(rank, uids, out_dir):
    """Communicator recovery: rank 1 fails a dense all-reduce combine (a plan it never executed),
    so rank 0's all-reduce waits on a peer that never comes, times out and aborts the communicator.  Both ranks then
    recreate it from a fresh id (pgpu_comm_recreate) and the next query combines correctly."""
    import time
    from pinot_amd import _lib as L
    from pinot_amd.combine import Communicator, combine_mode, combine_plan, union_dictionaries_comm
    from pinot_amd.executor import GpuTable
    import _oracle
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    stream = torch.cuda.current_stream().cuda_stream
    comm = Communicator(L.COMM_HOST, uids[0], WORLD, rank, 0)
    comm.set_timeout(3000)
    table = GpuTable(SCHEMA, device=0)
    lines = []
    try:
        handles = [table.pin_segment(_oracle.make_segment(SCHEMA, _segment_columns(rank * SEGS_PER_RANK + i)))
                   for i in range(SEGS_PER_RANK)]
        union_dictionaries_comm(table, ["d", "e", "f", "mi"], comm)
        q = parse_query(CASES["small"][0], num_groups_limit=CASES["small"][1])
        probe = table.plan(handles, q)
        nslots, nkeys, _ = probe.layout()
        mode, kinds = combine_mode(probe, comm, 1 << 62)
        probe.close()
        assert mode == L.COMBINE_ALL_REDUCE, mode
        d_table = torch.empty((nslots, nkeys), dtype=torch.int64, device="cuda")
        ptr = d_table.data_ptr()
        plan = table.plan(handles, q) if rank == 1 else table.plan_execute(handles, q, stream, ptr)
        t0 = time.monotonic()
        try:
            combine_plan(plan, comm, stream, mode, kinds, d_table=ptr)
            plan.finalize(stream, ptr)
            outcome = "ok"
        except L.PinotGpuError as e:
            outcome = "%d %s" % (e.code, e.message.replace("\n", " "))
        lines.append("%.3f %d %s" % (time.monotonic() - t0, int(comm.aborted), outcome))
        plan.close()
        # recovery: every rank recreates the communicator from a new id, then the query runs again
        comm.recreate(uids[1])
        lines.append("recreated %d" % int(comm.aborted))
        res = _run_dense_comm(table, handles, q, stream, False, comm)
        _dump(os.path.join(out_dir, "recovered_%d.npz" % rank), table, res, q)
    finally:
        with open(os.path.join(out_dir, "recovery_%d.txt" % rank), "w") as f:
            f.write("\n".join(lines))
        table.close()
        comm.close()


@pytest.mark.timeout(200)
def test_comm_recreate_after_rank_failure(oracle, gpu_lib, tmp_path):
    from pinot_amd import _lib as L
    from pinot_amd.combine import Communicator
    uids = [Communicator.unique_id(L.COMM_HOST), Communicator.unique_id(L.COMM_HOST)]
    ctx = mp.spawn(_recovery_worker, args=(uids, str(tmp_path)), nprocs=WORLD, join=False)
    t0 = time.time()
    while not ctx.join(timeout=5):
        if time.time() - t0 > 150:
            for p in ctx.processes:
                if p.is_alive():
                    p.kill()
            pytest.fail("ranks did not finish")
    logs = [open(tmp_path / ("recovery_%d.txt" % r)).read().split("\n") for r in range(WORLD)]
    # rank 1 fails its own check at once; rank 0's all-reduce gives up at the 3 s communicator timeout and aborts it
    assert logs[1][0].split(" ", 2)[2].startswith(str(L.PGPU_ERR_INVALID_ARGUMENT)), logs
    w0, ab0, out0 = logs[0][0].split(" ", 2)
    assert out0.startswith(str(L.PGPU_ERR_TIMEOUT)) and int(ab0) == 1 and float(w0) < 30, logs
    assert logs[0][1] == "recreated 0" and logs[1][1] == "recreated 0", logs
    q = parse_query(CASES["small"][0], num_groups_limit=CASES["small"][1])
    parts = [_load(tmp_path / ("recovered_%d.npz" % r)) for r in range(WORLD)]
    maps = [_as_map(*p) for p in parts]
    assert maps[0].keys() == maps[1].keys() and all((maps[0][k] == maps[1][k]).all() for k in maps[0])
    segs = [oracle.make_segment(SCHEMA, _segment_columns(s)) for s in range(WORLD * SEGS_PER_RANK)]
    _compare("recovered", maps[0], _as_map(*_oracle_arrays(oracle, SCHEMA, segs, q)), q, {"md"})
