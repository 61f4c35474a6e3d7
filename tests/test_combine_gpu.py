"""The cross-GPU combine inside the C ABI over RCCL (pgpu_comm, PGPU_COMM_RCCL) with a one-rank communicator on the
box's GPU: every combine mode runs its real RCCL calls (all-reduce, reduce-scatter, the grouped send/recv of the hash
exchange and of the row exchange, the all-gathers of the mode agreement) and the result must equal the oracle's
(GroupByCombineOperator.java:113-160, GroupByOrderByCombineOperator.java:170-181).  With one rank the merge is the
identity, so these tests pin the plumbing -- buffers, strides, kind agreement, finalize of the merged table -- and
the two-rank host-transport test (test_multi_rank_gpu.py, transport "comm") pins the merge arithmetic of the same
code."""
import numpy as np
import pytest
import torch

from pinot_amd import _lib as L
from pinot_amd.query import parse_query

pytestmark = pytest.mark.gpu

SCHEMA = [("d", "INT"), ("e", "INT"), ("f", "INT"), ("mi", "INT"), ("md", "DOUBLE")]
DOCS = 30000
CASES = [
    # (name, sql, numGroupsLimit, shard_bytes, expected mode)
    ("all_reduce", "SELECT COUNT(*), SUM(mi), MIN(mi), MAX(mi), SUM(md), AVG(md) FROM t WHERE f < 40 GROUP BY d",
     10 ** 9, 1 << 62, L.COMBINE_ALL_REDUCE),
    ("reduce_scatter", "SELECT SUM(mi), COUNT(*), MIN(md) FROM t GROUP BY d, e", 10 ** 9, 0, L.COMBINE_REDUCE_SCATTER),
    ("hash", "SELECT COUNT(*), SUM(mi), MIN(md), MAX(mi) FROM t WHERE f >= 10 GROUP BY e, mi", 10 ** 9, 0,
     L.COMBINE_HASH),
    ("rows", "SELECT COUNT(*), SUM(mi), MAX(md) FROM t GROUP BY e, f", 2000, 0, L.COMBINE_ROWS),
]


def _columns(seg):
    rng = np.random.default_rng(7000 + seg)
    return {"d": rng.integers(0, 40, DOCS).astype(np.int64), "e": rng.integers(0, 3000, DOCS).astype(np.int64),
            "f": rng.integers(0, 100, DOCS).astype(np.int64), "mi": rng.integers(-5000, 70000, DOCS).astype(np.int64),
            "md": rng.uniform(-1e6, 1e6, DOCS)}


@pytest.fixture(scope="module")
def rccl_table(gpu_lib):
    import _oracle
    from pinot_amd.combine import Communicator
    from pinot_amd.executor import GpuTable
    torch.cuda.set_device(0)
    table = GpuTable(SCHEMA, device=0)
    segs = [_oracle.make_segment(SCHEMA, _columns(s)) for s in range(3)]
    handles = [table.pin_segment(s) for s in segs]
    comm = Communicator(L.COMM_RCCL, Communicator.unique_id(L.COMM_RCCL), 1, 0, 0)
    yield table, handles, segs, comm
    comm.close()
    table.close()


def _check(oracle, res, segs, q, limit=None):
    from test_gpu_parity import assert_same
    kw = {"max_initial_capacity": min(10000, limit)} if limit and limit < 10 ** 9 else {}
    assert_same(res, oracle.run_groupby(SCHEMA, segs, q, **kw), q, SCHEMA)


@pytest.mark.parametrize("name,sql,limit,shard_bytes,expect", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("caller_table", [False, True])
def test_rccl_one_rank_combine_matches_oracle(oracle, rccl_table, name, sql, limit, shard_bytes, expect, caller_table):
    from pinot_amd.combine import combine_mode, combine_plan, combine_result_rows
    table, handles, segs, comm = rccl_table
    q = parse_query(sql, num_groups_limit=limit)
    stream = torch.cuda.Stream()
    s = stream.cuda_stream
    probe = table.plan(handles, q)
    mode, kinds = combine_mode(probe, comm, shard_bytes)
    probe.close()
    assert mode == expect
    if mode == L.COMBINE_ROWS:
        res = combine_result_rows(table, table.execute_groupby(handles, q, s), comm)
    else:
        d_table = None
        if caller_table and mode != L.COMBINE_HASH:
            with table.plan(handles, q) as p:
                ns, nk, _ = p.layout()
            d_table = torch.empty((ns, nk), dtype=torch.int64, device="cuda")
        ptr = d_table.data_ptr() if d_table is not None else None
        plan = table.plan_execute(handles, q, s, ptr)
        k0, kn = combine_plan(plan, comm, s, mode, kinds, d_table=ptr)
        if mode == L.COMBINE_REDUCE_SCATTER:
            assert k0 == 0 and kn == plan.layout()[1]
        res = plan.finalize(s, ptr)
        plan.close()
    _check(oracle, res, segs, q, limit)


def test_combine_mode_after_combine_is_rejected(rccl_table):
    from pinot_amd.combine import combine_mode, combine_plan
    table, handles, _, comm = rccl_table
    q = parse_query(CASES[1][1], num_groups_limit=CASES[1][2])
    stream = torch.cuda.Stream()  # held: the C ABI keeps only its handle
    s = stream.cuda_stream
    plan = table.plan_execute(handles, q, s)
    mode, kinds = combine_mode(plan, comm, 0)
    combine_plan(plan, comm, s, mode, kinds)
    with pytest.raises(L.PinotGpuError):
        combine_plan(plan, comm, s, mode, kinds)  # a table is merged once
    with pytest.raises(L.PinotGpuError):
        combine_plan(plan, comm, s, L.COMBINE_ROWS, kinds)
    plan.finalize(s)
    plan.close()
    stream.synchronize()


@pytest.mark.parametrize("name", ["all_reduce", "reduce_scatter", "hash"])
def test_plan_executed_again_after_combine_runs_as_planned(oracle, rccl_table, name):
    """pgpu_plan_combine changed the plan for good (an int64 SUM slot agreed as float64, the
    reduce-scattered shard, the merged hash table), so executing the plan again ran the scan with a float64 slot over
    an integer column and finalize returned the stale shard.  Now exec_prologue restores the planned state: execute,
    combine (with the int64 SUM forced to float64 -- what another rank's float64 sum would agree), execute again,
    finalize -- the answer is the plain one, integers exact."""
    from pinot_amd.combine import combine_mode, combine_plan
    table, handles, segs, comm = rccl_table
    sql, limit, shard_bytes = {c[0]: (c[1], c[2], c[3]) for c in CASES}[name]
    q = parse_query(sql, num_groups_limit=limit)
    stream = torch.cuda.Stream()
    s = stream.cuda_stream
    plan = table.plan(handles, q)
    mode, kinds = combine_mode(plan, comm, shard_bytes)
    forced = [L.SLOT_SUM_F64 if k == L.SLOT_SUM_I64 else k for k in kinds]
    assert forced != kinds  # the query has an integer SUM
    plan.execute(s)
    combine_plan(plan, comm, s, mode, forced)
    first = plan.finalize(s)
    _check(oracle, first, segs, q, limit)
    plan.execute(s)  # again, without a combine
    res = plan.finalize(s)
    plan.close()
    _check(oracle, res, segs, q, limit)  # integer SUMs compared exactly: a float64 slot read as int64 would differ
