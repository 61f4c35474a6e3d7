"""The multi-GPU query flow end to end on the device, world_size 2 (both ranks on the box's one GPU, gloo with
host-staged collectives; on a node the same code runs over RCCL): each rank pins its own segments, the ranks union
their group-by dictionaries (one key space), plan + execute streams into a caller-owned device table
(pgpu_plan_create_execute), the tables are merged with an all-reduce (small key spaces) or a reduce-scatter by key
range (large ones, then pgpu_plan_finalize_range per rank), and the merged answer must equal the oracle over the
union of all segments (GroupByCombineOperator semantics, core/operator/combine/GroupByCombineOperator.java:113-160).
This is bench.py's step for --gpus N."""
import datetime
import json
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pinot_amd.combine import allreduce_group_table, reduce_scatter_group_table, union_dictionaries
from pinot_amd.query import parse_query

pytestmark = pytest.mark.gpu

SCHEMA = [("d", "INT"), ("e", "INT"), ("f", "INT"), ("mi", "INT"), ("md", "DOUBLE")]
SMALL = "SELECT COUNT(*), SUM(mi), MIN(mi), MAX(mi), SUM(md) FROM t WHERE f < 40 GROUP BY d"
LARGE = "SELECT SUM(mi), COUNT(*) FROM t GROUP BY d, e"
WORLD = 2
SEGS_PER_RANK = 3
DOCS = 20000


def _segment_columns(seg_index):
    rng = np.random.default_rng(5000 + seg_index)
    d = rng.integers(0, 40, DOCS) + 7 * (seg_index % 3)  # ranks see different group values
    return {"d": d.astype(np.int64), "e": rng.integers(0, 3000, DOCS).astype(np.int64),
            "f": rng.integers(0, 100, DOCS).astype(np.int64),
            "mi": rng.integers(-5000, 70000, DOCS).astype(np.int64), "md": rng.uniform(-1e6, 1e6, DOCS)}


def _worker(rank, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # a rank that fails must not leave the other waiting in a collective forever
    dist.init_process_group("gloo", rank=rank, world_size=WORLD, timeout=datetime.timedelta(seconds=60))
    try:
        import _oracle
        from pinot_amd.executor import GpuTable
        torch.cuda.set_device(0)
        table = GpuTable(SCHEMA, device=0)
        mine = [rank * SEGS_PER_RANK + i for i in range(SEGS_PER_RANK)]
        handles = [table.pin_segment(_oracle.make_segment(SCHEMA, _segment_columns(s))) for s in mine]
        union_dictionaries(table, ["d", "e"])
        # a real stream: handle 0 (the default stream) means "the table's own stream" to the C ABI, and the
        # collectives' copies on torch's stream would not wait for the scan
        torch.cuda.set_stream(torch.cuda.Stream())
        stream = torch.cuda.current_stream().cuda_stream
        assert stream != 0
        for name, sql, shard in (("small", SMALL, False), ("large", LARGE, True)):
            q = parse_query(sql, num_groups_limit=10 ** 9)
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
            rows = [[[int(x) for x in k], [float(x) for x in v]] for k, v in res.as_dict().items()]
            with open(os.path.join(out_dir, "%s_%d.json" % (name, rank)), "w") as f:
                json.dump(rows, f)
        table.close()
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _load(path):
    with open(path) as f:
        return {tuple(k): v for k, v in json.load(f)}


def _run_ranks(tmp_path, limit_s=100):
    ctx = mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=False)
    t0 = time.time()
    while not ctx.join(timeout=5):
        if time.time() - t0 > limit_s:
            for p in ctx.processes:
                if p.is_alive():
                    p.kill()
            pytest.fail("ranks did not finish within %d s" % limit_s)


@pytest.mark.timeout(150)
def test_two_rank_query_flow_matches_oracle(oracle, gpu_lib, tmp_path):
    _run_ranks(tmp_path)
    segs = [oracle.make_segment(SCHEMA, _segment_columns(s)) for s in range(WORLD * SEGS_PER_RANK)]
    for name, sql, shard in (("small", SMALL, False), ("large", LARGE, True)):
        q = parse_query(sql, num_groups_limit=10 ** 9)
        exp = oracle.run_groupby(SCHEMA, segs, q, nthreads=4).groups
        parts = [_load(tmp_path / ("%s_%d.json" % (name, r))) for r in range(WORLD)]
        if shard:  # disjoint key ranges: the ranks' results together are the answer
            assert not set(parts[0]) & set(parts[1])
            got = dict(parts[0])
            got.update(parts[1])
        else:  # all-reduce: both ranks hold the whole answer
            assert parts[0] == parts[1], "all-reduce left the ranks with different answers"
            got = parts[0]
        missing, extra = set(exp) - set(got), set(got) - set(exp)
        assert not missing and not extra, (name, len(missing), len(extra), sorted(missing)[:5], sorted(extra)[:5])
        for key, vals in exp.items():
            for (fn, col), x, y in zip(q.aggregations, got[key], vals):
                if col == "md":
                    assert x == pytest.approx(float(y), rel=1e-9, abs=1e-6), (name, key)
                else:
                    assert x == float(y), (name, key, fn)
