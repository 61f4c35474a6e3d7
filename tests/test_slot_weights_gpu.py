"""Chunked scans weighted by CU slot (pgpu_config.slot_weight_step, r06): the weights only move tiles between the
workgroups of a launch, so every weighting -- none, the default, an extreme one -- returns the same groups, values and
statistics.  300 C3 segments of 1 M rows (36 900 tiles, >= 32 per workgroup of the 1 024-workgroup grid, so the
weighted split runs when the launch is alone on the table)."""
import pytest

from pinot_amd.executor import GpuTable
from pinot_amd.query import parse_query
from pinot_amd.workloads import WORKLOADS

pytestmark = pytest.mark.gpu

DOCS = 1_000_000
SEGS = 300


@pytest.fixture(scope="module")
def c3_table(gpu_lib):
    w = WORKLOADS["adanalytics"]()
    t = GpuTable(w.schema, device=0)
    handles = [t.generate_segment(w.gen, row0=i * DOCS, num_docs=DOCS) for i in range(SEGS)]
    yield t, handles, w
    t.close()


@pytest.mark.parametrize("sql", [
    None,  # the workload's query (two scan leaves in leap-frog, LEAP2 statistics)
    "SELECT COUNT(*), SUM(clicks), MAX(impressions) FROM t WHERE accountId IN (123456789, 4242) GROUP BY daysSinceEpoch",
    "SELECT COUNT(*), MIN(clicks) FROM t WHERE daysSinceEpoch BETWEEN 17600 AND 17610 GROUP BY accountId",
])
def test_weights_change_nothing_but_the_split(c3_table, sql):
    t, handles, w = c3_table
    q = parse_query(sql or w.sql, num_groups_limit=w.num_groups_limit)
    out = []
    for step in (0.0, 0.11, 3.0):
        t.set_config(slot_weight_step=step)
        r = t.execute_groupby(handles, q)
        out.append((r.as_dict(), r.stats.as_tuple()))
    t.set_config(slot_weight_step=0.11)
    assert out[0][0] and out[0] == out[1] == out[2]
