"""bench.py's rank plumbing on the CPU: `--gpus N` without a launcher starts N ranks itself, under a launcher
WORLD_SIZE must equal --gpus, more RCCL ranks than visible GPUs fail fast, and the spawner ends the other ranks when
one fails (a rank left waiting in a collective for a dead peer never returns)."""
import os
import subprocess
import sys
import textwrap
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launch_mode_cases():
    assert bench.launch_mode(1, {}, 0) == ("single", 1)
    assert bench.launch_mode(1, {}, 8) == ("single", 1)
    assert bench.launch_mode(8, {}, 8) == ("spawn", 8)
    assert bench.launch_mode(2, {"WORLD_SIZE": "2", "RANK": "1"}, 8) == ("rank", 2)
    assert bench.launch_mode(1, {"WORLD_SIZE": "1"}, 1) == ("rank", 1)
    # the host transport rehearses N ranks on fewer GPUs
    assert bench.launch_mode(2, {"PGPU_BENCH_BACKEND": "host"}, 1) == ("spawn", 2)
    with pytest.raises(SystemExit, match="8 GPU|1 GPU"):
        bench.launch_mode(8, {}, 1)
    with pytest.raises(SystemExit, match="WORLD_SIZE=4"):
        bench.launch_mode(8, {"WORLD_SIZE": "4"}, 8)
    with pytest.raises(SystemExit, match=">= 1"):
        bench.launch_mode(0, {}, 8)


def test_rank_env_is_a_launcher_rank():
    env = bench.rank_env({"PATH": "/bin", "WORLD_SIZE": "9", "PGPU_BENCH_PMC": "x", "MASTER_PORT": "1"}, 3, 8, 4242)
    assert env["RANK"] == env["LOCAL_RANK"] == "3"
    assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "8"
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "4242"
    assert "PGPU_BENCH_PMC" not in env and env["PATH"] == "/bin"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_segment_split_covers_every_segment():
    """Strong scaling: the ranks' segment ranges partition the workload's segments (main()'s arithmetic)."""
    for total in (1, 7, 100, 1000):
        for world in (1, 2, 3, 8):
            got = []
            for r in range(world):
                first = r * total // world
                got += list(range(first, (r + 1) * total // world))
            assert got == list(range(total))


def _script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def test_spawn_ranks_all_succeed(tmp_path):
    out = tmp_path / "seen"
    out.mkdir()
    script = _script(tmp_path, """
        import os, sys
        open(os.path.join(sys.argv[1], os.environ["RANK"]), "w").write(
            "%s %s %s %s" % (os.environ["WORLD_SIZE"], os.environ["LOCAL_RANK"], os.environ["MASTER_ADDR"],
                             os.environ.get("PGPU_BENCH_PMC", "-")))
    """)
    rc = bench.spawn_ranks(3, [str(out)], {"PGPU_BENCH_PMC": "p.json"}, poll_s=0.05, script=script)
    assert rc == 0
    seen = {f: open(os.path.join(out, f)).read().split() for f in os.listdir(out)}
    assert sorted(seen) == ["0", "1", "2"]
    assert all(v[0] == "3" and v[2] == "127.0.0.1" for v in seen.values())
    assert seen["0"][3] == "p.json" and seen["1"][3] == "-" and seen["2"][1] == "2"


def test_spawn_ranks_failure_ends_the_others(tmp_path):
    """Rank 1 fails at once; rank 0 would wait forever (as in a collective with a dead peer): the spawner returns
    rank 1's code after terminating rank 0."""
    script = _script(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(7)
        time.sleep(600)
    """)
    t0 = time.monotonic()
    rc = bench.spawn_ranks(2, [], poll_s=0.05, grace_s=5.0, script=script)
    assert rc == 7
    assert time.monotonic() - t0 < 60


def test_spawn_ranks_kills_a_rank_that_ignores_sigterm(tmp_path):
    script = _script(tmp_path, """
        import os, signal, sys, time
        if os.environ["RANK"] == "0":
            signal.signal(signal.SIGTERM, signal.SIG_IGN)
            time.sleep(600)
        time.sleep(0.5)
        sys.exit(3)
    """)
    t0 = time.monotonic()
    rc = bench.spawn_ranks(2, [], poll_s=0.05, grace_s=1.0, script=script)
    assert rc == 3
    assert time.monotonic() - t0 < 60


def test_bench_gpus_8_without_gpus_fails_fast():
    """`python3 bench.py --gpus 8` where fewer GPUs are visible (here: none) exits non-zero with the reason, before
    any segment is generated."""
    env = {k: v for k, v in os.environ.items() if k not in bench.DIST_ENV and k != "PGPU_BENCH_BACKEND"}
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert p.returncode != 0
    assert "RCCL takes one GPU per rank" in p.stderr
    assert p.stdout == ""
    assert time.monotonic() - t0 < 240


def test_bench_world_size_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)
    assert p.returncode != 0 and "must match" in p.stderr


def test_merge_partial_arrays_is_the_broker_merge():
    """The numpy merge the N > 1 parity leg uses: per group SUM / COUNT / AVG pairs add, MIN / MAX take min / max."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle
    aggs = [("COUNT", "*"), ("SUM", "m"), ("MIN", "m"), ("MAX", "m"), ("AVG", "m")]
    rng = np.random.default_rng(3)
    rows = [(int(k), float(v)) for k, v in zip(rng.integers(0, 50, 2000), rng.integers(-100, 100, 2000))]
    expect = {}
    for k, v in rows:
        e = expect.setdefault(k, [0, 0.0, v, v, 0.0, 0])
        e[0] += 1
        e[1] += v
        e[2] = min(e[2], v)
        e[3] = max(e[3], v)
        e[4] += v
        e[5] += 1
    parts = []
    for chunk in np.array_split(np.arange(len(rows)), 4):
        g = {}
        for i in chunk:
            k, v = rows[i]
            e = g.setdefault(k, [0, 0.0, v, v, 0.0, 0])
            e[0] += 1
            e[1] += v
            e[2] = min(e[2], v)
            e[3] = max(e[3], v)
            e[4] += v
            e[5] += 1
        ks = sorted(g)
        keys = np.array(ks, dtype=np.int64).reshape(-1, 1)
        vals = np.array([[g[k][0] for k in ks], [g[k][1] for k in ks], [g[k][2] for k in ks], [g[k][3] for k in ks],
                         [g[k][4] for k in ks]], dtype=np.float64)
        cnts = np.zeros_like(vals, dtype=np.int64)
        cnts[4] = [g[k][5] for k in ks]
        parts.append((keys, vals, cnts, (len(chunk), len(chunk), 2 * len(chunk), len(chunk))))
    keys, vals, cnts, stats = _oracle.merge_partial_arrays(parts, aggs)
    assert [int(k) for k in keys[:, 0]] == sorted(expect)
    for i, k in enumerate(keys[:, 0]):
        e = expect[int(k)]
        assert list(vals[:, i]) == [e[0], e[1], e[2], e[3], e[4]] and cnts[4, i] == e[5]
    assert stats == (2000, 2000, 4000, 2000)


def test_parse_config_fields():
    """bench.py --config: pgpu_config fields as integers / floats; the names must be the ABI's (GpuTable rejects
    unknown ones)."""
    from pinot_amd import _lib as L
    cfg = bench.parse_config("dense_selectivity=0.5,plan_cache=0, stream_chunks=3")
    assert cfg == {"dense_selectivity": 0.5, "plan_cache": 0, "stream_chunks": 3}
    assert set(cfg) <= set(L.CONFIG_FIELDS)
    assert bench.parse_config(None) == {} and bench.parse_config("") == {}
