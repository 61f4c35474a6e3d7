"""The host transport of pgpu_comm (comm.cpp) between processes, on the CPU: ids, the all-gather every combine mode's
agreement runs on, variable-length gathers (dictionary unions), and argument checks.  The device collectives of both
transports run in tests/test_multi_rank_gpu.py (host, two ranks on one GPU) and tests/test_combine_gpu.py (RCCL, one
rank)."""
import multiprocessing as mp
import struct

import pytest

from pinot_amd import _lib as L


def _rank(uid, rank, world, q):
    try:
        from pinot_amd.combine import Communicator
        c = Communicator(L.COMM_HOST, uid, world, rank, 0)
        got = c.allgather(struct.pack("<q", 100 + rank))
        var = c.allgather_var(b"x" * (rank * 3 + 1))
        c.barrier()
        mx = c.max(rank * 1.5)
        tot = c.sum_int(rank + 1)
        c.close()
        q.put((rank, [struct.unpack("<q", g)[0] for g in got], [len(v) for v in var], mx, tot))
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        q.put((rank, "error: %r" % e))


@pytest.mark.parametrize("world", [1, 2, 3])
def test_host_comm_allgather(world):
    uid = __import__("pinot_amd.combine", fromlist=["Communicator"]).Communicator.unique_id(L.COMM_HOST)
    assert uid.startswith(b"pgpu-comm-")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(uid, r, world, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict()
    for _ in range(world):
        item = q.get(timeout=60)
        out[item[0]] = item[1:]
    for p in procs:
        p.join(timeout=30)
    for r in range(world):
        assert not isinstance(out[r][0], str), out[r]
        gathered, lens, mx, tot = out[r]
        assert gathered == [100 + i for i in range(world)]
        assert lens == [i * 3 + 1 for i in range(world)]
        assert mx == (world - 1) * 1.5
        assert tot == world * (world + 1) // 2


def test_comm_bad_arguments():
    import ctypes
    lib = L.load()
    h = ctypes.c_void_p()
    uid = ctypes.create_string_buffer(b"not-an-id", L.COMM_ID_BYTES)
    assert lib.pgpu_comm_create(L.COMM_HOST, uid, 2, 0, 0, ctypes.byref(h)) == L.PGPU_ERR_INVALID_ARGUMENT
    assert lib.pgpu_comm_create(L.COMM_HOST, uid, 2, 2, 0, ctypes.byref(h)) == L.PGPU_ERR_INVALID_ARGUMENT
    assert lib.pgpu_comm_create(7, uid, 1, 0, 0, ctypes.byref(h)) == L.PGPU_ERR_INVALID_ARGUMENT
    assert lib.pgpu_comm_unique_id(7, uid) == L.PGPU_ERR_INVALID_ARGUMENT


def _pg_rank(rank, port, q):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from pinot_amd.combine import Communicator, union_dictionaries_comm
        c = Communicator.from_process_group(L.COMM_HOST, 0)

        class T:  # the two table methods union_dictionaries_comm uses
            def __init__(self, vals):
                self.vals = vals

            def dictionary(self, col):
                return list(self.vals)

            def add_dictionary_values(self, col, values):
                self.vals = sorted(set(self.vals) | set(values))
        t = T([3, 1, 7] if rank == 0 else [2, 7, 11])
        union_dictionaries_comm(t, ["k"], c)
        c.close()
        try:  # an unknown transport fails on every rank (no rank left waiting in a collective)
            Communicator.from_process_group(7, 0)
            bad = "no error"
        except L.PinotGpuError as e:
            bad = e.message
        q.put((rank, t.vals, bad))
    finally:
        dist.destroy_process_group()


def test_communicator_from_process_group():
    """bench.py's bootstrap: rank 0's id through a gloo process group, dictionary union over the communicator."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_pg_rank, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict((r, rest) for r, *rest in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=30)
    for r in range(2):
        vals, bad = out[r]
        assert vals == [1, 2, 3, 7, 11]
        assert "communicator" in bad


def _absent_peer_rank(uid, rank, q):
    """Rank 1 joins and leaves at once (as a peer that failed before the collective); rank 0's all-gather must end at
    its communicator timeout, not block, and the communicator is unusable afterwards."""
    import time
    try:
        from pinot_amd.combine import Communicator
        c = Communicator(L.COMM_HOST, uid, 2, rank, 0)
        if rank == 1:
            t0 = time.monotonic()
            c.close()  # no barrier on the way out: a peer's teardown never waits for the others
            q.put((rank, "closed", time.monotonic() - t0))
            return
        c.set_timeout(1500)
        t0 = time.monotonic()
        try:
            c.allgather(b"12345678")
            first = ("no error", 0)
        except L.PinotGpuError as e:
            first = (e.code, e.message)
        waited = time.monotonic() - t0
        try:
            c.allgather(b"12345678")
            second = ("no error", 0)
        except L.PinotGpuError as e:
            second = (e.code, e.message)
        t1 = time.monotonic()
        c.close()
        q.put((rank, first, second, waited, time.monotonic() - t1))
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        q.put((rank, "error: %r" % e))


def test_host_comm_absent_peer_times_out_and_aborts():
    """a rank that fails before a collective must not leave its peers blocked forever (the host
    transport gave up only after 600 s, and its destructor ran a barrier)."""
    import os
    from pinot_amd.combine import Communicator
    uid = Communicator.unique_id(L.COMM_HOST)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_absent_peer_rank, args=(uid, r, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict((item[0], item[1:]) for item in (q.get(timeout=120) for _ in range(2)))
    for p in procs:
        p.join(timeout=30)
    assert out[1][0] == "closed" and out[1][1] < 5, out[1]
    first, second, waited, close_s = out[0]
    assert first[0] == L.PGPU_ERR_TIMEOUT and "did not join" in first[1], first
    assert 1.0 <= waited < 30, waited
    assert second[0] == L.PGPU_ERR_DEVICE and "aborted" in second[1], second
    assert close_s < 5
    # the last rank out removed the control file
    assert not os.path.exists("/dev/shm/%s.ctl" % uid.rstrip(b"\0").decode())
