"""Cross-GPU combine: the dense group tables of all ranks are merged with collectives (RCCL over xGMI on the
node; gloo in the CPU tests) instead of GroupByCombineOperator's ConcurrentHashMap merge
(core/operator/combine/GroupByCombineOperator.java:113-160).

Small key spaces (C1-C4: kilobytes) are all-reduced, so every rank holds the merged table.  Large ones (C5: ~10M
groups, 160 MB per GPU) are reduce-scattered instead: rank r ends with the merged key range
[r * chunk, (r + 1) * chunk) and finalizes only that (pgpu_plan_finalize_range) -- half the link traffic of an
all-reduce, 1/N of the compaction and copy-back per rank, and the ranks' results are disjoint.

Every rank's table has the plan's layout ([num_slots][num_keys] 8-byte words, one row per accumulator) in the
table-global key space, so the merge is element-wise: COUNT and integer SUM rows add as int64, floating-point
SUM rows add as float64, MIN / MAX rows (order-preserving int64 keys) take min / max.  Rows of one kind are
reduced by a single collective.
"""
import ctypes

import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L

_OPS = {
    L.SLOT_COUNT: dist.ReduceOp.SUM,
    L.SLOT_SUM_I64: dist.ReduceOp.SUM,
    L.SLOT_SUM_F64: dist.ReduceOp.SUM,
    L.SLOT_MIN_KEY: dist.ReduceOp.MIN,
    L.SLOT_MAX_KEY: dist.ReduceOp.MAX,
}


def _staged(group):
    """gloo collectives on device tensors go through host copies (CPU tests use host tensors directly)."""
    return dist.get_backend(group) == "gloo"


def allreduce_group_table(table, slot_kinds, group=None):
    """In-place all-reduce of a [num_slots, num_keys] int64 tensor holding a plan's dense group table."""
    assert table.dtype == torch.int64 and table.dim() == 2 and table.shape[0] == len(slot_kinds)
    if table.is_cuda and _staged(group):
        host = table.cpu()
        allreduce_group_table(host, slot_kinds, group)
        table.copy_(host)
        return table
    kinds = list(slot_kinds)
    s = 0
    while s < len(kinds):
        e = s + 1
        while e < len(kinds) and _OPS[kinds[e]] == _OPS[kinds[s]] and \
                (kinds[e] == L.SLOT_SUM_F64) == (kinds[s] == L.SLOT_SUM_F64):
            e += 1
        rows = table[s:e]
        if kinds[s] == L.SLOT_SUM_F64:
            dist.all_reduce(rows.view(torch.float64), op=_OPS[kinds[s]], group=group)
        else:
            dist.all_reduce(rows, op=_OPS[kinds[s]], group=group)
        s = e
    return table


def shard_range(num_keys, world, rank):
    """Key range [begin, begin + count) of `rank` in a reduce-scattered table, and the padded chunk width."""
    chunk = -(-num_keys // world)
    begin = min(num_keys, rank * chunk)
    return begin, min(num_keys, begin + chunk) - begin, chunk


def reduce_scatter_group_table(table, slot_kinds, group=None):
    """Reduce-scatter of a [num_slots, num_keys] int64 dense group table by key range.  Returns (shard, key_begin,
    key_count): shard is a contiguous [num_slots, key_count] tensor with this rank's merged keys."""
    assert table.dtype == torch.int64 and table.dim() == 2 and table.shape[0] == len(slot_kinds)
    if table.is_cuda and _staged(group):
        shard, begin, count = reduce_scatter_group_table(table.cpu(), slot_kinds, group)
        return shard.to(table.device), begin, count
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    nslots, G = table.shape
    begin, count, chunk = shard_range(G, world, rank)
    out = torch.empty((nslots, chunk), dtype=torch.int64, device=table.device)
    for s, kind in enumerate(slot_kinds):
        row = table[s]
        if world * chunk != G:  # pad to world x chunk; padded keys have COUNT 0 and are never finalized
            row = torch.nn.functional.pad(row, (0, world * chunk - G))
        if kind == L.SLOT_SUM_F64:
            dist.reduce_scatter_tensor(out[s].view(torch.float64), row.view(torch.float64), op=_OPS[kind],
                                       group=group)
        else:
            dist.reduce_scatter_tensor(out[s], row, op=_OPS[kind], group=group)
    if count != chunk:
        out = out[:, :count].contiguous()
    return out, begin, count


def union_dictionaries(table, columns, group=None):
    """Makes every rank's table-global dictionary of `columns` the union over ranks (one all_gather_object per
    column at setup time), so all ranks' dense tables share one key space."""
    for col in columns:
        mine = table.dictionary(col)
        world = dist.get_world_size(group)
        gathered = [None] * world
        dist.all_gather_object(gathered, mine, group=group)
        union = sorted(set(v for vals in gathered for v in vals))
        table.add_dictionary_values(col, union)


# ---------------------------------------------------------------------------------------------- hash / row exchange
# Key spaces past 2^26 (hash-mode tables) and numGroupsLimit plans do not share a dense layout across ranks, so their
# merge is a hash-partitioned all-to-all (GroupByOrderByCombineOperator's IndexedTable.upsert across servers,
# core/operator/combine/GroupByOrderByCombineOperator.java:170-181): every group goes to one owner rank, which merges
# what it receives; the ranks end with disjoint groups, as Pinot servers return partial tables to the broker.
# numGroupsLimit applies per rank, as per server (each GPU is one server of the table).

def agreed_slot_kinds(kinds, group=None):
    """The slot kinds every rank exchanges in: a rank's int64 SUM travels as float64 when another rank's sum of the
    same slot is float64 (an int64 sum could overflow on that rank's segments: SumAggregationFunction's double)."""
    world = dist.get_world_size(group)
    gathered = [None] * world
    dist.all_gather_object(gathered, [int(k) for k in kinds], group=group)
    out = []
    for s, k in enumerate(kinds):
        ks = {g[s] for g in gathered}
        if ks <= {L.SLOT_SUM_I64, L.SLOT_SUM_F64}:
            out.append(L.SLOT_SUM_F64 if L.SLOT_SUM_F64 in ks else L.SLOT_SUM_I64)
        elif len(ks) == 1:
            out.append(int(k))
        else:
            raise ValueError("ranks disagree on slot %d: kinds %s" % (s, sorted(ks)))
    return out


def all_to_all_rows(send, counts, group=None):
    """send: [n, width] int64 records grouped by destination rank, counts[r] records for rank r.  Returns the
    [m, width] records every rank sent to this one (rank order)."""
    import numpy as np
    world = dist.get_world_size(group)
    width = send.shape[1]
    staged = _staged(group)
    dev = torch.device("cpu") if staged or not send.is_cuda else send.device
    cnt = torch.as_tensor(np.asarray(counts, dtype=np.int64), device=dev)
    rcnt = torch.empty_like(cnt)
    dist.all_to_all_single(rcnt, cnt, group=group)
    rc = [int(x) for x in rcnt.tolist()]
    src = send.to(dev).contiguous().view(-1)
    out = torch.empty((sum(rc), width), dtype=torch.int64, device=dev)
    if world == 1:
        out.copy_(send.to(dev))
    else:
        dist.all_to_all_single(out.view(-1), src, output_split_sizes=[c * width for c in rc],
                               input_split_sizes=[int(c) * width for c in counts], group=group)
    return out.to(send.device) if out.device != send.device else out


def exchange_hash_table(plan, group=None):
    """Cross-rank merge of an executed hash-mode plan (run without a caller table, on torch's current stream): its
    groups are split by owner on the device, exchanged with all_to_all (RCCL over xGMI on a node), and merged into
    this rank's table; plan.finalize(stream) then returns this rank's disjoint share of the merged groups."""
    world = dist.get_world_size(group)
    stream = torch.cuda.current_stream().cuda_stream
    nslots, _, kinds = plan.layout()
    kinds = agreed_slot_kinds(kinds, group)
    counts = plan.exchange_counts(stream, world)
    total = int(counts.sum())
    send = torch.empty((max(total, 1), 1 + nslots), dtype=torch.int64, device="cuda")
    plan.exchange_export(stream, world, kinds, send.data_ptr(), total)
    recv = all_to_all_rows(send[:total], counts, group)
    plan.exchange_merge(stream, kinds, recv.data_ptr() if recv.shape[0] else None, recv.shape[0])
    plan._exchange_keep = recv  # read by the merge kernel queued on the stream: alive until the plan is finalized
    return plan


def exchange_result(table, res, group=None):
    """Cross-rank merge of finalized results of any plan kind (numGroupsLimit plans, ARRAY_MAP key stages): the rows
    [dictIds, slot words] are split by owner on the host, exchanged with all_to_all, and merged by the owner
    (pgpu_result_merge_rows).  Returns this rank's disjoint share of the merged groups as a GroupByResult."""
    from .executor import _decode_result, _ResultHolder
    lib = table.lib
    world = dist.get_world_size(group)
    r = res._holder.r
    ns = ctypes.c_int32()
    kinds = (ctypes.c_int32 * 32)()
    L.check(lib.pgpu_result_slot_kinds(r, ctypes.byref(ns), kinds))
    mine = [kinds[i] for i in range(ns.value)]
    agreed = np.asarray(agreed_slot_kinds(mine, group), dtype=np.int32)
    # group ids index the ranks' dictionary snapshots: they must be the same (union_dictionaries before the query) --
    # compared by content, not only by size
    import hashlib
    digest = hashlib.sha256()
    for j, c in enumerate(res._query.group_by):
        digest.update(repr(list(table.result_dictionary(r, j, c))).encode())
    gathered = [None] * world
    dist.all_gather_object(gathered, digest.hexdigest(), group=group)
    if any(g != gathered[0] for g in gathered):
        raise ValueError("ranks' group-by dictionaries differ: union them before the query")
    nk = len(res._query.group_by)
    n = len(res)
    rows = np.empty((max(n, 1), nk + ns.value), dtype=np.int64)
    counts = np.zeros(world, dtype=np.int64)
    L.check(lib.pgpu_result_exchange_rows(r, world, L.ptr(agreed, ctypes.c_int32), L.ptr(rows, ctypes.c_int64),
                                          L.ptr(counts, ctypes.c_int64)))
    send = torch.from_numpy(rows[:n])
    if not _staged(group):
        send = send.cuda()
    recv = all_to_all_rows(send, counts, group).cpu().numpy()
    recv = np.ascontiguousarray(recv, dtype=np.int64)
    out = ctypes.c_void_p()
    L.check(lib.pgpu_result_merge_rows(r, L.ptr(recv, ctypes.c_int64) if len(recv) else None, len(recv),
                                       L.ptr(agreed, ctypes.c_int32), ctypes.byref(out)))
    return _decode_result(table, res._query, _ResultHolder(lib, out))


def plan_combine_mode(table, handles, query, group=None):
    """How this query's per-rank results merge, agreed by every rank: "dense" (element-wise all-reduce /
    reduce-scatter of the dense tables), "hash" (device all-to-all of hash-mode tables) or "rows" (host rows of the
    finalized results: numGroupsLimit plans and ARRAY_MAP key stages).  A rank whose segments make the query a
    numGroupsLimit plan puts every rank on the row path (the modes must match for the collectives to pair up)."""
    from . import _lib
    world = dist.get_world_size(group)
    probe = table.plan(handles, query)
    try:
        try:
            nslots, nkeys, kinds = probe.layout()
            mode = "dense" if nkeys > 0 else "hash"
        except _lib.PinotGpuError:
            mode = "rows"  # numGroupsLimit plan (its parts have their own tables)
        if mode == "hash":
            # ARRAY_MAP key stages (rank-local slot numbers in the keys) cannot exchange device records; the check
            # comes before the execution state, so the unexecuted probe answers it
            try:
                probe.exchange_counts(None, world)
            except _lib.PinotGpuError as e:
                if e.code == _lib.PGPU_ERR_UNSUPPORTED:
                    mode = "rows"
    finally:
        probe.close()
    gathered = [None] * world
    dist.all_gather_object(gathered, mode, group=group)
    # one mode on every rank, or the row exchange, which merges plans of any kind (a dense rank could not take part
    # in a hash exchange: its collectives would not pair up)
    return gathered[0] if len(set(gathered)) == 1 else "rows"


# ------------------------------------------------------------------------------------- the C ABI combine (pgpu_comm)
# The same merges as above, issued by libpinotgpu itself (include/pinotgpu.h, "communicator and the one-call
# cross-GPU combine"): what a Java server calls through JNI, with no torch in the process.  RCCL over xGMI on a node;
# the host transport runs the identical combine code with several ranks on one GPU (tests, rehearsals).

class Communicator:
    """pgpu_comm: one rank of a group of GPUs (RCCL) or of processes sharing a GPU (host transport)."""

    def __init__(self, kind, uid, nranks, rank, device):
        self.lib = L.load()
        self.kind = kind
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(uid), L.COMM_ID_BYTES)
        L.check(self.lib.pgpu_comm_create(kind, buf, nranks, rank, device, ctypes.byref(h)))
        self.handle = h
        self.rank, self.nranks, self.device = rank, nranks, device

    @staticmethod
    def unique_id(kind=L.COMM_RCCL):
        buf = ctypes.create_string_buffer(L.COMM_ID_BYTES)
        L.check(L.load().pgpu_comm_unique_id(kind, buf))
        return buf.raw

    @classmethod
    def from_process_group(cls, kind, device, group=None):
        """Rank 0 makes the id, the process group (any backend: gloo is enough) hands it to the others.  A failure
        on any rank raises PinotGpuError on every rank (no rank is left waiting in a collective)."""
        rank = dist.get_rank(group)
        box = [None]
        if rank == 0:
            try:
                box[0] = cls.unique_id(kind)
            except L.PinotGpuError as e:
                box[0] = ("error", str(e))
        dist.broadcast_object_list(box, src=0, group=group)
        if isinstance(box[0], tuple):
            raise L.PinotGpuError(L.PGPU_ERR_DEVICE, "communicator id: " + box[0][1])
        comm, err = None, None
        try:
            comm = cls(kind, box[0], dist.get_world_size(group), rank, device)
        except L.PinotGpuError as e:
            err = str(e)
        errs = [None] * dist.get_world_size(group)
        dist.all_gather_object(errs, err, group=group)
        if any(errs):
            if comm is not None:
                comm.close()
            raise L.PinotGpuError(L.PGPU_ERR_DEVICE, "communicator: " + "; ".join(e for e in errs if e))
        return comm

    def close(self):
        if getattr(self, "handle", None):
            self.lib.pgpu_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_timeout(self, ms):
        """pgpu_comm_set_timeout: waits on peers end with PGPU_ERR_TIMEOUT after `ms` (and abort the communicator)."""
        L.check(self.lib.pgpu_comm_set_timeout(self.handle, int(ms)))

    def abort(self):
        L.check(self.lib.pgpu_comm_abort(self.handle))

    @property
    def aborted(self):
        """pgpu_comm_status: the communicator was given up (an expired wait on a peer, or abort())."""
        v = ctypes.c_int32()
        L.check(self.lib.pgpu_comm_status(self.handle, ctypes.byref(v)))
        return bool(v.value)

    def recreate(self, uid):
        """pgpu_comm_recreate (collective): a fresh communicator of the same ranks from a new id, replacing an aborted
        one -- the server keeps serving after one rank's failed combine."""
        buf = ctypes.create_string_buffer(bytes(uid), L.COMM_ID_BYTES)
        L.check(self.lib.pgpu_comm_recreate(self.handle, buf))

    def allgather(self, data):
        """Every rank's `data` (bytes of one length on every rank), in rank order."""
        data = bytes(data)
        out = ctypes.create_string_buffer(max(1, len(data) * self.nranks))
        L.check(self.lib.pgpu_comm_allgather(self.handle, data, len(data), out))
        return [out.raw[i * len(data):(i + 1) * len(data)] for i in range(self.nranks)]

    def allgather_var(self, data):
        """Every rank's `data` (bytes of any length), in rank order."""
        import struct
        sizes = [struct.unpack("<q", b)[0] for b in self.allgather(struct.pack("<q", len(data)))]
        width = max(sizes)
        padded = self.allgather(bytes(data) + b"\0" * (width - len(data)))
        return [p[:n] for p, n in zip(padded, sizes)]

    def barrier(self):
        self.allgather(b"\0")

    def max(self, x):
        import struct
        return max(struct.unpack("<d", b)[0] for b in self.allgather(struct.pack("<d", float(x))))

    def sum_int(self, x):
        import struct
        return sum(struct.unpack("<q", b)[0] for b in self.allgather(struct.pack("<q", int(x))))


def union_dictionaries_comm(table, columns, comm):
    """union_dictionaries over a pgpu_comm (values travel as JSON: exact for ints, floats via repr, and strings)."""
    import json
    for col in columns:
        mine = json.dumps(list(table.dictionary(col))).encode()
        union = sorted(set(v for b in comm.allgather_var(mine) for v in json.loads(b.decode())))
        table.add_dictionary_values(col, union)


def combine_mode(plan, comm, shard_bytes):
    """(mode, kinds) every rank agrees on for this query (pgpu_plan_combine_mode, a collective)."""
    mode = ctypes.c_int32()
    kinds = (ctypes.c_int32 * 32)()
    L.check(plan.lib.pgpu_plan_combine_mode(plan.handle, comm.handle, int(shard_bytes), ctypes.byref(mode), kinds))
    ns = _num_slots(plan)
    return mode.value, [kinds[i] for i in range(ns)]


def _num_slots(plan):
    try:
        return plan.layout()[0]
    except L.PinotGpuError:  # numGroupsLimit plan: the kinds come with the rows
        return 0


def combine_plan(plan, comm, stream, mode, kinds=None, d_table=None, d_shard=None):
    """pgpu_plan_combine on the executed plan (ordered on `stream`); plan.finalize(stream, d_table) then returns this
    rank's share.  Returns (key_begin, key_count)."""
    k = np.ascontiguousarray(kinds, dtype=np.int32) if kinds else None
    kb, kc = ctypes.c_int64(), ctypes.c_int64()
    L.check(plan.lib.pgpu_plan_combine(plan.handle, comm.handle, ctypes.c_void_p(stream or 0),
                                       ctypes.c_void_p(d_table or 0), mode,
                                       L.ptr(k, ctypes.c_int32) if k is not None else None,
                                       ctypes.c_void_p(d_shard or 0), ctypes.byref(kb), ctypes.byref(kc)))
    return kb.value, kc.value


def combine_result_rows(table, res, comm):
    """pgpu_result_combine_rows: this rank's disjoint share of the merged finalized rows (ROWS mode)."""
    from .executor import _decode_result, _ResultHolder
    out = ctypes.c_void_p()
    L.check(table.lib.pgpu_result_combine_rows(res._holder.r, comm.handle, ctypes.byref(out)))
    return _decode_result(table, res._query, _ResultHolder(table.lib, out))
