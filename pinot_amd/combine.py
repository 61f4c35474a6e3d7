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
