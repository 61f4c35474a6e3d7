"""Cross-GPU combine: the dense group tables of all ranks are merged with collectives (RCCL over xGMI on the
node; gloo in the CPU tests) instead of GroupByCombineOperator's ConcurrentHashMap merge
(core/operator/combine/GroupByCombineOperator.java:113-160).

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


def allreduce_group_table(table, slot_kinds, group=None):
    """In-place all-reduce of a [num_slots, num_keys] int64 tensor holding a plan's dense group table."""
    assert table.dtype == torch.int64 and table.dim() == 2 and table.shape[0] == len(slot_kinds)
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
