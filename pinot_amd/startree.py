"""Star-tree indexes on the GPU path.

`StarTree.build` runs the host-side builder of libpinotgpu.so (pgpu_startree_build: BaseSingleTreeBuilder /
OnHeapSingleTreeBuilder, seglocal/startree/v2/builder/) over a segment in Pinot's byte format;
`GpuTable.attach_startree` pins one next to its segment (StarTreeIndexContainer at ImmutableSegmentLoader.java:
198-201).  Queries that fit a segment's star-tree (StarTreeUtils.isFitForStarTree, core/startree/StarTreeUtils.java:
151-176) then run on it: K5 traverses the tree (StarTreeFilterOperator) and K6 aggregates the pre-aggregated
documents (StarTreeGroupByExecutor); `QueryContext(..., use_star_tree=False)` is Pinot's debug option
useStarTree=false.
"""
import ctypes

import numpy as np

from . import _lib as L

FN_CODES = {"COUNT": L.AGG_COUNT, "SUM": L.AGG_SUM, "MIN": L.AGG_MIN, "MAX": L.AGG_MAX, "AVG": L.AGG_AVG}


class StarTree:
    """A built star-tree (host memory, owned by libpinotgpu.so until close())."""

    def __init__(self, handle, lib, schema):
        self.handle = handle
        self.lib = lib
        self.schema = schema

    @classmethod
    def build(cls, schema, segment, split_order, pairs, max_leaf_records=10000, skip_star_dims=()):
        """schema: [(name, type)]; segment: SegmentBuffers; split_order: column names; pairs: [(fn, column)] with
        column '*' for COUNT; skip_star_dims: column names of the split order without star nodes."""
        lib = L.load()
        names = [n for n, _ in schema]
        idx = {n: i for i, n in enumerate(names)}
        types = (ctypes.c_int32 * len(names))(*[L.TYPE_NAMES[t] if isinstance(t, str) else int(t) for _, t in schema])
        cols = (L.ColumnBuffers * len(names))()
        keep = []
        for i, name in enumerate(names):
            c = segment.columns[name]
            d = ctypes.create_string_buffer(bytes(c.dict_bytes), max(len(c.dict_bytes), 1))
            f = ctypes.create_string_buffer(bytes(c.fwd_bytes), max(len(c.fwd_bytes), 1))
            keep += [d, f]
            cols[i].cardinality = c.cardinality
            cols[i].bits_per_element = c.bits_per_element
            cols[i].entry_width = c.entry_width
            cols[i].padding_byte = c.padding_byte
            cols[i].fwd_format = c.fwd_format
            cols[i].dict = ctypes.cast(d, ctypes.c_void_p)
            cols[i].dict_len = len(c.dict_bytes)
            cols[i].fwd = ctypes.cast(f, ctypes.c_void_p)
            cols[i].fwd_len = len(c.fwd_bytes)
        desc = L.SegmentDesc(segment.num_docs, len(names), cols)
        split = (ctypes.c_int32 * len(split_order))(*[idx[c] for c in split_order])
        skip = [split_order.index(c) for c in skip_star_dims]
        skip_arr = (ctypes.c_int32 * max(len(skip), 1))(*skip)
        pc = (L.AggC * len(pairs))(*[L.AggC(FN_CODES[f.upper()], -1 if c == "*" else idx[c]) for f, c in pairs])
        h = ctypes.c_void_p()
        L.check(lib.pgpu_startree_build(ctypes.byref(desc), types, split, len(split_order), skip_arr, len(skip), pc,
                                        len(pairs), max_leaf_records, ctypes.byref(h)))
        st = cls(h, lib, schema)
        st.split_order = list(split_order)
        st.pairs = [(f.upper(), c) for f, c in pairs]
        return st

    def close(self):
        if self.handle:
            self.lib.pgpu_startree_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def desc(self):
        d = L.StarTreeDescC()
        L.check(self.lib.pgpu_startree_get_desc(self.handle, ctypes.byref(d)))
        return d

    def num_raw_records(self):
        n = ctypes.c_int32()
        L.check(self.lib.pgpu_startree_num_raw_records(self.handle, ctypes.byref(n)))
        return n.value

    def arrays(self):
        """Copies of the star-tree buffers: nodes [n,7] int32, per-dimension forward-index bytes, per-pair
        metric arrays (f64 or None, i64 or None)."""
        d = self.desc()
        nodes = np.ctypeslib.as_array(ctypes.cast(d.nodes, ctypes.POINTER(ctypes.c_int32)),
                                      shape=(d.num_nodes * 7,)).reshape(d.num_nodes, 7).copy()
        fwd = [ctypes.string_at(d.dim_fwd[k], d.dim_fwd_len[k]) for k in range(d.num_dims)]
        mf, mc = [], []
        for m in range(d.num_metrics):
            mf.append(np.ctypeslib.as_array(d.metric_f64[m], shape=(d.num_docs,)).copy()
                      if bool(d.metric_f64[m]) else None)
            mc.append(np.ctypeslib.as_array(d.metric_i64[m], shape=(d.num_docs,)).copy()
                      if bool(d.metric_i64[m]) else None)
        return {"num_docs": d.num_docs, "nodes": nodes, "dim_fwd": fwd, "metric_f64": mf, "metric_i64": mc,
                "dim_columns": [d.dim_columns[k] for k in range(d.num_dims)],
                "metrics": [(d.metrics[m].fn, d.metrics[m].column) for m in range(d.num_metrics)]}


def attach(table, segment_handle, star_tree):
    """Pins `star_tree` (a StarTree) for a pinned segment of `table` (a GpuTable)."""
    d = star_tree.desc()
    L.check(table.lib.pgpu_attach_startree(table.handle, segment_handle, ctypes.byref(d)))
