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
# AggregationFunctionType.getName() (segspi/AggregationFunctionType.java:29-34): the "<fn>__<col>" metric names
_FN_NAMES = {L.AGG_COUNT: "count", L.AGG_SUM: "sum", L.AGG_MIN: "min", L.AGG_MAX: "max", L.AGG_AVG: "avg"}
STAR_TREE_INDEX_FILE = "star_tree_index"           # StarTreeV2Constants.INDEX_FILE_NAME (:28)
STAR_TREE_INDEX_MAP_FILE = "star_tree_index_map"   # StarTreeV2Constants.INDEX_MAP_FILE_NAME (:29)
STAR_TREE_MAGIC = 0xBADDA55B00DAD00D                # OffHeapStarTree.MAGIC_MARKER (:39)
VAR_BYTE_TARGET_CHUNK = 1024 * 1024                 # SingleValueVarByteRawIndexCreator.TARGET_MAX_CHUNK_SIZE


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

    @classmethod
    def load(cls, schema, bits_per_element, index_bytes, index_map_text, num_docs, star_tree_id=0):
        """Star-tree `star_tree_id` of a segment from Pinot's files (pgpu_startree_load: StarTreeLoaderUtils.
        loadStarTreeV2): `index_bytes` = star_tree_index, `index_map_text` = star_tree_index_map, `num_docs` =
        metadata startree.v2.<id>.total.docs; bits_per_element: {column: segment bitsPerElement}."""
        lib = L.load()
        names = [n for n, _ in schema]
        cn = (ctypes.c_char_p * len(names))(*[n.encode() for n in names])
        bits = (ctypes.c_int32 * len(names))(*[int(bits_per_element.get(n, 0)) for n in names])
        buf = ctypes.create_string_buffer(bytes(index_bytes), max(len(index_bytes), 1))
        text = index_map_text.encode() if isinstance(index_map_text, str) else bytes(index_map_text)
        h = ctypes.c_void_p()
        L.check(lib.pgpu_startree_load(ctypes.cast(buf, ctypes.c_void_p), len(index_bytes), text, len(text),
                                       star_tree_id, num_docs, len(names), cn, bits, ctypes.byref(h)))
        st = cls(h, lib, schema)
        d = st.desc()
        st.split_order = [names[d.dim_columns[k]] for k in range(d.num_dims)]
        st.pairs = [(_FN_NAMES[d.metrics[m].fn].upper(), "*" if d.metrics[m].column < 0 else names[d.metrics[m].column])
                    for m in range(d.num_metrics)]
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


# ------------------------------------------------------------------------------------------- Pinot's file format
def _star_tree_buffer(split_order, nodes):
    """OffHeapStarTree buffer, little-endian (StarTreeBuilderUtils.serializeTree / writeHeader / writeNodes,
    seglocal/startree/StarTreeBuilderUtils.java:91-171): magic, version 1, header size, dimensions (index, name
    length, UTF-8 name), node count, then the 7-int node records in BFS order."""
    import struct
    names = [n.encode() for n in split_order]
    header = 20 + sum(8 + len(n) for n in names) + 4
    out = struct.pack("<qii", STAR_TREE_MAGIC - (1 << 64), 1, header) + struct.pack("<i", len(names))
    for i, n in enumerate(names):
        out += struct.pack("<ii", i, len(n)) + n
    out += struct.pack("<i", len(nodes))
    return out + np.ascontiguousarray(nodes, dtype="<i4").tobytes()


def _var_byte_avg_bytes(sums, counts):
    """AVG's function-column pair as SingleValueVarByteRawIndexCreator writes it (PASS_THROUGH, version 2;
    VarByteChunkSVForwardIndexWriter.putBytes :96-105): per chunk numDocsPerChunk int row offsets, then each row's
    AvgPair.toBytes (double sum, long count, big-endian)."""
    import struct
    n = len(sums)
    per = max(VAR_BYTE_TARGET_CHUNK // (16 + 4), 1)
    num_chunks = (n + per - 1) // per
    header = struct.pack(">iiiiiii", 2, num_chunks, per, 16, n, 0, 28)
    chunks, pos = [], 28 + 4 * num_chunks
    offsets = []
    for c in range(num_chunks):
        rows = range(c * per, min(n, (c + 1) * per))
        hdr = np.zeros(per, dtype=">i4")
        hdr[:len(rows)] = per * 4 + 16 * np.arange(len(rows))
        body = b"".join(struct.pack(">dq", float(sums[i]), int(counts[i])) for i in rows)
        chunk = hdr.tobytes() + body
        offsets.append(pos)
        pos += len(chunk)
        chunks.append(chunk)
    return header + b"".join(struct.pack(">i", o) for o in offsets) + b"".join(chunks)


def star_tree_files(star_trees, bits_per_element, max_leaf_records=10000):
    """Pinot's star-tree files of a segment for built StarTrees: (star_tree_index bytes, star_tree_index_map text,
    metadata.properties lines); bits_per_element: {column: the segment column's bitsPerElement}.  Per tree the combiner's order (StarTreeIndexCombiner.combine, seglocal/startree/v2/
    builder/StarTreeIndexCombiner.java:55-76): the star-tree buffer, each split-order dimension's fixed-bit forward
    index, each function-column pair's raw forward index (COUNT LONG, SUM / MIN / MAX DOUBLE, AVG AvgPair bytes)."""
    from .segment import raw_forward_index_bytes
    blob, lines, meta = [], [], ["startree.v2.count = %d" % len(star_trees)]
    off = 0

    def put(tree_id, column, kind, data):
        nonlocal off
        lines.append("%d.%s.%s.OFFSET = %d" % (tree_id, column, kind, off))
        lines.append("%d.%s.%s.SIZE = %d" % (tree_id, column, kind, len(data)))
        blob.append(data)
        off += len(data)

    for i, st in enumerate(star_trees):
        a = st.arrays()
        nd = a["num_docs"]
        put(i, "null", "STAR_TREE", _star_tree_buffer(st.split_order, a["nodes"]))
        for k, dim in enumerate(st.split_order):
            put(i, dim, "FORWARD_INDEX", a["dim_fwd"][k][:(nd * bits_per_element[dim] + 7) // 8])
        names = []
        for m, (fn, col) in enumerate(st.pairs):
            name = "%s__%s" % (fn.lower(), col)
            names.append(name)
            if fn.upper() == "AVG":
                data = _var_byte_avg_bytes(a["metric_f64"][m], a["metric_i64"][m])
            elif fn.upper() == "COUNT":
                data = raw_forward_index_bytes(L.LONG, a["metric_i64"][m])
            else:
                data = raw_forward_index_bytes(L.DOUBLE, a["metric_f64"][m])
            put(i, name, "FORWARD_INDEX", data)
        p = "startree.v2.%d." % i
        meta += [p + "total.docs = %d" % nd, p + "split.order = " + ",".join(st.split_order),
                 p + "function.column.pairs = " + ",".join(names), p + "max.leaf.records = %d" % max_leaf_records,
                 p + "skip.star.node.creation = "]
    return b"".join(blob), "\n".join(lines) + "\n", meta


def write_star_tree_files(segment_dir, star_trees, bits_per_element, max_leaf_records=10000):
    """Writes star_tree_index + star_tree_index_map into a (v1) segment directory and appends the star-tree keys to
    its metadata.properties (SegmentColumnarIndexCreator + MultipleTreesBuilder's output)."""
    import os
    from .segment_files import METADATA_FILE_NAME
    index, imap, meta = star_tree_files(star_trees, bits_per_element, max_leaf_records)
    with open(os.path.join(segment_dir, STAR_TREE_INDEX_FILE), "wb") as f:
        f.write(index)
    with open(os.path.join(segment_dir, STAR_TREE_INDEX_MAP_FILE), "w") as f:
        f.write(imap)
    with open(os.path.join(segment_dir, METADATA_FILE_NAME), "a") as f:
        f.write("\n".join(meta) + "\n")


def load_star_trees(segment_dir, schema, bits_per_element):
    """The star-trees of a v1 / v3 segment directory (StarTreeIndexContainer: metadata startree.v2.count, then
    star_tree_index + star_tree_index_map, copied as-is into v3 by SegmentV1V2ToV3FormatConverter.copyStarTreeV2)."""
    import os
    from .segment_files import METADATA_FILE_NAME, _parse_properties
    with open(os.path.join(segment_dir, METADATA_FILE_NAME)) as f:
        props = _parse_properties(f.read())
    n = int(props.get("startree.v2.count", "0"))
    if n == 0:
        return []
    with open(os.path.join(segment_dir, STAR_TREE_INDEX_FILE), "rb") as f:
        index = f.read()
    with open(os.path.join(segment_dir, STAR_TREE_INDEX_MAP_FILE)) as f:
        imap = f.read()
    return [StarTree.load(schema, bits_per_element, index, imap, int(props["startree.v2.%d.total.docs" % i]), i)
            for i in range(n)]
