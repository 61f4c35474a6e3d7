"""Pinot's own star-tree files (no device): the writer in pinot_amd/startree.py produces star_tree_index +
star_tree_index_map as StarTreeIndexCombiner / StarTreeBuilderUtils.serializeTree lay them out, and the product's
loader (pgpu_startree_load: StarTreeLoaderUtils.loadStarTreeV2 + OffHeapStarTree + the chunk forward-index readers)
reads back exactly the tree the builder made.  Malformed files are rejected with the reference's messages.  The
layout is pinned by the reference's source (no serialised star-tree ships with it): magic / version / header-length
/ buffer-size checks of OffHeapStarTree.java:45-80, chunk headers of BaseChunkSVForwardIndexReader.java:56-100."""
import os
import struct

import numpy as np
import pytest

import startree_common as SC
from pinot_amd import _lib as L
from pinot_amd import segment_files as SF
from pinot_amd.startree import StarTree, load_star_trees, star_tree_files, write_star_tree_files


@pytest.fixture(scope="module")
def built(oracle):
    rng = np.random.default_rng(7)
    cols = SC.c4_columns(rng, 40000, cards=(25, 9, 6, 4))
    seg = oracle.make_segment(SC.C4_SCHEMA, cols)
    st = StarTree.build(SC.C4_SCHEMA, seg, SC.C4_SPLIT, SC.C4_PAIRS, max_leaf_records=300)
    bits = {n: seg.columns[n].bits_per_element for n, _ in SC.C4_SCHEMA}
    return seg, st, bits, cols


def _same(a, b):
    assert a["num_docs"] == b["num_docs"]
    assert np.array_equal(a["nodes"], b["nodes"])
    assert a["dim_columns"] == b["dim_columns"]
    assert a["metrics"] == b["metrics"]
    for x, y in zip(a["dim_fwd"], b["dim_fwd"]):
        assert x == y
    for x, y in zip(a["metric_f64"] + a["metric_i64"], b["metric_f64"] + b["metric_i64"]):
        assert (x is None) == (y is None)
        if x is not None:
            assert np.array_equal(x, y)


def test_round_trip(built):
    seg, st, bits, _ = built
    index, imap, meta = star_tree_files([st], bits, 300)
    a = st.arrays()
    assert index[:8] == struct.pack("<Q", 0xBADDA55B00DAD00D)
    assert "0.null.STAR_TREE.OFFSET = 0" in imap and "0.sum__m.FORWARD_INDEX.SIZE" in imap
    assert "startree.v2.0.function.column.pairs = sum__m,count__*,min__m,max__m,avg__m,sum__md" in meta
    back = StarTree.load(SC.C4_SCHEMA, bits, index, imap, a["num_docs"])
    assert back.split_order == SC.C4_SPLIT
    assert back.pairs == [(f, c) for f, c in SC.C4_PAIRS]
    assert back.num_raw_records() == -1
    _same(a, back.arrays())


def test_two_trees_and_segment_dir(built, tmp_path):
    seg, st, bits, cols = built
    st2 = StarTree.build(SC.C4_SCHEMA, seg, ["d3", "d1"], [("COUNT", "*"), ("MAX", "md")], max_leaf_records=1000)
    path = str(tmp_path / "seg")
    SF.write_v1_segment_dir(path, SC.C4_SCHEMA, cols)
    write_star_tree_files(path, [st, st2], bits)
    v3 = SF.convert_v1_to_v3(path)
    for d in (path, v3):
        trees = load_star_trees(d, SC.C4_SCHEMA, bits)
        assert len(trees) == 2
        _same(st.arrays(), trees[0].arrays())
        _same(st2.arrays(), trees[1].arrays())
        assert trees[1].split_order == ["d3", "d1"]


def test_unknown_pairs_skipped_and_column_names(built):
    seg, st, bits, _ = built
    index, imap, _ = star_tree_files([st], bits)
    n = st.arrays()["num_docs"]
    # a pair of a function outside the GPU path (e.g. distinctCountHLL) is skipped, the rest still loads
    extra = b"\x00" * 64
    imap2 = imap + "0.distinctCountHLL__d1.FORWARD_INDEX.OFFSET = %d\n0.distinctCountHLL__d1.FORWARD_INDEX.SIZE = 64\n" \
        % len(index)
    back = StarTree.load(SC.C4_SCHEMA, bits, index + extra, imap2, n)
    assert len(back.pairs) == len(SC.C4_PAIRS)
    # a dimension name that is not a table column
    schema = [("x" if c == "d2" else c, t) for c, t in SC.C4_SCHEMA]
    with pytest.raises(L.PinotGpuError) as e:
        StarTree.load(schema, {("x" if k == "d2" else k): v for k, v in bits.items()}, index, imap, n)
    assert "d2" in e.value.message


def test_malformed(built):
    seg, st, bits, _ = built
    index, imap, _ = star_tree_files([st], bits)
    n = st.arrays()["num_docs"]
    bad = bytearray(index)
    bad[0] ^= 1
    with pytest.raises(L.PinotGpuError) as e:
        StarTree.load(SC.C4_SCHEMA, bits, bytes(bad), imap, n)
    assert "Invalid magic marker" in e.value.message
    bad = bytearray(index)
    bad[8] = 2
    with pytest.raises(L.PinotGpuError) as e:
        StarTree.load(SC.C4_SCHEMA, bits, bytes(bad), imap, n)
    assert "Invalid version" in e.value.message
    size = int([ln for ln in imap.splitlines() if ln.startswith("0.null.STAR_TREE.SIZE")][0].split("=")[1])
    short = imap.replace("0.null.STAR_TREE.SIZE = %d" % size, "0.null.STAR_TREE.SIZE = %d" % (size - 28))
    with pytest.raises(L.PinotGpuError) as e:
        StarTree.load(SC.C4_SCHEMA, bits, index, short, n)
    assert "buffer size mis-match" in e.value.message
    with pytest.raises(L.PinotGpuError):  # more documents than the forward indexes hold
        StarTree.load(SC.C4_SCHEMA, bits, index, imap, n + 100000)
    with pytest.raises(L.PinotGpuError):  # index map pointing past the file
        StarTree.load(SC.C4_SCHEMA, bits, index[:len(index) // 2], imap, n)
    with pytest.raises(L.PinotGpuError):
        StarTree.load(SC.C4_SCHEMA, bits, index, "garbage line without separator\n", n)
    # compressed metric chunks are declined (PASS_THROUGH only)
    line = [ln for ln in imap.splitlines() if ln.startswith("0.sum__m.FORWARD_INDEX.OFFSET")][0]
    off = int(line.split("=")[1])
    bad = bytearray(index)
    bad[off + 20:off + 24] = struct.pack(">i", 2)
    with pytest.raises(L.UnsupportedQueryError):
        StarTree.load(SC.C4_SCHEMA, bits, bytes(bad), imap, n)


def test_index_map_offsets_near_int64_max(built):
    """Offsets / sizes read from the index map text up to LLONG_MAX: the bounds check must not overflow (an
    OFFSET of 2^63-1 with SIZE 1 once passed as in-file and read far outside the buffer)."""
    seg, st, bits, _ = built
    index, imap, _ = star_tree_files([st], bits)
    n = st.arrays()["num_docs"]
    big = 2 ** 63 - 1
    lines = []
    for ln in imap.splitlines():
        if ln.startswith("0.null.STAR_TREE.OFFSET"):
            ln = "0.null.STAR_TREE.OFFSET = %d" % big
        elif ln.startswith("0.null.STAR_TREE.SIZE"):
            ln = "0.null.STAR_TREE.SIZE = 1"
        lines.append(ln)
    with pytest.raises(L.PinotGpuError):
        StarTree.load(SC.C4_SCHEMA, bits, index, "\n".join(lines) + "\n", n)
    # a metric chunk whose SIZE pushes offset + size past 2^63
    lines = []
    for ln in imap.splitlines():
        if ln.startswith("0.sum__m.FORWARD_INDEX.SIZE"):
            ln = "0.sum__m.FORWARD_INDEX.SIZE = %d" % big
        lines.append(ln)
    with pytest.raises(L.PinotGpuError):
        StarTree.load(SC.C4_SCHEMA, bits, index, "\n".join(lines) + "\n", n)
