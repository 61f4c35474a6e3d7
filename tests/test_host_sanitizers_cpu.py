"""The library's host parsers and builders under AddressSanitizer + UndefinedBehaviorSanitizer (tools/host_fuzz.cpp).

Every library source is compiled with host-only sanitizer flags into build/host_fuzz (pinot_amd.build.
build_host_fuzz); this test writes a seed corpus with the product's own writers -- raw forward indexes
(FixedByteChunkSVForwardIndexWriter layout, PASS_THROUGH / LZ4 / LZ4_LENGTH_PREFIXED, versions 2 and 3), DataTable V3
responses (DataTableImplV3.toBytes layout), bitmap inverted indexes (BitmapInvertedIndexWriter + portable Roaring,
with and without run containers) and star-tree files (star_tree_index + star_tree_index_map) -- and runs the
harness, which mutates each seed a few thousand times and also drives the inverted-index creator, the star-tree
builder and the filter-statistics replay with random inputs.  Pass = no sanitizer report (the harness exits non-zero
on the first one, and its output names the read).  No GPU is touched.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

import startree_common as SC
from pinot_amd import _lib as L
from pinot_amd import segment_files as SF
from pinot_amd.segment import raw_forward_index_bytes
from pinot_amd.startree import StarTree, star_tree_files
from test_broker_reduce_cpu import _meta, datatable

pytestmark = pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                                reason="hipcc is needed to build the sanitized harness")


@pytest.fixture(scope="module")
def harness():
    from pinot_amd import build
    return build.build_host_fuzz()


def _corpus(oracle, d):
    rng = np.random.default_rng(5)
    k = 0
    for t in (L.INT, L.LONG, L.FLOAT, L.DOUBLE):
        for version, comp in ((2, "PASS_THROUGH"), (3, "LZ4"), (2, "LZ4_LENGTH_PREFIXED")):
            n = int(rng.integers(1, 900))
            if t in (L.INT, L.LONG):
                vals = rng.integers(-50, 50, n)
            else:
                vals = np.round(rng.normal(size=n), 2)
            data = raw_forward_index_bytes(t, vals, version=version, docs_per_chunk=128, compression=comp)
            with open(os.path.join(d, "raw.%d.%d.%d.bin" % (t, n, k)), "wb") as f:
                f.write(data)
            k += 1
    tables = [
        datatable(["column11", "sum(column1)"], ["STRING", "DOUBLE"], [["P", 10.0], ["o", 3.0], ["", 7.0]], _meta(100)),
        datatable(["column11", "sum(column1)"], ["STRING", "DOUBLE"], [["o", 4.0], ["t", 1.0]], _meta(50)),
        datatable(["column17", "count(*)", "avg(column6)", "min(column6)"], ["INT", "LONG", "OBJECT", "DOUBLE"],
                  [[3, 5, (10.0, 4), 1.5], [-2, 1, (2.5, 1), -7.0]], _meta(9)),
        datatable(["column17", "count(*)", "avg(column6)", "min(column6)"], ["INT", "LONG", "OBJECT", "DOUBLE"],
                  [], _meta(0)),
    ]
    for i, b in enumerate(tables):
        with open(os.path.join(d, "dt.%d.bin" % i), "wb") as f:
            f.write(b)
    for i, (card, docs, sort, runs) in enumerate(((7, 5000, False, False), (3, 140000, True, True),
                                                  (40, 70000, False, True), (1, 10, False, False))):
        ids = rng.integers(0, card, docs)
        if sort:
            ids = np.sort(ids)
        with open(os.path.join(d, "inv.%d.%d.%d.bin" % (card, docs, i)), "wb") as f:
            f.write(SF.build_inverted_index(ids, card, run_optimize=runs))
    cols = SC.c4_columns(rng, 3000, cards=(9, 5, 4, 3))
    seg = oracle.make_segment(SC.C4_SCHEMA, cols)
    st = StarTree.build(SC.C4_SCHEMA, seg, SC.C4_SPLIT, SC.C4_PAIRS, max_leaf_records=40)
    bits = {n: seg.columns[n].bits_per_element for n, _ in SC.C4_SCHEMA}
    index, imap, _ = star_tree_files([st], bits)
    with open(os.path.join(d, "st.idx"), "wb") as f:
        f.write(index)
    with open(os.path.join(d, "st.map"), "w") as f:
        f.write(imap)
    with open(os.path.join(d, "st.args"), "w") as f:
        f.write("%d %d\n" % (st.arrays()["num_docs"], len(SC.C4_SCHEMA)))
        for n, _ in SC.C4_SCHEMA:
            f.write("%s %d\n" % (n, bits[n]))


def test_host_parsers_under_sanitizers(oracle, harness, tmp_path):
    _corpus(oracle, str(tmp_path))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", LSAN_OPTIONS="suppressions=" +
               os.path.join(os.path.dirname(__file__), "lsan.supp"))
    res = subprocess.run([harness, str(tmp_path), "1500", "17"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                         text=True, env=env, timeout=600)
    out = res.stdout
    assert res.returncode == 0, out[-6000:]
    assert "runtime error" not in out and "AddressSanitizer" not in out, out[-6000:]
    assert "host_fuzz calls:" in out
