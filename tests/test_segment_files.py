"""Pinot segment files (v1 directory, v3 columns.psf + index_map): writer, converter, reader.

Pinned by real Pinot-written segments (padding{Old,Null,Percent}.tar.gz, tests/golden/padding_segments.json): the
writer re-creates their dictionary and forward-index bytes exactly from the decoded values, and by the oracle's
own segment creator on seeded synthetic columns.
"""
import json
import os
import struct

import numpy as np
import pytest

from pinot_amd import _lib as L
from pinot_amd.segment import load_v1_segment_dir
from pinot_amd.segment_files import (MAGIC_MARKER, convert_v1_to_v3, load_segment_dir, num_bits_per_value,
                                     pack_msb_first, write_v1_segment_dir)

HERE = os.path.dirname(os.path.abspath(__file__))


def _padding():
    with open(os.path.join(HERE, "golden", "padding_segments.json")) as f:
        return json.load(f)


def _unpack(fwd, bits, n):
    b = np.unpackbits(np.frombuffer(fwd, dtype=np.uint8))[: n * bits].reshape(n, bits).astype(np.int64)
    return (b << np.arange(bits - 1, -1, -1)).sum(axis=1)


def _decode_column(c, n, pad):
    ids = _unpack(bytes.fromhex(c["fwd_hex"]), c["bitsPerElement"], n)
    d = bytes.fromhex(c["dict_hex"])
    typ = c["dataType"]
    if typ == "STRING":
        w = c["lengthOfEachEntry"]
        entries = [d[i * w:(i + 1) * w].rstrip(bytes([pad])).decode() for i in range(c["cardinality"])]
    else:
        entries = list(np.frombuffer(d, dtype={"INT": ">i4", "LONG": ">i8", "FLOAT": ">f4", "DOUBLE": ">f8"}[typ]))
    return [entries[i] for i in ids]


@pytest.mark.parametrize("name", ["paddingOld", "paddingNull", "paddingPercent"])
def test_writer_reproduces_pinot_written_segment(tmp_path, name):
    seg = _padding()[name]
    pad = 0 if "u0000" in seg["paddingCharacter"] else ord(seg["paddingCharacter"].replace("\\", "")[0])
    n = seg["totalDocs"]
    schema = [(col, c["dataType"]) for col, c in sorted(seg["columns"].items())]
    values = {col: _decode_column(c, n, pad) for col, c in seg["columns"].items()}
    out = write_v1_segment_dir(str(tmp_path / name), schema, values, pad_byte=pad)
    for col, c in seg["columns"].items():
        w = out.columns[col]
        assert (w.cardinality, w.bits_per_element) == (c["cardinality"], c["bitsPerElement"]), col
        assert w.dict_bytes.hex() == c["dict_hex"], col
        assert w.fwd_bytes.hex() == c["fwd_hex"], col
    back = load_v1_segment_dir(str(tmp_path / name))
    assert back.num_docs == n
    for col in seg["columns"]:
        assert back.columns[col] == out.columns[col], col


def test_num_bits_per_value():
    """PinotDataBitSet.getNumBitsPerValue (:59-70)."""
    assert [num_bits_per_value(m) for m in (0, 1, 2, 3, 4, 255, 256, 99999, 2 ** 31 - 1)] == \
        [1, 1, 2, 2, 3, 8, 9, 17, 31]


@pytest.mark.parametrize("bits", [1, 3, 9, 17, 31])
def test_pack_msb_first_matches_oracle(oracle, bits):
    rng = np.random.default_rng(bits)
    n = 1000
    ids = rng.integers(0, 2 ** bits, size=n)
    buf = pack_msb_first(ids, bits)
    assert len(buf) == (n * bits + 7) // 8
    np.testing.assert_array_equal(_unpack(buf, bits, n), ids)


def test_writer_matches_oracle_creator(oracle, tmp_path):
    rng = np.random.default_rng(5)
    n = 5000
    schema = [("i", "INT"), ("l", "LONG"), ("f", "FLOAT"), ("d", "DOUBLE"), ("s", "STRING")]
    vals = {"i": rng.integers(-50, 50, n).tolist(), "l": (rng.integers(0, 3000, n) * 10 ** 10).tolist(),
            "f": rng.integers(0, 200, n).astype(np.float32).tolist(),
            "d": (rng.random(n) * 1e6).round(3).tolist(),
            "s": ["k%d" % v for v in rng.integers(0, 300, n)]}
    seg = write_v1_segment_dir(str(tmp_path / "s"), schema, vals)
    ref = oracle.make_segment(schema, vals)
    for name, _ in schema:
        a, b = seg.columns[name], ref.columns[name]
        assert (a.cardinality, a.bits_per_element, a.entry_width) == (b.cardinality, b.bits_per_element,
                                                                       b.entry_width), name
        assert a.dict_bytes == bytes(b.dict_bytes), name
        assert a.fwd_bytes == bytes(b.fwd_bytes), name


def _synthetic(tmp_path, n=3000, seed=1):
    rng = np.random.default_rng(seed)
    schema = [("day", "INT"), ("acct", "LONG"), ("clicks", "INT"), ("name", "STRING")]
    vals = {"day": np.sort(rng.integers(17000, 17030, n)).tolist(), "acct": rng.integers(0, 500, n).tolist(),
            "clicks": rng.integers(0, 1000, n).tolist(), "name": ["n%d" % v for v in rng.integers(0, 7, n)]}
    path = str(tmp_path / ("seg%d" % seed))
    seg = write_v1_segment_dir(path, schema, vals, sorted_columns=("day",))
    return path, schema, vals, seg


def test_sorted_column_pairs(tmp_path):
    path, schema, vals, seg = _synthetic(tmp_path)
    c = seg.columns["day"]
    assert c.is_sorted and c.fwd_format == L.FWD_SORTED_PAIRS
    assert os.path.exists(os.path.join(path, "day.sv.sorted.fwd"))
    pairs = np.frombuffer(c.fwd_bytes, dtype=">i4").reshape(-1, 2)
    days = np.asarray(vals["day"])
    uniq = np.unique(days)
    for i, v in enumerate(uniq):
        docs = np.nonzero(days == v)[0]
        assert (pairs[i, 0], pairs[i, 1]) == (docs[0], docs[-1])
    with pytest.raises(ValueError):
        write_v1_segment_dir(str(tmp_path / "bad"), [("x", "INT")], {"x": [3, 1, 2]}, sorted_columns=("x",))


def test_v3_round_trip(tmp_path):
    path, schema, vals, seg = _synthetic(tmp_path)
    v3 = convert_v1_to_v3(path)
    assert sorted(os.listdir(v3)) == ["columns.psf", "index_map", "metadata.properties"]
    psf = open(os.path.join(v3, "columns.psf"), "rb").read()
    lines = open(os.path.join(v3, "index_map")).read().split("\n")
    starts = [int(ln.split(" = ")[1]) for ln in lines if ".startOffset = " in ln]
    assert len(starts) == 2 * len(schema)
    for s in starts:
        assert struct.unpack(">Q", psf[s:s + 8])[0] == MAGIC_MARKER
    back = load_segment_dir(path)
    assert back.num_docs == seg.num_docs
    for name, _ in schema:
        assert back.columns[name] == seg.columns[name], name
    assert load_segment_dir(v3).columns == back.columns
    meta = open(os.path.join(v3, "metadata.properties")).read()
    assert "segment.index.version = v3" in meta


def test_v3_column_names_with_dots(tmp_path):
    """SingleFileIndexDirectory.loadMap parses keys from the right: column names may contain '.'."""
    path = str(tmp_path / "dots")
    seg = write_v1_segment_dir(path, [("a.b.c", "INT")], {"a.b.c": [5, 1, 5, 2]})
    convert_v1_to_v3(path)
    assert load_segment_dir(path).columns["a.b.c"] == seg.columns["a.b.c"]


def test_v3_corrupt_marker_and_overrun(tmp_path):
    path, schema, vals, seg = _synthetic(tmp_path, n=100, seed=2)
    v3 = convert_v1_to_v3(path)
    psf_path = os.path.join(v3, "columns.psf")
    raw = bytearray(open(psf_path, "rb").read())
    raw[0] ^= 0xFF
    open(psf_path, "wb").write(bytes(raw))
    with pytest.raises(ValueError, match="magic marker"):
        load_segment_dir(path)
    raw[0] ^= 0xFF
    open(psf_path, "wb").write(bytes(raw[:-4]))
    with pytest.raises(ValueError, match="overruns"):
        load_segment_dir(path)


# ------------------------------------------------------------------------------------------- inverted index
def _decode_roaring(b):
    """Independent portable-format Roaring reader (the spec the writer and the C++ attach parser follow)."""
    cookie = struct.unpack_from("<I", b, 0)[0]
    if cookie & 0xFFFF == 12347:
        size = (cookie >> 16) + 1
        runbits = b[4:4 + (size + 7) // 8]
        pos = 4 + (size + 7) // 8
        offsets = size >= 4
    else:
        assert cookie == 12346
        size = struct.unpack_from("<I", b, 4)[0]
        runbits, pos, offsets = None, 8, True
    desc = [struct.unpack_from("<HH", b, pos + 4 * i) for i in range(size)]
    pos += 4 * size + (4 * size if offsets else 0)
    out = []
    for i, (key, c1) in enumerate(desc):
        card = c1 + 1
        if runbits is not None and (runbits[i >> 3] >> (i & 7)) & 1:
            nruns = struct.unpack_from("<H", b, pos)[0]
            runs = np.frombuffer(b, dtype="<u2", count=2 * nruns, offset=pos + 2).reshape(-1, 2)
            vals = np.concatenate([np.arange(int(s), int(s) + int(l) + 1) for s, l in runs])
            pos += 2 + 4 * nruns
        elif card <= 4096:
            vals = np.frombuffer(b, dtype="<u2", count=card, offset=pos).astype(np.int64)
            pos += 2 * card
        else:
            words = np.frombuffer(b, dtype="<u4", count=2048, offset=pos)
            vals = np.nonzero(np.unpackbits(words.view(np.uint8), bitorder="little"))[0]
            pos += 8192
        assert len(vals) == card
        out.append((key << 16) + np.asarray(vals, dtype=np.int64))
    assert pos == len(b)
    return np.concatenate(out) if out else np.zeros(0, np.int64)


@pytest.mark.parametrize("run_optimize", [False, True])
def test_roaring_serialisation_round_trip(run_optimize):
    from pinot_amd.segment_files import serialize_roaring
    rng = np.random.default_rng(3)
    cases = [np.array([0]), np.arange(70000), np.sort(rng.choice(300000, 5000, replace=False)),
             np.concatenate([np.arange(100, 9000), np.arange(65536 * 3 + 5, 65536 * 3 + 40)]),
             np.sort(rng.choice(200000, 150000, replace=False)), np.array([], dtype=np.int64)]
    for docs in cases:
        b = serialize_roaring(docs, run_optimize)
        np.testing.assert_array_equal(_decode_roaring(b), docs)


def test_inverted_index_files(tmp_path):
    from pinot_amd.segment_files import build_inverted_index
    rng = np.random.default_rng(4)
    n = 140000
    vals = {"a": rng.integers(0, 9, n).tolist(), "b": rng.integers(0, 3000, n).tolist()}
    path = str(tmp_path / "inv")
    seg = write_v1_segment_dir(path, [("a", "INT"), ("b", "INT")], vals, inverted_columns=("a", "b"),
                               run_optimize=True)
    for col in ("a", "b"):
        c = seg.columns[col]
        assert os.path.exists(os.path.join(path, col + ".bitmap.inv"))
        offs = np.frombuffer(c.inv_bytes[:4 * (c.cardinality + 1)], dtype=">i4")
        assert offs[0] == 4 * (c.cardinality + 1) and offs[-1] == len(c.inv_bytes)
        uniq = np.unique(vals[col])
        for d in (0, c.cardinality // 2, c.cardinality - 1):
            docs = _decode_roaring(c.inv_bytes[offs[d]:offs[d + 1]])
            np.testing.assert_array_equal(docs, np.nonzero(np.asarray(vals[col]) == uniq[d])[0])
    assert load_v1_segment_dir(path).columns == seg.columns
    convert_v1_to_v3(path)
    assert "a.inverted_index.startOffset" in open(os.path.join(path, "v3", "index_map")).read()
    assert load_segment_dir(path).columns == seg.columns
    assert build_inverted_index([], 0) == struct.pack(">i", 4)


def test_native_inverted_index_builder_matches_writer():
    """pgpu_build_inverted_index (host code of the library) writes the same bytes as the Python creator."""
    from pinot_amd.segment_files import build_column, build_inverted_index, build_inverted_index_native
    rng = np.random.default_rng(6)
    for n, card in ((1, 1), (5000, 3), (140000, 9), (70001, 2000)):
        c = build_column(L.INT, rng.integers(0, card, n).tolist(), is_sorted=False)
        ids = _unpack(c.fwd_bytes, c.bits_per_element, n)
        native = build_inverted_index_native(c.fwd_bytes, c.bits_per_element, n, c.cardinality)
        assert native == build_inverted_index(ids, c.cardinality)


def test_inverted_index_host_check():
    """pgpu_inverted_index_check: the attach-time validation of a bitmap.inv file, on the host (no device)."""
    import ctypes
    from pinot_amd.segment_files import build_inverted_index
    lib = L.load()
    rng = np.random.default_rng(8)

    def check(b, card, n):
        total = ctypes.c_int64(-1)
        buf = ctypes.create_string_buffer(bytes(b), max(len(b), 1))
        rc = lib.pgpu_inverted_index_check(ctypes.cast(buf, ctypes.c_void_p), len(b), card, n, ctypes.byref(total))
        return rc, total.value

    for n, card, runs in ((5000, 7, False), (140000, 3, True), (1, 1, False)):
        ids = np.sort(rng.integers(0, card, n)) if runs else rng.integers(0, card, n)
        b = build_inverted_index(ids, card, run_optimize=runs)
        assert check(b, card, n) == (0, n)
        assert check(b, card, n - 1)[0] == L.PGPU_ERR_INVALID_ARGUMENT or n == 1  # a docId past numDocs
        assert check(b[:-1], card, n)[0] == L.PGPU_ERR_INVALID_ARGUMENT           # truncated last bitmap
        assert check(b[:4 * card], card, n)[0] == L.PGPU_ERR_INVALID_ARGUMENT     # shorter than its offset header
        bad = bytearray(b)
        off = struct.unpack(">i", bytes(b[:4]))[0]
        bad[off:off + 4] = struct.pack("<I", 99)  # not a Roaring cookie
        assert check(bytes(bad), card, n)[0] == L.PGPU_ERR_INVALID_ARGUMENT
