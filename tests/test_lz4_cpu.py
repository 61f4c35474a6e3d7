"""LZ4 raw chunks and raw-value predicates, CPU side.

Two independent LZ4 block decoders -- the product's (rt_dict.cpp, reached through pgpu_raw_forward_index_values, the
decoder pgpu_pin_segment runs) and the oracle's (or_lz4_decompress / or_raw_decode) -- are checked against:
  - the reference's own vector: TestCompression.java round-trips "testing123" through LZ4 and LZ4_LENGTH_PREFIXED; a
    10-byte input is one literal-only sequence, token 0xA0 (LZ4 block format, lz4-java 1.7 -- absent from
    /root/reference, so the format is pinned by its published spec);
  - hand-built blocks exercising the format's corners (extended literal / match lengths, overlapping matches) and
    malformed ones (zero offset, offset before the output, truncation, output overflow) that must be rejected;
  - this repo's writer (pinot_amd.lz4 + segment.raw_forward_index_bytes) in FixedByteChunkSVForwardIndexTest's shape:
    10 009 values, 5 003 docs per chunk (a partial last chunk), versions 2 / 3, every compression it writes.
The oracle's raw-value predicate evaluators are pinned by NoDictionaryCompressionQueriesTest's LZ4 filter case
(1000 rows, every 10th = 1001, `LZ4_INTEGER > 1000`)."""
import ctypes
import struct

import numpy as np
import pytest

from pinot_amd import _lib as L
from pinot_amd import lz4
from pinot_amd.query import parse_query
from pinot_amd.segment import SegmentBuffers, build_raw_column, raw_forward_index_bytes

NUM_VALUES, PER_CHUNK = 10009, 5003


@pytest.fixture(scope="module")
def olib(oracle):
    lib = oracle.lib()
    lib.or_lz4_decompress.restype = ctypes.c_int64
    lib.or_lz4_decompress.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]
    lib.or_raw_decode.restype = ctypes.c_int
    lib.or_raw_decode.argtypes = [ctypes.POINTER(oracle.OrColumn), ctypes.c_char_p, ctypes.c_int64, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p]
    return lib


def _odecode(olib, block, cap):
    out = ctypes.create_string_buffer(max(cap, 1))
    n = olib.or_lz4_decompress(block, len(block), out, cap)
    return None if n < 0 else out.raw[:n]


def _product_values(raw, t, n):
    lib = L.load()
    i64 = np.zeros(max(n, 1), dtype=np.int64)
    f64 = np.zeros(max(n, 1), dtype=np.float64)
    rc = lib.pgpu_raw_forward_index_values(raw, len(raw), t, n, L.ptr(i64, ctypes.c_int64), L.ptr(f64, ctypes.c_double))
    return rc, i64[:n], f64[:n]


def _oracle_values(oracle, olib, raw, t, n):
    col = oracle.OrColumn(t, 0, 0, 4 if t in (L.INT, L.FLOAT) else 8, 0, 0, 0, None, None, 1, len(raw))
    i64 = np.zeros(max(n, 1), dtype=np.int64)
    f64 = np.zeros(max(n, 1), dtype=np.float64)
    rc = olib.or_raw_decode(ctypes.byref(col), raw, len(raw), n, i64.ctypes.data, f64.ctypes.data)
    return rc, i64[:n], f64[:n]


def test_reference_vector_testing123(olib):
    data = b"testing123"
    block = lz4.compress_block(data)
    assert block == b"\xa0" + data  # one literal-only sequence
    assert lz4.compress_with_length(data) == struct.pack("<i", 10) + block
    assert _odecode(olib, block, 10) == data


def _ints_column(block_bytes, n_values, codec=3):
    """A one-chunk INT raw forward index around a given LZ4 block (version 2)."""
    hdr = struct.pack(">iiiiiii", 2, 1, n_values, 4, n_values, codec, 28) + struct.pack(">i", 32)
    return hdr + block_bytes


def test_format_corners_both_decoders(oracle, olib):
    # overlapping match (run-length): 'a' + match(offset 1, length 14) + 5 literals = 20 x 'a'
    rle = bytes([0x1A]) + b"a" + b"\x01\x00" + bytes([0x50]) + b"aaaaa"
    assert _odecode(olib, rle, 64) == b"a" * 20
    # extended literal length (15 + 255 + 10 = 280 literals), then a long match (4 + 15 + 255 + 5 = 279 bytes)
    lits = bytes(range(256)) + bytes(range(24))
    blk = bytes([0xFF]) + bytes([255, 10]) + lits + b"\x00\x01" + bytes([255, 5]) + bytes([0x50]) + b"zzzzz"
    want = lits + (lits[24:] * 2)[:279] + b"zzzzz"  # offset 256: the copy repeats out[24:280]
    assert _odecode(olib, blk, 4096) == want
    for block, expect in ((rle, b"a" * 20), (blk, want)):
        n = len(expect) // 4  # a whole number of INT values: the chunk holds exactly the decoded bytes
        col = _ints_column(block, n)
        rc, i64, _ = _product_values(col, L.INT, n)
        assert rc == 0
        assert i64.tolist() == list(struct.unpack(">%di" % n, expect[:4 * n]))
    bad = [
        bytes([0x14]) + b"a" + b"\x00\x00",         # offset 0
        bytes([0x14]) + b"a" + b"\x05\x00" + bytes([0x50]) + b"aaaaa",  # offset before the start of the output
        bytes([0xF0]) + bytes([255]),                 # literal length runs off the input
        bytes([0x50]) + b"abc",                       # literals truncated
        bytes([0x14]) + b"a" + b"\x01",               # offset truncated
    ]
    for b in bad:
        assert _odecode(olib, b, 64) is None
        rc, _, _ = _product_values(_ints_column(b, 4), L.INT, 4)
        assert rc == L.PGPU_ERR_INVALID_ARGUMENT
    assert _odecode(olib, rle, 19) is None  # output overflow


def _values(t, rng, n, repetitive):
    if t == L.INT:
        v = rng.integers(0, 50, n) if repetitive else rng.integers(-2 ** 31, 2 ** 31, n)
    elif t == L.LONG:
        v = rng.integers(0, 7, n) * 10 ** 12 if repetitive else rng.integers(-2 ** 63, 2 ** 63 - 1, n, dtype=np.int64)
    elif t == L.FLOAT:
        v = np.float32(rng.integers(0, 9, n) * 0.5 if repetitive else rng.normal(0, 1e6, n)).astype(np.float64)
    else:
        v = (rng.integers(0, 9, n) * 0.25) if repetitive else rng.normal(0, 1e12, n)
    return v.tolist()


@pytest.mark.parametrize("compression", ["LZ4", "LZ4_LENGTH_PREFIXED", "PASS_THROUGH"])
@pytest.mark.parametrize("version", [2, 3])
@pytest.mark.parametrize("type_name", ["INT", "LONG", "FLOAT", "DOUBLE"])
def test_chunk_round_trip_product_and_oracle(oracle, olib, compression, version, type_name):
    t = L.TYPE_NAMES[type_name]
    rng = np.random.default_rng(hash((compression, version, type_name)) & 0xFFFF)
    vals = _values(t, rng, NUM_VALUES, repetitive=(version == 2))
    raw = raw_forward_index_bytes(t, vals, version, PER_CHUNK, compression)
    ver, nchunks, per, size, total, comp, start = struct.unpack(">iiiiiii", raw[:28])
    assert (ver, nchunks, per, total, start) == (version, 3, PER_CHUNK, NUM_VALUES, 28)
    assert comp == {"PASS_THROUGH": 0, "LZ4": 3, "LZ4_LENGTH_PREFIXED": 4}[compression]
    if compression != "PASS_THROUGH" and version == 2:  # repetitive values compress
        assert len(raw) < 28 + 3 * 4 + NUM_VALUES * size
    for rc, i64, f64 in (_product_values(raw, t, NUM_VALUES), _oracle_values(oracle, olib, raw, t, NUM_VALUES)):
        assert rc == 0
        assert f64.tolist() == [float(v) for v in vals]
        if t in (L.INT, L.LONG):
            assert i64.tolist() == [int(v) for v in vals]


def test_unsupported_codecs_and_corrupt_chunks(oracle, olib):
    vals = list(range(100))
    raw = bytearray(raw_forward_index_bytes(L.INT, vals, 2, 40, "LZ4"))
    for codec in (1, 2):  # SNAPPY, ZSTANDARD
        bad = bytearray(raw)
        bad[20:24] = struct.pack(">i", codec)
        assert _product_values(bytes(bad), L.INT, 100)[0] == L.PGPU_ERR_UNSUPPORTED
        assert _oracle_values(oracle, olib, bytes(bad), L.INT, 100)[0] == -2
    bad = bytearray(raw)
    bad[28:32] = struct.pack(">i", len(raw) + 5)  # chunk 0 starts past the end
    assert _product_values(bytes(bad), L.INT, 100)[0] == L.PGPU_ERR_INVALID_ARGUMENT
    assert _oracle_values(oracle, olib, bytes(bad), L.INT, 100)[0] == -1
    short = bytes(raw[:-3])  # the last chunk's block cut
    assert _product_values(short, L.INT, 100)[0] == L.PGPU_ERR_INVALID_ARGUMENT
    assert _oracle_values(oracle, olib, short, L.INT, 100)[0] == -1


def _nodict_rows(n=1000, seed=11):
    """NoDictionaryCompressionQueriesTest.createTestData: every 10th row 1001, the rest uniform in [0, 1000)."""
    rng = np.random.default_rng(seed)
    ints = [1001 if i % 10 == 0 else int(rng.integers(0, n)) for i in range(n)]
    longs = [1001 if i % 10 == 0 else int(rng.integers(0, n)) for i in range(n)]
    return ints, longs


def test_oracle_raw_filter_reference_case(oracle):
    """LZ4_INTEGER > 1000 selects exactly the rows holding 1001 (testLZ4IntegerFilterQueriesWithCompressionCodec);
    the same for PASS_THROUGH, and every predicate form agrees with numpy on the values."""
    ints, longs = _nodict_rows()
    schema = [("LZ4_INTEGER", "INT"), ("LZ4_LONG", "LONG"), ("PASS_THROUGH_INTEGER", "INT")]
    seg = SegmentBuffers(len(ints), {"LZ4_INTEGER": build_raw_column("INT", ints, compression="LZ4"),
                                     "LZ4_LONG": build_raw_column("LONG", longs, compression="LZ4"),
                                     "PASS_THROUGH_INTEGER": build_raw_column("INT", ints)})
    for col in ("LZ4_INTEGER", "PASS_THROUGH_INTEGER"):
        o = oracle.run_groupby(schema, [seg], parse_query("SELECT COUNT(*), SUM(LZ4_LONG) FROM t WHERE %s > 1000" % col))
        (vals,) = o.groups.values()
        assert vals[0] == 100 == sum(1 for v in ints if v > 1000)
        assert vals[1] == float(sum(lv for v, lv in zip(ints, longs) if v > 1000))
        assert o.stats[1] == len(ints)  # a raw scan counts every entry
    a = np.array(ints)
    for where, mask in [("LZ4_INTEGER = 1001", a == 1001), ("LZ4_INTEGER <> 1001", a != 1001),
                        ("LZ4_INTEGER IN (3, 5, 1001)", np.isin(a, [3, 5, 1001])),
                        ("LZ4_INTEGER NOT IN (3, 5, 1001)", ~np.isin(a, [3, 5, 1001])),
                        ("LZ4_INTEGER BETWEEN 10 AND 20", (a >= 10) & (a <= 20)),
                        ("LZ4_INTEGER < 10", a < 10), ("LZ4_INTEGER >= 999", a >= 999)]:
        o = oracle.run_groupby(schema, [seg], parse_query("SELECT COUNT(*) FROM t WHERE " + where))
        got = list(o.groups.values())[0][0] if o.groups else 0
        assert got == int(mask.sum()), where


@pytest.mark.parametrize("per_chunk", [2**31 - 1, 1 << 28])
def test_corrupted_chunk_header_is_rejected_before_allocating(per_chunk):
    """A header claiming an absurd numDocsPerChunk (and totalDocs) must fail as INVALID_ARGUMENT, not allocate a
    chunk buffer of per_chunk x entry bytes (INT32_MAX docs per chunk asked for ~17 GB)."""
    vals = np.arange(100, dtype=np.int64)
    raw = bytearray(raw_forward_index_bytes(L.LONG, vals, 3, 64, compression="LZ4"))
    struct.pack_into(">i", raw, 8, per_chunk)   # numDocsPerChunk
    struct.pack_into(">i", raw, 16, per_chunk)  # totalDocs
    rc, _, _ = _product_values(bytes(raw), L.LONG, 100)
    assert rc == L.PGPU_ERR_INVALID_ARGUMENT
