"""Pins the oracle's codec and dictionaries to the reference's golden bytes and bit-layout spec (CPU only).

- padding{Old,Null,Percent}.tar.gz: real Pinot-written v1 segments (tests/golden/padding_segments.json)
- FixedBitIntReaderTest.java:48-76 (seglocal-test/io/reader/impl/): every width 1..31 round-trips
- PinotDataBitSet.getNumBitsPerValue javadoc examples (PinotDataBitSet.java:45-58)
"""
import ctypes
import json
import os
import struct

import numpy as np
import pytest

from pinot_amd import _lib as L
from pinot_amd.segment import ColumnData, SegmentBuffers

HERE = os.path.dirname(os.path.abspath(__file__))


def _padding():
    with open(os.path.join(HERE, "golden", "padding_segments.json")) as f:
        return json.load(f)


def _np_unpack(buf, nbits, n):
    """Independent numpy decoder of the MSB-first layout (bit i*b is the MSB of value i)."""
    bits = np.unpackbits(np.frombuffer(buf, dtype=np.uint8))
    idx = np.arange(n)[:, None] * nbits + np.arange(nbits)[None, :]
    w = (1 << np.arange(nbits - 1, -1, -1)).astype(np.int64)
    return (bits[idx].astype(np.int64) * w).sum(axis=1)


def test_num_bits_per_value(oracle):
    o = oracle.lib()
    for v, b in [(0, 1), (1, 1), (2, 2), (9, 4), (113, 7), (255, 8), (256, 9), (65535, 16), (2 ** 31 - 1, 31)]:
        assert o.or_num_bits_per_value(v) == b


@pytest.mark.parametrize("name", ["paddingOld", "paddingNull", "paddingPercent"])
def test_padding_segment_bytes(oracle, name):
    seg = _padding()[name]
    o = oracle.lib()
    age = seg["columns"]["age"]
    fwd = bytes.fromhex(age["fwd_hex"]) + b"\0" * 8
    ids = [o.or_bitset_read_int(fwd, i, age["bitsPerElement"]) for i in range(seg["totalDocs"])]
    assert ids == [4, 2, 3, 0, 1]  # verified by hand in SURVEY.md §4
    assert list(_np_unpack(fwd, 3, 5)) == ids
    d = bytes.fromhex(age["dict_hex"])
    vals = list(struct.unpack(">5i", d))
    assert vals == sorted(vals) == [617, 824, 837, 1209, 1228]
    # the LONG time column and the FLOAT column decode to sorted dictionaries too
    assert list(struct.unpack(">5q", bytes.fromhex(seg["columns"]["outgoingName1"]["dict_hex"]))) == \
        sorted(struct.unpack(">5q", bytes.fromhex(seg["columns"]["outgoingName1"]["dict_hex"])))
    f = struct.unpack(">5f", bytes.fromhex(seg["columns"]["percent"]["dict_hex"]))
    assert list(f) == sorted(f)


def _padded_segment_column(seg, col):
    c = seg["columns"][col]
    pad = seg["paddingCharacter"]
    pad_byte = 0 if "u0000" in pad else ord(pad[0])
    return c, pad_byte


def test_string_dictionary_padding_lookup(oracle):
    """insertionIndexOf on padded string dictionaries: '%' legacy padding vs NUL padding order differently."""
    o = oracle.lib()
    o.or_dict_insertion_index_of.restype = ctypes.c_int
    o.or_dict_insertion_index_of.argtypes = [ctypes.POINTER(oracle.OrColumn), ctypes.c_char_p,
                                             ctypes.POINTER(ctypes.c_int)]
    segs = _padding()
    for name, expect_fwd in [("paddingOld", [1, 0, 0, 0, 1]), ("paddingNull", [0, 1, 1, 1, 0])]:
        c, pad = _padded_segment_column(segs[name], "name")
        fwd = bytes.fromhex(c["fwd_hex"]) + b"\0" * 8
        assert [o.or_bitset_read_int(fwd, i, 1) for i in range(5)] == expect_fwd
        d = ctypes.create_string_buffer(bytes.fromhex(c["dict_hex"]))
        col = oracle.OrColumn(L.STRING, 2, 1, c["lengthOfEachEntry"], pad, 0, 0, ctypes.cast(d, ctypes.c_void_p), None)
        err = ctypes.c_int()
        lynda = o.or_dict_insertion_index_of(ctypes.byref(col), b"lynda", ctypes.byref(err))
        lynda2 = o.or_dict_insertion_index_of(ctypes.byref(col), b"lynda 2.0", ctypes.byref(err))
        if pad == 0:
            assert (lynda, lynda2) == (0, 1)
        else:
            assert (lynda, lynda2) == (1, 0)


@pytest.mark.parametrize("nbits", list(range(1, 32)))
def test_fixed_bit_round_trip(oracle, nbits):
    """FixedBitIntReaderTest: random values of every width; read, bulk read and readDictIds agree."""
    o = oracle.lib()
    rng = np.random.default_rng(nbits)
    n = 1000
    vals = rng.integers(0, 1 << nbits, size=n, dtype=np.int64).astype(np.int32)
    buf = np.zeros(o.or_fwd_num_bytes(n, nbits) + 16, dtype=np.uint8)
    o.or_bitset_write_ints(buf.ctypes.data, 0, nbits, n, vals.ctypes.data)
    single = np.array([o.or_bitset_read_int(buf.ctypes.data, i, nbits) for i in range(n)], dtype=np.int32)
    np.testing.assert_array_equal(single, vals)
    bulk = np.zeros(n, dtype=np.int32)
    o.or_bitset_read_ints(buf.ctypes.data, 0, nbits, n, bulk.ctypes.data)
    np.testing.assert_array_equal(bulk, vals)
    np.testing.assert_array_equal(_np_unpack(buf.tobytes(), nbits, n), vals)
    for docs in (np.arange(100, 900, dtype=np.int32), np.sort(rng.choice(n, 300, replace=False)).astype(np.int32)):
        out = np.zeros(len(docs), dtype=np.int32)
        o.or_read_dict_ids(buf.ctypes.data, nbits, n, docs.ctypes.data, len(docs), out.ctypes.data)
        np.testing.assert_array_equal(out, vals[docs])


def test_bit9_reader_shift_spec(oracle):
    """FixedBitIntReader.Bit9Reader.read32 (:679-723): value 3 = ((i0 & 0x1f) << 4) | (i1 >>> 28)."""
    o = oracle.lib()
    rng = np.random.default_rng(9)
    words = rng.integers(0, 2 ** 32, size=9, dtype=np.uint64).astype(">u4")
    buf = words.tobytes() + b"\0" * 8
    i0, i1, i8 = int(words[0]), int(words[1]), int(words[8])
    assert o.or_bitset_read_int(buf, 0, 9) == i0 >> 23
    assert o.or_bitset_read_int(buf, 3, 9) == ((i0 & 0x1F) << 4) | (i1 >> 28)
    assert o.or_bitset_read_int(buf, 31, 9) == i8 & 0x1FF


def test_build_column_matches_pinot_layout(oracle):
    """The oracle's segment creator writes the same layout as the Pinot-written padding segments."""
    seg = oracle.make_segment([("age", "INT")], {"age": [1228, 837, 1209, 617, 824]})
    c = seg.columns["age"]
    assert c.cardinality == 5 and c.bits_per_element == 3
    assert c.dict_bytes.hex() == _padding()["paddingOld"]["columns"]["age"]["dict_hex"]
    assert c.fwd_bytes.hex() == _padding()["paddingOld"]["columns"]["age"]["fwd_hex"]


def test_strings_sorted_by_bytes(oracle):
    seg = oracle.make_segment([("s", "STRING")], {"s": ["b", "", "ab", "a", "b"]})
    c = seg.columns["s"]
    assert c.cardinality == 4 and c.entry_width == 2
    entries = [c.dict_bytes[i * 2:(i + 1) * 2].rstrip(b"\0") for i in range(4)]
    assert entries == [b"", b"a", b"ab", b"b"]
