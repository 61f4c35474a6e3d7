"""Raw (no-dictionary) fixed-width columns, CPU side: the FixedByteChunkSVForwardIndexWriter restatement
(pinot_amd.segment.raw_forward_index_bytes) read back by the oracle's FixedByteChunkSVForwardIndexReader
restatement -- the reference's own round-trip test (FixedByteChunkSVForwardIndexTest.java: 10 009 values, 5 003
docs per chunk so the last chunk is partial, versions 2 and 3 = 4- and 8-byte chunk offsets)."""
import ctypes
import struct

import numpy as np
import pytest

from pinot_amd import _lib as L
from pinot_amd.segment import build_raw_column, raw_forward_index_bytes

NUM_VALUES, PER_CHUNK = 10009, 5003


def _values(t, rng):
    if t == L.INT:
        return rng.integers(-2 ** 31, 2 ** 31, NUM_VALUES).tolist()
    if t == L.LONG:
        return rng.integers(-2 ** 63, 2 ** 63 - 1, NUM_VALUES, dtype=np.int64).tolist()
    if t == L.FLOAT:
        return np.float32(rng.normal(0, 1e6, NUM_VALUES)).astype(np.float64).tolist()
    return rng.normal(0, 1e12, NUM_VALUES).tolist()


@pytest.mark.parametrize("version", [2, 3])
@pytest.mark.parametrize("type_name", ["INT", "LONG", "FLOAT", "DOUBLE"])
def test_round_trip_through_the_oracle_reader(oracle, version, type_name):
    t = L.TYPE_NAMES[type_name]
    vals = _values(t, np.random.default_rng(version * 10 + t))
    raw = raw_forward_index_bytes(t, vals, version, PER_CHUNK)
    # header as BaseChunkSVForwardIndexWriter.writeHeader lays it out
    ver, nchunks, per, size, total, comp, start = struct.unpack(">iiiiiii", raw[:28])
    assert (ver, nchunks, per, total, comp, start) == (version, 2 + 1, PER_CHUNK, NUM_VALUES, 0, 28)
    assert size == (4 if t in (L.INT, L.FLOAT) else 8)
    lib = oracle.lib()
    lib.or_raw_get_double.restype = ctypes.c_double
    lib.or_raw_get_double.argtypes = [ctypes.POINTER(oracle.OrColumn), ctypes.c_int]
    buf = ctypes.create_string_buffer(raw, len(raw))
    col = oracle.OrColumn(t, 0, 0, size, 0, 0, 0, None, ctypes.cast(buf, ctypes.c_void_p), 1, len(raw))
    for i in list(range(0, NUM_VALUES, 97)) + [PER_CHUNK - 1, PER_CHUNK, NUM_VALUES - 1]:
        assert lib.or_raw_get_double(ctypes.byref(col), i) == float(vals[i]), i


def test_column_data_of_a_raw_column():
    c = build_raw_column("DOUBLE", [1.5, -2.0, 3.25])
    assert (c.cardinality, c.bits_per_element, c.entry_width, c.fwd_format) == (0, 0, 8, L.FWD_RAW_FIXED)
    assert c.dict_bytes == b"" and len(c.fwd_bytes) == 28 + 4 + 3 * 8
