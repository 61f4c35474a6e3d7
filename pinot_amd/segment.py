"""Host-side view of a Pinot ImmutableSegment as the GPU path consumes it: per column the dictionary bytes
(BIG_ENDIAN fixed width, BaseImmutableDictionary) and the forward-index bytes (FixedBitSVForwardIndexReaderV2
MSB-first packing, or SortedIndexReaderImpl pairs), exactly as they sit in PinotDataBuffers.

`load_v1_segment_dir` reads a v1 segment directory (metadata.properties + <col>.dict + <col>.sv.{un}sorted.fwd),
the on-disk form directly upstream of pinning (SegmentColumnarIndexCreator / SegmentDictionaryCreator;
segspi/V1Constants.java:25-103).
"""
import os
from dataclasses import dataclass, field

from . import _lib as L


@dataclass
class ColumnData:
    data_type: int
    cardinality: int
    bits_per_element: int
    entry_width: int
    dict_bytes: bytes
    fwd_bytes: bytes
    padding_byte: int = 0
    fwd_format: int = L.FWD_FIXED_BIT
    is_sorted: bool = False
    inv_bytes: bytes = None  # bitmap inverted index (<column>.bitmap.inv), if the column has one


@dataclass
class SegmentBuffers:
    num_docs: int
    columns: dict = field(default_factory=dict)  # name -> ColumnData

    def column_names(self):
        return list(self.columns)


def _parse_properties(text):
    props = {}
    for line in text.splitlines():
        line = line.strip()
        if not line or line.startswith("#") or "=" not in line:
            continue
        k, v = line.split("=", 1)
        props[k.strip()] = v.strip()
    return props


def _padding_byte(props):
    raw = props.get("segment.padding.character", "%")  # legacy segments default to '%'
    raw = raw.replace("\\\\", "\\")
    if raw in ("\\u0000", "\0", ""):
        return 0
    if raw.startswith("\\u"):
        return int(raw[2:], 16)
    return ord(raw[0])


def load_v1_segment_dir(path):
    """Reads a Pinot v1 segment directory into SegmentBuffers (dictionary-encoded single-value columns)."""
    with open(os.path.join(path, "metadata.properties")) as f:
        props = _parse_properties(f.read())
    num_docs = int(props["segment.total.docs"])
    pad = _padding_byte(props)
    cols = {}
    names = sorted({k[len("column."):-len(".cardinality")] for k in props
                    if k.startswith("column.") and k.endswith(".cardinality")})  # names may contain '.'
    for name in names:
        p = "column.%s." % name
        dtype = L.TYPE_NAMES[props[p + "dataType"]]
        card = int(props[p + "cardinality"])
        bits = int(props[p + "bitsPerElement"])
        width = {L.INT: 4, L.FLOAT: 4, L.LONG: 8, L.DOUBLE: 8}.get(dtype, int(props.get(p + "lengthOfEachEntry", 0)))
        with open(os.path.join(path, name + ".dict"), "rb") as f:
            d = f.read()
        sorted_fwd = os.path.join(path, name + ".sv.sorted.fwd")
        if os.path.exists(sorted_fwd):
            with open(sorted_fwd, "rb") as f:
                fwd = f.read()
            fmt = L.FWD_SORTED_PAIRS
        else:
            with open(os.path.join(path, name + ".sv.unsorted.fwd"), "rb") as f:
                fwd = f.read()
            fmt = L.FWD_FIXED_BIT
        inv_path = os.path.join(path, name + ".bitmap.inv")
        inv = None
        if os.path.exists(inv_path):
            with open(inv_path, "rb") as f:
                inv = f.read()
        cols[name] = ColumnData(dtype, card, bits, width, d, fwd, pad if dtype == L.STRING else 0, fmt,
                                props.get(p + "isSorted", "false") == "true", inv)
    return SegmentBuffers(num_docs, cols)
