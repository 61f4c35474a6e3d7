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
    range_bytes: bytes = None  # range index (<column>.bitmap.range, version 1 or 2), if the column has one


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


RAW_DOCS_PER_CHUNK = 1000  # SingleValueFixedByteRawIndexCreator.NUM_DOCS_PER_CHUNK (:36)
_RAW_FMT = {L.INT: ">i", L.LONG: ">q", L.FLOAT: ">f", L.DOUBLE: ">d"}


# ChunkCompressionType (segspi/compression/ChunkCompressionType.java:22)
COMPRESSION = {"PASS_THROUGH": 0, "SNAPPY": 1, "ZSTANDARD": 2, "LZ4": 3, "LZ4_LENGTH_PREFIXED": 4}


def raw_forward_index_bytes(data_type, values, version=2, docs_per_chunk=RAW_DOCS_PER_CHUNK,
                            compression="PASS_THROUGH"):
    """A no-dictionary fixed-width column as FixedByteChunkSVForwardIndexWriter writes it
    (BaseChunkSVForwardIndexWriter.java:71-193): header (version, numChunks, numDocsPerChunk, sizeOfEntry, then for
    version > 1 totalDocs, compression type, dataHeaderStart), the chunk offsets (int for version 2, long for 3; each
    the absolute position of its chunk), then the chunks: big-endian values back to back, each chunk compressed on
    its own (writeChunk; the last chunk holds the remaining docs) -- PASS_THROUGH as is, LZ4 as an LZ4 block,
    LZ4_LENGTH_PREFIXED as the little-endian decompressed length + the block (pinot_amd.lz4)."""
    import struct
    from . import lz4
    if version not in (2, 3):
        raise ValueError("raw forward index version %d (2 or 3)" % version)
    codec = COMPRESSION[compression]
    if codec not in (0, 3, 4):
        raise ValueError("writer supports PASS_THROUGH, LZ4 and LZ4_LENGTH_PREFIXED chunks")
    fmt = _RAW_FMT[data_type]
    size = struct.calcsize(fmt)
    n = len(values)
    num_chunks = (n + docs_per_chunk - 1) // docs_per_chunk
    entry = 4 if version == 2 else 8
    header_size = 7 * 4 + num_chunks * entry
    hdr = struct.pack(">iiiiiii", version, num_chunks, docs_per_chunk, size, n, codec, 7 * 4)
    cast = float if data_type in (L.FLOAT, L.DOUBLE) else int
    chunks, offsets, off = [], [], header_size
    for c in range(num_chunks):
        raw = b"".join(struct.pack(fmt, cast(v)) for v in values[c * docs_per_chunk:(c + 1) * docs_per_chunk])
        body = raw if codec == 0 else lz4.compress_block(raw) if codec == 3 else lz4.compress_with_length(raw)
        offsets.append(off)
        chunks.append(body)
        off += len(body)
    hdr += b"".join(struct.pack(">i" if version == 2 else ">q", o) for o in offsets)
    return hdr + b"".join(chunks)


def build_raw_column(type_name, values, version=2, docs_per_chunk=RAW_DOCS_PER_CHUNK, compression="PASS_THROUGH"):
    """ColumnData of a raw (no-dictionary) INT / LONG / FLOAT / DOUBLE column."""
    t = L.TYPE_NAMES[type_name] if isinstance(type_name, str) else int(type_name)
    fwd = raw_forward_index_bytes(t, values, version, docs_per_chunk, compression)
    return ColumnData(t, 0, 0, 4 if t in (L.INT, L.FLOAT) else 8, b"", fwd, fwd_format=L.FWD_RAW_FIXED)
