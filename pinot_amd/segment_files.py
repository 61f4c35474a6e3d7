"""Pinot segment files: the on-disk form directly upstream of pinning.

- `write_v1_segment_dir` is the dictionary-encoded single-value subset of Pinot's segment creator: sorted unique
  dictionary (`SegmentDictionaryCreator.java:89-233`: fixed-width big-endian numbers, strings padded to the longest
  entry with the segment's padding character and ordered by their padded bytes), MSB-first fixed-bit forward index
  of `ceil(numDocs * bits / 8)` bytes (`FixedBitSVForwardIndexWriter.java:39-50`, bits =
  `PinotDataBitSet.getNumBitsPerValue(card - 1)`, `PinotDataBitSet.java:59-70`), or, for a sorted column, the
  (minDocId, maxDocId) int32 pairs per dictId (`SingleValueSortedForwardIndexCreator`), and `metadata.properties`
  with the column keys of `SegmentColumnarIndexCreator.addColumnMetadataInfo` (`:623-680`).
- `convert_v1_to_v3` lays the same buffers into `v3/columns.psf` + `v3/index_map` the way
  `SegmentV1V2ToV3FormatConverter.copyIndexData` (`:139-170`) and `SingleFileIndexDirectory` (`:71-75,166-187,
  441-466`) do: per column dictionary then forward index, each buffer preceded by the 8-byte magic marker
  0xdeadbeefdeafbead, `index_map` lines `<column>.<index>.startOffset = O` / `.size = S` (S counts the marker).
- `load_segment_dir` reads either version into `SegmentBuffers` (v3 when a `v3/` subdirectory exists,
  `SegmentDirectoryPaths.java:33-61`); the v3 reader validates every marker (`SingleFileIndexDirectory.java:
  199-207`) and parses keys from the right, since column names may contain '.' (`:220-249`).

Host code only; the bytes it yields are what `GpuTable.pin_segment` copies into HBM verbatim.
"""
import os
import shutil
import struct

import numpy as np

from . import _lib as L
from .segment import ColumnData, SegmentBuffers, _padding_byte, _parse_properties, load_v1_segment_dir

MAGIC_MARKER = 0xDEADBEEFDEAFBEAD
INDEX_FILE_NAME = "columns.psf"
INDEX_MAP_FILE_NAME = "index_map"
METADATA_FILE_NAME = "metadata.properties"
V3_SUBDIRECTORY_NAME = "v3"

_NUM_DTYPES = {L.INT: ">i4", L.LONG: ">i8", L.FLOAT: ">f4", L.DOUBLE: ">f8"}
_TYPE_STR = {v: k for k, v in L.TYPE_NAMES.items()}


def num_bits_per_value(max_value):
    """PinotDataBitSet.getNumBitsPerValue (PinotDataBitSet.java:59-70): at least one bit."""
    return 1 if max_value <= 1 else int(max_value).bit_length()


def pack_msb_first(dict_ids, bits):
    """FixedBitIntReaderWriter.writeInt over a whole column: value i at bits [i*bits, (i+1)*bits), bit 0 = MSB of
    byte 0; ceil(n*bits/8) bytes (FixedBitSVForwardIndexWriter.java:41-43)."""
    ids = np.asarray(dict_ids, dtype=np.uint32)
    n = ids.size
    if n == 0:
        return b""
    shifts = np.arange(bits - 1, -1, -1, dtype=np.uint32)
    bitmat = ((ids[:, None] >> shifts[None, :]) & 1).astype(np.uint8)
    return np.packbits(bitmat.reshape(-1)).tobytes()[: (n * bits + 7) // 8]


def _build_dictionary(data_type, values, pad_byte):
    """Sorted unique dictionary + dictIds (SegmentDictionaryCreator.build)."""
    if data_type == L.STRING:
        raw = [v.encode("utf-8") if isinstance(v, str) else bytes(v) for v in values]
        width = max((len(b) for b in raw), default=0)
        padded = [b + bytes([pad_byte]) * (width - len(b)) for b in raw]
        uniq = sorted(set(padded))
        index = {b: i for i, b in enumerate(uniq)}
        ids = np.fromiter((index[b] for b in padded), dtype=np.int32, count=len(padded))
        return b"".join(uniq), ids, len(uniq), width
    arr = np.asarray(values, dtype=np.dtype(_NUM_DTYPES[data_type]).newbyteorder("="))
    uniq, ids = np.unique(arr, return_inverse=True)
    return uniq.astype(_NUM_DTYPES[data_type]).tobytes(), ids.astype(np.int32), int(uniq.size), \
        np.dtype(_NUM_DTYPES[data_type]).itemsize


def _sorted_pairs(ids, card):
    """SingleValueSortedForwardIndexCreator: int32 BE (minDocId, maxDocId) per dictId."""
    docs = np.arange(ids.size, dtype=np.int64)
    lo = np.full(card, np.iinfo(np.int32).max, dtype=np.int64)
    hi = np.full(card, np.iinfo(np.int32).min, dtype=np.int64)
    np.minimum.at(lo, ids, docs)
    np.maximum.at(hi, ids, docs)
    return np.stack([lo, hi], axis=1).astype(">i4").tobytes()


def build_column(data_type, values, pad_byte=0, is_sorted=None):
    """One dictionary-encoded SV column as Pinot's creator writes it. `is_sorted=None` detects sortedness the way
    the stats collector does (values non-decreasing in doc order)."""
    dict_bytes, ids, card, width = _build_dictionary(data_type, values, pad_byte)
    if is_sorted is None:
        is_sorted = bool(ids.size == 0 or np.all(ids[1:] >= ids[:-1]))
    bits = num_bits_per_value(card - 1)
    if is_sorted:
        fwd, fmt = _sorted_pairs(ids, card), L.FWD_SORTED_PAIRS
    else:
        fwd, fmt = pack_msb_first(ids, bits), L.FWD_FIXED_BIT
    entry_width = width
    return ColumnData(data_type, card, bits, entry_width, dict_bytes, fwd,
                      pad_byte if data_type == L.STRING else 0, fmt, bool(is_sorted))


def serialize_roaring(doc_ids, run_optimize=False):
    """Portable RoaringBitmap serialisation (RoaringBitmap 0.9.x `serialize`, little-endian) of sorted docIds:
    containers per 65536-doc key, ARRAY when cardinality <= 4096 else BITMAP (1024 u64); with `run_optimize` a
    container is stored as RUN when that is smaller (`runOptimize`), which switches to the 12347 cookie."""
    docs = np.asarray(doc_ids, dtype=np.int64)
    keys = np.unique(docs >> 16)
    conts = []
    for k in keys:
        low = (docs[(docs >> 16) == k] & 0xFFFF).astype(np.int64)
        card = low.size
        plain = low.astype("<u2").tobytes() if card <= 4096 else None
        if plain is None:
            bm = np.zeros(2048, dtype=np.uint32)
            np.bitwise_or.at(bm, low >> 5, (np.uint32(1) << (low & 31).astype(np.uint32)))
            plain = bm.astype("<u4").tobytes()
        kind, payload = "plain", plain
        if run_optimize:
            breaks = np.nonzero(np.diff(low) != 1)[0]
            starts = np.concatenate([[0], breaks + 1])
            ends = np.concatenate([breaks, [card - 1]])
            runs = np.stack([low[starts], low[ends] - low[starts]], axis=1).astype("<u2")
            run_bytes = struct.pack("<H", len(runs)) + runs.tobytes()
            if len(run_bytes) < len(plain):
                kind, payload = "run", run_bytes
        conts.append((int(k), card, kind, payload))
    size = len(conts)
    has_run = any(c[2] == "run" for c in conts)
    out = bytearray()
    if has_run:
        out += struct.pack("<I", 12347 | ((size - 1) << 16))
        rb = bytearray((size + 7) // 8)
        for i, c in enumerate(conts):
            if c[2] == "run":
                rb[i >> 3] |= 1 << (i & 7)
        out += rb
    else:
        out += struct.pack("<II", 12346, size)
    for k, card, _, _ in conts:
        out += struct.pack("<HH", k, card - 1)
    if not has_run or size >= 4:
        off = len(out) + 4 * size
        for _, _, _, payload in conts:
            out += struct.pack("<I", off)
            off += len(payload)
    for c in conts:
        out += c[3]
    return bytes(out)


def build_inverted_index(dict_ids, cardinality, run_optimize=False):
    """BitmapInvertedIndexWriter (seglocal/segment/creator/impl/inv/BitmapInvertedIndexWriter.java:37-75): big-endian
    int32 offsets of the (cardinality + 1) bitmap boundaries, counted from the start of the file, then each dictId's
    serialised RoaringBitmap of docIds."""
    ids = np.asarray(dict_ids, dtype=np.int64)
    order = np.argsort(ids, kind="stable")
    bounds = np.searchsorted(ids[order], np.arange(cardinality + 1))
    bitmaps = [serialize_roaring(np.sort(order[bounds[i]:bounds[i + 1]]), run_optimize) for i in range(cardinality)]
    offs = np.cumsum([4 * (cardinality + 1)] + [len(b) for b in bitmaps])
    return offs.astype(">i4").tobytes() + b"".join(bitmaps)


def build_range_index(dict_ids, cardinality, num_ranges=None):
    """RangeIndexCreator (version 1, seglocal/segment/creator/impl/inv/RangeIndexCreator.java) of a dictionary-encoded
    single-value column, whose values are its dictIds (DefaultIndexCreatorProvider.newRangeIndexCreator: INT): the
    values sorted, ranges of more than ceil(numValues / numRanges) values (default 20 ranges) cut where the value
    changes (seal()), then big-endian: version, value type name, range count, the ranges' first values + the last
    range's last value, the bitmap offsets (from the start of the file; the last one = the file size), and each
    range's serialised RoaringBitmap of docIds."""
    ids = np.asarray(dict_ids, dtype=np.int64)
    n = ids.size
    per_range = (n + (num_ranges or 20) - 1) // (num_ranges or 20)
    order = np.argsort(ids, kind="stable")
    vals = ids[order]
    ranges, start = [], 0
    for i in range(n):  # seal(): `if (i > start + boundary) { if (value changed) cut }`
        if i > start + per_range and vals[i] != vals[i - 1]:
            ranges.append((start, i - 1))
            start = i
    ranges.append((start, n - 1))
    out = bytearray(struct.pack(">i", 1))
    out += struct.pack(">i", 3) + b"INT"
    out += struct.pack(">i", len(ranges))
    for a, _ in ranges:
        out += struct.pack(">i", int(vals[a]))
    out += struct.pack(">i", int(vals[ranges[-1][1]]))
    bitmaps = [serialize_roaring(np.sort(order[a:b + 1])) for a, b in ranges]
    off = len(out) + 8 * (len(ranges) + 1)
    out += struct.pack(">q", off)
    for bm in bitmaps:
        off += len(bm)
        out += struct.pack(">q", off)
    return bytes(out) + b"".join(bitmaps)


def build_range_index_bitsliced_header(min_value=0):
    """The header of a version-2 (BitSlicedRangeIndexCreator) range index -- version, the column's minimum (dictId 0
    for a dictionary-encoded column) -- followed by a placeholder for its RangeBitmap body, which readers of this
    repository never parse: the index is exact, so the GPU path reads the matches from the forward index and scans
    no partial matches (BitSlicedRangeIndexReader.getPartiallyMatchingDocIds: null).  Format parity of the body is
    not claimed (RoaringBitmap 0.9.23's RangeBitmap is absent here)."""
    return struct.pack(">iq", 2, int(min_value)) + b"\0" * 16


def build_inverted_index_native(fwd_bytes, bits, num_docs, cardinality):
    """The same file from the library's host creator (pgpu_build_inverted_index; no GPU involved)."""
    import ctypes
    lib = L.load()
    fwd = ctypes.create_string_buffer(bytes(fwd_bytes), max(len(fwd_bytes), 1))
    n = ctypes.c_int64()
    L.check(lib.pgpu_build_inverted_index(fwd, len(fwd_bytes), bits, num_docs, cardinality, None, 0, ctypes.byref(n)))
    out = ctypes.create_string_buffer(max(n.value, 1))
    L.check(lib.pgpu_build_inverted_index(fwd, len(fwd_bytes), bits, num_docs, cardinality, out, n.value,
                                          ctypes.byref(n)))
    return out.raw[:n.value]


def _dict_ids(c, num_docs):
    """dictIds of every doc of a column (fixed-bit or sorted pairs)."""
    if c.fwd_format == L.FWD_SORTED_PAIRS:
        pairs = np.frombuffer(c.fwd_bytes, dtype=">i4").reshape(-1, 2).astype(np.int64)
        return np.repeat(np.arange(c.cardinality), np.maximum(pairs[:, 1] - pairs[:, 0] + 1, 0))
    b = c.bits_per_element
    bits = np.unpackbits(np.frombuffer(c.fwd_bytes, dtype=np.uint8))[: num_docs * b].reshape(num_docs, b)
    return (bits.astype(np.int64) << np.arange(b - 1, -1, -1)).sum(axis=1)


def _fwd_file_name(name, col):
    return name + (".sv.sorted.fwd" if col.fwd_format == L.FWD_SORTED_PAIRS else ".sv.unsorted.fwd")


def _metadata_lines(segment_name, table_name, num_docs, columns, pad_byte, version):
    pad = "\\u%04x" % pad_byte if pad_byte < 0x20 else chr(pad_byte)
    lines = ["segment.padding.character = " + pad,
             "segment.name = " + segment_name,
             "segment.table.name = " + table_name,
             "segment.dimension.column.names = " + ",".join(columns),
             "segment.metric.column.names = ",
             "segment.total.docs = %d" % num_docs]
    if version:
        lines.append("segment.index.version = " + version)
    for name, c in columns.items():
        p = "column.%s." % name
        lines += [p + "cardinality = %d" % c.cardinality,
                  p + "totalDocs = %d" % num_docs,
                  p + "dataType = " + _TYPE_STR[c.data_type],
                  p + "bitsPerElement = %d" % c.bits_per_element,
                  p + "lengthOfEachEntry = %d" % (c.entry_width if c.data_type == L.STRING else 0),
                  p + "columnType = DIMENSION",
                  p + "isSorted = " + ("true" if c.is_sorted else "false"),
                  p + "hasDictionary = true",
                  p + "isSingleValues = true",
                  p + "maxNumberOfMultiValues = 0",
                  p + "totalNumberOfEntries = %d" % num_docs]
    return "\n".join(lines) + "\n"


def write_v1_segment_dir(path, schema, values, segment_name="segment_0", table_name="table", pad_byte=0,
                         sorted_columns=(), inverted_columns=(), run_optimize=False):
    """Creates a v1 segment directory from column values; returns its SegmentBuffers.

    schema: [(name, "INT"|"LONG"|"FLOAT"|"DOUBLE"|"STRING")]; values: {name: sequence}. Columns named in
    `sorted_columns` are written with the sorted forward index (their values must be non-decreasing); columns named
    in `inverted_columns` also get a bitmap inverted index (`<column>.bitmap.inv`)."""
    os.makedirs(path, exist_ok=True)
    num_docs = len(values[schema[0][0]]) if schema else 0
    cols = {}
    for name, typ in schema:
        if len(values[name]) != num_docs:
            raise ValueError("column %s has %d values, expected %d" % (name, len(values[name]), num_docs))
        c = build_column(L.TYPE_NAMES[typ], values[name], pad_byte,
                         True if name in sorted_columns else False)
        if c.is_sorted and num_docs and c.fwd_format == L.FWD_SORTED_PAIRS:
            pairs = np.frombuffer(c.fwd_bytes, dtype=">i4").reshape(-1, 2)
            if np.any(pairs[1:, 0] != pairs[:-1, 1] + 1):
                raise ValueError("column %s is not sorted in doc order" % name)
        if name in inverted_columns:
            c.inv_bytes = build_inverted_index(_dict_ids(c, num_docs), c.cardinality, run_optimize)
            with open(os.path.join(path, name + ".bitmap.inv"), "wb") as f:
                f.write(c.inv_bytes)
        cols[name] = c
        with open(os.path.join(path, name + ".dict"), "wb") as f:
            f.write(c.dict_bytes)
        with open(os.path.join(path, _fwd_file_name(name, c)), "wb") as f:
            f.write(c.fwd_bytes)
    with open(os.path.join(path, METADATA_FILE_NAME), "w") as f:
        f.write(_metadata_lines(segment_name, table_name, num_docs, cols, pad_byte, None))
    return SegmentBuffers(num_docs, cols)


def convert_v1_to_v3(path):
    """SegmentV1V2ToV3FormatConverter: writes <path>/v3/{columns.psf,index_map,metadata.properties}."""
    v1 = load_v1_segment_dir(path)
    v3 = os.path.join(path, V3_SUBDIRECTORY_NAME)
    os.makedirs(v3, exist_ok=True)
    marker = struct.pack(">Q", MAGIC_MARKER)
    offset = 0
    index_map = []
    with open(os.path.join(v3, INDEX_FILE_NAME), "wb") as psf:
        for name in sorted(v1.columns):
            c = v1.columns[name]
            for index_name, buf in (("dictionary", c.dict_bytes), ("forward_index", c.fwd_bytes)):
                psf.write(marker)
                psf.write(buf)
                index_map.append("%s.%s.startOffset = %d" % (name, index_name, offset))
                index_map.append("%s.%s.size = %d" % (name, index_name, len(buf) + len(marker)))
                offset += len(buf) + len(marker)
        for name in sorted(v1.columns):  # inverted indexes follow every column's dictionary + forward index
            c = v1.columns[name]
            if c.inv_bytes is not None:
                psf.write(marker)
                psf.write(c.inv_bytes)
                index_map.append("%s.inverted_index.startOffset = %d" % (name, offset))
                index_map.append("%s.inverted_index.size = %d" % (name, len(c.inv_bytes) + len(marker)))
                offset += len(c.inv_bytes) + len(marker)
    with open(os.path.join(v3, INDEX_MAP_FILE_NAME), "w") as f:
        f.write("\n".join(index_map) + "\n")
    for star in ("star_tree_index", "star_tree_index_map"):  # copyStarTreeV2 (SegmentV1V2ToV3FormatConverter:182-190)
        if os.path.exists(os.path.join(path, star)):
            shutil.copyfile(os.path.join(path, star), os.path.join(v3, star))
    with open(os.path.join(path, METADATA_FILE_NAME)) as f:
        meta = [ln for ln in f.read().splitlines() if not ln.startswith("segment.index.version")]
    with open(os.path.join(v3, METADATA_FILE_NAME), "w") as f:
        f.write("\n".join(meta + ["segment.index.version = v3"]) + "\n")
    return v3


def _load_index_map(path):
    entries = {}
    with open(path) as f:
        for key, value in _parse_properties(f.read()).items():
            last = key.rfind(".")
            prev = key.rfind(".", 0, last) if last > 0 else -1
            if last < 0 or prev < 0:
                raise ValueError("malformed index_map key: %r" % key)
            prop, index_name, column = key[last + 1:], key[prev + 1:last], key[:prev]
            if prop not in ("startOffset", "size"):
                raise ValueError("invalid index_map key: %r" % key)
            entries.setdefault((column, index_name), {})[prop] = int(value)
    for k, e in entries.items():
        if e.get("startOffset", -1) < 0 or e.get("size", -1) < 0:
            raise ValueError("invalid index_map entry for %s" % (k,))
    return entries


def load_v3_segment_dir(v3_path):
    with open(os.path.join(v3_path, METADATA_FILE_NAME)) as f:
        props = _parse_properties(f.read())
    entries = _load_index_map(os.path.join(v3_path, INDEX_MAP_FILE_NAME))
    num_docs = int(props["segment.total.docs"])
    pad = _padding_byte(props)
    psf = np.memmap(os.path.join(v3_path, INDEX_FILE_NAME), dtype=np.uint8, mode="r") \
        if os.path.getsize(os.path.join(v3_path, INDEX_FILE_NAME)) else np.zeros(0, np.uint8)

    def buffer(column, index_name):
        e = entries.get((column, index_name))
        if e is None:
            raise ValueError("segment %s has no %s for column %s" % (v3_path, index_name, column))
        start, size = e["startOffset"], e["size"]
        if start + size > psf.size or size < 8:
            raise ValueError("index_map entry %s.%s overruns columns.psf" % (column, index_name))
        if struct.unpack(">Q", psf[start:start + 8].tobytes())[0] != MAGIC_MARKER:
            raise ValueError("missing magic marker at %d in %s" % (start, v3_path))
        return psf[start + 8:start + size].tobytes()

    cols = {}
    names = sorted({k[len("column."):-len(".cardinality")] for k in props
                    if k.startswith("column.") and k.endswith(".cardinality")})
    for name in names:
        p = "column.%s." % name
        dtype = L.TYPE_NAMES[props[p + "dataType"]]
        width = {L.INT: 4, L.FLOAT: 4, L.LONG: 8, L.DOUBLE: 8}.get(dtype, int(props.get(p + "lengthOfEachEntry", 0)))
        is_sorted = props.get(p + "isSorted", "false") == "true"
        cols[name] = ColumnData(dtype, int(props[p + "cardinality"]), int(props[p + "bitsPerElement"]), width,
                                buffer(name, "dictionary"), buffer(name, "forward_index"),
                                pad if dtype == L.STRING else 0,
                                L.FWD_SORTED_PAIRS if is_sorted else L.FWD_FIXED_BIT, is_sorted,
                                buffer(name, "inverted_index") if (name, "inverted_index") in entries else None)
    return SegmentBuffers(num_docs, cols)


def load_segment_dir(path):
    """ImmutableSegmentLoader's directory step: v3 if `<path>/v3` exists (or `path` is one), else v1."""
    if os.path.basename(os.path.normpath(path)) == V3_SUBDIRECTORY_NAME:
        return load_v3_segment_dir(path)
    v3 = os.path.join(path, V3_SUBDIRECTORY_NAME)
    if os.path.isdir(v3):
        return load_v3_segment_dir(v3)
    return load_v1_segment_dir(path)
