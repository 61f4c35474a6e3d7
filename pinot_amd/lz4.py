"""LZ4 block compression for raw (no-dictionary) forward-index chunks written by this repo's segment writer.

Pinot compresses raw chunks with lz4-java (net.jpountz.lz4 1.7.x; absent from /root/reference): LZ4 (ChunkCompressionType
3, seglocal/io/compression/LZ4Compressor.java) writes the bare LZ4 block, LZ4_LENGTH_PREFIXED (4,
LZ4WithLengthCompressor.java) the decompressed length as a little-endian int, then the block.  Readers only need a
valid block: this is a plain greedy compressor of the published LZ4 block format (sequences of token, literal-length
bytes, literals, 2-byte little-endian offset, match-length bytes; minimum match 4; the last 5 bytes are literals and
no match starts within the last 12), fast enough for test segments.  The reader that matters -- the product's -- is
in libpinotgpu.so (rt_dict.cpp, used at pin time), checked against the oracle's independent decoder.
"""
import struct

MIN_MATCH = 4
LAST_LITERALS = 5
MF_LIMIT = 12
MAX_OFFSET = 65535


def _put_len(out, n):
    while n >= 255:
        out.append(255)
        n -= 255
    out.append(n)


def _sequence(out, lit, match_len, offset):
    ll = len(lit)
    ml = match_len - MIN_MATCH if match_len else 0
    token = (min(ll, 15) << 4) | (min(ml, 15) if match_len else 0)
    out.append(token)
    if ll >= 15:
        _put_len(out, ll - 15)
    out += lit
    if match_len:
        out += struct.pack("<H", offset)
        if ml >= 15:
            _put_len(out, ml - 15)


def compress_block(data):
    """LZ4 block of `data` (bytes): greedy matches from a 4-byte hash table."""
    data = bytes(data)
    n = len(data)
    out = bytearray()
    if n < MF_LIMIT + 1:
        _sequence(out, data, 0, 0)
        return bytes(out)
    table = {}
    anchor = 0
    i = 0
    limit = n - MF_LIMIT  # no match may start at or after this
    while i < limit:
        key = data[i:i + 4]
        cand = table.get(key)
        table[key] = i
        if cand is None or i - cand > MAX_OFFSET:
            i += 1
            continue
        # extend the match forward, keeping the last LAST_LITERALS bytes as literals
        m = 4
        end = n - LAST_LITERALS
        while i + m < end and data[cand + m] == data[i + m]:
            m += 1
        _sequence(out, data[anchor:i], m, i - cand)
        for k in range(i + 1, min(i + m, limit)):  # index the matched span sparsely
            if (k & 3) == 0:
                table[data[k:k + 4]] = k
        i += m
        anchor = i
    _sequence(out, data[anchor:], 0, 0)
    return bytes(out)


def compress_with_length(data):
    """LZ4_LENGTH_PREFIXED chunk: little-endian decompressed length, then the block (LZ4CompressorWithLength)."""
    return struct.pack("<i", len(data)) + compress_block(data)
