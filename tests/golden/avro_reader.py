"""Minimal Avro object-container reader (null codec, records of nullable primitives).

Used only to turn the reference's test input ``pinot-core/src/test/resources/data/test_data-sv.avro`` into the
numeric fixture under tests/golden/ (see make_golden.py).  Implements the Avro 1.x container spec: header
(magic, metadata map, sync marker), then blocks of (count, byte size, records, sync).
"""
import json


class _Buf:
    def __init__(self, data, pos=0):
        self.d = data
        self.p = pos

    def long(self):
        shift = 0
        acc = 0
        while True:
            b = self.d[self.p]
            self.p += 1
            acc |= (b & 0x7F) << shift
            if not b & 0x80:
                break
            shift += 7
        return (acc >> 1) ^ -(acc & 1)  # zig-zag

    def bytes(self):
        n = self.long()
        v = self.d[self.p:self.p + n]
        self.p += n
        return v

    def raw(self, n):
        v = self.d[self.p:self.p + n]
        self.p += n
        return v


def _read_value(buf, typ):
    if isinstance(typ, list):  # union
        return _read_value(buf, typ[buf.long()])
    if isinstance(typ, dict):
        typ = typ["type"]
    if typ == "null":
        return None
    if typ in ("int", "long"):
        return buf.long()
    if typ == "string":
        return buf.bytes().decode("utf-8")
    if typ == "bytes":
        return bytes(buf.bytes())
    if typ == "boolean":
        v = buf.d[buf.p]
        buf.p += 1
        return bool(v)
    if typ in ("float", "double"):
        import struct
        n = 4 if typ == "float" else 8
        return struct.unpack("<f" if n == 4 else "<d", buf.raw(n))[0]
    raise ValueError("unsupported avro type %r" % (typ,))


def read_avro(path):
    """Returns (field_names, rows) where rows is a list of tuples in file order."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"Obj\x01":
        raise ValueError("not an avro container")
    buf = _Buf(data, 4)
    meta = {}
    while True:
        n = buf.long()
        if n == 0:
            break
        if n < 0:
            buf.long()
            n = -n
        for _ in range(n):
            k = buf.bytes().decode()
            meta[k] = bytes(buf.bytes())
    codec = meta.get("avro.codec", b"null").decode()
    if codec != "null":
        raise ValueError("codec %s not supported" % codec)
    schema = json.loads(meta["avro.schema"].decode())
    sync = buf.raw(16)
    fields = schema["fields"]
    names = [f["name"] for f in fields]
    rows = []
    while buf.p < len(data):
        count = buf.long()
        size = buf.long()
        end = buf.p + size
        for _ in range(count):
            rows.append(tuple(_read_value(buf, f["type"]) for f in fields))
        if buf.p != end:
            raise ValueError("block size mismatch")
        if buf.raw(16) != sync:
            raise ValueError("sync marker mismatch")
    return names, rows
