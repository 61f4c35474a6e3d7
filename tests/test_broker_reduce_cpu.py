"""Broker reduce of server DataTable V3 responses (pgpu_broker_reduce_sql, GroupByDataTableReducer.java:290-330)
on CPU: the server tables are written here byte by byte after DataTableImplV3.toBytes (DataTableImplV3.java:
183-290) -- header of 13 big-endian ints, exceptions, dictionary map, data schema, fixed-size rows, variable-size
data, then the metadata -- so the test also pins the reader against the format rather than against our writer."""
import struct

import pytest

from pinot_amd.executor import broker_reduce_sql
from pinot_amd.query import parse_query

META = {"numDocsScanned": (2, "q"), "numEntriesScannedInFilter": (3, "q"), "numEntriesScannedPostFilter": (4, "q"),
        "numSegmentsProcessed": (6, "i"), "numSegmentsMatched": (7, "i"), "totalDocs": (10, "q")}


def _s(x):
    b = x.encode()
    return struct.pack(">i", len(b)) + b


def datatable(names, types, rows, meta):
    """rows: lists of python values; STRING cells go through the per-column dictionary map, OBJECT cells are
    (sum, count) AvgPairs in the variable-size section."""
    dicts = {}
    fixed, var = b"", b""
    for row in rows:
        for n, t, v in zip(names, types, row):
            if t == "INT":
                fixed += struct.pack(">i", v)
            elif t == "LONG":
                fixed += struct.pack(">q", v)
            elif t == "DOUBLE":
                fixed += struct.pack(">d", v)
            elif t == "STRING":
                d = dicts.setdefault(n, {})
                fixed += struct.pack(">i", d.setdefault(v, len(d)))
            else:
                obj = struct.pack(">i", 4) + struct.pack(">dq", *v)  # ObjectType.AvgPair, AvgPair.toBytes
                fixed += struct.pack(">ii", len(var), 16)
                var += obj
    exc = struct.pack(">i", 0)
    dic = struct.pack(">i", len(dicts)) + b"".join(
        _s(c) + struct.pack(">i", len(m)) + b"".join(struct.pack(">i", i) + _s(v) for v, i in m.items())
        for c, m in dicts.items())
    sch = struct.pack(">i", len(names)) + b"".join(_s(n) for n in names) + b"".join(_s(t) for t in types)
    md = struct.pack(">i", len(meta)) + b"".join(
        struct.pack(">i", META[k][0]) + struct.pack(">" + META[k][1], v) for k, v in meta.items())
    off = 13 * 4
    hdr = struct.pack(">iii", 3, len(rows), len(names))
    for sec in (exc, dic, sch, fixed, var):
        hdr += struct.pack(">ii", off, len(sec))
        off += len(sec)
    return hdr + exc + dic + sch + fixed + var + struct.pack(">i", len(md)) + md


def _meta(docs):
    return {"numDocsScanned": docs, "numEntriesScannedInFilter": 0, "numEntriesScannedPostFilter": 2 * docs,
            "numSegmentsProcessed": 2, "numSegmentsMatched": 2, "totalDocs": docs}


def test_reduce_merges_orders_and_limits():
    names, types = ["column11", "sum(column1)"], ["STRING", "DOUBLE"]
    a = datatable(names, types, [["P", 10.0], ["o", 3.0], ["", 7.0]], _meta(100))
    b = datatable(names, types, [["o", 4.0], ["t", 1.0], ["P", 2.5]], _meta(50))
    q = parse_query("SELECT column11, SUM(column1) FROM t GROUP BY column11 ORDER BY SUM(column1) DESC LIMIT 3")
    r = broker_reduce_sql([a, b], q)
    assert r["resultTable"]["dataSchema"] == {"columnNames": names, "columnDataTypes": types}
    assert r["resultTable"]["rows"] == [["P", 12.5], ["", 7.0], ["o", 7.0]]  # tie: key order
    assert r["numDocsScanned"] == 150 and r["totalDocs"] == 150 and r["numEntriesScannedPostFilter"] == 300
    assert r["numServersQueried"] == 2


def test_reduce_avg_count_and_hidden_order_by_aggregation():
    names = ["column17", "count(*)", "avg(column6)", "min(column6)"]
    types = ["INT", "LONG", "OBJECT", "DOUBLE"]
    a = datatable(names, types, [[5, 2, (10.0, 2), 1.0], [9, 1, (7.0, 1), 7.0]], _meta(3))
    b = datatable(names, types, [[5, 1, (2.0, 1), 0.5], [1, 4, (4.0, 4), 0.0]], _meta(5))
    q = parse_query("SELECT column17, COUNT(*), AVG(column6) FROM t GROUP BY column17 ORDER BY MIN(column6) DESC")
    r = broker_reduce_sql([a, b], q)
    rt = r["resultTable"]
    assert rt["dataSchema"]["columnNames"] == ["column17", "count(*)", "avg(column6)"]
    assert rt["dataSchema"]["columnDataTypes"] == ["INT", "LONG", "DOUBLE"]
    assert rt["rows"] == [[9, 1, 7.0], [5, 3, 4.0], [1, 4, 1.0]]


def test_reduce_no_rows_and_bad_bytes():
    names, types = ["column11", "min(column6)"], ["STRING", "DOUBLE"]
    e = datatable(names, types, [], _meta(0))
    q = parse_query("SELECT column11, MIN(column6) FROM t GROUP BY column11 ORDER BY column11")
    r = broker_reduce_sql([e, e], q)
    assert r["resultTable"]["rows"] == [] and r["numDocsScanned"] == 0
    with pytest.raises(Exception):
        broker_reduce_sql([e[:20]], q)
    with pytest.raises(Exception):
        broker_reduce_sql([b"\0\0\0\2" + e[4:]], q)  # version 2


def _sections(dt):
    """(header ints, body) of a DataTable made by datatable()."""
    return list(struct.unpack(">13i", dt[:52])), dt[52:]


def _with_header(h, body):
    return struct.pack(">13i", *h) + body


def test_reduce_rejects_corrupted_tables():
    """Hand-corrupted server responses are rejected, never read outside their bytes."""
    names, types = ["column17", "count(*)", "avg(column6)"], ["INT", "LONG", "OBJECT"]
    good = datatable(names, types, [[5, 2, (10.0, 2)], [9, 1, (7.0, 1)]], _meta(3))
    q = parse_query("SELECT column17, COUNT(*), AVG(column6) FROM t GROUP BY column17")
    assert len(broker_reduce_sql([good], q)["resultTable"]["rows"]) == 2
    h, body = _sections(good)
    for k in range(5):  # a negative offset, then a negative length, for every section
        for field in (3 + 2 * k, 4 + 2 * k):
            bad = list(h)
            bad[field] = -8
            with pytest.raises(Exception):
                broker_reduce_sql([_with_header(bad, body)], q)
    bad = list(h)
    bad[9] = bad[10] = 0  # rows > 0 but no fixed-size section
    with pytest.raises(Exception):
        broker_reduce_sql([_with_header(bad, body)], q)
    bad = list(h)
    bad[1] = -1  # negative row count
    with pytest.raises(Exception):
        broker_reduce_sql([_with_header(bad, body)], q)
    # an AvgPair cell pointing before / past the variable-size data
    for off in (-16, 1 << 20):
        rows = bytearray(good)
        fixed_off = h[9]
        row_size = 4 + 8 + 8
        struct.pack_into(">i", rows, fixed_off + 12, off)  # first row's OBJECT offset
        with pytest.raises(Exception):
            broker_reduce_sql([bytes(rows)], q)
        _ = row_size


def test_reduce_double_keys_exact():
    """DOUBLE group keys that differ only past the 6th decimal stay distinct groups (keys compare by value)."""
    names, types = ["d", "count(*)"], ["DOUBLE", "LONG"]
    a = datatable(names, types, [[1e-7, 1], [2e-7, 2], [0.1 + 0.2, 3]], _meta(6))
    b = datatable(names, types, [[1e-7, 10], [0.3, 4], [-0.0, 5]], _meta(19))
    q = parse_query("SELECT d, COUNT(*) FROM t GROUP BY d ORDER BY d LIMIT 10")
    rows = broker_reduce_sql([a, b], q)["resultTable"]["rows"]
    assert rows == [[-0.0, 5], [1e-7, 11], [2e-7, 2], [0.3, 4], [0.1 + 0.2, 3]]


def test_reduce_reference_metadata_keys_and_nan():
    """Responses of a reference server carry metadata keys beyond the statistics (requestId, threadCpuTimeNs,
    traceInfo, ...; DataTable.java:90-110) -- decoded and skipped -- and a NaN aggregate is valid JSON."""
    names, types = ["column17", "sum(column6)"], ["INT", "DOUBLE"]
    meta = dict(_meta(4))
    dt = datatable(names, types, [[1, float("nan")], [2, 3.0]], meta)
    h, body = _sections(dt)
    # rebuild the metadata with extra reference keys appended
    extra = [(14, ">q", 123456789), (17, ">q", 42), (13, "s", "trace"), (8, ">i", 0), (9, ">q", -1)]
    md = struct.pack(">i", len(meta) + len(extra)) + b"".join(
        struct.pack(">i", META[k][0]) + struct.pack(">" + META[k][1], v) for k, v in meta.items())
    for ordinal, fmt, v in extra:
        md += struct.pack(">i", ordinal) + (_s(v) if fmt == "s" else struct.pack(fmt, v))
    end = max(h[3 + 2 * k] + h[4 + 2 * k] for k in range(5))
    dt2 = dt[:end] + struct.pack(">i", len(md)) + md
    q = parse_query("SELECT column17, SUM(column6) FROM t GROUP BY column17 ORDER BY column17")
    r = broker_reduce_sql([dt2], q)
    rows = r["resultTable"]["rows"]
    assert rows[1] == [2, 3.0]
    assert rows[0] == [1, "NaN"]  # Jackson's QUOTE_NON_NUMERIC_NUMBERS form: valid JSON
    assert r["numDocsScanned"] == 4
