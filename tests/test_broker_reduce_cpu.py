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
