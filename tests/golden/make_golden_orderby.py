"""Extracts the expected result tables of InterSegmentOrderBySingleValueQueriesTest.orderBySQLResultTableProvider
(pinot-core/src/test/java/org/apache/pinot/queries/InterSegmentOrderBySingleValueQueriesTest.java) as data:
query, rows (in order), data schema and execution statistics, for the queries the GPU path runs (SUM / COUNT / MIN /
MAX / AVG over identifier group-by columns; cases with transform expressions or other aggregation functions are
skipped).  The provider builds its lists with a handful of statements (literal lists, copy, reverse, subList),
replayed here; nothing of the reference runs.

    python tests/golden/make_golden_orderby.py /root/reference > tests/golden/kat_orderby_sql.json
"""
import json
import re
import sys

SRC = "pinot-core/src/test/java/org/apache/pinot/queries/InterSegmentOrderBySingleValueQueriesTest.java"


def java_values(text):
    """Literal list inside `new Object[]{...}`: strings, doubles, longs, ints."""
    out = []
    for m in re.finditer(r'"((?:[^"\\]|\\.)*)"|(-?\d+(?:\.\d+)?(?:[eE][+-]?\d+)?)([Ll])?', text):
        if m.group(1) is not None:
            out.append(m.group(1).replace("\\t", "\t").replace('\\"', '"'))
        elif m.group(3):
            out.append(int(m.group(2)))
        elif "." in m.group(2) or "e" in m.group(2).lower():
            out.append(float(m.group(2)))
        else:
            out.append(int(m.group(2)))
    return out


def main(root):
    src = open(root + "/" + SRC).read()
    start = src.index("public Object[][] orderBySQLResultTableProvider()")
    end = src.index("return data.toArray(", start)
    body = src[start:end]
    body = re.sub(r"//[^\n]*", "", body)
    body = re.sub(r'"\s*\+\s*"', "", body)  # Java string concatenation across lines
    state = {"numDocsScanned": 120000, "numEntriesScannedInFilter": 0, "numTotalDocs": 120000}
    results, schema, query, cases = [], None, None, []
    for stmt in body.split(";"):
        st = " ".join(stmt.split())
        m = re.search(r'query\s*=\s*"((?:[^"\\]|\\.)*)"', stmt)  # the raw statement keeps the query's whitespace
        if m:
            query = m.group(1).replace("\\t", "\t")
            continue
        if re.search(r"results = Lists ?\.newArrayList\(results\)", st):
            results = list(results)
            continue
        if "Collections.reverse(results)" in st:
            results.reverse()
            continue
        m = re.search(r"results = results\.subList\((\d+), (\d+)\)", st)
        if m:
            results = results[int(m.group(1)):int(m.group(2))]
            continue
        if re.search(r"results = new ArrayList<>\(0\)", st):
            results = []
            continue
        m = re.match(r"results\.add\(new Object\[\]\{([^}]*)\}\)$", st)
        if m:
            results.append(java_values(m.group(1)))
            continue
        if re.search(r"results = Lists ?\.newArrayList\(new Object", st):
            results = [java_values(b) for b in re.findall(r"new Object\[\]\{([^}]*)\}", st)]
            continue
        m = re.search(r"dataSchema = new DataSchema\(new String\[\]\{([^}]*)\}, new DataSchema\.ColumnDataType\[\]\{([^}]*)\}", st)
        if m:
            schema = {"columnNames": java_values(m.group(1)),
                      "columnDataTypes": re.findall(r"ColumnDataType\.([A-Z_]+)", m.group(2))}
            continue
        m = re.search(r"(numDocsScanned|numEntriesScannedInFilter|numEntriesScannedPostFilter|numTotalDocs) = (\d+)", st)
        if m:
            state[m.group(1)] = int(m.group(2))
            continue
        if st.startswith("data.add("):
            cases.append({"query": query, "rows": results, "dataSchema": schema,
                          "stats": [state["numDocsScanned"], state["numEntriesScannedInFilter"],
                                    state["numEntriesScannedPostFilter"], state["numTotalDocs"]]})
    ok = re.compile(r"^(sum|count|min|max|avg)\(", re.I)
    keep = []
    for c in cases:
        names = c["dataSchema"]["columnNames"]
        q = c["query"]
        funcs = re.findall(r"([A-Za-z]+)\(", q)
        if any(f.lower() not in ("sum", "count", "min", "max", "avg") for f in funcs):
            continue
        if any("(" in n and not ok.match(n) for n in names):
            continue
        keep.append(c)
    json.dump({"_source": SRC + " orderBySQLResultTableProvider (data extracted by tests/golden/make_golden_orderby.py); "
                                "4 segments = the KAT segment on 2 servers x 2 segments (BaseQueriesTest.java:209-242)",
               "cases": keep}, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
