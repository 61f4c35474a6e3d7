"""Extracts the aggregation KATs of InterSegmentAggregationSingleValueQueriesTest (SUM/COUNT/MIN/MAX/AVG) into
tests/golden/kat_inter_agg.json.  Reads the reference test source as text (expected numbers only; nothing of the
reference is run).  Run once in the build container:  python tests/golden/make_golden_inter_agg.py"""
import json
import os
import re

REF = "/root/reference/pinot-core/src/test/java/org/apache/pinot/queries/InterSegmentAggregationSingleValueQueriesTest.java"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat_inter_agg.json")
TESTS = ["testCount", "testMax", "testMin", "testSum", "testAvg"]
VARIANTS = [("no_filter", False, False), ("filter", True, False), ("group_by", False, True),
            ("filter_group_by", True, True)]


def main():
    src = open(REF).read()
    lines = src.splitlines()
    out = {"_source": "pinot-core/src/test/java/org/apache/pinot/queries/InterSegmentAggregationSingleValueQueriesTest.java",
           "_note": "4 segments (the test_data-sv.avro segment on 2 servers x 2 segments, BaseQueriesTest.java:209-242); "
                    "group_by variants append ' group by column9' and the value is the top group after PQL trimming "
                    "(descending, ascending for MIN); stats = numDocsScanned, numEntriesScannedInFilter, "
                    "numEntriesScannedPostFilter, numTotalDocs (inFilter depends on the reference's inverted/sorted "
                    "indexes when filtered)",
           "group_by_column": "column9", "cases": []}
    for t in TESTS:
        start = next(i for i, l in enumerate(lines) if re.search(r"public void %s\(\)" % t, l))
        body = []
        for l in lines[start + 1:]:
            if re.search(r"public void test", l):
                break
            body.append(l)
        text = "\n".join(body)
        query = re.search(r'String query = "([^"]+)";', text).group(1)
        calls = re.findall(r"testInterSegmentAggregationResult\(brokerResponse,\s*(\d+)L,\s*(\d+)L,\s*(\d+)L,\s*(\d+)L,"
                           r"\s*new String\[\]\{([^}]*)\}\)", text, re.S)
        assert len(calls) == 4, (t, len(calls))
        for (name, flt, gb), (docs, inf, post, total, vals) in zip(VARIANTS, calls):
            line = start + 1 + next(i for i, l in enumerate(body) if "testInterSegmentAggregationResult" in l) + 1
            out["cases"].append({"test": t, "variant": name, "query": query, "filter": flt, "group_by": gb,
                                 "stats": [int(docs), int(inf), int(post), int(total)],
                                 "values": [v.strip().strip('"') for v in vals.split(",")],
                                 "_cite": "InterSegmentAggregationSingleValueQueriesTest.java:%d" % line})
    json.dump(out, open(OUT, "w"), indent=1)
    print("wrote %d cases to %s" % (len(out["cases"]), OUT))


if __name__ == "__main__":
    main()
