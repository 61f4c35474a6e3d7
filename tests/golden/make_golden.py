"""Regenerates the golden input fixtures under tests/golden/ from files the reference's own tests hold.

    python tests/golden/make_golden.py /root/reference

Outputs (data only — no reference source is copied):
  sv_columns.npz          the 11 columns BaseSingleValueQueriesTest builds its segment from
                          (pinot-core/src/test/java/org/apache/pinot/queries/BaseSingleValueQueriesTest.java:49-115),
                          decoded from pinot-core/src/test/resources/data/test_data-sv.avro (30000 records).
                          INT columns -> int32 arrays; STRING columns -> <name>__blob (uint8) + <name>__off (int64).
  padding_segments.json   dictionary / forward-index bytes of the real Pinot-written v1 segments in
                          pinot-core/src/test/resources/data/padding{Old,Null,Percent}.tar.gz (codec golden vectors).
The expected outputs (kat_sv.json) are transcribed by hand from the reference tests, with file:line citations.
"""
import io
import json
import os
import sys
import tarfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from avro_reader import read_avro  # noqa: E402

INT_COLS = ["column1", "column3", "column6", "column7", "column9", "column17", "column18", "daysSinceEpoch"]
STR_COLS = ["column5", "column11", "column12"]


def main(ref_root):
    here = os.path.dirname(os.path.abspath(__file__))
    data_dir = os.path.join(ref_root, "pinot-core", "src", "test", "resources", "data")
    names, rows = read_avro(os.path.join(data_dir, "test_data-sv.avro"))
    out = {}
    for c in INT_COLS:
        i = names.index(c)
        out[c] = np.array([r[i] for r in rows], dtype=np.int32)
    for c in STR_COLS:
        i = names.index(c)
        enc = [r[i].encode("utf-8") for r in rows]
        off = np.zeros(len(enc) + 1, dtype=np.int64)
        off[1:] = np.cumsum([len(e) for e in enc])
        out[c + "__blob"] = np.frombuffer(b"".join(enc), dtype=np.uint8)
        out[c + "__off"] = off
    np.savez_compressed(os.path.join(here, "sv_columns.npz"), **out)

    segs = {}
    for name in ("paddingOld", "paddingNull", "paddingPercent"):
        with tarfile.open(os.path.join(data_dir, name + ".tar.gz")) as tf:
            files = {}
            for m in tf.getmembers():
                if m.isfile():
                    files[os.path.basename(m.name)] = tf.extractfile(m).read()
        props = {}
        for line in files["metadata.properties"].decode().splitlines():
            if "=" in line:
                k, v = line.split("=", 1)
                props[k.strip()] = v.strip()
        cols = {}
        for col in ("age", "name", "outgoingName1", "percent"):
            p = "column.%s." % col
            cols[col] = {
                "dataType": props[p + "dataType"],
                "cardinality": int(props[p + "cardinality"]),
                "bitsPerElement": int(props[p + "bitsPerElement"]),
                "lengthOfEachEntry": int(props[p + "lengthOfEachEntry"]),
                "dict_hex": files[col + ".dict"].hex(),
                "fwd_hex": files[col + ".sv.unsorted.fwd"].hex(),
            }
        segs[name] = {
            "paddingCharacter": props.get("segment.padding.character", "%"),  # absent in pre-0.3 segments: legacy %
            "totalDocs": int(props["segment.total.docs"]),
            "columns": cols,
        }
    with open(os.path.join(here, "padding_segments.json"), "w") as f:
        json.dump(segs, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
