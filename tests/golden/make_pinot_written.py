"""Copy the Pinot-written segment files the reference's own tests hold into tests/golden/pinot_written/
(data fixtures, byte for byte), with the expected values those tests assert (expected.json).

Sources (paths relative to the reference checkout):
* pinot-core/src/test/resources/data/fixedByteSVRDoubles.v1, fixedByteCompressed.v2, fixedByteRaw.v2:
  raw DOUBLE forward indexes written by FixedByteChunkForwardIndexWriter v1 (SNAPPY) / v2 (SNAPPY,
  PASS_THROUGH); FixedByteChunkSVForwardIndexTest.java:330-349 asserts value(doc i) == i + start.
* pinot-core/src/test/resources/data/paddingOld.tar.gz: a V1 segment directory (5 docs, dictionary-
  encoded INT / LONG / FLOAT / STRING columns; README: created with the pre-08/2016 '%' padding).
* pinot-integration-tests/src/test/resources/legacy/legacyRawInverted_OFFLINE_0.tar.gz and
  legacyRawInverted_v3_OFFLINE_0.tar.gz: a raw STRING column (VarByteChunkForwardIndexWriterV4,
  LZ4_LENGTH_PREFIXED) of 600 docs in V1 files and in V3 columns.psf + index_map;
  LegacyRawValueInvertedIndexMigrationIntegrationTest.java:93-104,196-243,300-310 asserts the counts.

    python tests/golden/make_pinot_written.py [/root/reference]
"""
import json
import os
import shutil
import sys
import tarfile

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "pinot_written")


def main(ref="/root/reference"):
    os.makedirs(OUT, exist_ok=True)
    data = os.path.join(ref, "pinot-core/src/test/resources/data")
    for f in ("fixedByteSVRDoubles.v1", "fixedByteCompressed.v2", "fixedByteRaw.v2"):
        shutil.copyfile(os.path.join(data, f), os.path.join(OUT, f))
    tars = [(os.path.join(data, "paddingOld.tar.gz"), "paddingOld"),
            (os.path.join(ref, "pinot-integration-tests/src/test/resources/legacy/legacyRawInverted_OFFLINE_0.tar.gz"),
             "legacyRawInverted_v1"),
            (os.path.join(ref, "pinot-integration-tests/src/test/resources/legacy/legacyRawInverted_v3_OFFLINE_0.tar.gz"),
             "legacyRawInverted_v3")]
    for tgz, name in tars:
        dst = os.path.join(OUT, name)
        shutil.rmtree(dst, ignore_errors=True)
        with tarfile.open(tgz) as t:
            for m in t.getmembers():
                if not m.isfile():
                    continue
                parts = m.name.split("/")[1:]  # drop the segment directory name
                if "v3" in parts and name.endswith("_v1"):
                    continue
                if name.endswith("_v3") and "v3" not in parts and not any(p.endswith(".properties") for p in parts):
                    continue
                target = os.path.join(dst, *parts)
                # members of the (untrusted) archive may only land inside this fixture's directory
                if os.path.isabs(m.name) or ".." in parts or \
                        not os.path.realpath(target).startswith(os.path.realpath(dst) + os.sep):
                    raise ValueError(f"tar member {m.name!r} escapes {dst}")
                os.makedirs(os.path.dirname(target), exist_ok=True)
                with t.extractfile(m) as src, open(target, "wb") as o:
                    o.write(src.read())
    expected = {
        "raw_doubles": {  # FixedByteChunkSVForwardIndexTest.testBackwardCompatibilityV1 / V2
            "fixedByteSVRDoubles.v1": {"num_docs": 10009, "start": 0.0},
            "fixedByteCompressed.v2": {"num_docs": 2000, "start": 100.2356},
            "fixedByteRaw.v2": {"num_docs": 2000, "start": 100.2356},
        },
        "legacy_raw_string": {  # LegacyRawValueInvertedIndexMigrationIntegrationTest
            "column": "category", "num_docs": 600,
            "counts": {"alpha": 300, "beta": 100, "gamma": 100, "delta": 100},
            "in_alpha_beta": 400, "not_eq_alpha": 300,
        },
        "padding_old": {  # metadata.properties of the segment (cardinality, bitsPerElement, time range)
            "num_docs": 5, "time_column": "outgoingName1", "start_time": 246, "end_time": 902,
            "cardinality": {"age": 5, "name": 2, "outgoingName1": 5, "percent": 5},
            "bits": {"age": 3, "name": 1, "outgoingName1": 3, "percent": 3},
        },
    }
    with open(os.path.join(OUT, "expected.json"), "w") as f:
        json.dump(expected, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
