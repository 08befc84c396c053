#!/usr/bin/env python3
"""Generate the committed golden fixtures from the reference's own test data.

Runs ONLY in the build container (it reads /root/reference, which does not exist on the
GPU box).  Outputs (committed, small):

  tests/golden/test_data_sv.npz   -- the 11 columns of pinot-core/src/test/resources/data/test_data-sv.avro
                                     that BaseSingleValueQueriesTest.java:95-105 puts into its segment,
                                     with Pinot's default-null substitution applied.
  tests/golden/simple_data_200001.npz -- simpleData200001.avro (QueryExecutorTest.java:159-192).
  tests/golden/padding_null/*     -- raw bytes of the Pinot-written v1 segment paddingNull.tar.gz
                                     (real on-disk forward index + dictionary bytes).

The expected answers themselves live in tests/golden/expected.json; they are transcribed
(by value, not code) from the reference tests cited there.

The Avro reader below implements the published Avro 1.x object-container format for the
subset these files use (codec "null", record of ["null", primitive] unions).
"""
import io
import json
import os
import sys
import tarfile

import numpy as np

REF = "/root/reference"
DATA = os.path.join(REF, "pinot-core/src/test/resources/data")
OUT = os.path.dirname(os.path.abspath(__file__))


def _read_long(b: io.BytesIO) -> int:
    shift = 0
    acc = 0
    while True:
        c = b.read(1)
        if not c:
            raise EOFError
        c = c[0]
        acc |= (c & 0x7F) << shift
        if not (c & 0x80):
            break
        shift += 7
    return (acc >> 1) ^ -(acc & 1)


def _read_bytes(b):
    n = _read_long(b)
    return b.read(n)


def read_avro(path):
    """Return (schema_fields, list_of_rows) for a codec-null Avro container file."""
    with open(path, "rb") as f:
        data = f.read()
    b = io.BytesIO(data)
    assert b.read(4) == b"Obj\x01"
    meta = {}
    while True:
        n = _read_long(b)
        if n == 0:
            break
        if n < 0:
            _read_long(b)
            n = -n
        for _ in range(n):
            k = _read_bytes(b).decode()
            meta[k] = _read_bytes(b)
    sync = b.read(16)
    codec = meta.get("avro.codec", b"null").decode()
    assert codec == "null", codec
    schema = json.loads(meta["avro.schema"])
    fields = schema["fields"]

    def read_value(t, bb):
        if isinstance(t, list):
            idx = _read_long(bb)
            return read_value(t[idx], bb)
        if t == "null":
            return None
        if t in ("int", "long"):
            return _read_long(bb)
        if t == "string":
            return _read_bytes(bb).decode("utf-8")
        if t == "boolean":
            return bb.read(1)[0] != 0
        if t == "double":
            return float(np.frombuffer(bb.read(8), "<f8")[0])
        if t == "float":
            return float(np.frombuffer(bb.read(4), "<f4")[0])
        raise NotImplementedError(t)

    rows = []
    while b.tell() < len(data):
        count = _read_long(b)
        size = _read_long(b)
        blk = io.BytesIO(b.read(size))
        for _ in range(count):
            rows.append({f["name"]: read_value(f["type"], blk) for f in fields})
        assert b.read(16) == sync
    return fields, rows


# Pinot default null values (pinot-spi FieldSpec.java): dimension/time INT -> Integer.MIN_VALUE,
# metric INT -> 0, dimension STRING -> "null".
INT_MIN = -(2 ** 31)


def make_test_data_sv():
    fields, rows = read_avro(os.path.join(DATA, "test_data-sv.avro"))
    # BaseSingleValueQueriesTest.java:95-105 schema
    spec = {
        "column1": ("INT", "METRIC"), "column3": ("INT", "METRIC"), "column5": ("STRING", "DIMENSION"),
        "column6": ("INT", "DIMENSION"), "column7": ("INT", "DIMENSION"), "column9": ("INT", "DIMENSION"),
        "column11": ("STRING", "DIMENSION"), "column12": ("STRING", "DIMENSION"),
        "column17": ("INT", "METRIC"), "column18": ("INT", "METRIC"), "daysSinceEpoch": ("INT", "TIME"),
    }
    cols = {}
    nulls = {}
    for name, (dt, ft) in spec.items():
        vals = [r[name] for r in rows]
        nulls[name] = sum(v is None for v in vals)
        if dt == "INT":
            dflt = 0 if ft == "METRIC" else INT_MIN
            cols[name] = np.array([dflt if v is None else v for v in vals], dtype=np.int32)
        else:
            cols[name] = np.array(["null" if v is None else v for v in vals], dtype=object)
    out = {k: (v if v.dtype != object else v.astype("U")) for k, v in cols.items()}
    np.savez_compressed(os.path.join(OUT, "test_data_sv.npz"), **out)
    print("test_data_sv: rows", len(rows), "nulls", {k: v for k, v in nulls.items() if v})


def make_simple_data():
    fields, rows = read_avro(os.path.join(DATA, "simpleData200001.avro"))
    names = [f["name"] for f in fields]
    out = {}
    for n in names:
        vals = [r[n] for r in rows]
        t = fields[names.index(n)]["type"]
        t = [x for x in t if x != "null"][0] if isinstance(t, list) else t
        if t in ("int", "long"):
            out[n] = np.array(vals, dtype=np.int64 if t == "long" else np.int32)
        elif t in ("double", "float"):
            out[n] = np.array(vals, dtype=np.float64)
        else:
            out[n] = np.array(vals).astype("U")
    np.savez_compressed(os.path.join(OUT, "simple_data_200001.npz"), **out)
    print("simpleData200001: rows", len(rows), "fields", [(f["name"], f["type"]) for f in fields])


def extract_padding():
    d = os.path.join(OUT, "padding_null")
    os.makedirs(d, exist_ok=True)
    with tarfile.open(os.path.join(DATA, "paddingNull.tar.gz")) as t:
        for m in t.getmembers():
            if m.isfile():
                data = t.extractfile(m).read()
                with open(os.path.join(d, os.path.basename(m.name)), "wb") as f:
                    f.write(data)


if __name__ == "__main__":
    if not os.path.isdir(DATA):
        sys.exit("reference data not present; fixtures are already committed")
    make_test_data_sv()
    make_simple_data()
    extract_padding()
