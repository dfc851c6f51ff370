"""Generates the golden fixtures under tests/golden/.  Run in the build container only:

    python tests/golden/make_golden.py

1. schema_hashes.json — schema hashes computed by the REFERENCE's own Python function
   ``compute_schema_hash`` / ``_compute_hash`` (python/pyfury/format/infer.py:160-190), loaded from
   /root/reference (read-only) by extracting just those two function definitions: importing the
   ``pyfury`` package raises ModuleNotFoundError here (its Cython extensions are unbuilt), an
   ordinary error.  The schemas are built with pyarrow, whose type ids are the ids the Java side
   hashes (java/fury-format/.../type/ArrowType.java:25-148).
2. known_answers.json — answers stated in the reference's own tests (copied as numbers/strings
   with their file:line), plus the hand-derived Bar row of SURVEY.md §8(c).
3. *.npz — seeded input columns + expected rows/offsets produced by the oracle restatement
   (oracle/row_oracle.c); regression fixtures for the device path (np.load allow_pickle=False).

Nothing here ships to, or is read on, the GPU box except the generated data files.
"""
from __future__ import annotations

import ast
import json
import os
import sys

import numpy as np
import pyarrow as pa

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
GOLDEN = os.path.dirname(os.path.abspath(__file__))
REF_INFER = "/root/reference/python/pyfury/format/infer.py"

from oracle import oracle as O  # noqa: E402
from fury_amd.types import schema_spec as fields_to_spec  # noqa: E402
from fury_amd.workloads import SCHEMAS, docs_struct_values, gen_columns  # noqa: E402


def load_reference_hash():
    src = open(REF_INFER).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef)
            and n.name in ("compute_schema_hash", "_compute_hash")]
    assert len(keep) == 2, "reference infer.py changed shape"
    mod = ast.Module(body=keep, type_ignores=[])
    ns = {"pa": pa}
    exec(compile(mod, REF_INFER, "exec"), ns)
    return ns["compute_schema_hash"]


def to_pa_type(f: O.F):
    t = f.type_id
    simple = {O.BOOL: pa.bool_(), O.INT8: pa.int8(), O.INT16: pa.int16(), O.INT32: pa.int32(),
              O.INT64: pa.int64(), O.FLOAT32: pa.float32(), O.FLOAT64: pa.float64(),
              O.STRING: pa.utf8(), O.BINARY: pa.binary(), O.DATE32: pa.date32(),
              O.TIMESTAMP: pa.timestamp("us"), O.DECIMAL: pa.decimal128(38, 18)}
    if t in simple:
        return simple[t]
    if t == O.LIST:
        return pa.list_(pa.field(f.children[0].name, to_pa_type(f.children[0]),
                                 f.children[0].nullable))
    if t == O.STRUCT:
        return pa.struct([pa.field(c.name, to_pa_type(c), c.nullable) for c in f.children])
    if t == O.MAP:
        return pa.map_(to_pa_type(f.children[0]), to_pa_type(f.children[1]))
    raise ValueError(t)


def main():
    ref_hash = load_reference_hash()
    hashes = {}
    for name, fields in SCHEMAS.items():
        schema = pa.schema([pa.field(f.name, to_pa_type(f), f.nullable) for f in fields])
        hashes[name] = {"fields": fields_to_spec(fields), "hash": int(ref_hash(schema))}
    with open(os.path.join(GOLDEN, "schema_hashes.json"), "w") as fh:
        json.dump({"source": "python/pyfury/format/infer.py:160-190 (reference, executed here)",
                   "schemas": hashes}, fh, indent=1)

    known = {
        "array_encoder_list_bar_bytes": {
            "value": 224, "ref": "java/fury-format/src/test/java/org/apache/fury/format/"
                                 "encoder/ArrayEncoderTest.java:56"},
        "array_encoder_nested_list_bar_bytes": {
            "value": 1576, "ref": "java/fury-format/src/test/java/org/apache/fury/format/"
                                  "encoder/ArrayEncoderTest.java:90"},
        "array_encoder_list_list_map_bytes": {
            "value": 10824, "ref": "java/fury-format/src/test/java/org/apache/fury/format/"
                                   "encoder/ArrayEncoderTest.java:124"},
        "cpp_row_to_string": {
            "value": "{f1=str, f2=1, f3=[2, 2], f4=Map([key1, key2], [1, 1]), "
                     "f5={n1=str, n2=1}}",
            "ref": "cpp/fury/row/row_test.cc:96-98"},
        "bar_row_hex": {
            "value": "0000000000000000" "0100000000000000" "0300000018000000" "7374720000000000",
            "ref": "SURVEY.md §8(c): Bar{f1=1,f2=\"str\"}, layout per "
                   "java/fury-format/.../writer/BinaryWriter.java:110-114,187-194"},
        "docs_struct_encode_bytes": {
            "value": 856, "ref": "BASELINE.json configs[0]; 8 hash + 16 bitmap + 104*8"},
    }
    with open(os.path.join(GOLDEN, "known_answers.json"), "w") as fh:
        json.dump(known, fh, indent=1)

    # Seeded regression fixtures (small) from the oracle restatement.
    for name, nrows in (("struct100", 64), ("mixed", 257), ("nested", 300),
                        ("narrow", 130), ("docs_struct", 1)):
        fields = SCHEMAS[name]
        if name == "docs_struct":
            cols = docs_struct_values(fields)
        else:
            cols = gen_columns(name, fields, nrows, seed=1234, start=0)
        rows, offs = O.encode(fields, cols, nrows)
        arrays = {"rows": rows, "row_offsets": offs}
        for k, c in enumerate(cols):
            for part in ("values", "validity", "offsets"):
                a = getattr(c, part)
                if a is not None:
                    arrays[f"c{k}_{part}"] = a
            if c.child:
                for part in ("values", "validity", "offsets"):
                    a = getattr(c.child[0], part)
                    if a is not None:
                        arrays[f"c{k}_child_{part}"] = a
        np.savez_compressed(os.path.join(GOLDEN, f"{name}.npz"), **arrays)
    print("golden fixtures written to", GOLDEN)


if __name__ == "__main__":
    main()
