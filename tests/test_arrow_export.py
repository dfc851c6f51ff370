"""CPU: the host Arrow export (fury_amd/arrow.py) over columns in the layout the device decode
produces — here produced by the oracle's decode — equals pyarrow arrays built from the values,
for flat and nested schemas (struct, map, list of lists / structs / strings)."""
import pyarrow as pa
import pytest

from fury_amd.arrow import columns_to_record_batch, pa_type
from fury_amd.beans import beans_to_columns, columns_to_beans
from fury_amd.workloads import SCHEMAS, gen_columns


def _check(oracle, fields, beans):
    n = len(beans)
    host = beans_to_columns(fields, beans)
    rows, offs = oracle.encode(fields, host, n)
    dec = oracle.decode(fields, rows, offs, n)
    assert columns_to_beans(fields, dec, n) == beans
    rb = columns_to_record_batch(fields, dec, n)
    rb.validate(full=True)
    for k, f in enumerate(fields):
        assert rb.column(k).equals(pa.array([b[f.name] for b in beans], type=pa_type(f))), f.name


def test_nested_export(oracle):
    from tests.test_device import _nested_beans, _nested_fields
    _check(oracle, _nested_fields(), _nested_beans(400, seed=3))


@pytest.mark.parametrize("name", ["mixed", "nested", "narrow", "foo"])
def test_named_schema_export(oracle, name):
    fields = SCHEMAS[name]
    if name == "foo":
        beans = [{"f1": i, "f2": None if i % 3 == 0 else f"s{i}", "f3": [f"x{j}" for j in range(i % 4)],
                  "f4": [(f"k{j}", j) for j in range(i % 3)] if i % 5 else None,
                  "f5": None if i % 7 == 0 else {"f1": i, "f2": "b"}} for i in range(60)]
    else:
        n = 200
        beans = columns_to_beans(fields, gen_columns(name, fields, n, seed=4), n)
        fields = [f for f in fields if f.type_id != 23]     # decimal values: bytes vs Decimal
        beans = [{f.name: b[f.name] for f in fields} for b in beans]
    _check(oracle, fields, beans)
