"""Arrow IPC messages (ArrowUtils.serializeRecordBatch / ArrowSerializers stream writers,
FMT/vectorized/ArrowUtils.java:63-72, ArrowSerializers.java:128-167).

The reference hands its columns to Arrow's MessageSerializer (arrow-vector 15.0.0, absent here);
parity is anchored on the Arrow IPC format itself: pyarrow (an independent Arrow implementation)
must read our Schema message as the schema TypeInference builds, and our RecordBatch message as
the arrays of the same values.  CPU: schema messages.  GPU: record batches gathered on the device
(with device-computed null counts)."""
from __future__ import annotations

import struct

import numpy as np
import pyarrow as pa
import pytest

from fury_amd import types as T
from fury_amd.arrow import pa_type
from fury_amd.workloads import SCHEMAS, gen_columns


def _expected_schema(fields):
    return pa.schema([pa.field(f.name, pa_type(f), f.nullable) for f in fields])


def _all_schemas():
    from tests.test_device import _nested_fields
    out = dict(SCHEMAS)
    out["deep_nested"] = _nested_fields()
    return out


@pytest.mark.parametrize("name", sorted(list(SCHEMAS) + ["deep_nested"]))
def test_ipc_schema_message_reads_back(name):
    from fury_amd.encoder import RowEncoder, ipc_schema_message
    fields = _all_schemas()[name]
    msg = ipc_schema_message(RowEncoder(fields, device="cpu"))
    cont, meta = struct.unpack_from("<Ii", msg)
    assert cont == 0xFFFFFFFF and meta % 8 == 0 and len(msg) == 8 + meta
    got = pa.ipc.read_schema(pa.py_buffer(msg))
    want = _expected_schema(fields)
    assert got.equals(want), f"{got}\n!=\n{want}"


def test_ipc_schema_stream_with_no_batches():
    """Schema message + end-of-stream marker is a valid, empty IPC stream."""
    from fury_amd.encoder import IPC_EOS, RowEncoder, ipc_schema_message
    fields = SCHEMAS["mixed"]
    data = ipc_schema_message(RowEncoder(fields, device="cpu")) + IPC_EOS
    table = pa.ipc.open_stream(pa.py_buffer(data)).read_all()
    assert table.num_rows == 0 and table.schema.equals(_expected_schema(fields))


def _beans_and_fields(name, n, seed):
    from fury_amd.beans import columns_to_beans
    from tests.test_device import _nested_beans, _nested_fields
    if name == "deep_nested":
        from fury_amd.beans import beans_to_columns
        fields = _nested_fields()
        beans = _nested_beans(n, seed=seed)
        return fields, beans_to_columns(fields, beans), beans
    fields = SCHEMAS[name]
    host = gen_columns(name, fields, n, seed=seed)
    return fields, host, columns_to_beans(fields, host, n)


@pytest.mark.gpu
@pytest.mark.parametrize("name,n", [("struct100", 1000), ("mixed", 1234), ("nested", 999),
                                    ("narrow", 300), ("deep_nested", 257), ("mixed", 1),
                                    ("mixed", 0)])
def test_ipc_record_batch_reads_back(name, n):
    """Device-gathered RecordBatch message: pyarrow reads the stream back as the same values,
    null counts included."""
    import torch
    from fury_amd.encoder import ArrowWriter, Encoders, column_to_device
    dev = torch.device("cuda:0")
    fields, host, beans = _beans_and_fields(name, n, seed=13)
    enc = Encoders.bean(fields, device=dev)
    b = enc.encode_batch([column_to_device(c, dev) for c in host], n)
    w = ArrowWriter(enc)
    w.write(b)
    msg = w.finish_as_ipc_message()
    assert msg.numel() % 64 == 0
    data = w.finish_as_ipc_stream()
    table = pa.ipc.open_stream(pa.py_buffer(data)).read_all()
    assert table.schema.equals(_expected_schema(fields))
    assert table.num_rows == n
    for k, f in enumerate(fields):
        if f.type_id == T.DECIMAL:
            continue      # decimal values compared bytewise in test_device
        ref = pa.array([bb[f.name] for bb in beans], type=pa_type(f))
        col = table.column(k).combine_chunks()
        col.validate(full=True)
        assert col.equals(ref), f"{name}.{f.name}"
        assert col.null_count == ref.null_count, f"{name}.{f.name} null_count"


@pytest.mark.gpu
def test_ipc_record_batch_large_struct100():
    """2M Struct-100 rows (1.6 GB body): one message, body bytes == the decoded columns."""
    import torch
    from fury_amd.encoder import Encoders, ipc_record_batch_message
    from fury_amd.workloads import Column
    dev = torch.device("cuda:0")
    fields = SCHEMAS["struct100"]
    n = 2_000_000
    g = torch.Generator(device=dev).manual_seed(4)
    cols = [Column(values=torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device=dev,
                                        generator=g)) for _ in fields]
    enc = Encoders.bean(fields, device=dev)
    b = enc.encode_batch(cols, n)
    out = enc.decode_batch(b, validity=False)          # non-null fields: no validity buffers
    msg = ipc_record_batch_message(enc, out, n)
    meta = int(np.frombuffer(msg[:8].cpu().numpy().tobytes(), dtype="<i4")[1])
    body = msg[8 + meta:]
    per = n * 8                               # 64-aligned: 16e6 % 64 == 0; no validity buffers
    assert body.numel() == 100 * per
    for k in (0, 1, 57, 99):
        assert torch.equal(body[k * per:(k + 1) * per], cols[k].values.view(torch.uint8))
