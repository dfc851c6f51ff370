"""Bounds-checked decode (GPU): a row whose slot, array or map header points outside the batch's row
bytes fails the way the reference fails -- IndexOutOfBoundsException from MemoryBuffer's bounds
checks (fury-core memory/MemoryBuffer.java:2500-2519 via UnsafeTrait.getBuffer / getBinary,
format/row/binary/UnsafeTrait.java:44-51,118-129; BinaryArray.pointTo's header read,
BinaryArray.java:69-78) and UnsupportedOperationException for map key / value arrays of different
lengths (BinaryMap.java:62-77) -- and nothing outside the batch is read: the decoded columns equal
the oracle's decode of the same rows with the offending value set null, so bytes past the batch
(guard bytes 0xAB) never reach an output.  A slot pointing at another row's bytes inside the batch
is legal in the reference (it reads the shared buffer) and decodes to the oracle's result.
Marked gpu."""
from __future__ import annotations

import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from fury_amd import types as T  # noqa: E402
from fury_amd.workloads import SCHEMAS, gen_columns  # noqa: E402
from tests.helpers import assert_columns_equal  # noqa: E402

GUARD = 4096


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda:0")


def _wide_fields(ncols):
    kinds = [T.INT64, T.STRING, T.FLOAT64, T.INT32, T.BINARY]
    out = []
    for k in range(ncols):
        t = kinds[k % len(kinds)]
        out.append(T.field(f"c{k:03d}", t))
    out[-1] = T.array_field(f"c{ncols - 1:03d}", T.INT64)
    return out


def _bm(n):
    return ((n + 63) // 64) * 8


def _encode(oracle, fields, n, seed, dev, **knobs):
    from fury_amd.encoder import Encoders, column_to_device
    host = gen_columns("bounds", fields, n, seed=seed, **knobs)
    enc = Encoders.bean(fields, device=dev)
    rows, offs = oracle.encode(fields, host, n)
    assert offs is not None
    return enc, host, rows.copy(), np.asarray(offs, dtype=np.int64).copy()


def _batch(enc, rows, offs, n, dev):
    """Device rows followed by GUARD bytes of 0xAB in the same allocation (the batch ends at
    offs[n])."""
    from fury_amd.encoder import RowBatch
    buf = np.full(len(rows) + GUARD, 0xAB, np.uint8)
    buf[:len(rows)] = rows
    t = torch.from_numpy(buf).to(dev)
    return RowBatch(t[:len(rows)], torch.from_numpy(offs).to(dev), n, enc.schema_hash)


def _slot_at(fields, rows, offs, i, k):
    p = int(offs[i]) + _bm(len(fields)) + 8 * k
    return p, struct.unpack_from("<q", rows, p)[0]


def _is_null(fields, rows, offs, i, k):
    return (rows[int(offs[i]) + (k >> 3)] >> (k & 7)) & 1


def _victim(fields, rows, offs, n, kinds):
    """A row in the middle of the batch and a non-null field of one of the type ids `kinds`."""
    for i in range(n // 2, n):
        for k, f in enumerate(fields):
            if f.type_id in kinds and not _is_null(fields, rows, offs, i, k):
                return i, k
    raise AssertionError("no victim")


def _set_null(fields, rows, offs, i, k):
    out = rows.copy()
    out[int(offs[i]) + (k >> 3)] |= 1 << (k & 7)
    return out


def _corrupt(fields, rows, offs, n, i, k, how):
    out = rows.copy()
    p, slot = _slot_at(fields, out, offs, i, k)
    rel, size = slot >> 32, slot & 0xFFFFFFFF
    total = int(offs[n])
    base = int(offs[i])
    if how == "offset_past_end":
        rel = total - base + 8
    elif how == "size_past_end":
        size = total - (base + rel) + 1
    elif how == "negative_size":
        size = 0x80000005
    elif how == "negative_offset":
        rel = -(base + 16)
    elif how == "huge_list_count":
        struct.pack_into("<q", out, base + rel, 1 << 30)
        return out
    struct.pack_into("<Q", out, p, ((rel & 0xFFFFFFFF) << 32) | (size & 0xFFFFFFFF))
    return out


FLAT = {
    "mixed": (lambda: SCHEMAS["mixed"], {T.STRING}),          # register-staged decode (<= 16)
    "wide33": (lambda: _wide_fields(33), {T.STRING, T.BINARY, T.LIST}),   # 17-256-field kernel
    "c4": (lambda: SCHEMAS["nested"], {T.LIST}),              # LIST of int64, register-staged
}


@pytest.mark.parametrize("schema", list(FLAT))
@pytest.mark.parametrize("how", ["offset_past_end", "size_past_end", "negative_size",
                                 "negative_offset", "huge_list_count"])
def test_flat_decode_out_of_bounds(oracle, dev, schema, how):
    from fury_amd.encoder import IndexOutOfBoundsException, column_to_host
    make, kinds = FLAT[schema]
    fields = make()
    if how == "huge_list_count":
        kinds = {T.LIST}
    elif how in ("size_past_end", "negative_size"):
        kinds = kinds - {T.LIST}          # a list's slot size is not read (BinaryArray.pointTo)
    if not any(f.type_id in kinds for f in fields):
        pytest.skip("schema has no such field")
    n = 3001
    enc, host, rows, offs = _encode(oracle, fields, n, 11, dev, null_pct=10, str_max=30,
                                    list_max=9)
    i, k = _victim(fields, rows, offs, n, kinds)
    bad = _corrupt(fields, rows, offs, n, i, k, how)
    batch = _batch(enc, bad, offs, n, dev)
    with pytest.raises(IndexOutOfBoundsException, match=f"row {i} "):
        enc.decode_batch(batch)
    # columns decoded without the check's exception: the oracle's columns with the value null
    cols = enc._decode(batch, True, False, None, None, "bound")
    with pytest.raises(IndexOutOfBoundsException):
        enc.device_status()
    want = _set_null(fields, rows, offs, i, k)
    ref = oracle.decode(fields, want, offs, n)
    assert_columns_equal(fields, [column_to_host(c) for c in cols], ref, n)
    # ArrowWriter path raises too; then the error state is clear and the intact rows decode
    from fury_amd.encoder import ArrowWriter
    with pytest.raises(IndexOutOfBoundsException):
        ArrowWriter(enc).write(batch)
    good = [column_to_host(c) for c in enc.decode_batch(_batch(enc, rows, offs, n, dev))]
    assert_columns_equal(fields, good, oracle.decode(fields, rows, offs, n), n)


def test_flat_decode_row_offset_out_of_bounds(oracle, dev):
    from fury_amd.encoder import IndexOutOfBoundsException
    fields = SCHEMAS["mixed"]
    n = 2000
    enc, host, rows, offs = _encode(oracle, fields, n, 3, dev, null_pct=10, str_max=30)
    bad_offs = offs.copy()
    bad_offs[777] = int(offs[n]) + 64
    with pytest.raises(IndexOutOfBoundsException, match="row 777 "):
        enc.decode_batch(_batch(enc, rows, bad_offs, n, dev))
    bad_offs = offs.copy()
    bad_offs[5] = -8
    with pytest.raises(IndexOutOfBoundsException, match="row 5 "):
        enc.decode_batch(_batch(enc, rows, bad_offs, n, dev))


@pytest.mark.parametrize("schema", ["mixed", "wide33"])
def test_slot_into_another_row_decodes_like_reference(oracle, dev, schema):
    """A string slot pointing at another row's string (inside the batch) is legal in the
    reference: the decode returns that string, as the oracle does."""
    from fury_amd.encoder import column_to_host
    fields = FLAT[schema][0]()
    n = 4000
    enc, host, rows, offs = _encode(oracle, fields, n, 5, dev, null_pct=10, str_max=30)
    i, k = _victim(fields, rows, offs, n, {T.STRING})
    j = None
    for cand in range(10, n):          # a donor far away (another tile): non-null, non-empty
        if abs(cand - i) > 600 and not _is_null(fields, rows, offs, cand, k):
            if _slot_at(fields, rows, offs, cand, k)[1] & 0xFFFFFFFF:
                j = cand
                break
    assert j is not None
    bad = rows.copy()
    _, sj = _slot_at(fields, rows, offs, j, k)
    abs_j = int(offs[j]) + (sj >> 32)
    rel = abs_j - int(offs[i])
    p, _ = _slot_at(fields, rows, offs, i, k)
    struct.pack_into("<Q", bad, p, ((rel & 0xFFFFFFFF) << 32) | (sj & 0xFFFFFFFF))
    got = [column_to_host(c) for c in enc.decode_batch(_batch(enc, bad, offs, n, dev))]
    assert_columns_equal(fields, got, oracle.decode(fields, bad, offs, n), n)


# ---- nested schemas: the level decode (fury_decode_prepare reports at prepare) ---------------

def _nested_batch(oracle, fields, n, seed, dev):
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders
    from tests.test_device import _random_value
    rng = np.random.default_rng(seed)
    beans = [{f.name: _random_value(f, rng) for f in fields} for _ in range(n)]
    host = beans_to_columns(fields, beans)
    enc = Encoders.bean(fields, device=dev)
    rows, offs = oracle.encode(fields, host, n)
    return enc, rows.copy(), np.asarray(offs, np.int64).copy()


def _value_at(fields, rows, offs, i, k):
    p, slot = _slot_at(fields, rows, offs, i, k)
    return int(offs[i]) + (slot >> 32), slot


@pytest.mark.parametrize("how", ["string_past_end", "list_count", "struct_out", "map_key_bytes",
                                 "map_count_mismatch", "list_elem_string"])
def test_nested_decode_out_of_bounds(oracle, dev, how):
    from fury_amd.encoder import IndexOutOfBoundsException, UnsupportedOperationException
    from fury_amd.encoder import column_to_host
    fields = SCHEMAS["foo"]          # f1 int, f2 string, f3 list<string>, f4 map<string,int>, f5 Bar
    names = [f.name for f in fields]
    n = 1500
    enc, rows, offs = _nested_batch(oracle, fields, n, 9, dev)
    total = int(offs[n])
    bad = rows.copy()
    exc = IndexOutOfBoundsException
    if how == "string_past_end":
        k = names.index("f2")
        i, _ = _victim(fields, rows, offs, n, {T.STRING})
        p, slot = _slot_at(fields, rows, offs, i, k)
        struct.pack_into("<Q", bad, p, (((total - int(offs[i]) + 8) & 0xFFFFFFFF) << 32) | 3)
    elif how in ("list_count", "list_elem_string"):
        k = names.index("f3")
        i = next(r for r in range(n // 2, n) if not _is_null(fields, rows, offs, r, k) and
                 struct.unpack_from("<q", rows, _value_at(fields, rows, offs, r, k)[0])[0] > 0)
        vp, _ = _value_at(fields, rows, offs, i, k)
        if how == "list_count":
            struct.pack_into("<q", bad, vp, 1 << 29)
        else:                         # the first element's (string) slot points past the end
            m = struct.unpack_from("<q", rows, vp)[0]
            ep = vp + 8 + _bm(m)
            if (rows[vp + 8] & 1) == 0:
                struct.pack_into("<Q", bad, ep, (((total - vp + 16) & 0xFFFFFFFF) << 32) | 4)
            else:
                pytest.skip("first element null")
    elif how == "struct_out":
        k = names.index("f5")
        i, _ = _victim(fields, rows, offs, n, {T.STRUCT})
        p, slot = _slot_at(fields, rows, offs, i, k)
        struct.pack_into("<Q", bad, p, (((total - int(offs[i]) - 8) & 0xFFFFFFFF) << 32) | 32)
    elif how in ("map_key_bytes", "map_count_mismatch"):
        k = names.index("f4")
        i = next(r for r in range(n // 2, n) if not _is_null(fields, rows, offs, r, k) and
                 struct.unpack_from("<q", rows, _value_at(fields, rows, offs, r, k)[0] + 8)[0] > 0)
        vp, _ = _value_at(fields, rows, offs, i, k)
        if how == "map_key_bytes":
            struct.pack_into("<q", bad, vp, total)
        else:
            kb = struct.unpack_from("<q", rows, vp)[0]
            cnt = struct.unpack_from("<q", rows, vp + 8 + kb)[0]
            struct.pack_into("<q", bad, vp + 8 + kb, cnt - 1)
            exc = UnsupportedOperationException
    with pytest.raises(exc):
        enc.decode_batch(_batch(enc, bad, offs, n, dev))
    # the error state is clear afterwards: the intact rows decode to the oracle's columns
    good = [column_to_host(c) for c in enc.decode_batch(_batch(enc, rows, offs, n, dev))]
    assert_columns_equal(fields, good, oracle.decode(fields, rows, offs, n), n)


def test_nested_row_offset_out_of_bounds(oracle, dev):
    from fury_amd.encoder import IndexOutOfBoundsException
    fields = SCHEMAS["foo"]
    n = 700
    enc, rows, offs = _nested_batch(oracle, fields, n, 4, dev)
    bad_offs = offs.copy()
    bad_offs[300] = int(offs[n]) + 8
    with pytest.raises(IndexOutOfBoundsException, match="row 300"):
        enc.decode_batch(_batch(enc, rows, bad_offs, n, dev))


def test_host_decode_out_of_bounds(oracle, dev):
    """The host-memory (JNI) decode reports the same exception synchronously."""
    from fury_amd.encoder import IndexOutOfBoundsException
    fields = SCHEMAS["mixed"]
    n = 1000
    enc, host, rows, offs = _encode(oracle, fields, n, 2, dev, null_pct=10, str_max=30)
    i, k = _victim(fields, rows, offs, n, {T.STRING})
    bad = _corrupt(fields, rows, offs, n, i, k, "offset_past_end")
    with pytest.raises(IndexOutOfBoundsException, match=f"row {i} "):
        enc.decode_host(bad, offs, n)
    enc.decode_host(rows, offs, n)


def test_device_errors_stay_on_their_stream(oracle, dev):
    """A malformed decode on stream A (error left pending: not yet taken) does not leak into an
    unrelated encode + decode on stream B run from another thread meanwhile -- those succeed,
    bit-exact -- and A's own status call still reports A's error (row and all), once.  (The
    error words are per stream: include/fury_row.h, asynchronous device errors.)"""
    import threading
    from fury_amd.encoder import IndexOutOfBoundsException, column_to_device, column_to_host
    fields = SCHEMAS["mixed"]
    n = 3001
    enc, host, rows, offs = _encode(oracle, fields, n, 11, dev, null_pct=10, str_max=30)
    i, k = _victim(fields, rows, offs, n, {T.STRING})
    bad = _batch(enc, _corrupt(fields, rows, offs, n, i, k, "offset_past_end"), offs, n, dev)
    good = _batch(enc, rows, offs, n, dev)
    dcols = [column_to_device(c, dev) for c in host]
    torch.cuda.synchronize()
    sa = torch.cuda.Stream(dev)
    enc._decode(bad, True, False, sa, None, "bound")      # raises on the device, not taken yet
    sa.synchronize()
    out = {}

    def other():
        try:
            sb = torch.cuda.Stream(dev)
            b2 = enc.encode_batch(dcols, n, stream=sb)
            cols = enc.decode_batch(good, stream=sb)
            sb.synchronize()
            out["rows"] = b2.rows.cpu().numpy()
            out["cols"] = [column_to_host(c) for c in cols]
        except Exception as e:          # noqa: BLE001 -- reported below
            out["err"] = e

    t = threading.Thread(target=other)
    t.start()
    t.join()
    assert "err" not in out, out.get("err")
    assert np.array_equal(out["rows"], rows)
    assert_columns_equal(fields, out["cols"], oracle.decode(fields, rows, offs, n), n)
    enc.device_status()                 # this thread's default stream: nothing pending
    with pytest.raises(IndexOutOfBoundsException, match=f"row {i} "):
        enc.device_status(sa)
    enc.device_status(sa)               # taken once


def test_error_slots_recycle_past_1024_streams(oracle, dev):
    """every stream that launches work holds one of 1024 device error slots until it is
    released (fury_stream_release), and slots are never shared.  1100 short-lived streams each run
    a decode and are released: the slots recycle, and an error raised on one of them (left
    pending, its stream kept) is still reported on that stream alone, after streams that reused
    other released slots ran clean decodes in between.  With every slot held, a call on a new
    stream fails loudly (FURY_ERR_DEVICE) instead of sharing a slot."""
    import ctypes
    from fury_amd import _native as N
    from fury_amd.encoder import FuryDeviceError, IndexOutOfBoundsException, column_to_host
    hip = ctypes.CDLL("libamdhip64.so")
    L = N.lib()
    fields = SCHEMAS["mixed"]
    n = 300
    enc, host, rows, offs = _encode(oracle, fields, n, 5, dev, null_pct=10, str_max=30)
    i, k = _victim(fields, rows, offs, n, {T.STRING})
    bad = _batch(enc, _corrupt(fields, rows, offs, n, i, k, "offset_past_end"), offs, n, dev)
    good = _batch(enc, rows, offs, n, dev)
    want = oracle.decode(fields, rows, offs, n)
    cols = enc.decode_batch(good)                       # outputs reused by every stream below
    torch.cuda.synchronize()
    base = L.fury_get_tuning(b"err_slots")

    def new_stream():
        h = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
        return h, torch.cuda.ExternalStream(h.value, device=dev)

    def drop(h):
        assert L.fury_stream_release(h) == 0
        assert hip.hipStreamDestroy(h) == 0

    held = None
    for j in range(1100):
        h, s = new_stream()
        if j == 700:                                    # the faulting stream stays open
            enc._decode(bad, True, False, s, None, "bound")
            s.synchronize()
            held = (h, s)
            continue
        enc.decode_into(good, cols, s)
        s.synchronize()
        drop(h)
    assert L.fury_get_tuning(b"err_slots") == base + 1
    assert_columns_equal(fields, [column_to_host(c) for c in cols], want, n)
    enc.device_status()                                 # nothing on this thread's stream
    with pytest.raises(IndexOutOfBoundsException, match=f"row {i} "):
        enc.device_status(held[1])
    enc.device_status(held[1])                          # taken once
    drop(held[0])
    assert L.fury_get_tuning(b"err_slots") == base
    # exhaustion: hold every free slot, then one more stream must fail loudly
    live = []
    try:
        while L.fury_get_tuning(b"err_slots") < 1024:
            h, s = new_stream()
            live.append(h)
            enc.decode_into(good, cols, s)
        h, s = new_stream()
        live.append(h)
        with pytest.raises(FuryDeviceError, match="error slots exhausted"):
            enc.decode_into(good, cols, s)
    finally:
        torch.cuda.synchronize()
        for h in live:
            drop(h)
    assert L.fury_get_tuning(b"err_slots") == base


@pytest.mark.gpu
def test_thread_exit_slot_quarantine(oracle, dev):
    """a thread that launches a failing decode on the null stream (torch's default) and
    exits without synchronising leaves its error slot QUARANTINED, not free: the kernel may still
    be running and raise into it.  New streams never receive it while it is quarantined; when
    the free slots run out the library synchronises the devices, drops the late error and reuses
    the slot -- a clean call on the stream that then gets it reports nothing."""
    import ctypes
    import threading
    from fury_amd import _native as N
    hip = ctypes.CDLL("libamdhip64.so")
    L = N.lib()
    fields = SCHEMAS["mixed"]
    n = 300
    enc, host, rows, offs = _encode(oracle, fields, n, 6, dev, null_pct=10, str_max=30)
    i, k = _victim(fields, rows, offs, n, {T.STRING})
    bad = _batch(enc, _corrupt(fields, rows, offs, n, i, k, "offset_past_end"), offs, n, dev)
    good = _batch(enc, rows, offs, n, dev)
    cols = enc.decode_batch(good)
    torch.cuda.synchronize()
    assert L.fury_trim_workspace(0) == 0              # start with an empty quarantine
    assert L.fury_get_tuning(b"err_slots_quarantined") == 0
    base = L.fury_get_tuning(b"err_slots")

    class _NullStream:            # the legacy null stream itself (handle 0): this thread's key
        cuda_stream = 0

    def worker():
        torch.cuda.set_device(dev)
        # one asynchronous launch that raises on the device; the thread exits without taking it
        enc.decode_into(bad, cols, stream=_NullStream())

    exits = L.fury_get_tuning(b"thread_key_exits")
    t = threading.Thread(target=worker)
    t.start()
    t.join()
    # join() returns when the Python thread state is gone; the OS thread's C++ thread_local
    # destructors (which quarantine the slot) run just after
    import time
    deadline = time.time() + 10
    while L.fury_get_tuning(b"err_slots_quarantined") < 1 and time.time() < deadline:
        time.sleep(0.01)
    assert L.fury_get_tuning(b"err_slots") == base, (
        f"thread_key_exits {exits} -> {L.fury_get_tuning(b'thread_key_exits')}, quarantined "
        f"{L.fury_get_tuning(b'err_slots_quarantined')}, last key kind "
        f"{L.fury_get_tuning(b'err_slot_last_key')}")
    assert L.fury_get_tuning(b"err_slots_quarantined") == 1

    def new_stream():
        h = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
        return h, torch.cuda.ExternalStream(h.value, device=dev)

    live = []
    try:
        # clean calls on new streams while the slot is quarantined: none of them sees the error
        for _ in range(8):
            h, s = new_stream()
            live.append(h)
            enc.decode_into(good, cols, s)
            enc.device_status(s)
        # take every never-used / free slot; the next stream drains the quarantine and gets the
        # quarantined slot, with the late error dropped
        while L.fury_get_tuning(b"err_slots") < 1024 - 1:
            h, s = new_stream()
            live.append(h)
            enc.decode_into(good, cols, s)
        assert L.fury_get_tuning(b"err_slots_quarantined") == 1
        h, s = new_stream()
        live.append(h)
        enc.decode_into(good, cols, s)
        enc.device_status(s)
        assert L.fury_get_tuning(b"err_slots_quarantined") == 0
        assert L.fury_get_tuning(b"err_slots") == 1024
    finally:
        torch.cuda.synchronize()
        for h in live:
            assert L.fury_stream_release(h) == 0
            assert hip.hipStreamDestroy(h) == 0
    assert L.fury_get_tuning(b"err_slots") == base
