"""GPU parity tests: the HIP path (through the C ABI) against the oracle restatement, on the
same seeded inputs.  Bar: bit-exact rows, bit-exact decoded columns.  Marked gpu."""
from __future__ import annotations

import json
import os
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from fury_amd import types as T  # noqa: E402
from fury_amd.workloads import SCHEMAS, Column, docs_struct_values, gen_columns  # noqa: E402
from tests.helpers import as_u8, assert_columns_equal  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch.device("cuda:0")


def _dev_cols(cols, dev):
    from fury_amd.encoder import column_to_device
    return [column_to_device(c, dev) for c in cols]


def _roundtrip(oracle, name, n, dev, seed=3, fields=None, cols=None, **knobs):
    from fury_amd.encoder import Encoders, column_to_host
    fields = fields or SCHEMAS[name]
    host = cols if cols is not None else gen_columns(name, fields, n, seed=seed, **knobs)
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch(_dev_cols(host, dev), n)
    torch.cuda.synchronize()
    want, want_offs = oracle.encode(fields, host, n)
    got = batch.rows.cpu().numpy()
    assert got.shape == want.shape, f"{name}: total bytes {got.shape} vs {want.shape}"
    if not np.array_equal(got, want):
        bad = np.nonzero(got != want)[0]
        raise AssertionError(f"{name}: {len(bad)} bytes differ, first at {bad[:8]}")
    if batch.row_offsets is not None:
        assert np.array_equal(batch.row_offsets.cpu().numpy(), want_offs)
    dec = [column_to_host(c) for c in enc.decode_batch(batch)]
    ref = oracle.decode(fields, want, want_offs, n)
    assert_columns_equal(fields, dec, ref, n)
    return enc, batch, host


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 255, 256, 257, 1000, 4097])
def test_struct100_bit_exact(oracle, dev, n):
    _roundtrip(oracle, "struct100", n, dev)


@pytest.mark.parametrize("name,n", [("mixed", 1), ("mixed", 257), ("mixed", 3000),
                                    ("nested", 1), ("nested", 700), ("nested", 5000),
                                    ("narrow", 129), ("narrow", 2000), ("beanb", 300),
                                    ("bar", 513), ("docs_struct", 999)])
def test_schemas_bit_exact(oracle, dev, name, n):
    _roundtrip(oracle, name, n, dev)


def test_docs_struct_java_random_values(oracle, dev):
    fields = SCHEMAS["docs_struct"]
    _roundtrip(oracle, "docs_struct", 1, dev, cols=docs_struct_values(fields))


def test_golden_fixtures(oracle, dev):
    from fury_amd.encoder import Encoders
    for name in ("struct100", "mixed", "nested", "narrow"):
        d = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
        fields = SCHEMAS[name]
        n = len(d["row_offsets"]) - 1
        cols = gen_columns(name, fields, n, seed=1234)
        enc = Encoders.bean(fields, device=dev)
        b = enc.encode_batch(_dev_cols(cols, dev), n)
        assert np.array_equal(b.rows.cpu().numpy(), d["rows"]), name


def test_special_float_bits_and_extremes(oracle, dev):
    """NaN payloads, -0.0, +-inf, int extremes survive as raw bits (doubleToRawLongBits)."""
    fields = [T.not_null_field("d", T.FLOAT64), T.not_null_field("f", T.FLOAT32),
              T.not_null_field("i", T.INT64), T.field("b", T.INT8), T.field("s", T.INT16)]
    d = np.array([0x7FF8000000000001, 0xFFF0000000000000, 0x8000000000000000,
                  0x7FF0000000000000, 0x7FF4DEADBEEF0000, 1, 0, 0x3FF0000000000000], np.uint64)
    f = np.array([0x7FC00001, 0xFF800000, 0x80000000, 0x7F800000, 0x7FA00005, 1, 0,
                  0x3F800000], np.uint32)
    i = np.array([-(2 ** 63), 2 ** 63 - 1, -1, 0, 1, 42, -42, 7], np.int64)
    b = np.array([-128, 127, -1, 0, 1, 5, 6, 7], np.int8)
    s = np.array([-32768, 32767, -1, 0, 1, 5, 6, 7], np.int16)
    vb = np.array([0b10110101], np.uint8)
    cols = [Column(values=d.view(np.float64)), Column(values=f.view(np.float32)),
            Column(values=i), Column(values=np.where(np.unpackbits(vb, bitorder="little")
                                                     .astype(bool), b, 0).astype(np.int8),
                                     validity=vb),
            Column(values=s, validity=None)]
    _roundtrip(oracle, None, 8, dev, fields=fields, cols=cols)


def test_strings_edge_lengths(oracle, dev):
    """Empty, 1, 7, 8, 9, long strings; unaligned Arrow offsets; multibyte UTF-8; nulls."""
    fields = [T.field("a", T.STRING), T.field("b", T.BINARY)]
    vals = ["", "x", "abcdefg", "abcdefgh", "abcdefghi", "é" * 37, None, "ü中😀", "z" * 300,
            None, "", "q" * 8191]
    from fury_amd.beans import beans_to_columns
    beans = [{"a": v, "b": (v.encode() if v is not None else None)} for v in vals]
    cols = beans_to_columns(fields, beans)
    _roundtrip(oracle, None, len(vals), dev, fields=fields, cols=cols)


def test_lists_edge_lengths(oracle, dev):
    """n = 0, 1, 63, 64, 65, 130; null lists; null elements; narrow element widths."""
    fields = [T.array_field("l", T.INT64), T.array_field("i", T.INT32),
              T.array_field("b", T.BOOL), T.array_field("s", T.INT16, elem_nullable=False)]
    lens = [0, 1, 63, 64, 65, 130, 2, 0]
    rng = np.random.default_rng(0)
    beans = []
    for k, m in enumerate(lens):
        if k == 6:
            beans.append({"l": None, "i": None, "b": None, "s": None})
            continue
        beans.append({
            "l": [None if (j % 7 == 3) else int(x) for j, x in
                  enumerate(rng.integers(-2**62, 2**62, m))],
            "i": [int(x) for x in rng.integers(-2**31, 2**31, m)],
            "b": [None if j % 5 == 0 else bool(j & 1) for j in range(m)],
            "s": [int(x) for x in rng.integers(-2**15, 2**15, m)],
        })
    from fury_amd.beans import beans_to_columns
    cols = beans_to_columns(fields, beans)
    _roundtrip(oracle, None, len(beans), dev, fields=fields, cols=cols)


def test_empty_batch(dev):
    from fury_amd.encoder import Encoders
    for name in ("struct100", "mixed"):
        fields = SCHEMAS[name]
        cols = gen_columns(name, fields, 0)
        enc = Encoders.bean(fields, device=dev)
        b = enc.encode_batch(_dev_cols(cols, dev), 0)
        assert b.rows.numel() == 0
        assert enc.decode_batch(b) is not None


def test_large_batch_with_long_strings_falls_back(oracle, dev):
    """Row ranges larger than the LDS stage take the direct-global path."""
    _roundtrip(oracle, "mixed", 2000, dev, str_max=600)
    _roundtrip(oracle, "nested", 1500, dev, list_max=200)


def test_single_object_api_matches_java_layout(dev):
    from fury_amd.encoder import ClassNotCompatibleException, Encoders
    enc = Encoders.bean(SCHEMAS["bar"], device=dev)
    kn = json.load(open(os.path.join(GOLDEN, "known_answers.json")))
    row = enc.to_row({"f1": 1, "f2": "str"})
    assert row.hex() == kn["bar_row_hex"]["value"]
    data = enc.encode({"f1": 1, "f2": "str"})
    assert struct.unpack_from("<q", data)[0] == 16567 and data[8:] == row
    assert enc.decode(data) == {"f1": 1, "f2": "str"}
    bad = struct.pack("<q", 16568) + row
    with pytest.raises(ClassNotCompatibleException):
        enc.decode(bad)


def test_frame_unframe_roundtrip(oracle, dev):
    """[int32 len][int64 hash][row] stream of Encoders.encode(MemoryBuffer, T)."""
    from fury_amd.encoder import ClassNotCompatibleException, Encoders
    for name, n in (("mixed", 300), ("struct100", 70)):
        fields = SCHEMAS[name]
        host = gen_columns(name, fields, n, seed=8)
        enc = Encoders.bean(fields, device=dev)
        b = enc.encode_batch(_dev_cols(host, dev), n)
        stream, fo = enc.frame(b)
        s = stream.cpu().numpy().tobytes()
        rows, offs = oracle.encode(fields, host, n)
        want = b"".join(struct.pack("<iq", int(offs[i + 1] - offs[i]) + 8, enc.schema_hash) +
                        rows[offs[i]:offs[i + 1]].tobytes() for i in range(n))
        assert s == want
        b2 = enc.unframe(stream, n)
        assert np.array_equal(b2.rows.cpu().numpy(), rows)
        other = Encoders.bean(SCHEMAS["bar"], device=dev)
        with pytest.raises(ClassNotCompatibleException):
            other.unframe(stream, n)


def test_fixed_paths_bit_exact(oracle, dev):
    """The fixed-width kernels the library ships (fast path: 8-byte columns, no validity; pair-mode
    decode and its fallback when a column is not 16-byte aligned; the general path: narrow types
    and validity) write the oracle's rows and decode them back, including ragged last tiles (odd
    row counts for the pair mode)."""
    from fury_amd.encoder import Encoders, column_to_host
    for n in (1, 3, 63, 65, 129, 1001):
        _roundtrip(oracle, "struct100", n, dev, seed=n)
        _roundtrip(oracle, "narrow", n, dev, seed=n)
    # a column at an 8- but not 16-byte aligned address: the decode takes the non-pair kernel
    fields = SCHEMAS["struct100"]
    n = 257
    host = gen_columns("struct100", fields, n, seed=5)
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch(_dev_cols(host, dev), n)
    cols = enc.alloc_columns(n, validity=False)
    pad = torch.empty(n * 8 + 8, dtype=torch.uint8, device=dev)
    cols[3].values = pad[8:]
    enc.decode_into(batch, cols)
    want, _ = oracle.encode(fields, host, n)
    ref = oracle.decode(fields, want, None, n)
    assert_columns_equal(fields, [column_to_host(c) for c in cols], ref, n)


def _roundtrips_var(oracle, dev, seed0):
    for name, n in (("mixed", 1), ("mixed", 513), ("mixed", 20_001), ("narrow", 1025),
                    ("nested", 4097), ("beanb", 700)):
        _roundtrip(oracle, name, n, dev, seed=n + seed0)
    _roundtrip(oracle, "mixed", 3000, dev, seed=seed0, str_max=600)   # tiles beyond the stage
    _roundtrip(oracle, "nested", 2000, dev, seed=seed0, list_max=200)


def test_var_decode_bit_exact(oracle, dev):
    """The variable-length decode (one pass, Arrow offsets chained across tiles by a decoupled
    look-back) decodes to the oracle's columns on ragged tiles and tiles beyond the LDS image."""
    from fury_amd import _native as N
    _roundtrips_var(oracle, dev, 0)
    assert N.lib().fury_get_tuning(b"lookback_timeouts") == 0


def test_var_decode_lookback_help_bit_exact(oracle, dev):
    """The variable-length decodes number tiles by blockIdx and let a look-back compute a silent
    predecessor's aggregate from its rows (look_back_help).  Tuning "lookback_help" makes every
    look-back help at once -- the path a late-dispatched predecessor takes -- and the results must
    still be the oracle's columns, for the register-staged (<= 16 fields) and the 17-256-field
    kernels."""
    from fury_amd import _native as N
    assert N.lib().fury_set_tuning(b"lookback_help", 1) == 0
    try:
        _roundtrips_var(oracle, dev, 32768)
        for ncols, n in ((33, 2049), (17, 20_001)):    # the 17-256-field kernel (decode_var_kernel)
            fields = _wide_fields(ncols)
            host = gen_columns("wide", fields, n, seed=ncols, null_pct=10, str_max=40, list_max=8)
            _roundtrip(oracle, None, n, dev, fields=fields, cols=host)
    finally:
        N.lib().fury_set_tuning(b"lookback_help", 0)
    assert N.lib().fury_get_tuning(b"lookback_timeouts") == 0


def _walks():
    from fury_amd import _native as N
    return N.lib().fury_get_tuning(b"unframe_walks")


def _unframe_both(enc, stream, n):
    """unframe by the speculative parallel parse and by the sequential walk (tuning 'unframe')."""
    from fury_amd import _native as N
    assert N.lib().fury_set_tuning(b"unframe", 1) == 0
    try:
        walked = enc.unframe(stream, n)
    finally:
        N.lib().fury_set_tuning(b"unframe", 0)
    return enc.unframe(stream, n), walked


@pytest.mark.parametrize("name,n", [("mixed", 5000), ("struct100", 3000), ("nested", 4097),
                                    ("narrow", 1), ("mixed", 257)])
def test_unframe_parallel_equals_walk(oracle, dev, name, n):
    """Speculative parallel parse == sequential walk == oracle rows, without falling back."""
    from fury_amd.encoder import Encoders
    fields = SCHEMAS[name]
    host = gen_columns(name, fields, n, seed=31)
    enc = Encoders.bean(fields, device=dev)
    stream, _ = enc.frame(enc.encode_batch(_dev_cols(host, dev), n))
    w0 = _walks()
    fast, walked = _unframe_both(enc, stream, n)
    assert _walks() == w0 + 1, "a clean stream must verify without the sequential walk"
    rows, offs = oracle.encode(fields, host, n)
    assert np.array_equal(fast.rows.cpu().numpy(), rows)
    assert np.array_equal(walked.rows.cpu().numpy(), rows)
    if fast.row_offsets is not None:
        assert np.array_equal(fast.row_offsets.cpu().numpy(), offs)


@pytest.mark.parametrize("name,n", [("mixed", 3001), ("struct100", 513), ("nested", 700)])
def test_stream_encode_decode(oracle, dev, name, n):
    """encode_stream / decode_stream: the Java encode(MemoryBuffer, T) loop's stream and back to
    the oracle's columns."""
    from fury_amd.encoder import column_to_host, Encoders
    fields = SCHEMAS[name]
    host = gen_columns(name, fields, n, seed=41)
    enc = Encoders.bean(fields, device=dev)
    s = enc.encode_stream(_dev_cols(host, dev), n)
    rows, offs = oracle.encode(fields, host, n)
    assert s.numel() == rows.nbytes + 12 * n
    dec = [column_to_host(c) for c in enc.decode_stream(s, n)]
    assert_columns_equal(fields, dec, oracle.decode(fields, rows, offs, n), n)


def _repairs():
    from fury_amd import _native as N
    return N.lib().fury_get_tuning(b"unframe_repairs")


def test_unframe_fake_header_in_payload(oracle, dev):
    """A row whose slots spell a plausible frame header ([len 16][schema hash]) is a false
    candidate: verification fails and the parallel repair (pointer doubling over the candidates)
    finds the real frame chain -- no sequential walk; results are still the oracle's."""
    from fury_amd.encoder import Encoders
    fields = SCHEMAS["struct100"]
    n = 600
    host = gen_columns("struct100", fields, n, seed=5)
    enc = Encoders.bean(fields, device=dev)
    h = enc.schema_hash & (2**64 - 1)
    f0 = host[0].values.view(np.uint64)
    f1 = host[1].values.view(np.uint64)
    for r in (0, 5, 599):
        f0[r] = np.uint64(16 | ((h & 0xFFFFFFFF) << 32))
        f1[r] = np.uint64(h >> 32)
    stream, _ = enc.frame(enc.encode_batch(_dev_cols(host, dev), n))
    w0, r0 = _walks(), _repairs()
    got = enc.unframe(stream, n)
    assert _walks() == w0, "fake headers are repaired in parallel, not walked"
    assert _repairs() == r0 + 1
    rows, _ = oracle.encode(fields, host, n)
    assert np.array_equal(got.rows.cpu().numpy(), rows)


def _stream_at(stream, shift, dev, tail=0):
    """The stream copied to byte offset `shift` of a fresh buffer (Java frames at any
    writerIndex), optionally followed by `tail` junk bytes."""
    buf = torch.full((stream.numel() + shift + tail + 64,), 0xA5, dtype=torch.uint8, device=dev)
    buf[shift:shift + stream.numel()] = stream
    return buf[shift:shift + stream.numel() + tail]


@pytest.mark.parametrize("shift", [1, 2, 3, 4, 5, 8, 9, 13])
@pytest.mark.parametrize("name,n", [("mixed", 2777), ("struct100", 300), ("nested", 1500)])
def test_unframe_any_byte_offset(oracle, dev, name, n, shift):
    """CodecBuilderTest.java:51-67 decodes a stream written after a 1-byte offset: streams at
    1..13-byte offsets parse in parallel (no walk, no repair) to the oracle's rows, and a
    two-row decode_stream at offset 1 round-trips like the Java test."""
    from fury_amd.encoder import Encoders, column_to_host
    fields = SCHEMAS[name]
    host = gen_columns(name, fields, n, seed=shift + n)
    enc = Encoders.bean(fields, device=dev)
    stream, _ = enc.frame(enc.encode_batch(_dev_cols(host, dev), n))
    s = _stream_at(stream, shift, dev, tail=7)
    w0, r0 = _walks(), _repairs()
    got = enc.unframe(s, n)
    assert (_walks(), _repairs()) == (w0, r0)
    rows, offs = oracle.encode(fields, host, n)
    assert np.array_equal(got.rows.cpu().numpy(), rows)
    if got.row_offsets is not None:
        assert np.array_equal(got.row_offsets.cpu().numpy(), offs)
    dec = [column_to_host(c) for c in enc.decode_stream(s, 2)]
    assert_columns_equal(fields, dec, oracle.decode(fields, rows[:offs[2]], offs[:3], 2), 2)


@pytest.mark.parametrize("shift", [0, 1, 6])
def test_unframe_fake_header_unaligned(oracle, dev, shift):
    """Fake headers in payloads at an unaligned base: repaired in parallel, oracle-exact."""
    from fury_amd.encoder import Encoders
    fields = SCHEMAS["mixed"]
    n = 5000
    host = gen_columns("mixed", fields, n, seed=9)
    enc = Encoders.bean(fields, device=dev)
    h = enc.schema_hash & (2**64 - 1)
    b = host[1].values.view(np.uint64)        # b: Long (slot 1) + c: Double (slot 2)
    c = host[2].values.view(np.uint64)
    va, vb = host[1].validity, host[2].validity
    for r in range(3, n, 97):                  # slots of b, c spell [len 24][hash] at word 4k
        b[r] = np.uint64(24 | ((h & 0xFFFFFFFF) << 32))
        c[r] = np.uint64(h >> 32)
        va[r >> 3] |= np.uint8(1 << (r & 7))
        vb[r >> 3] |= np.uint8(1 << (r & 7))
    stream, _ = enc.frame(enc.encode_batch(_dev_cols(host, dev), n))
    s = _stream_at(stream, shift, dev)
    w0, r0 = _walks(), _repairs()
    got = enc.unframe(s, n)
    assert _walks() == w0 and _repairs() == r0 + 1
    rows, offs = oracle.encode(fields, host, n)
    assert np.array_equal(got.rows.cpu().numpy(), rows)
    assert np.array_equal(got.row_offsets.cpu().numpy(), offs)


@pytest.mark.parametrize("shift", [0, 3])
def test_unframe_errors_match_decode(oracle, dev, shift):
    """Errors are Encoders.decode's: a frame with another schema's hash in the middle of the
    stream -> ClassNotCompatibleException; a stream cut inside a frame -> IndexOutOfBounds;
    asking for fewer frames than the stream holds -> that prefix."""
    from fury_amd.encoder import ClassNotCompatibleException, Encoders, FuryError
    fields = SCHEMAS["mixed"]
    n = 4000
    host = gen_columns("mixed", fields, n, seed=6)
    enc = Encoders.bean(fields, device=dev)
    stream, fo = enc.frame(enc.encode_batch(_dev_cols(host, dev), n))
    rows, offs = oracle.encode(fields, host, n)
    bad = stream.clone()
    p = int(fo[2500])
    bad[p + 4] ^= 1                            # frame 2500's schema hash
    with pytest.raises(ClassNotCompatibleException):
        enc.unframe(_stream_at(bad, shift, dev), n)
    short = enc.unframe(_stream_at(bad, shift, dev), 2500)     # the frames before it are fine
    assert np.array_equal(short.rows.cpu().numpy(), rows[:offs[2500]])
    with pytest.raises(FuryError):
        enc.unframe(_stream_at(stream[:-8], shift, dev), n)    # last frame runs past the end
    prefix = enc.unframe(_stream_at(stream, shift, dev), n - 1)
    assert np.array_equal(prefix.rows.cpu().numpy(), rows[:offs[n - 1]])


def test_unframe_large_fast_path(dev):
    """400k Struct-100 frames (331 MB stream): parallel parse round trip, no fallback."""
    from fury_amd.encoder import Encoders
    from fury_amd.workloads import Column as C
    fields = SCHEMAS["struct100"]
    n = 400_000
    g = torch.Generator(device=dev).manual_seed(9)
    cols = [C(values=torch.randint(-2**63, 2**63 - 1, (n,), dtype=torch.int64, device=dev,
                                   generator=g)) for _ in fields]
    enc = Encoders.bean(fields, device=dev)
    b = enc.encode_batch(cols, n)
    stream, _ = enc.frame(b)
    w0 = _walks()
    got = enc.unframe(stream, n)
    assert _walks() == w0
    assert torch.equal(got.rows, b.rows)
    del stream, got, b


def test_rows_to_arrow_matches_pyarrow(oracle, dev):
    """ArrowWriter path: device Arrow buffers == pyarrow arrays built from the same values."""
    import pyarrow as pa
    from fury_amd.arrow import pa_type
    from fury_amd.encoder import ArrowWriter, Encoders
    from fury_amd.beans import columns_to_beans
    for name, n in (("nested", 999), ("mixed", 1234), ("narrow", 300)):
        fields = SCHEMAS[name]
        host = gen_columns(name, fields, n, seed=21)
        enc = Encoders.bean(fields, device=dev)
        b = enc.encode_batch(_dev_cols(host, dev), n)
        w = ArrowWriter(enc)
        w.write(b)
        rb = w.finish_as_record_batch()
        rb.validate(full=True)
        beans = columns_to_beans(fields, host, n)
        for k, f in enumerate(fields):
            vals = [bb[f.name] for bb in beans]
            if f.type_id == T.DECIMAL:
                continue      # compared bytewise in test_schemas_bit_exact
            ref = pa.array(vals, type=pa_type(f))
            assert rb.column(k).equals(ref), f"{name}.{f.name}"


@pytest.mark.parametrize("rows", [3_000_000])
def test_struct100_full_size_roundtrip_property(dev, rows):
    """At bench scale: decode(encode(cols)) == cols byte-for-byte and every row's bitmap is
    zero (non-nullable primitives); a checksum of the row bytes equals the checksum of the
    interleaved columns computed independently with torch."""
    from fury_amd.encoder import Encoders
    fields = SCHEMAS["struct100"]
    g = torch.Generator(device=dev).manual_seed(5)
    cols = [Column(values=torch.randint(-2**63, 2**63 - 1, (rows,), dtype=torch.int64,
                                        device=dev, generator=g)) for _ in fields]
    enc = Encoders.bean(fields, device=dev)
    b = enc.encode_batch(cols, rows)
    r = b.rows.view(rows, 816)
    assert int(r[:, :16].abs().sum()) == 0
    slots = r[:, 16:].contiguous().view(torch.int64).view(rows, 100)
    stacked = torch.stack([c.values for c in cols], dim=1)
    assert torch.equal(slots, stacked)
    dec = enc.decode_batch(b, validity=False)
    for c, d in zip(cols, dec):
        assert torch.equal(c.values.view(torch.uint8), d.values)


def test_var_large_batch_hierarchical_scan(oracle, dev):
    """> 4096 workgroups: exercises the multi-level device scan of row sizes and of the Arrow
    offsets on decode; full byte comparison against the oracle."""
    _roundtrip(oracle, "mixed", 1_500_000, dev, seed=13)


# ---- nested schemas (generic engine) -------------------------------------------------------
def _nested_fields():
    inner = [T.field("a", T.INT32), T.array_field("l", T.INT64), T.field("s", T.STRING)]
    pt = [T.not_null_field("x", T.FLOAT64), T.not_null_field("y", T.FLOAT64)]
    return [
        T.not_null_field("id", T.INT64),
        T.struct_field("inner", inner),
        T.Field("ll", T.LIST, True, (T.Field("item", T.LIST, True, (T.field("item", T.INT32),)),)),
        T.map_field("m", T.field("key", T.STRING), T.field("value", T.INT32)),
        T.Field("pts", T.LIST, True, (T.struct_field("item", pt),)),
        T.Field("tags", T.LIST, True, (T.field("item", T.STRING),)),
        T.field("z", T.BOOL),
    ]


def _nested_beans(n, seed=0):
    rng = np.random.default_rng(seed)

    def maybe(v, p=0.1):
        return None if rng.random() < p else v

    def s(k):
        return "".join(chr(97 + int(x)) for x in rng.integers(0, 26, k))
    beans = []
    for i in range(n):
        beans.append({
            "id": int(rng.integers(-2**62, 2**62)),
            "inner": maybe({"a": maybe(int(rng.integers(-9, 9))),
                            "l": maybe([int(x) for x in rng.integers(-5, 5, rng.integers(0, 4))]),
                            "s": maybe(s(int(rng.integers(0, 12))))}),
            "ll": maybe([maybe([maybe(int(x)) for x in rng.integers(0, 99, rng.integers(0, 4))])
                         for _ in range(int(rng.integers(0, 4)))]),
            "m": maybe([(s(int(rng.integers(1, 6))), maybe(int(rng.integers(0, 9))))
                        for _ in range(int(rng.integers(0, 3)))]),
            "pts": maybe([maybe({"x": float(rng.random()), "y": float(rng.random())})
                          for _ in range(int(rng.integers(0, 3)))]),
            "tags": maybe([maybe(s(int(rng.integers(0, 9)))) for _ in range(int(rng.integers(0, 4)))]),
            "z": maybe(bool(rng.integers(0, 2))),
        })
    return beans


@pytest.mark.parametrize("n", [1, 7, 300, 2500])
def test_nested_schema_encode_decode(oracle, dev, n):
    from fury_amd.beans import beans_to_columns, columns_to_beans
    from fury_amd.encoder import Encoders, column_to_host
    from oracle import bean_oracle as B
    fields = _nested_fields()
    beans = _nested_beans(n, seed=n)
    host = beans_to_columns(fields, beans)
    enc = Encoders.bean(fields, device=dev)
    assert enc.nested
    batch = enc.encode_batch(_dev_cols(host, dev), n)
    want, want_offs = oracle.encode(fields, host, n)
    assert np.array_equal(batch.row_offsets.cpu().numpy(), want_offs)
    assert np.array_equal(batch.rows.cpu().numpy(), want)
    for i in range(min(n, 50)):
        assert want[want_offs[i]:want_offs[i + 1]].tobytes() == B.encode_row(fields, beans[i])
    dec = [column_to_host(c) for c in enc.decode_batch(batch)]
    assert columns_to_beans(fields, dec, n) == beans


def test_foo_bean_nested_struct_map(oracle, dev):
    """RowEncoderTest.Foo (list<string>, map<string,int>, nested Bar) on the device."""
    from fury_amd.encoder import Encoders
    from oracle import bean_oracle as B
    fields = SCHEMAS["foo"]
    enc = Encoders.bean(fields, device=dev)
    foo = {"f1": 2, "f2": "str", "f3": ["a", "b", "c"], "f4": [("k1", 1), ("k2", 2)],
           "f5": {"f1": 1, "f2": "str"}}
    row = enc.to_row(foo)
    assert row == B.encode_row(fields, foo)
    assert enc.from_row(row) == foo
    assert enc.decode(enc.encode(foo)) == foo


def test_nested_rows_to_arrow(dev):
    import pyarrow as pa
    from fury_amd.arrow import pa_type
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import ArrowWriter, Encoders
    fields = _nested_fields()
    n = 800
    beans = _nested_beans(n, seed=5)
    enc = Encoders.bean(fields, device=dev)
    b = enc.encode_batch(_dev_cols(beans_to_columns(fields, beans), dev), n)
    w = ArrowWriter(enc)
    w.write(b)
    rb = w.finish_as_record_batch()
    rb.validate(full=True)
    for k, f in enumerate(fields):
        ref = pa.array([bb[f.name] for bb in beans], type=pa_type(f))
        assert rb.column(k).equals(ref), f.name


# ---- single-pass decode (look-back scan of the Arrow offsets) --------------------------------
def test_many_var_columns_multi_chunk(oracle, dev):
    """13 STRING/LIST outputs: more than one look-back round per workgroup."""
    fields = ([T.field(f"s{i:02d}", T.STRING) for i in range(10)] +
              [T.array_field("la", T.INT64), T.array_field("lb", T.BOOL),
               T.array_field("lc", T.INT16, elem_nullable=False), T.field("x", T.INT32)])
    _roundtrip(oracle, None, 5000, dev, fields=fields,
               cols=gen_columns("many", fields, 5000, seed=21, null_pct=10, str_max=24,
                                list_max=9, elem_null_pct=10))


@pytest.mark.parametrize("name,n", [("mixed", 70_000), ("nested", 70_000), ("narrow", 20_000)])
def test_decode_into_scrubbed_buffers(oracle, dev, name, n):
    """decode_into over reused buffers holding garbage (offsets included) == oracle fromRow."""
    from fury_amd.encoder import Encoders, column_to_host
    fields = SCHEMAS[name]
    host = gen_columns(name, fields, n, seed=5)
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch(_dev_cols(host, dev), n)
    out = enc.decode_batch(batch)

    def scrub(c):
        for t in (c.values, c.offsets, c.validity):
            if t is not None:
                t.view(torch.uint8).fill_(0x5A)
        for x in c.child or []:
            scrub(x)
    for c in out:
        scrub(c)
    enc.decode_into(batch, out)
    enc.check_capacity(out, n)
    want, want_offs = oracle.encode(fields, host, n)
    assert_columns_equal(fields, [column_to_host(c) for c in out],
                         oracle.decode(fields, want, want_offs, n), n)


def test_decode_respects_capacity(dev):
    """Undersized payload buffers: nothing is written past them, offsets still complete."""
    from fury_amd.encoder import CapacityError, Encoders
    fields = [T.field("s", T.STRING), T.array_field("l", T.INT64)]
    n = 3000
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch(_dev_cols(gen_columns("cap", fields, n, seed=9, null_pct=5), dev), n)
    ref = enc.decode_batch(batch)
    ns = int(ref[0].offsets[n]); nl = int(ref[1].offsets[n])
    sbuf = torch.full((ns + 4096,), 0xAB, dtype=torch.uint8, device=dev)
    lbuf = torch.full((nl * 8 + 4096,), 0xCD, dtype=torch.uint8, device=dev)
    out = enc.decode_batch(batch)
    out[0].values = sbuf[: ns // 2]
    out[1].child[0].values = lbuf[: (nl // 3) * 8]
    enc.decode_into(batch, out)
    torch.cuda.synchronize()
    assert torch.equal(out[0].offsets, ref[0].offsets) and torch.equal(out[1].offsets, ref[1].offsets)
    assert torch.equal(sbuf[: ns // 2], ref[0].values[: ns // 2])
    assert bool((sbuf[ns // 2:] == 0xAB).all())
    assert torch.equal(lbuf[: (nl // 3) * 8], ref[1].child[0].values[: (nl // 3) * 8])
    assert bool((lbuf[(nl // 3) * 8:] == 0xCD).all())
    with pytest.raises(CapacityError):
        enc.check_capacity(out, n)


# ---- single-pass encode (fury_row_encode_measured) -------------------------------------------
@pytest.mark.parametrize("name,n", [("mixed", 1), ("mixed", 300_001), ("nested", 90_000),
                                    ("narrow", 5000), ("foo", 700)])
def test_encode_measured_matches_two_pass(dev, name, n):
    from fury_amd.encoder import Encoders
    fields = SCHEMAS[name]
    if name == "foo":
        from fury_amd.beans import beans_to_columns
        cols = _dev_cols(beans_to_columns(fields, [{"f1": i, "f2": str(i) * (i % 5),
                                                    "f3": [str(j) for j in range(i % 4)],
                                                    "f4": [(str(i), i)], "f5": {"f1": i, "f2": None}}
                                                   for i in range(n)]), dev)
    else:
        cols = _dev_cols(gen_columns(name, fields, n, seed=17), dev)
    enc = Encoders.bean(fields, device=dev)
    ref = enc.encode_batch(cols, n)
    total = ref.rows.numel()
    rows = torch.full((total + 4096,), 0xEE, dtype=torch.uint8, device=dev)
    offs = torch.full((n + 1,), -1, dtype=torch.int64, device=dev)
    enc.encode_measured_into(cols, n, rows[:total], offs)
    torch.cuda.synchronize()
    assert torch.equal(offs, ref.row_offsets)
    assert torch.equal(rows[:total], ref.rows)
    assert bool((rows[total:] == 0xEE).all())
    # undersized buffer: offsets still complete, nothing written past the capacity
    rows.fill_(0xEE)
    cap = (total // 3) & ~15
    enc.encode_measured_into(cols, n, rows[:cap], offs)
    torch.cuda.synchronize()
    assert torch.equal(offs, ref.row_offsets)
    assert bool((rows[cap:] == 0xEE).all())
    o = ref.row_offsets.cpu().numpy()
    end = int(o[int(np.searchsorted(o, cap, side="right")) - 1])   # rows ending by cap
    assert torch.equal(rows[:end], ref.rows[:end])


def test_encode_measured_fixed_capacity_error(dev):
    from fury_amd.encoder import CapacityError, Encoders
    fields = SCHEMAS["struct100"]
    enc = Encoders.bean(fields, device=dev)
    cols = _dev_cols(gen_columns("struct100", fields, 100), dev)
    rows = torch.empty(816 * 100, dtype=torch.uint8, device=dev)
    enc.encode_measured_into(cols, 100, rows, None)
    ref = enc.encode_batch(cols, 100)
    assert torch.equal(rows, ref.rows)
    with pytest.raises(CapacityError):
        enc.encode_measured_into(cols, 100, rows[:816 * 99], None)


def _encode_measured(enc, cols, n, dev):
    total_guess = enc.encode_batch(cols, n).rows.numel()
    rows = torch.full((total_guess + 64,), 0xEE, dtype=torch.uint8, device=dev)
    offs = torch.full((n + 1,), -1, dtype=torch.int64, device=dev)
    enc.encode_measured_into(cols, n, rows[:total_guess], offs)
    torch.cuda.synchronize()
    return rows, offs, total_guess


@pytest.mark.parametrize("case", ["mixed_multi_group", "long_strings", "long_lists", "edge_strings"])
def test_encode_measured_vs_oracle(oracle, dev, case):
    """fury_row_encode_measured (measure + encode in one call) against the oracle directly: rows
    and offsets bit-exact across several measure groups (1,024 rows) that straddle encode tiles,
    for oversized tiles that take the direct-to-HBM branch, and for edge-length strings; nothing
    is written past the rows."""
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders
    if case == "mixed_multi_group":
        fields, n = SCHEMAS["mixed"], 5 * 1024 + 77
        host = gen_columns("mixed", fields, n, seed=29)
    elif case == "long_strings":
        fields, n = SCHEMAS["mixed"], 2500
        host = gen_columns("mixed", fields, n, seed=31, str_max=600)
    elif case == "long_lists":
        fields, n = SCHEMAS["nested"], 1500
        host = gen_columns("nested", fields, n, seed=37, list_max=200)
    else:
        fields = [T.field("a", T.STRING), T.field("b", T.BINARY)]
        vals = ["", "x", "abcdefg", "abcdefgh", "abcdefghi", None, "z" * 300, "", "q" * 8191] * 150
        n = len(vals)
        host = beans_to_columns(fields, [{"a": v, "b": (v.encode() if v is not None else None)}
                                         for v in vals])
    want, want_offs = oracle.encode(fields, host, n)
    enc = Encoders.bean(fields, device=dev)
    cols = _dev_cols(host, dev)
    rows, offs, total = _encode_measured(enc, cols, n, dev)
    assert total == want.size
    assert np.array_equal(offs.cpu().numpy(), want_offs)
    assert np.array_equal(rows[:total].cpu().numpy(), want)
    assert bool((rows[total:] == 0xEE).all())


@pytest.mark.parametrize("name,n,knobs", [("mixed", 3000, {}), ("mixed", 2000, {"str_max": 600}),
                                          ("nested", 1500, {"list_max": 200}), ("mixed", 0, {})])
def test_decode_bound_sizing_matches_oracle(oracle, dev, name, n, knobs):
    """decode_batch(sizing="bound"): outputs sized from the row bytes, one decode pass, trimmed
    after -- columns equal the oracle's decode and the measured path's buffers exactly."""
    from fury_amd.encoder import Encoders, column_to_host
    fields = SCHEMAS[name]
    host = gen_columns(name, fields, n, seed=41, **knobs)
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch(_dev_cols(host, dev), n)
    got = enc.decode_batch(batch, sizing="bound")
    ref = enc.decode_batch(batch)
    torch.cuda.synchronize()
    want, want_offs = oracle.encode(fields, host, n)
    assert_columns_equal(fields, [column_to_host(c) for c in got],
                         oracle.decode(fields, want, want_offs, n), n)
    for a, b in zip(got, ref):
        if a.offsets is not None:
            assert torch.equal(a.offsets, b.offsets)
        if a.values is not None and b.values is not None:
            assert a.values.numel() == b.values.numel()
    with pytest.raises(ValueError):
        enc.decode_batch(batch, sizing="guess")


# ---- round 2: wide flat schemas (> 16 fields: the LDS-DMA encode / ticketed decode kernels) ----
def _wide_fields(ncols):
    """ncols fields cycling int32 / int64 / double / String / List<Long> / boolean / String,
    all nullable (boxed Java types), named so Descriptor order = index order."""
    kinds = [T.INT32, T.INT64, T.FLOAT64, T.STRING, "list", T.BOOL, T.STRING]
    out = []
    for i in range(ncols):
        k = kinds[i % len(kinds)]
        name = f"f{i:03d}"
        out.append(T.array_field(name, T.INT64) if k == "list" else T.field(name, k))
    return out


@pytest.mark.parametrize("ncols,n,str_max", [(17, 3001, 40), (33, 2049, 64), (64, 1500, 24),
                                             (17, 700, 600), (64, 257, 300)])
def test_wide_var_schemas_bit_exact(oracle, dev, ncols, n, str_max):
    """17 / 33 / 64-field flat schemas with strings, lists and 10 % nulls (long strings in the
    str_max = 300 / 600 cases overflow the LDS tiles): encode (measure + encode), encode_measured,
    decode, rows_to_arrow, and the sizing-pass decode mode — all oracle-exact."""
    from fury_amd import _native as N
    from fury_amd.encoder import ArrowWriter, Encoders, column_to_host
    fields = _wide_fields(ncols)
    host = gen_columns("wide", fields, n, seed=ncols + n, null_pct=10, str_max=str_max,
                       list_max=12, list_null_pct=10, elem_null_pct=10)
    enc, batch, _ = _roundtrip(oracle, None, n, dev, fields=fields, cols=host)
    want, want_offs = oracle.encode(fields, host, n)
    cols = _dev_cols(host, dev)
    rows, offs, total = _encode_measured(enc, cols, n, dev)
    assert np.array_equal(offs.cpu().numpy(), want_offs)
    assert np.array_equal(rows[:total].cpu().numpy(), want)
    assert bool((rows[total:] == 0xEE).all())
    ref = oracle.decode(fields, want, want_offs, n)
    w = ArrowWriter(enc)
    w.write(batch)
    assert_columns_equal(fields, [column_to_host(c) for c in w.finish()], ref, n)
    dec = [column_to_host(c) for c in enc.decode_batch(batch, sizing="bound")]
    assert_columns_equal(fields, dec, ref, n)
    assert N.lib().fury_get_tuning(b"lookback_timeouts") == 0


@pytest.mark.parametrize("engine", [1, 2, 0])
@pytest.mark.parametrize("ncols,n,str_max", [(17, 3001, 40), (33, 2049, 64), (64, 700, 300),
                                             (200, 300, 24)])
def test_wide_plan_engines(oracle, dev, engine, ncols, n, str_max):
    """The plan decode (fury_decode_prepare / execute, what decode_batch runs for 17-256 flat
    fields) through each engine of tuning wide_engine -- 1 the wide tiles, 2 the row walk (field
    groups past 16 counted fields), 0 auto by the average row -- decodes to the oracle's columns."""
    from fury_amd import _native as N
    from fury_amd.encoder import column_to_host
    fields = _wide_fields(ncols)
    host = gen_columns("wide", fields, n, seed=ncols * 3 + n, null_pct=10, str_max=str_max,
                       list_max=12, list_null_pct=10, elem_null_pct=10)
    enc, batch, _ = _roundtrip(oracle, None, n, dev, fields=fields, cols=host)
    want, want_offs = oracle.encode(fields, host, n)
    ref = oracle.decode(fields, want, want_offs, n)
    L = N.lib()
    old = L.fury_get_tuning(b"wide_engine")
    assert L.fury_set_tuning(b"wide_engine", engine) == 0
    try:
        dec = [column_to_host(c) for c in enc.decode_batch(batch)]
    finally:
        L.fury_set_tuning(b"wide_engine", old)
    assert_columns_equal(fields, dec, ref, n)


@pytest.mark.parametrize("engine", [1, 2, 0])
@pytest.mark.parametrize("ncols,n,str_max", [(17, 2049, 40), (33, 1500, 64), (64, 700, 300),
                                             (200, 300, 24)])
def test_wide_encode_engines(oracle, dev, engine, ncols, n, str_max):
    """The encode of a 17-256-field flat schema through each engine of tuning wide_enc_engine --
    1 the wide tiles, 2 the row-walk encode (rowenc.hip), 0 auto by the estimated row -- measured
    and two-pass: the rows are the oracle's bytes."""
    from fury_amd import _native as N
    from fury_amd.encoder import Encoders
    fields = _wide_fields(ncols)
    host = gen_columns("wide", fields, n, seed=ncols * 5 + n, null_pct=10, str_max=str_max,
                       list_max=12, list_null_pct=10, elem_null_pct=10)
    want, want_offs = oracle.encode(fields, host, n)
    L = N.lib()
    old = L.fury_get_tuning(b"wide_enc_engine")
    assert L.fury_set_tuning(b"wide_enc_engine", engine) == 0
    try:
        enc = Encoders.bean(fields, device=dev)
        cols = _dev_cols(host, dev)
        batch = enc.encode_batch(cols, n)
        rows, offs, total = _encode_measured(enc, cols, n, dev)
    finally:
        L.fury_set_tuning(b"wide_enc_engine", old)
    assert np.array_equal(batch.row_offsets.cpu().numpy(), want_offs)
    assert np.array_equal(batch.rows.cpu().numpy(), want)
    assert np.array_equal(offs.cpu().numpy(), want_offs)
    assert np.array_equal(rows[:total].cpu().numpy(), want)


_REG_MODES = {"bytes": [T.INT32, T.STRING, T.BOOL, T.INT64, T.STRING, T.FLOAT64],
              "lists": [T.INT64, "list", T.BOOL, T.FLOAT32, "list"],
              "all": [T.INT32, T.STRING, "list", T.BOOL, T.INT16]}


@pytest.mark.parametrize("mode", sorted(_REG_MODES))
@pytest.mark.parametrize("ncols", list(range(1, 17)))
def test_reg_decode_every_width_and_kind_mode(oracle, dev, mode, ncols):
    """The register-staged decode instances: K rounded up to {2, 3, 4, 6, 8, 12, 16} (padding
    columns), the kind modes strings-only / lists-only / all (var_dev.h kind_of), and both tile
    sizes (one vs several sequence columns) -- decode and rows->Arrow oracle-exact."""
    from fury_amd.encoder import ArrowWriter, column_to_host
    kinds = _REG_MODES[mode]
    fields = []
    for i in range(ncols):
        k = kinds[i % len(kinds)]
        fields.append(T.array_field(f"f{i:02d}", T.INT64) if k == "list" else T.field(f"f{i:02d}", k))
    n = 1300
    host = gen_columns("wide", fields, n, seed=ncols * 7 + len(mode), null_pct=10, str_max=40,
                       list_max=9, list_null_pct=10, elem_null_pct=10)
    enc, batch, _ = _roundtrip(oracle, None, n, dev, fields=fields, cols=host)
    want, want_offs = oracle.encode(fields, host, n)
    ref = oracle.decode(fields, want, want_offs, n)
    w = ArrowWriter(enc)
    w.write(batch)
    assert_columns_equal(fields, [column_to_host(c) for c in w.finish()], ref, n)


@pytest.mark.parametrize("pipe", [1, 2])
@pytest.mark.parametrize("mode", sorted(_REG_MODES))
@pytest.mark.parametrize("ncols,n", [(3, 1300), (5, 1300), (6, 400_001)])
def test_var_decode_pipe(oracle, dev, pipe, mode, ncols, n):
    """The persistent two-stage decode (tuning var_dec_pipe: 1 the planned tiles, two stages; 2
    half stages), instances K = 3 and 6: workgroups take tiles blockIdx, + gridDim, ... -- 400k rows
    give every workgroup several tiles -- and the decode and rows->Arrow are oracle-exact."""
    from fury_amd import _native as N
    from fury_amd.encoder import ArrowWriter, column_to_host
    kinds = _REG_MODES[mode]
    fields = []
    for i in range(ncols):
        k = kinds[i % len(kinds)]
        fields.append(T.array_field(f"f{i:02d}", T.INT64) if k == "list" else T.field(f"f{i:02d}", k))
    host = gen_columns("wide", fields, n, seed=ncols * 11 + len(mode), null_pct=10, str_max=40,
                       list_max=9, list_null_pct=10, elem_null_pct=10)
    L = N.lib()
    assert L.fury_set_tuning(b"var_dec_pipe", pipe) == 0
    try:
        enc, batch, _ = _roundtrip(oracle, None, n, dev, fields=fields, cols=host)
        want, want_offs = oracle.encode(fields, host, n)
        w = ArrowWriter(enc)
        w.write(batch)
        assert_columns_equal(fields, [column_to_host(c) for c in w.finish()],
                             oracle.decode(fields, want, want_offs, n), n)
    finally:
        L.fury_set_tuning(b"var_dec_pipe", 0)
    assert L.fury_get_tuning(b"lookback_timeouts") == 0


def test_wide_var_schema_large_batch(oracle, dev):
    """A 40-field schema over 300k rows (>1,000 workgroups chained by the look-back)."""
    fields = _wide_fields(40)
    n = 300_000
    host = gen_columns("wide", fields, n, seed=4, null_pct=10, str_max=20, list_max=6)
    _roundtrip(oracle, None, n, dev, fields=fields, cols=host)


# ---- round 2: rows as Java's RowEncoder.encode(obj) writes them (reused buffer) ---------------
def _nullable_fixed_fields():
    return [T.field("a", T.INT32), T.field("b", T.INT64), T.field("c", T.FLOAT64),
            T.field("d", T.BOOL), T.field("e", T.INT16), T.field("f", T.FLOAT32)]


@pytest.mark.parametrize("name,n", [("mixed", 3000), ("narrow", 1200), ("beanb", 900),
                                    ("nullable_fixed", 2000), ("wide33", 800), ("nested_deep", 400)])
def test_decode_java_encode_rows_with_stale_null_slots(oracle, dev, name, n):
    """RowEncoder.encode(obj) reuses one buffer (Encoders.java:146,191-198), so a null field's slot
    keeps the previous row's value (for a string or list: an offset/size that may point past this
    row).  The device must decode such rows exactly like the reference's fromRow, which never
    looks at a null field's slot: equal to oracle.decode of the same rows and to the decode of
    the canonical (toRow) rows."""
    from fury_amd.encoder import Encoders, RowBatch, column_to_host
    if name == "nullable_fixed":
        fields = _nullable_fixed_fields()
        host = gen_columns("nf", fields, n, seed=n, null_pct=30)
    elif name == "wide33":
        fields = _wide_fields(33)
        host = gen_columns("wide", fields, n, seed=n, null_pct=30, str_max=40)
    elif name == "nested_deep":
        from fury_amd.beans import beans_to_columns
        fields = _nested_fields()
        host = beans_to_columns(fields, _nested_beans(n, seed=11))
    else:
        fields = SCHEMAS[name]
        host = gen_columns(name, fields, n, seed=n, null_pct=30)
    canon, offs = oracle.encode(fields, host, n)
    java, joffs = oracle.encode(fields, host, n, reuse=True)
    assert np.array_equal(offs, joffs)
    assert not np.array_equal(canon, java), "the case must contain stale null slots"
    enc = Encoders.bean(fields, device=dev)
    rows = torch.from_numpy(java.copy()).to(dev)
    roffs = None if enc.schema().is_fixed else torch.from_numpy(joffs).to(dev)
    dec = [column_to_host(c) for c in enc.decode_batch(RowBatch(rows, roffs, n, enc.schema_hash))]
    want = oracle.decode(fields, java, joffs, n)
    assert_columns_equal(fields, dec, want, n)
    assert_columns_equal(fields, dec, oracle.decode(fields, canon, offs, n), n)
    if not enc.nested:
        from fury_amd.encoder import ArrowWriter
        w = ArrowWriter(enc)
        w.write(RowBatch(rows, roffs, n, enc.schema_hash))
        assert_columns_equal(fields, [column_to_host(c) for c in w.finish()], want, n)


# ---- round 2: explicit side streams, malformed rows under bound sizing ----------------------
@pytest.mark.parametrize("sizing", ["measure", "bound"])
def test_side_stream_encode_decode(oracle, dev, sizing):
    """encode_batch / decode_batch / unframe on a torch.cuda.Stream() that is not the current
    stream, held back by a spin kernel: output allocations and host reads wait for that stream,
    so sizes and bytes are still the oracle's."""
    from fury_amd.encoder import Encoders, column_to_host
    fields = SCHEMAS["mixed"]
    n = 20_000
    host = gen_columns("mixed", fields, n, seed=12)
    enc = Encoders.bean(fields, device=dev)
    cols = _dev_cols(host, dev)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    if hasattr(torch.cuda, "_sleep"):
        with torch.cuda.stream(s):
            torch.cuda._sleep(50_000_000)
    batch = enc.encode_batch(cols, n, stream=s)
    dec = enc.decode_batch(batch, stream=s, sizing=sizing)
    s.synchronize()
    want, want_offs = oracle.encode(fields, host, n)
    assert np.array_equal(batch.rows.cpu().numpy(), want)
    assert_columns_equal(fields, [column_to_host(c) for c in dec],
                         oracle.decode(fields, want, want_offs, n), n)


def test_bound_decode_falls_back_when_payload_exceeds_rows(oracle, dev):
    """Slots may point at any bytes of the batch (the reference reads the shared buffer): ten rows
    whose s1 covers the WHOLE batch make the column's payload ten times the row bytes, past the
    "bound" sizing -- decode_batch(sizing="bound") must re-decode with exact sizes and equal
    "measure" and the oracle.  A slot running past the batch raises IndexOutOfBoundsException
    under both sizings (test_bounds.py covers the rest)."""
    from fury_amd.encoder import Encoders, IndexOutOfBoundsException, RowBatch, column_to_host
    fields = SCHEMAS["mixed"]
    n = 1000
    host = gen_columns("mixed", fields, n, seed=2)
    enc = Encoders.bean(fields, device=dev)
    b = enc.encode_batch(_dev_cols(host, dev), n)
    total = b.rows.numel()
    offs = b.row_offsets.cpu().numpy()
    rows = b.rows.cpu().numpy().copy()
    slot_at = 8 + 8 * 3                               # s1's slot (field 3)
    for r in range(500, 510):
        base = int(offs[r])
        rows[base] &= ~np.uint8(1 << 3)               # s1 not null
        rel = (-base) & 0xFFFFFFFF
        rows[base + slot_at:base + slot_at + 8] = np.frombuffer(
            np.array([(rel << 32) | total], np.uint64).tobytes(), np.uint8)
    batch = RowBatch(torch.from_numpy(rows).to(dev), b.row_offsets, n, enc.schema_hash)
    got = enc.decode_batch(batch, sizing="bound")
    ref = enc.decode_batch(batch, sizing="measure")
    need = int(got[3].offsets[n])
    assert need > 10 * total - 1 and got[3].values.numel() >= need
    assert torch.equal(got[3].offsets, ref[3].offsets)
    assert torch.equal(got[3].values[:need], ref[3].values[:need])
    assert_columns_equal(fields, [column_to_host(c) for c in got],
                         oracle.decode(fields, rows, offs, n), n)
    r = 700
    base = int(offs[r])
    rows2 = rows.copy()
    rows2[base] &= ~np.uint8(1 << 3)
    rows2[base + slot_at:base + slot_at + 8] = np.frombuffer(
        np.array([(56 << 32) | total], np.uint64).tobytes(), np.uint8)   # runs past the batch
    bad = RowBatch(torch.from_numpy(rows2).to(dev), b.row_offsets, n, enc.schema_hash)
    for sizing in ("bound", "measure"):
        with pytest.raises(IndexOutOfBoundsException, match="row 700 "):
            enc.decode_batch(bad, sizing=sizing)


def test_c5_shard_size_property(oracle, dev):
    """C5 per-GPU shard: 12.5M Struct-100 rows (the last of 8 shards of 100M, global rows
    87.5M..100M, generated in HBM keyed by global row): decode(encode(cols)) == cols, every row
    bitmap is zero, every row's slots == the interleaved columns (checked in 1M-row chunks), and
    a sample of rows equals the oracle's encode of the same global rows."""
    from fury_amd.encoder import Encoders
    from fury_amd.shard import strong_shard
    from fury_amd.workloads import gen_columns_torch
    fields = SCHEMAS["struct100"]
    start, n = strong_shard(100_000_000, 8, 7)
    cols = gen_columns_torch("struct100", fields, n, seed=1234, start=start, device=dev)
    enc = Encoders.bean(fields, device=dev)
    b = enc.encode_batch(cols, n)
    r = b.rows.view(n, 816)
    step = 1_000_000
    for c0 in range(0, n, step):
        c1 = min(n, c0 + step)
        assert int(r[c0:c1, :16].abs().sum()) == 0
        slots = r[c0:c1, 16:].contiguous().view(torch.int64).view(c1 - c0, 100)
        assert torch.equal(slots, torch.stack([c.values.view(torch.int64)[c0:c1] for c in cols], 1))
    dec = enc.decode_batch(b, validity=False)
    for c, d in zip(cols, dec):
        assert torch.equal(c.values.view(torch.uint8), d.values)
    del dec
    for off in (0, n // 2, n - 300):
        host = gen_columns("struct100", fields, 300, seed=1234, start=start + off)
        want, _ = oracle.encode(fields, host, 300)
        assert np.array_equal(b.rows[off * 816:(off + 300) * 816].cpu().numpy(), want)


# ---- round 2: ArrayEncoder / MapEncoder batches on the device ---------------------------------
def _bar_item(name="item"):
    return T.struct_field(name, SCHEMAS["bar"])


def test_array_encoder_known_answer_224(dev):
    """ArrayEncoderTest.testListEncoder: 5 Bars -> encode() is 224 bytes; device bytes equal the
    bean restatement; decode(encode(x)) == x; toArray/fromArray round trip."""
    from fury_amd.encoder import Encoders
    from oracle import bean_oracle as B
    elem = _bar_item()
    enc = Encoders.array_encoder(elem, device=dev)
    bars = [{"f1": k, "f2": f"i{k}"} for k in range(5)]
    bs = enc.encode(bars)
    assert len(bs) == 224
    assert bs[:-8] == B.encode_array(elem, bars) and bs[-8:] == bytes(8)
    assert enc.decode(bs) == bars
    assert enc.from_array(enc.to_array(bars)) == bars


def test_array_encoder_known_answer_1576(dev):
    """ArrayEncoderTest.testNestListEncoder: List<List<List<Bar>>> -> 1576 bytes."""
    from fury_amd.encoder import Encoders
    from oracle import bean_oracle as B
    l1 = T.Field("item", T.LIST, True, (_bar_item(),))
    l2 = T.Field("item", T.LIST, True, (l1,))
    vals = [[[{"f1": k, "f2": f"s{k}"} for k in range(3)] for _ in range(i)] for i in range(5)]
    enc = Encoders.array_encoder(l2, device=dev)
    bs = enc.encode(vals)
    assert len(bs) == 1576
    assert bs[:-8] == B.encode_array(l2, vals)
    assert enc.decode(bs) == vals


def test_array_encoder_known_answer_10824(dev):
    """ArrayEncoderTest.testNestArrayWithMapEncoder: List<List<Map<Foo, List<Bar>>>> -> 10824."""
    from fury_amd.encoder import Encoders
    from oracle import bean_oracle as B
    key = T.Field("key", T.STRUCT, False, tuple(SCHEMAS["foo"]))
    value = T.Field("value", T.LIST, True, (_bar_item(),))
    m = T.Field("item", T.MAP, True, (key, value))
    l1 = T.Field("item", T.LIST, True, (m,))
    foo = {"f1": 2, "f2": "str", "f3": ["a", "b", "c"], "f4": [("k1", 1), ("k2", 2)],
           "f5": {"f1": 1, "f2": "str"}}
    vals = [[[(foo, [{"f1": j, "f2": f"x{j}"}])] for j in range(3)] for _ in range(10)]
    enc = Encoders.array_encoder(l1, device=dev)
    bs = enc.encode(vals)
    assert len(bs) == 10824
    assert bs[:-8] == B.encode_array(l1, vals)
    assert enc.decode(bs) == vals


def _collection_batch_case(kind, n, rng):
    bar = _bar_item()
    if kind == "list_bar":
        elem = bar
        vals = [[None if rng.random() < 0.1 else {"f1": int(rng.integers(-99, 99)),
                                                  "f2": None if rng.random() < 0.2 else "s" * int(rng.integers(0, 12))}
                 for _ in range(int(rng.integers(0, 6)))] for _ in range(n)]
    elif kind == "list_long":
        elem = T.field("item", T.INT64)
        vals = [[None if rng.random() < 0.1 else int(x) for x in rng.integers(-2**62, 2**62, int(rng.integers(0, 70)))]
                for _ in range(n)]
    elif kind == "list_str":
        elem = T.field("item", T.STRING)
        vals = [[None if rng.random() < 0.1 else "é" * int(rng.integers(0, 9)) for _ in range(int(rng.integers(0, 5)))]
                for _ in range(n)]
    else:   # list of list<int32>
        elem = T.Field("item", T.LIST, True, (T.field("item", T.INT32),))
        vals = [[None if rng.random() < 0.1 else [int(x) for x in rng.integers(0, 9, int(rng.integers(0, 4)))]
                 for _ in range(int(rng.integers(0, 4)))] for _ in range(n)]
    return elem, vals


@pytest.mark.parametrize("kind", ["list_bar", "list_long", "list_str", "list_list"])
def test_array_encoder_batch_vs_oracle(oracle, dev, kind):
    """A batch of top-level arrays (entry i = toArray(values[i])) encoded on the device: bytes and
    offsets == the columnar C restatement's LIST field bytes (row[16:], same layout), decode ==
    the oracle's decoded column, encode_measured == encode."""
    from fury_amd.beans import beans_to_columns, value_at
    from fury_amd.encoder import Encoders, column_to_host
    n = 1500
    elem, vals = _collection_batch_case(kind, n, np.random.default_rng(len(kind)))
    enc = Encoders.array_encoder(elem, device=dev)
    col = beans_to_columns([enc.field()], [{"value": v} for v in vals])[0]
    col.validity = None
    batch = enc.encode_batch([column_to_device_host(col, dev)], n)
    lf = enc.field()
    rows, offs = oracle.encode([lf], [col], n)
    sizes = np.diff(offs) - 16
    want = np.concatenate([rows[offs[i] + 16:offs[i + 1]] for i in range(n)])
    assert np.array_equal(batch.rows.cpu().numpy(), want)
    assert np.array_equal(np.diff(batch.row_offsets.cpu().numpy()), sizes)
    dec = column_to_host(enc.decode_batch(batch)[0])
    assert [value_at(lf, dec, i) for i in range(n)] == vals
    rows2 = torch.full((want.size + 64,), 0xEE, dtype=torch.uint8, device=dev)
    offs2 = torch.empty(n + 1, dtype=torch.int64, device=dev)
    enc.encode_measured_into([column_to_device_host(col, dev)], n, rows2[:want.size], offs2)
    assert torch.equal(rows2[:want.size], batch.rows) and torch.equal(offs2, batch.row_offsets)


def column_to_device_host(col, dev):
    from fury_amd.encoder import column_to_device
    return column_to_device(col, dev)


@pytest.mark.parametrize("kind", ["str_bar", "str_listlist_bar", "str_list_int", "bar_bar",
                                  "str_list_map"])
def test_map_encoder_shapes(oracle, dev, kind):
    """MapEncoderTest shapes (testMapEncoder, testNestListEncoder, testSimpleNestArrayWith-
    MapEncoder1, testKVStructMap, testNestArrayWithMapEncoder): toMap bytes == the bean
    restatement of MapEncoderBuilder, decode(encode(m)) == m, and the streaming form
    [int32 size][map] twice after a 1-byte offset decodes twice (CodecBuilderTest
    testStreamingEncode)."""
    from fury_amd.encoder import Encoders
    from oracle import bean_oracle as B
    bar = T.struct_field("value", SCHEMAS["bar"])
    skey = T.field("key", T.STRING)
    if kind == "str_bar":
        key, value = skey, bar
        m = [(f"i{k}", {"f1": k, "f2": f"i{k}"}) for k in range(5)]
    elif kind == "str_listlist_bar":
        key = skey
        value = T.Field("value", T.LIST, True, (T.Field("item", T.LIST, True, (_bar_item(),)),))
        m = [(str(i), [[{"f1": k, "f2": f"s{k}"} for k in range(3)] for _ in range(i)])
             for i in range(5)]
    elif kind == "str_list_int":
        key, value = skey, T.Field("value", T.LIST, True, (T.field("item", T.INT32),))
        m = [("k1", [1, 2])]
    elif kind == "bar_bar":
        key = T.Field("key", T.STRUCT, True, tuple(SCHEMAS["bar"]))
        value = bar
        m = [({"f1": 1, "f2": "a"}, {"f1": 2, "f2": None})]
    else:
        key = T.Field("key", T.STRUCT, True, tuple(SCHEMAS["foo"]))
        value = T.Field("value", T.LIST, True, (_bar_item(),))
        foo = {"f1": 2, "f2": "str", "f3": ["a", "b", "c"], "f4": [("k1", 1), ("k2", 2)],
               "f5": {"f1": 1, "f2": "str"}}
        inner = [[(foo, [{"f1": j, "f2": f"x{j}"}])] for j in range(3)]   # 3 one-entry maps
        value = T.Field("value", T.LIST, True, (T.map_field("item", key, value),))
        key = skey
        m = [(str(i), inner) for i in range(10)]
    enc = Encoders.map_encoder(key, value, device=dev)
    data = enc.encode(m)
    assert data == B.encode_map(key, value, m)
    assert enc.decode(data) == m and enc.from_map(enc.to_map(m)) == m
    buf = b"\xff" + enc.encode_stream(m) + enc.encode_stream(m)
    v1, p = enc.decode_stream(buf, 1)
    v2, p = enc.decode_stream(buf, p)
    assert v1 == m and v2 == m and p == len(buf)


def test_map_encoder_batch_vs_oracle(oracle, dev):
    """A batch of 3,000 top-level maps<String, Long> with null values: device bytes == the MAP
    field's bytes in the C restatement's rows, decode == values."""
    from fury_amd.beans import beans_to_columns, value_at
    from fury_amd.encoder import Encoders, column_to_host
    rng = np.random.default_rng(4)
    n = 3000
    vals = [[("k" * int(rng.integers(1, 9)), None if rng.random() < 0.2 else int(rng.integers(-9, 9)))
             for _ in range(int(rng.integers(0, 7)))] for _ in range(n)]
    enc = Encoders.map_encoder(T.field("key", T.STRING), T.field("value", T.INT64), device=dev)
    mf = enc._field
    col = beans_to_columns([mf], [{"value": v} for v in vals])[0]
    col.validity = None
    batch = enc.encode_batch([column_to_device_host(col, dev)], n)
    rows, offs = oracle.encode([mf], [col], n)
    want = np.concatenate([rows[offs[i] + 16:offs[i + 1]] for i in range(n)])
    assert np.array_equal(batch.rows.cpu().numpy(), want)
    dec = column_to_host(enc.decode_batch(batch)[0])
    assert [value_at(mf, dec, i) for i in range(n)] == vals


# ---- round 2: schemas wider than the kernel argument block (column table in device memory) ----
@pytest.mark.parametrize("ncols,n", [(300, 1500), (316, 777), (400, 1500), (1000, 129)])
def test_wide_fixed_fields(oracle, dev, ncols, n):
    """300 .. 1000 fixed-width fields (int8..int64, float, double, bool, date, timestamp; every
    third one nullable): beyond the argument block's 128 columns the general tile kernel reads the
    column table the host uploaded for the call; beyond 315 the column-block kernels (64 rows x 64
    fields per workgroup) take over.  Encode / decode / rows_to_arrow oracle-exact."""
    from fury_amd.encoder import ArrowWriter, column_to_host
    kinds = [T.INT64, T.FLOAT64, T.INT32, T.BOOL, T.INT16, T.FLOAT32, T.INT8, T.DATE32, T.TIMESTAMP]
    fields = [(T.field if i % 3 == 0 else T.not_null_field)(f"f{i:04d}", kinds[i % len(kinds)])
              for i in range(ncols)]
    host = gen_columns("wide", fields, n, seed=ncols, null_pct=15)
    enc, batch, _ = _roundtrip(oracle, None, n, dev, fields=fields, cols=host)
    assert enc.schema().is_fixed
    assert enc.schema().fixed_size == (ncols + 63) // 64 * 8 + 8 * ncols
    want, offs = oracle.encode(fields, host, n)
    w = ArrowWriter(enc)
    w.write(batch)
    assert_columns_equal(fields, [column_to_host(c) for c in w.finish()],
                         oracle.decode(fields, want, offs, n), n)


@pytest.mark.parametrize("ncols,n", [(100, 2000), (200, 700), (256, 300), (257, 500), (300, 900)])
def test_wide_var_schemas_beyond_arg_block(oracle, dev, ncols, n):
    """100 .. 300-field schemas with strings, lists, bools and nulls (multi-word row null bitmaps):
    encode (measure + encode), encode_measured, decode and rows_to_arrow oracle-exact.  Beyond 256
    fields the generic engine (row interpreter encode, plan-API decode) runs them."""
    from fury_amd.encoder import ArrowWriter, column_to_host
    fields = _wide_fields(ncols)
    host = gen_columns("wide", fields, n, seed=ncols, null_pct=20, str_max=48, list_max=9,
                       list_null_pct=10, elem_null_pct=10)
    enc, batch, _ = _roundtrip(oracle, None, n, dev, fields=fields, cols=host)
    want, want_offs = oracle.encode(fields, host, n)
    rows, offs, total = _encode_measured(enc, _dev_cols(host, dev), n, dev)
    assert np.array_equal(offs.cpu().numpy(), want_offs)
    assert np.array_equal(rows[:total].cpu().numpy(), want)
    w = ArrowWriter(enc)
    w.write(batch)
    assert_columns_equal(fields, [column_to_host(c) for c in w.finish()],
                         oracle.decode(fields, want, want_offs, n), n)


def _wide_nested_fields():
    """A bean with 60 scalar / string fields plus a nested bean, a map and a list of beans: 90
    schema nodes, beyond the argument block's 48."""
    fs = []
    for i in range(60):
        t = [T.INT64, T.STRING, T.INT32, T.FLOAT64, T.BOOL][i % 5]
        fs.append(T.field(f"a{i:02d}", t))
    inner = [T.field(f"i{j}", [T.INT32, T.STRING][j % 2]) for j in range(10)]
    fs.append(T.struct_field("b_inner", inner))
    fs.append(T.map_field("c_map", T.field("key", T.STRING), T.field("value", T.INT64)))
    fs.append(T.Field("d_list", T.LIST, True, (T.struct_field("item", SCHEMAS["bar"]),)))
    return fs


def _wide_nested_beans(fields, n, seed):
    rng = np.random.default_rng(seed)

    def val(f):
        if rng.random() < 0.15:
            return None
        t = f.type_id
        if t == T.INT64:
            return int(rng.integers(-2**62, 2**62))
        if t == T.INT32:
            return int(rng.integers(-2**31, 2**31))
        if t == T.FLOAT64:
            return float(rng.random())
        if t == T.BOOL:
            return bool(rng.integers(0, 2))
        if t == T.STRING:
            return "x" * int(rng.integers(0, 20))
        if t == T.STRUCT:
            return {c.name: val(c) for c in f.children}
        if t == T.MAP:
            return [("k" * int(rng.integers(1, 5)), int(rng.integers(0, 9)))
                    for _ in range(int(rng.integers(0, 4)))]
        if t == T.LIST:
            return [{"f1": int(rng.integers(0, 9)), "f2": "s" * int(rng.integers(0, 5))}
                    for _ in range(int(rng.integers(0, 4)))]
        raise ValueError(t)
    return [{f.name: val(f) for f in fields} for _ in range(n)]


@pytest.mark.parametrize("n", [1, 700, 5000])
def test_nested_schema_beyond_48_nodes(oracle, dev, n):
    """90-node nested schema: node table uploaded per call, decode cursors in the plan's count
    array.  Rows oracle-exact, decode == beans, the plan re-executes identically, Arrow ok."""
    from fury_amd.beans import beans_to_columns, columns_to_beans
    from fury_amd.encoder import Encoders, column_to_host
    fields = _wide_nested_fields()
    beans = _wide_nested_beans(fields, n, seed=n)
    host = beans_to_columns(fields, beans)
    enc = Encoders.bean(fields, device=dev)
    assert enc.nested
    batch = enc.encode_batch(_dev_cols(host, dev), n)
    want, want_offs = oracle.encode(fields, host, n)
    assert np.array_equal(batch.row_offsets.cpu().numpy(), want_offs)
    assert np.array_equal(batch.rows.cpu().numpy(), want)
    dec = [column_to_host(c) for c in enc.decode_batch(batch)]
    assert columns_to_beans(fields, dec, n) == beans
    assert_columns_equal(fields, dec, oracle.decode(fields, want, want_offs, n), n)
    rows, offs, total = _encode_measured(enc, _dev_cols(host, dev), n, dev)
    assert np.array_equal(rows[:total].cpu().numpy(), want)


# ---- round 2: level-by-level nested decode (levels.hip) vs the row interpreter ---------------
def _random_value(f, rng, depth=0):
    if f.nullable and rng.random() < 0.15:
        return None
    t = f.type_id
    if t == T.BOOL:
        return bool(rng.integers(0, 2))
    if t in (T.INT8, T.INT16, T.INT32, T.INT64, T.DATE32, T.TIMESTAMP):
        bits = {T.INT8: 7, T.INT16: 15, T.INT32: 31, T.DATE32: 31}.get(t, 62)
        return int(rng.integers(-2**bits, 2**bits))
    if t == T.FLOAT32:
        return float(np.float32(rng.standard_normal()))
    if t == T.FLOAT64:
        return float(rng.standard_normal())
    if t == T.STRING:
        return "".join(chr(97 + int(x)) for x in rng.integers(0, 26, int(rng.integers(0, 20))))
    if t == T.BINARY:
        return bytes(rng.integers(0, 256, int(rng.integers(0, 30))).astype(np.uint8))
    if t == T.DECIMAL:
        return bytes(rng.integers(0, 256, 16).astype(np.uint8))
    if t == T.STRUCT:
        return {c.name: _random_value(c, rng, depth + 1) for c in f.children}
    k = int(rng.integers(0, 6 if depth < 2 else 3))
    if t == T.LIST:
        return [_random_value(f.children[0], rng, depth + 1) for _ in range(k)]
    if t == T.MAP:
        return [(_random_value(f.children[0], rng, depth + 1),
                 _random_value(f.children[1], rng, depth + 1)) for _ in range(k)]
    raise ValueError(t)


def _engine_schemas():
    L = lambda name, e, nullable=True: T.Field(name, T.LIST, nullable, (e,))      # noqa: E731
    S = T.struct_field
    return {
        "nested7": _nested_fields(),
        "foo": SCHEMAS["foo"],
        "deep_lists": [L("a", L("item", L("item", T.field("item", T.BOOL)))),
                       L("b", L("item", T.field("item", T.STRING))), T.field("c", T.INT8)],
        "struct_chain": [S("s1", [S("s2", [S("s3", [T.field("x", T.INT16), T.field("d", T.DECIMAL),
                                                     T.field("b", T.BINARY)]),
                                           T.field("f", T.FLOAT32)]),
                                  L("l", S("item", [T.field("t", T.TIMESTAMP), T.field("q", T.BOOL)]))]),
                         T.not_null_field("k", T.INT64)],
        "maps": [T.map_field("m1", T.not_null_field("key", T.INT32),
                             L("value", T.field("item", T.STRING))),
                 L("lm", T.map_field("item", T.not_null_field("key", T.STRING),
                                     S("value", [T.field("v", T.FLOAT64), T.field("w", T.DATE32)]))),
                 T.map_field("m2", T.not_null_field("key", T.INT64), T.field("value", T.BOOL))],
    }


@pytest.mark.parametrize("name", ["nested7", "foo", "deep_lists", "struct_chain", "maps"])
def test_nested_decode_oracle_exact(oracle, dev, name):
    """The level-by-level nested decode returns the oracle's columns byte for byte on schemas with lists of lists of bools, struct chains
    with DECIMAL / BINARY / FLOAT32 / TIMESTAMP children, maps with scalar keys, lists of maps of
    structs; the plan re-executes identically; empty batch."""
    from fury_amd import _native as N
    from fury_amd.beans import beans_to_columns, columns_to_beans
    from fury_amd.encoder import Encoders, column_to_host
    fields = _engine_schemas()[name]
    rng = np.random.default_rng(len(name) * 7)
    n = 3001
    beans = [{f.name: _random_value(f, rng) for f in fields} for _ in range(n)]
    host = beans_to_columns(fields, beans)
    enc = Encoders.bean(fields, device=dev)
    assert enc.nested
    batch = enc.encode_batch(_dev_cols(host, dev), n)
    want, want_offs = oracle.encode(fields, host, n)
    assert np.array_equal(batch.rows.cpu().numpy(), want)
    dec = enc.decode_batch(batch)
    again = enc.decode_batch(batch)
    empty = enc.decode_batch(type(batch)(batch.rows, batch.row_offsets[:1], 0, batch.schema_hash))
    hdec = [column_to_host(c) for c in dec]
    assert_columns_equal(fields, hdec, oracle.decode(fields, want, want_offs, n), n)
    assert_columns_equal(fields, [column_to_host(c) for c in again], hdec, n)
    assert columns_to_beans(fields, hdec, n) == beans
    for f, c in zip(fields, empty):
        if c.offsets is not None:
            assert int(c.offsets[0].item()) == 0, f.name


def test_bound_calls_match(oracle, dev):
    """RowEncoder.bind_encode / bind_decode (argument blocks built once) issue the same calls as
    encode_measured_into / decode_into: oracle-exact rows and columns, repeatable."""
    from fury_amd.encoder import Encoders, column_to_host
    fields = SCHEMAS["mixed"]
    n = 5000
    host = gen_columns("mixed", fields, n, seed=4)
    enc = Encoders.bean(fields, device=dev)
    cols = _dev_cols(host, dev)
    batch = enc.encode_batch(cols, n)
    want, want_offs = oracle.encode(fields, host, n)
    rows = torch.zeros_like(batch.rows)
    offs = torch.zeros_like(batch.row_offsets)
    call = enc.bind_encode(cols, n, rows, offs, measured=True)
    call()
    call()
    assert np.array_equal(rows.cpu().numpy(), want) and np.array_equal(offs.cpu().numpy(), want_offs)
    out = enc.decode_batch(batch)
    ref = [column_to_host(c) for c in out]
    for c in out:
        for t in (c.values, c.validity, c.offsets):
            if t is not None:
                t.zero_()
    enc.bind_decode(batch, out)()
    assert_columns_equal(fields, [column_to_host(c) for c in out], ref, n)


def test_nested_large_batch_level_engine(oracle, dev):
    """600k depth-3 rows (several thousand workgroups per level, multi-block scans of every
    level's segments): device rows == C restatement, level-engine decode == its decode."""
    from fury_amd.beans import beans_to_columns
    from fury_amd.encoder import Encoders, column_to_host
    fields = _nested_fields()
    base = _nested_beans(20_000, seed=8)
    n = 600_000
    host = beans_to_columns(fields, (base * (n // len(base) + 1))[:n])
    enc = Encoders.bean(fields, device=dev)
    batch = enc.encode_batch(_dev_cols(host, dev), n)
    want, want_offs = oracle.encode(fields, host, n)
    assert np.array_equal(batch.row_offsets.cpu().numpy(), want_offs)
    assert np.array_equal(batch.rows.cpu().numpy(), want)
    dec = [column_to_host(c) for c in enc.decode_batch(batch)]
    assert_columns_equal(fields, dec, oracle.decode(fields, want, want_offs, n), n)


@pytest.mark.parametrize("order", ["short_first", "long_first", "alternating_blocks"])
def test_decode_skewed_row_sizes(oracle, dev, order):
    """Row sizes far from the batch average: the row-staged decode sizes its tiles, row stage and
    output images from the average (dec_tile_plan), so tiles of long rows read their tail rows from
    HBM and store columns that outgrow their image straight to HBM -- still bit-exact."""
    from fury_amd.beans import beans_to_columns
    fields = [T.field("a", T.INT32), T.field("s1", T.STRING), T.array_field("l", T.INT64),
              T.field("s2", T.BINARY)]
    rng = np.random.default_rng(11)
    n_short, n_long = 6000, 2500
    lengths = [0] * n_short + [1] * n_long
    if order == "long_first":
        lengths = lengths[::-1]
    elif order == "alternating_blocks":
        lengths = ([0] * 1500 + [1] * 600) * 4
    beans = []
    for i, longrow in enumerate(lengths):
        m = int(rng.integers(150, 400)) if longrow else int(rng.integers(0, 3))
        k = int(rng.integers(40, 90)) if longrow else int(rng.integers(0, 2))
        beans.append({
            "a": None if i % 13 == 5 else i,
            "s1": None if i % 17 == 2 else "".join(chr(97 + (i + j) % 26) for j in range(m)),
            "l": None if i % 19 == 4 else [None if j % 11 == 3 else i * 1000 + j for j in range(k)],
            "s2": bytes((i * 7 + j) & 0xFF for j in range(m // 2)),
        })
    cols = beans_to_columns(fields, beans)
    _roundtrip(oracle, None, len(beans), dev, fields=fields, cols=cols)


def _wide_all_kinds(ncols):
    """ncols fields cycling through every flat type the row format has -- each scalar, DECIMAL,
    STRING / BINARY and LIST of every fixed-width element type (nullable and not) -- all nullable
    at the top, named so Descriptor order = index order."""
    L = lambda name, e, en=True: T.Field(name, T.LIST, True, (T.Field("item", e, en, ()),))  # noqa: E731
    kinds = [T.BOOL, T.INT8, T.INT16, T.INT32, T.FLOAT32, T.DATE32, T.TIMESTAMP, T.DECIMAL,
             T.BINARY, T.STRING, T.FLOAT64, T.INT64, ("list", T.INT32, True),
             ("list", T.INT16, False), ("list", T.BOOL, True), ("list", T.INT8, True),
             ("list", T.FLOAT32, False), ("list", T.FLOAT64, True), ("list", T.DATE32, True),
             ("list", T.TIMESTAMP, True)]
    out = []
    for i in range(ncols):
        k = kinds[i % len(kinds)]
        name = f"f{i:03d}"
        out.append(L(name, k[1], k[2]) if isinstance(k, tuple) else T.field(name, k))
    return out


@pytest.mark.parametrize("ncols,n", [(20, 2001), (41, 1300), (100, 300)])
def test_wide_every_kind_bit_exact(oracle, dev, ncols, n):
    """17-256-field flat schemas carrying every flat type (the wide tiles: wide.hip): encode,
    encode_measured, decode, rows_to_arrow and the bound-sized decode == the oracle."""
    from fury_amd.encoder import ArrowWriter, column_to_host
    fields = _wide_all_kinds(ncols)
    host = gen_columns("wide", fields, n, seed=ncols * 3 + n, null_pct=10, str_max=30,
                       list_max=11, list_null_pct=10, elem_null_pct=10)
    enc, batch, _ = _roundtrip(oracle, None, n, dev, fields=fields, cols=host)
    want, want_offs = oracle.encode(fields, host, n)
    rows, offs, total = _encode_measured(enc, _dev_cols(host, dev), n, dev)
    assert np.array_equal(offs.cpu().numpy(), want_offs)
    assert np.array_equal(rows[:total].cpu().numpy(), want)
    ref = oracle.decode(fields, want, want_offs, n)
    w = ArrowWriter(enc)
    w.write(batch)
    assert_columns_equal(fields, [column_to_host(c) for c in w.finish()], ref, n)
    dec = [column_to_host(c) for c in enc.decode_batch(batch, sizing="bound")]
    assert_columns_equal(fields, dec, ref, n)


@pytest.mark.parametrize("seed", list(range(30)))
def test_random_flat_schemas(oracle, dev, seed):
    """Random flat schemas (1-120 fields of every flat type, lists of fixed-width elements,
    random nullability): the fixed-width, register-staged and wide kernels, whichever the field
    count picks -- encode, decode and rows_to_arrow == the oracle."""
    from fury_amd.encoder import ArrowWriter, column_to_host
    rng = np.random.default_rng(5000 + seed)
    scal = [T.BOOL, T.INT8, T.INT16, T.INT32, T.INT64, T.FLOAT32, T.FLOAT64, T.DATE32,
            T.TIMESTAMP, T.STRING, T.BINARY, T.DECIMAL]
    elem = [T.BOOL, T.INT8, T.INT16, T.INT32, T.INT64, T.FLOAT32, T.FLOAT64]
    nf = int(rng.choice([1, 3, 7, 16, 17, 33, 64, 65, 120]))
    var_p = float(rng.choice([0.0, 0.3, 0.6]))
    fields = []
    for i in range(nf):
        nullable = bool(rng.integers(0, 3))
        if rng.random() < var_p:
            if rng.random() < 0.4:
                e = elem[int(rng.integers(0, len(elem)))]
                fields.append(T.Field(f"f{i:03d}", T.LIST, nullable,
                                      (T.Field("item", e, bool(rng.integers(0, 2)), ()),)))
            else:
                fields.append(T.Field(f"f{i:03d}", [T.STRING, T.BINARY, T.DECIMAL][int(rng.integers(0, 3))], nullable, ()))
        else:
            fields.append(T.Field(f"f{i:03d}", scal[int(rng.integers(0, 9))], nullable, ()))
    n = int(rng.integers(1, 1500))
    host = gen_columns("wide", fields, n, seed=seed, null_pct=10, str_max=int(rng.integers(1, 60)),
                       list_max=int(rng.integers(1, 20)), list_null_pct=10, elem_null_pct=10)
    enc, batch, _ = _roundtrip(oracle, None, n, dev, fields=fields, cols=host)
    want, want_offs = oracle.encode(fields, host, n)
    ref = oracle.decode(fields, want, want_offs, n)
    w = ArrowWriter(enc)
    w.write(batch)
    assert_columns_equal(fields, [column_to_host(c) for c in w.finish()], ref, n)
