"""TEST INFRASTRUCTURE ONLY — value-level (bean-level) pure-Python restatement of the Java row
writer for SMALL cases: nested beans, lists of beans, maps.  It exists to reproduce the
reference's own known answers (ArrayEncoderTest 224 / 1576 / 10824 bytes, the C++ RowTest
ToString answer) and to cross-check the columnar C restatement (row_oracle.c) on random data:
two independent restatements of the same Java source.

Values: struct -> dict(name -> value) (None = null), list -> list, map -> list of (k, v) pairs in
iteration order, STRING -> str (UTF-8), BINARY -> bytes, DECIMAL -> 16 raw bytes, BOOL -> bool,
ints -> int, floats -> float (FLOAT32 packed as IEEE single).

FMT = java/fury-format/src/main/java/org/apache/fury/format
"""
from __future__ import annotations

import struct
from typing import Any, List, Sequence

from oracle.oracle import (BINARY, BOOL, DATE32, DECIMAL, F, FLOAT32, FLOAT64, INT8, INT16,
                           INT32, INT64, LIST, MAP, STRING, STRUCT, TIMESTAMP, WIDTH)

_PACK = {INT8: "<b", INT16: "<h", INT32: "<i", INT64: "<q", FLOAT32: "<f", FLOAT64: "<d",
         DATE32: "<i", TIMESTAMP: "<q"}


def _bitmap_bytes(n: int) -> int:                  # BitUtils.calculateBitmapWidthInBytes
    return ((n + 63) // 64) * 8


def _round8(n: int) -> int:                        # BinaryWriter.roundNumberOfBytesToNearestWord
    return n if n % 8 == 0 else n + 8 - n % 8


class Buffer:
    """MemoryBuffer: zero-filled growable bytearray with a writer index."""

    def __init__(self):
        self.data = bytearray(16)
        self.writer_index = 0

    def grow(self, needed: int):                   # MemoryBuffer.grow
        length = self.writer_index + needed
        if length > len(self.data):
            self.data.extend(bytes(length * 2 - len(self.data)))

    def put(self, off: int, b: bytes):
        self.data[off:off + len(b)] = b


class Writer:
    """BinaryWriter + BinaryRowWriter / BinaryArrayWriter (FMT/row/binary/writer/*.java)."""

    def __init__(self, buf: Buffer, is_array: bool, num_fields: int = 0, elem: F = None):
        self.buf = buf
        self.is_array = is_array
        self.start = 0
        self.bytes_before_bitmap = 8 if is_array else 0
        if is_array:
            w = WIDTH.get(elem.type_id, -1)
            self.elem_size = 8 if w < 0 else w
        else:
            self.header = _bitmap_bytes(num_fields)
            self.fixed_size = self.header + 8 * num_fields

    def reset_row(self):                           # BinaryRowWriter.reset :76-84
        b = self.buf
        self.start = b.writer_index
        b.grow(self.fixed_size)
        b.writer_index += self.fixed_size
        b.put(self.start, bytes(self.header))

    def reset_array(self, n: int):                 # BinaryArrayWriter.reset :91-118
        b = self.buf
        self.start = b.writer_index
        self.header = 8 + _bitmap_bytes(n)
        data = n * self.elem_size
        fixed_part = _round8(data)
        b.grow(self.header + fixed_part)
        b.put(self.start, struct.pack("<q", n))
        b.put(self.start + 8, bytes(self.header - 8))
        b.put(self.start + self.header + data, bytes(fixed_part - data))
        b.writer_index += self.header + fixed_part

    def offset(self, i: int) -> int:
        if self.is_array:
            return self.start + self.header + i * self.elem_size
        return self.start + self.header + 8 * i

    def set_null_at(self, i: int):
        p = self.start + self.bytes_before_bitmap + (i >> 3)
        self.buf.data[p] |= 1 << (i & 7)

    def set_not_null_at(self, i: int):
        p = self.start + self.bytes_before_bitmap + (i >> 3)
        self.buf.data[p] &= ~(1 << (i & 7)) & 0xFF

    def write_long(self, i: int, v: bytes):        # BinaryWriter.write(long/double)
        self.buf.put(self.offset(i), v)

    def write_narrow(self, i: int, v: bytes):
        off = self.offset(i)
        if self.is_array:
            self.set_not_null_at(i)
        else:
            self.buf.put(off, bytes(8))
        self.buf.put(off, v)

    def set_offset_and_size(self, i: int, absolute: int, size: int):
        rel = absolute - self.start
        self.write_long(i, struct.pack("<Q", ((rel << 32) | (size & 0xFFFFFFFF)) & (2**64 - 1)))

    def write_unaligned(self, i: int, data: bytes):  # :187-194
        b = self.buf
        n = len(data)
        rounded = _round8(n)
        b.grow(rounded)
        if n & 7:
            b.put(b.writer_index + ((n >> 3) << 3), bytes(8))
        b.put(b.writer_index, data)
        self.set_offset_and_size(i, b.writer_index, n)
        b.writer_index += rounded

    def write_directly(self, v: int):
        self.buf.grow(8)
        self.buf.put(self.buf.writer_index, struct.pack("<q", v))
        self.buf.writer_index += 8


def serialize(w: Writer, i: int, f: F, v: Any):
    """BaseBinaryEncoderBuilder.serializeFor (FMT/encoder/BaseBinaryEncoderBuilder.java:138-223)."""
    if v is None:
        w.set_null_at(i)
        return
    t = f.type_id
    if t == BOOL:
        w.write_narrow(i, bytes([1 if v else 0]))
    elif t in (INT8, INT16, INT32, FLOAT32, DATE32):
        w.write_narrow(i, struct.pack(_PACK[t], v))
    elif t in (INT64, FLOAT64, TIMESTAMP):
        w.write_long(i, struct.pack(_PACK[t], v))
    elif t == STRING:
        w.write_unaligned(i, v.encode("utf-8"))
    elif t == BINARY:
        w.write_unaligned(i, bytes(v))
    elif t == DECIMAL:
        b = w.buf
        b.grow(16)
        b.put(b.writer_index, bytes(v))
        w.set_offset_and_size(i, b.writer_index, 16)
        b.writer_index += 16
    elif t == LIST:
        offset = w.buf.writer_index
        aw = Writer(w.buf, True, elem=f.children[0])
        _serialize_array(aw, f.children[0], v)
        w.set_offset_and_size(i, offset, w.buf.writer_index - offset)
    elif t == STRUCT:
        offset = w.buf.writer_index
        rw = Writer(w.buf, False, num_fields=len(f.children))
        rw.reset_row()
        to_row(rw, f.children, v)
        w.set_offset_and_size(i, offset, w.buf.writer_index - offset)
    elif t == MAP:                                 # serializeForMap :298-357
        offset = w.buf.writer_index
        w.write_directly(-1)
        kw = Writer(w.buf, True, elem=f.children[0])
        _serialize_array(kw, f.children[0], [k for k, _ in v])
        w.buf.put(offset, struct.pack("<q", w.buf.writer_index - kw.start))
        vw = Writer(w.buf, True, elem=f.children[1])
        _serialize_array(vw, f.children[1], [x for _, x in v])
        w.set_offset_and_size(i, offset, w.buf.writer_index - offset)
    else:
        raise ValueError(f"unsupported type {t}")


def _serialize_array(aw: Writer, elem: F, values: list):
    aw.reset_array(len(values))
    for j, x in enumerate(values):
        serialize(aw, j, elem, x)


def to_row(w: Writer, fields: Sequence[F], bean: dict):
    for i, f in enumerate(fields):
        serialize(w, i, f, bean.get(f.name))


def encode_row(fields: Sequence[F], bean: dict) -> bytes:
    """RowEncoder.toRow(bean).toBytes() (Encoders.java:88-93)."""
    buf = Buffer()
    w = Writer(buf, False, num_fields=len(fields))
    w.reset_row()
    to_row(w, fields, bean)
    return bytes(buf.data[w.start:buf.writer_index])


def encode_array(elem: F, values: list) -> bytes:
    """ArrayEncoder.toArray(values) bytes (Encoders.java:360-369)."""
    buf = Buffer()
    aw = Writer(buf, True, elem=elem)
    _serialize_array(aw, elem, values)
    return bytes(buf.data[aw.start:buf.writer_index])


def encode_map(key: F, value: F, pairs: list) -> bytes:
    """MapEncoder.toMap(map) bytes (FMT/encoder/MapEncoderBuilder.java:152-208): the key writer
    writes writeDirectly(-1) at its writer index, the key array, then patches that word with the
    key array's size; the value writer (same buffer) appends the value array.  Result =
    [int64 keyArrayBytes][key BinaryArray][value BinaryArray] (BinaryMap.java:30-37)."""
    buf = Buffer()
    start = buf.writer_index
    kw = Writer(buf, True, elem=key)
    kw.write_directly(-1)
    _serialize_array(kw, key, [k for k, _ in pairs])
    buf.put(start, struct.pack("<q", buf.writer_index - kw.start))
    vw = Writer(buf, True, elem=value)
    _serialize_array(vw, value, [v for _, v in pairs])
    return bytes(buf.data[start:buf.writer_index])


def decode_array(elem: F, data: bytes) -> list:
    """ArrayEncoder.fromArray of a top-level BinaryArray at offset 0."""
    return read_array(data, 0, elem)


def decode_map(key: F, value: F, data: bytes) -> list:
    """MapEncoder.fromMap of a top-level BinaryMap at offset 0 (BinaryMap.pointTo :62-77)."""
    kb = struct.unpack_from("<q", data, 0)[0]
    keys = read_array(data, 8, key)
    vals = read_array(data, 8 + kb, value)
    if len(keys) != len(vals):
        raise ValueError("key / value count mismatch (UnsupportedOperationException)")
    return list(zip(keys, vals))


# ---------------------------------------------------------------------------------------------
# Reader + C++ Row::ToString formatting (cpp/fury/row/row.cc), used for the row_test.cc known
# answer.
# ---------------------------------------------------------------------------------------------
def read_value(base: bytes, off_slot: int, f: F, is_null: bool, container: bytes):
    if is_null:
        return None
    t = f.type_id
    slot = container[off_slot:off_slot + 8]
    if t == BOOL:
        return slot[0] != 0
    if t in _PACK:
        n = WIDTH[t]
        return struct.unpack(_PACK[t], container[off_slot:off_slot + n])[0]
    oas = struct.unpack("<q", slot)[0]
    rel, size = oas >> 32, oas & 0xFFFFFFFF
    data = container[base + rel: base + rel + size]
    if t == STRING:
        return data.decode("utf-8")
    if t in (BINARY, DECIMAL):
        return bytes(data)
    if t == LIST:
        return read_array(container, base + rel, f.children[0])
    if t == STRUCT:
        return read_row(container, base + rel, f.children)
    if t == MAP:
        kb = struct.unpack("<q", container[base + rel: base + rel + 8])[0]
        keys = read_array(container, base + rel + 8, f.children[0])
        vals = read_array(container, base + rel + 8 + kb, f.children[1])
        return list(zip(keys, vals))
    raise ValueError(t)


def read_row(buf: bytes, base: int, fields: Sequence[F]) -> dict:
    hdr = _bitmap_bytes(len(fields))
    out = {}
    for i, f in enumerate(fields):
        null = (buf[base + (i >> 3)] >> (i & 7)) & 1
        out[f.name] = read_value(base, base + hdr + 8 * i, f, bool(null), buf)
    return out


def read_array(buf: bytes, base: int, elem: F) -> list:
    n = struct.unpack("<q", buf[base:base + 8])[0]
    hdr = 8 + _bitmap_bytes(n)
    w = WIDTH.get(elem.type_id, -1)
    es = 8 if w < 0 else w
    res = []
    for j in range(n):
        null = (buf[base + 8 + (j >> 3)] >> (j & 7)) & 1
        res.append(read_value(base, base + hdr + es * j, elem, bool(null), buf))
    return res


def _fmt(f: F, v) -> str:
    if v is None:
        return "null"
    t = f.type_id
    if t == STRUCT:
        return "{" + ", ".join(f"{c.name}={_fmt(c, v[c.name])}" for c in f.children) + "}"
    if t == LIST:
        return "[" + ", ".join(_fmt(f.children[0], x) for x in v) + "]"
    if t == MAP:
        return ("Map([" + ", ".join(_fmt(f.children[0], k) for k, _ in v) + "], [" +
                ", ".join(_fmt(f.children[1], x) for _, x in v) + "])")
    if t in (FLOAT32, FLOAT64):
        return f"{v:g}"
    return str(v)


def row_to_string(fields: Sequence[F], row: bytes) -> str:
    """Format like C++ fury::Row::ToString (cpp/fury/row/row.cc)."""
    return _fmt(F("", STRUCT, True, list(fields)), read_row(row, 0, fields))
