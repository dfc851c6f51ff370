"""Synthetic workloads of BASELINE.json's configs: schemas and seeded column generators.

Schemas are written in slot order (Descriptor order: lexicographic Java field name,
fury-core type/Descriptor.java:324-332) with TypeInference's nullability (primitives non-null,
boxed/String/List nullable; TypeInference.java:136-238).

Values come from SplitMix64 keyed by (seed, column, GLOBAL row index), so any row range (a shard
of a multi-GPU run) reproduces exactly the rows a single-GPU run would generate.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from .types import (BINARY, BOOL, DATE32, DECIMAL, FLOAT32, FLOAT64, INT8, INT16, INT32, INT64,
                    LIST, MAP, STRING, STRUCT, TIMESTAMP, Field, array_field, field,
                    infer_bean_schema, map_field, not_null_field, struct_field, type_width)


@dataclass
class Column:
    """Arrow-style column (include/fury_row.h ``fury_column``); arrays are numpy (host) or
    torch tensors (device).  ``child`` is a list: LIST -> [elements], STRUCT -> children,
    MAP -> [keys, values]."""
    values: Optional[object] = None
    validity: Optional[object] = None
    offsets: Optional[object] = None
    child: Optional[List["Column"]] = None


# ---------------------------------------------------------------------------------------------
# Schemas
# ---------------------------------------------------------------------------------------------
def struct100() -> List[Field]:
    """C2/C5: f00..f99, even int64 / odd float64, primitive (non-null).  Zero-padded names so
    lexicographic order = numeric order."""
    return [not_null_field(f"f{i:02d}", INT64 if i % 2 == 0 else FLOAT64) for i in range(100)]


def docs_struct() -> List[Field]:
    """C1: docs/benchmarks `Struct` (java/benchmark/.../data/Struct.java:136-175): 104 primitive
    fields f0..f103 typed int/long/float/double by i % 4, sorted by Java name (f0, f1, f10,
    f100, ...)."""
    kinds = [INT32, INT64, FLOAT32, FLOAT64]
    fs = [(f"f{i}", not_null_field(f"f{i}", kinds[i % 4])) for i in range(104)]
    fs.sort(key=lambda p: p[0])
    return [f for _, f in fs]


def mixed() -> List[Field]:
    """C3: a:Integer, b:Long, c:Double, s1..s3:String — all nullable."""
    return [field("a", INT32), field("b", INT64), field("c", FLOAT64),
            field("s1", STRING), field("s2", STRING), field("s3", STRING)]


def nested() -> List[Field]:
    """C4: id:long, score:double, vals:List<Long>."""
    return [not_null_field("id", INT64), not_null_field("score", FLOAT64),
            array_field("vals", INT64, elem_nullable=True)]


def narrow() -> List[Field]:
    """Every fixed-width and var-length scalar type the device path handles, all nullable."""
    return [field("a_bool", BOOL), field("b_byte", INT8), field("c_short", INT16),
            field("d_int", INT32), field("e_float", FLOAT32), field("f_date", DATE32),
            field("g_ts", TIMESTAMP), field("h_dec", DECIMAL), field("i_bin", BINARY),
            field("j_double", FLOAT64), field("k_ints", LIST, True, (field("item", INT32),)),
            field("l_shorts", LIST, True, (not_null_field("item", INT16),)),
            field("m_long", INT64)]


def bar() -> List[Field]:
    """RowEncoderTest.Bar {int f1; String f2} (FMTT/encoder/RowEncoderTest.java:82-92)."""
    return [not_null_field("f1", INT32), field("f2", STRING)]


def beanb() -> List[Field]:
    """fury-test-core BeanB (test/bean/BeanB.java:28-38)."""
    return [not_null_field("f1", INT16), field("f2", INT32), not_null_field("f3", INT64),
            field("f4", FLOAT32), not_null_field("f5", FLOAT64),
            array_field("int_arr", INT32, elem_nullable=False),
            array_field("int_list", INT32, elem_nullable=True)]


def foo() -> List[Field]:
    """RowEncoderTest.Foo {int f1; String f2; List<String> f3; Map<String,Integer> f4; Bar f5}."""
    return [not_null_field("f1", INT32), field("f2", STRING), array_field("f3", STRING),
            map_field("f4", field("key", STRING), field("value", INT32)),
            struct_field("f5", bar())]


def beana() -> List[Field]:
    """fury-test-core BeanA (test/bean/BeanA.java:33-54) as TypeInference.inferSchema builds it
    (TypeInference.java:136-238): fields sorted by Java name with String.compareTo
    (Descriptor.java:324-332), renamed lower_underscore (:228), the transient ``f13`` skipped
    (Descriptor.java:391).  ``byte[]`` / ``int[]`` are primitive arrays (list of non-null items,
    :192-198), ``Iterable<BeanB>`` / ``List<BeanB>`` lists of nullable BeanB structs, ``int[][]``
    a list of nullable ``int[]`` lists, ``Map<String, BeanB>`` a map with a non-null String key
    (:204-213), BigDecimal a decimal(38, 18) (:173-177)."""
    def bean_b(name: str) -> Field:
        return struct_field(name, beanb())

    def lst(item: Field) -> Field:
        return Field("", LIST, True, (item,))

    java = [
        ("f1", not_null_field("", INT16)), ("f2", field("", INT32)),
        ("f3", not_null_field("", INT64)), ("f4", field("", FLOAT32)),
        ("f5", not_null_field("", FLOAT64)), ("beanB", bean_b("")),
        ("intArray", array_field("", INT32, elem_nullable=False)),
        ("bytes", array_field("", INT8, elem_nullable=False)),
        ("f12", not_null_field("", BOOL)), ("f15", field("", INT32)),
        ("f16", field("", DECIMAL)), ("f17", field("", STRING)),
        ("longStringField", field("", STRING)), ("doubleList", array_field("", FLOAT64)),
        ("beanBIterable", lst(bean_b("item"))), ("beanBList", lst(bean_b("item"))),
        ("stringBeanBMap", map_field("", field("key", STRING), bean_b("value"))),
        ("int2DArray", lst(array_field("item", INT32, elem_nullable=False))),
        ("double2DList", lst(array_field("item", FLOAT64))),
    ]
    return infer_bean_schema(java)


def row_test_fields() -> List[Field]:
    """The schema of cpp/fury/row/row_test.cc:31-44 (RowTest.Write): f1 utf8, f2 int32,
    f3 list<int32>, f4 map<utf8, float32>, f5 struct<n1 utf8, n2 int32>."""
    return [field("f1", STRING), field("f2", INT32), array_field("f3", INT32),
            map_field("f4", field("key", STRING), field("value", FLOAT32)),
            struct_field("f5", [field("n1", STRING), field("n2", INT32)])]


SCHEMAS: Dict[str, List[Field]] = {
    "struct100": struct100(), "docs_struct": docs_struct(), "mixed": mixed(),
    "nested": nested(), "narrow": narrow(), "bar": bar(), "beanb": beanb(), "foo": foo(),
    "beana": beana(), "row_test": row_test_fields(),
}

# ---------------------------------------------------------------------------------------------
# SplitMix64 generators (numpy, host)
# ---------------------------------------------------------------------------------------------
_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _keys(seed: int, col: int, rows: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        k = np.uint64((seed * 0x9E3779B97F4A7C15 + (col + 1) * 0xD1B54A32D192ED03)
                      & 0xFFFFFFFFFFFFFFFF)
        return splitmix64(rows.astype(np.uint64) ^ k)


def _validity_from_mask(valid: np.ndarray) -> np.ndarray:
    return np.packbits(valid.astype(np.uint8), bitorder="little")


def _gen_fixed(t: int, h: np.ndarray) -> np.ndarray:
    if t == FLOAT64:
        return ((h >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53)))
    if t == FLOAT32:
        return ((h >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / (1 << 24)))
    if t in (INT64, TIMESTAMP):
        return h.view(np.int64)
    w = type_width(t)
    dt = {1: np.int8, 2: np.int16, 4: np.int32}[w]
    return h.astype(dt)          # truncation of the 64-bit hash


def gen_column(f: Field, seed: int, col: int, start: int, n: int, null_pct: int,
               str_max: int = 32, list_max: int = 16, list_null_pct: int = 5,
               elem_null_pct: int = 0) -> Column:
    rows = np.arange(start, start + n, dtype=np.uint64)
    h = _keys(seed, col, rows)
    validity = None
    valid = np.ones(n, bool)
    pct = list_null_pct if f.type_id == LIST else null_pct
    if f.nullable and pct > 0:
        valid = (((h >> np.uint64(7)) % np.uint64(100)) >= np.uint64(pct))
        validity = _validity_from_mask(valid)
    t = f.type_id
    if t == BOOL:
        bitv = ((h >> np.uint64(3)) & np.uint64(1)).astype(bool) & valid
        return Column(values=_validity_from_mask(bitv), validity=validity)
    if type_width(t) > 0:
        v = _gen_fixed(t, h)
        if f.nullable and pct > 0:
            v = np.where(valid, v, np.zeros_like(v))
        return Column(values=np.ascontiguousarray(v), validity=validity)
    if t == DECIMAL:
        # decimal128 two's complement, |value| < 2**125 < 10**38 (fits precision 38)
        h2 = (_keys(seed, col + 1000, rows).view(np.int64) >> np.int64(3)).view(np.uint64)
        v = np.stack([h, h2], axis=1).view(np.uint8).reshape(n, 16).copy()
        v[~valid] = 0
        return Column(values=v.reshape(-1), validity=validity)
    if t in (STRING, BINARY):
        lens = ((h >> np.uint64(17)) % np.uint64(str_max + 1)).astype(np.int64)
        lens[~valid] = 0
        offsets = np.zeros(n + 1, np.int64)
        np.cumsum(lens, out=offsets[1:])
        total = int(offsets[-1])
        rid = np.repeat(rows, lens)
        pos = np.arange(total, dtype=np.int64) - np.repeat(offsets[:-1], lens)
        hb = splitmix64(_keys(seed, col + 2000, rid) ^ pos.astype(np.uint64))
        if t == STRING:
            data = (np.uint64(32) + hb % np.uint64(95)).astype(np.uint8)   # printable ASCII
        else:
            data = (hb >> np.uint64(13)).astype(np.uint8)
        return Column(values=data, validity=validity, offsets=offsets.astype(np.int32))
    if t == LIST:
        elem = f.children[0]
        lens = ((h >> np.uint64(19)) % np.uint64(list_max + 1)).astype(np.int64)
        lens[~valid] = 0
        offsets = np.zeros(n + 1, np.int64)
        np.cumsum(lens, out=offsets[1:])
        total = int(offsets[-1])
        rid = np.repeat(rows, lens)
        pos = np.arange(total, dtype=np.int64) - np.repeat(offsets[:-1], lens)
        eh = splitmix64(_keys(seed, col + 3000, rid) ^ (pos.astype(np.uint64) << np.uint64(32)))
        evalid = np.ones(total, bool)
        evalidity = None
        if elem.nullable and elem_null_pct > 0:
            evalid = ((eh >> np.uint64(5)) % np.uint64(100)) >= np.uint64(elem_null_pct)
            evalidity = _validity_from_mask(evalid)
        if elem.type_id == BOOL:
            ev = _validity_from_mask(((eh >> np.uint64(3)) & np.uint64(1)).astype(bool) & evalid)
        else:
            ev = _gen_fixed(elem.type_id, eh)
            ev = np.where(evalid, ev, np.zeros_like(ev))
        child = Column(values=np.ascontiguousarray(ev), validity=evalidity)
        return Column(validity=validity, offsets=offsets.astype(np.int32), child=[child])
    raise ValueError(f"no generator for type {t}")


# per-config generator knobs (BASELINE.json configs + SURVEY §8(d) table)
_KNOBS = {
    "struct100": dict(null_pct=0),
    "docs_struct": dict(null_pct=0),
    "mixed": dict(null_pct=10, str_max=32),
    "nested": dict(null_pct=0, list_max=16, list_null_pct=5),
    "narrow": dict(null_pct=10, str_max=40, list_max=70, list_null_pct=10, elem_null_pct=10),
    "bar": dict(null_pct=10),
    "beanb": dict(null_pct=10, list_max=5, list_null_pct=10, elem_null_pct=10),
}


def gen_columns(name: str, fields: Sequence[Field], n: int, seed: int = 1234,
                start: int = 0, **over) -> List[Column]:
    knobs = dict(_KNOBS.get(name, dict(null_pct=10)))
    knobs.update(over)
    return [gen_column(f, seed, k, start, n, **knobs) for k, f in enumerate(fields)]


def slice_columns(fields: Sequence[Field], cols: Sequence[Column], b: int, e: int) -> List[Column]:
    """Rows [b, e) of host columns as columns of their own: fixed values sliced, bitmaps re-packed
    from bit b, STRING / BINARY / LIST offsets rebased to 0 with their payload / child slices
    (the CPU baseline's per-thread batches)."""
    def bits(a, lo, hi):
        if a is None:
            return None
        u = np.unpackbits(np.asarray(a, np.uint8), bitorder="little")[lo:hi]
        return np.packbits(u, bitorder="little")

    out = []
    for f, c in zip(fields, cols):
        t = f.type_id
        if t == BOOL:
            out.append(Column(values=bits(c.values, b, e), validity=bits(c.validity, b, e)))
        elif type_width(t) > 0:
            out.append(Column(values=c.values[b:e], validity=bits(c.validity, b, e)))
        elif t == DECIMAL:
            out.append(Column(values=c.values[16 * b:16 * e], validity=bits(c.validity, b, e)))
        elif t in (STRING, BINARY):
            o = np.asarray(c.offsets)
            out.append(Column(values=c.values[o[b]:o[e]], validity=bits(c.validity, b, e),
                              offsets=(o[b:e + 1] - o[b]).astype(np.int32)))
        elif t == LIST:
            o = np.asarray(c.offsets)
            ch = c.child[0]
            if f.children[0].type_id == BOOL:
                cv = bits(ch.values, o[b], o[e])
            else:
                cv = ch.values[o[b]:o[e]]
            out.append(Column(validity=bits(c.validity, b, e),
                              offsets=(o[b:e + 1] - o[b]).astype(np.int32),
                              child=[Column(values=cv, validity=bits(ch.validity, o[b], o[e]))]))
        else:
            raise ValueError(f"no slice for type {t}")
    return out


def _u64_const(c: int):
    """A uint64 constant as the int64 with the same bits (torch has no uint64 arithmetic)."""
    c &= 0xFFFFFFFFFFFFFFFF
    return c - (1 << 64) if c >= 1 << 63 else c


def _t_shr(x, s: int):
    """Logical right shift of int64 tensors holding uint64 bits."""
    return (x >> s) & ((1 << (64 - s)) - 1)


def _t_splitmix64(x):
    z = x + _u64_const(0x9E3779B97F4A7C15)
    z = (z ^ _t_shr(z, 30)) * _u64_const(0xBF58476D1CE4E5B9)
    z = (z ^ _t_shr(z, 27)) * _u64_const(0x94D049BB133111EB)
    return z ^ _t_shr(z, 31)


def _t_keys(seed: int, col: int, rows):
    k = (seed * 0x9E3779B97F4A7C15 + (col + 1) * 0xD1B54A32D192ED03) & 0xFFFFFFFFFFFFFFFF
    return _t_splitmix64(rows ^ _u64_const(k))


def _t_umod(x, m: int):
    """x mod m for int64 tensors holding uint64 bits (numpy's uint64 %)."""
    hi = _t_shr(x, 32)
    lo = x & 0xFFFFFFFF
    return ((hi % m) * ((1 << 32) % m) + lo % m) % m


def _t_packbits(mask):
    """numpy.packbits(mask, bitorder="little") of a bool tensor."""
    import torch
    n = mask.numel()
    pad = (-n) % 8
    m = torch.nn.functional.pad(mask.to(torch.uint8), (0, pad)).view(-1, 8)
    w = (1 << torch.arange(8, device=mask.device, dtype=torch.int32))
    return (m.to(torch.int32) * w).sum(1).to(torch.uint8)


def _t_gen_fixed(t: int, h):
    import torch
    if t == FLOAT64:
        return _t_shr(h, 11).to(torch.float64) * (1.0 / (1 << 53))
    if t == FLOAT32:
        return _t_shr(h, 40).to(torch.float32) * (1.0 / (1 << 24))
    if t in (INT64, TIMESTAMP):
        return h
    if t in (INT32, DATE32):
        return _t_trunc(h, 32, torch.int32)
    if t == INT16:
        return _t_trunc(h, 16, torch.int16)
    if t == INT8:
        return _t_trunc(h, 8, torch.int8)
    raise ValueError(f"no torch generator for type {t}")


def gen_column_torch(f: Field, seed: int, col: int, start: int, n: int, null_pct: int,
                     str_max: int = 32, list_max: int = 16, list_null_pct: int = 5,
                     elem_null_pct: int = 0, device=None) -> Column:
    """``gen_column`` computed with torch on ``device``, bit for bit (the same SplitMix64 keys of
    (seed, column, GLOBAL row index)); for the configuration-size GPU tests and the bench, whose
    10M-row batches would take the numpy generator minutes."""
    import torch
    rows = torch.arange(start, start + n, dtype=torch.int64, device=device)
    h = _t_keys(seed, col, rows)
    validity = None
    valid = torch.ones(n, dtype=torch.bool, device=device)
    pct = list_null_pct if f.type_id == LIST else null_pct
    if f.nullable and pct > 0:
        valid = (_t_shr(h, 7) % 100) >= pct
        validity = _t_packbits(valid)
    t = f.type_id
    if t == BOOL:
        return Column(values=_t_packbits(((_t_shr(h, 3) & 1) != 0) & valid), validity=validity)
    if type_width(t) > 0:
        v = _t_gen_fixed(t, h)
        if f.nullable and pct > 0:
            v = torch.where(valid, v, torch.zeros_like(v))
        return Column(values=v.contiguous(), validity=validity)
    if t == DECIMAL:
        h2 = _t_keys(seed, col + 1000, rows) >> 3                  # arithmetic, as numpy's int64
        v = torch.stack([h, h2], 1).contiguous().view(torch.uint8).reshape(n, 16).clone()
        v[~valid] = 0
        return Column(values=v.reshape(-1), validity=validity)
    if t in (STRING, BINARY, LIST):
        mod = (str_max + 1) if t != LIST else (list_max + 1)
        lens = _t_shr(h, 17 if t != LIST else 19) % mod
        lens = torch.where(valid, lens, torch.zeros_like(lens))
        offsets = torch.zeros(n + 1, dtype=torch.int64, device=device)
        torch.cumsum(lens, 0, out=offsets[1:])
        total = int(offsets[-1].item())
        rid = torch.repeat_interleave(rows, lens, output_size=total)
        pos = torch.arange(total, dtype=torch.int64, device=device) - \
            torch.repeat_interleave(offsets[:-1], lens, output_size=total)
        if t != LIST:
            hb = _t_splitmix64(_t_keys(seed, col + 2000, rid) ^ pos)
            if t == STRING:
                data = (32 + _t_umod(hb, 95)).to(torch.uint8)      # printable ASCII
            else:
                data = (_t_shr(hb, 13) & 0xFF).to(torch.uint8)
            return Column(values=data, validity=validity, offsets=offsets.to(torch.int32))
        elem = f.children[0]
        eh = _t_splitmix64(_t_keys(seed, col + 3000, rid) ^ (pos << 32))
        evalid = torch.ones(total, dtype=torch.bool, device=device)
        evalidity = None
        if elem.nullable and elem_null_pct > 0:
            evalid = (_t_shr(eh, 5) % 100) >= elem_null_pct
            evalidity = _t_packbits(evalid)
        if elem.type_id == BOOL:
            ev = _t_packbits(((_t_shr(eh, 3) & 1) != 0) & evalid)
        else:
            ev = _t_gen_fixed(elem.type_id, eh)
            ev = torch.where(evalid, ev, torch.zeros_like(ev))
        child = Column(values=ev.contiguous(), validity=evalidity)
        return Column(validity=validity, offsets=offsets.to(torch.int32), child=[child])
    raise ValueError(f"no torch generator for type {t}")


def gen_columns_torch(name: str, fields: Sequence[Field], n: int, seed: int = 1234,
                      start: int = 0, device=None, **over) -> List[Column]:
    """``gen_columns`` computed with torch on ``device`` (the GPU for the bench, so 10M-row
    batches and 12.5M-row shards need no host generation or copy): bit for bit the same columns
    (tests/test_workloads.py checks it against the numpy generator)."""
    knobs = dict(_KNOBS.get(name, dict(null_pct=10)))
    knobs.update(over)
    return [gen_column_torch(f, seed, k, start, n, device=device, **knobs)
            for k, f in enumerate(fields)]


def _t_trunc(h, bits: int, dtype):
    """Two's-complement truncation of int64 bits to a narrower signed type (numpy astype)."""
    low = h & ((1 << bits) - 1)
    return (low - ((low >> (bits - 1)) << bits)).to(dtype)


def algorithmic_bytes_fixed(fields: Sequence[Field], nrows: int) -> dict:
    """SURVEY §8(d) / BASELINE.md §4 accounting for fixed-width schemas: encode reads the value
    columns and writes rows; decode the reverse."""
    col_bytes = sum(type_width(f.type_id) for f in fields) * nrows
    row_bytes = (((len(fields) + 63) // 64) * 8 + 8 * len(fields)) * nrows
    return {"encode": col_bytes + row_bytes, "decode": row_bytes + col_bytes,
            "total": 2 * (col_bytes + row_bytes), "col_bytes": col_bytes, "row_bytes": row_bytes}


# ---------------------------------------------------------------------------------------------
# java.util.Random restatement for the docs Struct values (Struct.java:112-134 uses
# new Random(17) over getDeclaredFields() declaration order).
# ---------------------------------------------------------------------------------------------
class JavaRandom:
    _MUL = 0x5DEECE66D
    _MASK = (1 << 48) - 1

    def __init__(self, seed: int):
        self.seed = (seed ^ self._MUL) & self._MASK

    def _next(self, bits: int) -> int:
        self.seed = (self.seed * self._MUL + 0xB) & self._MASK
        r = self.seed >> (48 - bits)
        if bits == 32 and r >= 1 << 31:
            r -= 1 << 32
        return r

    def next_int(self) -> int:
        return self._next(32)

    def next_long(self) -> int:
        v = ((self._next(32) << 32) + self._next(32)) & 0xFFFFFFFFFFFFFFFF
        return v - (1 << 64) if v >= 1 << 63 else v

    def next_float(self) -> float:
        return self._next(24) / float(1 << 24)

    def next_double(self) -> float:
        return ((self._next(26) << 27) + self._next(27)) * (1.0 / (1 << 53))

    def next_int_bound(self, bound: int) -> int:
        """Random.nextInt(int bound)."""
        if bound & -bound == bound:
            return (bound * self._next31()) >> 31
        while True:
            bits = self._next31()
            val = bits % bound
            if bits - val + (bound - 1) < 1 << 31:
                return val

    def _next31(self) -> int:
        self.seed = (self.seed * self._MUL + 0xB) & self._MASK
        return self.seed >> 17

    def next_bytes(self, n: int) -> bytes:
        """Random.nextBytes: little-endian bytes of successive nextInt() words."""
        out = bytearray()
        while len(out) < n:
            r = self.next_int() & 0xFFFFFFFF
            for _ in range(min(n - len(out), 4)):
                out.append(r & 0xFF)
                r >>= 8
        return bytes(out)


def _java_string_hash(s: str) -> int:
    h = 0
    for u in s.encode("utf-16-be").hex(" ", 2).split():
        h = (31 * h + int(u, 16)) & 0xFFFFFFFF
    return h


def java_hash_map_order(keys: Sequence[str]) -> List[str]:
    """Iteration order of a java.util.HashMap<String, ?> filled by put() in ``keys`` order
    (distinct keys, no treeified bins): table size 16 doubled while size > 0.75 * table; bucket
    = (h ^ (h >>> 16)) & (table - 1); buckets in index order, each in insertion order (resize
    splits keep it)."""
    cap = 16
    while len(keys) > cap * 3 // 4:
        cap *= 2
    def bucket(k):
        h = _java_string_hash(k)
        return (h ^ (h >> 16)) & (cap - 1)
    return [k for _, _, k in sorted((bucket(k), i, k) for i, k in enumerate(keys))]


def _java_random_string(size: int, rnd: "JavaRandom") -> str:
    """TestUtils.random(size, Random) (fury-test-core TestUtils.java:34-43): chars ' '..'z'."""
    return "".join(chr(32 + rnd.next_int_bound(ord("z") + 1 - 32)) for _ in range(size))


def create_beanb(arr_size: int) -> dict:
    """BeanB.createBeanB(arrSize) (fury-test-core test/bean/BeanB.java:39-65), new Random(37),
    as a bean dict keyed by the schema's field names."""
    rnd = JavaRandom(37)
    b = {"f1": ((rnd.next_int() + 2**15) & 0xFFFF) - 2**15, "f2": rnd.next_int(),
         "f3": rnd.next_long(), "f4": rnd.next_float(), "f5": rnd.next_double(),
         "int_arr": None, "int_list": None}
    if arr_size > 0:
        b["int_arr"] = [rnd.next_int() for _ in range(arr_size)]
        b["int_list"] = [rnd.next_int() for _ in range(arr_size)]
    return b


# BeanA.createBeanA's BigDecimal: unscaled 122222222222222225454657712222222222, scale 18
# (BeanA.java:67-68), as the 16-byte little-endian two's complement Arrow writes
# (DecimalUtility.writeBigDecimalToArrowBuf, BinaryWriter.writeDecimal :214-226).
BEANA_DECIMAL_UNSCALED = 122222222222222225454657712222222222


def decimal_bytes(unscaled: int) -> bytes:
    return unscaled.to_bytes(16, "little", signed=True)


def create_beana(arr_size: int) -> dict:
    """BeanA.createBeanA(arrSize) (fury-test-core test/bean/BeanA.java:56-137), value for value:
    new Random(37) drawn in the same order, f17 / long_string_field from TestUtils.random(n, 1),
    ``arr[i] = rnd.nextInt()`` in the int2DArray loop exactly as written (only the diagonal is
    set), map entries in java.util.HashMap iteration order, the transient f13 absent."""
    rnd = JavaRandom(37)
    a = {"f1": ((rnd.next_int() + 2**15) & 0xFFFF) - 2**15, "f2": rnd.next_int(),
         "f3": rnd.next_long(), "f4": rnd.next_float(), "f5": rnd.next_double()}
    a["f15"] = rnd.next_int()
    a["f12"] = True
    a["bean_b"] = create_beanb(arr_size)
    a["f16"] = decimal_bytes(BEANA_DECIMAL_UNSCALED)
    a["f17"] = _java_random_string(40, JavaRandom(1))
    a["long_string_field"] = _java_random_string(20, JavaRandom(1))
    for k in ("bytes", "double_list", "double2_d_list", "int_array", "int2_d_array",
              "bean_b_list", "string_bean_b_map", "bean_b_iterable"):
        a[k] = None
    if arr_size > 0:
        a["bytes"] = [b - 256 if b >= 128 else b for b in rnd.next_bytes(arr_size)]
        dl = [rnd.next_double() for _ in range(arr_size)]
        dl[0] = None
        a["double_list"] = dl
        a["double2_d_list"] = [[rnd.next_double() for _ in range(arr_size)]
                               for _ in range(arr_size)]
        a["int_array"] = [rnd.next_int() for _ in range(arr_size)]
        i2 = [[0] * arr_size for _ in range(arr_size)]
        for i in range(arr_size):
            for _ in range(arr_size):
                i2[i][i] = rnd.next_int()
        a["int2_d_array"] = i2
        a["bean_b_list"] = [create_beanb(arr_size) for _ in range(arr_size)]
        keys = [f"key{i}" for i in range(arr_size)]
        a["string_bean_b_map"] = [(k, create_beanb(arr_size)) for k in java_hash_map_order(keys)]
        a["bean_b_iterable"] = [create_beanb(arr_size) for _ in range(arr_size)]
    return a


def docs_struct_values(fields: Sequence[Field]) -> List[Column]:
    """One docs-Struct object as 1-row columns (values per Struct.createPOJO)."""
    rnd = JavaRandom(17)
    vals = {}
    for i in range(104):                          # declaration order f0..f103
        k = i % 4
        if k == 0:
            vals[f"f{i}"] = np.array([rnd.next_int()], np.int32)
        elif k == 1:
            vals[f"f{i}"] = np.array([rnd.next_long()], np.int64)
        elif k == 2:
            vals[f"f{i}"] = np.array([rnd.next_float()], np.float32)
        else:
            vals[f"f{i}"] = np.array([rnd.next_double()], np.float64)
    return [Column(values=vals[f.name]) for f in fields]
