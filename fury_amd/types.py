"""Schema types — the host-side mirror of ``org.apache.fury.format.type.DataTypes`` /
``TypeInference`` (java/fury-format/src/main/java/org/apache/fury/format/type/).

A schema is a list of :class:`Field` in slot order.  ``Field`` mirrors
``org.apache.arrow.vector.types.pojo.Field`` as TypeInference builds it: primitives are
non-nullable, boxed types / String / collections / beans are nullable, list elements are named
``item`` (DataTypes.ARRAY_ITEM_NAME, DataTypes.java:66), map children are ``key`` (non-null) and
``value`` (TypeInference.java:207-216).

Layout and schema hash are computed natively (``fury_schema_create`` in the C ABI); the helpers
here only describe fields.
"""
from __future__ import annotations

from dataclasses import dataclass, field as _dc_field
from typing import Dict, List, Sequence, Tuple

# Type ids = FMT/type/ArrowType.java:25-148 (also include/fury_row.h fury_type_id)
BOOL = 1
INT8 = 3
INT16 = 5
INT32 = 7
INT64 = 9
FLOAT32 = 11
FLOAT64 = 12
STRING = 13
BINARY = 14
DATE32 = 16
TIMESTAMP = 18
DECIMAL = 23
LIST = 25
STRUCT = 26
MAP = 30

TYPE_NAMES = {BOOL: "bool", INT8: "int8", INT16: "int16", INT32: "int32", INT64: "int64",
              FLOAT32: "float32", FLOAT64: "float64", STRING: "utf8", BINARY: "binary",
              DATE32: "date32", TIMESTAMP: "timestamp[us]", DECIMAL: "decimal128",
              LIST: "list", STRUCT: "struct", MAP: "map"}

# DataTypes.getTypeWidth (DataTypes.java:68-133): -1 for variable length.
_WIDTH = {BOOL: 1, INT8: 1, INT16: 2, INT32: 4, INT64: 8, FLOAT32: 4, FLOAT64: 8, DATE32: 4,
          TIMESTAMP: 8}


def type_width(type_id: int) -> int:
    return _WIDTH.get(type_id, -1)


@dataclass(frozen=True)
class Field:
    name: str
    type_id: int
    nullable: bool = True
    children: Tuple["Field", ...] = _dc_field(default_factory=tuple)

    def __post_init__(self):
        object.__setattr__(self, "children", tuple(self.children))

    def __repr__(self) -> str:
        inner = ""
        if self.children:
            inner = "<" + ", ".join(repr(c) for c in self.children) + ">"
        nn = "" if self.nullable else " not null"
        return f"{self.name}: {TYPE_NAMES.get(self.type_id, self.type_id)}{inner}{nn}"


# -- DataTypes-style constructors --------------------------------------------------------------
def field(name: str, type_id: int, nullable: bool = True, children: Sequence[Field] = ()) -> Field:
    """DataTypes.field(name, nullable, type, children) (DataTypes.java:309-336)."""
    return Field(name, type_id, nullable, tuple(children))


def not_null_field(name: str, type_id: int) -> Field:
    """DataTypes.notNullField (DataTypes.java:338-341)."""
    return Field(name, type_id, False)


def array_field(name: str, elem_type: int, elem_nullable: bool = True,
                elem_children: Sequence[Field] = ()) -> Field:
    """DataTypes.arrayField / primitiveArrayField (DataTypes.java:348-369): nullable list whose
    element field is named ``item``; primitive arrays (int[]...) have a non-null item."""
    return Field(name, LIST, True, (Field("item", elem_type, elem_nullable, tuple(elem_children)),))


def struct_field(name: str, children: Sequence[Field], nullable: bool = True) -> Field:
    """DataTypes.structField (bean fields are nullable structs, TypeInference.java:218-232)."""
    return Field(name, STRUCT, nullable, tuple(children))


def map_field(name: str, key: Field, value: Field) -> Field:
    """DataTypes.mapField: key field forced non-null (TypeInference.java:207-216)."""
    return Field(name, MAP, True, (Field("key", key.type_id, False, key.children),
                                   Field("value", value.type_id, value.nullable, value.children)))


def lower_camel_to_lower_underscore(s: str) -> str:
    """StringUtils.lowerCamelToLowerUnderscore (fury-core util/StringUtils.java:252-271)."""
    out, start = [], 0
    for i, ch in enumerate(s):
        if "A" <= ch <= "Z":
            out.append(s[start:i])
            out.append("_")
            out.append(ch.lower())
            start = i + 1
    if start < len(s):
        out.append(s[start:])
    return "".join(out)


def _java_compare_key(name: str):
    # String.compareTo compares UTF-16 code units.
    return name.encode("utf-16-be")


def infer_bean_schema(java_fields: Sequence[Tuple[str, Field]]) -> List[Field]:
    """TypeInference.inferSchema for a bean given as (javaFieldName, Field-with-any-name) pairs:
    sort by Java field name (Descriptor.java:324-332) and rename to lower_underscore
    (TypeInference.java:228)."""
    ordered = sorted(java_fields, key=lambda p: _java_compare_key(p[0]))
    return [Field(lower_camel_to_lower_underscore(jn), f.type_id, f.nullable, f.children)
            for jn, f in ordered]


def schema_spec(fields: Sequence[Field]) -> list:
    return [[f.name, f.type_id, bool(f.nullable), schema_spec(f.children)] for f in fields]


def schema_from_spec(spec: list) -> List[Field]:
    return [Field(n, t, bool(nl), tuple(schema_from_spec(ch))) for n, t, nl, ch in spec]


def is_fixed_schema(fields: Sequence[Field]) -> bool:
    return all(type_width(f.type_id) > 0 for f in fields)


def bitmap_bytes(n: int) -> int:
    """BitUtils.calculateBitmapWidthInBytes (fury-core memory/BitUtils.java:175-177)."""
    return ((n + 63) // 64) * 8


def fixed_size(fields: Sequence[Field]) -> int:
    """BinaryRowWriter fixedSize = bitmap + 8 * numFields (BinaryRowWriter.java:46-52)."""
    return bitmap_bytes(len(fields)) + 8 * len(fields)


Schema = List[Field]
SchemaDict = Dict[str, List[Field]]
