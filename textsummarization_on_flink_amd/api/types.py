"""Column types, schemas and rows of the streaming table API.

``DataTypes`` are the Flink-AI-Extended element types the reference's ``CodingUtils`` maps
(``CodingUtils.java:37-61,79-129``); ``TypeInformation`` mirrors the Flink basic type
infos they map to.  ``CodingUtils`` keeps the same two-way mapping and rejects the same
unsupported types.
"""
from __future__ import annotations

import enum
from typing import Any, Iterable, List, Optional, Sequence


class DataTypes(enum.Enum):
    STRING = "string"
    BOOL = "bool"
    INT_8 = "int8"
    INT_16 = "int16"
    INT_32 = "int32"
    INT_64 = "int64"
    FLOAT_16 = "float16"     # exists in FAE DataTypes; not supported by the coding (raises)
    FLOAT_32 = "float32"
    FLOAT_64 = "float64"
    UINT_8 = "uint8"         # unsupported (raises)
    UINT_16 = "uint16"       # Java char
    FLOAT_32_ARRAY = "float32_array"


class TypeInformation(enum.Enum):
    STRING_TYPE_INFO = str
    BOOLEAN_TYPE_INFO = bool
    BYTE_TYPE_INFO = "byte"
    SHORT_TYPE_INFO = "short"
    INT_TYPE_INFO = int
    LONG_TYPE_INFO = "long"
    FLOAT_TYPE_INFO = float
    DOUBLE_TYPE_INFO = "double"
    CHAR_TYPE_INFO = "char"
    DATE_TYPE_INFO = "date"
    VOID_TYPE_INFO = "void"
    BIG_INT_TYPE_INFO = "bigint"
    BIG_DEC_TYPE_INFO = "bigdec"
    INSTANT_TYPE_INFO = "instant"
    STRING_ARRAY_TYPE_INFO = "string[]"
    BOOLEAN_ARRAY_TYPE_INFO = "boolean[]"
    BYTE_ARRAY_TYPE_INFO = "byte[]"
    SHORT_ARRAY_TYPE_INFO = "short[]"
    INT_ARRAY_TYPE_INFO = "int[]"
    LONG_ARRAY_TYPE_INFO = "long[]"
    FLOAT_ARRAY_TYPE_INFO = "float[]"
    DOUBLE_ARRAY_TYPE_INFO = "double[]"
    CHAR_ARRAY_TYPE_INFO = "char[]"


_DT2TI = {
    DataTypes.STRING: TypeInformation.STRING_TYPE_INFO,
    DataTypes.BOOL: TypeInformation.BOOLEAN_TYPE_INFO,
    DataTypes.INT_8: TypeInformation.BYTE_TYPE_INFO,
    DataTypes.INT_16: TypeInformation.SHORT_TYPE_INFO,
    DataTypes.INT_32: TypeInformation.INT_TYPE_INFO,
    DataTypes.INT_64: TypeInformation.LONG_TYPE_INFO,
    DataTypes.FLOAT_32: TypeInformation.FLOAT_TYPE_INFO,
    DataTypes.FLOAT_64: TypeInformation.DOUBLE_TYPE_INFO,
    DataTypes.UINT_16: TypeInformation.CHAR_TYPE_INFO,
    DataTypes.FLOAT_32_ARRAY: TypeInformation.FLOAT_ARRAY_TYPE_INFO,
}
_TI2DT = {v: k for k, v in _DT2TI.items()}


def data_types_to_type_information(dt: DataTypes) -> TypeInformation:
    """CodingUtils.java:37-61."""
    try:
        return _DT2TI[dt]
    except KeyError:
        raise RuntimeError(f"Unsupported data type of {dt}") from None


def type_information_to_data_types(ti: TypeInformation) -> DataTypes:
    """CodingUtils.java:79-129."""
    try:
        return _TI2DT[ti]
    except KeyError:
        raise RuntimeError(f"Unsupported data type of {ti}") from None


def data_types_list_to_type_information(dts: Sequence[DataTypes]) -> List[TypeInformation]:
    return [data_types_to_type_information(d) for d in dts]


def type_information_list_to_data_types(tis: Sequence[TypeInformation]) -> List[DataTypes]:
    return [type_information_to_data_types(t) for t in tis]


def coerce(value: Any, dt: DataTypes):
    """Python value of a column of type ``dt``."""
    if value is None:
        return None
    if dt == DataTypes.STRING:
        if isinstance(value, (bytes, bytearray)):
            return value.decode("utf-8", errors="replace")
        return str(value)
    if dt == DataTypes.BOOL:
        return bool(value)
    if dt in (DataTypes.INT_8, DataTypes.INT_16, DataTypes.INT_32, DataTypes.INT_64):
        return int(value)
    if dt in (DataTypes.FLOAT_32, DataTypes.FLOAT_64):
        return float(value)
    if dt == DataTypes.UINT_16:
        s = value.decode() if isinstance(value, (bytes, bytearray)) else value
        return chr(s) if isinstance(s, int) else str(s)[:1]
    if dt == DataTypes.FLOAT_32_ARRAY:
        return [float(x) for x in value]
    raise RuntimeError(f"Unsupported data type of {dt}")


class TableSchema:
    def __init__(self, names: Sequence[str], types: Sequence):
        if len(names) != len(types):
            raise ValueError("Number of field names and field types must be equal.")
        if len(set(names)) != len(names):
            raise ValueError(f"Field names must be unique: {list(names)}")
        self._names = list(names)
        self._types = [t if isinstance(t, DataTypes) else type_information_to_data_types(t) for t in types]

    def get_field_names(self) -> List[str]:
        return list(self._names)

    def get_field_types(self) -> List[TypeInformation]:
        return data_types_list_to_type_information(self._types)

    def get_data_types(self) -> List[DataTypes]:
        return list(self._types)

    def get_field_count(self) -> int:
        return len(self._names)

    def index_of(self, name: str) -> int:
        try:
            return self._names.index(name)
        except ValueError:
            raise KeyError(f"no field {name!r} in {self._names}") from None

    def project(self, names: Sequence[str]) -> "TableSchema":
        return TableSchema(names, [self._types[self.index_of(n)] for n in names])

    getFieldNames, getFieldTypes, getFieldCount = get_field_names, get_field_types, get_field_count

    def __eq__(self, o):
        return isinstance(o, TableSchema) and self._names == o._names and self._types == o._types

    def __repr__(self):
        return "root\n" + "\n".join(f" |-- {n}: {t.name}" for n, t in zip(self._names, self._types))


class Row:
    """A positional record (Flink ``Row``)."""

    __slots__ = ("_f",)

    def __init__(self, *fields):
        self._f = list(fields)

    @classmethod
    def of(cls, *fields) -> "Row":
        return cls(*fields)

    @classmethod
    def with_arity(cls, n: int) -> "Row":
        return cls(*([None] * n))

    def get_arity(self) -> int:
        return len(self._f)

    def get_field(self, i: int):
        return self._f[i]

    def set_field(self, i: int, v) -> None:
        self._f[i] = v

    getArity, getField, setField = get_arity, get_field, set_field

    def as_dict(self, names: Sequence[str]) -> dict:
        return dict(zip(names, self._f))

    def __iter__(self):
        return iter(self._f)

    def __len__(self):
        return len(self._f)

    def __getitem__(self, i):
        return self._f[i]

    def __eq__(self, o):
        return isinstance(o, Row) and self._f == o._f

    def __hash__(self):
        return hash(tuple(map(repr, self._f)))

    def __repr__(self):
        return ",".join("null" if v is None else str(v) for v in self._f)


def parse_fields(spec) -> List[str]:
    """``"uuid,article, reference"`` or a list -> field names (``Table.select`` syntax)."""
    if isinstance(spec, str):
        return [s.strip() for s in spec.split(",") if s.strip()]
    return list(spec)


def schema_of(names: Iterable[str], types: Optional[Sequence[DataTypes]] = None) -> TableSchema:
    names = list(names)
    return TableSchema(names, list(types) if types is not None else [DataTypes.STRING] * len(names))
