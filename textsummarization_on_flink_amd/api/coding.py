"""Row <-> record codecs between the driver (table side) and worker processes
(``CodingUtils.java:131-206``).

A job config carries the codec description in its properties, exactly like the
reference's ``TFConfig`` (``INPUT_TF_EXAMPLE_CONFIG`` / ``OUTPUT_TF_EXAMPLE_CONFIG`` plus
``ENCODING_CLASS`` / ``DECODING_CLASS``).  Either side may be absent ("encode only",
"decode only", "neither" -- ``InputOutputTest.java:31-101``).

* ``ExampleCoding``: a row as a ``tf.Example`` (one feature per column; STRING -> bytes,
  integers/BOOL -> int64, FLOAT_* -> float, FLOAT_32_ARRAY -> float list), the format the
  reference's Python readers parse (``batcher.py:596-600``).
* ``CsvCoding``: the deprecated prototype's ``RowCSVCoding`` (fields joined with ``#``,
  ``Summarization.java:67-77``).
"""
from __future__ import annotations

import json
from typing import Dict, List, Optional, Sequence, Union

from ..data.example_proto import decode_example, encode_example, string_row_encoder
from .types import DataTypes, Row, TableSchema, coerce

INPUT_TF_EXAMPLE_CONFIG = "input_tf_example_config"
OUTPUT_TF_EXAMPLE_CONFIG = "output_tf_example_config"
ENCODING_CLASS = "sys:encoding_class"
DECODING_CLASS = "sys:decoding_class"
CSV_DELIM = "sys:delim"


class ExampleCoding:
    kind = "example"

    def __init__(self, names: Sequence[str], types: Sequence[DataTypes]):
        self.names, self.types = list(names), list(types)
        for t in self.types:
            if t in (DataTypes.FLOAT_16, DataTypes.UINT_8):
                raise RuntimeError(f"Unsupported data type of {t}")
        # all-STRING schemas (the streaming rows) take the precomputed fast path
        self._fast = string_row_encoder(self.names) if all(t == DataTypes.STRING for t in self.types) else None

    def _fields(self, row) -> List:
        if isinstance(row, dict):
            return [row.get(n) for n in self.names]
        return list(row)

    def encode(self, row: Union[Row, dict, Sequence]) -> bytes:
        vals = self._fields(row)
        if len(vals) != len(self.names):
            raise ValueError(f"row arity {len(vals)} != schema arity {len(self.names)}")
        if self._fast is not None:
            return self._fast(vals)
        feats = {}
        for n, t, v in zip(self.names, self.types, vals):
            if v is None:
                continue
            if t == DataTypes.STRING or t == DataTypes.UINT_16:
                feats[n] = [v if isinstance(v, (bytes, bytearray)) else str(v)]
            elif t == DataTypes.BOOL:
                feats[n] = [int(bool(v))]
            elif t in (DataTypes.INT_8, DataTypes.INT_16, DataTypes.INT_32, DataTypes.INT_64):
                feats[n] = [int(v)]
            elif t in (DataTypes.FLOAT_32, DataTypes.FLOAT_64):
                feats[n] = [float(v)]
            elif t == DataTypes.FLOAT_32_ARRAY:
                feats[n] = [float(x) for x in v] or [0.0][:0]
            else:
                raise RuntimeError(f"Unsupported data type of {t}")
        return encode_example(feats)

    def decode_dict(self, data: bytes) -> Dict[str, object]:
        ex = decode_example(data)
        out = {}
        for n, t in zip(self.names, self.types):
            v = ex.get(n)
            if v is None or (not v and t != DataTypes.FLOAT_32_ARRAY):
                out[n] = None
            else:
                out[n] = coerce(v if t == DataTypes.FLOAT_32_ARRAY else v[0], t)
        return out

    def decode(self, data: bytes) -> Row:
        d = self.decode_dict(data)
        return Row(*[d[n] for n in self.names])

    def describe(self) -> str:
        return json.dumps({"names": self.names, "types": [t.name for t in self.types], "objectType": "ROW",
                           "entryClass": "Row"})


class CsvCoding:
    kind = "csv"

    def __init__(self, names: Sequence[str], types: Sequence[DataTypes], delim: str = "#"):
        self.names, self.types, self.delim = list(names), list(types), delim

    def encode(self, row) -> bytes:
        vals = [row.get(n) for n in self.names] if isinstance(row, dict) else list(row)
        return self.delim.join("" if v is None else str(v) for v in vals).encode("utf-8")

    def decode_dict(self, data: bytes) -> Dict[str, object]:
        parts = data.decode("utf-8").split(self.delim)
        parts += [""] * (len(self.names) - len(parts))
        return {n: coerce(p, t) if p != "" or t == DataTypes.STRING else None
                for n, t, p in zip(self.names, self.types, parts)}

    def decode(self, data: bytes) -> Row:
        d = self.decode_dict(data)
        return Row(*[d[n] for n in self.names])

    def describe(self) -> str:
        return json.dumps({"names": self.names, "types": [t.name for t in self.types], "delim": self.delim})


def _from_desc(kind: str, desc: str):
    d = json.loads(desc)
    types = [DataTypes[t] for t in d["types"]]
    if kind == "csv":
        return CsvCoding(d["names"], types, d.get("delim", "#"))
    return ExampleCoding(d["names"], types)


class CodingUtils:
    """Static helpers with the reference's names (snake_case + Java aliases)."""

    @staticmethod
    def configure_encode_example_coding(properties: dict, names, types) -> None:
        c = ExampleCoding(names, _as_dt(types))
        properties[INPUT_TF_EXAMPLE_CONFIG] = c.describe()
        properties[ENCODING_CLASS] = "example"

    @staticmethod
    def configure_decode_example_coding(properties: dict, names, types) -> None:
        c = ExampleCoding(names, _as_dt(types))
        properties[OUTPUT_TF_EXAMPLE_CONFIG] = c.describe()
        properties[DECODING_CLASS] = "example"

    @staticmethod
    def configure_example_coding(properties: dict, encode_schema: Optional[TableSchema],
                                 decode_schema: Optional[TableSchema]) -> None:
        """CodingUtils.java:196-206: either schema may be None (configures one side only)."""
        if encode_schema is not None:
            CodingUtils.configure_encode_example_coding(properties, encode_schema.get_field_names(),
                                                        encode_schema.get_data_types())
        if decode_schema is not None:
            CodingUtils.configure_decode_example_coding(properties, decode_schema.get_field_names(),
                                                        decode_schema.get_data_types())

    @staticmethod
    def configure_csv_coding(properties: dict, encode_schema: Optional[TableSchema],
                             decode_schema: Optional[TableSchema], delim: str = "#") -> None:
        """The deprecated prototype's CSV row coding (Summarization.java:67-77)."""
        properties[CSV_DELIM] = delim
        if encode_schema is not None:
            properties[INPUT_TF_EXAMPLE_CONFIG] = CsvCoding(encode_schema.get_field_names(),
                                                            encode_schema.get_data_types(), delim).describe()
            properties[ENCODING_CLASS] = "csv"
        if decode_schema is not None:
            properties[OUTPUT_TF_EXAMPLE_CONFIG] = CsvCoding(decode_schema.get_field_names(),
                                                             decode_schema.get_data_types(), delim).describe()
            properties[DECODING_CLASS] = "csv"

    @staticmethod
    def input_coding(properties: dict):
        """Codec of driver->worker records, or None when no input is configured."""
        if INPUT_TF_EXAMPLE_CONFIG not in properties:
            return None
        return _from_desc(properties.get(ENCODING_CLASS, "example"), properties[INPUT_TF_EXAMPLE_CONFIG])

    @staticmethod
    def output_coding(properties: dict):
        if OUTPUT_TF_EXAMPLE_CONFIG not in properties:
            return None
        return _from_desc(properties.get(DECODING_CLASS, "example"), properties[OUTPUT_TF_EXAMPLE_CONFIG])

    from .types import (data_types_list_to_type_information, data_types_to_type_information,  # noqa: E402
                        type_information_list_to_data_types, type_information_to_data_types)
    data_types_to_type_information = staticmethod(data_types_to_type_information)
    type_information_to_data_types = staticmethod(type_information_to_data_types)
    data_types_list_to_type_information = staticmethod(data_types_list_to_type_information)
    type_information_list_to_data_types = staticmethod(type_information_list_to_data_types)
    dataTypesToTypeInformation = data_types_to_type_information
    typeInformationToDataTypes = type_information_to_data_types
    dataTypesListToTypeInformation = data_types_list_to_type_information
    configureExampleCoding = configure_example_coding


def _as_dt(types):
    from .types import type_information_to_data_types
    return [t if isinstance(t, DataTypes) else type_information_to_data_types(t) for t in types]
