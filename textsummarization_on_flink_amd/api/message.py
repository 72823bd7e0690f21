"""Wire format of the summarization app: JSON ``{uuid, article, summary, reference}``
(``Message.java:10-70``).

``MessageDeserializationSchema(max_count)`` keeps the reference's bounded-stream rule:
``is_end_of_stream`` turns true once more than ``max_count`` messages were deserialised,
so a source emits at most ``max_count`` rows (``MessageDeserializationSchema.java:22-40``).
``MessageSerializationSchema`` logs and returns empty bytes for a row it cannot encode
(``MessageSerializationSchema.java:14-27``).
"""
from __future__ import annotations

import json
import logging
import threading
from dataclasses import asdict, dataclass
from typing import Optional

from .types import DataTypes, Row, TableSchema

log = logging.getLogger(__name__)
FIELDS = ("uuid", "article", "summary", "reference")
MESSAGE_SCHEMA = TableSchema(list(FIELDS), [DataTypes.STRING] * 4)


@dataclass
class Message:
    uuid: Optional[str] = None
    article: Optional[str] = None
    summary: Optional[str] = None
    reference: Optional[str] = None

    def to_json(self) -> str:
        return json.dumps(asdict(self))

    @classmethod
    def from_json(cls, s) -> "Message":
        d = json.loads(s)
        return cls(**{k: d.get(k) for k in FIELDS})

    def to_row(self) -> Row:
        return Row(self.uuid, self.article, self.summary, self.reference)

    toRow = to_row

    @classmethod
    def from_row(cls, row) -> "Message":
        return cls(*[None if v is None else str(v) for v in list(row)[:4]])


class MessageDeserializationSchema:
    def __init__(self, max_count: int):
        self.max_count = max_count
        self._counter = 0
        self._lock = threading.Lock()

    def deserialize(self, data: bytes) -> Row:
        row = Message.from_json(data).to_row()
        with self._lock:
            self._counter += 1
        return row

    def is_end_of_stream(self, row) -> bool:
        return self._counter > self.max_count

    def get_produced_type(self) -> TableSchema:
        return MESSAGE_SCHEMA


class MessageSerializationSchema:
    def serialize(self, row) -> bytes:
        try:
            vals = list(row)
            if len(vals) != 4 or not all(v is None or isinstance(v, str) for v in vals):
                raise TypeError(f"not a 4-string row: {row!r}")
            return Message(*vals).to_json().encode("utf-8")
        except Exception as e:  # noqa: BLE001 -- reference behaviour: log and emit nothing
            log.error("Failed to parse JSON: %r", e)
            return b""
