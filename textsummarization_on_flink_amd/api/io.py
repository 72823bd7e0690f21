"""Sources and sinks of the streaming environment (``App.java:84-143``,
``TensorFlowTest.java:74,128-137``, ``SourceSinkTest.java:41-124``).

Sources (iterate rows; ``open``/``close``):
  ``CollectionSource``, ``JsonLinesSource`` (one Message JSON per line, optional follow),
  ``SocketSource`` (newline-delimited text or JSON from ``host:port``, the
  ``socketTextStream`` of ``testInferenceFromSocket``), ``RingSource`` (records pushed by
  another process into a native shm ring), ``TimedSource`` (the latency test's
  ``DummyTimedSource`` with checkpointable ``count`` state), ``KafkaSource`` (optional
  adapter, needs ``kafka-python``; not installed in this image -> clear error).
Sinks (``open(schema)``/``write(row)``/``flush``/``close``):
  ``PrintSink``, ``CollectSink`` (optionally timestamped), ``CallbackSink``,
  ``JsonLinesSink``, ``SocketSink``, ``KafkaSink`` (optional adapter).
"""
from __future__ import annotations

import json
import os
import socket
import sys
import time
from typing import Callable, Iterable, List, Optional, Sequence

from .message import FIELDS, MESSAGE_SCHEMA, Message, MessageDeserializationSchema, MessageSerializationSchema
from .types import DataTypes, Row, TableSchema


class Source:
    def open(self):
        pass

    def close(self):
        pass

    def field_names(self) -> List[str]:
        raise ValueError(f"{type(self).__name__} needs explicit field names")

    def field_types(self) -> Optional[List[DataTypes]]:
        return None

    def __iter__(self):
        raise NotImplementedError


class CollectionSource(Source):
    def __init__(self, rows: Iterable):
        self.rows = list(rows)

    def __iter__(self):
        return iter(self.rows)


class JsonLinesSource(Source):
    """Messages (or any JSON objects) one per line; ``follow`` tails a growing file until
    a line ``{"__end__": true}`` or ``idle_timeout_s`` without new data."""

    def __init__(self, path: str, fields: Sequence[str] = FIELDS, follow: bool = False, idle_timeout_s: float = 5.0):
        self.path, self.fields, self.follow, self.idle = path, list(fields), follow, idle_timeout_s

    def field_names(self):
        return list(self.fields)

    def __iter__(self):
        with open(self.path, encoding="utf-8") as f:
            last = time.time()
            while True:
                line = f.readline()
                if not line:
                    if not self.follow or time.time() - last > self.idle:
                        return
                    time.sleep(0.01)
                    continue
                last = time.time()
                line = line.strip()
                if not line:
                    continue
                d = json.loads(line)
                if d.get("__end__"):
                    return
                yield Row(*[d.get(k) for k in self.fields])


class SocketSource(Source):
    """Newline-delimited records from a TCP server; JSON objects -> fields, or raw text
    into a single field."""

    def __init__(self, host: str, port: int, fields: Sequence[str] = FIELDS, fmt: str = "json",
                 connect_timeout_s: float = 10.0):
        self.host, self.port, self.fields, self.fmt = host, port, list(fields), fmt
        self.connect_timeout_s = connect_timeout_s
        self._sock = None

    def field_names(self):
        return list(self.fields)

    def open(self):
        self._sock = socket.create_connection((self.host, self.port), timeout=self.connect_timeout_s)
        self._sock.settimeout(None)

    def __iter__(self):
        buf = b""
        while True:
            chunk = self._sock.recv(65536)
            if not chunk:
                break
            buf += chunk
            while b"\n" in buf:
                line, buf = buf.split(b"\n", 1)
                r = self._parse(line)
                if r is not None:
                    yield r
        if buf.strip():
            r = self._parse(buf)
            if r is not None:
                yield r

    def _parse(self, line: bytes):
        line = line.strip()
        if not line:
            return None
        if self.fmt == "json":
            d = json.loads(line)
            return Row(*[d.get(k) for k in self.fields])
        return Row(line.decode("utf-8", errors="replace"))

    def close(self):
        if self._sock is not None:
            self._sock.close()
            self._sock = None


class RingSource(Source):
    """Records from a native shm ring written by an ingestion process (decoded with a
    ``MessageDeserializationSchema``-like ``deserialize``)."""

    def __init__(self, ring_name: str, deserializer=None, fields: Sequence[str] = FIELDS):
        self.ring_name = ring_name
        self.deser = deserializer or MessageDeserializationSchema(1 << 62)
        self.fields = list(fields)
        self._ring = None

    def field_names(self):
        return list(self.fields)

    def open(self):
        from ..runtime.ring import RecordRing
        self._ring = RecordRing.open(self.ring_name)

    def __iter__(self):
        for rec in self._ring:
            row = self.deser.deserialize(rec)
            if self.deser.is_end_of_stream(row):
                return
            yield row

    def close(self):
        if self._ring is not None:
            self._ring.release()
            self._ring = None


class TimedSource(Source):
    """``DummyTimedSource`` (SourceSinkTest.java:71-124): ``n`` rows, one every
    ``interval_s``; ``count`` is checkpointable state (``snapshot_state`` /
    ``restore_state``), so a restored source resumes where it stopped."""

    def __init__(self, n: int, interval_s: float, make_row: Optional[Callable[[int], object]] = None,
                 fields: Sequence[str] = ("input",)):
        self.n, self.interval_s = n, interval_s
        self.make_row = make_row or (lambda i: Row(f"data-{i}"))
        self.fields = list(fields)
        self.count = 0
        self.emit_times: List[float] = []

    def field_names(self):
        return list(self.fields)

    def snapshot_state(self) -> dict:
        return {"count": self.count}

    def restore_state(self, state: dict) -> None:
        self.count = int(state.get("count", 0))

    def __iter__(self):
        while self.count < self.n:
            row = self.make_row(self.count)
            self.count += 1
            self.emit_times.append(time.time())
            yield row
            if self.count < self.n:
                time.sleep(self.interval_s)


class KafkaSource(Source):
    """Optional Kafka adapter (``FlinkKafkaConsumer`` + ``MessageDeserializationSchema``,
    ``App.java:134-139``).  Requires the ``kafka-python`` package."""

    def __init__(self, topic: str, bootstrap_servers: str = "127.0.0.1:9092", group_id: str = "bode",
                 deserializer=None, from_earliest: bool = True, fields: Sequence[str] = FIELDS):
        self.topic, self.bootstrap, self.group = topic, bootstrap_servers, group_id
        self.deser = deserializer or MessageDeserializationSchema(8)
        self.from_earliest = from_earliest
        self.fields = list(fields)
        self._c = None

    def field_names(self):
        return list(self.fields)

    def open(self):
        try:
            from kafka import KafkaConsumer  # type: ignore
        except ImportError as e:
            raise ImportError("KafkaSource needs the 'kafka-python' package; use JsonLinesSource / SocketSource / "
                              "RingSource instead") from e
        self._c = KafkaConsumer(self.topic, bootstrap_servers=self.bootstrap, group_id=self.group,
                                auto_offset_reset="earliest" if self.from_earliest else "latest")

    def __iter__(self):
        for msg in self._c:
            row = self.deser.deserialize(msg.value)
            if self.deser.is_end_of_stream(row):
                return
            yield row

    def close(self):
        if self._c is not None:
            self._c.close()


# ---------------------------------------------------------------------- sinks
class Sink:
    def open(self, schema: Optional[TableSchema]):
        self.schema = schema

    def write(self, row: Row):
        raise NotImplementedError

    def flush(self):
        pass

    def close(self):
        pass


class PrintSink(Sink):
    def __init__(self, prefix: str = "", stream=None):
        self.prefix, self.stream = prefix, stream

    def write(self, row):
        print(f"{self.prefix}{row!r}", file=self.stream or sys.stdout, flush=True)


class CollectSink(Sink):
    def __init__(self, timestamps: bool = False):
        self.rows: List[Row] = []
        self.times: List[float] = []
        self.timestamps = timestamps

    def write(self, row):
        self.rows.append(row)
        self.times.append(time.time())


class CallbackSink(Sink):
    def __init__(self, fn: Callable[[Row], None]):
        self.fn = fn

    def write(self, row):
        self.fn(row)


class JsonLinesSink(Sink):
    def __init__(self, path: str):
        self.path = path
        self._f = None

    def open(self, schema):
        super().open(schema)
        os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
        self._f = open(self.path, "a", encoding="utf-8", buffering=1)

    def write(self, row):
        names = self.schema.get_field_names() if self.schema else [f"f{i}" for i in range(len(row))]
        self._f.write(json.dumps(dict(zip(names, list(row)))) + "\n")

    def flush(self):
        if self._f:
            self._f.flush()

    def close(self):
        if self._f:
            self._f.close()
            self._f = None


class SocketSink(Sink):
    def __init__(self, host: str, port: int, serializer=None):
        self.host, self.port = host, port
        self.ser = serializer
        self._sock = None

    def open(self, schema):
        super().open(schema)
        self._sock = socket.create_connection((self.host, self.port), timeout=10.0)

    def write(self, row):
        if self.ser is not None:
            data = self.ser.serialize(row)
        else:
            names = self.schema.get_field_names() if self.schema else [f"f{i}" for i in range(len(row))]
            data = json.dumps(dict(zip(names, list(row)))).encode("utf-8")
        self._sock.sendall(data + b"\n")

    def close(self):
        if self._sock is not None:
            self._sock.close()
            self._sock = None


class KafkaSink(Sink):
    """Optional Kafka adapter (``FlinkKafkaProducer`` + ``MessageSerializationSchema``)."""

    def __init__(self, topic: str, bootstrap_servers: str = "127.0.0.1:9092", serializer=None):
        self.topic, self.bootstrap = topic, bootstrap_servers
        self.ser = serializer or MessageSerializationSchema()
        self._p = None

    def open(self, schema):
        super().open(schema)
        try:
            from kafka import KafkaProducer  # type: ignore
        except ImportError as e:
            raise ImportError("KafkaSink needs the 'kafka-python' package; use JsonLinesSink / SocketSink") from e
        self._p = KafkaProducer(bootstrap_servers=self.bootstrap)

    def write(self, row):
        self._p.send(self.topic, self.ser.serialize(row))

    def flush(self):
        if self._p:
            self._p.flush()

    def close(self):
        if self._p:
            self._p.close()


def message_rows(messages: Iterable[Message]) -> List[Row]:
    return [m.to_row() for m in messages]


__all__ = ["Source", "CollectionSource", "JsonLinesSource", "SocketSource", "RingSource", "TimedSource",
           "KafkaSource", "Sink", "PrintSink", "CollectSink", "CallbackSink", "JsonLinesSink", "SocketSink",
           "KafkaSink", "MESSAGE_SCHEMA", "message_rows"]
