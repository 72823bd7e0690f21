"""Lazy streaming table environment (replaces Flink's ``StreamExecutionEnvironment`` +
``StreamTableEnvironment`` for this framework's pipelines).

Programs build a DAG lazily -- sources, ``select``/``where``/``map`` operators, external
worker jobs (training / inference processes, ``stages.py``) and sinks -- and nothing runs
until ``env.execute()`` (the reference's "fit returns immediately, training runs at
execute()" model, ``App.java:102-103``).

Execution is push-based: each source runs on its own thread and pushes rows through the
operators; a row fans out to every downstream consumer (so one Kafka/socket input can
feed both a print sink and a model, ``App.java:97-102``); external jobs emit their result
rows from their output-drainer threads as soon as they land (emit-immediately, Issue-6).
Sinks serialise writes with a per-sink lock.  A node finishes when all its upstreams have
finished; an external job with an ``after`` dependency (train-then-infer in ONE job, the
reference's Issue-1) buffers its input until the dependency's workers have exited.
"""
from __future__ import annotations

import logging
import threading
from collections import deque
from typing import Callable, Iterable, List, Optional, Sequence

from .types import DataTypes, Row, TableSchema, parse_fields, schema_of

log = logging.getLogger(__name__)


# ---------------------------------------------------------------------- nodes
class Node:
    def __init__(self, env: "StreamEnvironment", schema: Optional[TableSchema], name: str = ""):
        self.env = env
        self.schema = schema
        self.name = name or type(self).__name__
        self.children: List["Node"] = []
        self.n_upstream = 0
        self._finished_up = 0
        self._lock = threading.Lock()
        env._nodes.append(self)

    def connect(self, child: "Node") -> "Node":
        self.children.append(child)
        child.n_upstream += 1
        return child

    def open(self):
        pass

    def process(self, row: Row):
        self.emit(row)

    def emit(self, row: Row):
        for c in self.children:
            c.process(row)

    def upstream_finished(self):
        with self._lock:
            self._finished_up += 1
            done = self._finished_up >= self.n_upstream
        if done:
            self.finish()

    def finish(self):
        for c in self.children:
            c.upstream_finished()

    def close(self):
        pass


class SourceNode(Node):
    def __init__(self, env, source, schema: TableSchema, name=""):
        super().__init__(env, schema, name or type(source).__name__)
        self.source = source

    def run(self):
        try:
            self.source.open()
            for rec in self.source:
                self.emit(rec if isinstance(rec, Row) else _to_row(rec, self.schema))
        finally:
            try:
                self.source.close()
            finally:
                self.finish()  # downstream jobs must see end-of-input even if the source failed


class SelectNode(Node):
    def __init__(self, env, parent_schema: TableSchema, fields: Sequence[str]):
        super().__init__(env, parent_schema.project(fields), "select(" + ",".join(fields) + ")")
        self.idx = [parent_schema.index_of(f) for f in fields]

    def process(self, row):
        self.emit(Row(*[row[i] for i in self.idx]))


class FuncNode(Node):
    def __init__(self, env, schema, fn: Callable, kind: str):
        super().__init__(env, schema, kind)
        self.fn, self.kind = fn, kind

    def process(self, row):
        if self.kind == "where":
            if self.fn(row):
                self.emit(row)
        else:
            out = self.fn(row)
            if out is not None:
                self.emit(out if isinstance(out, Row) else _to_row(out, self.schema))


class SinkNode(Node):
    def __init__(self, env, sink, schema):
        super().__init__(env, schema, type(sink).__name__)
        self.sink = sink
        self._wlock = threading.Lock()

    def open(self):
        self.sink.open(self.schema)

    def process(self, row):
        with self._wlock:
            self.sink.write(row)

    def finish(self):
        with self._wlock:
            self.sink.flush()

    def close(self):
        self.sink.close()


class ExternalNode(Node):
    """Rows -> worker job (coded records over shm rings) -> result rows."""

    def __init__(self, env, job_factory: Callable, input_coding, output_schema: Optional[TableSchema],
                 output_coding, name="external", after: Optional["ExternalNode"] = None):
        super().__init__(env, output_schema, name)
        self.job_factory = job_factory
        self.input_coding = input_coding
        self.output_coding = output_coding
        self.after = after
        self.job = None
        self._started = threading.Event()
        self._done = threading.Event()
        self._buf: deque = deque()
        self._buf_lock = threading.Lock()
        self.error: Optional[BaseException] = None

    def open(self):
        self.job = self.job_factory(self._on_output)
        if self.after is None:
            self._start()
        else:
            threading.Thread(target=self._start_after, daemon=True).start()

    def _start_after(self):
        self.after._done.wait()
        try:
            if self.after.error is None:
                self._start()
        except BaseException as e:  # noqa: BLE001
            self.error = e
            self.env._record_error(e)
        finally:
            if self.after.error is not None:
                self._done.set()

    def _start(self):
        self.job.start()
        with self._buf_lock:
            while self._buf:
                self.job.push(self._buf.popleft())
            self._started.set()
        if self.n_upstream == 0:  # decode-only job: no input stream
            threading.Thread(target=self._finish_job, daemon=True).start()

    def _on_output(self, rec: bytes):
        self.emit(self.output_coding.decode(rec))

    def process(self, row):
        if self.input_coding is None:
            return
        rec = self.input_coding.encode(row)
        if not self._started.is_set():
            with self._buf_lock:
                if not self._started.is_set():
                    self._buf.append(rec)
                    return
        self.job.push(rec)

    def finish(self):
        if self.after is not None and not self._started.is_set():
            threading.Thread(target=self._finish_when_started, daemon=True).start()
            return
        self._finish_job()

    def _finish_when_started(self):
        while not self._started.wait(0.1):
            if self._done.is_set():
                return
        self._finish_job()

    def _finish_job(self):
        try:
            self.job.finish()
        except BaseException as e:  # noqa: BLE001 -- surfaced by execute()
            self.error = e
            self.env._record_error(e)
        finally:
            self._done.set()
            super().finish()

    def close(self):
        if self.job is not None and not self._done.is_set():
            self.job.abort()


def _to_row(rec, schema: Optional[TableSchema]) -> Row:
    if isinstance(rec, Row):
        return rec
    if isinstance(rec, dict):
        return Row(*[rec.get(n) for n in schema.get_field_names()])
    if isinstance(rec, (list, tuple)):
        return Row(*rec)
    return Row(rec)


# ---------------------------------------------------------------------- Table
class Table:
    def __init__(self, env: "StreamEnvironment", node: Node):
        self.env = env
        self.node = node

    def get_schema(self) -> TableSchema:
        return self.node.schema

    getSchema = get_schema

    def print_schema(self):
        print(self.node.schema)

    printSchema = print_schema

    def select(self, fields) -> "Table":
        names = parse_fields(fields)
        return Table(self.env, self.node.connect(SelectNode(self.env, self.node.schema, names)))

    def where(self, pred: Callable[[Row], bool]) -> "Table":
        return Table(self.env, self.node.connect(FuncNode(self.env, self.node.schema, pred, "where")))

    filter = where

    def map(self, fn: Callable, names: Optional[Sequence[str]] = None,
            types: Optional[Sequence[DataTypes]] = None) -> "Table":
        schema = schema_of(names, types) if names is not None else self.node.schema
        return Table(self.env, self.node.connect(FuncNode(self.env, schema, fn, "map")))

    def add_sink(self, sink) -> "Table":
        self.node.connect(SinkNode(self.env, sink, self.node.schema))
        return self

    addSink = add_sink

    def print(self, prefix: str = "") -> "Table":
        from .io import PrintSink
        return self.add_sink(PrintSink(prefix))

    def collect(self) -> List[Row]:
        """Registers a collecting sink; the list fills during ``env.execute()``."""
        from .io import CollectSink
        s = CollectSink()
        self.add_sink(s)
        return s.rows

    def __repr__(self):
        return f"Table({self.node.name}, {self.node.schema.get_field_names() if self.node.schema else None})"


# ---------------------------------------------------------------------- environment
class StreamEnvironment:
    """One object plays both ``StreamExecutionEnvironment`` and ``StreamTableEnvironment``."""

    def __init__(self, parallelism: int = 1):
        self.parallelism = parallelism
        self._nodes: List[Node] = []
        self._errors: List[BaseException] = []
        self._elock = threading.Lock()
        self.executed = 0

    @classmethod
    def create_local_environment(cls, parallelism: int = 1) -> "StreamEnvironment":
        return cls(parallelism)

    createLocalEnvironment = create_local_environment
    get_execution_environment = create_local_environment

    @staticmethod
    def create(env: "StreamEnvironment") -> "StreamEnvironment":
        """``StreamTableEnvironment.create(streamEnv)``: the same object here."""
        return env

    # sources
    def from_source(self, source, fields=None, types: Optional[Sequence[DataTypes]] = None) -> Table:
        names = parse_fields(fields) if fields is not None else source.field_names()
        schema = schema_of(names, types if types is not None else getattr(source, "field_types", lambda: None)())
        return Table(self, SourceNode(self, source, schema))

    add_source = from_source

    def from_collection(self, rows: Iterable, fields, types: Optional[Sequence[DataTypes]] = None) -> Table:
        from .io import CollectionSource
        return self.from_source(CollectionSource(rows), fields, types)

    fromCollection = from_collection

    def from_data_stream(self, table_or_source, fields=None) -> Table:
        """``tableEnv.fromDataStream(stream, "uuid,article,summary,reference")``."""
        if isinstance(table_or_source, Table):
            if fields is None:
                return table_or_source
            names = parse_fields(fields)
            old = table_or_source.node.schema
            return table_or_source.map(lambda r: r, names, old.get_data_types()[:len(names)])
        return self.from_source(table_or_source, fields)

    fromDataStream = from_data_stream

    def to_append_stream(self, table: Table) -> Table:
        return table

    toAppendStream = to_append_stream

    def _record_error(self, e: BaseException):
        with self._elock:
            self._errors.append(e)

    def execute(self, job_name: str = "job"):
        """Run every registered node to completion; raises the first error."""
        from .worker import JobExecutionError
        nodes = list(self._nodes)
        self._nodes = []  # a new program may be built on the same env afterwards
        self._errors = []
        opened = []
        threads = []
        try:
            for n in reversed(nodes):  # sinks/jobs before sources
                n.open()
                opened.append(n)
            for n in nodes:
                if isinstance(n, SourceNode):
                    t = threading.Thread(target=self._guard(n.run), name=f"src-{n.name}", daemon=True)
                    t.start()
                    threads.append(t)
            for t in threads:
                t.join()
            for n in nodes:
                if isinstance(n, ExternalNode):
                    while not n._done.wait(0.1):
                        if self._errors:  # a failed source/job: abort the rest (close() below)
                            break
        except BaseException as e:  # noqa: BLE001
            self._record_error(e)
        finally:
            for n in opened:
                try:
                    n.close()
                except Exception as e:  # noqa: BLE001
                    self._record_error(e)
        self.executed += 1
        if self._errors:
            e = self._errors[0]
            if isinstance(e, JobExecutionError):
                raise e
            raise JobExecutionError(f"{job_name} failed: {e!r}") from e
        return {"job_name": job_name, "nodes": len(nodes)}

    def _guard(self, fn):
        def run():
            try:
                fn()
            except BaseException as e:  # noqa: BLE001
                self._record_error(e)
        return run


StreamExecutionEnvironment = StreamEnvironment
StreamTableEnvironment = StreamEnvironment
TableEnvironment = StreamEnvironment
