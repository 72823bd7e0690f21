"""Worker-process runtime: the replacement for Flink-AI-Extended's role launcher,
JVM<->Python data exchange and ``TFContext``.

Driver side (``WorkerJob``):
  * one Python process per worker (``worker_num``; one per GPU on a MI355X node), started
    with torchrun-style env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT)
    so ``torch.distributed`` (RCCL on GPU, gloo on CPU) rendezvouses over a TCPStore --
    the ZooKeeper + TF gRPC cluster of the reference;
  * per worker, an input and an output native shared-memory record ring
    (``runtime/ring.py`` over ``csrc/runtime/shm_ring.cpp``); input rows are encoded with
    the job's coding and distributed round-robin (Flink rebalance);
  * a drainer thread per output ring decodes result records and hands them downstream
    the moment they land (Issue-6 fix: results never lag behind inputs).
Worker side (``WorkerContext``, the ``TFContext`` equivalent passed to ``map_func``):
  role / index / cluster / properties, ``reader()`` (decoded input rows),
  ``flink_stream_dataset()`` (raw records), ``output_writer()``.

``ps_num`` must be 0: the parameter-server role is replaced by all-reduce (SURVEY PAR1).
"""
from __future__ import annotations

import importlib
import importlib.util
import json
import logging
import os
import socket
import subprocess
import sys
import tempfile
import threading
import time
import uuid as _uuid
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from ..runtime.ring import RecordRing, RingDrainer
from .coding import CodingUtils

log = logging.getLogger(__name__)
REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class JobExecutionError(RuntimeError):
    pass


@dataclass
class WorkerConfig:
    """``TFConfig(workerNum, psNum, properties, pythonFiles, funcName, envPath)``."""
    worker_num: int = 1
    ps_num: int = 0
    properties: Dict[str, str] = field(default_factory=dict)
    python_files: List[str] = field(default_factory=list)
    func_name: str = "main_on_flink"
    env_path: Optional[str] = None
    ring_capacity: int = 64 << 20
    timeout_s: float = 3600.0

    def validate(self):
        if self.ps_num:
            raise ValueError("ps_num > 0 is not supported: the parameter server is replaced by an RCCL all-reduce "
                             "across workers (set ps_num=0)")
        if self.worker_num < 1:
            raise ValueError("worker_num must be >= 1")
        if not self.python_files:
            raise ValueError("python scripts (train_scripts / inference_scripts) are required")


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# ---------------------------------------------------------------------- worker side
class _RingRowReader:
    """RowReader over the input ring (decoded dict rows; None at end of stream)."""

    def __init__(self, ring: Optional[RecordRing], coding):
        self.ring, self.coding = ring, coding

    def next_row(self, timeout: Optional[float] = None):
        if self.ring is None:
            return None
        rec = self.ring.pop(-1 if timeout is None else max(0, int(timeout * 1000)))
        if rec is None:
            return None
        return self.coding.decode_dict(rec) if self.coding else {"record": rec}

    def __iter__(self):
        while True:
            r = self.next_row()
            if r is None:
                return
            yield r


class OutputWriter:
    """Writes result rows to the output ring (``FlinkWriter``, ``flink_writer.py:17-37``)."""

    def __init__(self, ring: Optional[RecordRing], coding):
        self.ring, self.coding = ring, coding

    def write(self, row) -> None:
        if self.ring is None:
            raise RuntimeError("this job has no output schema (decode side not configured)")
        self.ring.push(row if isinstance(row, (bytes, bytearray)) else self.coding.encode(row))

    def write_result(self, uuid, article, summary, reference) -> None:
        self.write({"uuid": uuid, "article": article, "summary": summary, "reference": reference})

    def close(self) -> None:
        if self.ring is not None:
            self.ring.close()


class WorkerContext:
    def __init__(self, spec: dict):
        self.spec = spec
        self.role = spec.get("role", "worker")
        self.index = int(spec["index"])
        self.worker_num = int(spec["worker_num"])
        self.properties: Dict[str, str] = dict(spec["properties"])
        self.input_coding = CodingUtils.input_coding(self.properties)
        self.output_coding = CodingUtils.output_coding(self.properties)
        self._in = RecordRing.open(spec["input_ring"]) if spec.get("input_ring") else None
        self._out = RecordRing.open(spec["output_ring"]) if spec.get("output_ring") else None
        self._writer = OutputWriter(self._out, self.output_coding)

    # TFContext-style accessors
    def get_role_name(self) -> str:
        return self.role

    def get_index(self) -> int:
        return self.index

    def get_cluster(self) -> dict:
        return {"worker": [f"127.0.0.1:{self.spec.get('master_port', 0)}+{i}" for i in range(self.worker_num)]}

    get_tf_cluster = get_cluster

    def reader(self) -> _RingRowReader:
        return _RingRowReader(self._in, self.input_coding)

    def flink_stream_dataset(self):
        """Raw input records (bytes), like FAE's ``flink_stream_dataset``."""
        if self._in is None:
            return iter(())
        return iter(self._in)

    def output_writer(self) -> OutputWriter:
        return self._writer

    def close(self):
        self._writer.close()


def _load_entry(python_files: List[str], func_name: str) -> Callable:
    entry = python_files[0]
    for f in python_files:
        d = os.path.dirname(os.path.abspath(f)) if f.endswith(".py") else None
        if d and d not in sys.path:
            sys.path.insert(0, d)
    if entry.endswith(".py"):
        name = "flink_entry_" + os.path.splitext(os.path.basename(entry))[0]
        spec = importlib.util.spec_from_file_location(name, entry)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
    else:
        mod = importlib.import_module(entry)
    return getattr(mod, func_name)


def worker_main(spec_path: str) -> int:
    with open(spec_path) as f:
        spec = json.load(f)
    logging.basicConfig(level=logging.INFO, format=f"%(asctime)s w{spec['index']} %(levelname)s %(name)s: "
                                                   "%(message)s")
    ctx = WorkerContext(spec)
    try:
        fn = _load_entry(spec["python_files"], spec["func_name"])
        fn(ctx)
    finally:
        ctx.close()
    return 0


# ---------------------------------------------------------------------- driver side
class WorkerJob:
    """Launch ``worker_num`` processes running ``func_name`` from ``python_files``."""

    def __init__(self, config: WorkerConfig, on_output: Optional[Callable[[bytes], None]] = None,
                 name: str = "job"):
        config.validate()
        self.config = config
        self.on_output = on_output
        self.name = name
        self.procs: List[subprocess.Popen] = []
        self.in_rings: List[RecordRing] = []
        self.out_rings: List[RecordRing] = []
        self.drainers: List[RingDrainer] = []
        self._emit_lock = threading.Lock()
        self._rr = 0
        self._tmp = None
        self.has_input = CodingUtils.input_coding(config.properties) is not None
        self.has_output = CodingUtils.output_coding(config.properties) is not None

    def start(self):
        cfg = self.config
        tag = _uuid.uuid4().hex[:10]
        self._tmp = tempfile.mkdtemp(prefix=f"tsamd_{self.name}_")
        port = _free_port()
        py = os.path.join(cfg.env_path, "bin", "python") if cfg.env_path else sys.executable
        for i in range(cfg.worker_num):
            rin = RecordRing.create(f"/tsamd_{tag}_in{i}", cfg.ring_capacity) if self.has_input else None
            rout = RecordRing.create(f"/tsamd_{tag}_out{i}", cfg.ring_capacity) if self.has_output else None
            self.in_rings.append(rin)
            self.out_rings.append(rout)
            spec = {"role": "worker", "index": i, "worker_num": cfg.worker_num, "properties": cfg.properties,
                    "python_files": [os.path.abspath(f) if f.endswith(".py") else f for f in cfg.python_files],
                    "func_name": cfg.func_name, "input_ring": rin.name if rin else None,
                    "output_ring": rout.name if rout else None, "master_port": port}
            sp = os.path.join(self._tmp, f"worker{i}.json")
            with open(sp, "w") as f:
                json.dump(spec, f)
            env = dict(os.environ)
            env.update({"RANK": str(i), "LOCAL_RANK": str(i), "WORLD_SIZE": str(cfg.worker_num),
                        "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                        "PYTHONPATH": REPO_ROOT + os.pathsep + env.get("PYTHONPATH", "")})
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            from ..parallel.rccl_env import rccl_env
            rccl_env(env)  # RCCL's CU cap, before the worker initialises anything
            self.procs.append(subprocess.Popen([py, "-m", "textsummarization_on_flink_amd.api.worker", sp], env=env,
                                               cwd=os.getcwd()))
            if rout is not None:
                d = RingDrainer(rout, self._emit)
                d.start()
                self.drainers.append(d)

    def _emit(self, rec: bytes):
        # one drainer thread per worker: serialise the hand-off, downstream nodes and sinks
        # are single-threaded
        if self.on_output:
            with self._emit_lock:
                self.on_output(rec)

    def push(self, rec: bytes) -> None:
        """Round-robin a record to the workers' input rings."""
        if not self.has_input:
            return
        i = self._rr % len(self.in_rings)
        self._rr += 1
        while True:
            try:
                self.in_rings[i].push(rec, 200)
                return
            except TimeoutError:
                rc = self.procs[i].poll()
                if rc is not None:
                    if rc != 0:
                        raise JobExecutionError(f"{self.name}: worker {i} exited with code {rc}") from None
                    return  # the worker finished early (e.g. num_steps reached): its remaining input is dropped

    def finish(self, timeout_s: Optional[float] = None) -> None:
        """End of input: close input rings, wait for workers, drain outputs."""
        for r in self.in_rings:
            if r is not None:
                r.close()
        deadline = time.time() + (timeout_s or self.config.timeout_s)
        err = None
        for i, p in enumerate(self.procs):
            try:
                rc = p.wait(max(1.0, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                rc = p.wait()
                err = err or JobExecutionError(f"{self.name}: worker {i} timed out")
            if rc != 0:
                err = err or JobExecutionError(f"{self.name}: worker {i} exited with code {rc}")
                # a dead worker never closes its output ring; close it so the drainer ends
                if self.out_rings[i] is not None:
                    self.out_rings[i].close()
        for d in self.drainers:
            d.join()
            if d.error is not None:
                err = err or JobExecutionError(f"{self.name}: output drainer failed: {d.error!r}")
        self.release()
        if err:
            raise err

    def abort(self):
        for p in self.procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for r in self.out_rings:
            if r is not None:
                r.close()
        for d in self.drainers:
            d.join(5)
        self.release()

    def release(self):
        for r in self.in_rings + self.out_rings:
            if r is not None:
                r.release()
        self.in_rings, self.out_rings = [], []


if __name__ == "__main__":
    raise SystemExit(worker_main(sys.argv[1]))
