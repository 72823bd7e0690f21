"""Multi-process host input pipeline for the GPU trainer (reference
``batcher.py:246-272``: 16 example threads + 4 batch threads whose TF ops release the GIL).

In Python the threaded ``Batcher`` builds every Example (tokens -> ids, OOV maps, padding)
under the GIL, beside the thread that replays the train-step graphs; at B = 256 and ~21 ms
per step it would have to sustain ~12k examples/s.  ``ProcessBatcher`` moves all of it into
``workers`` forked processes:

  worker w:  .bin records k with k % world == rank and (k // world) % workers == w: every
             worker of every data-parallel rank walks the same shuffled file order per pass
             (one shared file-order seed), so each record is read by exactly one worker of
             one rank per pass
             -> Example -> length-bucketed batches (``bucketing_cache_size`` batches sorted by
             encoder length, shuffled) -> ``host_inputs`` -> ONE byte buffer in the engine's
             ``input_layout`` order -> a shared-memory SPSC ring (``runtime/ring.py``, native)
  trainer:   pops the next record round-robin over the rings and hands a ``PackedBatch`` to
             ``GraphTrainer.step``; ``set_batch`` copies the bytes into a pinned pack (one
             memcpy) and issues one H2D copy -- no per-example Python work in the trainer.

Workers are forked (never exec'd) and never touch the GPU; they end after a single pass
(``single_pass``) or when the trainer calls ``stop()``.  The threaded ``Batcher`` stays the
path for the CPU oracle, eval and decode.
"""
from __future__ import annotations

import json
import logging
import multiprocessing as mp
import os
import random
import struct
import uuid as _uuid
from typing import List, Optional

import numpy as np

from . import binfmt
from .batch import Batch, Example
from .vocab import Vocab, abstract2sents

log = logging.getLogger(__name__)
_HDR = struct.Struct("<I")


class _Shape:
    """``batch.enc_batch.shape`` for the engine's shape check, without the array."""

    def __init__(self, shape):
        self.shape = tuple(shape)


class PackedBatch:
    """What the GPU trainer needs of a Batch: the engine input pack (bytes in
    ``input_layout`` order) plus token accounting."""

    def __init__(self, host_pack: memoryview, enc_shape, n_tokens: int, n_padded: int, n_valid: int):
        self.host_pack = host_pack
        self.enc_batch = _Shape(enc_shape)
        self._tokens, self._padded, self.n_valid = n_tokens, n_padded, n_valid

    def num_tokens(self) -> int:
        return self._tokens

    def padded_tokens(self) -> int:
        return self._padded


def _push(ring, data: bytes) -> None:
    """Blocking push that gives up once the consumer closed the ring (trainer stopped)."""
    from ..runtime.ring import RingClosed
    while True:
        try:
            ring.push(data, timeout_ms=200)
            return
        except TimeoutError:
            if ring.closed:
                raise RingClosed(ring.name)


def _worker(w: int, n: int, ring_name: str, data_path: str, vocab: Vocab, hps, single_pass: bool, seed: int,
            pad_enc_to: Optional[int], D: int, cache: int, rank: int = 0, world: int = 1) -> None:
    from ..models.pointer_generator import host_inputs, input_layout, pack_host_inputs
    from ..runtime.ring import RecordRing, RingClosed
    ring = RecordRing.open(ring_name)
    B, T = hps.batch_size, pad_enc_to or hps.max_enc_steps
    layout, _ = input_layout(B, T, D)
    file_rng = random.Random(seed)  # identical in every worker of every rank: same file order per pass
    rng = random.Random(seed * 1009 + rank * n + w + 1)  # this worker's batch order
    failed = False
    try:
        def examples():
            k = 0  # index among this rank's records
            for rec in binfmt.example_generator(data_path, single_pass, file_rng, decode=False,
                                                shard=(rank, world)):
                mine = k % n == w
                k += 1
                if not mine:
                    continue
                for art, abs_ in binfmt.text_generator([binfmt.decode_example(rec)]):
                    yield Example(art, [s.strip() for s in abstract2sents(abs_)], vocab, hps)

        def emit(exs: List[Example]):
            b = Batch(exs, hps, vocab, pad_enc_to=pad_enc_to)
            if b.enc_batch.shape != (B, T):
                raise ValueError(f"batch shape {b.enc_batch.shape} != {(B, T)} (pad_enc_to must be max_enc_steps)")
            buf = pack_host_inputs(host_inputs(b, hps, D, sort_rows=True), layout)
            meta = json.dumps({"shape": [B, T], "tokens": b.num_tokens(), "padded": b.padded_tokens(),
                               "valid": int(b.valid.sum())}).encode()
            _push(ring, _HDR.pack(len(meta)) + meta + buf.tobytes())

        pending: List[Example] = []
        for ex in examples():
            pending.append(ex)
            if len(pending) >= B * cache:
                pending.sort(key=lambda e: e.enc_len)  # bucket by encoder length
                groups = [pending[i:i + B] for i in range(0, len(pending), B)]
                rng.shuffle(groups)
                for g in groups:
                    emit(g)
                pending = []
        if pending:  # single pass: the tail (a short last batch is padded with valid = 0 rows)
            pending.sort(key=lambda e: e.enc_len)
            for i in range(0, len(pending), B):
                g = pending[i:i + B]
                if len(g) == B or not hps.drop_last:
                    emit(g)
    except RingClosed:
        pass
    except BaseException as e:  # noqa: BLE001 -- reported to the trainer through the ring
        failed = True
        log.exception("loader worker %d failed", w)
        try:
            err = json.dumps({"error": repr(e)}).encode()
            ring.push(_HDR.pack(len(err)) + err, timeout_ms=1000)
        except Exception:  # noqa: BLE001
            pass
    finally:
        try:
            ring.close()
        except Exception:  # noqa: BLE001
            pass
        ring.release(unlink=False)
        # no atexit / finalizers of the parent's state in a forked child; a failed worker
        # exits non-zero so the trainer can tell a crash from the end of a pass
        os._exit(1 if failed else 0)


class ProcessBatcher:
    """``next_batch()`` -> PackedBatch | None (single pass exhausted); ``stop()``."""

    def __init__(self, data_path: str, vocab: Vocab, hps, single_pass: bool, workers: int, seed: int = 0,
                 pad_enc_to: Optional[int] = None, bucketing_cache_size: Optional[int] = None,
                 ring_bytes: int = 128 << 20, rank: int = 0, world: int = 1):
        """``rank`` / ``world``: this process's data-parallel share of the records (the same
        ``seed`` on every rank: it fixes the shared file order)."""
        from ..runtime.ring import RecordRing
        from ..utils.forking import fork_safe
        if workers < 1:
            raise ValueError("workers must be >= 1")
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world {world}")
        self.hps = hps
        self.D = hps.max_dec_steps
        self.single_pass = single_pass
        cache = 1 if single_pass else (bucketing_cache_size or 100)  # batcher.py:254
        tag = _uuid.uuid4().hex[:10]
        ctx = mp.get_context("fork")
        self.rings, self.procs = [], []
        with fork_safe():  # the children never collect the parent's (possibly GPU-owning) cycles
            for w in range(workers):
                ring = RecordRing.create(f"/tsamd_ld_{tag}_{w}", ring_bytes)
                p = ctx.Process(target=_worker, args=(w, workers, ring.name, data_path, vocab, hps, single_pass, seed,
                                                      pad_enc_to, self.D, cache, rank, world), daemon=True)
                p.start()
                self.rings.append(ring)
                self.procs.append(p)
        self._live = list(range(workers))
        self._rr = 0

    def next_batch(self, timeout: Optional[float] = None) -> Optional[PackedBatch]:
        """Next ready batch, trying the workers' rings round-robin (so a slow worker does
        not stall the others); None once every worker finished its single pass."""
        import time
        t0 = time.time()
        while self._live:
            n = len(self._live)
            for j in range(n):
                w = self._live[(self._rr + j) % n]
                try:
                    rec = self.rings[w].pop(timeout_ms=0 if j < n - 1 else 2)
                except TimeoutError:
                    if not self.procs[w].is_alive() and self.rings[w].stats()["pending_bytes"] == 0 \
                            and not self.rings[w].closed:
                        raise RuntimeError(f"loader worker {w} died (exit code {self.procs[w].exitcode})")
                    continue
                if rec is None:  # ring closed: the end of this worker's single pass, or a crash
                    self.procs[w].join(timeout=5)
                    code = self.procs[w].exitcode
                    if code or not self.single_pass:  # outside single_pass a worker never ends by itself
                        raise RuntimeError(f"loader worker {w} stopped (exit code {code})")
                    self._live.remove(w)
                    break
                self._rr = (self._rr + j + 1) % max(1, n)
                (hl,) = _HDR.unpack_from(rec, 0)
                meta = json.loads(rec[4:4 + hl])
                if "error" in meta:
                    raise RuntimeError(f"loader worker {w} failed: {meta['error']}")
                return PackedBatch(memoryview(rec)[4 + hl:], meta["shape"], meta["tokens"], meta["padded"],
                                   meta["valid"])
            if timeout is not None and time.time() - t0 > timeout:
                raise TimeoutError("no batch within timeout")
        return None

    def __iter__(self):
        while True:
            b = self.next_batch()
            if b is None:
                return
            yield b

    def stop(self):
        for r in self.rings:
            try:
                r.close()  # marks end of stream: a worker blocked in push() gets RingClosed
            except Exception:  # noqa: BLE001
                pass
        for p in self.procs:
            p.join(timeout=5)
            if p.is_alive():
                p.terminate()
        for r in self.rings:
            r.release(unlink=True)
        self.rings, self.procs, self._live = [], [], []

    def __del__(self):
        try:
            if self.procs:
                self.stop()
        except Exception:  # noqa: BLE001
            pass
