"""Stream-fed input pipelines at engine speed: packer processes between a worker's input
ring and the GPU engine (reference ``batcher.py:471-649``: ``AbstractFlinkReader`` /
``FlinkTrainBatcher`` / ``FlinkInferenceBatcher`` parse rows inside TF's C++ dataset runtime;
``App.java:83-132`` / ``run_summarization.py:370-399`` feed them).

A streaming worker (``flink_entry.main_on_flink``) receives coded rows on ONE shared-memory
input ring.  Decoding a row, tokenising its reference, building the Example / Batch and the
engine's input pack costs ~0.45 ms of Python per row -- a B = 256 train step consumes ~15k rows/s,
a 64-article beam batch ~6k/s -- so the trainer / decoder thread must not do it.  Here:

  input ring --(native fanout thread, ``RingPipe.fanout``)--> P packer rings
  packer p (forked process, never touches the GPU): rows -> Examples -> Batch -> ``host_inputs``
           -> ONE byte buffer in ``input_layout`` order -> its output ring
  engine thread: pops the packers' outputs (``PackedBatch``: one memcpy into the pinned pack,
           one H2D copy) -> GraphTrainer.step / DeviceBeamDecoder

Training (``StreamTrainPacker``): the fanout hands rows to packers in groups of B consecutive
rows (group k -> packer k % P) and the trainer pops packer k % P for batch k, so the batches and
their order are exactly those of the serial ``FlinkTrainBatcher`` (the last short batch padded
with ``valid = 0`` rows, or dropped with ``drop_last``).

Serving (``StreamDecodePacker``): rows go to packers one by one (round-robin); a packer takes the
rows already queued (up to ``n_articles``) and waits at most ``max_wait_s`` for more, like
``FlinkInferenceBatcher``.  It keeps each batch's strings (uuid, article, reference, in-article
OOVs) and ships only the pack; the decoder sends back the best hypothesis' token ids per article
and the packer turns them into result rows (ids -> words, [STOP] cut, sentence split --
``decode.py:159-185``) and encodes them onto its own result ring; a native fanin thread forwards
every result row to the worker's output ring the moment it lands (emit-immediately, Issue-6).
"""
from __future__ import annotations

import json
import logging
import multiprocessing as mp
import os
import struct
import time
import uuid as _uuid
from typing import List, Optional, Tuple

from .batch import Batch
from .batcher import IterRowReader, _StreamBatcher
from .loader import PackedBatch

log = logging.getLogger(__name__)
_HDR = struct.Struct("<I")


def _meta_record(meta: dict, payload: bytes = b"") -> bytes:
    m = json.dumps(meta).encode()
    return _HDR.pack(len(m)) + m + payload


def _split_record(rec: bytes):
    (hl,) = _HDR.unpack_from(rec, 0)
    return json.loads(rec[4:4 + hl]), memoryview(rec)[4 + hl:]


def _push(ring, data: bytes) -> None:
    """Blocking push that gives up once the consumer closed the ring."""
    from ..runtime.ring import RingClosed
    while True:
        try:
            ring.push(data, timeout_ms=200)
            return
        except TimeoutError:
            if ring.closed:
                raise RingClosed(ring.name)


class _Orphaned(Exception):
    pass


def _pop(ring, ppid: int):
    """Blocking pop that ends the packer if its parent (the stream worker) is gone."""
    while True:
        try:
            return ring.pop(timeout_ms=200)
        except TimeoutError:
            if os.getppid() != ppid:
                raise _Orphaned() from None


def default_packers(hps) -> int:
    """``--stream_packers`` (-1 = min(12, CPUs - 3): the driver, the engine thread and the
    fanout keep a core each)."""
    if getattr(hps, "stream_packers", -1) >= 0:
        return int(hps.stream_packers)
    return max(1, min(12, (os.cpu_count() or 4) - 3))


class _Pool:
    """P forked packer processes, each with an input ring (fed by the native fanout from the
    worker's input ring) and an output ring."""

    def __init__(self, target, n: int, extra_rings: int, ring_bytes: int, args: tuple):
        from ..runtime.ring import RecordRing
        self.interrupted = False
        from ..utils.forking import fork_safe
        if n < 1:
            raise ValueError("packers must be >= 1")
        tag = _uuid.uuid4().hex[:10]
        self.rings = [[RecordRing.create(f"/tsamd_sp_{tag}_{p}_{j}", ring_bytes) for j in range(2 + extra_rings)]
                      for p in range(n)]
        ctx = mp.get_context("fork")
        self.procs = []
        with fork_safe():  # the children never collect the parent's (possibly GPU-owning) cycles
            for p in range(n):
                pr = ctx.Process(target=target, args=(p, n, [r.name for r in self.rings[p]], *args), daemon=True)
                pr.start()
                self.procs.append(pr)
        self.pipes = []

    def check_alive(self, p: int) -> None:
        pr = self.procs[p]
        if not pr.is_alive() and pr.exitcode:
            raise RuntimeError(f"stream packer {p} died (exit code {pr.exitcode})")

    def pop(self, p: int, ring: int = 1, timeout_s: Optional[float] = None):
        """Blocking pop of packer p's ring ``ring``; None at its end of stream; raises if the
        packer died or reported an error."""
        t0 = time.time()
        while True:
            if self.interrupted:  # interrupt(): the consumer stopped before the stream ended
                return None
            try:
                rec = self.rings[p][ring].pop(timeout_ms=100)
            except TimeoutError:
                self.check_alive(p)
                if timeout_s is not None and time.time() - t0 > timeout_s:
                    raise
                continue
            if rec is None:
                self.procs[p].join(timeout=10)
                if self.procs[p].exitcode:
                    raise RuntimeError(f"stream packer {p} stopped (exit code {self.procs[p].exitcode})")
                return None
            meta, payload = _split_record(rec)
            if "error" in meta:
                raise RuntimeError(f"stream packer {p} failed: {meta['error']}")
            return meta, payload

    def check_feed(self) -> None:
        """At a consumer's end of stream: the input fanout (``pipes[0]``) must have ended at its
        source's end of stream.  A fanout that stopped on an error (a row larger than a packer
        ring, a packer ring closed early) also closes every packer input ring, which the packers
        cannot tell from a normal end -- so the error is raised here instead of the stream
        ending 'successfully' on truncated input."""
        if not self.pipes or self.pipes[0] is None:
            return
        fan, self.pipes[0] = self.pipes[0], None
        try:
            fan.join()
        except Exception as e:  # noqa: BLE001
            raise RuntimeError(f"stream input fanout failed: {e!r}") from e

    def stop(self):
        pipes = [p for p in self.pipes if p is not None]
        for pipe in pipes:
            pipe.stop()
        for pipe in pipes:
            try:
                pipe.join()
            except Exception as e:  # noqa: BLE001 -- cleanup (also on error paths): logged, not raised
                log.warning("stream pipe ended with %r", e)
        self.pipes = []
        for rs in self.rings:
            for r in rs:
                try:
                    r.close()  # producers blocked in push() see RingClosed; readers see end of stream
                except Exception:  # noqa: BLE001
                    pass
        for pr in self.procs:
            pr.join(timeout=5)
            if pr.is_alive():
                pr.terminate()
                pr.join(timeout=5)
        for rs in self.rings:
            for r in rs:
                r.release(unlink=True)
        self.rings, self.procs = [], []


def _packer_exit(failed: bool):
    # forked child: no atexit / finalizers of the parent's state
    os._exit(1 if failed else 0)


def _report(ring, e: BaseException):
    try:
        ring.push(_meta_record({"error": repr(e)}), timeout_ms=1000)
    except Exception:  # noqa: BLE001
        pass


# ---------------------------------------------------------------------- training
def _train_packer(p: int, n: int, names: List[str], coding, vocab, hps, T: int, D: int) -> None:
    from ..models.pointer_generator import host_inputs, input_layout, pack_host_inputs
    from ..runtime.ring import RecordRing, RingClosed
    rin, rout = RecordRing.open(names[0]), RecordRing.open(names[1])
    B = hps.batch_size
    layout, _ = input_layout(B, T, D)
    sb = _StreamBatcher(IterRowReader(()), vocab, hps)
    failed = False
    ppid = os.getppid()
    try:
        while True:
            exs = []
            while len(exs) < B:
                rec = _pop(rin, ppid)
                if rec is None:
                    break
                exs.append(sb._example(coding.decode_dict(rec)))
            if not exs or (len(exs) < B and hps.drop_last):
                break
            b = Batch(exs, hps, vocab, pad_enc_to=T)
            buf = pack_host_inputs(host_inputs(b, hps, D, sort_rows=True), layout)
            _push(rout, _meta_record({"shape": [B, T], "tokens": b.num_tokens(), "padded": b.padded_tokens(),
                                      "valid": len(exs)}, buf.tobytes()))
            if len(exs) < B:
                break
    except (RingClosed, _Orphaned):
        pass
    except BaseException as e:  # noqa: BLE001 -- reported to the trainer through the ring
        failed = True
        log.exception("stream train packer %d failed", p)
        _report(rout, e)
    finally:
        for r in (rout, rin):
            try:
                r.close()
            except Exception:  # noqa: BLE001
                pass
            r.release(unlink=False)
        _packer_exit(failed)


class StreamTrainPacker:
    """``next_batch()`` -> PackedBatch | None: the batches of ``FlinkTrainBatcher`` over the
    worker's input ring, built by ``packers`` processes (see the module docstring)."""

    def __init__(self, in_ring, coding, vocab, hps, packers: int, pad_enc_to: int, ring_bytes: int = 64 << 20):
        from ..runtime.ring import RingPipe
        self.hps, self.B, self.T, self.D = hps, hps.batch_size, pad_enc_to, hps.max_dec_steps
        self.pool = _Pool(_train_packer, packers, 0, ring_bytes, (coding, vocab, hps, pad_enc_to, self.D))
        # started after the fork: the forked packers must not inherit a running thread
        self.pool.pipes.append(RingPipe.fanout(in_ring, [r[0] for r in self.pool.rings], group=self.B))
        self.k = 0
        self.done = False

    def next_batch(self) -> Optional[PackedBatch]:
        if self.done:
            return None
        p = self.k % len(self.pool.procs)
        got = self.pool.pop(p)
        if got is None:  # packer p had no group k: the stream ended (or its feed failed: raises)
            self.done = True
            self.pool.check_feed()
            return None
        meta, payload = got
        self.k += 1
        return PackedBatch(payload, meta["shape"], meta["tokens"], meta["padded"], meta["valid"])

    def interrupt(self):
        """Make a pending / later ``next_batch`` return None within one 100 ms pop slice, without
        releasing anything (a prefetch thread may still be inside the pop; ``stop`` after it)."""
        self.pool.interrupted = True

    def stop(self):
        self.pool.stop()


# ---------------------------------------------------------------------- serving
def finish_rows(entries, results, vocab, hps, html_escape: bool = False):
    """(uuid, article, summary, reference) per decoded article: the best hypothesis' token ids
    (without [START]) -> words (in-article OOVs restored) -> cut at [STOP] -> sentences split
    at "." joined with two spaces (``decode.py:159-185``)."""
    from ..decode.decoder import flink_summary
    out = []
    for (uuid, article, ref_sents, oovs), ids in zip(entries, results):
        summary, reference = flink_summary(ids, vocab, oovs if hps.pointer_gen else None, ref_sents, html_escape)
        out.append((uuid, article, summary, reference))
    return out




_EX = struct.Struct("<iii")  # example record: (example id, encoder length, first target id) + enc + ext ids
_RES = struct.Struct("<i")   # result record: n, then n (example id, length) int32 pairs, then the ids


def _results(rec) -> List[Tuple[int, List[int]]]:
    """A result record -> [(example id, token ids)]."""
    import numpy as np
    n = _RES.unpack_from(rec, 0)[0]
    head = np.frombuffer(rec, dtype=np.int32, count=2 * n, offset=_RES.size).reshape(n, 2)
    body = np.frombuffer(rec, dtype=np.int32, offset=_RES.size + 8 * n).tolist()
    out, o = [], 0
    for e, L in head.tolist():
        out.append((e, body[o:o + L]))
        o += L
    return out


def _decode_packer(p: int, n: int, names: List[str], coding, out_coding, vocab, hps, T: int) -> None:
    """Rows -> Examples (strings kept here, the id arrays shipped); result token ids -> result
    rows.  Batches are formed by the decoder from whatever Examples are ready when it needs one
    (``StreamDecodePacker.poll``)."""
    import numpy as np
    from ..runtime.ring import RecordRing, RingClosed
    rin, rout, rres, rfin = (RecordRing.open(x) for x in names)
    sb = _StreamBatcher(IterRowReader(()), vocab, hps.replace(max_enc_steps=T))
    pending = {}   # example id -> (uuid, article, reference sentences, in-article OOVs)
    eid = 0
    in_open, failed = True, False
    ppid = os.getppid()
    fields = ("uuid", "article", "summary", "reference")

    def drain_results(block: bool):
        while pending:
            try:
                rec = rres.pop(timeout_ms=100 if block else 0)
            except TimeoutError:
                if block:
                    if os.getppid() != ppid:
                        raise _Orphaned() from None
                    continue
                return
            _finish(rec)
            if block:
                return

    def _try(ring, ms):
        try:
            return True, ring.pop(timeout_ms=ms)
        except TimeoutError:
            return False, None

    def _finish(rec):
        if rec is None:
            raise RuntimeError("decoder closed the result ring with examples pending")
        res = _results(rec)
        ents = [pending.pop(e) for e, _ids in res]
        for row in finish_rows(ents, [ids for _e, ids in res], vocab, hps, bool(hps.html_escape)):
            _push(rfin, out_coding.encode(dict(zip(fields, row))))

    try:
        while in_open or pending:
            if not in_open:
                drain_results(block=True)
                continue
            if pending:
                # results outstanding: check the result ring first and only peek at the input; an
                # idle wait is on the result ring (its poll backoff stays < 1 ms), so a finished
                # summary is written out within a fraction of a millisecond
                got, rr = _try(rres, 0)
                if got:
                    _finish(rr)
                    continue
                got, rec = _try(rin, 0)
                if not got:
                    got, rr = _try(rres, 1)
                    if got:
                        _finish(rr)
                    continue
            else:
                got, rec = _try(rin, 2)
                if not got:
                    if os.getppid() != ppid:
                        raise _Orphaned() from None
                    continue
            if rec is None:
                in_open = False
                rout.close()  # no more examples from this packer
                continue
            ex = sb._example(coding.decode_dict(rec))
            # the serial writer's rule (decoder.py handle): only a missing uuid gets a synthetic one
            pending[eid] = (ex.uuid if ex.uuid is not None else "uuid-%d-%d" % (p, eid), ex.original_article,
                            ex.original_abstract_sents, ex.article_oovs)
            enc = np.asarray(ex.enc_input, dtype=np.int32)
            ext = np.asarray(ex.enc_input_extend_vocab, dtype=np.int32)
            _push(rout, _EX.pack(eid, ex.enc_len, ex.target[0]) + enc.tobytes() + ext.tobytes())
            eid += 1
    except (RingClosed, _Orphaned):
        pass
    except BaseException as e:  # noqa: BLE001
        failed = True
        log.exception("stream decode packer %d failed", p)
        try:
            m = json.dumps({"error": repr(e)}).encode()
            rout.push(_EX.pack(-1, len(m), 0) + m, timeout_ms=1000)
        except Exception:  # noqa: BLE001
            pass
    finally:
        for r in (rout, rfin, rin, rres):
            try:
                r.close()
            except Exception:  # noqa: BLE001
                pass
            r.release(unlink=False)
        _packer_exit(failed)


class _DecodeRows:
    """The Batch fields ``host_inputs`` reads for a decode engine (D = 1), built from the
    packers' id arrays: padding rows copy the last real article with valid = 0, exactly like
    ``Batch``; decoder input [START], first target id, mask 1 (every dec_len >= 1)."""

    def __init__(self, items, Na: int, T: int, pad_id: int, start_id: int):
        import numpy as np
        n = len(items)
        rows = list(items) + [items[-1]] * (Na - n)
        self.enc_batch = np.full((Na, T), pad_id, dtype=np.int32)
        self.enc_batch_extend_vocab = np.full((Na, T), pad_id, dtype=np.int32)
        for i, (enc, ext, _t0) in enumerate(rows):
            self.enc_batch[i, :len(enc)] = enc
            self.enc_batch_extend_vocab[i, :len(ext)] = ext
        self.enc_lens = np.array([len(r[0]) for r in rows], dtype=np.int32)
        self.valid = np.zeros(Na, np.float32)
        self.valid[:n] = 1.0
        self.dec_batch = np.full((Na, 1), start_id, dtype=np.int32)
        self.target_batch = np.array([[r[2]] for r in rows], dtype=np.int32)
        self.dec_padding_mask = np.ones((Na, 1), np.float32)


class DecodePackedBatch(PackedBatch):
    """A serving batch: the engine pack plus (packer, example id) of every valid row."""

    def __init__(self, payload, Na: int, T: int, owners):
        super().__init__(payload, (Na, T), 0, 0, len(owners))
        self.owners = owners


class StreamDecodePacker:
    """Serving side: ``poll(block)`` -> DecodePackedBatch | None (end of stream) | NOT_READY;
    ``send_results(batch, token_id_lists)``; ``close()`` after the last result.  Result rows
    reach ``out_ring`` through the native fanin.

    A batch is formed when the decoder asks for one, from every Example the packers have ready
    (up to ``n_articles``): under load the batches are full, a lone request is decoded at once
    (after ``max_wait_s`` at most for company, ``FlinkInferenceBatcher``'s policy)."""

    NOT_READY = object()

    def __init__(self, in_ring, out_ring, coding, out_coding, vocab, hps, packers: int, n_articles: int, T: int,
                 max_wait_s: float, ring_bytes: int = 32 << 20):
        from ..data.vocab import PAD_TOKEN, START_DECODING
        from ..models.pointer_generator import input_layout
        from ..runtime.ring import RingPipe
        self.Na, self.T, self.max_wait_s = n_articles, T, max_wait_s
        self.hb = hps.replace(batch_size=n_articles)
        self.layout, _ = input_layout(n_articles, T, 1)
        self.pad_id, self.start_id = vocab.word2id(PAD_TOKEN), vocab.word2id(START_DECODING)
        self.pool = _Pool(_decode_packer, packers, 2, ring_bytes, (coding, out_coding, vocab, hps, T))
        rs = self.pool.rings
        self.pool.pipes.append(RingPipe.fanout(in_ring, [r[0] for r in rs], group=1))
        # result rows -> the worker's output ring (closed by the worker context at the end)
        self.fanin = RingPipe.fanin([r[3] for r in rs], out_ring, close_dst=False)
        self._live = list(range(len(rs)))
        self._rr = 0

    def _gather(self, items, owners) -> None:
        """Pop ready Examples round-robin over the packers (non-blocking) up to n_articles."""
        import numpy as np
        progress = True
        while progress and len(items) < self.Na and self._live:
            progress = False
            live = self._live[self._rr:] + self._live[:self._rr]
            for p in live:
                if len(items) >= self.Na:
                    break
                try:
                    rec = self.pool.rings[p][1].pop(timeout_ms=0)
                except TimeoutError:
                    continue
                if rec is None:  # packer p's input ended and all its examples were handed out
                    self._live.remove(p)
                    continue
                progress = True
                eid, L, t0 = _EX.unpack_from(rec, 0)
                if eid < 0:
                    raise RuntimeError(f"stream packer {p} failed: {json.loads(rec[_EX.size:])['error']}")
                a = np.frombuffer(rec, dtype=np.int32, count=2 * L, offset=_EX.size)
                items.append((a[:L], a[L:], t0))
                owners.append((p, eid))
            if self._live:
                self._rr = (self._rr + 1) % len(self._live)

    def poll(self, block: bool):
        from ..models.pointer_generator import host_inputs, pack_host_inputs
        items, owners = [], []
        self._gather(items, owners)
        if not items:
            if not self._live:
                self.pool.check_feed()
                return None
            if not block:
                return self.NOT_READY
            spins = 0
            while not items and self._live:
                time.sleep(0.0002)
                spins += 1
                if spins % 500 == 0:
                    for p in self._live:
                        self.pool.check_alive(p)
                self._gather(items, owners)
            if not items:
                self.pool.check_feed()
                return None
        if self.max_wait_s > 0 and len(items) < self.Na:
            deadline = time.time() + self.max_wait_s
            while len(items) < self.Na and self._live and time.time() < deadline:
                time.sleep(0.0002)
                self._gather(items, owners)
        rows = _DecodeRows(items, self.Na, self.T, self.pad_id, self.start_id)
        buf = pack_host_inputs(host_inputs(rows, self.hb, 1, need_grad=False), self.layout)
        return DecodePackedBatch(memoryview(buf), self.Na, self.T, owners)

    def send_results(self, batch: DecodePackedBatch, ids: List[List[int]]) -> None:
        """Best-hypothesis token ids (after [START]) per valid row, routed to the packers: one
        binary record per packer, (example id, length) int32 pairs then the ids (``_results``)."""
        import numpy as np
        per = {}
        for (p, eid), t in zip(batch.owners, ids):
            per.setdefault(p, []).append((eid, t))
        for p, r in per.items():
            head = np.array([(e, len(t)) for e, t in r], dtype=np.int32).reshape(-1)
            body = np.concatenate([np.asarray(t, dtype=np.int32) for _e, t in r]) if r else np.zeros(0, np.int32)
            _push(self.pool.rings[p][2], _RES.pack(len(r)) + head.tobytes() + body.tobytes())

    def close(self) -> None:
        """After the last result: end the result rings, let the packers flush, join the fanin."""
        for rs in self.pool.rings:
            rs[2].close()
        for pr in self.pool.procs:
            pr.join()
        bad = [p for p, pr in enumerate(self.pool.procs) if pr.exitcode]
        self.fanin.join()
        self.pool.stop()
        if bad:
            raise RuntimeError(f"stream packers {bad} failed")

    def stop(self):
        self.fanin.stop()
        try:
            self.fanin.join()
        except Exception:  # noqa: BLE001
            pass
        self.pool.stop()
