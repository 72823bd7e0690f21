"""Host input pipeline (reference ``batcher.py:222-649``).

``Batcher``      -- example-reader threads -> example queue -> batch threads (length
                    bucketing over ``bucketing_cache_size`` batches, shuffled batch order)
                    -> batch queue; a watchdog restarts dead threads.  ``single_pass``
                    uses one reader / one batcher / no bucketing and ends with ``None``.
                    Decode mode repeats one example ``batch_size`` times (beam-as-batch,
                    ``batcher.py:337-340``) or, for the batched device beam search, packs
                    ``batch_size`` DISTINCT articles (``decode_distinct=True``).
``RawTextBatcher`` -- one example per raw text file (``batcher.py:382-395``).
``FlinkTrainBatcher`` / ``FlinkInferenceBatcher`` -- batches from a row stream
                    (the worker context's reader, ``batcher.py:471-649``), references
                    sentence/word tokenised like the reference's nltk calls.

Fixes of reference defects:
  * Issue-5 / quirk 3: a short final batch no longer hangs (single_pass) or indexes past
    the end (FlinkTrainBatcher); it is padded with ``valid = 0`` rows (or dropped with
    ``hps.drop_last``);
  * ``FlinkInferenceBatcher`` can micro-batch several articles for the device beam search
    with a bounded wait, so streaming latency stays low (Issue-6 spirit).
"""
from __future__ import annotations

import glob
import logging
import queue
import random
import threading
import time
from typing import Callable, Iterable, Iterator, List, Optional, Sequence, Tuple

from . import binfmt
from .batch import Batch, Example
from .tokenize import sent_tokenize, word_tokenize
from .vocab import Vocab, abstract2sents

log = logging.getLogger(__name__)
_END = object()


def reference_to_sentences(reference: str) -> List[str]:
    """``[' '.join(word_tokenize(s)) for s in sent_tokenize(reference)]`` (batcher.py:579,643)."""
    return [" ".join(word_tokenize(s)) for s in sent_tokenize(reference)]


def _ex_text(v) -> str:
    if isinstance(v, (bytes, bytearray)):
        return v.decode("utf-8", errors="replace")
    if isinstance(v, (list, tuple)):
        return _ex_text(v[0]) if v else ""
    return "" if v is None else str(v)


class Batcher:
    BATCH_QUEUE_MAX = 100

    def __init__(self, data_path: str, vocab: Vocab, hps, single_pass: bool,
                 example_source: Optional[Callable[[], Iterator[Tuple[str, List[str], Optional[str]]]]] = None,
                 decode_distinct: bool = False, num_example_threads: Optional[int] = None,
                 num_batch_threads: Optional[int] = None, bucketing_cache_size: Optional[int] = None,
                 watchdog_secs: float = 60.0, seed: Optional[int] = None, pad_enc_to: Optional[int] = None,
                 rank: int = 0, world: int = 1):
        """``rank`` / ``world``: read only this data-parallel rank's share of the .bin records
        (record k of a pass goes to rank k % world; every rank passes the same ``seed``, which
        fixes the shared file order)."""
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world {world}")
        if world > 1 and seed is None:
            # the k % world record shards are disjoint only if every rank walks the same file
            # order, which the shared seed fixes
            raise ValueError("data-parallel Batcher (world > 1) needs a seed shared by every rank")
        self._shard = (rank, world)
        self._file_seed = seed
        self._data_path = data_path
        self._vocab = vocab
        self._hps = hps
        self._single_pass = single_pass
        self._source = example_source or self._bin_source
        self._decode_distinct = decode_distinct
        self._pad_enc_to = pad_enc_to
        self._rng = random.Random(seed if world == 1 else (None if seed is None else seed * 1009 + rank + 1))
        self._batch_queue: "queue.Queue" = queue.Queue(self.BATCH_QUEUE_MAX)
        self._example_queue: "queue.Queue" = queue.Queue(self.BATCH_QUEUE_MAX * hps.batch_size)
        if single_pass:
            n_ex, n_b, cache = 1, 1, 1
        else:
            n_ex, n_b, cache = 16, 4, 100  # batcher.py:251-254
        self._num_example_q_threads = num_example_threads or n_ex
        self._num_batch_q_threads = num_batch_threads or n_b
        self._bucketing_cache_size = bucketing_cache_size or cache
        if single_pass:
            self._num_example_q_threads = self._num_batch_q_threads = 1
        self._finished_reading = False
        self._stop = threading.Event()
        self.errors: List[BaseException] = []
        self._example_q_threads = [self._start(self.fill_example_queue) for _ in range(self._num_example_q_threads)]
        self._batch_q_threads = [self._start(self.fill_batch_queue) for _ in range(self._num_batch_q_threads)]
        self._watch_thread = None
        if not single_pass:
            self._watchdog_secs = watchdog_secs
            self._watch_thread = self._start(self.watch_threads)

    # ------------------------------------------------------------------ threads
    def _start(self, fn) -> threading.Thread:
        t = threading.Thread(target=self._guard(fn), daemon=True)
        t.start()
        return t

    def _guard(self, fn):
        def run():
            try:
                fn()
            except BaseException as e:  # noqa: BLE001 -- recorded; the watchdog restarts the thread
                if not self._stop.is_set():
                    log.error("batcher thread died: %r", e)
                    self.errors.append(e)
        return run

    def _bin_source(self) -> Iterator[Tuple[str, List[str], Optional[str]]]:
        file_rng = random.Random(self._rng.random() if self._shard[1] == 1 else random.Random(self._file_seed).random())
        gen = binfmt.text_generator(binfmt.example_generator(self._data_path, self._single_pass, file_rng,
                                                            shard=self._shard))
        for article, abstract in gen:
            yield article, [s.strip() for s in abstract2sents(abstract)], None

    def _put(self, q: "queue.Queue", item) -> bool:
        while not self._stop.is_set():
            try:
                q.put(item, timeout=0.1)
                return True
            except queue.Full:
                continue
        return False

    def _get(self, q: "queue.Queue"):
        while not self._stop.is_set():
            try:
                return q.get(timeout=0.1)
            except queue.Empty:
                continue
        return _END

    def fill_example_queue(self):
        for article, abstract_sentences, uuid in self._source():
            ex = Example(article, abstract_sentences, self._vocab, self._hps, uuid=uuid)
            if not self._put(self._example_queue, ex):
                return
        if self._single_pass:
            log.info("single_pass mode is on, so we've finished reading dataset. This thread is stopping.")
            self._finished_reading = True
            self._put(self._example_queue, _END)
        elif not self._stop.is_set():
            raise RuntimeError("single_pass mode is off but the example generator is out of data; error.")

    def _make_batch(self, exs: List[Example]) -> Batch:
        return Batch(exs, self._hps, self._vocab, pad_enc_to=self._pad_enc_to)

    def fill_batch_queue(self):
        hps = self._hps
        while not self._stop.is_set():
            if hps.mode == "decode" and not self._decode_distinct:
                ex = self._get(self._example_queue)
                if ex is _END:
                    self._put(self._batch_queue, _END)
                    return
                self._put(self._batch_queue, self._make_batch([ex] * hps.batch_size))
                continue
            inputs, ended = [], False
            for _ in range(hps.batch_size * self._bucketing_cache_size):
                ex = self._get(self._example_queue)
                if ex is _END:
                    ended = True
                    break
                inputs.append(ex)
            if self._stop.is_set():
                return
            if hps.mode != "decode":
                inputs = sorted(inputs, key=lambda e: e.enc_len)  # bucket by encoder length
            groups = [inputs[i:i + hps.batch_size] for i in range(0, len(inputs), hps.batch_size)]
            if groups and len(groups[-1]) < hps.batch_size and hps.drop_last:
                groups = groups[:-1]
            if not self._single_pass:
                self._rng.shuffle(groups)
            for g in groups:
                self._put(self._batch_queue, self._make_batch(g))
            if ended:
                self._put(self._batch_queue, _END)
                return

    def watch_threads(self):
        while not self._stop.wait(self._watchdog_secs):
            for idx, t in enumerate(self._example_q_threads):
                if not t.is_alive():
                    log.error("Found example queue thread dead. Restarting.")
                    self._example_q_threads[idx] = self._start(self.fill_example_queue)
            for idx, t in enumerate(self._batch_q_threads):
                if not t.is_alive():
                    log.error("Found batch queue thread dead. Restarting.")
                    self._batch_q_threads[idx] = self._start(self.fill_batch_queue)

    # ------------------------------------------------------------------ consumer
    def next_batch(self, timeout: Optional[float] = None) -> Optional[Batch]:
        """Next Batch; ``None`` once a single pass is exhausted."""
        if self._batch_queue.qsize() == 0:
            log.debug("Bucket input queue is empty when calling next_batch. Bucket queue size: %i, "
                      "Input queue size: %i", self._batch_queue.qsize(), self._example_queue.qsize())
        t0 = time.time()
        while True:
            try:
                b = self._batch_queue.get(timeout=0.1)
                break
            except queue.Empty:
                if self.errors and self._single_pass:
                    raise RuntimeError("batcher thread failed") from self.errors[0]
                if timeout is not None and time.time() - t0 > timeout:
                    raise TimeoutError("no batch within timeout")
        if b is _END:
            self._batch_queue.put(_END)  # every later call also sees end-of-data
            log.info("Finished reading dataset in single_pass mode.")
            return None
        return b

    def __iter__(self):
        while True:
            b = self.next_batch()
            if b is None:
                return
            yield b

    def stop(self):
        self._stop.set()


class RawTextBatcher(Batcher):
    """Inference on raw text files: the whole file is the article (word-tokenised) and the
    reference (``batcher.py:382-395``)."""

    def __init__(self, data_path, vocab, hps, single_pass, **kw):
        kw.setdefault("example_source", self._raw_source)
        super().__init__(data_path, vocab, hps, single_pass, **kw)

    def _raw_source(self):
        filelist = sorted(glob.glob(self._data_path))
        if not filelist:
            raise FileNotFoundError(f"Error: Empty filelist at {self._data_path}")
        while True:
            for f in filelist:
                with open(f, encoding="utf-8", errors="replace") as fh:
                    text = fh.read()
                yield " ".join(word_tokenize(text)), [text], f
            if self._single_pass:
                return


# ---------------------------------------------------------------------- row streams
class RowReader:
    """Protocol of a row stream: ``next_row(timeout)`` -> dict | None (end of stream),
    raises ``TimeoutError``.  ``IterRowReader`` adapts any iterable of dicts."""

    def next_row(self, timeout: Optional[float] = None):
        raise NotImplementedError


class IterRowReader(RowReader):
    def __init__(self, rows: Iterable[dict]):
        self._it = iter(rows)

    def next_row(self, timeout=None):
        return next(self._it, None)


class _StreamBatcher:
    def __init__(self, reader: RowReader, vocab: Vocab, hps):
        self._reader, self._vocab, self._hps = reader, vocab, hps
        self._eof = False

    def _example(self, row) -> Example:
        uuid = _ex_text(row.get("uuid"))
        article = _ex_text(row.get("article"))
        if getattr(self._hps, "flink_tokenize_article", False):
            article = " ".join(word_tokenize(article))
        reference = _ex_text(row.get("reference"))
        return Example(article, reference_to_sentences(reference), self._vocab, self._hps, uuid=uuid)

    def _read(self, timeout=None):
        if self._eof:
            return None
        r = self._reader.next_row(timeout)
        if r is None:
            self._eof = True
        return r


class FlinkTrainBatcher(_StreamBatcher):
    """``batch_size`` stream rows per Batch (``batcher.py:588-649``).  The last short
    batch is padded with ``valid = 0`` rows (the reference raised IndexError) or dropped
    with ``hps.drop_last``."""

    def __init__(self, reader, vocab, hps, pad_enc_to: Optional[int] = None):
        super().__init__(reader, vocab, hps)
        self._pad_enc_to = pad_enc_to

    def next_batch(self) -> Optional[Batch]:
        exs = []
        while len(exs) < self._hps.batch_size:
            r = self._read()
            if r is None:
                break
            exs.append(self._example(r))
        if not exs or (len(exs) < self._hps.batch_size and self._hps.drop_last):
            return None
        return Batch(exs, self._hps, self._vocab, pad_enc_to=self._pad_enc_to)


class FlinkInferenceBatcher(_StreamBatcher):
    """Decode batches from the stream (``batcher.py:539-585``).

    ``n_articles == 1``: one row, replicated ``batch_size`` (= beam) times -- the host
    beam search layout.  ``n_articles > 1``: up to ``n_articles`` distinct rows for the
    device beam search; after the first row arrives it takes every row already queued and
    waits at most ``max_wait_s`` for more, so a trickle of requests is still answered
    promptly (``tools/stream_latency.py``: p50 18 ms at one request per 50 ms, no wait)."""

    def __init__(self, reader, vocab, hps, n_articles: int = 1, max_wait_s: float = 0.0,
                 pad_enc_to: Optional[int] = None):
        super().__init__(reader, vocab, hps)
        self.n_articles = n_articles
        self.max_wait_s = max_wait_s
        self._pad_enc_to = pad_enc_to

    def next_batch(self) -> Optional[Batch]:
        r = self._read()
        if r is None:
            return None
        if self.n_articles == 1:
            ex = self._example(r)
            return Batch([ex] * self._hps.batch_size, self._hps, self._vocab, pad_enc_to=self._pad_enc_to)
        exs = [self._example(r)]
        deadline = time.time() + self.max_wait_s
        while len(exs) < self.n_articles:
            # requests already queued always join the batch; beyond those, wait at most until
            # the deadline (max_wait_s = 0: decode immediately with whatever has arrived)
            left = max(0.0, deadline - time.time())
            try:
                r = self._read(left)
            except TimeoutError:
                break
            if r is None:
                break
            exs.append(self._example(r))
        return Batch(exs, self._hps.replace(batch_size=self.n_articles), self._vocab, pad_enc_to=self._pad_enc_to)


FlinkBatcher = FlinkInferenceBatcher  # legacy name (batcher.py:413-468, dead code in the reference)


def examples_from_rows(rows: Sequence[dict], vocab: Vocab, hps) -> List[Example]:
    b = _StreamBatcher(IterRowReader(rows), vocab, hps)
    return [b._example(r) for r in rows]
