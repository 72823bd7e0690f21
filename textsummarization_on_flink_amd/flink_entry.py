"""Worker entry point for the streaming API: ``main_on_flink(context)``
(reference ``run_summarization.py:370-426``; SURVEY 3.1, 3.2, 2.10 "Python entry contract").

The job's hyper-parameter string (``--mode=train ...``, first token a placeholder) is read
from ``context.properties[<hyper_params_key>]`` and parsed leniently.  ``mode=train`` runs
``training_on_flink`` (stream rows -> ``FlinkTrainBatcher`` -> trainer; ``worker_num > 1``
is synchronous data parallel over RCCL/gloo with lock-step end-of-stream), ``mode=decode``
runs ``inference_on_flink`` (stream rows -> beam search -> ``FlinkWriter`` results,
emitted per article).  There is no ``ps`` role: ``ps_num`` must be 0.
"""
from __future__ import annotations

import logging

import torch

from textsummarization_on_flink_amd.config import parse_hyperparam_string
from textsummarization_on_flink_amd.parallel.dist import DistInfo, SyncedBatcher, init_from_env

log = logging.getLogger("flink_entry")
DEFAULT_KEY = "TF_Hyperparameter"


class FlinkWriter:
    """Result sink of the decoder (``flink_writer.py:17-37``): one row
    ``(uuid, article, summary, reference)`` per decoded article, written immediately."""

    def __init__(self, context):
        self._w = context.output_writer()

    def write_result(self, uuid, article, summary, reference):
        self._w.write_result(uuid, article, summary, reference)

    def close(self):
        self._w.close()


def _hps(context):
    key = context.properties.get("sys:hyper_params_key", DEFAULT_KEY)
    return parse_hyperparam_string(context.properties.get(key, ""))


def _gpu() -> bool:
    # device_count() does not initialise the GPU: packer processes are forked after this
    return torch.cuda.device_count() > 0


def _stream_packers(context, hps) -> int:
    """Packer processes for this stream worker (0 = rows are parsed on the engine thread): GPU
    workers with an input ring and a static-shape engine (``data/stream_pack.py``)."""
    from textsummarization_on_flink_amd.data.stream_pack import default_packers
    if not _gpu() or context._in is None or context.input_coding is None:
        return 0
    if hps.mode == "train" and not hps.pad_enc_to_max:
        return 0
    if hps.mode == "decode" and (max(1, hps.decode_batch) == 1 or context._out is None):
        return 0
    return default_packers(hps)


def training_on_flink(context, hps, info: DistInfo, packer=None):
    """Stream rows -> batches -> trainer.  With ``packer`` (a ``StreamTrainPacker`` forked
    before the GPU was touched) the batches come pre-packed from its processes; the batch
    sequence is the one ``FlinkTrainBatcher`` builds."""
    from textsummarization_on_flink_amd import cli
    from textsummarization_on_flink_amd.data.batcher import FlinkTrainBatcher
    from textsummarization_on_flink_amd.train.loop import setup_training
    vocab, hps = cli.default_setup(hps, info)
    if hps.mode != "train":
        raise ValueError("The 'mode' flag must be one of train/eval/decode")
    if packer is not None:
        inner = packer
    else:
        pad = hps.max_enc_steps if (_gpu() and hps.pad_enc_to_max) else None
        inner = FlinkTrainBatcher(context.reader(), vocab, hps, pad_enc_to=pad)
    # lock-step end of stream: one host-side agreement per check window (never a per-step sync)
    synced = SyncedBatcher(inner, info, window=max(1, int(hps.check_every)))
    try:
        setup_training(hps, vocab, synced, info=info, metrics=cli.metrics_for(hps, info))
    finally:
        synced.close()
        if packer is not None:
            packer.stop()


def _serve_packed(context, hps, vocab, pool):
    """Streaming decode at engine speed: pre-packed batches from the packer processes ->
    pipelined device beam search -> best token ids back to the packer that holds the batch's
    strings (it writes the result rows; a native fanin forwards them to the output ring)."""
    from collections import deque
    import time
    from textsummarization_on_flink_amd import cli
    from textsummarization_on_flink_amd.decode.decoder import SECS_UNTIL_NEW_CKPT
    from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
    params, _, _ = cli.load_params_for_decode(hps, vocab, "cuda")
    dev = DeviceBeamDecoder(hps, vocab, params, n_articles=hps.decode_batch, T=hps.max_enc_steps,
                            use_graph=hps.graph, keep_attn=False)
    fifo = deque()
    t_load = time.time()

    def batches():
        nonlocal t_load
        while True:
            if not fifo and not hps.single_pass and time.time() - t_load > SECS_UNTIL_NEW_CKPT:
                cli.load_params_into(hps, params)  # nothing in flight: reload (decode.py:155-157)
                dev.refresh_weights()
                t_load = time.time()
            b = pool.poll(block=not fifo)
            if b is pool.NOT_READY:
                yield dev.FLUSH
                continue
            if b is None:
                return
            fifo.append(b)
            yield b

    n = 0
    for hyps in dev.decode_batches(batches()):
        b = fifo.popleft()
        pool.send_results(b, [[int(t) for t in h.tokens[1:]] for h in hyps])
        n += len(hyps)
    pool.close()
    log.info("stream decode: %d articles", n)
    return n


def inference_on_flink(context, hps, pool=None):
    from textsummarization_on_flink_amd import cli
    from textsummarization_on_flink_amd.data.batcher import FlinkInferenceBatcher
    if _gpu():
        torch.cuda.set_device(context.get_index() % torch.cuda.device_count())
    vocab, hps = cli.default_setup(hps)
    if pool is not None:
        try:
            return _serve_packed(context, hps, vocab, pool)
        except BaseException:
            pool.stop()
            raise
    writer = FlinkWriter(context)
    reader = context.reader()
    dec = cli.build_decoder(hps, vocab, lambda h, n, pad: FlinkInferenceBatcher(
        reader, vocab, h.replace(batch_size=h.beam_size), n_articles=n, pad_enc_to=pad,
        max_wait_s=hps.stream_max_wait_ms / 1000.0), writer=writer)
    dec.decode(with_rouge=False)


def _fork_packers(context, hps):
    """Fork the stream packer processes (before anything initialises the GPU)."""
    from textsummarization_on_flink_amd.data.vocab import Vocab
    n = _stream_packers(context, hps)
    if not n:
        return None
    vocab = Vocab(hps.vocab_path, hps.vocab_size)
    if hps.mode == "train":
        from textsummarization_on_flink_amd.data.stream_pack import StreamTrainPacker
        return StreamTrainPacker(context._in, context.input_coding, vocab, hps, n, hps.max_enc_steps)
    from textsummarization_on_flink_amd.data.stream_pack import StreamDecodePacker
    hd = hps.replace(batch_size=hps.beam_size)  # default_setup's decode-mode batch size
    return StreamDecodePacker(context._in, context._out, context.input_coding, context.output_coding, vocab, hd, n,
                              max(1, hps.decode_batch), hps.max_enc_steps, hps.stream_max_wait_ms / 1000.0)


def main_on_flink(context):
    hps = _hps(context)
    if context.get_role_name() == "ps":
        raise ValueError("ps role is not supported (ps_num must be 0): gradients are all-reduced across workers")
    if hps.mode not in ("train", "decode"):
        raise ValueError("The 'mode' flag must be one of train/eval/decode")
    packers = _fork_packers(context, hps)
    try:
        if hps.mode == "train":
            info = init_from_env(timeout_s=hps.dist_timeout_s)
            training_on_flink(context, hps, info, packers)
        else:
            inference_on_flink(context, hps, packers)
    finally:
        if packers is not None:
            packers.stop()


class AbstractFlinkWriter:
    """Generic result-writer template (``flink_writer.py:40-89``): subclasses name the output
    fields in ``_fields()``; ``write_result(*values)`` sends one row to the stream."""

    def __init__(self, context):
        self._w = context.output_writer()

    def _fields(self):
        raise NotImplementedError

    def write_result(self, *values):
        self._w.write(dict(zip(self._fields(), values)))

    def close(self):
        self._w.close()


def test_trainer_on_flink(context):
    """``FlinkTestTrainer`` (``train.py:12-55``): a plumbing stub that only pulls batches from
    the stream (select it with ``train_map_func="test_trainer_on_flink"``)."""
    from textsummarization_on_flink_amd import cli
    from textsummarization_on_flink_amd.data.batcher import FlinkTrainBatcher
    vocab, hps = cli.default_setup(_hps(context))
    batcher = FlinkTrainBatcher(context.reader(), vocab, hps)
    n = 0
    while True:
        b = batcher.next_batch()
        if b is None:
            break
        n += 1
        log.info("pulled batch %d: %s", n, b.uuids)
    return n
