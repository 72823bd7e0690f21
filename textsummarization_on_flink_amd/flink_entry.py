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
from textsummarization_on_flink_amd.parallel.dist import DistInfo, all_reduce_scalar, init_from_env

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


class SyncedBatcher:
    """DP lock-step: every rank gets a batch or all stop (avoids a collective hang when
    the row stream ends unevenly across workers)."""

    def __init__(self, inner, info: DistInfo):
        self.inner, self.info = inner, info

    def next_batch(self):
        b = self.inner.next_batch()
        if self.info.enabled:
            have = all_reduce_scalar(0.0 if b is None else 1.0, self.info)
            if have < self.info.world:
                return None
        return b


def _hps(context):
    key = context.properties.get("sys:hyper_params_key", DEFAULT_KEY)
    return parse_hyperparam_string(context.properties.get(key, ""))


def training_on_flink(context, hps, info: DistInfo):
    from textsummarization_on_flink_amd import cli
    from textsummarization_on_flink_amd.data.batcher import FlinkTrainBatcher
    from textsummarization_on_flink_amd.train.loop import setup_training
    vocab, hps = cli.default_setup(hps, info)
    if hps.mode != "train":
        raise ValueError("The 'mode' flag must be one of train/eval/decode")
    pad = hps.max_enc_steps if torch.cuda.is_available() else None
    batcher = SyncedBatcher(FlinkTrainBatcher(context.reader(), vocab, hps, pad_enc_to=pad), info)
    setup_training(hps, vocab, batcher, info=info, metrics=cli.metrics_for(hps, info))


def inference_on_flink(context, hps):
    from textsummarization_on_flink_amd import cli
    from textsummarization_on_flink_amd.data.batcher import FlinkInferenceBatcher
    if torch.cuda.is_available():
        torch.cuda.set_device(context.get_index() % torch.cuda.device_count())
    vocab, hps = cli.default_setup(hps)
    writer = FlinkWriter(context)
    reader = context.reader()
    dec = cli.build_decoder(hps, vocab, lambda h, n, pad: FlinkInferenceBatcher(
        reader, vocab, h.replace(batch_size=h.beam_size), n_articles=n, pad_enc_to=pad,
        max_wait_s=hps.stream_max_wait_ms / 1000.0), writer=writer)
    dec.decode(with_rouge=False)


def main_on_flink(context):
    hps = _hps(context)
    if context.get_role_name() == "ps":
        raise ValueError("ps role is not supported (ps_num must be 0): gradients are all-reduced across workers")
    if hps.mode == "train":
        info = init_from_env(timeout_s=hps.dist_timeout_s)
        training_on_flink(context, hps, info)
    elif hps.mode == "decode":
        inference_on_flink(context, hps)
    else:
        raise ValueError("The 'mode' flag must be one of train/eval/decode")


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
