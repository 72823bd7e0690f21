"""The user-facing paths on the MI355X backends: CLI train/resume (hipGraph HIP-kernel
trainer) and single-pass decode (batched device beam search), and the streaming API
(fit -> execute -> transform) with GPU worker processes."""
import glob

import pytest

from textsummarization_on_flink_amd import cli
from textsummarization_on_flink_amd.api import Row, app
from textsummarization_on_flink_amd.api.io import CollectionSource, CollectSink
from textsummarization_on_flink_amd.api.message import FIELDS
from textsummarization_on_flink_amd.train import checkpoint as ckpt

from helpers import GPU_FLAGS, gpu_corpus, make_dataset

pytestmark = pytest.mark.gpu


def _flags(tmp, d, vp, *extra, split="train"):
    return [f"--data_path={d}/{split}_*", f"--vocab_path={vp}", f"--log_root={tmp}/log", "--exp_name=exp",
            *GPU_FLAGS, *extra]


def test_cli_train_resume_decode_on_gpu(tmp_path):
    d, vp, _ = make_dataset(str(tmp_path), per_file=12, corpus=gpu_corpus())
    assert cli.main(_flags(tmp_path, d, vp, "--mode=train", "--num_steps=3", "--check_every=1")) == 0
    # default cadence: the host reads the flags / loss every check_every=10 steps and after the last
    assert cli.main(_flags(tmp_path, d, vp, "--mode=train", "--num_steps=2")) == 0
    assert ckpt.latest_checkpoint(f"{tmp_path}/log/exp/train").endswith("model.ckpt-5")
    import json
    recs = [json.loads(x) for x in open(f"{tmp_path}/log/exp/metrics_train.jsonl")]
    assert [r["step"] for r in recs] == [1, 2, 3, 5] and all(r["loss"] > 0 for r in recs)
    assert [r["steps"] for r in recs] == [1, 1, 1, 2]
    assert cli.main(_flags(tmp_path, d, vp, "--mode=decode", "--single_pass=1", split="test")) == 0
    dec = glob.glob(f"{tmp_path}/log/exp/decode_*")
    assert len(dec) == 1
    assert len(glob.glob(f"{dec[0]}/decoded/*_decoded.txt")) == 24
    assert "ROUGE-1" in open(f"{dec[0]}/ROUGE_results.txt").read()


def test_streaming_fit_then_transform_on_gpu(tmp_path):
    import os
    c = gpu_corpus(1)
    make_dataset(str(tmp_path), corpus=c)
    os.replace(f"{tmp_path}/vocab", f"{tmp_path}/vocab")
    extra = list(GPU_FLAGS)
    rows = [Row(*[r[k] for k in FIELDS]) for r in c.rows(16)]
    js = app.start_training(CollectionSource(rows), str(tmp_path), extra + ["--num_steps=2"], extra, echo=False)
    assert ckpt.latest_checkpoint(f"{tmp_path}/log/pretrained_model/train").endswith("model.ckpt-2")
    sink = CollectSink()
    q = [Row(*[r[k] for k in FIELDS]) for r in c.rows(10, "q")]
    app.start_inference(js, CollectionSource(q), [sink], str(tmp_path), extra, echo=False)
    assert sorted(r[0] for r in sink.rows) == sorted(f"q-{i}" for i in range(10))


def test_stream_fit_runs_at_engine_speed(tmp_path):
    """Throughput of the streaming fit path (rows -> worker input ring -> native fanout -> stream
    packer processes -> GraphTrainer) against the engine alone on the same batch shape: production
    width (hidden 256, emb 128, enc 400 -> dec 100, coverage), vocab 5k, batch 64, 40 steps.  The
    steady-state windows of the worker's metrics must reach 70% of the engine's tokens/s (the full
    shape: tools/stream_throughput.py, profiles/r4/)."""
    import json
    import time

    import torch

    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer

    V, B, steps = 5000, 64, 40
    c = SyntheticCorpus(vocab_size=V, seed=3)
    c.vocab(V).save(f"{tmp_path}/vocab")
    # the engine alone
    hps = HParams(batch_size=B, vocab_size=V, coverage=True)
    batches = make_batches(hps, c.vocab(V), c, 4, pad_enc_to=400)
    tr = GraphTrainer(hps, V, B=B, T=400)
    for b in batches[:2]:
        tr.step(b)
    torch.cuda.synchronize()
    t0, toks = time.time(), 0
    for i in range(20):
        tr.step(batches[i % 4])
        toks += batches[i % 4].num_tokens()
    torch.cuda.synchronize()
    engine_tps = toks / (time.time() - t0)
    del tr
    torch.cuda.empty_cache()
    # the streaming job
    rows = [Row(*[r[k] for k in FIELDS]) for r in c.rows(B * steps)]
    metrics = f"{tmp_path}/m.jsonl"
    flags = [f"--vocab_size={V}", f"--batch_size={B}", "--num_steps=0", "--check_every=10", "--tensorboard=0",
             f"--metrics_path={metrics}"]
    app.start_training(CollectionSource(rows), str(tmp_path), flags, flags, echo=False)
    win = [json.loads(x) for x in open(metrics)][1:]  # the first window holds the graph capture
    stream_tps = sum(w["tokens_per_sec"] * w["step_ms"] * w["steps"] for w in win) / sum(
        w["step_ms"] * w["steps"] for w in win)
    assert sum(w["steps"] for w in win) >= 30
    assert stream_tps >= 0.7 * engine_tps, (stream_tps, engine_tps)


def test_stream_transform_runs_at_engine_speed(tmp_path):
    """Throughput of the streaming transform path (rows -> worker input ring -> stream packer
    processes -> demand-formed decode batches -> DeviceBeamDecoder -> binary result records ->
    sink) against the decoder alone on the same shape: hidden 256, enc 400, dec 100, beam 4,
    vocab 5k, 16-article batches.  Summaries/s over the timed rows must reach 70% of the
    decoder's (the full shape: tools/stream_throughput.py, profiles/r4/stream.md)."""
    import os
    import threading
    import time

    import torch

    from textsummarization_on_flink_amd.api.io import CallbackSink, Source
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
    from textsummarization_on_flink_amd.models.params import build_params

    V, NA, warm, timed = 5000, 16, 32, 320
    c = SyntheticCorpus(vocab_size=V, seed=5)
    c.vocab(V).save(f"{tmp_path}/vocab")
    # the decoder alone
    hps = HParams(mode="decode", batch_size=NA, beam_size=4, coverage=True, vocab_size=V)
    params = build_params(hps, V, device="cuda", seed=1)
    batches = make_batches(hps, c.vocab(V), c, 1 + timed // NA, pad_enc_to=hps.max_enc_steps)
    dec = DeviceBeamDecoder(hps, c.vocab(V), params, n_articles=NA, T=hps.max_enc_steps, keep_attn=False)
    dec.decode(batches[0])
    torch.cuda.synchronize()
    t0, n = time.perf_counter(), 0
    for hyps in dec.decode_batches(batches[1:]):
        n += len(hyps)
    torch.cuda.synchronize()
    engine_sps = n / (time.perf_counter() - t0)
    del dec
    torch.cuda.empty_cache()
    # the streaming job, from a random-init checkpoint
    train_dir = os.path.join(tmp_path, "log", "pretrained_model", "train")
    os.makedirs(train_dir)
    ckpt.Saver(train_dir).save(build_params(HParams(vocab_size=V, coverage=True), V, device="cpu", seed=1), 0)
    rows = c.rows(warm + timed, "q")
    warm_ids = {r["uuid"] for r in rows[:warm]}

    class Gated(Source):
        def __init__(self):
            self.warm = threading.Event()
            self.t_start = None

        def field_names(self):
            return list(FIELDS)

        def __iter__(self):
            for i, r in enumerate(rows):
                if i == warm:
                    self.warm.wait(600)
                    self.t_start = time.time()
                yield Row(r["uuid"], r["article"], "", r["reference"])

    src, lock, got = Gated(), threading.Lock(), {"warm": 0, "timed": 0, "t_last": None}

    def on_row(row):
        with lock:
            if row[0] in warm_ids:
                got["warm"] += 1
                if got["warm"] == warm:
                    src.warm.set()
            else:
                got["timed"] += 1
                got["t_last"] = time.time()

    flags = [f"--vocab_size={V}", "--coverage=1", f"--decode_batch={NA}", "--stream_max_wait_ms=0"]
    app.start_inference(None, src, [CallbackSink(on_row)], str(tmp_path), flags, echo=False)
    assert got["timed"] == timed
    stream_sps = timed / (got["t_last"] - src.t_start)
    assert stream_sps >= 0.7 * engine_sps, (stream_sps, engine_sps)
