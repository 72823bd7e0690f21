"""Throughput of the streaming (Flink-API) paths on one GPU -- the reference's primary
execution path: ``App.startTraining`` / ``startInference`` -> ``TFEstimator.fit`` /
``TFModel.transform`` (``App.java:83-132``, ``run_summarization.py:370-399``).

  fit:        CollectionSource(N synthetic CNN/DM-shaped rows) -> select -> SummarizationEstimator.fit
              -> env.execute(): the worker process receives coded rows on its input ring; the
              stream packer processes (data/stream_pack.py) turn them into engine batches for
              GraphTrainer (B = 256, H = 256, E = 128, enc 400 -> dec 100, V = 50k, coverage).
              Reported: train tokens/s from the worker's metrics windows (``check_every`` steps
              each, the first ``--skip-windows`` dropped: warm-up and graph capture), the same
              token definition as bench.py.
  transform:  a random-init checkpoint; ``--warm`` rows answered first (worker start, graph
              capture), then N rows emitted as fast as the driver can; reported: result rows/s
              from the first timed row's emission to the last result's arrival at the sink
              (64 articles x beam 4 per device batch).

  python tools/stream_throughput.py [--fit-rows 20480] [--transform-rows 10240] [--out F.jsonl]
"""
import argparse
import json
import os
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FIELDS = ["uuid", "article", "summary", "reference"]
MODEL = ["--vocab_size=50000", "--hidden_dim=256", "--emb_dim=128", "--max_enc_steps=400", "--max_dec_steps=100",
         "--coverage=1"]


def _rows(corpus, n, prefix):
    t = time.time()
    rows = corpus.rows(n, prefix)
    print(f"# {n} rows generated in {time.time() - t:.1f} s", file=sys.stderr, flush=True)
    return rows


def run_fit(a, root, corpus):
    from textsummarization_on_flink_amd.api import app
    from textsummarization_on_flink_amd.api.io import CollectionSource
    rows = _rows(corpus, a.fit_rows, "t")
    metrics = os.path.join(root, "fit_metrics.jsonl")
    extra = MODEL + [f"--batch_size={a.batch}", "--num_steps=0", "--save_model_secs=0", "--check_every=10",
                     f"--metrics_path={metrics}", "--tensorboard=0", f"--stream_packers={a.packers}"]
    src = CollectionSource([tuple(r[f] for f in FIELDS) for r in rows])
    t0 = time.time()
    app.start_training(src, root, extra, echo=False)
    wall = time.time() - t0
    win = [json.loads(x) for x in open(metrics)]
    win = [w for w in win if "tokens_per_sec" in w]
    steady = win[a.skip_windows:] or win
    toks = sum(w["tokens_per_sec"] * w["step_ms"] * w["steps"] / 1e3 for w in steady)
    secs = sum(w["step_ms"] * w["steps"] / 1e3 for w in steady)
    rec = {"metric": "stream_fit_train_tokens_per_sec", "value": round(toks / secs, 1), "unit": "tokens/s",
           "rows": a.fit_rows, "batch": a.batch, "steps": sum(w["steps"] for w in win),
           "steady_steps": sum(w["steps"] for w in steady),
           "ms_per_step_steady": round(1e3 * secs / sum(w["steps"] for w in steady), 3),
           "windows_tokens_per_sec": [round(w["tokens_per_sec"]) for w in win], "wall_s": round(wall, 1),
           "packers": a.packers, "config": "H=256 E=128 V=50k enc400 dec100 coverage, synthetic rows, random init"}
    print(json.dumps(rec), flush=True)
    return rec


def engine_decode(root, corpus, na, n_batches=12):
    """The decoder alone (bench_decode.py's loop) with the checkpoint the streaming job served --
    a random-init one, or the one the fit just trained, whose decode differs -- on synthetic
    batches of the same shape: the fair denominator for the streaming transform."""
    import torch
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import make_batches
    from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
    from textsummarization_on_flink_amd.models.params import build_params
    from textsummarization_on_flink_amd.train import checkpoint as ckpt
    hps = HParams(mode="decode", batch_size=na, beam_size=4, coverage=True, vocab_size=50000)
    params = build_params(hps, 50000, device="cuda")
    ckpt.restore(ckpt.latest_checkpoint(os.path.join(root, "log", "pretrained_model", "train")), params,
                 load_adagrad=False, strict=False)
    vocab = corpus.vocab(50000)
    batches = make_batches(hps, vocab, corpus, n_batches + 1, pad_enc_to=hps.max_enc_steps)
    dec = DeviceBeamDecoder(hps, vocab, params, n_articles=na, T=hps.max_enc_steps, keep_attn=False)
    dec.decode(batches[0])
    torch.cuda.synchronize()
    t0, n, steps = time.perf_counter(), 0, 0
    for hyps in dec.decode_batches(batches[1:]):
        n += len(hyps)
        steps += dec.finished_steps
    torch.cuda.synchronize()
    sps = round(n / (time.perf_counter() - t0), 1)
    del dec, params
    torch.cuda.empty_cache()
    return sps, round(steps / n_batches, 1)


def run_transform(a, root, corpus):
    from textsummarization_on_flink_amd.api import app
    from textsummarization_on_flink_amd.api.io import CallbackSink, Source
    from textsummarization_on_flink_amd.api.table import Row
    rows = _rows(corpus, a.warm + a.transform_rows, "q")
    warm_ids = {r["uuid"] for r in rows[:a.warm]}

    class GatedSource(Source):
        def __init__(self):
            self.warm = threading.Event()
            self.t_start = None

        def field_names(self):
            return list(FIELDS)

        def __iter__(self):
            for i, r in enumerate(rows):
                if i == a.warm:
                    self.warm.wait(900)
                    self.t_start = time.time()
                yield Row(r["uuid"], r["article"], "", r["reference"])

    src = GatedSource()
    lock = threading.Lock()
    got = {"warm": 0, "timed": 0, "t_last": None}

    def on_row(row):
        with lock:
            if row[0] in warm_ids:
                got["warm"] += 1
                if got["warm"] == a.warm:
                    src.warm.set()
            else:
                got["timed"] += 1
                got["t_last"] = time.time()

    extra = MODEL + [f"--decode_batch={a.decode_batch}", f"--stream_max_wait_ms={a.max_wait_ms}",
                     f"--stream_packers={a.packers}"]
    t0 = time.time()
    app.start_inference(None, src, [CallbackSink(on_row)], root, extra, echo=False)
    wall = time.time() - t0
    el = got["t_last"] - src.t_start
    eng_sps, eng_steps = engine_decode(root, corpus, a.decode_batch)
    rec = {"metric": "stream_transform_summaries_per_sec", "value": round(got["timed"] / el, 1),
           "engine_same_ckpt_summaries_per_sec": eng_sps, "engine_decode_steps_per_batch": eng_steps,
           "ratio_vs_engine": round(got["timed"] / el / eng_sps, 3),
           "unit": "summaries/s", "rows": a.transform_rows, "answered": got["timed"], "timed_s": round(el, 2),
           "decode_batch": a.decode_batch, "beam": 4, "wall_s": round(wall, 1), "packers": a.packers,
           "config": "H=256 E=128 V=50k enc400 dec100 beam4 coverage, synthetic rows, random init"}
    print(json.dumps(rec), flush=True)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fit-rows", type=int, default=20480)
    ap.add_argument("--transform-rows", type=int, default=10240)
    ap.add_argument("--warm", type=int, default=128)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--decode-batch", type=int, default=64)
    ap.add_argument("--max-wait-ms", type=float, default=0.0)
    ap.add_argument("--packers", type=int, default=-1)
    ap.add_argument("--skip-windows", type=int, default=1)
    ap.add_argument("--only", choices=("fit", "transform"), default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus
    from textsummarization_on_flink_amd.models.params import build_params
    from textsummarization_on_flink_amd.train import checkpoint as ckpt
    root = tempfile.mkdtemp(prefix="tsamd_thr_")
    corpus = SyntheticCorpus(seed=11)
    corpus.vocab(50000).save(os.path.join(root, "vocab"))
    recs = []
    if a.only in (None, "fit"):
        recs.append(run_fit(a, root, corpus))
    if a.only in (None, "transform"):
        train_dir = os.path.join(root, "log", "pretrained_model", "train")
        if not os.path.exists(os.path.join(train_dir, "checkpoint")):
            os.makedirs(train_dir, exist_ok=True)
            ckpt.Saver(train_dir).save(build_params(HParams(vocab_size=50000, coverage=True), 50000, device="cpu",
                                                    seed=1), 0)
        recs.append(run_transform(a, root, corpus))
    if a.out:
        with open(a.out, "a") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
