"""Per-request latency of streaming summarisation on the GPU (the Issue-6 concern of
``SourceSinkTest.java:41-62``: a result must leave as soon as it is ready, not one record
late).

Builds a full-size model (H=256, E=128, V=50k, enc 400, dec 100, coverage; random init,
saved as checkpoint 0), then runs ``app.start_inference`` -- the same streaming job as the
reference App: source -> select -> SummarizationModel.transform (worker process, shared-
memory rings, device beam search) -> sink -- with a timed source emitting one CNN/DM-shaped
article every ``--interval-ms``.  Latency = sink receipt time - source emit time per uuid.
With random weights STOP is rarely chosen, so most requests decode all 100 steps: the
worst case.  Prints one JSON line per micro-batch wait setting (``--stream_max_wait_ms``).

  python tools/stream_latency.py [--requests 60] [--interval-ms 50] [--waits 0,20]
"""
import argparse
import json
import os
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=60)
    ap.add_argument("--interval-ms", type=float, default=50.0)
    ap.add_argument("--waits", default="0,20")
    ap.add_argument("--decode-batch", type=int, default=64)
    a = ap.parse_args()
    from textsummarization_on_flink_amd.api import app
    from textsummarization_on_flink_amd.api.io import CallbackSink, Source
    from textsummarization_on_flink_amd.api.table import Row
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus
    from textsummarization_on_flink_amd.models.params import build_params
    from textsummarization_on_flink_amd.train import checkpoint as ckpt

    root = tempfile.mkdtemp(prefix="tsamd_lat_")
    corpus = SyntheticCorpus(seed=4)
    corpus.vocab(50000).save(os.path.join(root, "vocab"))
    hps = HParams(vocab_size=50000, coverage=True)
    train_dir = os.path.join(root, "log", "pretrained_model", "train")
    os.makedirs(train_dir, exist_ok=True)
    ckpt.Saver(train_dir).save(build_params(hps, 50000, device="cpu", seed=1), 0)
    rows = corpus.rows(a.requests + 1, "r")
    fields = ["uuid", "article", "summary", "reference"]

    class GatedSource(Source):
        """Request 0 warms the worker up (process start, weights, graph capture); the timed
        requests start only after its answer arrived, one every interval."""

        def __init__(self):
            self.warm = threading.Event()
            self.emit = {}

        def field_names(self):
            return list(fields)

        def __iter__(self):
            for i in range(a.requests + 1):
                if i == 1:
                    self.warm.wait(600)
                elif i > 1:
                    time.sleep(a.interval_ms / 1000.0)
                self.emit[rows[i]["uuid"]] = time.time()
                yield Row(rows[i]["uuid"], rows[i]["article"], "", rows[i]["reference"])

    for wait in [float(x) for x in a.waits.split(",")]:
        recv, lock = {}, threading.Lock()
        src = GatedSource()

        def on_row(row, src=src, recv=recv):
            with lock:
                recv[row[0]] = time.time()
            if row[0] == rows[0]["uuid"]:
                src.warm.set()

        extra = ["--vocab_size=50000", f"--decode_batch={a.decode_batch}", f"--stream_max_wait_ms={wait}"]
        t0 = time.time()
        app.start_inference(None, src, [CallbackSink(on_row)], root, extra, echo=False)
        wall = time.time() - t0
        lat = sorted(1e3 * (recv[r["uuid"]] - src.emit[r["uuid"]]) for r in rows[1:] if r["uuid"] in recv)
        pct = lambda xs, q: round(xs[min(len(xs) - 1, int(q * len(xs)))], 1)
        print(json.dumps({"metric": "stream_request_latency_ms", "interval_ms": a.interval_ms, "max_wait_ms": wait,
                          "decode_batch": a.decode_batch, "requests": a.requests, "answered": len(lat),
                          "p50_ms": pct(lat, 0.5), "p90_ms": pct(lat, 0.9), "p99_ms": pct(lat, 0.99),
                          "max_ms": round(lat[-1], 1), "warmup_request_ms": round(
                              1e3 * (recv[rows[0]["uuid"]] - src.emit[rows[0]["uuid"]]), 1),
                          "wall_s": round(wall, 1),
                          "config": "H=256 E=128 V=50k enc400 dec100 beam4 coverage, random-init weights"}),
              flush=True)


if __name__ == "__main__":
    main()
