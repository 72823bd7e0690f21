"""End-to-end training throughput of the real CLI path (``cli --mode=train``: .bin files ->
batcher -> GraphTrainer -> checkpoints), for comparison with ``bench.py`` (which feeds
pre-built batches).

  python tools/cli_throughput.py [--examples 20000] [--steps 60] [--batch 256] [--workers 8]
                                 [--threaded] [--host-only]

Writes a synthetic CNN/DM-shaped dataset (1000-example .bin chunks, 50k vocab) under --root,
runs the CLI in a child process and prints one JSON line: steady-state tokens/s and ms per
step from the metrics JSONL (windows of ``--check_every`` steps, the first windows -- graph
capture, loader warm-up -- dropped).  ``--host-only`` times the batcher alone (batches/s the
host pipeline sustains without the GPU).  ``--threaded`` uses the threaded Batcher instead of
the worker processes.
"""
import argparse
import glob
import json
import multiprocessing as mp
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _write_chunk(args):
    path, n, seed = args
    from textsummarization_on_flink_amd.data import binfmt
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus
    c = SyntheticCorpus(seed=seed)
    binfmt.write_bin(path, [{"article": a, "abstract": s} for a, s in c.examples(n)])
    return path


def make_data(root, n, procs=8):
    d = os.path.join(root, "data")
    os.makedirs(d, exist_ok=True)
    chunks = [(os.path.join(d, f"train_{i:04d}.bin"), 1000, 100 + i) for i in range((n + 999) // 1000)]
    todo = [c for c in chunks if not os.path.exists(c[0])]
    if todo:
        with mp.get_context("fork").Pool(procs) as pool:
            pool.map(_write_chunk, todo)
    vp = os.path.join(root, "vocab")
    if not os.path.exists(vp):
        from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus
        SyntheticCorpus(seed=0).vocab(50000).save(vp)
    return os.path.join(d, "train_*.bin"), vp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default="/tmp/tsamd_cli")
    ap.add_argument("--examples", type=int, default=20000)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--check-every", type=int, default=10)
    ap.add_argument("--threaded", action="store_true")
    ap.add_argument("--host-only", action="store_true")
    a = ap.parse_args()
    t0 = time.time()
    pattern, vp = make_data(a.root, a.examples)
    gen_s = time.time() - t0
    flags = [f"--data_path={pattern}", f"--vocab_path={vp}", f"--batch_size={a.batch}", "--max_enc_steps=400",
             "--max_dec_steps=100", "--coverage=1", "--vocab_size=50000"]
    if a.host_only:
        from textsummarization_on_flink_amd.config import parse_flags
        from textsummarization_on_flink_amd.data.vocab import Vocab
        hps = parse_flags(["--mode=train", *flags], known_only=True)
        vocab = Vocab(vp, 50000)
        if a.threaded:
            from textsummarization_on_flink_amd.data.batcher import Batcher
            b = Batcher(pattern, vocab, hps, single_pass=False, seed=1, pad_enc_to=400)
        else:
            from textsummarization_on_flink_amd.data.loader import ProcessBatcher
            b = ProcessBatcher(pattern, vocab, hps, single_pass=False, workers=a.workers, seed=1, pad_enc_to=400)
        t1 = time.time()  # from construction: includes the bucket fills (100 batches per bucket)
        for _ in range(a.steps):
            b.next_batch()
        dt = time.time() - t1
        b.stop()
        print(json.dumps({"mode": "host_only", "loader": "threaded" if a.threaded else f"processes x{a.workers}",
                          "batch": a.batch, "batches_per_s": round(a.steps / dt, 2),
                          "examples_per_s": round(a.steps * a.batch / dt, 1)}), flush=True)
        return 0
    log_root = os.path.join(a.root, "log")
    exp = f"run_{int(time.time())}"
    cmd = [sys.executable, "-m", "textsummarization_on_flink_amd.cli", "--mode=train", *flags,
           f"--log_root={log_root}", f"--exp_name={exp}", f"--num_steps={a.steps}",
           f"--check_every={a.check_every}", "--save_model_secs=0", "--tensorboard=0",
           f"--loader_workers={0 if a.threaded else a.workers}"]
    t1 = time.time()
    rc = subprocess.call(cmd, cwd=REPO)
    wall = time.time() - t1
    if rc != 0:
        print(json.dumps({"error": f"cli exited {rc}"}))
        return rc
    recs = [json.loads(x) for x in open(glob.glob(os.path.join(log_root, exp, "metrics_train.jsonl"))[0])]
    recs = [r for r in recs if "tokens_per_sec" in r]
    steady = recs[2:] if len(recs) > 3 else recs[-1:]
    tps = sorted(r["tokens_per_sec"] for r in steady)
    ms = sorted(r["step_ms"] for r in steady)
    print(json.dumps({"mode": "cli_train", "loader": "threaded" if a.threaded else f"processes x{a.workers}",
                      "batch": a.batch, "steps": a.steps, "windows": len(steady),
                      "tokens_per_sec_median": round(tps[len(tps) // 2], 1),
                      "ms_per_step_median": round(ms[len(ms) // 2], 3), "wall_s": round(wall, 1),
                      "datagen_s": round(gen_s, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
