"""Data parallelism through the production GPU engine (``GraphTrainer``: three captured
backward graphs, per-bucket async all-reduce, 1/world folded into the optimizer kernel).

Two ranks share the one GPU of the test box over ``gloo`` (RCCL refuses two ranks on one
device); after 3 steps the ranks must hold bit-identical parameters, and the DP=2 update
must equal DP=1 on the concatenated batch within bf16 tolerance.  Variants: the bf16
gradient wire format, and the ordering used when the persistent LSTM fills the GPU (the
encoder-backward graph waits for the in-flight bucket all-reduces).
Reference: worker replication ``run_summarization.py:402-426``, ``HasClusterConfig.java:20-29``.
"""
import os

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

T, D, V, STEPS = 48, 12, 600, 3
# (rows per rank, emb_dim, hidden_dim): the small model of the multi-block attention kernels, and
# the projected-context row attention with the dead-step skipping (hidden 256, emb 128, 64 rows)
SMALL, PROJ = (8, 64, 64), (64, 128, 256)


def _hps(batch, dims=SMALL):
    from textsummarization_on_flink_amd.config import HParams
    return HParams(batch_size=batch, max_enc_steps=T, max_dec_steps=D, vocab_size=V, emb_dim=dims[1],
                   hidden_dim=dims[2], coverage=True, trunc_norm_init_std=0.05)


def _examples(dims=SMALL):
    from helpers import gpu_corpus
    from textsummarization_on_flink_amd.data.batch import Example
    from textsummarization_on_flink_amd.data.vocab import abstract2sents
    c = gpu_corpus(5)
    vocab = c.vocab()
    B = dims[0]
    hps = _hps(B, dims)
    return vocab, [Example(a, [x.strip() for x in abstract2sents(s)], vocab, hps) for a, s in c.examples(2 * B * STEPS)]


def _batch(exs, rows, vocab, dims=SMALL):
    from textsummarization_on_flink_amd.data.batch import Batch
    return Batch([exs[i] for i in rows], _hps(len(rows), dims), vocab, pad_enc_to=T)


def _rank(rank, world, port, q, compress, exclusive, dims=SMALL):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from textsummarization_on_flink_amd.parallel.dist import init_from_env
        from textsummarization_on_flink_amd.train.trainer import GraphTrainer
        info = init_from_env(backend="gloo")
        vocab, exs = _examples(dims)
        B = dims[0]
        hps = _hps(B, dims).replace(grad_compress=compress)
        tr = GraphTrainer(hps, vocab.size(), B=B, T=T, device="cuda:0", info=info)
        if dims == PROJ:
            assert tr.engine.proj_attn and tr.engine.skip_pad
        tr.lstm_exclusive = exclusive
        init = tr.params.flat.clone()
        for k in range(STEPS):
            out = tr.step(_batch(exs, range(2 * B * k + B * rank, 2 * B * k + B * rank + B), vocab, dims))
        vals = tr.check_finite(out)
        q.put((rank, (tr.params.flat - init).cpu(), tr.params.flat.cpu(), vals["total_loss"]))
        torch.distributed.destroy_process_group()
    except BaseException as e:  # noqa: BLE001
        q.put((rank, repr(e), None, None))
        raise


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("compress,exclusive,tol,dims", [("none", False, 3e-2, SMALL), ("bf16", True, 5e-2, SMALL),
                                                        ("none", False, 3e-2, PROJ)])
def test_graph_trainer_dp2_matches_dp1(compress, exclusive, tol, dims):
    """PROJ: each rank sorts its own rows by live decoder steps, DP=1 sorts the concatenation."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q, compress, exclusive, dims)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, delta, flat, loss = q.get(timeout=110)
        assert flat is not None, delta
        res[r] = (delta, flat, loss)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    assert torch.equal(res[0][1], res[1][1]), "ranks diverged"
    # DP=1 on the concatenated batch (rows of both ranks), same init (same seed)
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer
    vocab, exs = _examples(dims)
    B = dims[0]
    tr = GraphTrainer(_hps(2 * B, dims), vocab.size(), B=2 * B, T=T, device="cuda:0")
    init = tr.params.flat.clone()
    for k in range(STEPS):
        tr.step(_batch(exs, range(2 * B * k, 2 * B * k + 2 * B), vocab, dims))
    tr.check_finite(tr.out)
    d1 = (tr.params.flat - init).cpu()
    d2 = res[0][0]
    rel = float((d2 - d1).norm() / d1.norm())
    assert rel < tol, rel


def test_bench_launches_its_own_ranks():
    """``python bench.py --gpus 2`` without torchrun env starts both ranks itself (before any
    GPU call in the parent) and reports the world size the process group observed."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--steps", "2", "--warmup", "1", "--batch", "16", "--enc", "64", "--dec", "8",
                        "--vocab", "2000", "--hidden", "64", "--emb", "64", "--pool", "2",
                        "--decode-batches", "2", "--decode-articles", "8", "--config5-steps", "0"],
                       capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2" and rec["config"]["backend"] == "gloo"
    assert rec["value"] > 0 and rec["beam4_summaries_per_sec"] > 0
