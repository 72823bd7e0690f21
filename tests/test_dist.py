"""Data parallelism on CPU (gloo, world_size 2 and 8): bucketed async all-reduce and DP=2 training
equivalent to DP=1 on the concatenated batch (SURVEY 4 "distributed tier", 7.5-6)."""
import os

import pytest
import torch
import torch.multiprocessing as mp

from helpers import tiny_corpus


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from textsummarization_on_flink_amd.parallel.dist import init_from_env
    return init_from_env(backend="gloo")


def _reducer_worker(rank, world, port, q):
    info = _init(rank, world, port)
    from textsummarization_on_flink_amd.parallel.dist import GradAllReducer
    g = torch.arange(100, dtype=torch.float32) * (rank + 1)
    red = GradAllReducer(g, info, bounds=[30, 70])
    assert [b.numel() for b in red.buckets] == [30, 40, 30]
    red.bucket_ready(0)
    red.bucket_ready(1)
    red()
    q.put((rank, g.tolist()))
    torch.distributed.destroy_process_group()


def _reducer_bf16_worker(rank, world, port, q):
    info = _init(rank, world, port)
    from textsummarization_on_flink_amd.parallel.dist import GradAllReducer
    g = torch.arange(100, dtype=torch.float32) * (rank + 1)
    red = GradAllReducer(g, info, bounds=[30, 70], compress="bf16", average=False)
    red.bucket_ready(0)
    red.wait_issued()  # bucket 0 complete; its fp32 copy-back happens in __call__
    red()
    q.put((rank, g.tolist()))
    torch.distributed.destroy_process_group()


def _train_worker(rank, world, port, q, batches_state):
    info = _init(rank, world, port)
    from textsummarization_on_flink_amd.train.cpu_trainer import CpuTrainer
    hps, vsize, batches = batches_state
    tr = CpuTrainer(hps, vsize, info=info)
    for b in batches[rank]:
        vals = tr.check_finite(tr.step(b))
    q.put((rank, tr.params.flat.clone().numpy(), vals))  # by value: the sender may exit before the read
    torch.distributed.destroy_process_group()


def _spawn(fn, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q, *args)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return dict((o[0], o[1:]) for o in out)


def test_bucketed_async_allreduce_averages():
    res = _spawn(_reducer_worker, 2)
    want = [float(i) * 1.5 for i in range(100)]
    assert res[0][0] == pytest.approx(want) and res[1][0] == pytest.approx(want)


def test_bf16_compressed_allreduce_sums():
    """bf16 wire format: the fp32 buffer receives the (bf16-rounded) SUM; averaging is left
    to the optimizer (average=False, as the GPU trainer uses it)."""
    res = _spawn(_reducer_bf16_worker, 2)
    want = [float(torch.tensor(3.0 * i).bfloat16()) for i in range(100)]
    assert res[0][0] == pytest.approx(want, rel=1e-2) and res[1][0] == res[0][0]


@pytest.mark.parametrize("world", [2, 8])
def test_dp_matches_dp1_on_concatenated_batch(world):
    """DP=world (2, and the 8-rank node layout rehearsed over gloo on the CPU) == DP=1 on the
    concatenated batch: every rank ends with the same parameters as one process stepping on
    all the rows (gradient sum over ranks, 1/world average, clip and Adagrad after it)."""
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.batch import Batch, Example
    from textsummarization_on_flink_amd.data.vocab import abstract2sents
    from textsummarization_on_flink_amd.train.cpu_trainer import CpuTrainer
    c = tiny_corpus(3)
    vocab = c.vocab()
    n = 16  # rows per step over all ranks
    bs = n // world
    hps = HParams(hidden_dim=16, emb_dim=8, vocab_size=200, max_enc_steps=30, max_dec_steps=8, batch_size=bs,
                  coverage=True)
    exs = [Example(a, [x.strip() for x in abstract2sents(s)], vocab, hps) for a, s in c.examples(2 * n)]
    # two steps; each step: rank r gets rows [n k + bs r, n k + bs (r + 1)); DP1 gets all n rows (same padding)
    per_rank = {r: [Batch(exs[n * k + bs * r: n * k + bs * (r + 1)], hps, vocab, pad_enc_to=30) for k in range(2)]
                for r in range(world)}
    res = _spawn(_train_worker, world, (hps, vocab.size(), per_rank))
    hpsn = hps.replace(batch_size=n)
    tr = CpuTrainer(hpsn, vocab.size())
    for k in range(2):
        tr.step(Batch(exs[n * k: n * (k + 1)], hpsn, vocab, pad_enc_to=30))
    for r in range(1, world):
        assert (res[0][0] == res[r][0]).all()  # ranks stay identical
    assert torch.allclose(torch.from_numpy(res[0][0]), tr.params.flat, atol=1e-5, rtol=1e-4)


def _cli_rank(rank, world, port, q, flags):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    from textsummarization_on_flink_amd import cli
    try:
        cli.main(flags)
        q.put((rank, "ok"))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, f"err:{type(e).__name__}"))
        raise


def test_dead_rank_surfaces_and_training_restarts_from_latest(tmp_path):
    """Fault injection: rank 1 dies at step 1 -> rank 0 errors out within the collective
    timeout (no hang) after checkpointing; a relaunch resumes from that checkpoint."""
    from helpers import TINY_FLAGS, make_dataset
    d, vp, _ = make_dataset(str(tmp_path))
    flags = [f"--data_path={d}/train_*", f"--vocab_path={vp}", f"--log_root={tmp_path}/log", "--exp_name=exp",
             *TINY_FLAGS, "--mode=train", "--num_steps=4", "--fault_kill_step=1", "--fault_kill_rank=1",
             "--dist_timeout_s=20"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cli_rank, args=(r, 2, port, q, flags)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert procs[1].exitcode == 17          # the injected hard exit
    assert procs[0].exitcode not in (0, None)  # surfaced as an error, not a hang
    from textsummarization_on_flink_amd.train import checkpoint as ckpt
    latest = ckpt.latest_checkpoint(f"{tmp_path}/log/exp/train")
    assert latest is not None and latest.endswith("model.ckpt-1")
    # restart from latest on a fresh single-process launch
    from textsummarization_on_flink_amd import cli
    import unittest.mock as um
    with um.patch("torch.cuda.is_available", lambda: False):
        assert cli.main([f for f in flags if not f.startswith("--fault_kill")] + ["--num_steps=2"]) == 0
    assert ckpt.latest_checkpoint(f"{tmp_path}/log/exp/train").endswith("model.ckpt-3")


def _cli_rank_report(rank, world, port, q, flags):
    """One CLI training rank that reports its parameter checksum and global step at the end."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    from textsummarization_on_flink_amd.train import loop
    seen = {}
    orig = loop.run_training

    def spy(trainer, *a, **k):
        seen["start"] = trainer.global_step
        out = orig(trainer, *a, **k)
        seen["end"] = trainer.global_step
        seen["sum"] = float(trainer.params.flat.double().sum())
        return out
    loop.run_training = spy
    from textsummarization_on_flink_amd import cli
    cli.main(flags)
    q.put((rank, seen))


def test_dp_checkpoint_saved_on_rank0_resumes_on_all_ranks(tmp_path):
    """SURVEY 4 distributed tier: a 2-rank job checkpoints on rank 0 only; a relaunched 2-rank job
    resumes every rank from that checkpoint (same start step, identical parameters after the
    resumed steps)."""
    from helpers import TINY_FLAGS, make_dataset
    from textsummarization_on_flink_amd.train import checkpoint as ckpt
    d, vp, _ = make_dataset(str(tmp_path))
    flags = [f"--data_path={d}/train_*", f"--vocab_path={vp}", f"--log_root={tmp_path}/log", "--exp_name=exp",
             *TINY_FLAGS, "--mode=train", "--num_steps=2"]
    first = _spawn(_cli_rank_report, 2, flags)
    assert first[0][0]["start"] == first[1][0]["start"] == 0
    assert ckpt.latest_checkpoint(f"{tmp_path}/log/exp/train").endswith("model.ckpt-2")
    second = _spawn(_cli_rank_report, 2, flags)
    assert second[0][0]["start"] == second[1][0]["start"] == 2  # both ranks resumed from rank 0's checkpoint
    assert second[0][0]["end"] == second[1][0]["end"] == 4
    assert second[0][0]["sum"] == second[1][0]["sum"]  # the ranks stay identical
    assert ckpt.latest_checkpoint(f"{tmp_path}/log/exp/train").endswith("model.ckpt-4")


def _poison_worker(rank, world, port, q):
    """Rank 1 alone sees a persistent-LSTM error word: after poison_where on its last bucket and
    the bucketed all-reduce, EVERY rank holds a non-finite gradient (so every rank's optimizer
    kernel skips the step and every rank raises at the same check)."""
    info = _init(rank, world, port)
    from textsummarization_on_flink_amd.parallel.dist import GradAllReducer, poison_where
    g = torch.ones(100)
    err = torch.tensor([1 if rank == 1 else 0], dtype=torch.int32)
    red = GradAllReducer(g, info, bounds=[30, 70], average=False)
    red.bucket_ready(0)
    red.bucket_ready(1)
    poison_where(err, g[-1:])
    red()
    healthy = torch.ones(10)
    poison_where(torch.zeros(1, dtype=torch.int32), healthy[-1:])
    q.put((rank, bool(torch.isfinite(g).all()), float(g[0]), bool(torch.isfinite(healthy).all())))
    torch.distributed.destroy_process_group()


def test_lstm_error_on_one_rank_skips_the_step_on_all_ranks():
    res = _spawn(_poison_worker, 2)
    for r in (0, 1):
        finite, g0, healthy_finite = res[r]
        assert not finite and g0 == 2.0 and healthy_finite


@pytest.mark.parametrize("defer,dw_side", [(True, False), (False, False), (True, True), (False, True)])
def test_bucket_issue_order_leaves_only_the_embedding(defer, dw_side):
    """GraphTrainer's replay order (train/trainer.py replay_phases / issue_plan) with a recording
    reducer over the real flat-gradient layout of the bench model: every bucket except the
    embedding's is issued before the last phase graph is queued, so at most the 25.6 MB embedding
    gradient is all-reduced with nothing left to overlap; with the decoder weight gradients
    deferred beside the encoder BPTT their bucket goes out right after that phase; with the vocab dW
    beside the decoder loop (dw_side) phase 1 issues bucket 0 itself (GraphTrainer._Phase1)."""
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.models.params import FlatParams, param_specs
    from textsummarization_on_flink_amd.models.pointer_generator import HipPointerGenerator
    from textsummarization_on_flink_amd.parallel.dist import DistInfo, GradAllReducer
    from textsummarization_on_flink_amd.train.trainer import BPTT_PHASE, issue_plan, replay_phases

    hps = HParams(coverage=True)
    specs = param_specs(hps, 50000)
    offs, o = {}, 0
    for sp in specs:
        n = 1
        for d in sp.shape:
            n *= d
        offs[sp.name] = o
        o += n
    bounds = [offs[nm] for nm in HipPointerGenerator.PHASE_FIRST_PARAM]
    red = GradAllReducer(torch.zeros(o), DistInfo(0, 2, 0, "gloo"), bounds=bounds, average=False)
    assert len(red.buckets) == 4
    events = []

    class G:
        def __init__(self, i):
            self.i = i

        def replay(self):
            events.append(("graph", self.i))
            if dw_side and self.i == 1:
                events.append(("bucket", 0))  # _Phase1: from the side stream, before the decoder graph ends

    class Rec:
        def bucket_ready(self, b):
            events.append(("bucket", b))

        def wait_issued(self):
            events.append(("wait",))

    replay_phases([G(i) for i in range(4)], Rec(), issue_plan(defer, dw_side), BPTT_PHASE, lstm_exclusive=True)
    issued_before_last = {e[1] for e in events[:events.index(("graph", 3))] if e[0] == "bucket"}
    assert issued_before_last == {0, 1, 2}
    assert [e for e in events if e[0] == "bucket"].count(("bucket", 0)) == 1
    assert events.index(("bucket", 0)) == events.index(("graph", 1 if dw_side else 0)) + 1
    assert events.index(("wait",)) == events.index(("graph", BPTT_PHASE)) - 1  # no RCCL beside the full-grid BPTT
    if defer:
        assert events.index(("bucket", 1)) == events.index(("graph", 2)) + 1
    else:
        assert events.index(("bucket", 1)) == events.index(("graph", 1)) + 1 + dw_side
    left = sum(red.buckets[b].numel() * 4 for b in range(4) if b not in issued_before_last)
    assert left == 50000 * 128 * 4 <= 26 * 2 ** 20  # the embedding only


class _ListBatcher:
    def __init__(self, n):
        self.items = list(range(n))

    def next_batch(self):
        return self.items.pop(0) if self.items else None


def _synced_worker(rank, world, port, q, lengths, window):
    info = _init(rank, world, port)
    from textsummarization_on_flink_amd.parallel.dist import SyncedBatcher
    sb = SyncedBatcher(_ListBatcher(lengths[rank]), info, window=window)
    got = []
    while True:
        b = sb.next_batch()
        if b is None:
            break
        got.append(b)
    sb.close()
    q.put((rank, got, sb.collectives))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("lengths,window", [((23, 17), 5), ((10, 10), 5), ((3, 40), 4), ((0, 7), 3)])
def test_synced_batcher_stops_every_rank_at_the_same_step(lengths, window):
    """Stream-fed DP (flink_entry.training_on_flink): streams that end unevenly across ranks stop
    every rank after the same number of batches (the shortest stream's), with ONE blocking host
    collective per window of batches -- not one per batch (no per-step host sync)."""
    res = _spawn(_synced_worker, 2, lengths, window)
    n = min(lengths)
    for r in range(2):
        got, coll = res[r]
        assert got == list(range(n)), (r, got)
        assert coll <= n // window + 1, (r, coll)


def _synced_nccl_layout_worker(rank, world, port, q, lengths, window):
    """The production GPU layout: the default group is the gradient backend (RCCL there; gloo
    stands in for it here) and the window agreement runs on the dedicated gloo group cpu_group()
    creates when the default backend is "nccl" -- with a gradient-sized collective on the default
    group after every batch, interleaved with the agreement collectives."""
    import dataclasses
    info = _init(rank, world, port)
    from textsummarization_on_flink_amd.parallel import dist as D
    nccl_info = dataclasses.replace(info, backend="nccl")
    grp = D.cpu_group(nccl_info)
    assert grp is not None and grp is not torch.distributed.group.WORLD
    sb = D.SyncedBatcher(_ListBatcher(lengths[rank]), nccl_info, window=window)
    assert sb._group is grp
    got, grads = [], []
    while True:
        b = sb.next_batch()
        if b is None:
            break
        got.append(b)
        g = torch.full((4096,), float(rank + 1))
        torch.distributed.all_reduce(g)  # the step's gradient all-reduce on the default group
        grads.append(float(g[0]))
    sb.close()
    after = torch.ones(1)
    torch.distributed.all_reduce(after)  # every rank reaches the next collective after the stop
    q.put((rank, got, sb.collectives, grads, float(after[0])))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("lengths,window", [((23, 17), 5), ((3, 40), 4)])
def test_synced_batcher_on_dedicated_gloo_group_beside_gradient_collectives(lengths, window):
    """SyncedBatcher under the NCCL default backend agrees on a dedicated gloo subgroup
    (dist.new_group(backend="gloo")): every rank stops after the shortest stream's batch count,
    each step's default-group all-reduce pairs up across ranks (sum = 1 + 2), and every rank
    reaches a later collective."""
    res = _spawn(_synced_nccl_layout_worker, 2, lengths, window)
    n = min(lengths)
    for r in range(2):
        got, coll, grads, after = res[r]
        assert got == list(range(n)), (r, got)
        assert coll <= n // window + 1
        assert grads == [3.0] * n and after == 2.0


class _BlockingBatcher:
    """A stream that blocks in next_batch until stopped (a training run ended before its stream)."""
    def __init__(self):
        import threading
        self.n = 0
        self.stopped = threading.Event()

    def next_batch(self):
        if self.n < 3:
            self.n += 1
            return self.n
        self.stopped.wait(30)
        return None

    def interrupt(self):
        self.stopped.set()


def test_synced_batcher_close_stops_a_blocked_source_promptly():
    """close() before the stream ends must interrupt the inner source before joining
    the prefetch thread, not wait out the join timeout with the thread blocked in
    next_batch() (flink_entry then releases the rings under it)."""
    import time
    from textsummarization_on_flink_amd.parallel.dist import DistInfo, SyncedBatcher
    inner = _BlockingBatcher()
    sb = SyncedBatcher(inner, DistInfo(rank=0, world=2, backend="gloo"), window=2, group=object())
    time.sleep(0.3)  # the prefetch thread took the 3 batches and blocks in next_batch
    t0 = time.monotonic()
    sb.close()
    assert time.monotonic() - t0 < 1.0 and inner.stopped.is_set()
    assert not sb._thread.is_alive()


def _agree_worker(rank, world, port, q, fits_on_rank1):
    info = _init(rank, world, port)
    import sys as _sys
    _sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from textsummarization_on_flink_amd.parallel import dist as D

    def trial(c):
        if rank == 1 and c > fits_on_rank1:  # an OOM on one rank only
            raise torch.cuda.OutOfMemoryError(f"HIP out of memory (injected, batch {c})")
        return f"trainer-{c}"

    got = bench.agree_largest((2048, 1024, 512), trial, info, D, "cpu")
    # a collective after the search: every rank must reach it (no rank left behind in a trial)
    total = D.all_reduce_scalar(1.0, info, op="sum", device="cpu")
    q.put((rank, got, total))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("fits_on_rank1,want", [(1024, 1024), (2048, 2048), (0, None)])
def test_capacity_search_agrees_when_one_rank_runs_out_of_memory(fits_on_rank1, want):
    """bench.py's config #5 batch sizing: an OOM injected on rank 1 only makes EVERY rank step down
    to the same batch (or all skip when nothing fits), then both reach the next collective: no
    rank-local skip that would leave its peer blocked in an all-reduce."""
    res = _spawn(_agree_worker, 2, fits_on_rank1)
    for r in range(2):
        (c, trial_result), total = res[r]
        assert c == want and total == 2.0
        assert trial_result == (None if want is None else f"trainer-{want}")
