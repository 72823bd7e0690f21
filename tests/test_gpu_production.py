"""Numerics at the production (bench) shape, not toy shapes: B=256 articles, T=400 encoder
steps (CNN/DM-shaped lengths, most articles truncated), D=100 decoder steps, V=50k --
the persistent LSTM at grid 128, the XCD-ordered attention kernels, 196 vocab tiles.

* one forward + backward of the HIP engine vs the fp32 oracle (``models.reference``)
  run on the same GPU: loss, coverage loss, attention distributions, p_gen and every
  parameter gradient;
* the hipGraph-captured train step (GraphTrainer replay) vs the same step run eagerly;
* a 50-step loss curve of the HIP trainer vs the fp32 oracle trainer on the same
  batches (B=32, T=400, V=50k): the bf16 path must track the fp32 one step by step.
Reference semantics: ``model.py:199-285``, ``attention_decoder.py:79-180``.
"""
import json
import math
import os

import numpy as np
import pytest
import torch

from textsummarization_on_flink_amd.config import HParams
from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
from textsummarization_on_flink_amd.models.params import build_params
from textsummarization_on_flink_amd.models.reference import ReferencePointerGenerator, batch_to_tensors
from helpers import grad_mismatches, grad_rel

pytestmark = pytest.mark.gpu

T, D, V = 400, 100, 50000


def _rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


def _hps(B, **kw):
    return HParams(batch_size=B, max_enc_steps=T, max_dec_steps=D, vocab_size=V, coverage=True, pointer_gen=True,
                   **kw)


def _batches(hps, n, seed):
    corpus = SyntheticCorpus(vocab_size=V, seed=seed)
    vocab = corpus.vocab(V)
    return vocab, make_batches(hps, vocab, corpus, n, pad_enc_to=T)


def _oracle_check(hps, B, T_, D_, seed, cov_tol=2e-2):
    """One forward + backward of the HIP engine vs the fp32 oracle (autograd) on the same GPU:
    loss, coverage loss, attention distributions, p_gen and every parameter gradient."""
    from textsummarization_on_flink_amd.models.pointer_generator import HipPointerGenerator
    corpus = SyntheticCorpus(vocab_size=hps.vocab_size, seed=seed)
    vocab = corpus.vocab(hps.vocab_size)
    (batch,) = make_batches(hps, vocab, corpus, 1, pad_enc_to=T_)
    params = build_params(hps, vocab.size(), device="cuda", seed=3)
    params.enable_grad()
    eng = HipPointerGenerator(hps, vocab.size(), params, B=B, T=T_, D=D_)
    eng.set_batch(batch)
    out = eng.forward(need_grad=True)
    eng.backward()
    torch.cuda.synchronize()
    eng.check_lstm_err()
    got = {k: v.detach().clone() for k, v in out.items()}
    g_hip = params.grad.clone()
    att, pg = eng.w["ATT"].clone(), eng.w["pg"].clone()
    # steps past a row's last loss-weighted decoder step are not computed (skip_pad_steps): compare
    # the attention and p_gen of live steps only
    live = torch.arange(D_, device="cuda")[:, None] < eng.w["dlen"].long()[None, :]  # [D, B]
    src = eng.w["row_src"].long().clone()  # engine row b is batch row src[b] (rows sorted by live steps)
    kinds = {"persistent_lstm": eng.persistent_lstm, "fused_vocab": eng.fused_vocab, "row_attn": eng.row_attn,
             "row_attn_bwd": eng.row_attn_bwd, "split": eng.split, "proj_attn": eng.proj_attn}
    del eng
    torch.cuda.empty_cache()
    flat = params.flat.detach().clone().requires_grad_(True)
    W = {n: flat[o:o + c].view(params.view(n).shape) for n, (o, c) in params.offsets.items()}
    ref = ReferencePointerGenerator(hps, vocab.size()).forward(W, batch_to_tensors(batch, "cuda"))
    ref["total_loss"].backward()
    g_ref = flat.grad
    assert abs(float(got["loss"]) - float(ref["loss"])) < 1e-2 * abs(float(ref["loss"]))
    assert abs(float(got["coverage_loss"]) - float(ref["coverage_loss"])) < cov_tol * abs(float(ref["coverage_loss"]))
    assert _rel(att[live], ref["attn_dists"].detach()[:, src][live]) < 2e-2
    assert _rel(pg[live], ref["p_gens"].detach()[:, src][live]) < 2e-2
    bad = grad_mismatches(params, g_hip, g_ref)
    assert not bad, bad
    kinds["grad_rel"] = grad_rel(params, g_hip, g_ref)
    return kinds


def test_bench_shape_with_every_weight_gradient_on_wgrad_tt(monkeypatch):
    """The bench shape against the fp32 oracle with every eligible long-K weight gradient on the
    deterministic split-K wgrad_tt (threshold 0; deterministic mode runs the decoder-side ones
    inline, where they take it too): encoder x^T.dz / h^T.dz (K = T.B = 102400, layer 0's M = 128
    with the operand roles swapped), decoder cell / output-projection / attention / W_h (K = D.B)."""
    from textsummarization_on_flink_amd.models import pointer_generator as pgm
    monkeypatch.setattr(pgm, "WGRAD_TT_MIN", 0)
    monkeypatch.setenv("TSAMD_DETERMINISTIC", "1")
    _oracle_check(_hps(256, trunc_norm_init_std=0.05), 256, T, D, seed=13)


def test_bench_shape_with_vocab_dw_on_the_split_bmm_and_unpadded(monkeypatch):
    """The vocab weight gradient's other paths against the fp32 oracle: the 4-way split-K batched
    GEMM over the padded dlogits rows (config #5's path, threshold 0 here), and the unpadded
    layout (TSAMD_VOCAB_PAD=0: the round-5 GEMMs at V = 50k)."""
    from textsummarization_on_flink_amd.models import pointer_generator as pgm
    monkeypatch.setattr(pgm, "VOCAB_DW_SPLIT_MIN", 0)
    _oracle_check(_hps(256, trunc_norm_init_std=0.05), 256, T, D, seed=17)
    monkeypatch.setattr(pgm, "VOCAB_PAD", False)
    monkeypatch.setattr(pgm, "DE_BF16", False)
    monkeypatch.setattr(pgm, "CTX_NATIVE", False)
    _oracle_check(_hps(256, trunc_norm_init_std=0.05), 256, T, D, seed=19)


def test_bench_shape_matches_fp32_oracle():
    kinds = _oracle_check(_hps(256, trunc_norm_init_std=0.05), 256, T, D, seed=11)
    assert kinds["persistent_lstm"] and kinds["fused_vocab"] and kinds["row_attn_bwd"] and kinds["proj_attn"]
    # the small parameters whose gradients are near zero at a larger init (coverage w_c, the p_gen
    # bias, the reduce-state biases: attention_decoder.py:72-73, 164-168; model.py:111-114) are
    # each checked on their own at this init, at the same relative bound as the large ones
    rel = kinds["grad_rel"]
    small = [n for n in rel if n.endswith(("coverage/w_c", "calculate_pgen/Linear/Bias", "bias_reduce_c",
                                           "bias_reduce_h"))]
    assert len(small) == 4, small
    assert all(rel[n] < 5e-2 for n in small), {n: rel[n] for n in small}


@pytest.mark.parametrize("B", [8, 128, 512, 1024])
def test_config5_shape_matches_fp32_oracle(B):
    """Config #5's model (hidden 512, 2-layer bi-LSTM encoder, enc 800, V = 50k, coverage) against
    the fp32 oracle, D = 20 decoder steps: B = 8 runs the multi-block attention kernels, B >= 128
    the row-resident forward and backward at A = 1024 (2 / 4 row groups); all use the fused
    H = 512 vocab head; B = 128 the 8-wave persistent LSTM forward and 16-row BPTT, B = 512 the 32-row-team ones,
    B = 1024 two launches of them.  The upper layer's input gradients go through the merged
    two-direction GEMM (gemm_bt_merge) straight into the lower layer's step frame."""
    hps = HParams(batch_size=B, max_enc_steps=800, max_dec_steps=20, vocab_size=V, coverage=True, pointer_gen=True,
                  hidden_dim=512, emb_dim=128, enc_layers=2, trunc_norm_init_std=0.05)
    kinds = _oracle_check(hps, B, 800, 20, seed=21)
    assert kinds["persistent_lstm"] and kinds["fused_vocab"]
    assert kinds["row_attn"] == (B >= 128) and kinds["row_attn_bwd"] == (B >= 128) and kinds["proj_attn"] == (B >= 128)


def test_graph_replay_equals_eager_train_step():
    """Three optimizer steps through the captured graphs == the same steps launched eagerly."""
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer
    B = 256
    hps = _hps(B)
    vocab, batches = _batches(hps, 3, seed=12)
    res = []
    for use_graph in (True, False):
        tr = GraphTrainer(hps, vocab.size(), B=B, T=T, device="cuda:0", use_graph=use_graph)
        init = tr.params.flat.clone()
        losses = []
        for b in batches:
            losses.append(float(tr.check_finite(tr.step(b))["total_loss"]))
        res.append(((tr.params.flat - init).clone(), tr.params.accum.clone(), losses))
        del tr
        torch.cuda.empty_cache()
    (d_g, acc_g, l_g), (d_e, acc_e, l_e) = res
    np.testing.assert_allclose(l_g, l_e, rtol=1e-4)
    assert _rel(d_g, d_e) < 1e-3, _rel(d_g, d_e)
    assert _rel(acc_g, acc_e) < 1e-4


def test_loss_curve_tracks_fp32_oracle_50_steps():
    """50 optimizer steps of the captured bf16 engine vs the fp32 oracle trainer on the same
    batches: two independent trajectories (bf16 and fp32 weights and updates)."""
    from textsummarization_on_flink_amd.train.cpu_trainer import CpuTrainer
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer
    B, steps = 32, 50
    hps = _hps(B)
    vocab, batches = _batches(hps, 10, seed=13)
    hip = GraphTrainer(hps, vocab.size(), B=B, T=T, device="cuda:0")
    ora = CpuTrainer(hps, vocab.size(), device="cuda:0")
    assert torch.equal(hip.params.flat, ora.params.flat)  # same seeded init
    lh, lo = [], []
    for i in range(steps):
        b = batches[i % len(batches)]
        lh.append(float(hip.check_finite(hip.step(b))["total_loss"]))
        lo.append(float(ora.check_finite(ora.step(b))["total_loss"]))
    lh, lo = np.array(lh), np.array(lo)
    dev = np.abs(lh - lo) / lo
    # bf16 vs fp32 trajectories separate slowly, and once the model starts fitting its ten
    # batches (steps ~40+) the gap is also sensitive to the summation order of fp32 atomics,
    # which any change of the launch schedule perturbs (a bit-identical weight repack moved
    # step 46 from < 2% to 4.7%): tight bound while tracking, loose bound late, mean overall.
    # (test_loss_teacher_forced_50_steps below pins the per-step error with one bound.)
    info = (dev.max(), int(dev.argmax()), lh.tolist(), lo.tolist())
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/loss_curve_50.jsonl", "a") as f:
        f.write(json.dumps({"mode": "trajectories", "dev_max": float(dev.max()), "argmax": int(dev.argmax()),
                            "loss_hip": np.round(lh, 4).tolist(), "loss_fp32": np.round(lo, 4).tolist()}) + "\n")
    assert dev[:40].max() < 0.02, info
    assert dev.max() < 0.08 and dev.mean() < 0.015, info
    assert lh[-5:].mean() < lh[:5].mean()  # and it learns


def test_loss_teacher_forced_50_steps(monkeypatch):
    """Deterministic mode (TSAMD_DETERMINISTIC=1), 50 optimizer steps of the captured bf16
    engine; before every step the fp32 oracle evaluates the SAME batch at the engine's own
    current (fp32 master) parameters.  The two independent trajectories of the test above drift
    apart once the model fits (bf16 vs fp32 updates compound, measured up to 6.7 % of the
    initial loss late); pinned per step, the engine's error is a step-local quantity and ONE
    bound holds over all 50 steps."""
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer
    monkeypatch.setenv("TSAMD_DETERMINISTIC", "1")
    B, steps = 32, 50
    hps = _hps(B)
    vocab, batches = _batches(hps, 10, seed=13)
    hip = GraphTrainer(hps, vocab.size(), B=B, T=T, device="cuda:0")
    assert hip.engine.det
    ref = ReferencePointerGenerator(hps, vocab.size())
    P = hip.params
    lh, lo = [], []
    for i in range(steps):
        b = batches[i % len(batches)]
        with torch.no_grad():
            W = {n: P.flat[o:o + c].view(P.view(n).shape) for n, (o, c) in P.offsets.items()}
            lo.append(float(ref.forward(W, batch_to_tensors(b, "cuda"))["total_loss"]))
        lh.append(float(hip.check_finite(hip.step(b))["total_loss"]))
    lh, lo = np.array(lh), np.array(lo)
    dev = np.abs(lh - lo) / lo
    with open("gpurun_out/loss_curve_50.jsonl", "a") as f:
        f.write(json.dumps({"mode": "teacher_forced_det", "dev_max": float(dev.max()), "argmax": int(dev.argmax()),
                            "loss_hip": np.round(lh, 4).tolist(), "loss_fp32": np.round(lo, 4).tolist()}) + "\n")
    assert dev.max() < 1e-4, (dev.max(), int(dev.argmax()), lh.tolist(), lo.tolist())  # measured 2.3e-6
    assert lh[-5:].mean() < lh[:5].mean()


@pytest.mark.parametrize("split", ["2", "4", "2/1", "1/2"])
def test_row_split_streams_match_single_chain(monkeypatch, split):
    """The decoder recurrences run as ``split`` row groups on parallel streams (``fwd/bwd``: a
    different group count for the backward loop, TSAMD_SPLIT_BWD); the result must equal the
    single-chain launch sequence (same kernels on row slices)."""
    from textsummarization_on_flink_amd.models.pointer_generator import HipPointerGenerator
    B = 64
    hps = _hps(B, trunc_norm_init_std=0.05).replace(max_dec_steps=20)
    vocab, (batch,) = _batches(hps, 1, seed=14)
    got = []
    for sp in ("1/1", split if "/" in split else f"{split}/{split}"):
        fw, bw = sp.split("/")
        monkeypatch.setenv("TSAMD_SPLIT", fw)
        monkeypatch.setenv("TSAMD_SPLIT_BWD", bw)
        params = build_params(hps, vocab.size(), device="cuda", seed=5).enable_grad()
        eng = HipPointerGenerator(hps, vocab.size(), params, B=B, T=T, D=20)
        assert (eng.split, eng.split_bwd) == (int(fw), int(bw))
        eng.set_batch(batch)
        out = eng.forward(need_grad=True)
        eng.backward()
        torch.cuda.synchronize()
        got.append((float(out["total_loss"]), eng.w["ATT"].clone(), params.grad.clone()))
    assert abs(got[0][0] - got[1][0]) < 1e-5 * abs(got[0][0])
    assert _rel(got[1][1], got[0][1]) < 1e-6
    assert _rel(got[1][2], got[0][2]) < 1e-4


def test_deferred_weight_gradients_match_inline(monkeypatch):
    """The decoder-side weight gradients deferred onto a side stream beside the encoder BPTT
    (TSAMD_DEFER_WGRAD, default on) give
    the gradients of the inline order, in eager mode and through the captured phase graphs."""
    from textsummarization_on_flink_amd.models.pointer_generator import HipPointerGenerator
    B = 256
    hps = _hps(B, trunc_norm_init_std=0.05).replace(max_dec_steps=24)
    vocab, (batch,) = _batches(hps, 1, seed=15)
    got = []
    for defer in ("0", "1"):
        monkeypatch.setenv("TSAMD_DEFER_WGRAD", defer)
        params = build_params(hps, vocab.size(), device="cuda", seed=6).enable_grad()
        eng = HipPointerGenerator(hps, vocab.size(), params, B=B, T=T, D=24)
        assert eng.defer_wgrad == (defer == "1")
        eng.set_batch(batch)
        eng.forward(need_grad=True)
        eng.backward()
        torch.cuda.synchronize()
        eager = params.grad.clone()
        g = [torch.cuda.CUDAGraph() for _ in range(3)]
        from textsummarization_on_flink_amd.utils.graphs import capture_guard
        with capture_guard():
            with torch.cuda.graph(g[0]):
                eng.forward(need_grad=True)
                eng.backward_head()
            with torch.cuda.graph(g[1]):
                eng.backward_mid()
            with torch.cuda.graph(g[2]):
                eng.backward_tail()
        for x in g:
            x.replay()
        torch.cuda.synchronize()
        got.append((eager, params.grad.clone()))
    for a, b in ((got[0][0], got[1][0]), (got[0][0], got[1][1]), (got[0][0], got[0][1])):
        assert _rel(b, a) < 1e-5, _rel(b, a)


def test_config5_batch2048_graph_replays():
    """Config #5 at batch 2048 (3.4G-element gate buffers, 10G-element dlogits, ~239 GB): the
    captured step replays over distinct batches.  This shape used to fault the GPU on the second
    replay (a device radix sort of the embedding ids inside the captured backward; the order is
    now sorted on the host with the batch) -- profiles/r3/b2048_fault.md."""
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer
    hps = HParams(batch_size=2048, max_enc_steps=800, max_dec_steps=100, vocab_size=50000, hidden_dim=512,
                  emb_dim=128, coverage=True, pointer_gen=True, enc_layers=2)
    corpus = SyntheticCorpus(vocab_size=50000, seed=1000)
    batches = make_batches(hps, corpus.vocab(50000), corpus, 3, pad_enc_to=800)
    tr = GraphTrainer(hps, 50000, B=2048, T=800, device="cuda")
    losses = []
    try:
        for b in batches + batches[:1]:
            out = tr.step(b)
            torch.cuda.synchronize()
            losses.append(tr.check_finite(out)["total_loss"])
    finally:
        del tr
        torch.cuda.empty_cache()
    assert all(math.isfinite(x) for x in losses) and losses[-1] < losses[0], losses


@pytest.mark.parametrize("B,split", [(64, "0"), (256, "1"), (256, "2"), (256, "4")])
def test_deterministic_mode_bit_identical(monkeypatch, B, split):
    """TSAMD_DETERMINISTIC=1: no fp32 atomics in the step (fixed-order embedding / bias /
    attention-parameter reductions, row attention backward, inline weight gradients), so two
    trainings from the same init on the same batches end with bit-identical parameters and
    Adagrad accumulators after 5 captured steps -- with the decoder recurrences as ``split`` row
    groups on parallel streams (0: the default), whose per-row arithmetic is the same on any
    stream, so every split gives the single chain's bits; and the result stays close to the
    default (atomic) path."""
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer
    hps = _hps(B)
    vocab, batches = _batches(hps, 3, seed=17)
    res = {}
    runs = [("det1", "1", split), ("det2", "1", split), ("atomic", "0", "0")]
    if split not in ("0", "1"):
        runs.append(("chain", "1", "1"))
    for mode, det, sp in runs:
        monkeypatch.setenv("TSAMD_DETERMINISTIC", det)
        monkeypatch.setenv("TSAMD_SPLIT", sp)
        tr = GraphTrainer(hps, vocab.size(), B=B, T=T, device="cuda:0")
        assert tr.engine.det == (det == "1")
        if sp != "0":
            assert tr.engine.split == int(sp)
        for i in range(5):
            tr.check_finite(tr.step(batches[i % len(batches)]))
        # bit patterns (torch.equal is False for NaN == NaN even when the bits agree)
        res[mode] = (tr.params.flat.clone().view(torch.int32), tr.params.accum.clone().view(torch.int32))
        offsets = tr.params.offsets
        del tr
        torch.cuda.empty_cache()

    def differ(a, b):
        """(buffer, slice or padding, differing elements, first differing offsets) of params / accumulators"""
        out = []
        for j, name in ((0, "param"), (1, "accum")):
            x, y = res[a][j], res[b][j]
            pad = torch.ones_like(x, dtype=torch.bool)
            for n, (o, c) in offsets.items():
                pad[o:o + c] = False
                d = (x[o:o + c] != y[o:o + c]).nonzero().flatten()
                if d.numel():
                    out.append((name, n, int(d.numel()), c, d[:6].tolist()))
            d = ((x != y) & pad).nonzero().flatten()
            if d.numel():
                out.append((name, "padding", int(d.numel()), int(pad.sum()), d[:6].tolist()))
        return out

    for other in ("det2", "chain"):
        if other in res:
            same = torch.equal(res["det1"][0], res[other][0]) and torch.equal(res["det1"][1], res[other][1])
            if not same:
                for d in differ("det1", other):
                    print(other, *d, flush=True)
            assert same, other
    assert _rel(res["det1"][0].view(torch.float32), res["atomic"][0].view(torch.float32)) < 1e-3


@pytest.mark.parametrize("det", ["1", "0"])
def test_vocab_dw_beside_decoder_loop_matches_inline(monkeypatch, det):
    """TSAMD_VOCAB_DW_SIDE: the vocab dW graph replayed on a side stream beside the decoder backward
    graph (GraphTrainer._Phase1) trains like the dW inside the vocab-backward graph -- bit-identical
    in deterministic mode (same GEMM, only its timing moves), close with the atomic path (compact
    vocab buckets: one dW graph per bucket, batches of different live-row counts)."""
    from textsummarization_on_flink_amd.train import trainer as trm
    B = 256
    hps = _hps(B)
    vocab, batches = _batches(hps, 3, seed=23)
    monkeypatch.setenv("TSAMD_DETERMINISTIC", det)
    res = []
    for side in (False, True):
        monkeypatch.setattr(trm, "VOCAB_DW_SIDE", side)
        tr = trm.GraphTrainer(hps, vocab.size(), B=B, T=T, device="cuda:0")
        assert tr.dw_side == side
        for i in range(4):
            tr.check_finite(tr.step(batches[i % len(batches)]))
        assert bool(tr.g_dw) == side and (len(tr.g_dw) == len(tr.engine.vocab_buckets) or det == "1" or not side)
        res.append((tr.params.flat.clone(), tr.params.accum.clone()))
        del tr
        torch.cuda.empty_cache()
    if det == "1":
        assert torch.equal(res[0][0].view(torch.int32), res[1][0].view(torch.int32))
        assert torch.equal(res[0][1].view(torch.int32), res[1][1].view(torch.int32))
    else:
        assert _rel(res[1][0], res[0][0]) < 1e-4 and _rel(res[1][1], res[0][1]) < 1e-4


def test_bptt_phase_beside_cus_held_like_rccl(monkeypatch):
    """The data-parallel co-residency guard (train/trainer.py): RCCL collective kernels hold at most
    RCCL_MAX_CHANNELS CUs (one workgroup per channel, capped in every rank's environment), and a
    persistent-LSTM grid that leaves that many CUs free may run beside in-flight all-reduces.
    Here a kernel holds exactly LSTM_RCCL_RESERVE_CUS CUs (one workgroup per CU through its whole-LDS
    request, spinning on the clock) while the captured B = 256 step replays, encoder BPTT included:
    no hand-off timeout (lstm_err 0) and gradients bit-equal to the solo step (deterministic mode)."""
    from textsummarization_on_flink_amd.ops import ops
    from textsummarization_on_flink_amd.parallel.rccl_env import RCCL_MAX_CHANNELS
    from textsummarization_on_flink_amd.train.trainer import LSTM_RCCL_RESERVE_CUS, GraphTrainer
    k = ops()
    monkeypatch.setenv("TSAMD_DETERMINISTIC", "1")
    B = 256
    hps = _hps(B)
    vocab, (batch,) = _batches(hps, 1, seed=21)
    tr = GraphTrainer(hps, vocab.size(), B=B, T=T, device="cuda:0")
    eng = tr.engine
    reserve = max(LSTM_RCCL_RESERVE_CUS, RCCL_MAX_CHANNELS)
    grid, cap = int(k.lstm_persistent_grid(eng.H, B)), int(k.lstm_persistent_capacity(eng.H))
    assert eng.persistent_lstm and 0 < grid <= cap - reserve  # the shape the DP trainer lets RCCL overlap
    snap = (tr.params.flat.clone(), tr.params.accum.clone())
    tr.check_finite(tr.step(batch))  # capture + one step

    def step(hold: bool):
        tr.params.flat.copy_(snap[0])
        tr.params.accum.copy_(snap[1])
        eng.pack()
        times = torch.zeros(2 * reserve, dtype=torch.long, device="cuda")
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        if hold:
            with torch.cuda.stream(side):  # held for 300 ms: the whole step (~20 ms) runs beside it
                k.cu_hold(times, reserve, 300.0, int(k.cu_hold_max_lds()))
        tr.step(batch)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        return tr.params.grad.clone().view(torch.int32), int(eng.w["lstm_err"].item()), times.cpu()

    g_solo, err_solo, _ = step(False)
    g_held, err_held, times = step(True)
    assert err_solo == 0 and err_held == 0
    t0, t1 = times[0::2], times[1::2]
    assert int(t0.max()) < int(t1.min())  # every holding workgroup was resident at once
    assert torch.equal(g_solo, g_held)
