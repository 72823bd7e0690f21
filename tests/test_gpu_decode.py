"""Device beam search: final_topk / beam_step kernels vs references, graph == eager, and
end-to-end agreement with the host beam search over the PyTorch oracle."""
import numpy as np
import pytest
import torch

from textsummarization_on_flink_amd.config import HParams
from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
from textsummarization_on_flink_amd.models.params import build_params
from textsummarization_on_flink_amd.models.reference import ReferencePointerGenerator

pytestmark = pytest.mark.gpu


def test_final_topk_matches_materialised_distribution():
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    torch.manual_seed(0)
    Na, beam, V, T, K = 5, 4, 3000, 96, 8
    R = Na * beam
    logits = torch.randn(R, V, device="cuda") * 3
    bias = torch.randn(V, device="cuda")
    pg = torch.rand(R, device="cuda")
    lens = torch.randint(20, T + 1, (Na,), device="cuda", dtype=torch.int32)
    ext = torch.randint(0, V + 20, (Na, T), device="cuda", dtype=torch.int32)
    ext[:, :10] = ext[:, 10:20]  # duplicates
    attn = torch.rand(R, T, device="cuda")
    mask = (torch.arange(T, device="cuda")[None] < lens.repeat_interleave(beam)[:, None]).float()
    attn = attn * mask
    attn = attn / attn.sum(1, keepdim=True)
    ids = torch.zeros(R, K, dtype=torch.int32, device="cuda")
    lp = torch.zeros(R, K, device="cuda")
    S = int(k.topk_parts(V))
    pms = torch.zeros(R, S, 2, device="cuda")
    pv = torch.zeros(R, S, K, device="cuda")
    pi = torch.zeros(R, S, K, dtype=torch.int32, device="cuda")
    k.final_topk(logits, bias, pg, attn, ext, lens, ids, lp, pms, pv, pi, R, V, T, K, beam)
    # reference: materialise [R, V + 20]
    vd = torch.softmax(logits + bias, 1)
    fd = torch.cat([pg[:, None] * vd, torch.zeros(R, 20, device="cuda")], 1)
    fd = fd.scatter_add(1, ext.repeat_interleave(beam, 0).long(), (1 - pg[:, None]) * attn)
    rp, ri = torch.topk(fd, K, 1)
    assert torch.equal(ids.long(), ri)
    torch.testing.assert_close(lp, torch.log(rp), rtol=1e-4, atol=1e-5)
    # baseline mode
    k.final_topk(logits, bias, None, None, ext, lens, ids, lp, pms, pv, pi, R, V, T, K, beam)
    rp, ri = torch.topk(vd, K, 1)
    assert torch.equal(ids.long(), ri)


def _py_beam_step(state, ids, lps, t, beam, K, stop, min_dec):
    """numpy mirror of beam_search.py:126-154 for Na articles."""
    Na = len(state["done"])
    for a in range(Na):
        base = a * beam
        if state["done"][a]:
            state["gidx"][base:base + beam] = np.arange(base, base + beam)
            continue
        norig = 1 if t == 0 else beam
        cands = []
        for i in range(norig):
            for j in range(K):
                cands.append((state["lp"][base + i] + lps[base + i, j], i, int(ids[base + i, j])))
        order = sorted(range(len(cands)), key=lambda c: cands[c][0], reverse=True)
        nh, new = 0, []
        for c in order:
            v, i, tok = cands[c]
            if tok == stop:
                if t >= min_dec:
                    state["res"][a].append((v / (t + 2), t, i))
            else:
                new.append((v, tok, i))
            if len(new) == beam or len(state["res"][a]) == beam:
                break
        if len(state["res"][a]) >= beam:
            state["done"][a] = 1
        for kk in range(beam):
            v, tok, i = new[min(kk, len(new) - 1)]
            state["lp"][base + kk] = v
            state["latest"][base + kk] = tok
            state["gidx"][base + kk] = base + i


def test_beam_step_kernel_matches_python():
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    rng = np.random.default_rng(1)
    Na, beam, K, stop, min_dec, maxD = 6, 4, 8, 3, 2, 12
    R = Na * beam
    dev = {n: torch.zeros(s, dtype=d, device="cuda") for n, s, d in [
        ("lp", (R,), torch.float32), ("latest", (R,), torch.int32), ("gidx", (R,), torch.int32),
        ("th", (maxD, R), torch.int32), ("ph", (maxD, R), torch.int32), ("done", (Na,), torch.int32),
        ("rc", (Na,), torch.int32), ("rs", (R,), torch.float32), ("rl", (R,), torch.int32),
        ("rst", (R,), torch.int32), ("rp", (R,), torch.int32), ("step", (1,), torch.int32),
        ("ctr", (1,), torch.int32), ("att", (R, 7), torch.float32), ("ah", (maxD, R, 7), torch.float32),
        ("pg", (R,), torch.float32), ("pgh", (maxD, R), torch.float32)]}
    st = {"lp": np.zeros(R, np.float32), "latest": np.zeros(R, np.int64), "gidx": np.arange(R),
          "done": np.zeros(Na, np.int64), "res": [[] for _ in range(Na)]}
    for t in range(maxD):
        ids = rng.integers(0, 40, (R, K)).astype(np.int32)
        ids[rng.random((R, K)) < 0.15] = stop
        for r in range(R):  # distinct ids per row like top_k
            ids[r] = rng.permutation(40)[:K]
            if rng.random() < 0.3:
                ids[r, rng.integers(0, K)] = stop
        lps = np.sort(np.log(rng.random((R, K)).astype(np.float32)), 1)[:, ::-1].copy()
        dev["att"].uniform_()
        dev["pg"].uniform_()
        k.beam_step(torch.from_numpy(ids).cuda(), torch.from_numpy(lps).cuda(), dev["lp"], dev["latest"], dev["gidx"],
                    dev["th"], dev["ph"], dev["done"], dev["rc"], dev["rs"], dev["rl"], dev["rst"], dev["rp"],
                    dev["step"], dev["ctr"], dev["att"], dev["ah"], dev["pg"], dev["pgh"], 7, Na, beam, K, stop,
                    min_dec, maxD)
        assert int(dev["step"].item()) == t + 1 and int(dev["ctr"].item()) == 0  # kernel advances the step
        torch.testing.assert_close(dev["ah"][t], dev["att"], rtol=0, atol=0)
        torch.testing.assert_close(dev["pgh"][t], dev["pg"], rtol=0, atol=0)
        _py_beam_step(st, ids, lps, t, beam, K, stop, min_dec)
        np.testing.assert_array_equal(dev["done"].cpu().numpy(), st["done"])
        live = np.repeat(st["done"] == 0, beam)
        np.testing.assert_allclose(dev["lp"].cpu().numpy()[live], st["lp"][live], rtol=1e-6)
        np.testing.assert_array_equal(dev["latest"].cpu().numpy()[live], st["latest"][live])
        np.testing.assert_array_equal(dev["gidx"].cpu().numpy(), st["gidx"])
        rc = dev["rc"].cpu().numpy()
        for a in range(Na):
            assert rc[a] == len(st["res"][a])
            got = dev["rs"].cpu().numpy()[a * beam:a * beam + rc[a]]
            np.testing.assert_allclose(got, [x[0] for x in st["res"][a]], rtol=1e-6)


def _peaked_setup(coverage, Na=8, T=48, V=600, pointer_gen=True):
    hps = HParams(batch_size=Na, max_enc_steps=T, max_dec_steps=20, min_dec_steps=3, beam_size=4, vocab_size=V,
                  emb_dim=64, hidden_dim=64, coverage=coverage, pointer_gen=pointer_gen, trunc_norm_init_std=0.5,
                  rand_unif_init_mag=0.3)
    corpus = SyntheticCorpus(vocab_size=V, raw_vocab=3 * V, seed=2, art_mean=40, art_sd=10, sent_mean=4)
    vocab = corpus.vocab(V)
    batch = make_batches(hps, vocab, corpus, 1, pad_enc_to=T)[0]
    params = build_params(hps, vocab.size(), device="cuda", seed=3)
    return hps, vocab, batch, params


@pytest.mark.parametrize("coverage,pointer_gen", [(True, True), (False, True), (False, False)])
def test_device_beam_graph_equals_eager_and_tracks_oracle(coverage, pointer_gen):
    from textsummarization_on_flink_amd.data.batch import Batch, Example
    from textsummarization_on_flink_amd.decode.beam_search import OracleStepModel, run_beam_search
    from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
    hps, vocab, batch, params = _peaked_setup(coverage, pointer_gen=pointer_gen)
    dg = DeviceBeamDecoder(hps, vocab, params, n_articles=hps.batch_size, T=hps.max_enc_steps, use_graph=True)
    hg = dg.decode(batch)
    de = DeviceBeamDecoder(hps, vocab, params, n_articles=hps.batch_size, T=hps.max_enc_steps, use_graph=False)
    he = de.decode(batch)
    assert [h.tokens for h in hg] == [h.tokens for h in he]
    # host beam search over the fp32 oracle, one article at a time (reference decode path)
    flat = params.flat
    W = {n: flat[o:o + c].view(params.view(n).shape) for n, (o, c) in params.offsets.items()}
    model = OracleStepModel(ReferencePointerGenerator(hps, vocab.size()), W, hps, device="cuda")
    hps1 = hps.replace(batch_size=hps.beam_size)
    agree = 0
    for a in range(hps.batch_size):
        ex = Example(batch.original_articles[a], batch.original_abstracts_sents[a], vocab, hps1)
        b1 = Batch([ex] * hps.beam_size, hps1, vocab, pad_enc_to=hps.max_enc_steps)
        best = run_beam_search(model, vocab, b1, hps)
        n = min(len(best.tokens), len(hg[a].tokens), 6)
        agree += best.tokens[:n] == hg[a].tokens[:n]
    assert agree >= hps.batch_size - 2, agree
    if dg.keep_attn:
        assert len(hg[0].attn_dists) == len(hg[0].tokens) - 1


@pytest.mark.parametrize("overlap,flush,group", [(False, False, 1), (False, False, 2), (False, False, 4),
                                                 (False, True, 4), (True, False, 1), (True, True, 1)])
def test_pipelined_decode_batches_equal_batch_by_batch(overlap, flush, group):
    """decode_batches (results snapshotted to pinned memory, backtracked while the next batch
    runs; overlap: the next batch's encoder on a side stream beside the decode steps; group: up to
    that many queued batches encoded as one pass -- 2: a pair then the third alone, 4: all three in
    one 4-batch pass with a repeated batch filling the rows) == decode() batch by batch: same
    summaries in the same order."""
    from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
    hps, vocab, batch, params = _peaked_setup(True, pointer_gen=True)
    corpus = SyntheticCorpus(vocab_size=hps.vocab_size, raw_vocab=3 * hps.vocab_size, seed=9, art_mean=40, art_sd=10,
                             sent_mean=4)
    more = make_batches(hps, vocab, corpus, 2, pad_enc_to=hps.max_enc_steps)
    batches = [batch] + more
    d = DeviceBeamDecoder(hps, vocab, params, n_articles=hps.batch_size, T=hps.max_enc_steps, use_graph=True)
    seq = [[h.tokens for h in d.decode(b)] for b in batches]
    d.overlap_encoder = overlap
    d.group_enc = group
    # flush: a streaming source with nothing queued between batches (FLUSH from the encoder
    # look-ahead, then a batch from the last-chunk poll, which was not pre-encoded)
    src = [x for b in batches for x in (b, d.FLUSH)] if flush else batches
    piped = [[h.tokens for h in hy] for hy in d.decode_batches(src)]
    assert piped == seq


@pytest.mark.parametrize("B,K1,K2,N,use_add", [(20, 256, 512, 256, False), (37, 512, 0, 128, True),
                                               (64, 256, 256, 512, False), (33, 512, 512, 256, True),
                                               (16, 1024, 1024, 128, False)])
def test_linear2_matches_fp32(B, K1, K2, N, use_add):
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    torch.manual_seed(1)
    a1 = torch.randn(B, K1, device="cuda").bfloat16()
    a2 = torch.randn(B, K2, device="cuda").bfloat16() if K2 else None
    Wt = (torch.randn(N, K1 + K2, device="cuda") * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda")
    add = torch.randn(B, N, device="cuda") if use_add else None
    A = a1.float() if a2 is None else torch.cat([a1.float(), a2.float()], 1)
    ref = A @ Wt.float().t() + bias + (add if add is not None else 0)
    out = add.clone() if use_add else torch.zeros(B, N, device="cuda")
    outb = torch.zeros(B, N, device="cuda", dtype=torch.bfloat16)
    k.linear2(a1, K1, a2, K2, Wt, bias, out if use_add else None, out, outb, B, N)
    torch.cuda.synchronize()
    assert (out - ref).abs().max().item() < 1e-3 * ref.abs().max().item() + 1e-4
    assert (outb.float() - ref).abs().max().item() < 1e-2 * ref.abs().max().item()


@pytest.mark.parametrize("R", [256, 37])
def test_linear2_pair_matches_two_linear2(R):
    """The beam step's pair launch at the shipped shape (H=256, A=512, E=128): problem 0 is the
    attention query s = [c, h].W_s + b (N = A = 512), problem 1 the in-place x-merge
    x += ctx.W_in[E:] (M = E = 128 < N, add aliases out; column tiles past M exit early).
    Both must equal separate linear2 launches and the fp32 reference; R = 37 is not a
    multiple of 16 (partial row tile)."""
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    torch.manual_seed(3)
    H, A, E = 256, 512, 128
    c = torch.randn(R, H, device="cuda").bfloat16()
    h = torch.randn(R, H, device="cuda").bfloat16()
    ctx = torch.randn(R, A, device="cuda").bfloat16()
    WsT = (torch.randn(A, 2 * H, device="cuda") * 0.05).bfloat16()
    bs = torch.randn(A, device="cuda")
    WicT = (torch.randn(E, A, device="cuda") * 0.05).bfloat16()
    x0 = torch.randn(R, E, device="cuda")
    s_pair, x_pair = torch.zeros(R, A, device="cuda"), x0.clone()
    k.linear2_pair(c, H, h, H, WsT, bs, None, s_pair, None, A, ctx, A, None, 0, WicT, None, x_pair, x_pair, None, E, R)
    s_one, x_one = torch.zeros(R, A, device="cuda"), x0.clone()
    k.linear2(c, H, h, H, WsT, bs, None, s_one, None, R, A)
    k.linear2(ctx, A, None, 0, WicT, None, x_one, x_one, None, R, E)
    torch.cuda.synchronize()
    assert torch.equal(s_pair, s_one) and torch.equal(x_pair, x_one)
    s_ref = torch.cat([c.float(), h.float()], 1) @ WsT.float().t() + bs
    x_ref = x0 + ctx.float() @ WicT.float().t()
    assert (s_pair - s_ref).abs().max().item() < 1e-3 * s_ref.abs().max().item() + 1e-4
    assert (x_pair - x_ref).abs().max().item() < 1e-3 * x_ref.abs().max().item() + 1e-4


def test_pgen_matches_fp32():
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    torch.manual_seed(2)
    R, A, H, E = 30, 512, 256, 128
    ctx, c, x = torch.randn(R, A, device="cuda"), torch.randn(R, H, device="cuda"), torch.randn(R, E, device="cuda")
    h = torch.randn(R, H, device="cuda").bfloat16()
    w = torch.randn(A + 2 * H + E, device="cuda") * 0.05
    b = torch.randn(1, device="cuda")
    pg = torch.zeros(R, device="cuda")
    k.pgen(ctx, c, h, x, w, b, pg, R, A, H, E)
    ref = torch.sigmoid(torch.cat([ctx, c, h.float(), x], 1) @ w + b)
    torch.cuda.synchronize()
    assert (pg - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("pointer,V,H,bias_kind", [
    (True, 3000, 128, "rand"), (False, 3000, 128, "rand"), (True, 600, 64, "rand"), (False, 600, 64, "rand"),
    (False, 50000, 256, "rand"), (True, 50000, 512, "rand"), (False, 3000, 512, "rand"),
    (True, 50000, 256, "zipf"), (False, 50000, 256, "zipf"), (True, 3000, 128, "flat")])
def test_fused_vocab_topk_matches_materialised_path(pointer, V, H, bias_kind):
    """vocab_topk (MFMA logits + per-tile (max, sum exp) partials, then a select that reads
    only the K best tiles of each row) == the library GEMM + final_topk path; V=600 has
    fewer vocab tiles than K.  bias_kind "zipf": a trained model's frequency-shaped output
    bias over a frequency-sorted vocabulary (the best tiles are full of entries above the
    tile bound: the select's group-maxima bound prunes them); "flat": every logit equal
    (ties broken by id)."""
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    torch.manual_seed(5)
    Na, beam, T, K = 5, 4, 96, 8
    R = Na * beam
    X = (torch.randn(R, H, device="cuda")).bfloat16()
    W = (torch.randn(H, V, device="cuda") * 0.3).bfloat16()
    bias = torch.randn(V, device="cuda")
    if bias_kind == "zipf":
        W = (W.float() * 0.05).bfloat16()
        bias = -1.5 * torch.log1p(torch.arange(V, device="cuda", dtype=torch.float32)) + 0.05 * bias
    elif bias_kind == "flat":
        W = torch.zeros_like(W)
        bias = torch.full((V,), 0.25, device="cuda")
    lens = torch.randint(20, T + 1, (Na,), device="cuda", dtype=torch.int32)
    ext = torch.randint(0, V + 20, (Na, T), device="cuda", dtype=torch.int32)
    ext[:, :10] = ext[:, 10:20]
    pg = torch.rand(R, device="cuda") if pointer else None
    attn = None
    if pointer:
        attn = torch.rand(R, T, device="cuda")
        mask = (torch.arange(T, device="cuda")[None] < lens.repeat_interleave(beam)[:, None]).float()
        attn = attn * mask
        attn = attn / attn.sum(1, keepdim=True)
    logits = torch.mm(X, W, out_dtype=torch.float32)
    S = int(k.topk_parts(V))
    ids0 = torch.zeros(R, K, dtype=torch.int32, device="cuda")
    lp0 = torch.zeros(R, K, device="cuda")
    k.final_topk(logits, bias, pg, attn, ext, lens, ids0, lp0, torch.zeros(R, S, 2, device="cuda"),
                 torch.zeros(R, S, K, device="cuda"), torch.zeros(R, S, K, dtype=torch.int32, device="cuda"),
                 R, V, T, K, beam)
    nt = int(k.vocab_topk_parts(V, H))
    ids1 = torch.zeros(R, K, dtype=torch.int32, device="cuda")
    lp1 = torch.zeros(R, K, device="cuda")
    lg = torch.zeros(R, V, device="cuda")
    k.vocab_topk(X, W.t().contiguous(), bias, pg, attn, ext, lens, ids1, lp1, lg, torch.zeros(R, nt, 2, device="cuda"),
                 R, V, H, T, K, beam)
    torch.cuda.synchronize()
    assert (lg - (logits + bias)).abs().max().item() < 1e-3
    bad = (ids0 != ids1).any(1).nonzero().flatten().tolist()
    assert not bad, (bad, ids0[bad[:2]].tolist(), ids1[bad[:2]].tolist(), lp0[bad[:2]].tolist(), lp1[bad[:2]].tolist())
    assert (lp0 - lp1).abs().max().item() < 1e-3


@pytest.mark.parametrize("coverage", [True, False])
def test_row_attention_decode_production_width(coverage, monkeypatch):
    """Beam decode at the production width (H=256, E=128: A=512, where the decode step uses
    the row-resident attention kernel with rep = beam) against the multi-block attention
    kernels (TSAMD_DEC_ROW_ATTN=0): same precision but a different summation order, so the
    first 6 tokens agree on >= 90% of the articles and full summaries on >= 70%.  Against the host beam search over the fp32 oracle the first 6 tokens must
    agree on >= 70%: with random weights, bf16 rounding flips beams at near-ties and the
    untrained recurrence amplifies it (tools/decode_agreement.py: full-summary agreement 6/10
    with coverage, 1/10 without, identical for both attention paths; larger inits agree less)."""
    from textsummarization_on_flink_amd.data.batch import Batch, Example
    from textsummarization_on_flink_amd.decode.beam_search import OracleStepModel, run_beam_search
    from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
    Na, T, V = 10, 64, 2000
    hps = HParams(batch_size=Na, max_enc_steps=T, max_dec_steps=24, min_dec_steps=3, beam_size=4, vocab_size=V,
                  emb_dim=128, hidden_dim=256, coverage=coverage, pointer_gen=True, trunc_norm_init_std=0.5,
                  rand_unif_init_mag=0.3)
    corpus = SyntheticCorpus(vocab_size=V, raw_vocab=3 * V, seed=5, art_mean=50, art_sd=10, sent_mean=4)
    vocab = corpus.vocab(V)
    batch = make_batches(hps, vocab, corpus, 1, pad_enc_to=T)[0]
    params = build_params(hps, vocab.size(), device="cuda", seed=4)
    row = DeviceBeamDecoder(hps, vocab, params, n_articles=Na, T=T, use_graph=True)
    assert row.row_attn
    hr = row.decode(batch)
    monkeypatch.setenv("TSAMD_DEC_ROW_ATTN", "0")
    mb = DeviceBeamDecoder(hps, vocab, params, n_articles=Na, T=T, use_graph=True)
    assert not mb.row_attn
    hm = mb.decode(batch)
    same = sum(a.tokens == b.tokens for a, b in zip(hr, hm))
    same6 = sum(a.tokens[:6] == b.tokens[:6] for a, b in zip(hr, hm))
    assert same >= 0.7 * Na and same6 >= 0.9 * Na, (same, same6)
    flat = params.flat
    W = {n: flat[o:o + c].view(params.view(n).shape) for n, (o, c) in params.offsets.items()}
    model = OracleStepModel(ReferencePointerGenerator(hps, vocab.size()), W, hps, device="cuda")
    hps1 = hps.replace(batch_size=hps.beam_size)
    agree = 0
    for a in range(Na):
        ex = Example(batch.original_articles[a], batch.original_abstracts_sents[a], vocab, hps1)
        b1 = Batch([ex] * hps.beam_size, hps1, vocab, pad_enc_to=T)
        agree += run_beam_search(model, vocab, b1, hps).tokens[:6] == hr[a].tokens[:6]
    assert agree >= 0.7 * Na, agree


@pytest.mark.parametrize("coverage,pointer_gen,H", [(True, True, 256), (False, True, 256), (False, False, 256),
                                                    (True, True, 512)])
def test_fused_decode_step_equals_unfused(coverage, pointer_gen, H):
    """The 6-launch decode step (parent / token gathers inside the cell, x-merge and attention
    kernels; beam bookkeeping in the vocab select kernel's tail) == the 8-launch step
    (beam_gather ... beam_step): same arithmetic on the same values, so the same summaries and
    attention histories bit for bit (scores to 1e-6: the bookkeeping's final division may be
    compiled differently inside the select kernel); graph-captured."""
    from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
    Na, T, V = 16, 120, 3000
    hps = HParams(mode="decode", batch_size=Na, max_enc_steps=T, max_dec_steps=30, min_dec_steps=5, beam_size=4,
                  vocab_size=V, emb_dim=128, hidden_dim=H, coverage=coverage, pointer_gen=pointer_gen,
                  trunc_norm_init_std=0.05)
    corpus = SyntheticCorpus(vocab_size=V, raw_vocab=3 * V, seed=8, art_mean=100, art_sd=20, sent_mean=5)
    vocab = corpus.vocab(V)
    batch = make_batches(hps, vocab, corpus, 1, pad_enc_to=T)[0]
    params = build_params(hps, vocab.size(), device="cuda", seed=9)
    res = []
    for fused in (True, False):
        d = DeviceBeamDecoder(hps, vocab, params, n_articles=Na, T=T, use_graph=True)
        assert d.fused_step
        d.fused_step = fused
        hy = d.decode(batch)
        res.append(([h.tokens for h in hy], [h.avg_log_prob for h in hy], [np.stack(h.attn_dists) for h in hy],
                    [np.array(h.p_gens, dtype=np.float64) if pointer_gen else None for h in hy]))
    assert res[0][0] == res[1][0]
    np.testing.assert_allclose(res[0][1], res[1][1], rtol=1e-6)
    for a, b in zip(res[0][2], res[1][2]):
        np.testing.assert_array_equal(a, b)
    if pointer_gen:  # p_gen histories (each row workgroup stores its own entry in the fused step)
        for a, b in zip(res[0][3], res[1][3]):
            np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)
