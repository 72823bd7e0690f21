"""attn_bwd_step (one launch per decoder step: da, de, ds, dcov) against a plain PyTorch fp32
reference of the same math, at A = 512 (bench, 4-position kernel) and A = 1024 (config #5,
16 features per lane, 256 positions per block).  T = 300 leaves partial blocks; lens of 1, a
few, and T leave fully masked blocks and masked tail groups.

Reference semantics (attention_decoder.py:79-129, model.py:463-480 of the reference): scores
e_i = v . tanh(F_i + s + w_c cov_i), a = masked softmax(e), ctx = sum_i a_i E_i, coverage loss
sum_i min(a_i, cov_i), cov_{t+1} = cov_t + a_t.  The kernels read F stored multiplied by 2 log2(e)
(the engine's F GEMM runs on W_h * 2 log2(e)): each test passes that operand and checks against the
reference on the same values divided back.
"""
import pytest
import torch

from textsummarization_on_flink_amd.ops import ops

pytestmark = pytest.mark.gpu

KF = 2.8853900817779268  # 2 log2(e): the kernels read F stored pre-scaled by it (attn_common.h)


def _scaled(F):
    """(kernel operand, reference features) of bf16 features F: the operand is F * 2 log2(e)
    rounded to bf16, the reference its exact value divided back."""
    Fk = (F.float() * KF).bfloat16()
    return Fk, Fk.float() / KF


def _reference(E, F, s, v, wc, cov, a, dctx, Ga, dnext, g, lens):
    B, T, A = E.shape
    mask = torch.arange(T, device=E.device)[None, :] < lens[:, None].long()
    u = F.float() + s[:, None, :] + wc[None, None, :] * cov[:, :, None]
    sech2 = 1 - torch.tanh(u) ** 2
    r = Ga + dnext + g[:, None] * (a <= cov).float()
    da = r + torch.einsum("bta,ba->bt", E.float(), dctx)
    da = torch.where(mask, da, torch.zeros_like(da))
    S = (a * da).sum(1, keepdim=True)
    de = torch.where(mask, a * (da - S), torch.zeros_like(da))
    ds = torch.einsum("bt,bta->ba", de, sech2) * v[None, :]
    hc = torch.einsum("bta,a->bt", sech2, v * wc)
    dcov = dnext + torch.where(mask, g[:, None] * (a > cov).float() + de * hc, torch.zeros_like(de))
    return de, ds, dcov


@pytest.mark.parametrize("A", [512, 1024])
def test_attn_bwd_step_matches_fp32(A):
    k = ops()
    B, T = 6, 300
    gen = torch.Generator(device="cuda").manual_seed(A)
    dev = "cuda"

    def r(*shape, s=1.0):
        return torch.randn(*shape, generator=gen, device=dev) * s

    lens = torch.tensor([T, 1, 5, 129, 257, 300], dtype=torch.int32, device=dev)
    mask = torch.arange(T, device=dev)[None, :] < lens[:, None].long()
    E, F = r(B, T, A, s=0.5).bfloat16(), r(B, T, A, s=0.5).bfloat16()
    s, v, wc = r(B, A, s=0.3), r(A, s=0.1), r(A, s=0.1)
    cov = torch.rand(B, T, generator=gen, device=dev) * mask
    a = torch.softmax(r(B, T).masked_fill(~mask, float("-inf")), -1)
    ctx = torch.einsum("bt,bta->ba", a, E.float())
    dctx, Ga, dnext = r(B, A, s=0.1), r(B, T, s=0.1), r(B, T, s=0.1)
    g = torch.full((B,), 0.7, device=dev)
    de, ds, dcov = torch.zeros(B, T, device=dev), torch.zeros(B, A, device=dev), torch.zeros(B, T, device=dev)
    Fk, Fr = _scaled(F)
    k.attn_bwd_step(E, Fk, s, v, wc, cov, a, dctx, ctx, Ga, dnext, g, lens, de, ds, dcov, B, T, A)
    torch.cuda.synchronize()
    want = _reference(E, Fr, s, v, wc, cov, a, dctx, Ga, dnext, g, lens)
    for name, got, ref in zip(("de", "ds", "dcov"), (de, ds, dcov), want):
        err = float((got - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
        assert err < 2e-3, (name, err)


@pytest.mark.parametrize("A,Na,rep", [(512, 16, 4), (512, 6, 4), (1024, 8, 4), (512, 64, 1)])
def test_attn_fwd_row_matches_fp32(A, Na, rep):
    """attn_fwd_row: scores, masked softmax, context, coverage update and coverage loss against
    fp32, with rep hypothesis rows per encoder row (beam decode).  Na * rep = 64 and 32 rows take
    the XCD-grouped workgroup -> row map (rows of one article on one XCD), 24 the identity map."""
    k = ops()
    T, B = 300, Na * rep
    gen = torch.Generator(device="cuda").manual_seed(A + Na)
    dev = "cuda"

    def r(*shape, s=1.0):
        return torch.randn(*shape, generator=gen, device=dev) * s

    lens = torch.randint(1, T + 1, (Na,), generator=gen, device=dev, dtype=torch.int32)
    lens[0] = T
    E, F = r(Na, T, A, s=0.5).bfloat16(), r(Na, T, A, s=0.5).bfloat16()
    s, v, wc = r(B, A, s=0.3), r(A, s=0.1), r(A, s=0.5)
    rl = lens.long().repeat_interleave(rep)
    mask = torch.arange(T, device=dev)[None, :] < rl[:, None]
    cov = torch.rand(B, T, generator=gen, device=dev) * mask
    a, cov_out, cl = torch.zeros(B, T, device=dev), torch.zeros(B, T, device=dev), torch.zeros(B, device=dev)
    ctx, ctx_bf = torch.zeros(B, A, device=dev), torch.zeros(B, A, device=dev, dtype=torch.bfloat16)
    Fk, Fr = _scaled(F)
    k.attn_fwd_row(Fk, E, s, v, wc, cov, lens, a, cov_out, cl, ctx, ctx_bf, B, T, A, rep)
    torch.cuda.synchronize()
    Fr, Er = Fr.repeat_interleave(rep, 0), E.float().repeat_interleave(rep, 0)
    e = torch.einsum("bta,a->bt", torch.tanh(Fr + s[:, None, :] + wc[None, None, :] * cov[:, :, None]), v)
    a_ref = torch.softmax(e.masked_fill(~mask, float("-inf")), -1)
    ctx_ref = torch.einsum("bt,bta->ba", a_ref, Er)
    checks = (("a", a, a_ref), ("ctx", ctx, ctx_ref), ("cov_out", cov_out, cov + a_ref),
              ("covloss", cl, torch.minimum(a_ref, cov).sum(1)), ("ctx_bf", ctx_bf.float(), ctx_ref))
    for name, got, ref in checks:
        err = float((got - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
        assert err < (1e-2 if name == "ctx_bf" else 2e-3), (name, err)


@pytest.mark.parametrize("A", [512, 1024])
def test_attn_bwd_row_matches_fp32(A):
    """attn_bwd_row (one workgroup per row) against the fp32 reference of the fused attention
    backward step, A = 512 (parameters in registers) and 1024 (in LDS); lens of 1, a few and T."""
    k = ops()
    B, T = 6, 300
    gen = torch.Generator(device="cuda").manual_seed(78)
    dev = "cuda"

    def r(*shape, s=1.0):
        return torch.randn(*shape, generator=gen, device=dev) * s

    lens = torch.tensor([T, 1, 5, 129, 257, 300], dtype=torch.int32, device=dev)
    mask = torch.arange(T, device=dev)[None, :] < lens[:, None].long()
    E, F = r(B, T, A, s=0.5).bfloat16(), r(B, T, A, s=0.5).bfloat16()
    s, v, wc = r(B, A, s=0.3), r(A, s=0.1), r(A, s=0.1)
    cov = torch.rand(B, T, generator=gen, device=dev) * mask
    a = torch.softmax(r(B, T).masked_fill(~mask, float("-inf")), -1)
    ctx = torch.einsum("bt,bta->ba", a, E.float())
    dctx, Ga, dnext = r(B, A, s=0.1), r(B, T, s=0.1), r(B, T, s=0.1)
    g = torch.full((B,), 0.7, device=dev)
    de, dcov = torch.full((B, T), float("nan"), device=dev), torch.full((B, T), float("nan"), device=dev)
    ds = torch.full((B, A), float("nan"), device=dev)
    Fk, Fr = _scaled(F)
    k.attn_bwd_row(E, Fk, s, v, wc, cov, a, dctx, ctx, Ga, dnext, g, lens, de, ds, dcov, B, T, A)
    torch.cuda.synchronize()
    got_ds = ds
    want = _reference(E, Fr, s, v, wc, cov, a, dctx, Ga, dnext, g, lens)
    for name, got, ref in zip(("de", "ds", "dcov"), (de, got_ds, dcov), want):
        err = float((got - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
        assert err < 2e-3, (name, err)


@pytest.mark.parametrize("A", [512, 1024])
def test_attn_fwd_rowp_matches_fp32(A):
    """attn_fwd_rowp (projected context, training): a, coverage, coverage loss and
    g = sum_i a_i G_i against fp32; lens of 1, a few, a partial last group and T."""
    k = ops()
    B, T, EG = 6, 300, 128
    gen = torch.Generator(device="cuda").manual_seed(A + 5)
    dev = "cuda"

    def r(*shape, s=1.0):
        return torch.randn(*shape, generator=gen, device=dev) * s

    lens = torch.tensor([T, 1, 5, 130, 257, 299], dtype=torch.int32, device=dev)
    mask = torch.arange(T, device=dev)[None, :] < lens[:, None].long()
    F, G = r(B, T, A, s=0.5).bfloat16(), r(B, T, EG, s=0.5).bfloat16()
    s, v, wc = r(B, A, s=0.3), r(A, s=0.1), r(A, s=0.5)
    cov = torch.rand(B, T, generator=gen, device=dev) * mask
    a, cov_out, cl = (torch.full((B, T), float("nan"), device=dev), torch.zeros(B, T, device=dev),
                      torch.zeros(B, device=dev))
    gx, gxb = torch.zeros(B, EG, device=dev), torch.zeros(B, EG, device=dev, dtype=torch.bfloat16)
    Fk, Fr = _scaled(F)
    ab = torch.full((B, T), float("nan"), device=dev, dtype=torch.bfloat16)
    k.attn_fwd_rowp(Fk, G, s, v, wc, cov, lens, a, cov_out, cl, gx, gxb, B, T, A, None, 0, ab)
    torch.cuda.synchronize()
    e = torch.einsum("bta,a->bt", torch.tanh(Fr + s[:, None, :] + wc[None, None, :] * cov[:, :, None]), v)
    a_ref = torch.softmax(e.masked_fill(~mask, float("-inf")), -1)
    g_ref = torch.einsum("bt,bte->be", a_ref, G.float())
    assert torch.equal(ab, a.bfloat16())  # the bf16 twin of a, written by the same kernel
    checks = (("a", a, a_ref), ("g", gx, g_ref), ("cov_out", cov_out, cov + a_ref),
              ("covloss", cl, torch.minimum(a_ref, cov).sum(1)), ("g_bf", gxb.float(), g_ref))
    for name, got, ref in checks:
        err = float((got - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
        assert err < (1e-2 if name == "g_bf" else 2e-3), (name, err)


@pytest.mark.parametrize("A", [512, 1024])
@pytest.mark.parametrize("last", [False, True])
def test_attn_bwd_rowp_matches_fp32(A, last):
    """attn_bwd_rowp: the backward step with da_i = r_i + dx . G_i (dx = None: the last decoder
    step) against the fp32 reference, which is the E-form with dctx . E_i = dx . G_i when
    G = E . W and dctx = W . dx."""
    k = ops()
    B, T, EG = 6, 300, 128
    gen = torch.Generator(device="cuda").manual_seed(91 + A)
    dev = "cuda"

    def r(*shape, s=1.0):
        return torch.randn(*shape, generator=gen, device=dev) * s

    lens = torch.tensor([T, 1, 5, 129, 258, 300], dtype=torch.int32, device=dev)
    mask = torch.arange(T, device=dev)[None, :] < lens[:, None].long()
    G, F = r(B, T, EG, s=0.5).bfloat16(), r(B, T, A, s=0.5).bfloat16()
    s, v, wc = r(B, A, s=0.3), r(A, s=0.1), r(A, s=0.1)
    cov = torch.rand(B, T, generator=gen, device=dev) * mask
    a = torch.softmax(r(B, T).masked_fill(~mask, float("-inf")), -1)
    gv = torch.einsum("bt,bte->be", a, G.float())
    dx = None if last else r(B, EG, s=0.1)
    Ga, dnext = r(B, T, s=0.1), r(B, T, s=0.1)
    g = torch.full((B,), 0.7, device=dev)
    de, dcov = torch.full((B, T), float("nan"), device=dev), torch.full((B, T), float("nan"), device=dev)
    ds = torch.full((B, A), float("nan"), device=dev)
    Fk, Fr = _scaled(F)
    k.attn_bwd_rowp(G, Fk, s, v, wc, cov, a, dx, gv, Ga, dnext, g, lens, de, ds, dcov, B, T, A, None, 0)
    torch.cuda.synchronize()
    # the E-form reference with "E" = G and "dctx" = dx (zero at the last step)
    want = _reference(G, Fr, s, v, wc, cov, a, torch.zeros(B, EG, device=dev) if last else dx, Ga, dnext, g, lens)
    for name, got, ref in zip(("de", "ds", "dcov"), (de, ds, dcov), want):
        err = float((got - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
        assert err < 2e-3, (name, err)
