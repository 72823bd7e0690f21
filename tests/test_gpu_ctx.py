"""Batched attention-context GEMMs (csrc/kernels/ctx_bmm.hip) against fp32 einsums of the same
bf16 operands: the decoder's context a . enc_out for all steps (step-major output + bf16 twin),
its attention gradient dctx . enc_out^T (stored or accumulated into the step-major dA) and its
encoder-output gradient a^T . dctx -- D below / at the 128-row limit, T not a multiple of 64 (the
K tail of ctx_fwd, the partial t tiles of ctx_da / ctx_de), A = 128 .. 512."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(8, 400, 100, 512), (5, 136, 37, 256), (3, 72, 128, 128), (2, 8, 1, 128), (4, 200, 16, 384)]


def _k():
    from textsummarization_on_flink_amd.ops import ops
    return ops()


def _close(got, ref, tol=1e-4):
    err = float((got.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
    assert err < tol, err


def _ops(B, T, D, A, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    att = torch.rand(D, B, T, device="cuda", generator=g).bfloat16()
    enc = torch.randn(B, T, A, device="cuda", generator=g).bfloat16()
    dctx = torch.randn(D, B, A, device="cuda", generator=g).bfloat16()
    return att, enc, dctx


@pytest.mark.parametrize("B,T,D,A", SHAPES)
def test_ctx_fwd_matches_fp32(B, T, D, A):
    k = _k()
    assert k.ctx_bmm_ok(B, T, D, A)
    att, enc, _ = _ops(B, T, D, A, B + T + D + A)
    ctx = torch.full((D, B, A), float("nan"), device="cuda")
    ctxb = torch.zeros(D, B, A, device="cuda", dtype=torch.bfloat16)
    k.ctx_fwd(att, enc, ctx, ctxb, B, T, D, A)
    torch.cuda.synchronize()
    ref = torch.einsum("dbt,bta->dba", att.float(), enc.float())
    _close(ctx, ref)
    assert torch.equal(ctxb, ctx.bfloat16())


@pytest.mark.parametrize("acc", [False, True])
@pytest.mark.parametrize("B,T,D,A", SHAPES)
def test_ctx_da_matches_fp32(B, T, D, A, acc):
    k = _k()
    _, enc, dctx = _ops(B, T, D, A, 7 * B + T + D + A)
    g = torch.Generator(device="cuda").manual_seed(1)
    base = torch.randn(D, B, T, device="cuda", generator=g)
    full = torch.full((D * B * T + 64,), 12345.0, device="cuda")
    da = full[:D * B * T].view(D, B, T)
    da.copy_(base) if acc else da.fill_(float("nan"))
    k.ctx_da(dctx, enc, da, B, T, D, A, acc)
    torch.cuda.synchronize()
    ref = torch.einsum("dba,bta->dbt", dctx.float(), enc.float()) + (base if acc else 0)
    _close(da, ref)
    assert bool((full[D * B * T:] == 12345.0).all())


@pytest.mark.parametrize("B,T,D,A", SHAPES)
def test_ctx_de_matches_fp32(B, T, D, A):
    k = _k()
    att, _, dctx = _ops(B, T, D, A, 3 * B + T + D + A)
    full = torch.full((B * T * A + 64,), 12345.0, device="cuda")
    de = full[:B * T * A].view(B, T, A)
    de.fill_(float("nan"))
    k.ctx_de(att, dctx, de, B, T, D, A)
    torch.cuda.synchronize()
    ref = torch.einsum("dbt,dba->bta", att.float(), dctx.float())
    _close(de, ref)
    assert bool((full[B * T * A:] == 12345.0).all())


@pytest.mark.parametrize("B,T,D,A", SHAPES[:3])
def test_ctx_de_into_bf16(B, T, D, A):
    """bf16 dE mode: a^T . dctx stored in bf16 (the engine's bf16 encoder-output gradient, to which the
    W_h GEMM adds dF . W_h^T): the fp32 result rounded once."""
    k = _k()
    att, _, dctx = _ops(B, T, D, A, 5 * B + T + D + A)
    de = torch.full((B, T, A), float("nan"), device="cuda", dtype=torch.bfloat16)
    k.ctx_de(att, dctx, de, B, T, D, A)
    de32 = torch.empty(B, T, A, device="cuda")
    k.ctx_de(att, dctx, de32, B, T, D, A)
    torch.cuda.synchronize()
    assert torch.equal(de, de32.bfloat16())
    ref = torch.einsum("dbt,dba->bta", att.float(), dctx.float())
    _close(de, ref, 1e-2)


def test_ctx_bmm_declines_unsupported_shapes():
    k = _k()
    assert not k.ctx_bmm_ok(4, 100, 129, 512)  # D > 128
    assert not k.ctx_bmm_ok(4, 101, 100, 512)  # T % 8
    assert not k.ctx_bmm_ok(4, 400, 100, 320)  # A % 128
