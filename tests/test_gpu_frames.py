"""Layout / reduction helper kernels of csrc/kernels/frames.hip against plain PyTorch:
to_step_frame (embedding gather into the [2][T][B][W] step frame, bw direction reversed per
length), from_step_frame (fw + reversed bw input gradients), transpose_bta (W_h feature
transpose) and cast_colsum (bf16 copy + bias-gradient column sums)."""
import pytest
import torch

from textsummarization_on_flink_amd.ops import ops

pytestmark = pytest.mark.gpu


def _rev(lens, T):
    t = torch.arange(T).view(1, T).expand(len(lens), T)
    L = lens.view(-1, 1)
    return torch.where(t < L, L - 1 - t, t).contiguous()


@pytest.mark.parametrize("B,T,W", [(5, 7, 16), (16, 33, 128)])
def test_to_and_from_step_frame(B, T, W):
    k = ops()
    g = torch.Generator().manual_seed(B + T)
    lens = torch.randint(1, T + 1, (B,), generator=g)
    lens[0] = T
    rev = _rev(lens, T)
    V = 50
    emb = torch.randn(V, W, generator=g).to(torch.bfloat16)
    ids = torch.randint(0, V, (B, T), generator=g)
    out = torch.empty(2, T, B, W, dtype=torch.bfloat16, device="cuda")
    k.to_step_frame(emb.cuda(), ids.cuda(), rev.cuda(), out, B, T, W, 0)
    fw = emb[ids].permute(1, 0, 2)                                  # [T][B][W]
    bw = emb[torch.gather(ids, 1, rev)].permute(1, 0, 2)
    torch.testing.assert_close(out.cpu(), torch.stack([fw, bw]), rtol=0, atol=0)
    # doff: the bw direction reads columns doff.. of a [B, T, 2W] source
    src = torch.randn(B, T, 2 * W, generator=g)
    out2 = torch.empty(2, T, B, W, device="cuda")
    k.to_step_frame(src.cuda(), None, rev.cuda(), out2, B, T, W, W)
    ref_bw = torch.gather(src[:, :, W:], 1, rev.unsqueeze(-1).expand(B, T, W)).permute(1, 0, 2)
    torch.testing.assert_close(out2.cpu(), torch.stack([src[:, :, :W].permute(1, 0, 2), ref_bw]), rtol=0, atol=0)
    # from_step_frame: out[b][t] = in[0][t][b] + in[1][rev[b][t]][b]
    x = torch.randn(2, T, B, W, generator=g)
    o = torch.empty(B, T, W, device="cuda")
    k.from_step_frame(x.cuda(), rev.cuda(), o, B, T, W)
    ref = x[0].permute(1, 0, 2) + torch.gather(x[1].permute(1, 0, 2), 1, rev.unsqueeze(-1).expand(B, T, W))
    torch.testing.assert_close(o.cpu(), ref, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("B,T,A", [(2, 64, 64), (3, 101, 128)])
def test_transpose_bta(B, T, A):
    k = ops()
    x = torch.randn(B, T, A, generator=torch.Generator().manual_seed(T)).to(torch.bfloat16).cuda()
    y = torch.empty(B, A, T, dtype=torch.bfloat16, device="cuda")
    k.transpose_bta(x, y, B, T, A)
    torch.testing.assert_close(y, x.transpose(1, 2), rtol=0, atol=0)


@pytest.mark.parametrize("N,C", [(1, 4), (37, 128), (25600, 256), (999, 512), (100, 1024)])
def test_cast_colsum(N, C):
    k = ops()
    x = torch.randn(N, C, generator=torch.Generator().manual_seed(N + C)).cuda()
    xb = torch.empty(N, C, dtype=torch.bfloat16, device="cuda")
    cs = torch.full((C,), 0.5, device="cuda")  # accumulates onto what is there
    k.cast_colsum(x, xb, cs, N, C)
    torch.testing.assert_close(xb, x.to(torch.bfloat16), rtol=0, atol=0)
    ref = x.double().sum(0) + 0.5
    torch.testing.assert_close(cs.double(), ref, rtol=1e-5, atol=1e-4 * (N ** 0.5))


@pytest.mark.parametrize("N,C,bf", [(25600, 1, False), (1, 3, False), (102400, 1024, True), (25600, 1024, True),
                                    (25600, 50000, True), (999, 130, False), (256, 256, False), (37, 514, True)])
def test_colsum_deterministic_matches_fp64(N, C, bf):
    """colsum (frames.hip): column sums of a tall fp32 / bf16 matrix in an order fixed by (N, C) --
    the deterministic replacement of torch sum(0) for the bias gradients -- vs an fp64 sum; two
    runs give the same bits; acc adds onto the output."""
    k = ops()
    g = torch.Generator(device="cuda").manual_seed(N + C)
    x = torch.randn(N, C, device="cuda", generator=g)
    if bf:
        x = x.bfloat16()
    out = torch.empty(C, device="cuda")
    k.colsum(x, out, N, C, False)
    ref = x.double().sum(0)
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=2e-5 * (N ** 0.5))
    again = torch.full((C,), 0.25, device="cuda")
    for _ in range(3):
        o2 = torch.empty(C, device="cuda")
        k.colsum(x, o2, N, C, False)
        assert torch.equal(o2.view(torch.int32), out.view(torch.int32))
    k.colsum(x, again, N, C, True)
    torch.testing.assert_close(again.double(), ref + 0.25, rtol=1e-5, atol=2e-5 * (N ** 0.5))


@pytest.mark.parametrize("K,M,N,strided", [(1000, 128, 128, False), (25600, 256, 512, False), (3001, 128, 256, True),
                                           (130, 512, 128, True), (25600, 256, 5000, False), (3001, 256, 200, True)])
def test_wgrad_tn_matches_fp32(K, M, N, strided):
    """wgrad.hip: out[M][N] += a[K][M]^T b[K][N] (split-K MFMA, transposed LDS reads, fp32
    atomics) vs an fp32 matmul, including K not a multiple of the k-step, N not a multiple of
    the 128-column tile (the vocab dW shape: M = 256, N = V), row-strided operand views and an
    output slice of a wider matrix."""
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    g = torch.Generator(device="cuda").manual_seed(K + M)
    pad = 8 if strided else 0
    a = (torch.randn(K, M + pad, device="cuda", generator=g) * 0.2).bfloat16()[:, :M]
    b = (torch.randn(K, N + pad, device="cuda", generator=g) * 0.2).bfloat16()[:, :N]
    big = torch.zeros(M, N + 2 * pad, device="cuda")
    out = big[:, pad:pad + N] if strided else big[:, :N]
    k.wgrad_tn(a, b, out)
    ref = a.float().t() @ b.float()
    err = float((out - ref).abs().max() / ref.abs().max())
    assert err < 1e-4, err
    if strided:  # nothing written outside the slice
        assert float(big[:, :pad].abs().max()) == 0 and float(big[:, pad + N:].abs().max()) == 0


@pytest.mark.parametrize("B,T,H", [(5, 7, 16), (16, 33, 64)])
def test_step_frame_hop_equals_from_then_to_step_frame(B, T, H):
    """step_frame_hop (upper layer's step-frame input gradients straight into the lower layer's
    output-gradient step frame) == from_step_frame followed by to_step_frame (doff = H), bit for bit."""
    k = ops()
    g = torch.Generator().manual_seed(B * T + H)
    lens = torch.randint(1, T + 1, (B,), generator=g)
    lens[0] = T
    rev = _rev(lens, T).cuda()
    dxs = torch.randn(2, T * B, 2 * H, generator=g).cuda()
    dx = torch.empty(B, T, 2 * H, device="cuda")
    k.from_step_frame(dxs, rev, dx, B, T, 2 * H)
    ref = torch.empty(B, T, 2 * H, device="cuda")  # [2][T][B][H] in the engine's dout buffer
    k.to_step_frame(dx, None, rev, ref, B, T, H, H)
    out = torch.full((B, T, 2 * H), float("nan"), device="cuda")
    k.step_frame_hop(dxs, rev, out, B, T, H)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("P,Q,R", [(6, 5, 512), (3, 7, 12), (256, 100, 400)])
def test_tr01_transposes_casts_and_accumulates(P, Q, R):
    """tr01: fp32 [P][Q][R] -> [Q][P][R] (copy or accumulate) and the bf16 twin in one pass."""
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    g = torch.Generator(device="cuda").manual_seed(P + Q + R)
    x = torch.randn(P, Q, R, device="cuda", generator=g)
    out = torch.full((Q, P, R), float("nan"), device="cuda")
    outb = torch.full((Q, P, R), float("nan"), device="cuda", dtype=torch.bfloat16)
    k.tr01(x, out, outb, P, Q, R, False)
    torch.cuda.synchronize()
    assert torch.equal(out, x.transpose(0, 1))
    assert torch.equal(outb, x.transpose(0, 1).bfloat16())
    base = torch.randn(Q, P, R, device="cuda", generator=g)
    acc = base.clone()
    k.tr01(x, acc, None, P, Q, R, True)
    torch.cuda.synchronize()
    assert torch.equal(acc, base + x.transpose(0, 1))
