"""Hand-written MFMA GEMM (csrc/kernels/gemm_mfma.hip) against an fp32 PyTorch matmul of the same
bf16 operands: plain rows (fp32 / bf16 out, bias, beta = 1 accumulate, partial row tiles, 128-wide
column tiles) and the encoder step-frame gather of its A rows (the embedding table by token id,
or the layer below's batch-frame output; the bw direction reversed within each length) -- the
rows to_step_frame used to write for the library GEMM."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _k():
    from textsummarization_on_flink_amd.ops import ops
    return ops()


def _close(got, ref, tol=2e-3):
    err = float((got.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
    assert err < tol, err


@pytest.mark.parametrize("M,N,K,out_bf16,bias,beta", [(1000, 512, 256, False, True, False),
                                                      (256, 256, 64, False, False, False),
                                                      (777, 384, 128, True, True, False),
                                                      (4096, 2048, 1024, False, False, True),
                                                      (300, 128, 192, True, False, False)])
def test_gemm_bt_plain_matches_fp32(M, N, K, out_bf16, bias, beta):
    k = _k()
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    Bt = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g) if bias else None
    c0 = torch.randn(M, N, device="cuda", generator=g)
    # the output is the head of a taller buffer: the rows after M must keep their sentinel (the
    # epilogue's row-range guard covers every store of a partial row tile)
    full = torch.full((M + 256, N), 12345.0, device="cuda", dtype=torch.bfloat16 if out_bf16 else torch.float32)
    out = full[:M]
    if beta:
        out.copy_(c0)
    else:
        out.fill_(float("nan"))
    k.gemm_bt(A, Bt, out, 1.0 if beta else 0.0, b, None, None, 0, 0, 0, None)
    torch.cuda.synchronize()
    ref = A.float() @ Bt.float().t() + (b if bias else 0) + (c0 if beta else 0)
    _close(out, ref, 1e-2 if out_bf16 else 2e-3)
    assert bool((full[M:] == 12345.0).all())


@pytest.mark.parametrize("ids", [True, False])
@pytest.mark.parametrize("direction", [0, 1])
def test_gemm_bt_step_frame_gather_matches_to_step_frame(ids, direction):
    """out[(t, b)] = src[row(b, tt)] . W with tt = t (fw) or rev[b][t] (bw) -- bit-identical to the
    library path's to_step_frame + GEMM operands (same bf16 rows), equal to fp32 within rounding."""
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    B, T, K, N, V = 48, 37, 128, 512, 3000
    g = torch.Generator(device="cuda").manual_seed(11 + direction)
    lens = torch.randint(1, T + 1, (B,), generator=g, device="cuda")
    t = torch.arange(T, device="cuda")
    rev = torch.where(t[None, :] < lens[:, None], lens[:, None] - 1 - t[None, :], t[None, :]).long().contiguous()
    if ids:
        src = torch.randn(V, K, device="cuda", generator=g).bfloat16()
        tok = torch.randint(0, V, (B, T), generator=g, device="cuda").long()
    else:
        src = torch.randn(B * T, K, device="cuda", generator=g).bfloat16()
        tok = None
    W = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).bfloat16()
    out = torch.full((T * B, N), float("nan"), device="cuda")
    xsf = torch.full((T * B, K), float("nan"), device="cuda").bfloat16()
    k.gemm_bt(src, W, out, 0.0, None, tok, rev, B, T, direction, xsf)
    torch.cuda.synchronize()
    tt = t[None, :].expand(B, T) if direction == 0 else rev
    rows = tok.gather(1, tt) if ids else torch.arange(B, device="cuda")[:, None] * T + tt
    A = src[rows.t().reshape(-1)]  # step frame: m = t * B + b
    ref = A.float() @ W.float().t()
    _close(out, ref)
    assert torch.equal(xsf, A)  # the step-frame copy of the gathered rows (what to_step_frame wrote)


@pytest.mark.parametrize("mode", [6, 2, 1])
def test_gemm_bt_merge_matches_two_direction_sum(mode):
    """AMODE 2: out[m] = [dz_fw row | dz_bw row] . [Kx_fw ; Kx_bw], the row of half h read at step t or
    rev[b][t] (mode bit h), m = t * B + b or b * T + t (bit 2) -- the per-direction GEMMs plus
    from_step_frame (mode 6) / step_frame_hop's two outputs (modes 2, 1) it replaces."""
    k = _k()
    B, T, Kh, N = 40, 29, 256, 128
    g = torch.Generator(device="cuda").manual_seed(100 + mode)
    lens = torch.randint(1, T + 1, (B,), generator=g, device="cuda")
    t = torch.arange(T, device="cuda")
    rev = torch.where(t[None, :] < lens[:, None], lens[:, None] - 1 - t[None, :], t[None, :]).long().contiguous()
    dz = torch.randn(2, T, B, Kh, device="cuda", generator=g).bfloat16()
    Bt = (torch.randn(N, 2 * Kh, device="cuda", generator=g) * Kh ** -0.5).bfloat16()
    full = torch.full((T * B + 64, N), 12345.0, device="cuda")
    out = full[:T * B]
    k.gemm_bt_merge(dz, Bt, out, rev, B, T, mode)
    torch.cuda.synchronize()
    bb = torch.arange(B, device="cuda")[:, None].expand(B, T)
    tt = t[None, :].expand(B, T)
    t0 = rev if mode & 1 else tt
    t1 = rev if mode & 2 else tt
    A = torch.cat([dz[0][t0, bb], dz[1][t1, bb]], -1)  # [B][T][2 Kh]: rows of output (b, t)
    ref = A.float() @ Bt.float().t()
    if not mode & 4:
        ref = ref.transpose(0, 1)  # step frame: m = t * B + b
    _close(out.view(ref.shape), ref)
    assert bool((full[T * B:] == 12345.0).all())


@pytest.mark.parametrize("K,M,N,acc", [(4096, 256, 256, False), (6400, 512, 384, False), (8192, 128, 512, False),
                                       (3200, 256, 1024, True), (64, 256, 128, False)])
def test_wgrad_tt_matches_fp32_and_is_deterministic(K, M, N, acc):
    """wgrad_tt (wgrad.hip): out (+)= a[K][M]^T . b[K][N] by 256 x BN MFMA tiles with the K range
    split over workgroups into fp32 slabs summed in split order -- against an fp32 matmul of the
    same bf16 operands; bit-identical on a repeat (no atomics); M = 128 runs with the operand
    roles swapped (transposed slab sum); the rows after the output keep their sentinel."""
    k = _k()
    g = torch.Generator(device="cuda").manual_seed(K + M + N)
    a = (torch.randn(K, M, device="cuda", generator=g) * 0.1).bfloat16()
    b = (torch.randn(K, N, device="cuda", generator=g) * 0.1).bfloat16()
    c0 = torch.randn(M, N, device="cuda", generator=g)
    full = torch.full((M + 64, N), 12345.0, device="cuda")
    out = full[:M]
    out.copy_(c0) if acc else out.fill_(float("nan"))
    ws = torch.empty(int(k.wgrad_tt_ws(M, N, K)), device="cuda")
    assert k.wgrad_tt(a, b, out, ws, acc)
    torch.cuda.synchronize()
    ref = a.float().t() @ b.float() + (c0 if acc else 0)
    _close(out, ref, 1e-4)
    assert bool((full[M:] == 12345.0).all())
    if not acc:
        again = torch.empty_like(out)
        k.wgrad_tt(a, b, again, ws, False)
        assert torch.equal(again, out)


def test_wgrad_tt_declines_unsupported_shapes():
    k = _k()
    a = torch.zeros(100, 96, device="cuda", dtype=torch.bfloat16)
    b = torch.zeros(100, 64, device="cuda", dtype=torch.bfloat16)
    assert int(k.wgrad_tt_ws(96, 64, 100)) == 0
    assert not k.wgrad_tt(a, b, torch.empty(96, 64, device="cuda"), torch.empty(1, device="cuda"), False)


@pytest.mark.parametrize("M,N", [(256, 256), (128, 512)])
def test_wgrad_tt_writes_an_unaligned_gradient_slice(M, N):
    """The output may be a slice of the flat gradient buffer at any 4-byte offset (the parameter
    offsets are not 16-byte aligned): the slab sum falls back to scalar stores there."""
    k = _k()
    K = 2048
    g = torch.Generator(device="cuda").manual_seed(M + N)
    a = (torch.randn(K, M, device="cuda", generator=g) * 0.1).bfloat16()
    b = (torch.randn(K, N, device="cuda", generator=g) * 0.1).bfloat16()
    flat = torch.full((M * N + 8,), 7.0, device="cuda")
    out = flat[1:1 + M * N].view(M, N)
    ws = torch.empty(int(k.wgrad_tt_ws(M, N, K)), device="cuda")
    assert k.wgrad_tt(a, b, out, ws, False)
    torch.cuda.synchronize()
    _close(out, a.float().t() @ b.float(), 1e-4)
    assert float(flat[0]) == 7.0 and bool((flat[1 + M * N:] == 7.0).all())


@pytest.mark.parametrize("M,N,K,acc", [(16000, 256, 50048, False), (1000, 512, 8192, True), (300, 128, 4096, False)])
def test_gemm_bt_splitk_matches_fp32_and_is_deterministic(M, N, K, acc):
    """Split-K gemm_bt (the vocab input gradient dX = dlogits . W^T, K = the padded vocabulary):
    S K-splits into fp32 slabs summed in split order -- against an fp32 matmul of the same bf16
    operands, bit-identical on a repeat, rows past M untouched; partial last row tile."""
    k = _k()
    n = int(k.gemm_bt_splitk_ws(M, N, K))
    assert n > 0, "the shape should split"
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = (torch.randn(M, K, device="cuda", generator=g) * 0.05).bfloat16()
    Bt = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    c0 = torch.randn(M, N, device="cuda", generator=g)
    full = torch.full((M + 16, N), 12345.0, device="cuda")
    out = full[:M]
    out.copy_(c0) if acc else out.fill_(float("nan"))
    ws = torch.empty(n, device="cuda")
    assert k.gemm_bt_splitk(A, Bt, out, ws, acc)
    torch.cuda.synchronize()
    ref = A.float() @ Bt.float().t() + (c0 if acc else 0)
    _close(out, ref, 1e-4)
    assert bool((full[M:] == 12345.0).all())
    if not acc:
        again = torch.empty_like(out)
        k.gemm_bt_splitk(A, Bt, again, ws, False)
        assert torch.equal(again, out)
    assert int(k.gemm_bt_splitk_ws(131072, 512, 4096)) == 0  # many tiles: no split, the caller's other path


@pytest.mark.parametrize("N,nv", [(1152, 1000), (32896, 32800)])
def test_wgrad_tt_narrow_output_drops_padding_columns(N, nv):
    """b wider than out (the padded dlogits rows, Vp = 128-aligned): out gets b's first nv columns
    only, through the slab sum (N = 1152: 9 tiles, split K) or stored straight into out (N =
    32896: 257 tiles, one split, no slab); the columns after it keep their sentinel."""
    k = _k()
    K, M = 2048, 256
    g = torch.Generator(device="cuda").manual_seed(3)
    a = (torch.randn(K, M, device="cuda", generator=g) * 0.1).bfloat16()
    b = (torch.randn(K, N, device="cuda", generator=g) * 0.1).bfloat16()
    full = torch.full((M, nv + 24), 7.0, device="cuda")
    out = full[:, :nv]
    ws = torch.empty(max(1, int(k.wgrad_tt_ws(M, N, K))), device="cuda")
    assert k.wgrad_tt(a, b, out, ws, False)
    torch.cuda.synchronize()
    _close(out, (a.float().t() @ b.float())[:, :nv], 1e-4)
    assert bool((full[:, nv:] == 7.0).all())
