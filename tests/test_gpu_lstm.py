"""Persistent weight-resident LSTM (one launch, granule hand-offs) vs the per-step kernels:
same layouts, same TF LSTMCell semantics (variable lengths, frozen rows, step frame)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(H, B, T, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    r = lambda *s, sc=1.0: (torch.randn(*s, device="cuda", generator=g) * sc)
    lens = torch.randint(1, T + 1, (B,), device="cuda", generator=g, dtype=torch.int32)
    lens[0] = T
    lens[-1] = 1
    gx = r(2, T, B, 4 * H, sc=0.5)
    W = r(2, 4 * H, H, sc=1.0 / H ** 0.5).bfloat16()          # Wt [2][4H][H]
    Wn = W.transpose(1, 2).contiguous()                        # [2][H][4H]
    hs = torch.zeros(2, T + 1, B, H, device="cuda", dtype=torch.bfloat16)
    cs = torch.zeros(2, T + 1, B, H, device="cuda")
    hs[:, 0] = r(2, B, H, sc=0.3).bfloat16()
    cs[:, 0] = r(2, B, H, sc=0.3)
    return g, r, lens, gx, W.contiguous(), Wn, hs, cs


# (512, <= 256): the 8-wave forward and 16-row BPTT; (512, > 256): the 4-wave 32-row-team forward
# (RT = 2) and the 16-wave 32-row-team BPTT (one launch at 300, a partial last tile);
# (256, 600), (512, 600) and (512, 1100):
# more row tiles than one resident grid holds -> consecutive launches over row-tile ranges
@pytest.mark.parametrize("H,B,T", [(64, 16, 9), (128, 37, 20), (256, 64, 33), (256, 200, 12), (256, 600, 7),
                                   (256, 40, 25), (128, 30, 11), (512, 40, 21), (512, 64, 200), (512, 300, 9),
                                   (512, 600, 6), (512, 1100, 5)])
def test_persistent_matches_step_kernels(H, B, T):
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    assert int(k.lstm_persistent_grid(H, B)) > 0
    if (H, B) in ((256, 600), (512, 600), (512, 1100)):
        assert int(k.lstm_persistent_launches(H, B)) > 1
    g, r, lens, gx, Wt, Wn, hs0, cs0 = _setup(H, B, T, 7 + H + B)
    bias = torch.randn(2, 4 * H, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5)) * 0.2
    res = {}
    for mode in ("step", "persistent"):
        hs, cs = hs0.clone(), cs0.clone()
        acts = torch.zeros(2, T, B, 4 * H, device="cuda")
        # the persistent kernels write every position of out (zeros past the length): start from NaN
        out = torch.full((B, T, 2 * H), 0.0 if mode == "step" else float("nan"), device="cuda", dtype=torch.bfloat16)
        err = torch.zeros(1, device="cuda", dtype=torch.int32)
        if mode == "step":
            for s in range(T):
                k.lstm_enc_fwd_step(gx, bias, Wt, hs, cs, acts, out, lens, s, T, B, H)
        else:
            xf = torch.zeros(int(k.lstm_persistent_xbuf(H, B, False)), device="cuda", dtype=torch.long)
            k.lstm_fwd_persistent(gx, bias, Wt, hs, cs, acts, out, lens, xf, err, T, B, H)
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        # backward on the forward's own activations
        gb = torch.Generator(device="cuda").manual_seed(99)
        dout = torch.randn(2, T, B, H, device="cuda", generator=gb) * 0.1
        dh_fin = torch.randn(2, B, H, device="cuda", generator=gb) * 0.1
        dcc = torch.randn(2, B, H, device="cuda", generator=gb) * 0.1
        dz = torch.zeros(2, T, B, 4 * H, device="cuda", dtype=torch.bfloat16)
        if mode == "step":
            for s in reversed(range(T)):
                k.lstm_enc_bwd_step(dz, Wn, dout, dh_fin, dcc, acts, cs, lens, s, T, B, H)
        else:
            xb = torch.zeros(int(k.lstm_persistent_xbuf(H, B, True)), device="cuda", dtype=torch.long)
            db = torch.full((2, 4 * H), 0.25, device="cuda")  # accumulates onto what is there
            dcc0 = dcc.clone()
            dcc_init = dcc.clone()
            k.lstm_bwd_persistent(dz, Wn, dout, dh_fin, dcc, acts, cs, lens, xb, err, db, T, B, H, False)
            # the same gradient in the BATCH frame ([B][T][2H], bw half at the reversed position), read
            # by the kernel directly (what the top layer's to_step_frame pass used to rebuild): same bits
            t = torch.arange(T, device="cuda")
            ln = lens.long()[:, None]
            rev = torch.where(t[None, :] < ln, ln - 1 - t[None, :], t[None, :])
            dE = torch.cat([dout[0].transpose(0, 1),
                            dout[1].transpose(0, 1)[torch.arange(B, device="cuda")[:, None], rev]], -1).contiguous()
            dz2 = torch.zeros_like(dz)
            xb.zero_()
            k.lstm_bwd_persistent(dz2, Wn, dE, dh_fin, dcc0, acts, cs, lens, xb, err, None, T, B, H, True)
            torch.cuda.synchronize()
            assert torch.equal(dz2, dz) and torch.equal(dcc0, dcc)
            # the batch-frame gradient in bf16 (the engine's bf16 dE): the same bits as the fp32 read
            # of the same rounded values
            dEb = dE.bfloat16()
            outs = []
            for src in (dEb, dEb.float()):
                dzx, dcx = torch.zeros_like(dz), dcc_init.clone()
                xb.zero_()
                k.lstm_bwd_persistent(dzx, Wn, src, dh_fin, dcx, acts, cs, lens, xb, err, None, T, B, H, True)
                outs.append((dzx, dcx))
            torch.cuda.synchronize()
            assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        if mode != "step":
            # gate-bias gradient from the kernel's fp32 register sums vs the column sum of the
            # bf16 dz it wrote (each term rounded to bf16: ~1e-3 relative)
            ref = dz.float().sum(dim=(1, 2)) + 0.25
            torch.testing.assert_close(db, ref, rtol=2e-2, atol=1e-2 * float(ref.abs().max()))
        res[mode] = dict(hs=hs.float(), cs=cs, acts=acts, out=out.float(), dz=dz.float(), dc=dcc)
    a, b = res["step"], res["persistent"]
    for name, tol in [("hs", 3e-2), ("cs", 3e-2), ("acts", 2e-2), ("out", 3e-2), ("dz", 3e-2), ("dc", 3e-2)]:
        diff = (a[name] - b[name]).abs()
        assert diff.max().item() < tol, (name, diff.max().item())
        assert diff.mean().item() < 2e-3, (name, diff.mean().item())
    # frozen rows: final state equals the state at their length
    L = int(lens[-1])
    assert torch.equal(res["persistent"]["hs"][:, T, -1], res["persistent"]["hs"][:, L, -1])


def test_persistent_repeated_launches_reset_tags():
    """Graph-style replays: the hand-off buffer is zeroed before every launch, so a second
    launch on the same buffers gives identical results."""
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    H, B, T = 256, 48, 17
    g, r, lens, gx, Wt, Wn, hs0, cs0 = _setup(H, B, T, 3)
    xf = torch.zeros(int(k.lstm_persistent_xbuf(H, B, False)), device="cuda", dtype=torch.long)
    err = torch.zeros(1, device="cuda", dtype=torch.int32)
    bias = torch.zeros(2, 4 * H, device="cuda")
    outs = []
    for _ in range(3):
        hs, cs = hs0.clone(), cs0.clone()
        acts = torch.zeros(2, T, B, 4 * H, device="cuda")
        out = torch.zeros(B, T, 2 * H, device="cuda", dtype=torch.bfloat16)
        xf.zero_()
        k.lstm_fwd_persistent(gx, bias, Wt, hs, cs, acts, out, lens, xf, err, T, B, H)
        outs.append(out.clone())
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])


def test_persistent_lstm_with_concurrent_kernels():
    """Co-residency under concurrent work (the data-parallel case: RCCL kernels of an earlier
    gradient bucket run beside the BPTT).  The persistent launches need all their workgroups
    resident; a long GEMM stream on a second HIP stream holds CUs while they start, so early
    team members spin until the others get CUs.  Results must equal the solo launches and no
    hand-off may time out (lstm_err stays 0)."""
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    H, B, T = 256, 256, 40
    g, r, lens, gx, Wt, Wn, hs0, cs0 = _setup(H, B, T, 11)
    bias = torch.zeros(2, 4 * H, device="cuda")
    xf = torch.zeros(int(k.lstm_persistent_xbuf(H, B, False)), device="cuda", dtype=torch.long)
    xb = torch.zeros(int(k.lstm_persistent_xbuf(H, B, True)), device="cuda", dtype=torch.long)
    err = torch.zeros(1, device="cuda", dtype=torch.int32)
    dout = torch.randn(2, T, B, H, device="cuda", generator=g) * 0.1
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)

    def run(side_load):
        hs, cs = hs0.clone(), cs0.clone()
        acts = torch.zeros(2, T, B, 4 * H, device="cuda")
        out = torch.zeros(B, T, 2 * H, device="cuda", dtype=torch.bfloat16)
        dz = torch.zeros(2, T, B, 4 * H, device="cuda", dtype=torch.bfloat16)
        dcc = torch.zeros(2, B, H, device="cuda")
        dhf = torch.zeros(2, B, H, device="cuda")
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        if side_load:
            with torch.cuda.stream(side):
                for _ in range(30):  # ~ms of GEMMs occupying every CU while the LSTM launches start
                    a @ a
        xf.zero_()
        k.lstm_fwd_persistent(gx, bias, Wt, hs, cs, acts, out, lens, xf, err, T, B, H)
        if side_load:
            with torch.cuda.stream(side):
                for _ in range(30):
                    a @ a
        xb.zero_()
        k.lstm_bwd_persistent(dz, Wn, dout, dhf, dcc, acts, cs, lens, xb, err, None, T, B, H, False)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        return out.clone(), dz.clone()

    solo = run(False)
    busy = run(True)
    assert int(err.item()) == 0
    assert torch.equal(solo[0], busy[0]) and torch.equal(solo[1], busy[1])


@pytest.mark.parametrize("H,B", [(256, 512), (512, 256)])
def test_persistent_lstm_stress_full_grid(H, B):
    """Stress of the inter-workgroup hand-off: 40 back-to-back forward + BPTT
    launches at a grid that fills the chip (B = 512 at H = 256: 256 workgroups, one per CU;
    H = 512: 8-wave teams), each bit-identical to the first and without a hand-off timeout.
    A stale read of a peer's granule (XCD-local L2 coherence, tag reuse across launches)
    would show up as a differing launch."""
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    T = 48
    assert int(k.lstm_persistent_grid(H, B)) > 0
    g, r, lens, gx, Wt, Wn, hs0, cs0 = _setup(H, B, T, 21 + H)
    bias = torch.randn(2, 4 * H, device="cuda", generator=g) * 0.1
    xf = torch.zeros(int(k.lstm_persistent_xbuf(H, B, False)), device="cuda", dtype=torch.long)
    xb = torch.zeros(int(k.lstm_persistent_xbuf(H, B, True)), device="cuda", dtype=torch.long)
    err = torch.zeros(1, device="cuda", dtype=torch.int32)
    dout = torch.randn(2, T, B, H, device="cuda", generator=g) * 0.1
    hs, cs = hs0.clone(), cs0.clone()
    acts = torch.zeros(2, T, B, 4 * H, device="cuda")
    out = torch.zeros(B, T, 2 * H, device="cuda", dtype=torch.bfloat16)
    dz = torch.zeros(2, T, B, 4 * H, device="cuda", dtype=torch.bfloat16)
    dcc = torch.zeros(2, B, H, device="cuda")
    dhf = torch.zeros(2, B, H, device="cuda")
    ref = None
    for it in range(40):
        hs.copy_(hs0)
        cs.copy_(cs0)
        xf.zero_()
        k.lstm_fwd_persistent(gx, bias, Wt, hs, cs, acts, out, lens, xf, err, T, B, H)
        dcc.zero_()
        dhf.zero_()
        xb.zero_()
        k.lstm_bwd_persistent(dz, Wn, dout, dhf, dcc, acts, cs, lens, xb, err, None, T, B, H, False)
        if ref is None:
            ref = (out.clone(), dz.clone(), dcc.clone())
        elif it % 8 == 0 or it == 39:
            torch.cuda.synchronize()
            assert torch.equal(out, ref[0]) and torch.equal(dz, ref[1]) and torch.equal(dcc, ref[2]), it
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    assert torch.equal(out, ref[0]) and torch.equal(dz, ref[1])


# The input projection inside the recurrence (FX, encoder layer 0, E = 128) against the same
# recurrence fed gx = x . W_x from an fp32 matmul: 4-wave H <= 256 kernels (W_x in registers),
# the H = 512 32-row-team kernel (W_x / x staged in LDS, single-buffered h tile), several
# launches over row-tile ranges (256, 600), and a partial last tile (512, 300).
@pytest.mark.parametrize("H,B,T", [(64, 16, 9), (128, 37, 20), (256, 64, 33), (256, 600, 7), (512, 300, 9),
                                   (512, 512, 40)])
def test_persistent_input_projection_matches_gx_path(H, B, T):
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    E = 128
    assert bool(k.lstm_persistent_fx_ok(H, B, E))
    g, r, lens, _, Wt, _, hs0, cs0 = _setup(H, B, T, 11 + H + B)
    xsf = r(2, T, B, E, sc=0.5).bfloat16()
    WxT = r(2, 4 * H, E, sc=1.0 / E ** 0.5).bfloat16()           # [d][u * 4 + g][E]
    bias = torch.randn(2, 4 * H, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5)) * 0.2
    gx = torch.stack([xsf[d].float().reshape(T * B, E) @ WxT[d].float().t() for d in range(2)]).view(2, T, B, 4 * H)
    res = {}
    for mode in ("gx", "fx"):
        hs, cs = hs0.clone(), cs0.clone()
        acts = torch.full((2, T, B, 4 * H), float("nan"), device="cuda")
        out = torch.full((B, T, 2 * H), float("nan"), device="cuda", dtype=torch.bfloat16)
        err = torch.zeros(1, device="cuda", dtype=torch.int32)
        xf = torch.zeros(int(k.lstm_persistent_xbuf(H, B, False)), device="cuda", dtype=torch.long)
        if mode == "gx":
            k.lstm_fwd_persistent(gx, bias, Wt, hs, cs, acts, out, lens, xf, err, T, B, H)
        else:
            k.lstm_fwd_persistent_fx(xsf, WxT[0].contiguous(), WxT[1].contiguous(), bias, Wt, hs, cs, acts, out, lens,
                                     xf, err, T, B, H)
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        res[mode] = (hs, cs, acts, out)
    t = torch.arange(T, device="cuda")
    live = (t[None, :] < lens.long()[:, None]).t()                # [T][B]
    for name, a, b in zip(("hs", "cs"), res["gx"][:2], res["fx"][:2]):
        torch.testing.assert_close(b.float(), a.float(), rtol=2e-2, atol=2e-2, msg=name)
    ag, af = res["gx"][2], res["fx"][2]
    m = live[None, :, :, None].expand_as(ag)
    torch.testing.assert_close(af[m], ag[m], rtol=1e-2, atol=1e-2)
    assert not torch.isnan(res["fx"][3]).any()                    # every out position written
    torch.testing.assert_close(res["fx"][3].float(), res["gx"][3].float(), rtol=2e-2, atol=2e-2)
