"""Attention kernels at a chosen shape with random operands, cold or warm in the caches.

The row kernels stream F and E ([rows, T, A] bf16) once per launch; whether those bytes come
from HBM or from the 256 MB MALL decides the time.  NG > 1 cycles the launches over NG
disjoint row groups (NG * rows * T * A * 4 bytes apart), as the training step does at
batch NG * rows; NG = 1 re-reads one group (warm).  A plain reduction over the same bytes
(torch.sum of F and E) gives the streaming reference.

  MB=256 T=800 A=1024 NG=4 python tools/attn_micro_c5.py     (config #5, one row group)
  MB=256 T=400 A=512  NG=1 python tools/attn_micro_c5.py     (bench default, warm)
(FEAT=0 skips the post-loop feature-gradient pass, D decoder steps, timed in ms.)
Prints one JSON line: microseconds per launch and the effective GB/s of F + E.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, n, it=30):
    for i in range(2 * n):
        fn(i % n)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for i in range(it):
        fn(i % n)
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) * 1e3 / it, 2)


def main():
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    MB, T, A, NG = (int(os.environ.get(x, d)) for x, d in (("MB", "256"), ("T", "800"), ("A", "1024"), ("NG", "4")))
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    F = (torch.randn(NG, MB, T, A, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    E = (torch.randn(NG, MB, T, A, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    s = torch.randn(MB, A, device=dev, generator=g) * 0.5
    v = torch.randn(A, device=dev, generator=g) * 0.05
    wc = torch.randn(A, device=dev, generator=g) * 0.05
    cov = torch.rand(MB, T, device=dev, generator=g)
    lens = torch.full((MB,), T, dtype=torch.int32, device=dev)
    att = torch.softmax(torch.randn(MB, T, device=dev, generator=g), 1)
    cov_out, covloss = torch.empty_like(cov), torch.empty(MB, device=dev)
    ctx, ctxb = torch.empty(MB, A, device=dev), torch.empty(MB, A, device=dev, dtype=torch.bfloat16)
    dctx, ga = torch.randn(MB, A, device=dev, generator=g) * 0.1, torch.randn(MB, T, device=dev, generator=g) * 0.1
    dcn, gcl = torch.randn(MB, T, device=dev, generator=g) * 0.1, torch.rand(MB, device=dev)
    de, ds, dco = torch.empty(MB, T, device=dev), torch.empty(MB, A, device=dev), torch.empty(MB, T, device=dev)
    gb = NG * MB * T * A * 4 / 1e9 / NG  # bytes of F + E per launch, GB
    res = {"MB": MB, "T": T, "A": A, "NG": NG, "MB_FE": round(gb * 1e3, 1),
           "env": {x: os.environ[x] for x in os.environ if x.startswith("TSAMD_")}}

    def bw(us):
        return round(gb / (us * 1e-6), 1)

    out = torch.empty(MB, device=dev)
    res["sum_FE"] = timeit(lambda i: (torch.sum(F[i].view(MB, -1), 1, dtype=torch.float32, out=out),
                                      torch.sum(E[i].view(MB, -1), 1, dtype=torch.float32, out=out)), NG)
    if k.attn_row_ok(A, T):
        res["fwd_row"] = timeit(lambda i: k.attn_fwd_row(F[i], E[i], s, v, wc, cov, lens, att, cov_out, covloss, ctx,
                                                         ctxb, MB, T, A, 1), NG)
        res["bwd_row"] = timeit(lambda i: k.attn_bwd_row(E[i], F[i], s, v, wc, cov, att, dctx, ctx, ga, dcn, gcl, lens,
                                                         de, ds, dco, MB, T, A), NG)
    if k.attn_rowp_ok(A, T, 128):  # projected context: F and G = enc_out . W_in[E:] (128 wide)
        Gp = (torch.randn(NG, MB, T, 128, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        gx, gxb = torch.empty(MB, 128, device=dev), torch.empty(MB, 128, device=dev, dtype=torch.bfloat16)
        dxp = torch.randn(MB, 128, device=dev, generator=g) * 0.1
        res["fwd_rowp"] = timeit(lambda i: k.attn_fwd_rowp(F[i], Gp[i], s, v, wc, cov, lens, att, cov_out, covloss, gx,
                                                           gxb, MB, T, A, None, 0, None), NG)
        res["bwd_rowp"] = timeit(lambda i: k.attn_bwd_rowp(Gp[i], F[i], s, v, wc, cov, att, dxp, gx, ga, dcn, gcl, lens,
                                                           de, ds, dco, MB, T, A, None, 0), NG)
        gbp = MB * T * (A + 128) * 2 / 1e9  # F + G bytes per launch
        for key in ("fwd_rowp", "bwd_rowp"):
            res[key + "_GBs"] = round(gbp / (res[key] * 1e-6), 1)
    res["bwd_step"] = timeit(lambda i: (ds.zero_(), k.attn_bwd_step(E[i], F[i], s, v, wc, cov, att, dctx, ctx, ga, dcn,
                                                                    gcl, lens, de, ds, dco, MB, T, A)), NG)
    if os.environ.get("FEAT", "1") == "1":  # the post-loop dF / dv / dwc pass over D decoder steps
        D = int(os.environ.get("D", "100"))
        S_all = torch.randn(D, MB, A, device=dev, generator=g) * 0.5
        cov_all = torch.rand(D, MB, T, device=dev, generator=g)
        de_all = torch.randn(D, MB, T, device=dev, generator=g) * 0.01
        dF = torch.empty(MB, T, A, device=dev, dtype=torch.bfloat16)
        dv, dwc = torch.zeros(64, A, device=dev), torch.zeros(64, A, device=dev)
        res["bwd_feat_ms"] = round(timeit(lambda i: k.attn_bwd_feat(F[i], S_all, v, wc, cov_all, de_all, lens, dF, dv,
                                                                     dwc, D, MB, T, A, None), NG, it=3) / 1e3, 3)
    for key in ("sum_FE", "fwd_row", "bwd_row", "bwd_step"):
        if key in res:
            res[key + "_GBs"] = bw(res[key])
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
