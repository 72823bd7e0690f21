"""Times the three batched context GEMMs of the pointer-generator step (library bmm) and
layout alternatives, one HIP-event time per op (median of 20).

  ctx = a . enc_out      [B][D,T] x [B][T,A]  (a stored [D][B][T])       forward
  da  = dctx . enc_out^T [B][D,A] x [B][A,T]  (dctx stored [D][B][A])    backward
  dE  = a^T . dctx       [B][T,D] x [B][D,A]                             backward

usage: python tools/ctx_bmm_micro.py [--B 256 --T 400 --D 100 --A 512]
"""
import argparse
import json

import torch

F32, BF = torch.float32, torch.bfloat16


def timed(fn, n=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--T", type=int, default=400)
    ap.add_argument("--D", type=int, default=100)
    ap.add_argument("--A", type=int, default=512)
    ap.add_argument("--native", action="store_true", help="also time the hand-written kernels")
    a = ap.parse_args()
    B, T, D, A = a.B, a.T, a.D, a.A
    dev = "cuda"
    att = torch.randn(D, B, T, device=dev).to(BF)
    enc = torch.randn(B, T, A, device=dev).to(BF)
    dctx = torch.randn(D, B, A, device=dev).to(BF)
    ctx = torch.empty(B, D, A, device=dev, dtype=F32)
    da = torch.empty(B, D, T, device=dev, dtype=F32)
    dE = torch.empty(B, T, A, device=dev, dtype=F32)
    att_c = att.transpose(0, 1).contiguous()
    dctx_c = dctx.transpose(0, 1).contiguous()
    r = dict(B=B, T=T, D=D, A=A)
    r["ctx_bmm"] = timed(lambda: torch.bmm(att.permute(1, 0, 2), enc, out_dtype=F32, out=ctx))
    r["ctx_bmm_contig_a"] = timed(lambda: torch.bmm(att_c, enc, out_dtype=F32, out=ctx))
    r["ctx_bmm_bf16_out"] = timed(lambda: torch.bmm(att_c, enc))
    r["da_bmm"] = timed(lambda: torch.bmm(dctx.permute(1, 0, 2), enc.transpose(1, 2), out_dtype=F32, out=da))
    r["da_bmm_contig"] = timed(lambda: torch.bmm(dctx_c, enc.transpose(1, 2), out_dtype=F32, out=da))
    r["dE_bmm"] = timed(lambda: torch.bmm(att.permute(1, 2, 0), dctx.permute(1, 0, 2), out_dtype=F32, out=dE))
    r["dE_bmm_contig"] = timed(lambda: torch.bmm(att_c.transpose(1, 2), dctx_c, out_dtype=F32, out=dE))
    mb = lambda n: n / 1e6  # noqa: E731
    r["bytes_MB"] = dict(enc=mb(enc.numel() * 2), att=mb(att.numel() * 2), ctx_f32=mb(ctx.numel() * 4),
                         da_f32=mb(da.numel() * 4), dE_f32=mb(dE.numel() * 4))
    if a.native:
        import sys
        import os
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from textsummarization_on_flink_amd.ops import load
        k = load()
        CTX = torch.empty(D, B, A, device=dev, dtype=F32)
        CTXb = torch.empty(D, B, A, device=dev, dtype=BF)
        dA = torch.zeros(D, B, T, device=dev, dtype=F32)
        tr = torch.empty(B * D * max(A, T), device=dev)
        r["ctx_bmm_tr01"] = timed(lambda: (torch.bmm(att.permute(1, 0, 2), enc, out_dtype=F32, out=ctx),
                                           k.tr01(ctx, CTX, CTXb, B, D, A, False)))
        r["da_bmm_tr01"] = timed(lambda: (torch.bmm(dctx.permute(1, 0, 2), enc.transpose(1, 2), out_dtype=F32, out=da),
                                          k.tr01(da, dA, None, B, D, T, True)))
        r["ctx_native"] = timed(lambda: k.ctx_fwd(att, enc, CTX, CTXb, B, T, D, A))
        r["da_native"] = timed(lambda: k.ctx_da(dctx, enc, dA, B, T, D, A, True))
        r["dE_native"] = timed(lambda: k.ctx_de(att, dctx, dE, B, T, D, A))
        dEb = torch.zeros(B, T, A, device=dev, dtype=BF)
        r["dE_native_bf16"] = timed(lambda: k.ctx_de(att, dctx, dEb, B, T, D, A))
        # the rest of dE: dF . W_h^T over B * T rows (fp32 beta = 1 after the fp32 dE, or bf16 out first)
        dF = (torch.randn(B * T, A, device=dev) * 0.01).to(BF)
        Wh = (torch.randn(A, A, device=dev) * 0.05).to(BF)
        r["dFWh_blt_f32_beta1"] = timed(lambda: k.blt_mm(dF, Wh, dE.view(B * T, A), False, True, 1.0, None))
        r["dFWh_blt_bf16"] = timed(lambda: k.blt_mm(dF, Wh, dEb.view(B * T, A), False, True, 0.0, None))
        r["dFWh_gemm_bt_bf16"] = timed(lambda: k.gemm_bt(dF, Wh, dEb.view(B * T, A), 0.0, None, None, None, 0, 0, 0, None))
        r["dFWh_blt_bf16_beta1"] = timed(lambda: k.blt_mm(dF, Wh, dEb.view(B * T, A), False, True, 1.0, None))
        del tr
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
