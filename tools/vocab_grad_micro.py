"""Vocab-projection gradient GEMMs of the headline step (compact rows M = 16000 live decoder
rows, H = 256, V = 50k):

  dW[H][V] = X^T . dlogits      (K = M rows)
  dX[M][H] = dlogits . W^T      (K = V)

What ran in round 5/6 (dW: 4-way split-K torch.bmm + torch.sum; dX: hipBLASLt at K = 50000)
against the padded layout (dlogits rows and the bf16 W of Vp = 50048 = 391 x 128 columns, the
pad columns zero: the vocab head writes them) on the library and on the hand-written kernels
(dW: wgrad_tt, one split stored straight into the [H][V] gradient; dX: gemm_bt split-K + the
ordered slab sum).  HIP-event time per call and the error against an fp32 matmul of the same
bf16 operands; one JSON line.

  python tools/vocab_grad_micro.py [--M 16000 --H 256 --V 50000]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from textsummarization_on_flink_amd.ops import ops  # noqa: E402

F32, BF = torch.float32, torch.bfloat16


def timed(fn, it=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) * 1e3 / it, 1)


def rel(x, ref):
    return float((x - ref).norm() / ref.norm())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=16000)
    ap.add_argument("--H", type=int, default=256)
    ap.add_argument("--V", type=int, default=50000)
    a = ap.parse_args()
    k = ops()
    M, H, V = a.M, a.H, a.V
    Vp = -(-V // 128) * 128
    g = torch.Generator(device="cuda").manual_seed(0)
    x = (torch.randn(M, H + 8, device="cuda", generator=g) * 0.5).to(BF)  # outb rows (ld H + 8, as the model)
    dlp = torch.zeros(M, Vp, device="cuda", dtype=BF)
    dlp[:, :V] = (torch.randn(M, V, device="cuda", generator=g) * 1e-3).to(BF)
    owp = torch.zeros(H, Vp, device="cuda", dtype=BF)
    owp[:, :V] = (torch.randn(H, V, device="cuda", generator=g) * 0.05).to(BF)
    dl = dlp[:, :V].contiguous()
    ow = owp[:, :V].contiguous()
    xe = x[:, :H]
    r = dict(M=M, H=H, V=V, Vp=Vp, gflop_each=round(2 * M * H * V / 1e9, 1))
    refW = xe.float().t() @ dl.float()
    refX = dl.float() @ ow.float().t()
    dW = torch.empty(H, V, device="cuda", dtype=F32)
    dWp = torch.empty(H, Vp, device="cuda", dtype=F32)
    dX = torch.empty(M, H, device="cuda", dtype=F32)

    def dw_bmm():
        parts = torch.bmm(x.view(4, M // 4, H + 8)[:, :, :H].transpose(1, 2), dl.view(4, M // 4, V), out_dtype=F32)
        torch.sum(parts, 0, out=dW)
    if M % 4 == 0:
        r["dW_bmm4_sum_V"] = timed(dw_bmm)
    r["dW_blt_V"] = timed(lambda: k.blt_mm(xe, dl, dW, True, False, 0.0, None))
    r["dW_blt_Vp"] = timed(lambda: k.blt_mm(xe, dlp, dWp, True, False, 0.0, None))
    r["dW_blt_Vp_copy"] = timed(lambda: (k.blt_mm(xe, dlp, dWp, True, False, 0.0, None), dW.copy_(dWp[:, :V])))
    ws_n = int(k.wgrad_tt_ws(H, Vp, M))
    if ws_n:
        ws = torch.empty(ws_n, device="cuda", dtype=F32)
        dW.zero_()
        if k.wgrad_tt(xe, dlp, dW, ws, False):
            r["dW_wgrad_tt_Vp"] = timed(lambda: k.wgrad_tt(xe, dlp, dW, ws, False))
            r["dW_wgrad_tt_rel"] = rel(dW, refW)
            r["dW_wgrad_tt_ws_floats"] = ws_n
        else:
            r["dW_wgrad_tt_Vp"] = "declined"
    r["dX_blt_V"] = timed(lambda: k.blt_mm(dl, ow, dX, False, True, 0.0, None))
    r["dX_blt_Vp"] = timed(lambda: k.blt_mm(dlp, owp, dX, False, True, 0.0, None))
    r["dX_blt_Vp_rel"] = rel(dX, refX)
    ws_n = int(k.gemm_bt_splitk_ws(M, H, Vp))
    r["dX_splitk_ws_floats"] = ws_n
    if ws_n:
        ws2 = torch.empty(ws_n, device="cuda", dtype=F32)
        dX.zero_()
        if k.gemm_bt_splitk(dlp, owp, dX, ws2, False):
            r["dX_gemm_bt_splitk_Vp"] = timed(lambda: k.gemm_bt_splitk(dlp, owp, dX, ws2, False))
            r["dX_gemm_bt_splitk_rel"] = rel(dX, refX)
            d1 = dX.clone()
            k.gemm_bt_splitk(dlp, owp, dX, ws2, False)
            r["dX_gemm_bt_splitk_bitwise_repeat"] = bool(torch.equal(d1, dX))
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
