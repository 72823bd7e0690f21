"""The deterministic split-K weight-gradient GEMM (wgrad.hip wgrad_tt: 256 x 256 / 128 tiles,
LDS-DMA staged K-major operands read by ds_read_b64_tr_b16, fp32 slabs summed in split order)
vs the torch split-K path (pointer_generator.wgrad_into: bmm + torch.sum) and hipBLASLt (blt_mm)
at the encoder weight-gradient shapes: B = 256 (K = T.B = 102400) and config #5 at batch 2048
(K = 800 x 2048 = 1638400).  Error vs fp32 and HIP-event time per call; one JSON line per shape.

  python tools/wgrad_tt_micro.py [--quick]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from textsummarization_on_flink_amd.models import pointer_generator as pgm  # noqa: E402
from textsummarization_on_flink_amd.ops import ops  # noqa: E402


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


def main():
    k = ops()
    quick = "--quick" in sys.argv
    g = torch.Generator(device="cuda").manual_seed(0)
    shapes = [("enc_x_b256", 102400, 128, 1024), ("enc_h_b256", 102400, 256, 1024),
              ("enc_x_l0_c5", 1638400, 128, 2048), ("enc_x_l1_c5", 1638400, 1024, 2048), ("enc_h_c5", 1638400, 512, 2048)]
    if quick:
        shapes = shapes[:2] + [("enc_h_c5q", 409600, 512, 2048)]
    for name, K, M, N in shapes:
        a = (torch.randn(K, M, device="cuda", generator=g) * 0.1).bfloat16()
        b = (torch.randn(K, N, device="cuda", generator=g) * 0.1).bfloat16()
        ref = a.float().t() @ b.float()
        ws = torch.empty(int(k.wgrad_tt_ws(M, N, K)), device="cuda")
        out = torch.full((M, N), float("nan"), device="cuda")
        assert k.wgrad_tt(a, b, out, ws, False)
        err = float((out - ref).abs().max() / ref.abs().max())
        out2 = torch.empty(M, N, device="cuda")
        pgm.wgrad_into(out2, a, b)
        err_lib = float((out2 - ref).abs().max() / ref.abs().max())
        out3 = out.clone()
        k.wgrad_tt(a, b, out3, ws, False)
        flop = 2.0 * K * M * N
        t_tt = timed(lambda: k.wgrad_tt(a, b, out, ws, False))
        t_lib = timed(lambda: pgm.wgrad_into(out2, a, b))
        t_blt = timed(lambda: k.blt_mm(a, b, out2, True, False, 0.0, None))
        print(json.dumps({"shape": name, "K": K, "M": M, "N": N, "err": err, "err_split_k": err_lib,
                          "bitwise_repeat": bool(torch.equal(out, out3)), "ws_mb": round(ws.numel() * 4 / 2 ** 20, 1),
                          "wgrad_tt_us": t_tt, "wgrad_tt_TF": round(flop / t_tt / 1e6, 1),
                          "split_k_us": t_lib, "split_k_TF": round(flop / t_lib / 1e6, 1),
                          "blt_mm_us": t_blt, "blt_mm_TF": round(flop / t_blt / 1e6, 1)}), flush=True)
        del a, b, ref, ws, out, out2, out3
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
