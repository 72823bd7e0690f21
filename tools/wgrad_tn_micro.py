"""The custom weight-gradient kernel (wgrad.hip: split-K MFMA, LDS transposed reads, fp32
atomics, no inter-workgroup waits) vs the library split-K path (pointer_generator.wgrad_into)
at the training step's weight-gradient shapes (B=256, D=100, T=400): error vs fp32 and
HIP-event time per call.  Prints one JSON line per shape.

  python tools/wgrad_tn_micro.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from textsummarization_on_flink_amd.models.pointer_generator import wgrad_into  # noqa: E402
from textsummarization_on_flink_amd.ops import ops  # noqa: E402


def timed(fn, it=20):
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
    g = torch.Generator(device="cuda").manual_seed(0)
    shapes = [("out_proj_h", 25600, 256, 256), ("out_proj_ctx", 25600, 512, 256), ("cell_x", 25600, 128, 1024),
              ("cell_h", 25600, 256, 1024), ("lin_ctx", 25344, 512, 128), ("att_c", 25600, 256, 512),
              ("W_h", 102400, 512, 512),
              # encoder weight gradients x^T.dz / h^T.dz: B = 256 (K = T.B = 102400) and config #5 (819200)
              ("enc_x_b256", 102400, 128, 1024), ("enc_h_b256", 102400, 256, 1024),
              ("enc_x_l0_c5", 819200, 128, 2048), ("enc_x_l1_c5", 819200, 1024, 2048), ("enc_h_c5", 819200, 512, 2048)]
    for name, K, M, N in shapes:
        a = (torch.randn(K, M, device="cuda", generator=g) * 0.1).bfloat16()
        b = (torch.randn(K, N, device="cuda", generator=g) * 0.1).bfloat16()
        ref = a.float().t() @ b.float()
        out = torch.zeros(M, N, device="cuda")
        k.wgrad_tn(a, b, out)
        err = float((out - ref).abs().max() / ref.abs().max())
        out2 = torch.empty(M, N, device="cuda")
        wgrad_into(out2, a, b)
        err_lib = float((out2 - ref).abs().max() / ref.abs().max())

        def custom():
            out.zero_()
            k.wgrad_tn(a, b, out)
        print(json.dumps({"shape": name, "K": K, "M": M, "N": N, "err": err, "err_lib": err_lib,
                          "custom_us": timed(custom), "zero_us": timed(lambda: out.zero_()),
                          "library_us": timed(lambda: wgrad_into(out2, a, b))}), flush=True)


if __name__ == "__main__":
    main()
