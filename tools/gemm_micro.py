"""Hand-written MFMA GEMM (gemm_bt) vs hipBLASLt (blt_mm, the fastest of its candidates) on the
engine's activation-GEMM shapes; HIP-event times of graph-captured repeats, random bf16 data.

  python tools/gemm_micro.py [--reps 10]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # name, M, N, K, out dtype
    ("c5_gx_l1", 819200, 2048, 1024, "f32"), ("c5_gx_l0", 819200, 2048, 128, "f32"),
    ("c5_F", 819200, 1024, 1024, "bf16"), ("c5_dx_l1", 819200, 1024, 2048, "f32"),
    ("b256_gx", 102400, 1024, 128, "f32"), ("b256_F", 102400, 512, 512, "bf16"),
    ("sq4096", 4096, 4096, 4096, "f32"), ("sq8192", 8192, 8192, 8192, "bf16"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    import torch
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    torch.manual_seed(0)
    for name, M, N, K, od in SHAPES:
        if a.only and a.only not in name:
            continue
        A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        Bt = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        out = torch.empty(M, N, device="cuda", dtype=torch.float32 if od == "f32" else torch.bfloat16)
        res = {"shape": name, "M": M, "N": N, "K": K, "out": od}
        runs = {"gemm_bt": lambda: k.gemm_bt(A, Bt, out, 0.0, None, None, None, 0, 0, 0, None),
                "blt_mm": lambda: k.blt_mm(A, Bt, out, False, True, 0.0, None)}
        ref = None
        for tag, fn in runs.items():
            fn()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.float().clone() if M * N <= 1 << 26 else out[:4096].float().clone()
            else:
                cmp = out.float() if M * N <= 1 << 26 else out[:4096].float()
                res["max_rel_diff"] = float((cmp - ref).abs().max() / ref.abs().max())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(a.reps):
                    fn()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1000 / a.reps
            res[f"{tag}_us"] = round(us, 1)
            res[f"{tag}_TF"] = round(2.0 * M * N * K / us / 1e6, 1)
        print(json.dumps(res), flush=True)
        del A, Bt, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
