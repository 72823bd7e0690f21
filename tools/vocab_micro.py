"""Micro-benchmark of the decode vocab head (vocab_topk.hip) against yardsticks.

Times, for R rows x V vocab x H hidden: the fused head (logits kernel + select), a library
GEMM writing the same fp32 logits (torch.mm), and a plain fp32 fill of the logits array (the
HBM write floor).  Run under rocprofv3 --kernel-trace --stats for the per-kernel split.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from textsummarization_on_flink_amd import ops


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=256)
    ap.add_argument("--vocab", type=int, default=50000)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--T", type=int, default=400)
    ap.add_argument("--beam", type=int, default=4)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--no-pointer", action="store_true")
    a = ap.parse_args()
    k = ops.load(build_if_missing=False)
    R, V, H, T, K = a.rows, a.vocab, a.hidden, a.T, 2 * a.beam
    dev = "cuda"
    torch.manual_seed(0)
    X = (torch.randn(R, H, device=dev) * 0.5).to(torch.bfloat16)
    WT = (torch.randn(V, H, device=dev) * 0.05).to(torch.bfloat16)
    W = WT.t().contiguous()
    bias = torch.randn(V, device=dev) * 0.1
    Na = R // a.beam
    pg = None if a.no_pointer else torch.rand(R, device=dev)
    att = None if a.no_pointer else torch.softmax(torch.randn(R, T, device=dev), 1)
    ext = torch.randint(0, V + 50, (Na, T), device=dev, dtype=torch.int32)
    lens = torch.full((Na,), T, device=dev, dtype=torch.int32)
    ids = torch.zeros(R, K, device=dev, dtype=torch.int32)
    lp = torch.zeros(R, K, device=dev)
    logits = torch.empty(R, V, device=dev)
    parts = torch.empty(R, int(k.vocab_topk_parts(V)), 2, device=dev)
    res = {
        "fused_head_us": timeit(lambda: k.vocab_topk(X, WT, bias, pg, att, ext, lens, ids, lp, logits, parts,
                                                     R, V, H, T, K, a.beam), a.iters),
        "torch_mm_fp32_out_us": timeit(lambda: torch.mm(X, W, out_dtype=torch.float32, out=logits), a.iters),
        "fill_logits_us": timeit(lambda: logits.fill_(1.0), a.iters),
    }
    res["logits_MB"] = R * V * 4 / 1e6
    print(json.dumps(res))


if __name__ == "__main__":
    main()
