"""HIP-event timings of the beam-decode step kernels at the bench shape (64 articles x beam 4,
T = 400, A = 512, H = 256, V = 50k): the per-hypothesis row attention vs the article-level
split attention (attention_beam.hip), each launch sequence captured in a hipGraph of N copies.

  python tools/decode_kernels_micro.py [--na 64] [--T 400] [--reps 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps, torch):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(5):
        g.replay()
    t1.record()
    torch.cuda.synchronize()
    return 1000.0 * t0.elapsed_time(t1) / (5 * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--na", type=int, default=64)
    ap.add_argument("--T", type=int, default=400)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import torch
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    Na, T, A, rep = a.na, a.T, 512, 4
    B = Na * rep
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s, sc=1.0: torch.randn(*s, generator=g, device=dev) * sc
    lens = torch.full((Na,), T, dtype=torch.int32, device=dev)
    E, F = r(Na, T, A, sc=0.5).bfloat16(), r(Na, T, A, sc=0.5).bfloat16()
    s, v, wc = r(B, A, sc=0.3), r(A, sc=0.1), r(A, sc=0.5)
    cov_src, a_src = torch.rand(B, T, device=dev), torch.rand(B, T, device=dev) * 0.01
    gidx = torch.arange(B, dtype=torch.int32, device=dev)
    att, ctx = torch.zeros(B, T, device=dev), torch.zeros(B, A, device=dev)
    ctxb, keep = torch.zeros(B, A, device=dev, dtype=torch.bfloat16), torch.zeros(B, T, device=dev)
    out = {}
    out["attn_fwd_row_beam_us"] = timed(lambda: k.attn_fwd_row_beam(F, E, s, v, wc, cov_src, a_src, keep, gidx, lens,
                                                                    att, ctx, ctxb, B, T, A, rep), a.reps, torch)
    for S in sorted({int(k.attn_beam_chunks(Na, T)), 4, 8, 16}):
        e_buf, pm, pctx = torch.zeros(B, T, device=dev), torch.zeros(B, S, 2, device=dev), torch.zeros(B, S, A,
                                                                                                       device=dev)
        out[f"attn_beam_S{S}_us"] = timed(lambda: k.attn_beam(F, E, s, v, wc, None, cov_src, a_src, keep, gidx, lens,
                                                              e_buf, pm, pctx, att, ctx, ctxb, B, T, A, rep, S),
                                          a.reps, torch)
    out.update({"Na": Na, "T": T, "A": A, "default_S": int(k.attn_beam_chunks(Na, T))})
    print(json.dumps({k_: (round(v_, 2) if isinstance(v_, float) else v_) for k_, v_ in out.items()}), flush=True)


if __name__ == "__main__":
    main()
