"""Issue cost of the attention kernels' tanh form (exp2 + rcp, attn_common.h rsig2) against the
clamped rational with one rcp (probes.hip tanh_rat2) inside a score-like reduction over
register-resident data: elements per second over the whole GPU, and accuracy vs fp64.

  python tools/tanh_probe.py [--iters 4096] [--reps 5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--threads", type=int, default=256 * 1024 * 4)
    a = ap.parse_args()
    import torch
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    inp = torch.randn(1024, device="cuda") * 2
    out = torch.empty(a.threads, device="cuda")
    res = {"threads": a.threads, "iters": a.iters, "elements_per_thread_iter": 8}
    for mode, name in ((0, "exp_rcp"), (1, "rational_1rcp")):
        k.tanh_tput(inp, out, 16, mode)
        torch.cuda.synchronize()
        best = None
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            k.tanh_tput(inp, out, a.iters, mode)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        el = a.threads * a.iters * 8
        res[name] = {"ms": round(best, 3), "G_elements_per_s": round(el / best / 1e6, 1), "checksum": float(out.sum())}
        x = torch.linspace(-20, 20, 4_000_001, device="cuda")
        t, s2 = torch.empty_like(x), torch.empty_like(x)
        k.tanh_eval(x, t, s2, mode)
        ref = torch.tanh(x.double())
        res[name]["max_abs_err_tanh"] = float((t.double() - ref).abs().max())
        res[name]["max_abs_err_sech2"] = float((s2.double() - (1 - ref * ref)).abs().max())
    res["rational_vs_exp_time"] = round(res["rational_1rcp"]["ms"] / res["exp_rcp"]["ms"], 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
