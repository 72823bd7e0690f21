"""Training vocab head micro-benchmark at the bench shape (N = D*B = 25600 rows, V = 50k,
H = 256): HIP-event time of the fused pass 1 (logits -> per-tile LSE partials + row stats)
and pass 2 (recomputed logits -> bf16 dlogits + bias gradient).  Synthetic inputs.

  python tools/vocab_train_micro.py [--rows 25600] [--reps 2] [--ldd 50000,50048,...]

--ldd: pass 2 with dlogits rows of these lengths (>= V; the pad columns are never written and stay zero): the row
stride's effect on the dlogits stores (profiles/r6/vocab_grad.md).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from textsummarization_on_flink_amd.ops import ops  # noqa: E402


def timed(fn, it):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=25600)
    ap.add_argument("--vocab", type=int, default=50000)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--ldd", type=str, default="")
    a = ap.parse_args()
    k = ops()
    N, V, H = a.rows, a.vocab, a.hidden
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(0)
    ldx = H + 8
    X = (torch.randn(N, ldx, generator=g) * 0.5).to(dev, torch.bfloat16)
    WT = (torch.randn(V, H, generator=g) * 0.1).to(dev, torch.bfloat16)
    bias = (torch.randn(V, generator=g) * 0.1).to(dev)
    target = torch.randint(0, V + 50, (N,), generator=g).to(dev, torch.int32)
    nt = int(k.vocab_train_tiles(V, H))
    part = torch.empty(nt * N * 2, device=dev)
    zg, lse, pv = (torch.empty(N, device=dev) for _ in range(3))
    alpha = torch.rand(N, generator=g).to(dev)
    dl = torch.empty(N, V, dtype=torch.bfloat16, device=dev)
    db = torch.zeros(V, device=dev)
    ref = None
    for rep in range(a.reps):
        fwd = lambda: k.vocab_train_fwd(X, WT, bias, target, part, zg, lse, pv, N, V, H, ldx, None, None)
        bwd = lambda: k.vocab_train_bwd(X, WT, bias, target, lse, alpha, dl, db, N, V, H, ldx, None, None, None, None)
        r = {"rep": rep, "rows": N, "fwd_us": timed(fwd, a.iters), "bwd_us": timed(bwd, a.iters)}
        db.zero_()
        fwd()
        bwd()
        torch.cuda.synchronize()
        cur = (lse.clone(), dl[:64].float().clone(), db.clone())
        if ref is None:
            ref = cur
        else:
            r["lse_maxdiff"] = (cur[0] - ref[0]).abs().max().item()
            r["dl_maxdiff"] = (cur[1] - ref[1]).abs().max().item()
            r["db_rel"] = ((cur[2] - ref[2]).abs().max() / ref[2].abs().max()).item()
        print(json.dumps(r), flush=True)
    for ld in [int(v) for v in a.ldd.split(",") if v]:
        dlp = torch.zeros(N, ld, dtype=torch.bfloat16, device=dev)  # pad columns: zero, never written
        bwd = lambda: k.vocab_train_bwd(X, WT, bias, target, lse, alpha, dlp, db, N, V, H, ldx, None, None, None, None)
        r = {"ldd": ld, "row_bytes": 2 * ld, "bwd_us": timed(bwd, a.iters)}
        r["pad_zero"] = bool((dlp[:, V:] == 0).all().item()) if ld > V else None
        r["same_dl"] = bool(torch.equal(dlp[:64, :V], dl[:64]))
        print(json.dumps(r), flush=True)
        del dlp


if __name__ == "__main__":
    main()
