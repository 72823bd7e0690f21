"""Decode vocab head micro-benchmark at the beam-4 / 64-article shape (R=256 rows, V=50k,
H=256, T=400, K=8): HIP-event time of one vocab_topk call (logits + select kernels).  Run it
under ``rocprofv3 --kernel-trace --stats`` for the per-kernel split.  Synthetic inputs."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from textsummarization_on_flink_amd.ops import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=256)
    ap.add_argument("--vocab", type=int, default=50000)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--enc", type=int, default=400)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    k = ops()
    R, V, H, T, K, beam = a.rows, a.vocab, a.hidden, a.enc, 8, 4
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (torch.randn(R, H, generator=g) * 0.5).to(dev, torch.bfloat16)
    WT = (torch.randn(V, H, generator=g) * 0.1).to(dev, torch.bfloat16)
    bias = (torch.randn(V, generator=g) * 0.1).to(dev)
    pg = torch.rand(R, generator=g).to(dev)
    attn = torch.softmax(torch.randn(R, T, generator=g), 1).to(dev)
    ext = torch.randint(4, V + 50, (R // beam, T), generator=g, dtype=torch.int32).to(dev)
    lens = torch.full((R // beam,), T, dtype=torch.int32, device=dev)
    ids = torch.empty(R, K, dtype=torch.int32, device=dev)
    lp = torch.empty(R, K, device=dev)
    lg = torch.empty(R, V, device=dev)
    nt = int(k.vocab_topk_parts(V, H))
    pms = torch.empty(R, nt, 2, device=dev)

    def run():
        k.vocab_topk(X, WT, bias, pg, attn, ext, lens, ids, lp, lg, pms, R, V, H, T, K, beam)

    for _ in range(5):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"vocab_topk_us": round(e0.elapsed_time(e1) * 1000 / a.iters, 2), "R": R, "V": V, "H": H}))


if __name__ == "__main__":
    main()
