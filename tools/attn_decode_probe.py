"""Attribution of the beam-decode attention forward (attn_fwd_row_kernel<1, 12>: 256 hypothesis
rows, A = 512, T = 400): HIP-event time per launch with parts compiled out (PROBE bits: 1 no
score arithmetic, 2 no context accumulation, 4 no E loads, 8 no F / E loads) and with the rows'
sharing of encoder rows varied (rep = hypotheses per article: 1 = every row its own article,
4 = beam decode, 256 = one article for all).  Probe results are wrong by design; only times are
used (profiles/r6/decode_attention_probe.md).  Synthetic inputs."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from textsummarization_on_flink_amd.ops import ops  # noqa: E402


def main():
    k = ops()
    B, T, A = 256, 400, 512
    g = torch.Generator(device="cpu").manual_seed(0)
    out = {"B": B, "T": T, "A": A}
    for rep in (1, 4, 256):
        na = B // rep
        F = (torch.randn(na, T, A, generator=g) * 0.5).to("cuda", torch.bfloat16)
        E = (torch.randn(na, T, A, generator=g) * 0.5).to("cuda", torch.bfloat16)
        s = (torch.randn(B, A, generator=g) * 0.5).cuda()
        v = (torch.randn(A, generator=g) * 0.1).cuda()
        wc = (torch.randn(A, generator=g) * 0.1).cuda()
        cov = torch.rand(B, T, generator=g).cuda()
        lens = torch.full((na,), T, dtype=torch.int32, device="cuda")
        a = torch.empty(B, T, device="cuda")
        ctx = torch.empty(B, A, device="cuda")
        for p, n in ((0, "full"), (1, "no_score"), (2, "no_ctx"), (3, "no_math"), (4, "no_E_loads"), (8, "no_loads"),
                     (11, "loop_only")):
            if rep != 4 and p not in (0,):
                continue
            for _ in range(10):
                k.attn_fwd_row_probe(F, E, s, v, wc, cov, lens, a, ctx, B, T, rep, p)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(200):
                k.attn_fwd_row_probe(F, E, s, v, wc, cov, lens, a, ctx, B, T, rep, p)
            e1.record()
            torch.cuda.synchronize()
            out[f"rep{rep}_{n}"] = round(e0.elapsed_time(e1) * 1000 / 200, 2)
        del F, E
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
