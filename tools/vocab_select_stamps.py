"""Per-phase attribution of the decode select kernel (vocab_select_kernel, span path) at the
beam-4 / 64-article shape: thread 0 of every row stamps s_memtime (shader cycles) at the phase
boundaries of a stamped build of the kernel; prints the median cycles of each phase over rows
(profiles/r6/decode_select_stamps.md).  Synthetic inputs, as tools/vocab_micro.py."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from textsummarization_on_flink_amd.ops import ops  # noqa: E402

PHASES = ["pgen+clear", "partials+hash", "block_max", "lse+gkey", "tile_cands", "rank1", "rt2+gkey3",
          "cands2", "rank2", "copy_cands", "rank3", "tail"]


def main():
    k = ops()
    R, V, H, T, K, beam = 256, 50000, 256, 400, 8, 4
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (torch.randn(R, H, generator=g) * 0.5).to("cuda", torch.bfloat16)
    WT = (torch.randn(V, H, generator=g) * 0.1).to("cuda", torch.bfloat16)
    bias = (torch.randn(V, generator=g) * 0.1).cuda()
    pg = torch.rand(R, generator=g).cuda()
    attn = torch.softmax(torch.randn(R, T, generator=g), 1).cuda()
    ext = torch.randint(4, V + 50, (R // beam, T), generator=g, dtype=torch.int32).cuda()
    lens = torch.full((R // beam,), T, dtype=torch.int32, device="cuda")
    ids = torch.empty(R, K, dtype=torch.int32, device="cuda")
    lp = torch.empty(R, K, device="cuda")
    lg = torch.empty(R, V, device="cuda")
    nt = int(k.vocab_topk_parts(V, H))
    pms = torch.empty(R, nt, 2, device="cuda")
    st = torch.zeros(R, 16, dtype=torch.int64, device="cuda")
    k.vocab_select_stamps(st)
    for _ in range(20):
        k.vocab_topk(X, WT, bias, pg, attn, ext, lens, ids, lp, lg, pms, R, V, H, T, K, beam)
    torch.cuda.synchronize()
    k.vocab_select_stamps(None)
    s = st[:, :13].double()
    d = (s[:, 1:] - s[:, :-1])
    med = d.median(0).values.tolist()
    out = {"rows": R, "total_cycles_median": float((s[:, 12] - s[:, 0]).median()),
           "phase_cycles_median": {n: round(v) for n, v in zip(PHASES, med)},
           "start_spread_cycles": float(s[:, 0].max() - s[:, 0].min())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
