"""attn_bwd_step at config #5's shape (A = 1024, T = 800, 256 rows per launch).  Random
operands.  Prints one JSON line: microseconds per launch, effective E+F bandwidth and a digest
of the outputs (tools only; the tests compare the paths).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    B, T, A = int(os.environ.get("MICRO_B", "256")), int(os.environ.get("MICRO_T", "800")), 1024
    g = torch.Generator(device="cuda").manual_seed(0)
    dev, F32, BF = "cuda", torch.float32, torch.bfloat16

    def r(*shape, s=1.0, dt=F32):
        return (torch.randn(*shape, generator=g, device=dev) * s).to(dt)

    E, F = r(B, T, A, s=0.5, dt=BF), r(B, T, A, s=0.5, dt=BF)
    s, v, wc = r(B, A, s=0.3), r(A, s=0.1), r(A, s=0.1)
    cov = torch.rand(B, T, generator=g, device=dev)
    a = torch.softmax(r(B, T), -1)
    dctx, ctx, Ga, dnext = r(B, A, s=0.1), r(B, A, s=0.1), r(B, T, s=0.1), r(B, T, s=0.1)
    gcl = torch.ones(B, device=dev)
    lens = torch.randint(T // 2, T + 1, (B,), generator=g, device=dev, dtype=torch.int32)
    lens[0] = T
    if os.environ.get("MICRO_FULL"):
        lens.fill_(T)
    de, ds, dcov = (torch.zeros(B, T, device=dev), torch.zeros(B, A, device=dev), torch.zeros(B, T, device=dev))

    def run():
        k.attn_bwd_step(E, F, s, v, wc, cov, a, dctx, ctx, Ga, dnext, gcl, lens, de, ds, dcov, B, T, A)

    run()
    torch.cuda.synchronize()
    out = [de.clone(), ds.clone(), dcov.clone()]
    it = 30
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(it):
        run()
    en.record()
    torch.cuda.synchronize()
    us = st.elapsed_time(en) * 1e3 / it
    gb = 2 * float(lens.sum()) * A * 2 / 1e9
    print(json.dumps({"variant": "default", "full": bool(os.environ.get("MICRO_FULL")), "B": B, "T": T, "A": A,
                      "us": round(us, 1), "ef_TBps": round(gb / us * 1e3, 2),
                      "digest": [round(float(x.double().abs().sum()), 4) for x in out]}), flush=True)
    torch.save([x.cpu() for x in out], f"gpurun_out/attn_a1024_{'default'}.pt")


if __name__ == "__main__":
    main()
