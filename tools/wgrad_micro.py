"""Weight-gradient GEMMs (long K, small M x N): library GEMM vs split-K batched GEMM."""
import json
import torch

F32, BF = torch.float32, torch.bfloat16


def t(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(it):
        fn()
    e.record(); torch.cuda.synchronize()
    return round(s.elapsed_time(e) * 1e3 / it, 1)


res = {}
for (K, M, N) in [(102400, 512, 512), (102400, 128, 1024), (102400, 256, 1024), (25600, 256, 256), (25600, 128, 128),
                  (25600, 256, 512), (25600, 128, 1024)]:
    a = torch.randn(K, M, device="cuda").to(BF)
    b = torch.randn(K, N, device="cuda").to(BF)
    ref = torch.mm(a.t(), b, out_dtype=F32)
    r = {"mm": t(lambda: torch.mm(a.t(), b, out_dtype=F32))}
    for S in (8, 16, 32, 64):
        if K % S:
            continue
        try:
            out = torch.empty(M, N, device="cuda")

            def f():
                p = torch.bmm(a.view(S, K // S, M).transpose(1, 2), b.view(S, K // S, N), out_dtype=F32)
                torch.sum(p, 0, out=out)
            f()
            err = (out - ref).abs().max().item() / ref.abs().max().item()
            r[f"split{S}"] = t(f)
            r[f"err{S}"] = f"{err:.1e}"
        except Exception as e:  # noqa
            r[f"split{S}"] = str(e)[:80]
    res[f"K{K}_M{M}_N{N}"] = r
print(json.dumps(res, indent=0))
