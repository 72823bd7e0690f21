"""Vocab-projection GEMMs of one training step (N = D*B rows, H = 256, V = 50k):
library GEMM vs split-K batched GEMM for the input gradient dout = dlogits . W^T
(K = V is long while the output [N, H] is only N/256 x 1 tiles of 256x256)."""
import json
import sys

import torch

F32, BF = torch.float32, torch.bfloat16


def t(fn, it=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(it):
        fn()
    e.record(); torch.cuda.synchronize()
    return round(s.elapsed_time(e) * 1e3 / it, 1)


N = int(sys.argv[1]) if len(sys.argv) > 1 else 25600
H, V = 256, 50000
dl = (torch.randn(N, V, device="cuda") * 1e-3).to(BF)
W = torch.randn(H, V, device="cuda").to(BF)
WT = W.t().contiguous()
ob = torch.randn(N, H + 8, device="cuda").to(BF)
bias = torch.randn(V, device="cuda").to(BF)
lg = torch.empty(N, V, device="cuda", dtype=BF)
grad = torch.zeros((H + 1) * V, device="cuda")
ref = torch.mm(dl, W.t(), out_dtype=F32)
r = {"N": N,
     "logits_addmm_bf16": t(lambda: torch.addmm(bias, ob[:, :H], W, out=lg)),
     "dWb_M257": t(lambda: torch.mm(ob[:, :H + 1].t(), dl, out_dtype=F32, out=grad.view(H + 1, V))),
     "dX_mm": t(lambda: torch.mm(dl, W.t(), out_dtype=F32)),
     "dX_mm_WT": t(lambda: torch.mm(dl, WT, out_dtype=F32))}
out = torch.empty(N, H, device="cuda")
for S in (2, 4, 5, 8, 10, 20, 25):
    Vs = V // S

    def f():
        p = torch.bmm(dl.view(N, S, Vs).transpose(0, 1), WT.view(S, Vs, H), out_dtype=F32)
        torch.sum(p, 0, out=out)
    try:
        f()
        err = (out - ref).abs().max().item() / ref.abs().max().item()
        r[f"dX_split{S}"] = t(f)
        r[f"err{S}"] = f"{err:.1e}"
    except Exception as e:  # noqa: BLE001
        r[f"dX_split{S}"] = str(e)[:100]
print(json.dumps(r))
