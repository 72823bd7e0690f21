"""Timing of the output-projection gradient variants (dW = outb^T . dl, db = colsum(dl))."""
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


N, H, V = 25600, 256, 50000
dl = (torch.randn(N, V, device="cuda") * 1e-3).to(BF)
ob = torch.zeros(N, H + 8, device="cuda", dtype=BF)
ob[:, :H] = torch.randn(N, H, device="cuda").to(BF)
ob[:, H] = 1
grad = torch.zeros((H + 1) * V, device="cuda")
buf = torch.zeros(V, H + 8, device="cuda")
buf2 = torch.zeros(H + 64, V, device="cuda")
ob64 = torch.zeros(N, H + 64, device="cuda", dtype=BF)
W = torch.randn(H, V, device="cuda").to(BF)
bias = torch.randn(V, device="cuda").to(BF)
lg = torch.empty(N, V, device="cuda", dtype=BF)
r = {
    "dW_M256": t(lambda: torch.mm(ob[:, :H].t(), dl, out_dtype=F32, out=grad[:H * V].view(H, V))),
    "db_sum": t(lambda: grad[H * V:].copy_(dl.sum(0, dtype=F32))),
    "dWb_M257": t(lambda: torch.mm(ob[:, :H + 1].t(), dl, out_dtype=F32, out=grad.view(H + 1, V))),
    "dWbT_N264": t(lambda: torch.mm(dl.t(), ob, out_dtype=F32, out=buf)),
    "dWbT_N264_plus_copy": t(lambda: (torch.mm(dl.t(), ob, out_dtype=F32, out=buf),
                                      grad.view(H + 1, V).copy_(buf[:, :H + 1].t()))),
    "dWb_M320": t(lambda: torch.mm(ob64.t(), dl, out_dtype=F32, out=buf2)),
    "dX": t(lambda: torch.mm(dl, W.t(), out_dtype=F32)),
    "logits_addmm_bf16": t(lambda: torch.addmm(bias, ob[:, :H], W, out=lg)),
    "logits_mm_fp32": t(lambda: torch.mm(ob[:, :H], W, out_dtype=F32)),
}
print(json.dumps(r))
