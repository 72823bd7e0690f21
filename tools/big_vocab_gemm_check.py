"""The vocab-head library GEMMs of the unfused (H=512) training path at large batches, checked
against the same products computed over small row chunks (normal-size GEMMs):

  * logits = outb . W + b   [N, H] x [H, V] -> bf16 [N, V]
  * dW|db  = [outb | 1]^T . dlogits  (K = N rows, the [N, V] operand past 2^32 elements)
  * dX     = dlogits . W^T   [N, V] x [V, H]

N = D x B = 100 x B.  Usage: python tools/big_vocab_gemm_check.py B [B ...]
"""
import json
import sys

import torch


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-30))


def check(B, H=512, V=50000, D=100):
    dev = "cuda"
    N = D * B
    torch.manual_seed(B)
    out = {"B": B, "N": N, "nv_elems": N * V}
    xe = torch.randn(N, H + 8, device=dev, dtype=torch.bfloat16)
    xe[:, H] = 1.0
    W = (torch.randn(H, V, device=dev) * 0.05).to(torch.bfloat16)
    bias = torch.randn(V, device=dev, dtype=torch.bfloat16)
    logits = torch.empty(N, V, device=dev, dtype=torch.bfloat16)
    torch.addmm(bias, xe[:, :H], W, out=logits)
    C = 12800
    errs = []
    for r0 in (0, N // 2, N - C):
        ref = torch.addmm(bias, xe[r0:r0 + C, :H].clone(), W)
        errs.append(rel(logits[r0:r0 + C], ref))
    out["logits_rel"] = max(errs)
    dl = logits  # reuse as dlogits (values only matter for the comparison)
    dW = torch.empty(H + 1, V, device=dev, dtype=torch.float32)
    torch.mm(xe[:, :H + 1].t(), dl, out_dtype=torch.float32, out=dW)
    ref = torch.zeros(H + 1, V, device=dev, dtype=torch.float32)
    for r0 in range(0, N, C):
        ref += torch.mm(xe[r0:r0 + C, :H + 1].t().contiguous(), dl[r0:r0 + C].clone(), out_dtype=torch.float32)
    out["dW_rel"] = rel(dW, ref)
    del ref, dW
    dX = torch.mm(dl, W.t(), out_dtype=torch.float32)
    errs = []
    for r0 in (0, N // 2, N - C):
        errs.append(rel(dX[r0:r0 + C], torch.mm(dl[r0:r0 + C].clone(), W.t().contiguous(), out_dtype=torch.float32)))
    out["dX_rel"] = max(errs)
    torch.cuda.synchronize()
    out["ok"] = all(out[k] < 1e-2 for k in ("logits_rel", "dW_rel", "dX_rel"))
    return out


def main():
    ok = True
    for b in (int(x) for x in (sys.argv[1:] or ["1024", "2048"])):
        r = check(b)
        print(json.dumps(r), flush=True)
        ok &= r["ok"]
        torch.cuda.empty_cache()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
