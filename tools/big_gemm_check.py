"""Library GEMMs at the config #5 batch-2048 shapes: do hipBLASLt's plain and strided-batched
paths address operands past 2^31 elements / 4 GB correctly?

The engine at H=512, 2 layers, T=800, B=2048 runs (per encoder direction and layer):
  * gx = x_sf . Kxi        [T*B, 1024] x [1024, 2048] -> fp32 [T*B, 2048]  (3.36G outputs)
  * dxs = dz . Kx^T        [T*B, 2048] x [2048, 1024]                      (3.36G-element A)
  * dW  = x_sf^T . dz      split-K as bmm over 32 batches of 51200 rows    (batch offsets up to 3.25G)
Each result is compared against the same product of small contiguous slices copied out of the
big operands (so only the big-operand addressing differs).  Prints one JSON line per check.
"""
import json
import sys

import torch


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-30))


def main():
    dev = "cuda"
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    T, din, G = 800, 1024, 2048
    K = T * B
    torch.manual_seed(0)
    x = torch.randn(K, din, device=dev, dtype=torch.bfloat16)
    W = torch.randn(din, G, device=dev, dtype=torch.bfloat16) * 0.03
    res = []
    # 1. plain GEMM, fp32 output past 2^31 elements
    out = torch.empty(K, G, device=dev, dtype=torch.float32)
    torch.mm(x, W, out_dtype=torch.float32, out=out)
    for r0 in (0, K // 2, K - 256):
        ref = torch.mm(x[r0:r0 + 256].clone(), W, out_dtype=torch.float32)
        res.append({"check": "mm_out_big", "row0": r0, "rel": rel(out[r0:r0 + 256], ref)})
    del out
    torch.cuda.synchronize()
    print(json.dumps(res[-3:]), flush=True)
    # 2. plain GEMM, A operand past 2^31 elements
    dz = torch.randn(K, G, device=dev, dtype=torch.bfloat16)
    Kx = torch.randn(din, G, device=dev, dtype=torch.bfloat16) * 0.03
    o2 = torch.mm(dz, Kx.t(), out_dtype=torch.float32)
    for r0 in (0, K // 2, K - 256):
        ref = torch.mm(dz[r0:r0 + 256].clone(), Kx.t().contiguous(), out_dtype=torch.float32)
        res.append({"check": "mm_a_big", "row0": r0, "rel": rel(o2[r0:r0 + 256], ref)})
    del o2
    torch.cuda.synchronize()
    print(json.dumps(res[-3:]), flush=True)
    # 3. split-K strided-batched GEMM (wgrad_into's S = 32 path)
    S = 32
    parts = torch.bmm(x.reshape(S, K // S, din).transpose(1, 2), dz.reshape(S, K // S, G), out_dtype=torch.float32)
    for s in (0, S // 2, S - 1):
        a = x[s * (K // S):(s + 1) * (K // S)].clone()
        b = dz[s * (K // S):(s + 1) * (K // S)].clone()
        ref = torch.mm(a.t(), b, out_dtype=torch.float32)
        res.append({"check": "bmm_splitk", "batch": s, "offset_elems": s * (K // S) * G, "rel": rel(parts[s], ref)})
    torch.cuda.synchronize()
    print(json.dumps(res[-3:]), flush=True)
    bad = [r for r in res if not (r["rel"] < 1e-2)]
    print(json.dumps({"B": B, "ok": not bad, "bad": bad}), flush=True)
    return 0 if not bad else 1


if __name__ == "__main__":
    sys.exit(main())
