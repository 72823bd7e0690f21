"""Attribution of the decode vocab logits kernel (vocab_logits_span_kernel, R = 256, V = 50k, H = 256):
HIP-event time per launch with parts of the kernel compiled out (PROBE bits: 1 no logits stores,
2 no epilogue math, 4 no MFMAs).  The probe variants give wrong results by design; only their
times are used (profiles/r6/decode_vocab_span.md).  Synthetic inputs."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from textsummarization_on_flink_amd.ops import ops  # noqa: E402


def main():
    k = ops()
    R, V, H = int(os.environ.get("ROWS", 256)), 50000, 256
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (torch.randn(R, H, generator=g) * 0.5).to("cuda", torch.bfloat16)
    WT = (torch.randn(V, H, generator=g) * 0.1).to("cuda", torch.bfloat16)
    bias = (torch.randn(V, generator=g) * 0.1).cuda()
    nt = int(k.vocab_topk_parts(V, H))
    lg = torch.empty(max(R * V, 8 * nt * R * 32), device="cuda")  # the span-major probe writes [8 nt waves][R][32]
    pms = torch.empty(R, nt, 2, device="cuda")
    if os.environ.get("PMC"):  # counter pass: a few production launches only
        for _ in range(5):
            k.vocab_span_probe(X, WT, bias, lg, pms, R, V, 0)
        torch.cuda.synchronize()
        return
    names = {0: "full", 1: "no_store", 3: "no_store_no_math", 4: "no_mfma", 5: "no_mfma_no_store", 7: "loads_only",
             8: "temporal_store", 16: "span_major_store", 32: "bf16_store"}
    out = {"R": R, "V": V, "H": H}
    for rep in range(2):
        for p, n in names.items():
            for _ in range(20):
                k.vocab_span_probe(X, WT, bias, lg, pms, R, V, p)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(300):
                k.vocab_span_probe(X, WT, bias, lg, pms, R, V, p)
            e1.record()
            torch.cuda.synchronize()
            out[n] = round(e0.elapsed_time(e1) * 1000 / 300, 2)
    k.vocab_span_probe(X, WT, bias, lg, pms, R, V, 0)
    ref = torch.mm(X, WT.t(), out_dtype=torch.float32) + bias
    torch.cuda.synchronize()
    out["max_err_full"] = float((lg[:R * V].view(R, V) - ref).abs().max())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
