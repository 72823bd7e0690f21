"""The encoder-side GEMMs of a config #5 training step (hidden 512, 2 layers, T = 800, batch
MB_B), each as the engine issues it and with alternatives, HIP events, random bf16 operands.
Prints one JSON line: milliseconds per call and the achieved TFLOP/s.

  B=1024 python tools/gemm_c5.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

F32, BF = torch.float32, torch.bfloat16


def timeit(fn, it=5):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    from textsummarization_on_flink_amd.models.pointer_generator import wgrad_into
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    B, T, H = int(os.environ.get("B", "1024")), 800, 512
    N = B * T
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: (torch.randn(*s, device=dev, generator=g) * 0.1).to(BF)
    res = {"B": B, "rows": N}

    def rec(name, ms, flop):
        res[name] = round(ms, 3)
        res[name + "_TF"] = round(flop / (ms * 1e-3) / 1e12, 1)

    x2, x1, dz, hs = r(N, 2 * H), r(N, 128), r(N, 4 * H), r(N, H)
    kx2, kx1, wh = r(2 * H, 4 * H), r(128, 4 * H), r(2 * H, 2 * H)
    gx = torch.empty(N, 4 * H, device=dev)
    rec("fwd_gx_l2", timeit(lambda: torch.mm(x2, kx2, out_dtype=F32, out=gx)), 2 * N * 2 * H * 4 * H)
    rec("fwd_gx_l1", timeit(lambda: torch.mm(x1, kx1, out_dtype=F32, out=gx)), 2 * N * 128 * 4 * H)
    Fo = torch.empty(N, 2 * H, device=dev, dtype=BF)
    rec("fwd_F", timeit(lambda: torch.mm(x2, wh, out=Fo)), 2 * N * 2 * H * 2 * H)
    del gx
    o2 = torch.empty(2 * H, 4 * H, device=dev)
    oh = torch.empty(H, 4 * H, device=dev)
    f = 2 * N * 2 * H * 4 * H
    rec("wg_x2_bmm", timeit(lambda: wgrad_into(o2, x2, dz)), f)
    rec("wg_x2_tn", timeit(lambda: (o2.zero_(), k.wgrad_tn(x2, dz, o2))), f)
    rec("wg_x2_mm", timeit(lambda: torch.mm(x2.t(), dz, out_dtype=F32, out=o2)), f)
    f = 2 * N * H * 4 * H
    rec("wg_h_bmm", timeit(lambda: wgrad_into(oh, hs, dz)), f)
    rec("wg_h_tn", timeit(lambda: (oh.zero_(), k.wgrad_tn(hs, dz, oh))), f)
    rec("wg_h_mm", timeit(lambda: torch.mm(hs.t(), dz, out_dtype=F32, out=oh)), f)
    dx = torch.empty(N, 2 * H, device=dev)
    rec("dx_l2", timeit(lambda: torch.mm(dz, kx2.t(), out_dtype=F32, out=dx)), 2 * N * 4 * H * 2 * H)
    dxb = torch.empty(N, 2 * H, device=dev, dtype=BF)
    rec("dx_l2_bf16out", timeit(lambda: torch.mm(dz, kx2.t(), out=dxb)), 2 * N * 4 * H * 2 * H)
    ow = torch.empty(2 * H, 2 * H, device=dev)
    f = 2 * N * 2 * H * 2 * H
    rec("wg_wh_bmm", timeit(lambda: wgrad_into(ow, x2, Fo)), f)
    rec("wg_wh_tn", timeit(lambda: (ow.zero_(), k.wgrad_tn(x2, Fo, ow))), f)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
