"""Persistent-LSTM launch timing (HIP events): forward and BPTT per (H, B, T), one JSON line
per shape with the microseconds per launch and per recurrence step.

  python tools/lstm_micro.py 256:256:400 512:256:400 512:128:800
(The 4-wave forward runs below H = 512, the 8-wave one at H = 512; the BPTT always has 8 waves.)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, it=5):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / it


def main():
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    for spec in sys.argv[1:] or ["256:256:400", "512:256:400"]:
        H, B, T = (int(x) for x in spec.split(":"))
        g = torch.Generator(device="cuda").manual_seed(0)
        lens = torch.full((B,), T, device="cuda", dtype=torch.int32)
        gx = torch.randn(2, T, B, 4 * H, device="cuda", generator=g) * 0.5
        W = (torch.randn(2, 4 * H, H, device="cuda", generator=g) / H ** 0.5).bfloat16()
        Wn = W.transpose(1, 2).contiguous()
        bias = torch.zeros(2, 4 * H, device="cuda")
        hs = torch.zeros(2, T + 1, B, H, device="cuda", dtype=torch.bfloat16)
        cs = torch.zeros(2, T + 1, B, H, device="cuda")
        acts = torch.zeros(2, T, B, 4 * H, device="cuda")
        out = torch.zeros(B, T, 2 * H, device="cuda", dtype=torch.bfloat16)
        err = torch.zeros(1, device="cuda", dtype=torch.int32)
        xf = torch.zeros(int(k.lstm_persistent_xbuf(H, B, False)), device="cuda", dtype=torch.long)
        xb = torch.zeros(int(k.lstm_persistent_xbuf(H, B, True)), device="cuda", dtype=torch.long)
        dout = torch.randn(2, T, B, H, device="cuda", generator=g) * 0.1
        dh_fin = torch.zeros(2, B, H, device="cuda")
        dcc = torch.zeros(2, B, H, device="cuda")
        dz = torch.zeros(2, T, B, 4 * H, device="cuda", dtype=torch.bfloat16)
        db = torch.zeros(2, 4 * H, device="cuda")

        def fwd():
            xf.zero_()
            k.lstm_fwd_persistent(gx, bias, W, hs, cs, acts, out, lens, xf, err, T, B, H)

        def bwd():
            xb.zero_()
            k.lstm_bwd_persistent(dz, Wn, dout, dh_fin, dcc, acts, cs, lens, xb, err, db, T, B, H, False)

        tf, tb = timeit(fwd), timeit(bwd)
        print(json.dumps({"H": H, "B": B, "T": T, "nw": "auto",
                          "grid": int(k.lstm_persistent_grid(H, B)), "launches": int(k.lstm_persistent_launches(H, B)),
                          "fwd_us": round(tf, 1), "bwd_us": round(tb, 1), "fwd_us_per_step": round(tf / T, 2),
                          "bwd_us_per_step": round(tb / T, 2), "err": int(err.item())}), flush=True)
        del gx, acts, dz, dout, out, hs, cs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
