"""Per-step decoder kernels at the training shapes (one row group): HIP-event time per call of
dec_cell_fwd, linear2 (attention query s = [c, h] . W_s), dec_bwd_cell and dec_bwd_dz, at
hidden 256 (bench config) and 512 (config #5).  Synthetic inputs.

  python tools/dec_kernels_micro.py [--rows 128,256] [--hidden 256,512]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from textsummarization_on_flink_amd.ops import ops  # noqa: E402


def timed(fn, it=50):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) * 1e3 / it, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="128,256")
    ap.add_argument("--hidden", default="256,512")
    a = ap.parse_args()
    k = ops()
    E = 128
    for H in [int(x) for x in a.hidden.split(",")]:
        A = 2 * H
        for B in [int(x) for x in a.rows.split(",")]:
            r = lambda *s, dt=torch.float32: (torch.randn(*s, device="cuda") * 0.1).to(dt)
            bf = torch.bfloat16
            XG, ctxp, hprev, cprev = r(B, 4 * H), r(B, A, dt=bf), r(B, H, dt=bf), r(B, H)
            WcT = r(4 * H, H + A, dt=bf)
            c_out, cb, hb, act = r(B, H), r(B, H, dt=bf), r(B, H, dt=bf), r(B, 4 * H)
            WsT, bs, s_out = r(A, 2 * H, dt=bf), r(A), r(B, A)
            dz, Wbig = r(B, 4 * H, dt=bf), r(E + H + A, 4 * H, dt=bf)
            dx, dctx, dh = r(B, E), r(B, A), r(B, H)
            ds, Ws = r(B, A), r(A, 2 * H, dt=bf)
            dcc = r(B, H)
            res = {"H": H, "A": A, "rows": B,
                   "dec_cell_fwd_us": timed(lambda: k.dec_cell_fwd(XG, ctxp, hprev, cprev, WcT, c_out, cb, hb, act,
                                                                   B, H, A, None, 0)),
                   "linear2_sproj_us": timed(lambda: k.dec_sproj(cb, hb, WsT, bs, s_out, B, H, A, None, 0)),
                   "dec_bwd_dz_us": timed(lambda: k.dec_bwd_dz(dz, Wbig, None, None, dx, dctx, dh, B, E, H, A, None, 0))}
            try:
                res["dec_bwd_cell_us"] = timed(lambda: k.dec_bwd_cell(ds, Ws, None, dh, dh, dcc, act, c_out, cprev, dz,
                                                                      B, H, A, None, 0))
            except RuntimeError as e:  # noqa: BLE001
                res["dec_bwd_cell_us"] = str(e)[:80]
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
