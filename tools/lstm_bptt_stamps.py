"""Attribution of the H = 512, 32-row-team encoder BPTT step (lstm_bwd_persistent32_kernel, the
config #5 backward): a STAMP build of the production kernel sums s_memtime deltas per step phase
in thread 0 of every workgroup, and this tool prints the mean per step over the workgroups:

  0 loads issued      the step's dout / activation / c loads issued, own partial dh from LDS
  1 hand-off wait     polling the peers' partial-dh granules of the previous step
  2 cell backward     dz for the lane's 2 rows (waits for the loads), dz slice -> LDS
  3 barrier 1         the team's dz slice complete
  4 MFMA              this wave's partial dh (2 x 2 tiles, K = 256)
  5 publish           partial dh -> own LDS slot or the destination's granules
  6 dz stores + barrier 2

Synthetic operands (random activations; lengths T for every row).  Timed without stamps too.

  python tools/lstm_bptt_stamps.py [H:B:T ...]     (default 512:1024:800)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

PHASES = ["loads_issued", "handoff_wait", "cell_backward", "barrier1", "mfma", "publish", "dz_store_barrier2"]


def main():
    from textsummarization_on_flink_amd.ops import ops
    k = ops()
    for spec in sys.argv[1:] or ["512:1024:800"]:
        H, B, T = (int(x) for x in spec.split(":"))
        g = torch.Generator(device="cuda").manual_seed(0)
        lens = torch.full((B,), T, device="cuda", dtype=torch.int32)
        W = (torch.randn(2, 4 * H, H, device="cuda", generator=g) / H ** 0.5).bfloat16()
        Wn = W.transpose(1, 2).contiguous()
        cs = torch.rand(2, T + 1, B, H, device="cuda", generator=g) - 0.5
        acts = torch.rand(2, T, B, 4 * H, device="cuda", generator=g)
        err = torch.zeros(1, device="cuda", dtype=torch.int32)
        xb = torch.zeros(int(k.lstm_persistent_xbuf(H, B, True)), device="cuda", dtype=torch.long)
        dout = torch.randn(2, T, B, H, device="cuda", generator=g) * 0.1
        dh_fin = torch.zeros(2, B, H, device="cuda")
        dcc = torch.zeros(2, B, H, device="cuda")
        dz = torch.zeros(2, T, B, 4 * H, device="cuda", dtype=torch.bfloat16)
        db = torch.zeros(2, 4 * H, device="cuda")

        def bwd():
            xb.zero_()
            k.lstm_bwd_persistent(dz, Wn, dout, dh_fin, dcc, acts, cs, lens, xb, err, db, T, B, H, False)

        def timed(it=3):
            bwd()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(it):
                bwd()
            e.record()
            torch.cuda.synchronize()
            return s.elapsed_time(e) * 1e3 / it

        t_plain = timed()
        nteam = 2 * ((B + 31) // 32)
        st = torch.zeros(nteam * (H // 64) * 8, device="cuda", dtype=torch.long)
        k.lstm_bwd_stamps(st)
        t_stamp = timed()
        bwd()
        torch.cuda.synchronize()
        k.lstm_bwd_stamps(None)
        v = st.view(-1, 8).double()
        live = v[:, 7] > 0
        per_step = (v[live, :7] / v[live, 7:8]).mean(0)
        tot = float(per_step.sum())
        spread = (v[live, :7] / v[live, 7:8]).std(0)
        res = {"H": H, "B": B, "T": T, "us_plain": round(t_plain, 1), "us_per_step_plain": round(t_plain / T, 2),
               "us_stamped": round(t_stamp, 1), "workgroups": int(live.sum()), "steps": int(v[live, 7].max()),
               "cycles_per_step": round(tot, 1),
               "phases_cycles": {p: round(float(c), 1) for p, c in zip(PHASES, per_step)},
               "phases_share": {p: round(float(c) / tot, 3) for p, c in zip(PHASES, per_step)},
               "phases_std_over_workgroups": {p: round(float(c), 1) for p, c in zip(PHASES, spread)},
               "err": int(err.item())}
        # the s_memtime clock against the event time of the stamped launch
        res["memtime_hz_est"] = round(tot * T / (t_stamp * 1e-6) / 1e6, 1)
        print(json.dumps(res), flush=True)
        del acts, dz, dout, cs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
