"""Find where two deterministic-mode runs diverge (TSAMD_DETERMINISTIC=1).

Builds two engines on the same parameters and batch (B=256, T=400, D=100, V=50k, coverage),
runs forward + backward on each ITERS times (eager, or through GraphTrainer with --graph) and
after every run compares every engine buffer and the parameter gradient bit for bit, printing
the buffers that differ (first differing index and values).  One JSON line per iteration.

  TSAMD_DETERMINISTIC=1 python tools/det_diff.py [--iters 6] [--graph]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--dirty", type=float, default=0.0,
                    help="GB of random junk allocated and freed (not released) before building each engine, so "
                         "uninitialised memory differs between the two")
    a = ap.parse_args()
    os.environ.setdefault("TSAMD_DETERMINISTIC", "1")
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.models.params import build_params
    from textsummarization_on_flink_amd.models.pointer_generator import HipPointerGenerator

    V = 50000
    hps = HParams(batch_size=a.batch, max_enc_steps=400, max_dec_steps=100, vocab_size=V, coverage=True,
                  pointer_gen=True)
    corpus = SyntheticCorpus(vocab_size=V, seed=17)
    vocab = corpus.vocab(V)
    batches = make_batches(hps, vocab, corpus, 3, pad_enc_to=400)
    def junk(i):
        if a.dirty > 0:
            chunks = [torch.full((int(a.dirty * 2 ** 28) // 8,), float(i + 1) * 1e30, device="cuda") for _ in range(8)]
            for c in chunks:
                c[::7] = float("nan")
            del chunks  # back to the caching allocator, not to the driver
    trs, engs = [], []
    for i in range(2):
        junk(i)
        if a.graph:
            from textsummarization_on_flink_amd.train.trainer import GraphTrainer
            trs.append(GraphTrainer(hps, vocab.size(), B=a.batch, T=400, device="cuda:0"))
            engs.append(trs[-1].engine)
        else:
            p = build_params(hps, vocab.size(), device="cuda", seed=3).enable_grad()
            engs.append(HipPointerGenerator(hps, vocab.size(), p, B=a.batch, T=400))
    for it in range(a.iters):
        b = batches[it % len(batches)]
        for i, e in enumerate(engs):
            if a.graph:
                trs[i].step(b)
            else:
                e.set_batch(b)
                e.forward(need_grad=True)
                e.backward()
        torch.cuda.synchronize()
        diffs = []
        for k in sorted(engs[0].w):
            x, y = engs[0].w[k], engs[1].w[k]
            if x is None or not torch.is_tensor(x) or x.shape != y.shape:
                continue
            xv, yv = x.reshape(-1), y.reshape(-1)
            if x.dtype in (torch.float32, torch.bfloat16):
                ne = (xv != yv) & ~(torch.isnan(xv.float()) & torch.isnan(yv.float()))
            else:
                ne = xv != yv
            n = int(ne.sum())
            if n:
                j = int(ne.nonzero()[0])
                diffs.append({"buf": k, "n": n, "first": j, "a": float(xv[j]), "b": float(yv[j])})
        gx, gy = engs[0].p.grad, engs[1].p.grad
        ng = int((gx != gy).sum())
        if ng:
            j = int((gx != gy).nonzero()[0])
            names = [n for n, (o, c) in engs[0].p.offsets.items() if o <= j < o + c]
            diffs.append({"buf": "grad", "n": ng, "first": j, "param": names[0] if names else None})
        print(json.dumps({"iter": it, "graph": a.graph, "ndiff": len(diffs), "diffs": diffs[:12]}), flush=True)


if __name__ == "__main__":
    main()
