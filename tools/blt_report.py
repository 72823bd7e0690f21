"""What blt_mm's per-shape search picked in a training step: trains a few graph steps at the
bench shape (or config #5 with C5=1), then prints one JSON line per tuned GEMM key:
M, N, K, transposes, hipBLASLt's first heuristic pick's time, the kept pick's time (us).

  python tools/blt_report.py            (B = 256 bench shape)
  C5=1 python tools/blt_report.py       (config #5, batch 1024)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.ops import ops
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer

    c5 = os.environ.get("C5", "0") == "1"
    B, T, H, L = (1024, 800, 512, 2) if c5 else (256, 400, 256, 1)
    hps = HParams(batch_size=B, max_enc_steps=T, max_dec_steps=100, vocab_size=50000, hidden_dim=H, emb_dim=128,
                  coverage=True, pointer_gen=True, enc_layers=L)
    corpus = SyntheticCorpus(vocab_size=50000, seed=1000)
    vocab = corpus.vocab(50000)
    batches = make_batches(hps, vocab, corpus, 2, pad_enc_to=T)
    tr = GraphTrainer(hps, vocab.size(), B=B, T=T, device="cuda:0")
    for i in range(3):
        tr.step(batches[i % 2])
    torch.cuda.synchronize()
    st = list(ops().blt_stats())
    keys, tuned, calls = int(st[0]), int(st[1]), int(st[2])
    rows = [st[3 + 8 * i:3 + 8 * (i + 1)] for i in range(tuned)]
    tot_h = tot_p = 0.0
    for M, N, K, ta, tb, hu, pu, nc in rows:
        tot_h += hu
        tot_p += pu
        print(json.dumps({"M": int(M), "N": int(N), "K": int(K), "ta": int(ta), "tb": int(tb),
                          "heuristic0_us": round(hu, 1), "pick_us": round(pu, 1), "candidates": int(nc)}), flush=True)
    print(json.dumps({"config": "config5" if c5 else "b256", "keys": keys, "tuned": tuned, "calls": calls,
                      "sum_heuristic0_us": round(tot_h, 1), "sum_pick_us": round(tot_p, 1)}), flush=True)


if __name__ == "__main__":
    main()
