"""Beam-4 decode (64 articles, bench_decode.py's loop) with trained weights instead of random
init: trains ``--train-steps`` GraphTrainer steps on synthetic batches first (0 = random init),
then decodes.  Prints one JSON line; run under rocprofv3 --kernel-trace --stats to see which
decode kernels cost more with trained weights.

  python tools/decode_trained_prof.py --train-steps 80
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--train-steps", type=int, default=80)
    ap.add_argument("--batches", type=int, default=6)
    a = ap.parse_args()
    import torch
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer

    corpus = SyntheticCorpus(vocab_size=50000, seed=11)
    vocab = corpus.vocab(50000)
    hps = HParams(batch_size=256, coverage=True, vocab_size=50000)
    tr = GraphTrainer(hps, vocab.size(), B=256, T=400)
    if a.train_steps:
        tb = make_batches(hps, vocab, corpus, 4, pad_enc_to=400)
        for i in range(a.train_steps):
            out = tr.step(tb[i % 4])
        loss = float(out["loss"])
    else:
        loss = None
    torch.cuda.synchronize()
    params = tr.params
    dh = HParams(mode="decode", batch_size=64, beam_size=4, coverage=True, vocab_size=50000)
    batches = make_batches(dh, vocab, corpus, a.batches + 1, pad_enc_to=400)
    dec = DeviceBeamDecoder(dh, vocab, params, n_articles=64, T=400, keep_attn=False)
    dec.decode(batches[0])
    torch.cuda.synchronize()
    t0, n, steps, stops = time.perf_counter(), 0, 0, 0
    for hyps in dec.decode_batches(batches[1:]):
        n += len(hyps)
        steps += dec.finished_steps
        stops += sum(1 for h in hyps if len(h.tokens) < dh.max_dec_steps + 1)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"train_steps": a.train_steps, "train_loss": loss, "summaries_per_sec": round(n / el, 1),
                      "ms_per_batch": round(1e3 * el / a.batches, 2), "decode_steps_per_batch": steps / a.batches,
                      "summaries_shorter_than_max": stops, "summaries": n}), flush=True)


if __name__ == "__main__":
    main()
