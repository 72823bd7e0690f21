"""Prototype A/B: one DeviceBeamDecoder over 64-article batches against two decoders over
32-article halves, each on its own HIP stream and host thread, so one half's kernels fill the
other's launch gaps.  Prints one JSON line per variant (summaries/s).

  python tools/decode_split_proto.py [--batches 8]
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--articles", type=int, default=64)
    a = ap.parse_args()
    import torch
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
    from textsummarization_on_flink_amd.models.params import build_params

    NA = a.articles
    corpus = SyntheticCorpus(vocab_size=50000, seed=7)
    vocab = corpus.vocab(50000)
    hps = HParams(mode="decode", batch_size=NA, beam_size=4, coverage=True, vocab_size=50000)
    params = build_params(hps, vocab.size(), device="cuda")
    full = make_batches(hps, vocab, corpus, a.batches + 1, pad_enc_to=hps.max_enc_steps)
    hh = hps.replace(batch_size=NA // 2)
    halves = [make_batches(hh, vocab, SyntheticCorpus(vocab_size=50000, seed=70 + i), a.batches + 1,
                           pad_enc_to=hps.max_enc_steps) for i in range(2)]

    def one():
        dec = DeviceBeamDecoder(hps, vocab, params, n_articles=NA, T=hps.max_enc_steps, keep_attn=False)
        dec.decode(full[0])
        torch.cuda.synchronize()
        t0, n = time.perf_counter(), 0
        for hyps in dec.decode_batches(full[1:]):
            n += len(hyps)
        torch.cuda.synchronize()
        return n / (time.perf_counter() - t0)

    def split():
        decs = [DeviceBeamDecoder(hh, vocab, params, n_articles=NA // 2, T=hps.max_enc_steps, keep_attn=False)
                for _ in range(2)]
        streams = [torch.cuda.Stream() for _ in range(2)]
        for d, s, bs in zip(decs, streams, halves):
            with torch.cuda.stream(s):
                d.decode(bs[0])
        torch.cuda.synchronize()
        counts = [0, 0]
        go = threading.Barrier(3)

        def work(i):
            with torch.cuda.stream(streams[i]):
                go.wait()
                for hyps in decs[i].decode_batches(halves[i][1:]):
                    counts[i] += len(hyps)
                streams[i].synchronize()

        th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
        for t in th:
            t.start()
        go.wait()
        t0 = time.perf_counter()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        return sum(counts) / (time.perf_counter() - t0)

    for name, fn in (("one_decoder", one), ("two_halves_two_streams", split), ("one_decoder", one),
                     ("two_halves_two_streams", split)):
        print(json.dumps({"variant": name, "summaries_per_sec": round(fn(), 1), "articles": NA,
                          "batches": a.batches}), flush=True)


if __name__ == "__main__":
    main()
