"""Probe: beam-4 decode of a 64-article batch as ONE 64-article decoder vs TWO 32-article decoders
whose captured step graphs run concurrently on two streams (the latency-bound kernels of one half
-- cell, projections, vocab select -- beside the bandwidth-bound attention / vocab logits of the
other).  Random-init weights, synthetic CNN/DM-shaped articles (every batch runs all 100 steps).
Prints one JSON line: summaries/s of each arrangement.

  python tools/decode_dual_probe.py [--batches 4]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=4)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--layers", type=int, default=1)
    ap.add_argument("--enc", type=int, default=400)
    a = ap.parse_args()
    import torch
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
    from textsummarization_on_flink_amd.models.params import build_params

    V = 50000
    res = {"hidden": a.hidden, "layers": a.layers, "enc": a.enc, "batches": a.batches}
    corpus = SyntheticCorpus(vocab_size=V, seed=7)
    vocab = corpus.vocab(V)

    def hp(n):
        return HParams(mode="decode", batch_size=n, beam_size=4, coverage=True, vocab_size=V, hidden_dim=a.hidden,
                       enc_layers=a.layers, max_enc_steps=a.enc)

    params = build_params(hp(64), vocab.size(), device="cuda")
    # one 64-article decoder
    full = make_batches(hp(64), vocab, corpus, a.batches + 1, pad_enc_to=a.enc)
    dec = DeviceBeamDecoder(hp(64), vocab, params, n_articles=64, T=a.enc, keep_attn=False)
    dec.decode(full[0])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in full[1:]:
        dec.decode(b)
    torch.cuda.synchronize()
    res["one_64"] = round(64 * a.batches / (time.perf_counter() - t0), 1)
    del dec
    torch.cuda.empty_cache()
    # two 32-article decoders, concurrent on two streams
    halves = make_batches(hp(32), vocab, corpus, 2 * (a.batches + 1), pad_enc_to=a.enc)
    decs = [DeviceBeamDecoder(hp(32), vocab, params, n_articles=32, T=a.enc, keep_attn=False) for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def pair(ba, bb):
        gens = []
        for d, b, s in zip(decs, (ba, bb), streams):
            s.wait_stream(torch.cuda.current_stream())
            gens.append(d.run_chunks(b))
        alive = [True, True]
        while any(alive):
            for i in range(2):
                if alive[i]:
                    with torch.cuda.stream(streams[i]):
                        try:
                            next(gens[i])
                        except StopIteration:
                            alive[i] = False
        out = []
        for d, s in zip(decs, streams):
            with torch.cuda.stream(s):
                out.append(d.results())
        for s in streams:
            torch.cuda.current_stream().wait_stream(s)
        return out

    for d, b in zip(decs, halves[:2]):  # capture each decoder's graph
        d.decode(b)
    torch.cuda.synchronize()
    pair(halves[0], halves[1])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(1, a.batches + 1):
        pair(halves[2 * i], halves[2 * i + 1])
    torch.cuda.synchronize()
    res["two_32_concurrent"] = round(64 * a.batches / (time.perf_counter() - t0), 1)
    # the same two decoders one after the other (no overlap)
    t0 = time.perf_counter()
    for i in range(1, a.batches + 1):
        decs[0].decode(halves[2 * i])
        decs[1].decode(halves[2 * i + 1])
    torch.cuda.synchronize()
    res["two_32_serial"] = round(64 * a.batches / (time.perf_counter() - t0), 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
