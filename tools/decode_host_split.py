"""Where a beam-4 decode batch's wall time goes (64 articles, bench config #4 shape): host time
spent queueing the encoder + decode chunks (run), the GPU tail still running when run returns,
and the host result fetch + backtracking (results).  Prints one line per batch.

  python tools/decode_host_split.py [--batches 4]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=4)
    a = ap.parse_args()
    import torch
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
    from textsummarization_on_flink_amd.models.params import build_params
    hps = HParams(mode="decode", batch_size=64, beam_size=4, coverage=True, vocab_size=50000)
    corpus = SyntheticCorpus(vocab_size=50000, seed=7)
    vocab = corpus.vocab(50000)
    batches = make_batches(hps, vocab, corpus, a.batches + 1, pad_enc_to=hps.max_enc_steps)
    params = build_params(hps, vocab.size(), device="cuda")
    dec = DeviceBeamDecoder(hps, vocab, params, n_articles=64, T=hps.max_enc_steps, keep_attn=False)
    dec.decode(batches[0])
    torch.cuda.synchronize()
    for b in batches[1:]:
        t0 = time.perf_counter()
        dec.run(b)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        dec.results(64)
        t3 = time.perf_counter()
        print(f"run (host queueing) {1e3 * (t1 - t0):.2f} ms, GPU tail {1e3 * (t2 - t1):.2f} ms, "
              f"results {1e3 * (t3 - t2):.2f} ms, total {1e3 * (t3 - t0):.2f} ms", flush=True)


if __name__ == "__main__":
    main()
