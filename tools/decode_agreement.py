"""Agreement of the device beam search (bf16 kernels) with the host beam search over the fp32
oracle, at the production width (H=256, E=128) and small T / V, for a few init scales:
prints one JSON line per setting with the number of articles whose full summary (and whose
first 6 / 12 tokens) match.  Diagnostic for choosing test thresholds: bf16 rounding flips
beams at near-ties, which random weights produce more often the flatter the init.

  python tools/decode_agreement.py [--articles 10] [--steps 24]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--articles", type=int, default=10)
    ap.add_argument("--steps", type=int, default=24)
    a = ap.parse_args()
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.batch import Batch, Example
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.decode.beam_search import OracleStepModel, run_beam_search
    from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
    from textsummarization_on_flink_amd.models.params import build_params
    from textsummarization_on_flink_amd.models.reference import ReferencePointerGenerator
    Na, T, V = a.articles, 64, 2000
    for std, mag in ((0.5, 0.3), (1.0, 0.5), (2.0, 1.0)):
        for cov in (True, False):
            hps = HParams(batch_size=Na, max_enc_steps=T, max_dec_steps=a.steps, min_dec_steps=3, beam_size=4,
                          vocab_size=V, emb_dim=128, hidden_dim=256, coverage=cov, pointer_gen=True,
                          trunc_norm_init_std=std, rand_unif_init_mag=mag)
            corpus = SyntheticCorpus(vocab_size=V, raw_vocab=3 * V, seed=5, art_mean=50, art_sd=10, sent_mean=4)
            vocab = corpus.vocab(V)
            batch = make_batches(hps, vocab, corpus, 1, pad_enc_to=T)[0]
            params = build_params(hps, vocab.size(), device="cuda", seed=4)
            hyps = DeviceBeamDecoder(hps, vocab, params, n_articles=Na, T=T, use_graph=True).decode(batch)
            W = {n: params.flat[o:o + c].view(params.view(n).shape) for n, (o, c) in params.offsets.items()}
            model = OracleStepModel(ReferencePointerGenerator(hps, vocab.size()), W, hps, device="cuda")
            hps1 = hps.replace(batch_size=hps.beam_size)
            full = p6 = p12 = 0
            lens = []
            for i in range(Na):
                ex = Example(batch.original_articles[i], batch.original_abstracts_sents[i], vocab, hps1)
                ref = run_beam_search(model, vocab, Batch([ex] * 4, hps1, vocab, pad_enc_to=T), hps).tokens
                got = hyps[i].tokens
                full += ref == got
                p6 += ref[:6] == got[:6]
                p12 += ref[:12] == got[:12]
                lens.append(len(ref))
            print(json.dumps({"init_std": std, "unif_mag": mag, "coverage": cov, "articles": Na, "full": full,
                              "prefix6": p6, "prefix12": p12, "mean_len": sum(lens) / Na}), flush=True)


if __name__ == "__main__":
    main()
