"""Beam-4 decode throughput (summaries/s) on MI355X -- BASELINE config #4.

pointer-generator+coverage, hidden 256, emb 128, enc 400, max_dec 100, min_dec 35,
vocab 50k, beam 4, 64 articles per device batch (256 hypothesis rows), random-init
weights, synthetic CNN/DM-shaped articles.  A summary is complete when beam_size
hypotheses reached [STOP] after min_dec_steps or max_dec_steps were run; with random
weights [STOP] is essentially never chosen, so every batch runs all 100 steps (the
worst case).  Timed: encoder + every decode step + host backtracking; excluded: text
tokenisation.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--articles", type=int, default=64)
    ap.add_argument("--beam", type=int, default=4)
    ap.add_argument("--batches", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-pipeline", dest="pipelined", action="store_false",
                    help="decode batch by batch (host backtracking not overlapped with the next batch)")
    ap.add_argument("--vocab", type=int, default=50000)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--layers", type=int, default=1, help="encoder bi-LSTM layers (config #5: 2)")
    ap.add_argument("--enc", type=int, default=400, help="max encoder steps (config #5: 800)")
    ap.add_argument("--unfused-step", action="store_true",
                    help="A/B: the 8-launch decode step (separate beam_step) instead of the fused beam tail")
    args = ap.parse_args()
    import torch
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
    from textsummarization_on_flink_amd.models.params import build_params

    hps = HParams(mode="decode", batch_size=args.articles, beam_size=args.beam, coverage=True, vocab_size=args.vocab,
                  hidden_dim=args.hidden, enc_layers=args.layers, max_enc_steps=args.enc)
    corpus = SyntheticCorpus(vocab_size=args.vocab, seed=7)
    vocab = corpus.vocab(args.vocab)
    batches = make_batches(hps, vocab, corpus, args.batches + args.warmup, pad_enc_to=hps.max_enc_steps)
    params = build_params(hps, vocab.size(), device="cuda")
    dec = DeviceBeamDecoder(hps, vocab, params, n_articles=args.articles, T=hps.max_enc_steps,
                            use_graph=not args.no_graph, keep_attn=False)
    if args.unfused_step:
        dec.fused_step = False
    for b in batches[:args.warmup]:
        dec.decode(b)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    steps = 0
    per = []
    tb = time.perf_counter()
    if args.pipelined:
        # host result backtracking of batch i overlapped with batch i+1 on the GPU
        for hyps in dec.decode_batches(batches[args.warmup:]):
            per.append(time.perf_counter() - tb)
            tb = time.perf_counter()
            n += len(hyps)
            steps += dec.finished_steps
    else:
        for b in batches[args.warmup:]:
            tb = time.perf_counter()
            hyps = dec.decode(b)  # synchronous: results() reads the device buffers
            per.append(time.perf_counter() - tb)
            n += len(hyps)
            steps += dec.steps_run
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"metric": "beam4_summaries_per_sec", "value": round(n / el, 2), "unit": "summaries/s",
                      "n_gpus": 1, "higher_is_better": True, "dtype": "bf16",
                      "data": "synthetic (CNN/DM-shaped, random-init weights)",
                      "ms_per_batch": round(1000 * el / args.batches, 2), "decode_steps_per_batch": steps / args.batches,
                      "ms_per_batch_min": round(1000 * min(per), 2),
                      "ms_per_batch_median": round(1000 * sorted(per)[len(per) // 2], 2),
                      "config": {"model": f"pointer-generator+coverage hidden={args.hidden} emb=128 enc={args.enc} "
                                          f"dec<=100 vocab={args.vocab} enc_layers={args.layers}",
                                 "beam": args.beam, "articles_per_batch": args.articles,
                                 "rows": args.articles * args.beam, "graph": not args.no_graph,
                                 "pipelined": args.pipelined, "fused_step": bool(dec.fused_step)}}))


if __name__ == "__main__":
    main()
