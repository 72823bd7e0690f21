"""Wall-time breakdown of one training step by phase, without profiler distortion.

Builds the bench-shaped engine (defaults: pointer-gen + coverage, H=256, E=128, T=400, D=100,
V=50k, B=256), runs two eager steps so every buffer holds realistic values, then captures each
phase of the step as its own hipGraph and times its replays with HIP events:
encoder forward | decoder forward loop | head forward (+vocab loss) | backward_head |
backward_mid | backward_tail | optimizer.  Prints one JSON line (ms per phase).

  python tools/phase_micro.py [--batch B] [--hidden H] [--enc T] [--layers L]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--enc", type=int, default=400)
    ap.add_argument("--layers", type=int, default=1)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.models.params import build_params
    from textsummarization_on_flink_amd.models.pointer_generator import HipPointerGenerator

    V = 50000
    hps = HParams(batch_size=a.batch, max_enc_steps=a.enc, max_dec_steps=100, vocab_size=V, hidden_dim=a.hidden,
                  emb_dim=128, coverage=True, pointer_gen=True, enc_layers=a.layers)
    corpus = SyntheticCorpus(vocab_size=V, seed=3)
    vocab = corpus.vocab(V)
    batch = make_batches(hps, vocab, corpus, 1, pad_enc_to=a.enc)[0]
    params = build_params(hps, vocab.size(), device="cuda").enable_grad().enable_adagrad(hps.adagrad_init_acc)
    eng = HipPointerGenerator(hps, vocab.size(), params, B=a.batch, T=a.enc)
    eng.set_batch(batch)
    for _ in range(2):
        eng.train_step()
    torch.cuda.synchronize()
    phases = [("encoder_fwd", eng._encoder_forward), ("decoder_fwd", eng._decoder_forward),
              ("head_fwd", lambda: eng._head_forward(True)), ("backward_head", eng.backward_head),
              ("backward_mid", eng.backward_mid), ("backward_tail", eng.backward_tail),
              ("optimizer", eng.optimizer_step)]
    graphs = []
    pool = torch.cuda.graph_pool_handle()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _, fn in phases:  # warm-up on a side stream (allocations settle)
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    from textsummarization_on_flink_amd.utils.graphs import capture_guard
    with capture_guard():
        for _, fn in phases:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                fn()
            graphs.append(g)
    torch.cuda.synchronize()
    res = {"batch": a.batch, "hidden": a.hidden, "enc": a.enc, "layers": a.layers}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(phases) + 1)]
    tot = [0.0] * len(phases)
    for _ in range(a.iters):
        ev[0].record()
        for i, g in enumerate(graphs):
            g.replay()
            ev[i + 1].record()
        torch.cuda.synchronize()
        for i in range(len(phases)):
            tot[i] += ev[i].elapsed_time(ev[i + 1])
    for (n, _), t in zip(phases, tot):
        res[n] = round(t / a.iters, 3)
    res["total"] = round(sum(tot) / a.iters, 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
