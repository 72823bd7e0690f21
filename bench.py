"""Headline benchmark: pointer-generator (+coverage) training throughput on MI355X.

Metric (BASELINE.json / BASELINE.md): train tokens/sec for the whole job = sum over
ranks of non-pad encoder tokens (enc_lens) + non-pad decoder tokens (dec_padding_mask)
per optimizer step / steady-state wall time per step.  Config: hidden 256, emb 128,
enc 400 -> dec 100, vocab 50k, pointer-gen with coverage loss, bf16 compute (fp32 master
weights + Adagrad accumulators), synthetic CNN/DM-shaped data, random-init weights.
Weak scaling: the per-GPU batch is fixed, global batch = batch x N.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
       (N > 1 is launched by torch.distributed.run; one rank per GPU, RCCL all-reduce.)

Timed region per step: H2D copy of the batch, forward + backward (one hipGraph replay),
gradient all-reduce (RCCL), clip + Adagrad + weight repack (second hipGraph) -- i.e. the
complete optimizer step; only synthetic text generation/tokenisation is done ahead of
time (like a prefetching loader).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BASELINE_TOKENS_PER_S = 6700.0  # See et al. 2017 on a K40m, <=6.7k tokens/s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch (rows); 256 keeps the persistent LSTM grid at 128 of 256 CUs so the overlapped RCCL all-reduce always finds free CUs")
    ap.add_argument("--no-coverage", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--pool", type=int, default=4, help="distinct synthetic batches cycled per rank")
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--emb", type=int, default=128)
    ap.add_argument("--enc", type=int, default=400)
    ap.add_argument("--dec", type=int, default=100)
    ap.add_argument("--vocab", type=int, default=50000)
    ap.add_argument("--layers", type=int, default=1, help="stacked bi-LSTM encoder layers (config #5: 2)")
    ap.add_argument("--backend", default=None, help="process-group backend override (default nccl = RCCL; gloo "
                                                    "lets several ranks share one GPU for a plumbing check)")
    args = ap.parse_args()

    import torch
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.parallel import dist as D
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer

    info = D.init_from_env(backend=args.backend)
    if info.world != args.gpus and not (info.world == 1 and args.gpus == 1):
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={info.world}", file=sys.stderr)
    dev_id = info.local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_id)
    hps = HParams(batch_size=args.batch, max_enc_steps=args.enc, max_dec_steps=args.dec, vocab_size=args.vocab,
                  hidden_dim=args.hidden, emb_dim=args.emb, coverage=not args.no_coverage, pointer_gen=True,
                  enc_layers=args.layers)
    corpus = SyntheticCorpus(vocab_size=args.vocab, seed=1000 + info.rank)
    vocab = corpus.vocab(args.vocab)
    batches = make_batches(hps, vocab, corpus, args.pool, pad_enc_to=args.enc)
    tr = GraphTrainer(hps, vocab.size(), B=args.batch, T=args.enc, device=f"cuda:{dev_id}", info=info,
                      use_graph=not args.no_graph)

    for i in range(args.warmup):
        out = tr.step(batches[i % len(batches)])
    if args.warmup:
        tr.check_finite(out)
    torch.cuda.synchronize()
    D.barrier(info)
    torch.cuda.synchronize()
    tokens = 0
    padded = 0
    t0 = time.perf_counter()
    for i in range(args.steps):
        b = batches[i % len(batches)]
        out = tr.step(b)
        tokens += b.num_tokens()
        padded += b.padded_tokens()
    torch.cuda.synchronize()
    D.barrier(info)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    vals = tr.check_finite(out)
    elapsed_max = D.all_reduce_scalar(elapsed, info, op="max", device=tr.device)
    tok_all = D.all_reduce_scalar(float(tokens), info, op="sum", device=tr.device)
    pad_all = D.all_reduce_scalar(float(padded), info, op="sum", device=tr.device)
    value = tok_all / elapsed_max
    if info.is_chief:
        rec = {
            "metric": "train_tokens_per_sec",
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": info.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed_max / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_TOKENS_PER_S, 2),
            "dtype": "bf16",
            "data": "synthetic (CNN/DM-shaped, random-init weights)",
            "config": {
                "model": f"pointer-generator{'+coverage' if hps.coverage else ''} hidden={hps.hidden_dim} "
                         f"emb={hps.emb_dim} enc={hps.max_enc_steps} dec={hps.max_dec_steps} vocab={hps.vocab_size}"
                         + (f" enc_layers={hps.enc_layers}" if hps.enc_layers > 1 else ""),
                "global_batch": args.batch * info.world,
                "per_gpu_batch": args.batch,
                "seq_len": f"{hps.max_enc_steps}->{hps.max_dec_steps}",
                "parallelism": f"dp{info.world}",
                "padded_tokens_per_sec": round(pad_all / elapsed_max, 1),
                "loss": round(vals.get("total_loss", float("nan")), 4),
                "graph": not args.no_graph,
            },
        }
        print(json.dumps(rec), flush=True)
    if info.enabled:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
