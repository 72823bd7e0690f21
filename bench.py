"""Headline benchmark: pointer-generator (+coverage) training throughput on MI355X, plus the
beam-4 decode throughput as a secondary field of the same JSON line.

Metric (BASELINE.json / BASELINE.md): train tokens/sec for the whole job = sum over
ranks of non-pad encoder tokens (enc_lens) + non-pad decoder tokens (dec_padding_mask)
per optimizer step / steady-state wall time per step.  Config: hidden 256, emb 128,
enc 400 -> dec 100, vocab 50k, pointer-gen with coverage loss, bf16 compute (fp32 master
weights + Adagrad accumulators), synthetic CNN/DM-shaped data, random-init weights.
Weak scaling: the per-GPU batch is fixed, global batch = batch x N.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]

Multi-GPU: one process per GPU, torch.distributed over RCCL (backend "nccl"), gradients
all-reduced in four buckets overlapped with the backward.  Either launch it with
``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`` (RANK /
WORLD_SIZE / MASTER_* come from the environment), or run ``python bench.py --gpus N``
directly: without WORLD_SIZE in the environment this process starts the N rank processes
itself (torchrun-style env, rendezvous on 127.0.0.1) before anything touches the GPU,
relays their output and exits with the worst exit code.  ``n_gpus`` in the JSON is the
world size the process group reports.

Timed region per step: H2D copy of the batch, forward + backward (four phase-graph
replays), gradient all-reduce (RCCL), clip + Adagrad + weight repack (the optimizer hipGraph)
-- the complete optimizer step; only synthetic text generation/tokenisation is done ahead
of time (like a prefetching loader).  The W warmup steps include the graph captures.

Secondary (BASELINE config #4, ``beam4_summaries_per_sec``): after the training timing,
every rank decodes ``--decode-batches`` batches of 64 articles x beam 4 (hipGraph-captured
device beam search, fresh random-init weights, encoder included, host backtracking
included, tokenisation excluded); the value is the sum over ranks of completed summaries
divided by the slowest rank's wall time.  ``--decode-batches 0`` skips it.

Secondary (BASELINE config #5, ``config5_tokens_per_sec`` / ``config5_beam4_summaries_per_sec``):
hidden 512, 2-layer encoder, enc 800, per-GPU batch sized for the GPU's HBM (the largest of
2048 / 1024 / 512 whose captured step fits EVERY rank, agreed before any gradient collective;
``config5_peak_mem_gb`` reports the footprint), ``--config5-steps`` timed steps after two warm-up
steps (graph capture + one replay of the other batch), the same timed region as the headline;
then 8 beam-4 decode batches at that size.  ``--config5-steps 0`` skips it.
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BASELINE_TOKENS_PER_S = 6700.0  # See et al. 2017 on a K40m, <=6.7k tokens/s


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", default="256", help="per-GPU batch (rows), or 'auto': the largest of 2048/1024/512/256/128 "
                                                   "whose training step fits every rank's GPU memory (config #5 sizing)")
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
    ap.add_argument("--grad-compress", default="none", choices=("none", "bf16"),
                    help="gradient all-reduce wire format (fp32 master weights either way)")
    ap.add_argument("--decode-batches", type=int, default=10, help="timed beam-4 decode batches (0 = skip)")
    ap.add_argument("--decode-articles", type=int, default=64)
    ap.add_argument("--port", type=int, default=0, help="rendezvous port when launching ranks (0 = free port)")
    ap.add_argument("--config5-steps", type=int, default=10,
                    help="BASELINE config #5 (hidden 512, 2-layer encoder, enc 800, the HBM-sized per-GPU batch) timed "
                         "train steps + 4 beam-4 decode batches, reported as config5_* fields (0 = skip).  Every step "
                         "packs its batch on the host; the first one's pack (~40 ms at batch 2048) has no GPU work "
                         "to hide behind, so 10 steps rather than 5 keep that start-up cost from reading as ~7 ms/step")
    return ap.parse_args(argv)


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv, port: int = 0) -> int:
    """Start ``n`` rank processes of this script (one per GPU) and wait for them.  Runs
    before anything initialises the GPU in this process (torch is not even imported)."""
    from textsummarization_on_flink_amd.parallel.rccl_env import rccl_env  # torch-free
    port = port or _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        rccl_env(env)  # RCCL's CU cap before the rank touches the GPU (parallel/rccl_env.py)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0:
                    rc = rc or code
                    for q in procs:  # one rank failed: the others would block in a collective
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


def _timed(fn, info, D, torch):
    torch.cuda.synchronize()
    D.barrier(info)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = fn()
    torch.cuda.synchronize()
    D.barrier(info)
    torch.cuda.synchronize()
    return res, time.perf_counter() - t0


def main(argv=None):
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus, sys.argv[1:] if argv is None else list(argv), args.port)

    import torch
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.parallel import dist as D
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer

    info = D.init_from_env(backend=args.backend)
    if info.enabled:
        assert torch.distributed.get_world_size() == info.world
    if info.world != args.gpus:
        print(f"warning: --gpus {args.gpus} but the process group has {info.world} ranks", file=sys.stderr)
    dev_id = info.local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_id)
    hps = HParams(batch_size=256 if args.batch == "auto" else int(args.batch), max_enc_steps=args.enc, max_dec_steps=args.dec, vocab_size=args.vocab,
                  hidden_dim=args.hidden, emb_dim=args.emb, coverage=not args.no_coverage, pointer_gen=True,
                  enc_layers=args.layers, grad_compress=args.grad_compress)
    corpus = SyntheticCorpus(vocab_size=args.vocab, seed=1000 + info.rank)
    vocab = corpus.vocab(args.vocab)
    if args.batch == "auto":
        B = pick_batch(args, hps, vocab, corpus, info, D, torch, dev_id)
    else:
        B = int(args.batch)
    args.batch = B
    hps = hps.replace(batch_size=B)
    batches = make_batches(hps, vocab, corpus, args.pool, pad_enc_to=args.enc)
    tr = GraphTrainer(hps, vocab.size(), B=B, T=args.enc, device=f"cuda:{dev_id}", info=info,
                      use_graph=not args.no_graph)

    for i in range(args.warmup):
        out = tr.step(batches[i % len(batches)])
    if args.warmup:
        tr.check_finite(out)

    def train_loop():
        tokens = padded = 0
        o = None
        for i in range(args.steps):
            b = batches[i % len(batches)]
            o = tr.step(b)
            tokens += b.num_tokens()
            padded += b.padded_tokens()
        return o, tokens, padded

    (out, tokens, padded), elapsed = _timed(train_loop, info, D, torch)
    vals = tr.check_finite(out)
    elapsed_max = D.all_reduce_scalar(elapsed, info, op="max", device=tr.device)
    elapsed_min = D.all_reduce_scalar(elapsed, info, op="min", device=tr.device)
    # diagnostics, after the timed region: per-phase wall time of a few more steps (HIP events
    # between the phase graphs; ms_allreduce = the all-reduce wait exposed after the backward)
    tr.timing = True
    ph = {}
    nph = 3
    for i in range(nph):
        tr.step(batches[i % len(batches)])
        for k_, v_ in tr.phase_ms().items():
            ph[k_] = ph.get(k_, 0.0) + v_ / nph
    tr.timing = False
    ph = {k_: round(D.all_reduce_scalar(v_, info, op="max", device=tr.device), 3) for k_, v_ in ph.items()}
    tok_all = D.all_reduce_scalar(float(tokens), info, op="sum", device=tr.device)
    pad_all = D.all_reduce_scalar(float(padded), info, op="sum", device=tr.device)
    value = tok_all / elapsed_max

    dec = None
    if args.decode_batches > 0:
        dec = bench_decode(args, info, D, torch, dev_id)
    peak_gb = torch.cuda.max_memory_allocated() / 2 ** 30
    eng_flags = {"persistent_lstm": bool(tr.engine.persistent_lstm), "proj_attn": bool(tr.engine.proj_attn),
                 "skip_pad_steps": bool(tr.engine.skip_pad), "decoder_row_groups": int(tr.engine.split)}
    from textsummarization_on_flink_amd.models import pointer_generator as _pg
    if _pg.BLT:  # library GEMMs through blt_mm: GEMM shapes seen / given a timed candidate search
        st = tr.engine.k.blt_stats()
        eng_flags["blt_mm"] = {"keys": int(st[0]), "tuned": int(st[1])}
    # which activation GEMMs ran on the hand-written kernel (fixed table, not per-run timing)
    eng_flags["gemm_dispatch"] = _pg.gemm_bt_stats()
    c5 = None
    if args.config5_steps > 0 and args.hidden != 512:
        del tr, batches
        torch.cuda.empty_cache()
        # no rank-local OOM handling here: bench_config5 agrees on a batch that fits every rank
        # before any collective (a rank that skipped alone would leave its peers in an all-reduce)
        c5 = bench_config5(args, info, D, torch, dev_id)

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
                "backend": info.backend if info.enabled else "none",
                "grad_allreduce": ("bf16" if args.grad_compress == "bf16" else "fp32") if info.enabled else "none",
                "padded_tokens_per_sec": round(pad_all / elapsed_max, 1),
                "ms_per_step_rank_min": round(1000.0 * elapsed_min / args.steps, 3),
                "ms_allreduce_exposed": ph.get("ms_allreduce"),
                "phase_ms_max_over_ranks": ph,
                "loss": round(vals.get("total_loss", float("nan")), 4),
                "graph": not args.no_graph,
                # projected-context attention and skipped dead decoder steps (loss and gradients
                # unchanged; the metric counts non-pad tokens either way): README "Performance"
                **eng_flags,
                "peak_mem_gb": round(peak_gb, 1),
                "gpu_mem_gb": round(torch.cuda.get_device_properties(dev_id).total_memory / 2 ** 30, 1),
            },
        }
        if dec is not None:
            rec.update(dec)
        if c5 is not None:
            rec.update(c5)
        print(json.dumps(rec), flush=True)
    if info.enabled:
        torch.distributed.destroy_process_group()
    return 0


AUTO_BATCHES = (2048, 1024, 512, 256, 128)


def _oom_type():
    import torch
    return torch.cuda.OutOfMemoryError


def agree_largest(cands, trial, info, D, device):
    """Rank-agreed capacity search: ``trial(c)`` runs rank-locally (no collectives inside) for
    each candidate, largest first; a ``torch.cuda.OutOfMemoryError`` (and only that: any other
    error is real) marks it as not fitting on this rank.  The ranks all-reduce MIN of their
    success flags after each trial, so every rank returns the same ``(c, trial result)`` -- or
    ``(None, None)`` when no candidate fits everywhere -- before any gradient collective runs.
    A rank never skips or falls back on its own."""
    oom = _oom_type()
    for c in cands:
        res, ok = None, 1.0
        try:
            res = trial(c)
        except oom as e:
            print(f"capacity search: {c} does not fit ({str(e).splitlines()[0][:120]})", file=sys.stderr)
            ok = 0.0
        _empty_cache()
        if D.all_reduce_scalar(ok, info, op="min", device=device) > 0:
            return c, res
        res = None
        _empty_cache()
    return None, None


def _empty_cache():
    import torch
    if torch.cuda.is_available():
        torch.cuda.empty_cache()


def pick_batch(args, hps, vocab, corpus, info, D, torch, dev_id) -> int:
    """``--batch auto``: the largest per-GPU batch whose captured training step fits EVERY
    rank's memory (``agree_largest``: a trainer without collectives, one captured step per
    candidate); the smallest candidate if none does."""
    from textsummarization_on_flink_amd.data.synthetic import make_batches
    from textsummarization_on_flink_amd.parallel.dist import DistInfo
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer

    def trial(B):
        h = hps.replace(batch_size=B)
        b = make_batches(h, vocab, corpus, 1, pad_enc_to=args.enc)[0]
        tr = GraphTrainer(h, vocab.size(), B=B, T=args.enc, device=f"cuda:{dev_id}", info=DistInfo(),
                          use_graph=not args.no_graph)
        tr.step(b)  # graph capture included: the peak allocation happens here
        torch.cuda.synchronize()
        return None

    B, _ = agree_largest(AUTO_BATCHES, trial, info, D, f"cuda:{dev_id}")
    return B if B is not None else AUTO_BATCHES[-1]


CONFIG5 = dict(hidden=512, layers=2, enc=800)  # BASELINE.json config #5 (run_summarization.py:62-66)
CONFIG5_BATCHES = (2048, 1024, 512)            # "batch sized for 288 GB HBM": the largest that fits


def bench_config5(args, info, D, torch, dev_id):
    """BASELINE config #5 on the same clock as the headline: hidden 512, 2-layer bi-LSTM encoder,
    enc 800 -> dec 100, the largest per-GPU batch of CONFIG5_BATCHES whose captured step fits every
    rank (weak scaling), same timed region as the headline (H2D, phase-graph replays, all-reduce,
    optimizer graph); then 4 batches of 64-article beam-4 decode at that size.

    The batch is found by ``agree_largest`` before any collective: each rank captures a trainer
    without collectives at the candidate size (its two warm-up steps); on one rank that trainer is
    the timed one, on several ranks the data-parallel trainer is built at the agreed size."""
    import argparse as _ap
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.parallel.dist import DistInfo
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer
    c = CONFIG5
    hps = HParams(batch_size=CONFIG5_BATCHES[0], max_enc_steps=c["enc"], max_dec_steps=args.dec,
                  vocab_size=args.vocab, hidden_dim=c["hidden"], emb_dim=args.emb, coverage=not args.no_coverage,
                  pointer_gen=True, enc_layers=c["layers"], grad_compress=args.grad_compress)
    corpus = SyntheticCorpus(vocab_size=args.vocab, seed=2000 + info.rank)
    vocab = corpus.vocab(args.vocab)
    dev = f"cuda:{dev_id}"
    torch.cuda.reset_peak_memory_stats(dev_id)

    def warm(tr, batches):
        out = None
        for b in batches:  # warm-up: graph capture, then a replay of each batch (each live-row bucket's head graph)
            out = tr.step(b)
        tr.check_finite(out)

    def trial(B):
        h = hps.replace(batch_size=B)
        batches = make_batches(h, vocab, corpus, 2, pad_enc_to=c["enc"])
        tr = GraphTrainer(h, vocab.size(), B=B, T=c["enc"], device=dev, info=DistInfo(), use_graph=not args.no_graph)
        warm(tr, batches)
        torch.cuda.synchronize()
        return (tr if not info.enabled else None), batches

    B, got = agree_largest(CONFIG5_BATCHES, trial, info, D, dev)
    if B is None:
        return {"config5_error": f"no per-GPU batch of {CONFIG5_BATCHES} fits every rank"}
    tr, batches = got
    if tr is None:  # data parallel: the trial trainer had no collectives
        tr = GraphTrainer(hps.replace(batch_size=B), vocab.size(), B=B, T=c["enc"], device=dev, info=info,
                          use_graph=not args.no_graph)
        warm(tr, batches)
    n_warm = len(batches)
    # the footprint of the CHOSEN batch: the capacity search's peak also holds larger candidates'
    # partial allocations and the freed trial trainer (reported apart)
    trial_peak = torch.cuda.max_memory_allocated(dev_id) / 2 ** 30
    torch.cuda.reset_peak_memory_stats(dev_id)

    def loop():
        tokens = 0
        o = None
        for i in range(args.config5_steps):
            b = batches[(i + 1) % 2]
            o = tr.step(b)
            tokens += b.num_tokens()
        return o, tokens

    (out, tokens), el = _timed(loop, info, D, torch)
    tr.check_finite(out)
    el_max = D.all_reduce_scalar(el, info, op="max", device=tr.device)
    tok_all = D.all_reduce_scalar(float(tokens), info, op="sum", device=tr.device)
    peak = D.all_reduce_scalar(torch.cuda.max_memory_allocated(dev_id) / 2 ** 30, info, op="max", device=tr.device)
    del tr, batches
    torch.cuda.empty_cache()
    rec = {"config5_tokens_per_sec": round(tok_all / el_max, 1),
           "config5_ms_per_step": round(1000.0 * el_max / args.config5_steps, 3),
           "config5_peak_mem_gb": round(peak, 1),
           "config5_search_peak_mem_gb": round(D.all_reduce_scalar(trial_peak, info, op="max", device=dev), 1),
           "config5_config": {"model": f"pointer-generator+coverage hidden={c['hidden']} emb={args.emb} "
                                       f"enc={c['enc']} dec={args.dec} vocab={args.vocab} enc_layers={c['layers']}",
                              "per_gpu_batch": B, "global_batch": B * info.world,
                              "batch_sizing": f"largest of {list(CONFIG5_BATCHES)} whose step fits every rank",
                              "steps": args.config5_steps, "warmup": n_warm}}
    if args.decode_batches > 0:
        # 8 batches (4 before round 6): the decoder encodes up to 8 queued batches in one pass
        # (decode/device_beam.py group_enc), so a 4-batch run padded half of that pass
        a5 = _ap.Namespace(**{**vars(args), "hidden": c["hidden"], "layers": c["layers"], "enc": c["enc"],
                              "decode_batches": 8})
        d5 = bench_decode(a5, info, D, torch, dev_id)
        rec["config5_beam4_summaries_per_sec"] = d5["beam4_summaries_per_sec"]
        rec["config5_beam4_ms_per_batch"] = d5["beam4_ms_per_batch"]
    return rec


def bench_decode(args, info, D, torch, dev_id):
    """Beam-4 decode, config #4 (64 articles x beam 4 per batch), on every rank."""
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
    from textsummarization_on_flink_amd.models.params import build_params

    hps = HParams(mode="decode", batch_size=args.decode_articles, beam_size=4, coverage=not args.no_coverage,
                  vocab_size=args.vocab, hidden_dim=args.hidden, emb_dim=args.emb, max_enc_steps=args.enc,
                  max_dec_steps=args.dec, enc_layers=args.layers)
    corpus = SyntheticCorpus(vocab_size=args.vocab, seed=7 + info.rank)
    vocab = corpus.vocab(args.vocab)
    pool = make_batches(hps, vocab, corpus, 3, pad_enc_to=hps.max_enc_steps)
    params = build_params(hps, vocab.size(), device=f"cuda:{dev_id}")
    dec = DeviceBeamDecoder(hps, vocab, params, n_articles=args.decode_articles, T=hps.max_enc_steps,
                            use_graph=not args.no_graph, keep_attn=False)
    dec.decode(pool[0])  # warm-up: graph capture

    def loop():
        # pipelined: batch i's host backtracking runs while batch i+1 is on the GPU; the loop
        # ends when the last batch's results are on the host
        n = steps = 0
        for hyps in dec.decode_batches([pool[1 + i % 2] for i in range(args.decode_batches)]):
            n += len(hyps)
            steps += dec.finished_steps
        return n, steps

    (n, steps), el = _timed(loop, info, D, torch)
    el_max = D.all_reduce_scalar(el, info, op="max", device=f"cuda:{dev_id}")
    n_all = D.all_reduce_scalar(float(n), info, op="sum", device=f"cuda:{dev_id}")
    return {"beam4_summaries_per_sec": round(n_all / el_max, 1),
            "beam4_ms_per_batch": round(1000.0 * el_max / args.decode_batches, 3),
            "beam4_config": {"articles_per_batch": args.decode_articles, "beam": 4, "batches": args.decode_batches,
                             "decode_steps_per_batch": steps / args.decode_batches, "min_dec_steps": hps.min_dec_steps,
                             "max_dec_steps": hps.max_dec_steps, "graph": not args.no_graph}}


if __name__ == "__main__":
    sys.exit(main())
