"""``run_summarization``-compatible command line (reference ``run_summarization.py:295-367``).

    python -m textsummarization_on_flink_amd.cli --mode=train  --data_path=... --vocab_path=... \\
        --log_root=... --exp_name=... [--coverage=1] [--num_steps=N]
    python -m textsummarization_on_flink_amd.cli --mode=eval   ...
    python -m textsummarization_on_flink_amd.cli --mode=decode ... [--single_pass=1] [--inference=1]

Same flag names/defaults (``config.HParams``), same directory layout
(``<log_root>/<exp_name>/{train,eval,decode*}``), same mode semantics:
  * train: Batcher -> trainer (MI355X hipGraph engine on GPU, oracle on CPU), checkpoints
    every ``save_model_secs``, ``--convert_to_coverage_model`` / ``--restore_best_model``
    one-shot utilities;
  * eval: running-average loss, best-model checkpoints;
  * decode: beam search -> ROUGE files + ROUGE at the end of ``single_pass`` (or attn-vis
    JSON in continuous mode, reloading the checkpoint every 60 s); on a GPU the batched
    device beam search decodes ``decode_batch`` articles at once;
  * ``--inference``: raw text files in, summaries out (``RawTextBatcher``).
Multi-GPU training: launch with ``torchrun --nproc-per-node N`` (one rank per GPU, RCCL).
"""
from __future__ import annotations

import logging
import os
import sys
from typing import Optional, Sequence

import torch

from .config import HParams, check_hps, parse_flags
from .data.batcher import Batcher, RawTextBatcher
from .data.vocab import Vocab
from .parallel.dist import DistInfo, init_from_env
from .utils.logs import setup_logging

log = logging.getLogger("textsummarization_on_flink_amd")


def default_setup(hps: HParams, info: Optional[DistInfo] = None):
    """run_summarization.py:295-330 -> (vocab, hps)."""
    setup_logging(logging.INFO, log_file=hps.log_file or None,
                  rank=info.rank if (info is not None and info.enabled) else None)
    log.info("Starting seq2seq_attention in %s mode...", hps.mode)
    log_root = os.path.join(hps.log_root, hps.exp_name) if hps.exp_name else hps.log_root
    if not os.path.exists(log_root):
        if hps.mode == "train":
            os.makedirs(log_root, exist_ok=True)
        else:
            raise FileNotFoundError("Logdir %s doesn't exist. Run in train mode to create it." % log_root)
    hps = hps.replace(log_root=log_root)
    vocab = Vocab(hps.vocab_path, hps.vocab_size)
    if hps.mode == "decode":
        hps = hps.replace(batch_size=hps.beam_size)
    check_hps(hps)
    torch.manual_seed(hps.seed + (info.rank if info else 0))
    return vocab, hps


def metrics_for(hps, info: Optional[DistInfo] = None):
    from .train.loop import MetricsLogger
    chief = info is None or info.is_chief
    path = hps.metrics_path or (os.path.join(hps.log_root, f"metrics_{hps.mode}.jsonl") if hps.log_root else "")
    tb_dir = None
    if hps.tensorboard and hps.log_root and hps.mode in ("train", "eval") and not hps.inference:
        tb_dir = os.path.join(hps.log_root, hps.mode)  # Supervisor(logdir=train) / eval summary_writer
    return MetricsLogger(path or None, enabled=chief, tb_dir=tb_dir)


def load_params_for_decode(hps, vocab, device, retries: Optional[int] = None):
    from .models.params import build_params
    from .train import checkpoint as ckpt
    params = build_params(hps, vocab.size(), device=device, seed=hps.seed)
    path, step = ckpt.load_ckpt(hps.log_root, params, "train", max_retries=hps.load_retries if retries is None
                                else retries, load_adagrad=False)
    return params, path, step


def build_decoder(hps, vocab, batcher_factory, writer=None, device: Optional[str] = None, decode_dir=None):
    """BeamSearchDecoder over the device beam search (GPU) or the host beam search over
    the oracle step model (CPU).  ``batcher_factory(hps, n_articles, pad_enc_to)``."""
    from .decode.decoder import BeamSearchDecoder
    device = device or ("cuda" if torch.cuda.is_available() else "cpu")
    params, path, _ = load_params_for_decode(hps, vocab, device)
    ckpt_name = "ckpt-" + path.split("-")[-1] if hps.single_pass else None
    if device.startswith("cuda"):
        from .decode.device_beam import DeviceBeamDecoder
        n = max(1, hps.decode_batch)
        dev = DeviceBeamDecoder(hps, vocab, params, n_articles=n, T=hps.max_enc_steps, use_graph=hps.graph)
        batcher = batcher_factory(hps, n, hps.max_enc_steps)

        def reload():
            load_params_into(hps, params)
            dev.refresh_weights()
        return BeamSearchDecoder(None, batcher, vocab, hps, writer=writer, device_beam=dev, ckpt_name=ckpt_name,
                                 html_escape=hps.html_escape, reload_fn=reload, decode_dir=decode_dir)
    from .decode.beam_search import OracleStepModel
    from .models.reference import ReferencePointerGenerator
    from .train.cpu_trainer import _Views
    model = OracleStepModel(ReferencePointerGenerator(hps, vocab.size()), _Views(params, params.flat), hps, device)
    batcher = batcher_factory(hps, 1, None)
    return BeamSearchDecoder(model, batcher, vocab, hps, writer=writer, ckpt_name=ckpt_name,
                             html_escape=hps.html_escape, reload_fn=lambda: load_params_into(hps, params),
                             decode_dir=decode_dir)


def load_params_into(hps, params):
    from .train import checkpoint as ckpt
    ckpt.load_ckpt(hps.log_root, params, "train", max_retries=hps.load_retries, load_adagrad=False)


def loader_workers(hps) -> int:
    """Worker processes of the multi-process input pipeline for GPU training: ``--loader_workers``
    (0 = the threaded Batcher), default (-1) min(8, CPUs - 2).  The threaded Batcher builds
    ~0.7k examples/s under the GIL; the B = 256 step consumes ~12k/s."""
    if hps.mode != "train" or hps.inference or not hps.pad_enc_to_max or torch.cuda.device_count() == 0:
        return 0
    if hps.loader_workers >= 0:
        return hps.loader_workers
    return max(1, min(8, (os.cpu_count() or 4) - 2))


def main(argv: Optional[Sequence[str]] = None) -> int:
    hps = parse_flags(sys.argv[1:] if argv is None else argv, known_only=True)
    loader = None
    nw = loader_workers(hps)
    if nw:
        # fork the loader workers before anything initialises the GPU (init_from_env does
        # under data parallelism); device_count() above does not
        from .data.loader import ProcessBatcher
        # rank-disjoint shares of the records: every rank uses the same seed (the shared
        # file order) and reads the records k with k % WORLD_SIZE == RANK
        rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
        loader = ProcessBatcher(hps.data_path, Vocab(hps.vocab_path, hps.vocab_size), hps,
                                single_pass=hps.single_pass, workers=nw, seed=hps.seed, rank=rank, world=world,
                                pad_enc_to=hps.max_enc_steps)
    info = init_from_env(timeout_s=hps.dist_timeout_s) if hps.mode == "train" else DistInfo()
    vocab, hps = default_setup(hps, info)
    metrics = metrics_for(hps, info)
    try:
        if hps.inference:
            log.info("Inference Mode")
            dec = build_decoder(hps, vocab, lambda h, n, pad: RawTextBatcher(
                h.data_path, vocab, h.replace(batch_size=h.beam_size if n == 1 else n), single_pass=h.single_pass,
                decode_distinct=n > 1, pad_enc_to=pad))
            dec.decode(with_rouge=False)
        elif hps.mode == "train":
            if loader is not None:  # Example/Batch construction in the forked workers
                batcher = loader
            else:
                pad = hps.max_enc_steps if (torch.cuda.device_count() > 0 and hps.pad_enc_to_max) else None
                batcher = Batcher(hps.data_path, vocab, hps, single_pass=hps.single_pass, seed=hps.seed,
                                  pad_enc_to=pad, rank=info.rank, world=info.world)
            from .train.loop import setup_training
            try:
                setup_training(hps, vocab, batcher, info=info, metrics=metrics)
            finally:
                batcher.stop()
        elif hps.mode == "eval":
            batcher = Batcher(hps.data_path, vocab, hps, single_pass=hps.single_pass, seed=hps.seed,
                              pad_enc_to=hps.max_enc_steps if torch.cuda.is_available() else None)
            from .train.loop import run_eval
            run_eval(hps, vocab, batcher, metrics=metrics)
        elif hps.mode == "decode":
            dec = build_decoder(hps, vocab, lambda h, n, pad: Batcher(
                h.data_path, vocab, h.replace(batch_size=h.beam_size if n == 1 else n), single_pass=h.single_pass,
                decode_distinct=n > 1, pad_enc_to=pad))
            res = dec.decode()
            if res is not None:
                log.info("ROUGE: %s", {k: v for k, v in res.items() if k.endswith("f_score")})
        else:
            raise ValueError("The 'mode' flag must be one of train/eval/decode")
    finally:
        metrics.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
