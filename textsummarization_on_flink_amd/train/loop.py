"""Train / eval loops, backend selection, metrics and fault injection
(reference ``run_summarization.py:105-292``, ``train.py:57-125``).

* ``make_trainer``: the MI355X ``GraphTrainer`` when a GPU is present, else the oracle
  ``CpuTrainer`` -- same interface, so these loops are backend-agnostic.
* ``run_training``: batch -> step -> log -> NaN guard -> metrics; checkpoints on the chief
  every ``save_model_secs`` (Supervisor, ``run_summarization.py:192-200``) and at exit;
  ``num_steps`` counts steps relative to the restored step (``StopAtStepHook``,
  ``train.py:78``); ``KeyboardInterrupt`` saves and stops.
* ``run_eval``: reload latest train checkpoint, eval loss, ``running_avg_loss`` (decay
  0.99, clipped at 12) and keep the 3 best as ``eval/bestmodel-<step>`` with the
  ``checkpoint_best`` state file.
* ``MetricsLogger``: structured JSONL (step, loss, coverage_loss, global_norm, tokens/s,
  step_ms) -- replaces TensorBoard summaries (``model.py:270-300``).
* ``--debug``: ``NonFiniteWatch`` scans parameters, gradients and activations after every
  step and stops with a report of the non-finite tensors (tfdbg ``has_inf_or_nan``,
  ``run_summarization.py:216-218``).
* fault injection (``hps.fault_nan_step`` / ``hps.fault_kill_step`` + ``fault_kill_rank``):
  a NaN gradient at step k (exercises the device NaN guard and the "Loss is not finite"
  stop) or a hard exit of one rank (exercises restart-from-latest).
"""
from __future__ import annotations

import json
import logging
import os
import time
from typing import Dict, Optional

import torch

from ..parallel.dist import DistInfo, all_reduce_scalar, barrier, broadcast_params, broadcast_scalar
from ..utils.debug import NonFiniteWatch
from . import checkpoint as ckpt
from .trainer import NonFiniteLossError

log = logging.getLogger(__name__)


class MetricsLogger:
    """JSONL metrics plus (optionally) TensorBoard scalars in ``tb_dir`` -- the reference's
    summary tags: ``loss``, ``coverage_loss``, ``total_loss``, ``global_norm`` (train,
    ``model.py:270-300``) and ``running_avg_loss/decay=0.990000`` (eval,
    ``run_summarization.py:124-127``); flushed every 100 records (``:243-244``)."""

    TB_RENAME = {"eval_loss": "loss", "running_avg_loss": "running_avg_loss/decay=0.990000"}

    def __init__(self, path: Optional[str], enabled: bool = True, tb_dir: Optional[str] = None):
        self.path = path if enabled else None
        self._f = None
        if self.path:
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
            self._f = open(self.path, "a", buffering=1)
        self._tb = None
        self._n = 0
        if tb_dir and enabled:
            from ..utils.tensorboard import EventWriter
            self._tb = EventWriter(tb_dir)

    def log(self, **kv):
        if self._f:
            kv.setdefault("time", time.time())
            self._f.write(json.dumps(kv, sort_keys=True) + "\n")
        if self._tb is not None and "step" in kv:
            sc = {self.TB_RENAME.get(k, k): float(v) for k, v in kv.items()
                  if k not in ("step", "time") and isinstance(v, (int, float)) and not isinstance(v, bool)}
            self._tb.add_scalars(int(kv["step"]), sc)
            self._n += 1
            if self._n % 100 == 0:
                self._tb.flush()

    def close(self):
        if self._f:
            self._f.close()
            self._f = None
        if self._tb is not None:
            self._tb.close()
            self._tb = None


def make_trainer(hps, vsize: int, info: Optional[DistInfo] = None, device: Optional[str] = None, params=None):
    """GPU: hipGraph HIP-kernel trainer (static shapes B x max_enc_steps).  CPU: oracle."""
    use_gpu = (device or ("cuda" if torch.cuda.is_available() else "cpu")).startswith("cuda")
    if use_gpu:
        from .trainer import GraphTrainer
        return GraphTrainer(hps, vsize, B=hps.batch_size, T=hps.max_enc_steps, info=info, params=params,
                            use_graph=hps.graph)
    from .cpu_trainer import CpuTrainer
    return CpuTrainer(hps, vsize, info=info, params=params)


def calc_running_avg_loss(loss: float, running_avg_loss: float, decay: float = 0.99) -> float:
    """run_summarization.py:105-129 (first value taken as is; clipped at 12)."""
    if running_avg_loss == 0:
        running_avg_loss = loss
    else:
        running_avg_loss = running_avg_loss * decay + (1 - decay) * loss
    return min(running_avg_loss, 12)


def _fault(hps, trainer, step: int, info: DistInfo):
    if getattr(hps, "fault_nan_step", -1) == step:
        log.warning("fault injection: NaN gradient at step %d", step)
        trainer.poison_next = True
    if getattr(hps, "fault_kill_step", -1) == step and info.rank == getattr(hps, "fault_kill_rank", 0):
        log.warning("fault injection: rank %d exits at step %d", info.rank, step)
        os._exit(17)


def run_training(trainer, batcher, hps, info: Optional[DistInfo] = None, saver: Optional[ckpt.Saver] = None,
                 metrics: Optional[MetricsLogger] = None, num_steps: Optional[int] = None,
                 save_model_secs: Optional[float] = None, log_every: Optional[int] = None) -> Dict[str, float]:
    """Train until ``num_steps`` more steps (0/None = until the batcher ends).

    The host never waits on the GPU between checks: a GPU trainer (``trainer.host_sync_free``)
    reads the loss, the NaN-guard flag and the persistent-LSTM error word only every
    ``hps.check_every`` steps (and after the last step).  The flags are sticky, so a
    non-finite step anywhere in the window stops training at the check ("Loss is not
    finite. Stopping.", ``train.py:107-108``); the device NaN guard has already skipped that
    step's update.  The CPU oracle trainer is synchronous anyway and checks every step.
    Loss lines and metrics are emitted at checks (``log_every`` > 0 enables them); tokens/s
    is measured over the whole window, and the token count is all-reduced once per check."""
    info = info or DistInfo()
    num_steps = hps.num_steps if num_steps is None else num_steps
    save_model_secs = hps.save_model_secs if save_model_secs is None else save_model_secs
    log_every = getattr(hps, "log_every", 1) if log_every is None else log_every
    check_every = max(1, int(getattr(hps, "check_every", 1))) if getattr(trainer, "host_sync_free", False) else 1
    start = trainer.global_step
    last_save = time.time()
    watch = NonFiniteWatch(trainer) if getattr(hps, "debug", False) and hasattr(trainer, "named_debug_tensors") \
        else None
    vals: Dict[str, float] = {}
    win_t0, win_tokens, win_steps = time.time(), 0.0, 0
    out = None

    def check():
        nonlocal vals, win_t0, win_tokens, win_steps
        vals = trainer.check_finite(out)  # host sync; raises "Loss is not finite. Stopping."
        dt = time.time() - win_t0
        toks = all_reduce_scalar(win_tokens, info)
        if log_every:
            log.info("step %d: seconds for training step: %.3f loss: %f%s", trainer.global_step, dt / win_steps,
                     vals["loss"], f" coverage_loss: {vals['coverage_loss']:f}" if "coverage_loss" in vals else "")
            if metrics:
                extra = trainer.phase_ms() if getattr(trainer, "timing", False) else {}
                metrics.log(step=trainer.global_step, step_ms=dt * 1e3 / win_steps, steps=win_steps,
                            tokens_per_sec=toks / max(dt, 1e-9), **extra, **vals)
        win_t0, win_tokens, win_steps = time.time(), 0.0, 0

    try:
        while not num_steps or trainer.global_step - start < num_steps:
            batch = batcher.next_batch()
            if batch is None:
                break
            _fault(hps, trainer, trainer.global_step - start, info)
            out = trainer.step(batch)
            win_tokens += float(batch.num_tokens())
            win_steps += 1
            if watch is not None and watch.check(trainer.global_step):
                raise NonFiniteLossError("Loss is not finite. Stopping. (--debug: has_inf_or_nan tripped)")
            if trainer.global_step % check_every == 0:
                check()
            if saver and info.is_chief and save_model_secs and time.time() - last_save >= save_model_secs:
                saver.save(trainer.params, trainer.global_step)
                last_save = time.time()
        if win_steps:
            check()
    except KeyboardInterrupt:
        log.info("Caught keyboard interrupt on worker. Stopping supervisor...")
    finally:
        if saver and info.is_chief and trainer.global_step > start:
            saver.save(trainer.params, trainer.global_step)
        barrier(info)
    return vals


def setup_training(hps, vocab, batcher, info: Optional[DistInfo] = None, metrics: Optional[MetricsLogger] = None,
                   device: Optional[str] = None):
    """``setup_training`` (run_summarization.py:181-209): train dir, optional coverage
    conversion / best-model restore (which exit, as in the reference), restore-from-latest
    (Supervisor auto-restore), then the training loop."""
    info = info or DistInfo()
    train_dir = os.path.join(hps.log_root, "train")
    os.makedirs(train_dir, exist_ok=True)
    trainer = make_trainer(hps, vocab.size(), info=info, device=device)
    if hps.convert_to_coverage_model:
        if not hps.coverage:
            raise ValueError("To convert your non-coverage model to a coverage model, run with "
                             "convert_to_coverage_model=True and coverage=True")
        return ckpt.convert_to_coverage_model(hps.log_root, trainer.params) if info.is_chief else None
    if hps.restore_best_model:
        return ckpt.restore_best_model(hps.log_root, trainer.params) if info.is_chief else None
    # only the chief reads the checkpoint (it wrote them): another rank may not see the file, or
    # see it half-written, and a restore error there would leave rank 0 blocked in the broadcast
    latest = ckpt.latest_checkpoint(train_dir) if info.is_chief else None
    if latest:
        trainer.global_step = ckpt.restore(latest, trainer.params, load_adagrad=True)
        if hasattr(trainer, "engine"):
            trainer.engine.pack()
        log.info("Restored %s at step %d", latest, trainer.global_step)
    if info.enabled:
        # resume on every rank from the chief's state
        broadcast_params(trainer.params.flat, info)
        if trainer.params.accum is not None:
            broadcast_params(trainer.params.accum, info)
        trainer.global_step = broadcast_scalar(trainer.global_step, info, trainer.params.flat.device)
        if hasattr(trainer, "engine"):
            trainer.engine.pack()
    saver = ckpt.Saver(train_dir, max_to_keep=hps.max_to_keep) if info.is_chief else None
    if info.is_chief:
        write_embedding_projector(train_dir, vocab)
    if getattr(hps, "profile_phases", False) and hasattr(trainer, "timing"):
        trainer.timing = True
    return trainer, run_training(trainer, batcher, hps, info=info, saver=saver, metrics=metrics)


def write_embedding_projector(train_dir: str, vocab) -> str:
    """vocab_metadata.tsv + projector_config.pbtxt for the embedding projector
    (``model.py:185-197``, ``data.py:93-105``)."""
    meta = os.path.join(train_dir, "vocab_metadata.tsv")
    vocab.write_metadata(meta)
    with open(os.path.join(train_dir, "projector_config.pbtxt"), "w") as f:
        f.write('embeddings {\n  tensor_name: "seq2seq/embedding/embedding"\n  metadata_path: "%s"\n}\n' % meta)
    return meta


def run_eval(hps, vocab, batcher, max_iters: Optional[int] = None, device: Optional[str] = None,
             metrics: Optional[MetricsLogger] = None, load_retries: int = 6, load_sleep_s: float = 10.0):
    """Eval loop (run_summarization.py:247-292).  Returns (best_loss, running_avg_loss)."""
    trainer = make_trainer(hps, vocab.size(), device=device)
    eval_dir = os.path.join(hps.log_root, "eval")
    saver = ckpt.Saver(eval_dir, max_to_keep=3, prefix="bestmodel", latest_filename="checkpoint_best")
    running_avg_loss, best_loss = 0.0, None
    it = 0
    while max_iters is None or it < max_iters:
        _, step = ckpt.load_ckpt(hps.log_root, trainer.params, "train", max_retries=load_retries,
                                 sleep_s=load_sleep_s)
        if hasattr(trainer, "engine"):
            trainer.engine.pack()
        batch = batcher.next_batch()
        if batch is None:
            break
        t0 = time.time()
        res = trainer.eval_step(batch)
        log.info("seconds for batch: %.2f loss: %f", time.time() - t0, res["loss"])
        running_avg_loss = calc_running_avg_loss(res["loss"], running_avg_loss)
        log.info("running_avg_loss: %f", running_avg_loss)
        if metrics:
            metrics.log(step=step, eval_loss=res["loss"], running_avg_loss=running_avg_loss,
                        **{k: v for k, v in res.items() if k != "loss"})
        if best_loss is None or running_avg_loss < best_loss:
            log.info("Found new best model with %.3f running_avg_loss. Saving to %s", running_avg_loss,
                     os.path.join(eval_dir, "bestmodel"))
            saver.save(trainer.params, step, with_adagrad=False)
            best_loss = running_avg_loss
        it += 1
    return best_loss, running_avg_loss
