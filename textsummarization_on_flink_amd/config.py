"""Hyper-parameters and the run_summarization-compatible flag system.

Same flag names and defaults as the reference (``run_summarization.py:47-88``), parsed
leniently like ``tf.app.flags.FLAGS(argv, known_only=True)`` (``run_summarization.py:420``)
so a Flink-style space-joined hyper-parameter string (``App.java:55-81``, first token a
placeholder program name) can be fed straight in.  The model-visible subset mirrors the
``hps`` namedtuple (``run_summarization.py:320-327``) plus the MI355X-side knobs
(dtype, static-shape padding, graph capture).
"""
from __future__ import annotations

import argparse
import dataclasses
import json
from dataclasses import dataclass, field, fields
from typing import List, Optional, Sequence


def _bool(v) -> bool:
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("1", "true", "t", "yes", "y"):
        return True
    if s in ("0", "false", "f", "no", "n", ""):
        return False
    raise ValueError(f"not a boolean: {v!r}")


@dataclass
class HParams:
    # where to find data (run_summarization.py:48-49)
    data_path: str = ""
    vocab_path: str = ""
    # important settings (:52-55)
    mode: str = "train"
    num_steps: int = 0
    single_pass: bool = False
    inference: bool = False
    # where to save output (:58-59)
    log_root: str = ""
    exp_name: str = ""
    # hyperparameters (:62-74)
    hidden_dim: int = 256
    emb_dim: int = 128
    batch_size: int = 16
    max_enc_steps: int = 400
    max_dec_steps: int = 100
    beam_size: int = 4
    min_dec_steps: int = 35
    vocab_size: int = 50000
    lr: float = 0.15
    adagrad_init_acc: float = 0.1
    rand_unif_init_mag: float = 0.02
    trunc_norm_init_std: float = 1e-4
    max_grad_norm: float = 2.0
    # pointer-generator / coverage (:77-81)
    pointer_gen: bool = True
    coverage: bool = False
    cov_loss_wt: float = 1.0
    # utility (:84-88)
    convert_to_coverage_model: bool = False
    restore_best_model: bool = False
    debug: bool = False
    # ---- MI355X-native knobs (not in the reference) ----
    enc_layers: int = 1            # >1 = stacked bi-LSTM (BASELINE config #5 generalisation)
    seed: int = 111                # tf.set_random_seed(111), run_summarization.py:329
    pad_enc_to_max: bool = True    # static shapes for hipGraph capture (padding is masked)
    graph: bool = True             # capture the train step / decode step in hipGraphs
    decode_batch: int = 64         # articles decoded together (beam-as-batch x articles)
    stream_max_wait_ms: float = 0.0   # streaming decode: queued requests always share a batch; after
                                      # the first, wait at most this long for more (0 = no waiting)
    save_model_secs: int = 60      # Supervisor(save_model_secs=60), run_summarization.py:199
    max_to_keep: int = 3           # Saver(max_to_keep=3)
    log_every: int = 1
    drop_last: bool = False        # Issue-5 fix: pad (False) or drop (True) a short final batch
    metrics_path: str = ""         # JSONL metrics file ("" = <log_root>/metrics_<mode>.jsonl)
    tensorboard: bool = True       # also write TensorBoard scalar event files (train/ and eval/)
    html_escape: bool = False      # fix quirk: make_html_safe discards its result in the reference
    load_retries: int = 6          # bounded checkpoint-load retries (util.py:29-41 retried forever)
    fault_nan_step: int = -1       # fault injection: NaN gradient at this (relative) step
    fault_kill_step: int = -1      # fault injection: hard-exit rank fault_kill_rank at this step
    fault_kill_rank: int = 0
    dist_timeout_s: int = 600      # collective timeout: a dead rank surfaces as an error, not a hang
    profile_phases: bool = False   # per-phase step timing (HIP events) into the metrics JSONL
    flink_tokenize_article: bool = False  # quirk 4: the Flink path whitespace-splits the raw article
    log_file: str = ""             # rotating log file, 100 MB x 20 (log4j2.xml); one file per rank
    check_every: int = 10          # host reads loss / NaN / LSTM-error flags every N steps (1 = every step)
    grad_compress: str = "none"    # DP gradient all-reduce wire format: none (fp32) | bf16
    loader_workers: int = -1       # GPU training input pipeline: N worker processes (0 = threaded Batcher,
                                   # -1 = min(8, CPUs - 2)); see data/loader.py
    stream_packers: int = -1       # streaming (Flink-API) GPU workers: N packer processes parse rows into
                                   # engine batches (0 = on the engine thread, -1 = min(12, CPUs - 3));
                                   # see data/stream_pack.py

    # ------------------------------------------------------------------ helpers
    def replace(self, **kw) -> "HParams":
        return dataclasses.replace(self, **kw)

    def to_dict(self):
        return dataclasses.asdict(self)

    def to_json(self) -> str:
        return json.dumps(self.to_dict(), sort_keys=True)

    @classmethod
    def from_dict(cls, d):
        names = {f.name for f in fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})


_FIELD_TYPES = {f.name: f.type for f in fields(HParams)}


def _caster(tp):
    tp = str(tp)
    if tp == "bool":
        return _bool
    if tp == "int":
        return int
    if tp == "float":
        return float
    return str


def build_arg_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="run_summarization", allow_abbrev=False)
    defaults = HParams()
    for name, tp in _FIELD_TYPES.items():
        c = _caster(tp)
        if c is _bool:
            # absl-style: --flag, --noflag, --flag=1/0/true/false
            p.add_argument(f"--{name}", nargs="?", const=True, default=getattr(defaults, name), type=_bool)
            p.add_argument(f"--no{name}", dest=name, action="store_false")
        else:
            p.add_argument(f"--{name}", type=c, default=getattr(defaults, name))
    return p


def parse_flags(argv: Optional[Sequence[str]] = None, known_only: bool = True, base: Optional[HParams] = None
                ) -> HParams:
    """Parse reference-style flags.  ``argv[0]`` is a program name placeholder only when it
    does not start with ``--`` (``App.java:56`` passes "run_summarization.py")."""
    argv = list(argv or [])
    if argv and not argv[0].startswith("-"):
        argv = argv[1:]
    p = build_arg_parser()
    if base is not None:
        p.set_defaults(**base.to_dict())
    ns, unknown = p.parse_known_args(argv)
    if unknown and not known_only:
        raise SystemExit(f"unknown flags: {unknown}")
    return HParams.from_dict(vars(ns))


def parse_hyperparam_string(s: str, base: Optional[HParams] = None) -> HParams:
    """Parse the space-joined hyper-parameter property (``TFEstimator.java:52``)."""
    return parse_flags([t for t in s.split(" ") if t], known_only=True, base=base)


def decode_hps(hps: HParams) -> HParams:
    """Decode-mode overrides: ``batch_size = beam_size`` (run_summarization.py:312-313) and
    the one-step decoder (``max_dec_steps=1`` for the model, :344-345).  The batcher keeps
    the full ``max_dec_steps`` for the decode loop bound."""
    return hps.replace(batch_size=hps.beam_size)


def check_hps(hps: HParams) -> None:
    if hps.mode not in ("train", "eval", "decode"):
        raise ValueError("The 'mode' flag must be one of train/eval/decode")
    if hps.single_pass and hps.mode != "decode":
        raise ValueError("The single_pass flag should only be True in decode mode")  # :316-317
    if hps.convert_to_coverage_model and not hps.coverage:
        raise ValueError("To convert your non-coverage model to a coverage model, run with "
                         "convert_to_coverage_model=True and coverage=True")  # :188


@dataclass
class ModelDims:
    """Shapes the kernels are specialised on."""
    V: int
    E: int
    H: int
    T: int
    D: int
    layers: int = 1

    @property
    def A(self) -> int:
        return 2 * self.H
