"""Checkpoint / resume in the reference's TF1 format.

* ``model.ckpt-<step>.{index,data-00000-of-00001}`` tensor bundles (native C++ codec), the
  text ``checkpoint`` state file, ``max_to_keep`` rotation (``Saver(max_to_keep=3)``,
  ``run_summarization.py:192``) and ``save_model_secs`` cadence;
* variable names of the reference graph + ``<var>/Adagrad`` slots + ``global_step``;
* eval best-model tracking (``eval/bestmodel-<step>`` + ``checkpoint_best``,
  ``run_summarization.py:250-288``);
* ``convert_to_coverage_model`` / ``restore_best_model`` (``run_summarization.py:132-178``);
* ``load_ckpt`` with BOUNDED retries (the reference loops forever, ``util.py:29-41``,
  SURVEY 2.9 item 10);
* ``inspect_checkpoint`` NaN/Inf scanner (``inspect_checkpoint.py:11-45``).

Only the chief (rank 0) writes; every rank reads.
"""
from __future__ import annotations

import glob
import logging
import os
import re
import time
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..runtime.tf_bundle import list_bundle, load_bundle, save_bundle

log = logging.getLogger(__name__)
GLOBAL_STEP = "global_step"
SLOT = "/Adagrad"


# ------------------------------------------------------------------ state file
def write_state(ckpt_dir: str, paths: List[str], latest_filename: str = "checkpoint") -> None:
    rel = [os.path.relpath(p, ckpt_dir) if os.path.isabs(p) and p.startswith(ckpt_dir) else p for p in paths]
    lines = [f'model_checkpoint_path: "{rel[-1]}"'] + [f'all_model_checkpoint_paths: "{p}"' for p in rel]
    tmp = os.path.join(ckpt_dir, latest_filename + ".tmp")
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, os.path.join(ckpt_dir, latest_filename))


def read_state(ckpt_dir: str, latest_filename: Optional[str] = None) -> Optional[Tuple[str, List[str]]]:
    p = os.path.join(ckpt_dir, latest_filename or "checkpoint")
    if not os.path.exists(p):
        return None
    latest, allp = None, []
    for line in open(p):
        m = re.match(r'\s*(model_checkpoint_path|all_model_checkpoint_paths):\s*"(.*)"', line)
        if not m:
            continue
        v = m.group(2)
        v = v if os.path.isabs(v) else os.path.join(ckpt_dir, v)
        if m.group(1) == "model_checkpoint_path":
            latest = v
        else:
            allp.append(v)
    if latest is None:
        return None
    return latest, allp


def latest_checkpoint(ckpt_dir: str, latest_filename: Optional[str] = None) -> Optional[str]:
    st = read_state(ckpt_dir, latest_filename)
    return st[0] if st else None


def _delete(prefix: str):
    for f in glob.glob(prefix + ".index") + glob.glob(prefix + ".data-*") + glob.glob(prefix + ".meta"):
        try:
            os.remove(f)
        except OSError:
            pass


# ------------------------------------------------------------------ save / restore
def params_to_tensors(params, global_step: int, with_adagrad: bool = True) -> Dict[str, np.ndarray]:
    out = {}
    for n, t in params.items():
        out[n] = t.detach().float().cpu().numpy()
    if with_adagrad and params.accum is not None:
        for n in params.names:
            out[n + SLOT] = params.view(n, params.accum).detach().float().cpu().numpy()
    out[GLOBAL_STEP] = np.array(int(global_step), dtype=np.int32)
    return out


class Saver:
    """tf.train.Saver-like manager for one directory."""

    def __init__(self, ckpt_dir: str, max_to_keep: int = 3, prefix: str = "model.ckpt",
                 latest_filename: str = "checkpoint"):
        self.dir = ckpt_dir
        self.max_to_keep = max_to_keep
        self.prefix = prefix
        self.latest_filename = latest_filename
        os.makedirs(ckpt_dir, exist_ok=True)

    def save(self, params, global_step: int, with_adagrad: bool = True, name: Optional[str] = None) -> str:
        path = os.path.join(self.dir, name or f"{self.prefix}-{int(global_step)}")
        save_bundle(path, params_to_tensors(params, global_step, with_adagrad))
        st = read_state(self.dir, self.latest_filename)
        paths = [p for p in (st[1] if st else []) if p != path] + [path]
        if self.max_to_keep and len(paths) > self.max_to_keep:
            for old in paths[:-self.max_to_keep]:
                _delete(old)
            paths = paths[-self.max_to_keep:]
        write_state(self.dir, paths, self.latest_filename)
        log.info("Saved checkpoint %s", path)
        return path


def restore(prefix: str, params, load_adagrad: bool = True, skip=lambda name: False, strict: bool = True) -> int:
    """Load a bundle into FlatParams; returns global_step (0 if absent)."""
    t = load_bundle(prefix)
    import torch
    missing = []
    for n in params.names:
        if skip(n):
            continue
        if n in t:
            params.view(n).copy_(torch.from_numpy(np.ascontiguousarray(t[n])).reshape(params.view(n).shape))
        else:
            missing.append(n)
        if load_adagrad and params.accum is not None and (n + SLOT) in t:
            params.view(n, params.accum).copy_(torch.from_numpy(np.ascontiguousarray(t[n + SLOT])).reshape(
                params.view(n).shape))
    if strict and missing:
        raise KeyError(f"checkpoint {prefix} lacks variables: {missing}")
    return int(np.asarray(t[GLOBAL_STEP]).reshape(-1)[0]) if GLOBAL_STEP in t else 0


def load_ckpt(log_root: str, params, ckpt_dir: str = "train", max_retries: int = 6, sleep_s: float = 10.0,
              load_adagrad: bool = True) -> Tuple[str, int]:
    """Restore the latest checkpoint of ``log_root/ckpt_dir`` (``checkpoint_best`` for eval),
    retrying a bounded number of times (util.py:29-41 retried forever)."""
    latest_filename = "checkpoint_best" if ckpt_dir == "eval" else None
    d = os.path.join(log_root, ckpt_dir)
    err = None
    for attempt in range(max_retries + 1):
        try:
            path = latest_checkpoint(d, latest_filename)
            if path is None:
                raise FileNotFoundError(f"no checkpoint state in {d}")
            step = restore(path, params, load_adagrad=load_adagrad)
            log.info("Loaded checkpoint %s (step %d)", path, step)
            return path, step
        except Exception as e:  # noqa: BLE001 -- retried, then re-raised
            err = e
            if attempt < max_retries:
                log.info("Failed to load checkpoint from %s (%s). Sleeping for %.0f secs...", d, e, sleep_s)
                time.sleep(sleep_s)
    raise RuntimeError(f"could not load a checkpoint from {d} after {max_retries + 1} attempts") from err


def convert_to_coverage_model(log_root: str, params) -> str:
    """Restore all non-coverage, non-Adagrad variables from the latest train checkpoint into
    a freshly initialised coverage model and save it as ``<ckpt>_cov_init``."""
    path = latest_checkpoint(os.path.join(log_root, "train"))
    if path is None:
        raise FileNotFoundError("no train checkpoint to convert")
    step = restore(path, params, load_adagrad=False, skip=lambda n: "coverage" in n, strict=True)
    new = path + "_cov_init"
    save_bundle(new, params_to_tensors(params, step, with_adagrad=True))
    st = read_state(os.path.join(log_root, "train"))
    write_state(os.path.join(log_root, "train"), (st[1] if st else []) + [new])
    log.info("saved coverage-initialised model to %s", new)
    return new


def restore_best_model(log_root: str, params) -> str:
    """Copy eval/bestmodel-N (without Adagrad) into train/model-N with fresh Adagrad slots."""
    best = latest_checkpoint(os.path.join(log_root, "eval"), "checkpoint_best")
    if best is None:
        raise FileNotFoundError("no eval best model")
    step = restore(best, params, load_adagrad=False)
    name = os.path.basename(best).replace("bestmodel", "model")
    out = os.path.join(log_root, "train", name)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    save_bundle(out, params_to_tensors(params, step, with_adagrad=True))
    st = read_state(os.path.join(log_root, "train"))
    write_state(os.path.join(log_root, "train"), (st[1] if st else []) + [out])
    return out


def inspect_checkpoint(prefix: str) -> Dict[str, List[str]]:
    """Classify every variable as finite / all inf-nan / some inf-nan."""
    t = load_bundle(prefix)
    res = {"finite": [], "all_infnan": [], "some_infnan": []}
    for k in sorted(t):
        a = np.asarray(t[k])
        if not np.issubdtype(a.dtype, np.floating) or np.all(np.isfinite(a)):
            res["finite"].append(k)
        elif not np.any(np.isfinite(a)):
            res["all_infnan"].append(k)
        else:
            res["some_infnan"].append(k)
    return res


def main_inspect(argv=None):
    import sys
    argv = argv if argv is not None else sys.argv[1:]
    if len(argv) != 1:
        raise SystemExit("Usage: python -m textsummarization_on_flink_amd.train.checkpoint <ckpt prefix>\n"
                         "Note: Do not include the .data .index or .meta part of the model checkpoint in file_name.")
    r = inspect_checkpoint(argv[0])
    print("\nFINITE VARIABLES:")
    print("\n".join(r["finite"]))
    print("\nVARIABLES THAT ARE ALL INF/NAN:")
    print("\n".join(r["all_infnan"]))
    print("\nVARIABLES THAT CONTAIN SOME FINITE, SOME INF/NAN VALUES:")
    print("\n".join(r["some_infnan"]))
    print("")
    ok = not r["all_infnan"] and not r["some_infnan"]
    print("CHECK PASSED: checkpoint contains no inf/NaN values" if ok else
          "CHECK FAILED: checkpoint contains some inf/NaN values")
    return 0 if ok else 1


if __name__ == "__main__":
    raise SystemExit(main_inspect())
