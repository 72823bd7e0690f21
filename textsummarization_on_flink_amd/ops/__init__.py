"""Loader for the in-tree gfx950 kernel library (``_C.so``, built by ``_build.py``).

The HIP kernels are the only GPU compute path: ``ops()`` raises if the library is
missing or fails to load, so a GPU run can never fall back to eager PyTorch silently.

TSAMD_KERNEL_DEBUG=1 loads the bounds-checked build ``_C_debug.so`` instead (data-dependent
indices -- token ids, lengths, beam back-pointers -- checked in the kernels and clamped;
``debug_check()`` raises on the first failed check).
"""
from __future__ import annotations

import os
import threading

import torch

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEBUG = os.environ.get("TSAMD_KERNEL_DEBUG", "0") == "1"
# TSAMD_C_LIB: another in-tree build of the library (same-box A/B of a kernel change)
_LIB = os.path.join(_PKG, os.environ.get("TSAMD_C_LIB") or ("_C_debug.so" if DEBUG else "_C.so"))
# check ids of csrc/kernels/dcheck.h
DEBUG_CHECKS = {1: "to_step_frame row id", 2: "step-frame reversal index", 3: "embedding-gradient token id",
                4: "attention encoder length", 5: "pointer-loss / copy-mass encoder length",
                6: "beam parent row", 7: "beam latest token"}
_lock = threading.Lock()
_loaded = False


def library_path() -> str:
    return _LIB


def load(build_if_missing: bool = True):
    global _loaded
    with _lock:
        if _loaded:
            return torch.ops.tsamd
        if not os.path.exists(_LIB) and build_if_missing:
            from .. import _build
            _build.build_kernels(debug=DEBUG)
        if not os.path.exists(_LIB):
            raise RuntimeError(f"HIP kernel library not found at {_LIB}; run `python -m textsummarization_on_flink_amd._build`")
        torch.ops.load_library(_LIB)
        _loaded = True
        return torch.ops.tsamd


def ops():
    """The torch.ops namespace of the kernels; loads (and builds if needed) on first use."""
    return load()


def is_loaded() -> bool:
    return _loaded


class KernelBoundsError(RuntimeError):
    pass


def debug_check(clear: bool = True) -> None:
    """Raise KernelBoundsError if a bounds check of the debug build failed (no-op for the
    release build).  Synchronises the device."""
    k = ops()
    if not int(k.debug_enabled()):
        return
    import torch as _t
    _t.cuda.synchronize()
    cid, blk, thr, val = (int(x) for x in k.debug_status().tolist())
    if clear:
        k.debug_clear()
    if cid:
        raise KernelBoundsError(f"kernel bounds check failed: {DEBUG_CHECKS.get(cid, cid)} "
                                f"(block {blk}, thread {thr}, value {val})")

