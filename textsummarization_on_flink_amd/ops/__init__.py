"""Loader for the in-tree gfx950 kernel library (``_C.so``, built by ``_build.py``).

The HIP kernels are the only GPU compute path: ``ops()`` raises if the library is
missing or fails to load, so a GPU run can never fall back to eager PyTorch silently.
"""
from __future__ import annotations

import os
import threading

import torch

_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C.so")
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
            _build.build_kernels()
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
