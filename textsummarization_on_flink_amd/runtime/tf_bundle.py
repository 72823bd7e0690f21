"""TF1 V2 checkpoint (tensor bundle) files without TensorFlow, via the native C++
reader/writer in ``csrc/runtime/tf_bundle.cpp``.

``save_bundle(prefix, {name: array})`` writes ``prefix.index`` + ``prefix.data-00000-of-00001``;
``load_bundle(prefix)`` reads them back (crc32c-verified).  Variable names/shapes are the
reference's (``seq2seq/...``, ``<var>/Adagrad``, ``global_step``), so checkpoints written
here use the pointer-generator layout and the reference's TF1 checkpoints load here.
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict
from typing import Dict

import numpy as np

from .native import lib

# TF DataType enum
DT = {np.dtype("float32"): 1, np.dtype("float64"): 2, np.dtype("int32"): 3, np.dtype("int64"): 9,
      np.dtype("float16"): 19, np.dtype("uint8"): 4, np.dtype("int8"): 6, np.dtype("int16"): 5, np.dtype("bool"): 10}
DT_INV = {v: k for k, v in DT.items()}
DT_BFLOAT16 = 14


def save_bundle(prefix: str, tensors: Dict[str, object]) -> None:
    L = lib()
    w = L.tsb_writer_open(prefix.encode())
    if not w:
        raise OSError(f"cannot open checkpoint for writing: {prefix}")
    try:
        for name, t in tensors.items():
            if hasattr(t, "detach"):
                t = t.detach().cpu().numpy()
            a = np.require(np.asarray(t), requirements="C")  # keeps 0-d scalars 0-d
            if a.dtype not in DT:
                raise TypeError(f"unsupported dtype {a.dtype} for {name}")
            dims = (C.c_int64 * max(1, a.ndim))(*a.shape)
            rc = L.tsb_writer_add(w, name.encode(), DT[a.dtype], a.ndim, dims, a.ctypes.data_as(C.c_void_p),
                                  a.nbytes)
            if rc != 0:
                raise OSError(f"tsb_writer_add({name}) failed: {rc}")
    finally:
        rc = L.tsb_writer_finish(w)
    if rc != 0:
        raise OSError(f"tsb_writer_finish failed: {rc}")


def list_bundle(prefix: str) -> Dict[str, tuple]:
    """name -> (numpy dtype or 'bfloat16', shape)."""
    L = lib()
    r = L.tsb_reader_open(prefix.encode(), 1)
    if not r:
        raise OSError(f"not a readable tensor bundle: {prefix}")
    out = OrderedDict()
    try:
        for i in range(L.tsb_reader_num(r)):
            name, dt, shape, _ = _entry(L, r, i)
            out[name] = (DT_INV.get(dt, "bfloat16" if dt == DT_BFLOAT16 else dt), shape)
    finally:
        L.tsb_reader_close(r)
    return out


def _entry(L, r, i):
    buf = C.create_string_buffer(4096)
    dt, nd, nb = C.c_int(), C.c_int(), C.c_int64()
    dims = (C.c_int64 * 8)()
    rc = L.tsb_reader_entry(r, i, buf, 4096, C.byref(dt), C.byref(nd), dims, C.byref(nb))
    if rc != 0:
        raise OSError(f"tsb_reader_entry failed: {rc}")
    return buf.value.decode(), dt.value, tuple(dims[k] for k in range(nd.value)), nb.value


def load_bundle(prefix: str, verify: bool = True) -> Dict[str, np.ndarray]:
    L = lib()
    r = L.tsb_reader_open(prefix.encode(), int(verify))
    if not r:
        raise OSError(f"not a readable tensor bundle (or corrupt index): {prefix}")
    out = OrderedDict()
    try:
        for i in range(L.tsb_reader_num(r)):
            name, dt, shape, nbytes = _entry(L, r, i)
            if dt == DT_BFLOAT16:
                raw = np.empty(nbytes // 2, np.uint16)
                rc = L.tsb_reader_read(r, i, raw.ctypes.data_as(C.c_void_p), int(verify))
                arr = (raw.astype(np.uint32) << 16).view(np.float32).reshape(shape)
            else:
                npdt = DT_INV.get(dt)
                if npdt is None:
                    raise TypeError(f"unsupported TF dtype {dt} for {name}")
                arr = np.empty(shape, npdt)
                if arr.nbytes != nbytes:
                    raise OSError(f"size mismatch for {name}: {arr.nbytes} vs {nbytes}")
                rc = L.tsb_reader_read(r, i, arr.ctypes.data_as(C.c_void_p), int(verify))
            if rc == -4:
                raise OSError(f"crc32c mismatch reading {name} from {prefix}")
            if rc != 0:
                raise OSError(f"tsb_reader_read({name}) failed: {rc}")
            out[name] = arr
    finally:
        L.tsb_reader_close(r)
    return out
