"""ctypes binding of the host-side native runtime ``_rt.so`` (built from csrc/runtime)."""
from __future__ import annotations

import ctypes as C
import os
import threading

_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_rt.so")
_lock = threading.Lock()
_lib = None


def lib():
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(_LIB):
            from .. import _build
            _build.build_runtime()
        L = C.CDLL(_LIB)
        vp, i32, i64, u32, u64 = C.c_void_p, C.c_int, C.c_int64, C.c_uint32, C.c_uint64
        sig = {
            "tsb_crc32c": (u32, [vp, u64]),
            "tsb_crc32c_masked": (u32, [vp, u64]),
            "tsb_writer_open": (vp, [C.c_char_p]),
            "tsb_writer_add": (i32, [vp, C.c_char_p, i32, i32, C.POINTER(i64), vp, i64]),
            "tsb_writer_finish": (i32, [vp]),
            "tsb_reader_open": (vp, [C.c_char_p, i32]),
            "tsb_reader_num": (i32, [vp]),
            "tsb_reader_entry": (i32, [vp, i32, C.c_char_p, i32, C.POINTER(i32), C.POINTER(i32), C.POINTER(i64),
                                       C.POINTER(i64)]),
            "tsb_reader_read": (i32, [vp, i32, vp, i32]),
            "tsb_reader_close": (None, [vp]),
            "ring_create": (vp, [C.c_char_p, u64]),
            "ring_open": (vp, [C.c_char_p]),
            "ring_push": (i32, [vp, vp, u32, i64]),
            "ring_pop": (i64, [vp, vp, u64, i64, C.POINTER(u64)]),
            "ring_close_writer": (None, [vp]),
            "ring_is_closed": (i32, [vp]),
            "ring_pending_bytes": (u64, [vp]),
            "ring_records_in": (u64, [vp]),
            "ring_records_out": (u64, [vp]),
            "ring_capacity": (u64, [vp]),
            "ring_release": (None, [vp, i32]),
            "ring_fanout_start": (vp, [vp, C.POINTER(vp), i32, i64]),
            "ring_fanin_start": (vp, [C.POINTER(vp), i32, vp, i32]),
            "ring_pipe_count": (i64, [vp]),
            "ring_pipe_stop": (None, [vp]),
            "ring_pipe_join": (i64, [vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
        return L


def crc32c(data: bytes, masked: bool = False) -> int:
    b = C.create_string_buffer(bytes(data), len(data))
    f = lib().tsb_crc32c_masked if masked else lib().tsb_crc32c
    return int(f(b, len(data)))
