"""Shared-memory SPSC record ring (native, ``csrc/runtime/shm_ring.cpp``) -- the replacement
for Flink-AI-Extended's JVM<->Python queue.

``RecordRing.create(name, capacity)`` on the producer side, ``RecordRing.open(name)`` on
the consumer side (any process).  ``push(bytes)`` / ``pop()`` block with timeouts;
``close()`` marks end-of-stream so a drained consumer gets ``None``.

``RingDrainer`` runs the consumer loop on a dedicated thread and hands every record to a
callback as soon as it lands -- the Issue-6 fix (results must not lag one record behind
because reads and writes share one thread).
"""
from __future__ import annotations

import ctypes as C
import threading
from typing import Callable, Iterator, Optional

from .native import lib


class RingClosed(Exception):
    pass


class RecordRing:
    def __init__(self, handle, name: str, owner: bool):
        if not handle:
            raise OSError(f"cannot create/open ring {name}")
        self._h = handle
        self.name = name
        self.owner = owner
        self._buf = C.create_string_buffer(1 << 16)

    @classmethod
    def create(cls, name: str, capacity: int = 64 << 20) -> "RecordRing":
        if not name.startswith("/"):
            name = "/" + name
        return cls(lib().ring_create(name.encode(), capacity), name, True)

    @classmethod
    def open(cls, name: str) -> "RecordRing":
        if not name.startswith("/"):
            name = "/" + name
        return cls(lib().ring_open(name.encode()), name, False)

    def push(self, data: bytes, timeout_ms: int = -1) -> None:
        rc = lib().ring_push(self._h, data, len(data), timeout_ms)
        if rc == -1:
            raise TimeoutError("ring full")
        if rc == -2:
            raise RingClosed(self.name)
        if rc == -3:
            raise ValueError(f"record of {len(data)} bytes exceeds ring capacity")

    def pop(self, timeout_ms: int = -1) -> Optional[bytes]:
        """Next record; None at end of stream; TimeoutError if nothing within timeout."""
        need = C.c_uint64(0)
        while True:
            n = lib().ring_pop(self._h, self._buf, len(self._buf), timeout_ms, C.byref(need))
            if n >= 0:
                return self._buf.raw[:n]
            if n == -2:
                return None
            if n == -1:
                raise TimeoutError("ring empty")
            if n == -3:
                self._buf = C.create_string_buffer(int(need.value) * 2)
                continue
            raise OSError(f"ring_pop failed: {n}")

    def __iter__(self) -> Iterator[bytes]:
        while True:
            r = self.pop()
            if r is None:
                return
            yield r

    def close(self) -> None:
        lib().ring_close_writer(self._h)

    @property
    def closed(self) -> bool:
        return bool(lib().ring_is_closed(self._h))

    def stats(self):
        L = lib()
        return {"in": int(L.ring_records_in(self._h)), "out": int(L.ring_records_out(self._h)),
                "pending_bytes": int(L.ring_pending_bytes(self._h)), "capacity": int(L.ring_capacity(self._h))}

    def release(self, unlink: Optional[bool] = None) -> None:
        if self._h:
            lib().ring_release(self._h, int(self.owner if unlink is None else unlink))
            self._h = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


class RingPipe:
    """A native forwarding thread between rings (``shm_ring.cpp`` ring pipes; no GIL on the
    record path).  ``fanout``: record k of ``src`` -> ``dsts[(k // group) % n]``, the
    destinations closed at the source's end of stream.  ``fanin``: every record of any source
    -> ``dst`` the moment it lands, ``dst`` closed once all sources are closed and drained."""

    def __init__(self, handle, keep):
        if not handle:
            raise OSError("cannot start ring pipe")
        self._h, self._keep = handle, keep  # keep the rings alive while the thread uses them

    @classmethod
    def fanout(cls, src: RecordRing, dsts, group: int = 1) -> "RingPipe":
        arr = (C.c_void_p * len(dsts))(*[d._h for d in dsts])
        return cls(lib().ring_fanout_start(src._h, arr, len(dsts), int(group)), (src, list(dsts)))

    @classmethod
    def fanin(cls, srcs, dst: RecordRing, close_dst: bool = True) -> "RingPipe":
        arr = (C.c_void_p * len(srcs))(*[s._h for s in srcs])
        return cls(lib().ring_fanin_start(arr, len(srcs), dst._h, int(close_dst)), (list(srcs), dst))

    @property
    def count(self) -> int:
        return int(lib().ring_pipe_count(self._h)) if self._h else -1

    def stop(self) -> None:
        if self._h:
            lib().ring_pipe_stop(self._h)

    def join(self) -> int:
        """Wait for the thread; records forwarded (raises if a destination was closed early)."""
        if not self._h:
            return 0
        n = int(lib().ring_pipe_join(self._h))
        self._h = None
        if n == -2:
            raise RingClosed("ring pipe: a destination ring was closed by its consumer")
        if n < 0:
            raise OSError(f"ring pipe failed: {n}")
        return n

    def __del__(self):
        try:
            if self._h:
                self.stop()
                lib().ring_pipe_join(self._h)
        except Exception:
            pass


class RingDrainer(threading.Thread):
    """Consumer thread: pops records and calls ``on_record`` immediately (Issue-6 fix)."""

    def __init__(self, ring: RecordRing, on_record: Callable[[bytes], None], poll_ms: int = 50):
        super().__init__(daemon=True)
        self.ring = ring
        self.on_record = on_record
        self.poll_ms = poll_ms
        self.error: Optional[BaseException] = None
        self.count = 0

    def run(self):
        try:
            while True:
                try:
                    r = self.ring.pop(self.poll_ms)
                except TimeoutError:
                    continue
                if r is None:
                    return
                self.on_record(r)
                self.count += 1
        except BaseException as e:  # noqa: BLE001 -- surfaced via .error
            self.error = e
