"""TensorBoard scalar event files without TensorFlow.

The reference logs its scalars through ``tf.summary`` into the Supervisor's /
MonitoredTrainingSession's summary writer: ``loss``, ``coverage_loss``, ``total_loss``,
``global_norm`` in ``<log_root>/train`` (``model.py:270-278,300``;
``run_summarization.py:238-244``) and ``running_avg_loss/decay=0.990000`` in
``<log_root>/eval`` (``run_summarization.py:124-127``).  This module writes the same
``events.out.tfevents.<time>.<host>`` files so TensorBoard reads them unchanged:

  record  = uint64 length | uint32 masked_crc32c(length) | payload | uint32 masked_crc32c(payload)
  Event   = {1: wall_time (double), 2: step (int64), 3: file_version (string) | 5: summary}
  Summary = {1: repeated Value},  Value = {1: tag (string), 2: simple_value (float)}

The crc32c comes from the native runtime (``csrc/runtime/tf_bundle.cpp``), the same
routine the TF checkpoint writer uses.  ``read_events`` parses the files back (tests).
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Dict, Iterator, List, Optional, Tuple

from ..runtime.native import crc32c


def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _bytes_field(field: int, data: bytes) -> bytes:
    return _key(field, 2) + _varint(len(data)) + data


def encode_event(wall_time: float, step: int, scalars: Optional[Dict[str, float]] = None,
                 file_version: Optional[str] = None) -> bytes:
    ev = _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(int(step))
    if file_version is not None:
        ev += _bytes_field(3, file_version.encode())
    if scalars:
        summ = b"".join(_bytes_field(1, _bytes_field(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(v)))
                        for tag, v in scalars.items())
        ev += _bytes_field(5, summ)
    return ev


def frame(payload: bytes) -> bytes:
    n = struct.pack("<Q", len(payload))
    return n + struct.pack("<I", crc32c(n, masked=True)) + payload + struct.pack("<I", crc32c(payload, masked=True))


class EventWriter:
    """Append-only scalar writer (``tf.summary.FileWriter`` equivalent)."""

    def __init__(self, logdir: str, filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}{filename_suffix}"
        self.path = os.path.join(logdir, name)
        self._f = open(self.path, "ab")
        self._f.write(frame(encode_event(time.time(), 0, file_version="brain.Event:2")))
        self._f.flush()

    def add_scalars(self, step: int, scalars: Dict[str, float], wall_time: Optional[float] = None) -> None:
        if self._f is None or not scalars:
            return
        self._f.write(frame(encode_event(time.time() if wall_time is None else wall_time, step, scalars)))

    def flush(self) -> None:
        if self._f:
            self._f.flush()

    def close(self) -> None:
        if self._f:
            self._f.close()
            self._f = None


# ---------------------------------------------------------------------- reading back
def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    shift = n = 0
    while True:
        c = b[i]
        i += 1
        n |= (c & 0x7F) << shift
        shift += 7
        if not c & 0x80:
            return n, i


def _fields(b: bytes) -> Iterator[Tuple[int, int, object]]:
    i = 0
    while i < len(b):
        k, i = _read_varint(b, i)
        f, wt = k >> 3, k & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 1:
            v, i = b[i:i + 8], i + 8
        elif wt == 5:
            v, i = b[i:i + 4], i + 4
        elif wt == 2:
            n, i = _read_varint(b, i)
            v, i = b[i:i + n], i + n
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield f, wt, v


def read_events(path: str) -> List[dict]:
    """Parse an event file, verifying both CRCs of every record."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        hdr = data[i:i + 8]
        (n,) = struct.unpack("<Q", hdr)
        (hc,) = struct.unpack("<I", data[i + 8:i + 12])
        if hc != crc32c(hdr, masked=True):
            raise ValueError("corrupt length crc")
        payload = data[i + 12:i + 12 + n]
        (pc,) = struct.unpack("<I", data[i + 12 + n:i + 16 + n])
        if pc != crc32c(payload, masked=True):
            raise ValueError("corrupt payload crc")
        i += 16 + n
        ev = {"scalars": {}}
        for fld, _, v in _fields(payload):
            if fld == 1:
                ev["wall_time"] = struct.unpack("<d", v)[0]
            elif fld == 2:
                ev["step"] = v
            elif fld == 3:
                ev["file_version"] = v.decode()
            elif fld == 5:
                for f2, _, val in _fields(v):
                    if f2 != 1:
                        continue
                    tag, sv = None, None
                    for f3, _, x in _fields(val):
                        if f3 == 1:
                            tag = x.decode()
                        elif f3 == 2:
                            sv = struct.unpack("<f", x)[0]
                    ev["scalars"][tag] = sv
        out.append(ev)
    return out
