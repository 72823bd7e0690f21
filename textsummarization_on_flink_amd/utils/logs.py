"""Logging setup: console + optional size-rotated file.

Equivalent of the reference's log4j2 configuration (``src/main/resources/log4j2.xml:3-23``:
console appender plus a rolling file ``target/log/tensorflow-on-flink.log``, 100 MB x 20).
Idempotent: calling it again replaces the handlers it installed before, so a worker that
re-initialises (restart after a failure) does not duplicate every line.
"""
from __future__ import annotations

import logging
import logging.handlers
import os
from typing import Optional

FORMAT = "%(asctime)s %(levelname)s %(name)s: %(message)s"
ROLL_BYTES = 100 * 1024 * 1024
ROLL_COUNT = 20
_MARK = "_tsamd_handler"


def setup_logging(level=logging.INFO, log_file: Optional[str] = None, max_bytes: int = ROLL_BYTES,
                  backup_count: int = ROLL_COUNT, rank: Optional[int] = None) -> logging.Logger:
    """Configure the root logger: a console handler and, when ``log_file`` is given, a
    ``RotatingFileHandler`` (``max_bytes`` x ``backup_count``).  ``rank`` (multi-GPU) is
    added to every record and appended to the file name, one file per rank."""
    root = logging.getLogger()
    for h in list(root.handlers):
        if getattr(h, _MARK, False):
            root.removeHandler(h)
            h.close()
    fmt = FORMAT if rank is None else FORMAT.replace("%(name)s", f"[rank {rank}] %(name)s")
    console = logging.StreamHandler()
    console.setFormatter(logging.Formatter(fmt))
    setattr(console, _MARK, True)
    root.addHandler(console)
    if log_file:
        if rank is not None:
            stem, ext = os.path.splitext(log_file)
            log_file = f"{stem}.rank{rank}{ext}"
        os.makedirs(os.path.dirname(os.path.abspath(log_file)), exist_ok=True)
        fh = logging.handlers.RotatingFileHandler(log_file, maxBytes=max_bytes, backupCount=backup_count)
        fh.setFormatter(logging.Formatter(fmt))
        setattr(fh, _MARK, True)
        root.addHandler(fh)
    root.setLevel(level)
    return root


def project_root() -> str:
    """Project root directory (reference ``SysUtils.java:4-6`` uses ``user.dir``)."""
    return os.getcwd()
