"""utils: rotating log setup (log4j2.xml equivalent) and the non-finite tensor report."""
import logging
import logging.handlers
import os

import torch

from textsummarization_on_flink_amd.utils import NonFiniteWatch, nonfinite_report, setup_logging


def test_setup_logging_rotates_and_is_idempotent(tmp_path):
    path = str(tmp_path / "l" / "app.log")
    setup_logging(logging.INFO, log_file=path, max_bytes=2000, backup_count=3)
    setup_logging(logging.INFO, log_file=path, max_bytes=2000, backup_count=3)  # no duplicate handlers
    lg = logging.getLogger("tsamd.test")
    for i in range(200):
        lg.info("line %04d %s", i, "x" * 40)
    files = sorted(os.listdir(tmp_path / "l"))
    assert files == ["app.log", "app.log.1", "app.log.2", "app.log.3"]
    assert all(os.path.getsize(tmp_path / "l" / f) <= 2100 for f in files)
    text = open(path).read()
    assert text.count("line 0199") == 1  # one handler, one copy of each record
    setup_logging(logging.INFO)  # back to console only
    assert not any(isinstance(h, logging.handlers.RotatingFileHandler) for h in logging.getLogger().handlers)


def test_setup_logging_per_rank_file(tmp_path):
    path = str(tmp_path / "r.log")
    setup_logging(logging.INFO, log_file=path, rank=3)
    logging.getLogger("tsamd.test").info("hello")
    setup_logging(logging.INFO)
    assert "[rank 3]" in open(tmp_path / "r.rank3.log").read()


def test_nonfinite_report_and_watch():
    a = torch.zeros(10)
    b = torch.tensor([1.0, float("nan"), float("inf"), -float("inf")])
    c = torch.arange(4)  # integer tensors are skipped
    rep = nonfinite_report([("a", a), ("b", b), ("c", c)])
    assert rep == [("b", 1, 2)]

    class T:
        def named_debug_tensors(self):
            yield "grad/x", b
            yield "param/y", a

    assert [r[0] for r in NonFiniteWatch(T()).check(7)] == ["grad/x"]
