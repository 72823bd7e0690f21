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


def test_tensorboard_event_roundtrip(tmp_path):
    from textsummarization_on_flink_amd.utils.tensorboard import EventWriter, read_events
    w = EventWriter(str(tmp_path / "train"))
    w.add_scalars(1, {"loss": 7.5, "coverage_loss": 0.25})
    w.add_scalars(2, {"loss": 7.25, "global_norm": 1.5})
    w.close()
    evs = read_events(w.path)
    assert evs[0]["file_version"] == "brain.Event:2"
    assert [e["step"] for e in evs[1:]] == [1, 2]
    assert evs[1]["scalars"] == {"loss": 7.5, "coverage_loss": 0.25}
    assert evs[2]["scalars"]["global_norm"] == 1.5
    raw = bytearray(open(w.path, "rb").read())
    raw[-6] ^= 0xFF  # corrupt the last payload: the masked crc32c must catch it
    open(w.path, "wb").write(bytes(raw))
    import pytest
    with pytest.raises(ValueError):
        read_events(w.path)


def test_metrics_logger_writes_reference_summary_tags(tmp_path):
    from textsummarization_on_flink_amd.train.loop import MetricsLogger
    from textsummarization_on_flink_amd.utils.tensorboard import read_events
    m = MetricsLogger(str(tmp_path / "m.jsonl"), tb_dir=str(tmp_path / "eval"))
    m.log(step=3, eval_loss=6.0, running_avg_loss=6.5)
    m.close()
    (f,) = [p for p in os.listdir(tmp_path / "eval") if p.startswith("events.out.tfevents.")]
    sc = read_events(str(tmp_path / "eval" / f))[1]["scalars"]
    assert sc == {"loss": 6.0, "running_avg_loss/decay=0.990000": 6.5}
