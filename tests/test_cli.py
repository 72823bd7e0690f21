"""run_summarization-compatible CLI end to end on the CPU oracle backend:
train -> checkpoint -> resume -> eval (best model) -> decode single_pass (ROUGE files) ->
raw-text inference -> coverage conversion -> restore best; NaN fault injection."""
import glob
import json
import os

import pytest

from textsummarization_on_flink_amd import cli
from textsummarization_on_flink_amd.train import checkpoint as ckpt
from textsummarization_on_flink_amd.train.trainer import NonFiniteLossError

from helpers import TINY_FLAGS, make_dataset


@pytest.fixture
def ds(tmp_path):
    d, vp, _ = make_dataset(str(tmp_path))
    return tmp_path, d, vp


def _flags(tmp, d, vp, *extra, split="train"):
    return [f"--data_path={d}/{split}_*", f"--vocab_path={vp}", f"--log_root={tmp}/log", "--exp_name=exp",
            *TINY_FLAGS, *extra]


def test_train_resume_eval_decode(ds, monkeypatch):
    monkeypatch.setattr("torch.cuda.is_available", lambda: False)
    tmp, d, vp = ds
    assert cli.main(_flags(tmp, d, vp, "--mode=train", "--num_steps=3")) == 0
    train_dir = f"{tmp}/log/exp/train"
    latest = ckpt.latest_checkpoint(train_dir)
    assert latest and latest.endswith("model.ckpt-3")
    # metrics JSONL: one record per step with loss / global_norm / tokens/s
    recs = [json.loads(x) for x in open(f"{tmp}/log/exp/metrics_train.jsonl")]
    assert [r["step"] for r in recs] == [1, 2, 3]
    assert all(r["loss"] > 0 and r["global_norm"] > 0 and r["tokens_per_sec"] > 0 for r in recs)
    # TensorBoard scalars next to the checkpoints, with the reference's summary tags
    from textsummarization_on_flink_amd.utils.tensorboard import read_events
    (ev,) = glob.glob(f"{train_dir}/events.out.tfevents.*")
    tb = read_events(ev)[1:]
    assert [e["step"] for e in tb] == [1, 2, 3]
    assert {"loss", "total_loss", "global_norm"} <= set(tb[0]["scalars"])
    # resume: num_steps is relative to the restored step (StopAtStepHook semantics)
    assert cli.main(_flags(tmp, d, vp, "--mode=train", "--num_steps=2")) == 0
    assert ckpt.latest_checkpoint(train_dir).endswith("model.ckpt-5")
    # eval: single pass over val, best model saved with checkpoint_best
    from textsummarization_on_flink_amd.config import parse_flags
    from textsummarization_on_flink_amd.data.batcher import Batcher
    from textsummarization_on_flink_amd.train.loop import run_eval
    vocab, hps = cli.default_setup(parse_flags(_flags(tmp, d, vp, "--mode=eval", split="val")))
    best, avg = run_eval(hps, vocab, Batcher(hps.data_path, vocab, hps, single_pass=False, seed=0), max_iters=3)
    assert best is not None and best <= 12
    assert ckpt.latest_checkpoint(f"{tmp}/log/exp/eval", "checkpoint_best").endswith("bestmodel-5")
    # decode single pass: ROUGE files for every test example + results file
    assert cli.main(_flags(tmp, d, vp, "--mode=decode", "--single_pass=1", split="test")) == 0
    dec_dirs = glob.glob(f"{tmp}/log/exp/decode_*")  # dataset name: first of train/val/test in the path
    assert len(dec_dirs) == 1 and dec_dirs[0].endswith("ckpt-5")
    assert len(glob.glob(f"{dec_dirs[0]}/decoded/*_decoded.txt")) == 24
    assert len(glob.glob(f"{dec_dirs[0]}/reference/*_reference.txt")) == 24
    assert "ROUGE-1" in open(f"{dec_dirs[0]}/ROUGE_results.txt").read()


def test_inference_raw_text_and_conversions(ds, monkeypatch):
    monkeypatch.setattr("torch.cuda.is_available", lambda: False)
    tmp, d, vp = ds
    assert cli.main(_flags(tmp, d, vp, "--mode=train", "--num_steps=1", "--coverage=0")) == 0
    raw = tmp / "raw"
    raw.mkdir()
    for i in range(3):
        (raw / f"story{i}.txt").write_text(f"w{i} w1 w2 w3 . w4 w5 w6 w7 w8 . w9 w10")
    assert cli.main(_flags(tmp, d, vp, "--mode=decode", "--inference=1", "--single_pass=1") +
                    [f"--data_path={raw}/*.txt"]) == 0
    dec = glob.glob(f"{tmp}/log/exp/decode_*")
    assert dec and len(glob.glob(f"{dec[0]}/decoded/*")) == 3
    # coverage conversion: non-coverage ckpt -> <ckpt>_cov_init with coverage/w_c present
    assert cli.main(_flags(tmp, d, vp, "--mode=train", "--coverage=1", "--convert_to_coverage_model=1")) == 0
    conv = ckpt.latest_checkpoint(f"{tmp}/log/exp/train")
    assert conv.endswith("_cov_init")
    from textsummarization_on_flink_amd.runtime.tf_bundle import list_bundle
    names = list(list_bundle(conv))
    assert any("coverage/w_c" in n for n in names)


def test_restore_best_model(ds, monkeypatch):
    monkeypatch.setattr("torch.cuda.is_available", lambda: False)
    tmp, d, vp = ds
    assert cli.main(_flags(tmp, d, vp, "--mode=train", "--num_steps=2")) == 0
    from textsummarization_on_flink_amd.config import parse_flags
    from textsummarization_on_flink_amd.data.batcher import Batcher
    from textsummarization_on_flink_amd.train.loop import run_eval
    vocab, hps = cli.default_setup(parse_flags(_flags(tmp, d, vp, "--mode=eval", split="val")))
    run_eval(hps, vocab, Batcher(hps.data_path, vocab, hps, single_pass=False, seed=0), max_iters=1)
    assert cli.main(_flags(tmp, d, vp, "--mode=train", "--restore_best_model=1")) == 0
    assert os.path.exists(f"{tmp}/log/exp/train/model-2.index")


def test_nan_fault_injection_stops_training(ds, monkeypatch):
    monkeypatch.setattr("torch.cuda.is_available", lambda: False)
    tmp, d, vp = ds
    with pytest.raises(NonFiniteLossError, match="Loss is not finite"):
        cli.main(_flags(tmp, d, vp, "--mode=train", "--num_steps=5", "--fault_nan_step=2"))
    # the guard skipped the poisoned update; the two good steps were checkpointed on exit
    latest = ckpt.latest_checkpoint(f"{tmp}/log/exp/train")
    assert latest.endswith("model.ckpt-3")
    assert ckpt.inspect_checkpoint(latest)["some_infnan"] == []


def test_non_train_mode_requires_logdir(ds):
    tmp, d, vp = ds
    with pytest.raises(FileNotFoundError, match="Run in train mode"):
        cli.main(_flags(tmp, d, vp, "--mode=decode"))
    with pytest.raises(ValueError, match="single_pass"):
        cli.main(_flags(tmp, d, vp, "--mode=train", "--single_pass=1"))


def test_debug_watch_names_nonfinite_tensors(ds, monkeypatch, caplog):
    """--debug (tfdbg has_inf_or_nan): the step whose gradients carry NaN stops training and
    the report names the offending tensors."""
    monkeypatch.setattr("torch.cuda.is_available", lambda: False)
    tmp, d, vp = ds
    with pytest.raises(NonFiniteLossError, match="has_inf_or_nan"):
        cli.main(_flags(tmp, d, vp, "--mode=train", "--num_steps=5", "--fault_nan_step=1", "--debug=1"))
    msgs = [r.getMessage() for r in caplog.records if "has_inf_or_nan" in r.getMessage()]
    assert msgs and "grad/" in msgs[0]


def test_log_file_rotating_handler(ds, monkeypatch):
    monkeypatch.setattr("torch.cuda.is_available", lambda: False)
    tmp, d, vp = ds
    log_file = f"{tmp}/logs/run.log"
    cli.main(_flags(tmp, d, vp, "--mode=train", "--num_steps=1", f"--log_file={log_file}"))
    text = open(log_file).read()
    assert "Starting seq2seq_attention in train mode" in text
