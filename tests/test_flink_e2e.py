"""End-to-end streaming pipeline on the CPU oracle backend, mirroring the reference's
TensorFlowTest (testModelTraining, testInferenceAfterTraining, testJsonExportImport,
testPipeline) plus the fixes: train+infer in ONE job (Issue-1), DP over 2 workers."""
import glob
import os

import pytest

from textsummarization_on_flink_amd.api import (Pipeline, Row, SelectColTransformer, StreamEnvironment,
                                                SummarizationModel)
from textsummarization_on_flink_amd.api import app
from textsummarization_on_flink_amd.api.io import CollectionSource, JsonLinesSink, JsonLinesSource
from textsummarization_on_flink_amd.api.message import FIELDS, Message
from textsummarization_on_flink_amd.train import checkpoint as ckpt

from helpers import TINY_FLAGS, make_dataset

EXTRA = [f for f in TINY_FLAGS] + ["--max_to_keep=3"]


@pytest.fixture
def root(tmp_path, monkeypatch):
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    d, vp, corpus = make_dataset(str(tmp_path))
    os.replace(vp, str(tmp_path / "vocab"))
    return tmp_path, corpus


def _rows(corpus, n, prefix="uuid"):
    return [Row(*[r[k] for k in FIELDS]) for r in corpus.rows(n, prefix)]


def test_model_training_then_inference(root):
    tmp, corpus = root
    js = app.start_training(CollectionSource(_rows(corpus, 8)), str(tmp), EXTRA + ["--num_steps=2"], EXTRA,
                            echo=False)
    latest = ckpt.latest_checkpoint(f"{tmp}/log/pretrained_model/train")
    assert latest and latest.endswith("model.ckpt-2")
    # testJsonExportImport: the model JSON restores every inference param
    m = SummarizationModel().load_json(js)
    assert m.get_inference_selected_cols() == ["uuid", "article", "reference"]
    assert "--mode=decode" in m.get_inference_hyper_params()
    # testInferenceAfterTraining: a NEW environment consumes the JSON
    out_path = tmp / "out.jsonl"
    app.start_inference(js, CollectionSource(_rows(corpus, 5, "q")), [JsonLinesSink(str(out_path))], str(tmp),
                        EXTRA, echo=False)
    msgs = [Message.from_json(x) for x in open(out_path)]
    assert sorted(m.uuid for m in msgs) == [f"q-{i}" for i in range(5)]
    assert all(isinstance(m.summary, str) and m.reference for m in msgs)


def test_train_and_infer_in_one_job_pipeline(root):
    """Issue-1 fixed: Pipeline(fit) with an Estimator and the fitted model's transform run in
    ONE env.execute(); inference starts after training has written its checkpoint."""
    tmp, corpus = root
    env = StreamEnvironment()
    t = env.from_collection(_rows(corpus, 8), ",".join(FIELDS))
    est = app.create_estimator(str(tmp), EXTRA + ["--num_steps=1"], EXTRA)
    fitted = Pipeline().append_stage(est).fit(env, t)
    model = fitted.get_stages()[0]
    q = env.from_collection(_rows(corpus, 3, "q"), ",".join(FIELDS))
    out = Pipeline().append_stage(SelectColTransformer().set_selected_cols(["uuid", "article", "reference"])) \
        .append_stage(model).transform(env, q).collect()
    env.execute()
    assert ckpt.latest_checkpoint(f"{tmp}/log/pretrained_model/train").endswith("model.ckpt-1")
    assert sorted(r[0] for r in out) == ["q-0", "q-1", "q-2"]


def test_data_parallel_training_two_workers(root):
    """worker_num=2: two worker processes, gloo all-reduce, lock-step end of stream; only
    the chief writes the checkpoint."""
    tmp, corpus = root
    jsonl = tmp / "train.jsonl"
    with open(jsonl, "w") as f:
        for r in corpus.rows(16):
            f.write(Message(**r).to_json() + "\n")
    app.start_training(JsonLinesSource(str(jsonl)), str(tmp), EXTRA + ["--num_steps=0"], EXTRA, worker_num=2,
                       echo=False)
    # 16 rows / 2 workers / batch 4 = 2 steps on each rank
    latest = ckpt.latest_checkpoint(f"{tmp}/log/pretrained_model/train")
    assert latest.endswith("model.ckpt-2")
    assert len(glob.glob(f"{tmp}/log/pretrained_model/train/*.index")) == 1
