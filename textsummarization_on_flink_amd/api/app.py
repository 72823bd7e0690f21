"""End-to-end streaming summarization app (reference ``App.java:28-208``).

  train:     source(train rows) -> Table(uuid,article,summary,reference) -> print
             -> SummarizationEstimator.fit -> env.execute() -> model.to_json()
  inference: source(input rows) -> select(uuid,article,reference) -> SummarizationModel
             .load_json(json).transform -> print + sink(output)

Kafka topics (``flink_train`` / ``flink_input`` / ``flink_output``) become pluggable
sources/sinks: JSON-lines files or TCP sockets by default, Kafka when ``kafka-python`` is
available.  Hyper-parameters mirror ``App.java:55-81`` (``--batch_size=2``,
``--coverage=1``, ``--num_steps=1`` for training; ``--mode=decode --single_pass=1
--inference=1`` for serving).

    python -m textsummarization_on_flink_amd.api.app --root DIR --train-jsonl train.jsonl \\
        --input-jsonl in.jsonl --output-jsonl out.jsonl [--extra-flag=--hidden_dim=64 ...]
"""
from __future__ import annotations

import argparse
import logging
import os
from typing import List, Optional, Sequence

from .io import JsonLinesSink, JsonLinesSource, KafkaSink, KafkaSource, PrintSink
from .message import FIELDS
from .stages import SummarizationEstimator, SummarizationModel
from .table import StreamEnvironment
from .types import DataTypes

log = logging.getLogger(__name__)
MAX_ROW_COUNT = 8
TRAIN_TOPIC, INPUT_TOPIC, OUTPUT_TOPIC = "flink_train", "flink_input", "flink_output"
CONSUMER_GROUP, KAFKA_ADDRESS = "bode", "127.0.0.1:9092"
HYPERPARAMETER_KEY = "TF_Hyperparameter"
SCRIPTS = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "flink_entry.py")]
MAP_FUNC = "main_on_flink"


def inference_hyperparameter(root: str, exp_name: str = "pretrained_model", extra: Sequence[str] = ()) -> List[str]:
    return ["run_summarization.py", "--mode=decode", f"--data_path={root}/data/test_input",
            f"--vocab_path={root}/vocab", f"--log_root={root}/log", f"--exp_name={exp_name}", "--batch_size=2",
            "--max_enc_steps=400", "--max_dec_steps=100", "--coverage=1", "--single_pass=1", "--inference=1",
            *extra]


def train_hyperparameter(root: str, exp_name: str = "pretrained_model", extra: Sequence[str] = ()) -> List[str]:
    return ["run_summarization.py", "--mode=train", f"--data_path={root}/data/train_input",
            f"--vocab_path={root}/vocab", f"--log_root={root}/log", f"--exp_name={exp_name}", "--batch_size=2",
            "--max_enc_steps=400", "--max_dec_steps=100", "--coverage=1", "--num_steps=1", *extra]


def create_model(root: str, extra: Sequence[str] = (), worker_num: int = 1) -> SummarizationModel:
    """App.java:145-160."""
    return (SummarizationModel()
            .set_zookeeper_conn_str("127.0.0.1:2181").set_worker_num(worker_num).set_ps_num(0)
            .set_inference_scripts(SCRIPTS).set_inference_map_func(MAP_FUNC)
            .set_inference_hyper_params_key(HYPERPARAMETER_KEY)
            .set_inference_hyper_params(inference_hyperparameter(root, extra=extra))
            .set_inference_env_path(None)
            .set_inference_selected_cols(["uuid", "article", "reference"])
            .set_inference_output_cols(list(FIELDS))
            .set_inference_output_types([DataTypes.STRING] * 4))


def create_estimator(root: str, extra_train: Sequence[str] = (), extra_infer: Sequence[str] = (),
                     worker_num: int = 1) -> SummarizationEstimator:
    """App.java:162-187."""
    return (SummarizationEstimator()
            .set_zookeeper_conn_str("127.0.0.1:2181").set_worker_num(worker_num).set_ps_num(0)
            .set_train_scripts(SCRIPTS).set_train_map_func(MAP_FUNC)
            .set_train_hyper_params_key(HYPERPARAMETER_KEY)
            .set_train_hyper_params(train_hyperparameter(root, extra=extra_train))
            .set_train_env_path(None)
            .set_train_selected_cols(["uuid", "article", "reference"])
            .set_train_output_cols(["uuid"])
            .set_train_output_types([DataTypes.STRING])
            .set_inference_scripts(SCRIPTS).set_inference_map_func(MAP_FUNC)
            .set_inference_hyper_params_key(HYPERPARAMETER_KEY)
            .set_inference_hyper_params(inference_hyperparameter(root, extra=extra_infer))
            .set_inference_env_path(None)
            .set_inference_selected_cols(["uuid", "article", "reference"])
            .set_inference_output_cols(list(FIELDS))
            .set_inference_output_types([DataTypes.STRING] * 4))


def start_training(source, root: str, extra_train: Sequence[str] = (), extra_infer: Sequence[str] = (),
                   worker_num: int = 1, echo: bool = True) -> str:
    """App.java:83-106 -> model JSON."""
    env = StreamEnvironment.create_local_environment(1)
    inp = env.from_source(source, list(FIELDS))
    if echo:
        inp.print_schema()
        inp.print()
    model = create_estimator(root, extra_train, extra_infer, worker_num).fit(env, inp)
    env.execute("train")
    js = model.to_json()
    log.info("trained model: %s", js)
    return js


def start_inference(model_json: Optional[str], source, sinks=(), root: str = ".", extra: Sequence[str] = (),
                    worker_num: int = 1, echo: bool = True):
    """App.java:108-132."""
    env = StreamEnvironment.create_local_environment(1)
    inp = env.from_source(source, list(FIELDS))
    if echo:
        inp.print()
    inp = inp.select("uuid,article,reference")
    model = create_model(root, extra, worker_num)
    if model_json is not None:
        model.load_json(model_json)
    out = model.transform(env, inp)
    if echo:
        out.print()
    for s in sinks:
        out.add_sink(s)
    env.execute("inference")
    return out


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--root", required=True, help="dir holding vocab, data/ and log/")
    p.add_argument("--train-jsonl")
    p.add_argument("--input-jsonl")
    p.add_argument("--output-jsonl")
    p.add_argument("--kafka", action="store_true", help="use Kafka topics instead of JSONL files")
    p.add_argument("--workers", type=int, default=1)
    p.add_argument("--extra-flag", action="append", default=[], help="extra run_summarization flag (repeatable)")
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    js = None
    if a.kafka:
        js = start_training(KafkaSource(TRAIN_TOPIC, KAFKA_ADDRESS, CONSUMER_GROUP), a.root, a.extra_flag,
                            a.extra_flag, a.workers)
        start_inference(js, KafkaSource(INPUT_TOPIC, KAFKA_ADDRESS, CONSUMER_GROUP), [KafkaSink(OUTPUT_TOPIC)],
                        a.root, a.extra_flag, a.workers)
        return 0
    if a.train_jsonl:
        js = start_training(JsonLinesSource(a.train_jsonl), a.root, a.extra_flag, a.extra_flag, a.workers)
    if a.input_jsonl:
        sinks = [JsonLinesSink(a.output_jsonl)] if a.output_jsonl else [PrintSink()]
        start_inference(js, JsonLinesSource(a.input_jsonl), sinks, a.root, a.extra_flag, a.workers)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
