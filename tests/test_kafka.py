"""Kafka path of the streaming app (reference ``App.java:134-143``: FlinkKafkaConsumer /
FlinkKafkaProducer with ``MessageDeserializationSchema`` / ``MessageSerializationSchema``),
exercised through an in-memory fake ``kafka`` module injected into ``sys.modules`` (no broker,
no package).  Checks the consumer/producer wiring, the reference's end-of-stream rule
(``MessageDeserializationSchema.java:34-40``: the stream ends once more than max_count
messages were deserialized) and the full train -> serve job of ``app.main(["--kafka"])``."""
import json
import os
import sys
import types

import pytest

from textsummarization_on_flink_amd.api import app
from textsummarization_on_flink_amd.api.io import KafkaSink, KafkaSource
from textsummarization_on_flink_amd.api.message import FIELDS, Message, MessageDeserializationSchema
from textsummarization_on_flink_amd.train import checkpoint as ckpt

from helpers import TINY_FLAGS, make_dataset


class FakeBroker:
    def __init__(self):
        self.topics = {}
        self.consumers = []
        self.producers = []

    def module(self):
        broker = self

        class Msg:
            def __init__(self, value):
                self.value = value

        class KafkaConsumer:
            def __init__(self, topic, bootstrap_servers=None, group_id=None, auto_offset_reset="latest"):
                self.topic, self.bootstrap, self.group, self.reset = topic, bootstrap_servers, group_id, auto_offset_reset
                self.closed = False
                broker.consumers.append(self)

            def __iter__(self):  # a real consumer blocks for more; the fake ends with the topic
                for v in list(broker.topics.get(self.topic, [])):
                    yield Msg(v)

            def close(self):
                self.closed = True

        class KafkaProducer:
            def __init__(self, bootstrap_servers=None):
                self.bootstrap = bootstrap_servers
                self.flushed = self.closed = False
                broker.producers.append(self)

            def send(self, topic, value):
                assert isinstance(value, bytes)
                broker.topics.setdefault(topic, []).append(value)

            def flush(self):
                self.flushed = True

            def close(self):
                self.closed = True

        m = types.ModuleType("kafka")
        m.KafkaConsumer, m.KafkaProducer = KafkaConsumer, KafkaProducer
        return m


@pytest.fixture
def broker(monkeypatch):
    b = FakeBroker()
    monkeypatch.setitem(sys.modules, "kafka", b.module())
    return b


def _msg(i, prefix="uuid"):
    return Message(f"{prefix}-{i}", f"article number {i} . it has words .", "", f"reference {i} .").to_json().encode()


def test_source_reads_topic_until_end_of_stream(broker):
    broker.topics["t"] = [_msg(i) for i in range(12)]
    src = KafkaSource("t", "10.0.0.1:9092", "grp", deserializer=MessageDeserializationSchema(8))
    src.open()
    rows = list(src)
    src.close()
    c = broker.consumers[0]
    assert (c.topic, c.bootstrap, c.group, c.reset) == ("t", "10.0.0.1:9092", "grp", "earliest")
    assert c.closed
    # counter > max_count ends the stream: the 9th message is deserialized but not emitted
    assert [r[0] for r in rows] == [f"uuid-{i}" for i in range(8)]
    assert list(rows[3]) == [f"uuid-3", "article number 3 . it has words .", "", "reference 3 ."]


def test_sink_serializes_rows_and_skips_bad_ones(broker):
    sink = KafkaSink("out", "h:1")
    sink.open(None)
    sink.write(("a", "b", "c", "d"))
    sink.write(("only", "three", "fields"))  # reference: log and emit empty bytes
    sink.flush()
    sink.close()
    p = broker.producers[0]
    assert p.bootstrap == "h:1" and p.flushed and p.closed
    first, bad = broker.topics["out"]
    assert Message.from_json(first) == Message("a", "b", "c", "d")
    assert bad == b""


def test_missing_package_is_a_clear_error(monkeypatch):
    monkeypatch.setitem(sys.modules, "kafka", None)
    with pytest.raises(ImportError, match="kafka-python"):
        KafkaSource("t").open()
    with pytest.raises(ImportError, match="kafka-python"):
        KafkaSink("t").open(None)


def test_app_kafka_train_then_serve(broker, tmp_path, monkeypatch):
    """``App.main --kafka``: train from flink_train, then summarise flink_input into flink_output."""
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    _, vp, corpus = make_dataset(str(tmp_path))
    os.replace(vp, str(tmp_path / "vocab"))
    rows = corpus.rows(14, "k")
    enc = lambda r, pre: Message(r["uuid"].replace("k", pre), r["article"], r["summary"], r["reference"]).to_json().encode()
    broker.topics[app.TRAIN_TOPIC] = [enc(r, "train") for r in rows[:10]]
    broker.topics[app.INPUT_TOPIC] = [enc(r, "q") for r in rows[10:]]
    extra = [f"--extra-flag={f}" for f in TINY_FLAGS] + ["--extra-flag=--num_steps=2"]
    assert app.main(["--root", str(tmp_path), "--kafka", *extra]) == 0
    # consumers: train topic then input topic, group "bode", broker address of App.java
    assert [c.topic for c in broker.consumers] == [app.TRAIN_TOPIC, app.INPUT_TOPIC]
    assert all(c.group == app.CONSUMER_GROUP and c.bootstrap == app.KAFKA_ADDRESS for c in broker.consumers)
    assert ckpt.latest_checkpoint(f"{tmp_path}/log/pretrained_model/train")
    out = [Message.from_json(v) for v in broker.topics[app.OUTPUT_TOPIC]]
    assert sorted(m.uuid for m in out) == sorted(r["uuid"].replace("k", "q") for r in rows[10:])
    assert all(isinstance(m.summary, str) and m.reference for m in out)
    assert all(json.loads(v).keys() >= set(FIELDS) for v in broker.topics[app.OUTPUT_TOPIC])
