"""Pipeline API parity: Params/JSON, DataTypes coding, lazy tables, worker jobs mirroring
the reference's InputOutputTest (encode+decode / encode only / decode only / neither) and
SourceSinkTest (results are emitted immediately, Issue-6)."""
import os
import time

import pytest

from textsummarization_on_flink_amd.api import (CodingUtils, CollectSink, CsvCoding, DataTypes, ExampleCoding,
                                                JobExecutionError, Message, MessageDeserializationSchema,
                                                MessageSerializationSchema, Params, Pipeline, Row,
                                                SelectColTransformer, StreamEnvironment, SummarizationEstimator,
                                                SummarizationModel, TableSchema, TimedSource, TypeInformation,
                                                WorkerConfig, run_python)
from textsummarization_on_flink_amd.api.params import HasClusterConfig

STUBS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "flink_stubs.py")


# ---------------------------------------------------------------------- params
def test_params_defaults_required_and_json():
    m = SummarizationModel()
    assert m.get_worker_num() == 1 and m.getPsNum() == 0
    assert m.get_zookeeper_conn_str() == "127.0.0.1:2181"
    assert m.get_inference_hyper_params() == [] and m.get_inference_env_path() is None
    with pytest.raises(ValueError, match="inference_scripts"):
        m.get_inference_scripts()
    m.setWorkerNum(3).set_inference_output_types([DataTypes.STRING, DataTypes.FLOAT_32_ARRAY])
    m.set_inference_scripts(["a.py", "b.py"]).set_inference_map_func("main_on_flink")
    js = m.to_json()
    m2 = SummarizationModel().load_json(js)
    assert m2.get_worker_num() == 3
    assert m2.get_inference_output_types() == [DataTypes.STRING, DataTypes.FLOAT_32_ARRAY]
    assert m2.get_inference_scripts() == ["a.py", "b.py"]
    assert Params.from_json(js) == m.get_params()
    # Flink-ML layout: name -> JSON-encoded value
    import json
    assert json.loads(js)["worker_num"] == "3"
    # load_json overlays
    m3 = SummarizationModel().set_worker_num(5).set_ps_num(0)
    m3.load_json('{"worker_num": "2"}')
    assert m3.get_worker_num() == 2 and m3.get(HasClusterConfig.PS_NUM) == 0


def test_estimator_passes_all_inference_params_to_model():
    est = (SummarizationEstimator().set_worker_num(2).set_train_scripts([STUBS]).set_train_map_func("f")
           .set_train_hyper_params_key("K").set_train_selected_cols(["input"]).set_train_output_cols([])
           .set_train_output_types([]).set_inference_scripts([STUBS]).set_inference_map_func("g")
           .set_inference_hyper_params_key("K2").set_inference_hyper_params(["x", "--mode=decode"])
           .set_inference_selected_cols(["input"]).set_inference_output_cols(["output"])
           .set_inference_output_types([DataTypes.STRING]))
    env = StreamEnvironment()
    model = est.fit(env, env.from_collection([Row("a")], "input"))
    assert model.get_inference_hyper_params_key() == "K2"  # reference defect fixed
    assert model.get_worker_num() == 2 and model.get_inference_map_func() == "g"


# ---------------------------------------------------------------------- types / coding
def test_data_types_mapping_and_unsupported():
    for dt in [DataTypes.STRING, DataTypes.BOOL, DataTypes.INT_8, DataTypes.INT_16, DataTypes.INT_32,
               DataTypes.INT_64, DataTypes.FLOAT_32, DataTypes.FLOAT_64, DataTypes.UINT_16, DataTypes.FLOAT_32_ARRAY]:
        assert CodingUtils.type_information_to_data_types(CodingUtils.data_types_to_type_information(dt)) == dt
    with pytest.raises(RuntimeError, match="Unsupported"):
        CodingUtils.data_types_to_type_information(DataTypes.FLOAT_16)
    with pytest.raises(RuntimeError, match="Unsupported"):
        CodingUtils.type_information_to_data_types(TypeInformation.DATE_TYPE_INFO)
    with pytest.raises(RuntimeError):
        CodingUtils.type_information_to_data_types(TypeInformation.DOUBLE_ARRAY_TYPE_INFO)


def test_example_and_csv_coding_roundtrip():
    names = ["s", "b", "i8", "i64", "f", "d", "c", "arr"]
    types = [DataTypes.STRING, DataTypes.BOOL, DataTypes.INT_8, DataTypes.INT_64, DataTypes.FLOAT_32,
             DataTypes.FLOAT_64, DataTypes.UINT_16, DataTypes.FLOAT_32_ARRAY]
    c = ExampleCoding(names, types)
    row = Row("héllo", True, -3, 1 << 40, 0.5, 2.25, "x", [1.0, -2.5])
    assert c.decode(c.encode(row)) == row
    assert c.decode(c.encode({"s": "a"})) == Row("a", None, None, None, None, None, None, None)
    csv = CsvCoding(["a", "b"], [DataTypes.STRING, DataTypes.INT_32])
    assert csv.encode(Row("x y", 7)) == b"x y#7"
    assert csv.decode(b"x y#7") == Row("x y", 7)
    props = {}
    CodingUtils.configure_example_coding(props, TableSchema(["a"], [DataTypes.STRING]), None)
    assert CodingUtils.input_coding(props) is not None and CodingUtils.output_coding(props) is None


def test_message_schemas():
    m = Message("u", "art", "sum", "ref")
    assert Message.from_json(m.to_json()) == m
    d = MessageDeserializationSchema(2)
    rows = []
    for i in range(5):
        r = d.deserialize(Message(f"u{i}", "a", "", "r").to_json().encode())
        if d.is_end_of_stream(r):
            break
        rows.append(r)
    assert [r[0] for r in rows] == ["u0", "u1"]  # bounded at max_count
    assert MessageSerializationSchema().serialize(Row(1, 2)) == b""  # logs, emits nothing


# ---------------------------------------------------------------------- lazy tables
def test_lazy_table_ops_and_fanout():
    env = StreamEnvironment.create_local_environment(1)
    t = env.from_collection([Row(f"u{i}", f"article {i}.", "", f"ref {i}.") for i in range(6)],
                            "uuid,article,summary,reference")
    a = t.select("uuid, reference").collect()
    b = t.where(lambda r: int(r[0][1:]) % 2 == 0).map(lambda r: Row(r[0].upper()), ["U"]).collect()
    assert a == [] and b == []  # nothing runs before execute()
    env.execute()
    assert a == [Row(f"u{i}", f"ref {i}.") for i in range(6)]
    assert b == [Row("U0"), Row("U2"), Row("U4")]
    with pytest.raises(KeyError):
        t.select("nope")


# ---------------------------------------------------------------------- worker jobs (InputOutputTest)
def _cfg(func, n=1):
    return WorkerConfig(worker_num=n, ps_num=0, properties={}, python_files=[STUBS], func_name=func, timeout_s=120)


def _data(n=10):
    return [Row(f"data-{i}") for i in range(n)]


@pytest.mark.parametrize("workers", [1, 2])
def test_example_coding_both_sides(workers):
    env = StreamEnvironment()
    out = run_python(env, env.from_collection(_data(), "input"), _cfg("test_example_coding", workers),
                     TableSchema(["output"], [DataTypes.STRING]))
    rows = out.collect()
    env.execute()
    assert sorted(r[0] for r in rows) == sorted(f"data-{i}" for i in range(10))


def test_example_coding_without_encode():
    env = StreamEnvironment()
    rows = run_python(env, None, _cfg("test_example_coding_without_encode"),
                      TableSchema(["output"], [DataTypes.STRING])).collect()
    env.execute()
    assert [r[0] for r in rows] == [f"output-{i}" for i in range(10)]


def test_example_coding_without_decode_and_nothing():
    env = StreamEnvironment()
    assert run_python(env, env.from_collection(_data(), "input"), _cfg("test_example_coding_without_decode"),
                      None) is None
    env.execute()
    env2 = StreamEnvironment()
    run_python(env2, None, _cfg("test_example_coding_with_nothing"), None)
    env2.execute()


def test_worker_failure_surfaces_and_ps_rejected():
    env = StreamEnvironment()
    run_python(env, env.from_collection(_data(3), "input"), _cfg("test_fail"),
               TableSchema(["output"], [DataTypes.STRING]))
    with pytest.raises(JobExecutionError, match="exited with code"):
        env.execute()
    cfg = _cfg("test_example_coding")
    cfg.ps_num = 1
    with pytest.raises(ValueError, match="ps_num"):
        cfg.validate()


def test_typed_rows_through_worker():
    names = ["s", "i", "f", "arr"]
    types = [DataTypes.STRING, DataTypes.INT_64, DataTypes.FLOAT_64, DataTypes.FLOAT_32_ARRAY]
    env = StreamEnvironment()
    src = [Row("a", 1, 0.5, [1.0, 2.0]), Row("b", -7, 3.25, [])]
    rows = run_python(env, env.from_collection(src, names, types), _cfg("test_types"),
                      TableSchema(names, types)).collect()
    env.execute()
    assert rows == src


def test_source_sink_emits_immediately():
    """SourceSinkTest: result k must reach the sink before input k+1 is produced."""
    n, interval = 8, 0.25
    src = TimedSource(n, interval)
    env = StreamEnvironment()
    sink = CollectSink()
    run_python(env, env.from_source(src), _cfg("test_source_sink"),
               TableSchema(["output", "t"], [DataTypes.STRING, DataTypes.FLOAT_64])).add_sink(sink)
    env.execute()
    assert [r[0] for r in sink.rows] == [f"data-{i}" for i in range(n)]
    # skip the first rows (worker process start-up); afterwards every result lands
    # before the next input is emitted
    for k in range(n // 2, n - 1):
        assert sink.times[k] < src.emit_times[k + 1], (k, sink.times[k], src.emit_times[k + 1])


def test_timed_source_state_snapshot_restore():
    s = TimedSource(5, 0.0)
    it = iter(s)
    next(it), next(it)
    snap = s.snapshot_state()
    s2 = TimedSource(5, 0.0)
    s2.restore_state(snap)
    assert [r[0] for r in s2] == ["data-2", "data-3", "data-4"]


def test_pipeline_json_roundtrip_and_select_transformer():
    p = Pipeline().append_stage(SelectColTransformer().set_selected_cols(["uuid", "article"])) \
        .append_stage(SummarizationModel().set_worker_num(2))
    p2 = Pipeline().load_json(p.to_json())
    assert [type(s).__name__ for s in p2.get_stages()] == ["SelectColTransformer", "SummarizationModel"]
    assert p2.get_stages()[1].get_worker_num() == 2
    env = StreamEnvironment()
    t = env.from_collection([Row("u", "a", "s", "r")], "uuid,article,summary,reference")
    rows = Pipeline([p2.get_stages()[0]]).transform(env, t).collect()
    env.execute()
    assert rows == [Row("u", "a")]
