"""Pipeline stages: ``Estimator`` / ``Model`` / ``Transformer`` / ``Pipeline`` and the
summarization estimator/model (reference ``TFEstimator.java``, ``TFModel.java``; Flink-ML
1.9 interfaces).

``SummarizationEstimator.fit(env, table)`` wires a TRAIN worker job into the lazy DAG and
returns a ``SummarizationModel`` carrying only inference metadata (weights live in
``<log_root>/<exp_name>/train``, as in the reference); the job runs at ``env.execute()``.
``SummarizationModel.transform(env, table)`` wires an INFERENCE worker job and returns its
output table (``uuid, article, summary, reference``).

Deliberate fixes:
  * the fitted model also receives ``inference_hyper_params_key`` (the reference forgot it,
    ``TFEstimator.java:86-96``, so ``fit -> transform`` without ``loadJson`` failed);
  * train and inference in ONE job (Issue-1): a model transformed in the same environment
    as its ``fit`` starts its workers after training finished, buffering input meanwhile;
  * ``Pipeline.fit`` with an Estimator stage works (it was commented out in the reference
    test because of Issue-1).
"""
from __future__ import annotations

import importlib
import json
from typing import List, Optional

from .coding import CodingUtils
from .params import (HasClusterConfig, HasInferenceOutputCols, HasInferenceOutputTypes, HasInferencePythonConfig,
                     HasInferenceSelectedCols, HasTrainOutputCols, HasTrainOutputTypes, HasTrainPythonConfig,
                     HasTrainSelectedCols, Params, WithParams)
from .table import ExternalNode, StreamEnvironment, Table
from .types import TableSchema
from .worker import WorkerConfig, WorkerJob

HYPER_PARAMS_KEY_PROP = "sys:hyper_params_key"


class PipelineStage(WithParams):
    def to_json(self) -> str:
        return self.get_params().to_json()

    def load_json(self, s: str):
        self.get_params().load_json(s)
        return self

    toJson, loadJson = to_json, load_json


class Transformer(PipelineStage):
    def transform(self, env: StreamEnvironment, table: Table) -> Table:
        raise NotImplementedError


class Model(Transformer):
    pass


class Estimator(PipelineStage):
    def fit(self, env: StreamEnvironment, table: Table) -> Model:
        raise NotImplementedError


class SelectColTransformer(Transformer):
    """A pure table transformer (``TensorFlowTest.java:263-279``)."""
    from .params import ParamInfo as _PI
    SELECTED_COLS = _PI("selectedCols", list, "Names of the columns to select", True)

    def set_selected_cols(self, cols):
        return self.set(self.SELECTED_COLS, list(cols))

    def get_selected_cols(self):
        return self.get(self.SELECTED_COLS)

    setSelectedCols, getSelectedCols = set_selected_cols, get_selected_cols

    def transform(self, env, table):
        return table.select(self.get_selected_cols())


def _stage_class_name(stage) -> str:
    return f"{type(stage).__module__}:{type(stage).__qualname__}"


def _load_stage_class(name: str):
    mod, _, qual = name.partition(":")
    obj = importlib.import_module(mod)
    for part in qual.split("."):
        obj = getattr(obj, part)
    return obj


class Pipeline(Estimator):
    """Chains stages; ``fit`` fits each Estimator on the running table and transforms the
    table for the next stage; ``transform`` applies every stage (all must be Transformers)."""

    def __init__(self, stages: Optional[List[PipelineStage]] = None):
        self.stages: List[PipelineStage] = list(stages or [])

    def append_stage(self, stage: PipelineStage) -> "Pipeline":
        self.stages.append(stage)
        return self

    appendStage = append_stage

    def get_stages(self):
        return list(self.stages)

    def need_fit(self) -> bool:
        return any(isinstance(s, Estimator) for s in self.stages)

    def fit(self, env, table) -> "Pipeline":
        last_est = max((i for i, s in enumerate(self.stages) if isinstance(s, Estimator)), default=-1)
        out = []
        for i, s in enumerate(self.stages):
            if isinstance(s, Estimator):
                m = s.fit(env, table)
                out.append(m)
                if i < last_est:
                    table = m.transform(env, table)
            else:
                out.append(s)
                if i < last_est:
                    table = s.transform(env, table)
        return Pipeline(out)

    def transform(self, env, table) -> Table:
        for s in self.stages:
            if not isinstance(s, Transformer):
                raise TypeError(f"stage {type(s).__name__} is not a Transformer; fit the pipeline first")
            table = s.transform(env, table)
        return table

    def to_json(self) -> str:
        return json.dumps([{"stageClassName": _stage_class_name(s), "stageJson": s.to_json()} for s in self.stages])

    def load_json(self, s: str) -> "Pipeline":
        for d in json.loads(s):
            stage = _load_stage_class(d["stageClassName"])()
            stage.load_json(d["stageJson"])
            self.stages.append(stage)
        return self

    toJson, loadJson = to_json, load_json


# ---------------------------------------------------------------------- summarization stages
def _job_factory(config: WorkerConfig, name: str):
    return lambda on_output: WorkerJob(config, on_output=on_output, name=name)


class SummarizationModel(Model, HasClusterConfig, HasInferencePythonConfig, HasInferenceSelectedCols,
                         HasInferenceOutputCols, HasInferenceOutputTypes):
    """TFModel.java:29-87."""

    def __init__(self):
        self._after = None  # (env, ExternalNode) of the training job that produced this model

    def configure_input_table(self, raw: Table) -> Table:
        return raw.select(self.get_inference_selected_cols())

    def configure_output_schema(self) -> TableSchema:
        return TableSchema(self.get_inference_output_cols(), self.get_inference_output_types())

    def configure_config(self) -> WorkerConfig:
        key = self.get_inference_hyper_params_key()
        props = {"zookeeper_connect_str": self.get_zookeeper_conn_str(), HYPER_PARAMS_KEY_PROP: key,
                 key: " ".join(self.get_inference_hyper_params())}
        return WorkerConfig(self.get_worker_num(), self.get_ps_num(), props, list(self.get_inference_scripts()),
                            self.get_inference_map_func(), self.get_inference_env_path())

    def transform(self, env: StreamEnvironment, table: Table) -> Table:
        inp = self.configure_input_table(table)
        out_schema = self.configure_output_schema()
        cfg = self.configure_config()
        CodingUtils.configure_example_coding(cfg.properties, inp.get_schema(), out_schema)
        cfg.validate()
        after = self._after[1] if self._after and self._after[0] is env else None
        node = ExternalNode(env, _job_factory(cfg, "inference"), CodingUtils.input_coding(cfg.properties),
                            out_schema, CodingUtils.output_coding(cfg.properties), name="inference", after=after)
        inp.node.connect(node)
        return Table(env, node)


class SummarizationEstimator(Estimator, HasClusterConfig, HasTrainPythonConfig, HasInferencePythonConfig,
                             HasTrainSelectedCols, HasTrainOutputCols, HasTrainOutputTypes, HasInferenceSelectedCols,
                             HasInferenceOutputCols, HasInferenceOutputTypes):
    """TFEstimator.java:26-108."""

    def configure_input_table(self, raw: Table) -> Optional[Table]:
        cols = self.get_train_selected_cols()
        return raw.select(cols) if len(cols) else None

    def configure_output_schema(self) -> Optional[TableSchema]:
        cols = self.get_train_output_cols()
        return TableSchema(cols, self.get_train_output_types()) if len(cols) else None

    def configure_config(self) -> WorkerConfig:
        key = self.get_train_hyper_params_key()
        props = {"zookeeper_connect_str": self.get_zookeeper_conn_str(), HYPER_PARAMS_KEY_PROP: key,
                 key: " ".join(self.get_train_hyper_params())}
        return WorkerConfig(self.get_worker_num(), self.get_ps_num(), props, list(self.get_train_scripts()),
                            self.get_train_map_func(), self.get_train_env_path())

    def fit(self, env: StreamEnvironment, table: Table) -> SummarizationModel:
        inp = self.configure_input_table(table)
        out_schema = self.configure_output_schema()
        cfg = self.configure_config()
        CodingUtils.configure_example_coding(cfg.properties, inp.get_schema() if inp is not None else None,
                                             out_schema)
        cfg.validate()
        out_coding = CodingUtils.output_coding(cfg.properties)
        node = ExternalNode(env, _job_factory(cfg, "train"), CodingUtils.input_coding(cfg.properties), out_schema,
                            out_coding, name="train")
        if inp is not None:
            inp.node.connect(node)
        self.train_output = Table(env, node) if out_schema is not None else None
        m = SummarizationModel()
        for info in (HasClusterConfig.ZOOKEEPER_CONNECT_STR, HasClusterConfig.WORKER_NUM, HasClusterConfig.PS_NUM,
                     HasInferencePythonConfig.INFERENCE_SCRIPTS, HasInferencePythonConfig.INFERENCE_MAP_FUNC,
                     HasInferencePythonConfig.INFERENCE_HYPER_PARAMS_KEY,
                     HasInferencePythonConfig.INFERENCE_HYPER_PARAMS, HasInferencePythonConfig.INFERENCE_ENV_PATH,
                     HasInferenceSelectedCols.INFERENCE_SELECTED_COLS, HasInferenceOutputCols.INFERENCE_OUTPUT_COLS,
                     HasInferenceOutputTypes.INFERENCE_OUTPUT_TYPES):
            if self.get_params().contains(info) or info.has_default_value:
                m.set(info, self.get(info))
        m._after = (env, node)
        return m


TFEstimator = SummarizationEstimator
TFModel = SummarizationModel


def run_python(env: StreamEnvironment, input_table: Optional[Table], config: WorkerConfig,
               output_schema: Optional[TableSchema], name: str = "python") -> Optional[Table]:
    """``TFUtils.train / inference`` equivalent: run ``config.func_name`` from
    ``config.python_files`` in ``worker_num`` processes over ``input_table`` (None = no
    input) and return the output table (None when ``output_schema`` is None)."""
    CodingUtils.configure_example_coding(config.properties, input_table.get_schema() if input_table is not None
                                         else None, output_schema)
    config.validate()
    node = ExternalNode(env, _job_factory(config, name), CodingUtils.input_coding(config.properties), output_schema,
                        CodingUtils.output_coding(config.properties), name=name)
    if input_table is not None:
        input_table.node.connect(node)
    return Table(env, node) if output_schema is not None else None
