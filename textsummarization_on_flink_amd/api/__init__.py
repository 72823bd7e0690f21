"""Flink-ML-style pipeline API over a lazy streaming table environment (SURVEY 2.1 J1-J19,
2.10): Params/ParamInfo/WithParams, DataTypes/TableSchema/Row, StreamEnvironment/Table,
sources & sinks, CodingUtils, Estimator/Model/Transformer/Pipeline, the summarization
estimator/model, and the worker-process runtime."""
from .coding import CodingUtils, CsvCoding, ExampleCoding
from .io import (CallbackSink, CollectionSource, CollectSink, JsonLinesSink, JsonLinesSource, KafkaSink, KafkaSource,
                 PrintSink, RingSource, SocketSink, SocketSource, TimedSource)
from .message import Message, MessageDeserializationSchema, MessageSerializationSchema
from .params import (HasClusterConfig, HasInferenceOutputCols, HasInferenceOutputTypes, HasInferencePythonConfig,
                     HasInferenceSelectedCols, HasTrainOutputCols, HasTrainOutputTypes, HasTrainPythonConfig,
                     HasTrainSelectedCols, ParamInfo, Params, WithParams)
from .stages import (Estimator, Model, Pipeline, PipelineStage, SelectColTransformer, SummarizationEstimator,
                     SummarizationModel, TFEstimator, TFModel, Transformer, run_python)
from .table import StreamEnvironment, StreamExecutionEnvironment, StreamTableEnvironment, Table, TableEnvironment
from .types import DataTypes, Row, TableSchema, TypeInformation
from .worker import JobExecutionError, WorkerConfig, WorkerContext
