"""MI355X-native abstractive summarization (pointer-generator + coverage) training and
serving framework with a Flink-ML-style Estimator/Model/Pipeline API.

Capabilities of yangzichuang/TextSummarization-On-Flink, re-designed for AMD Instinct
MI355X (gfx950): hand-written HIP/CDNA4 kernels for the recurrences, attention and the
fused pointer loss, hipGraph-captured steps, data parallelism over RCCL/xGMI.
"""
__version__ = "0.1.0"
