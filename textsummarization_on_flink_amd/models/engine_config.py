"""Execution choices of the HIP engine: ONE documented object instead of scattered
environment reads.

Every field has a measured-best default (``auto`` ones depend on the shape and are resolved by
the engine).  ``EngineConfig.from_env()`` reads the ``TSAMD_*`` variables below (once, when an
engine is built); code can also pass a config explicitly.

| Variable                  | Field              | Default / meaning |
|---------------------------|--------------------|-------------------|
| TSAMD_LSTM_PERSISTENT     | persistent_lstm    | 1: one persistent weight-resident launch per bi-LSTM pass; 0: per-step kernels |
| TSAMD_ROW_ATTN            | row_attn           | auto (B >= 64): one workgroup per row; 0 / 1 force |
| TSAMD_SPLIT               | split              | auto (2 groups from B = 256, 4 from B = 1024): decoder row groups on parallel streams |
| TSAMD_SPLIT_BWD           | split_bwd          | auto (= split): row groups of the decoder backward loop |
| TSAMD_FUSED_VOCAB_TRAIN   | fused_vocab_train  | 1: training vocab head with the logits only in MFMA accumulators; 0: library GEMM + ptr_loss |
| TSAMD_FUSED_VOCAB         | fused_vocab_decode | 1: decode vocab head + top-k fused; 0: GEMM + final_topk |
| TSAMD_PROJ_ATTN           | proj_attn          | 1: training row attention streams G = enc_out . W_in[E:] (emb_dim wide) instead of enc_out; 0: enc_out |
| TSAMD_SKIP_PAD_STEPS      | skip_pad_steps     | 1: the projected-context attention kernels skip (row, step) pairs past the row's last loss-weighted decoder step; 0: compute them |
| TSAMD_DEC_ROW_ATTN        | decode_row_attn    | 1: beam-decode attention through the row kernel; 0: score + softmax kernels |
| TSAMD_COMPACT_VOCAB_GRAD  | compact_vocab_grad | 1: with skip_pad_steps, the vocab-head dlogits of the live 32-row blocks are written compacted and the two gradient GEMMs run over those rows only (bucketed block counts); 0: every row |
| TSAMD_DEFER_WGRAD         | defer_wgrad        | 1: decoder-side weight gradients beside the encoder BPTT (B >= 256); 0: inline |
| TSAMD_DETERMINISTIC       | deterministic      | 0; 1: fixed-order reductions instead of fp32 atomics (bit-reproducible steps) |
| TSAMD_KERNEL_DEBUG        | (ops loader)       | 0; 1: the bounds-checked kernel library ``_C_debug.so`` |
"""
from __future__ import annotations

import os
from dataclasses import dataclass, fields, replace
from typing import Mapping, Optional


def _flag(env: Mapping[str, str], name: str, default: bool) -> bool:
    v = env.get(name, "")
    return default if v == "" else v != "0"


def _tri(env: Mapping[str, str], name: str) -> Optional[bool]:
    v = env.get(name, "")
    return None if v == "" else v != "0"


@dataclass(frozen=True)
class EngineConfig:
    persistent_lstm: bool = True
    row_attn: Optional[bool] = None
    split: int = 0
    split_bwd: int = 0
    fused_vocab_train: bool = True
    fused_vocab_decode: bool = True
    proj_attn: bool = True
    skip_pad_steps: bool = True
    decode_row_attn: bool = True
    compact_vocab_grad: bool = True
    defer_wgrad: bool = True
    deterministic: bool = False

    @classmethod
    def from_env(cls, env: Optional[Mapping[str, str]] = None, **overrides) -> "EngineConfig":
        env = os.environ if env is None else env
        cfg = cls(
            persistent_lstm=_flag(env, "TSAMD_LSTM_PERSISTENT", True),
            row_attn=_tri(env, "TSAMD_ROW_ATTN"),
            split=int(env.get("TSAMD_SPLIT", "0") or 0),
            split_bwd=int(env.get("TSAMD_SPLIT_BWD", "0") or 0),
            fused_vocab_train=_flag(env, "TSAMD_FUSED_VOCAB_TRAIN", True),
            fused_vocab_decode=_flag(env, "TSAMD_FUSED_VOCAB", True),
            proj_attn=_flag(env, "TSAMD_PROJ_ATTN", True),
            skip_pad_steps=_flag(env, "TSAMD_SKIP_PAD_STEPS", True),
            decode_row_attn=_flag(env, "TSAMD_DEC_ROW_ATTN", True),
            compact_vocab_grad=_flag(env, "TSAMD_COMPACT_VOCAB_GRAD", True),
            defer_wgrad=_flag(env, "TSAMD_DEFER_WGRAD", True),
            deterministic=_flag(env, "TSAMD_DETERMINISTIC", False),
        )
        return replace(cfg, **overrides) if overrides else cfg

    def as_dict(self):
        return {f.name: getattr(self, f.name) for f in fields(self)}
