"""Pointer-generator parameter set, named and shaped exactly like the reference's TF1
checkpoint variables (``model.py:111-114,206-231``,
``attention_decoder.py:66-73,91-93,150,165-173,218-227``).

All trainable tensors are views into ONE contiguous fp32 buffer (``flat``), and their
gradients into one contiguous fp32 ``grad`` buffer.  That single buffer is what the
fused clip+Adagrad kernel updates, what the data-parallel all-reduce reduces (in
buckets), and what the checkpoint writer walks -- no per-tensor launches anywhere.

Initialisers follow TF: ``random_uniform(+-rand_unif_init_mag, seed=123)`` for the LSTM
kernels, ``truncated_normal(std=trunc_norm_init_std)`` for embedding / reduce-state /
output projection, TF's default Glorot-uniform for ``W_h``, ``v``, ``w_c`` and every
``linear`` Matrix, zeros for ``linear`` and LSTM biases.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch

P = "seq2seq"
DEC = f"{P}/decoder/attention_decoder"


@dataclass
class ParamSpec:
    name: str
    shape: Tuple[int, ...]
    init: str  # 'unif' | 'tnorm' | 'glorot' | 'zeros'


def enc_prefix(layer: int) -> str:
    return f"{P}/encoder" if layer == 0 else f"{P}/encoder/layer_{layer}"


def param_specs(hps, vsize: int) -> List[ParamSpec]:
    """Ordered so that backward produces gradients roughly front-to-back (output
    projection first, embedding last): contiguous all-reduce buckets fill in order."""
    E, H = hps.emb_dim, hps.hidden_dim
    A = 2 * H
    s: List[ParamSpec] = [
        ParamSpec(f"{P}/output_projection/w", (H, vsize), "tnorm"),
        ParamSpec(f"{P}/output_projection/v", (vsize,), "tnorm"),
        ParamSpec(f"{DEC}/AttnOutputProjection/Linear/Matrix", (H + A, H), "glorot"),
        ParamSpec(f"{DEC}/AttnOutputProjection/Linear/Bias", (H,), "zeros"),
    ]
    if hps.pointer_gen:
        s += [ParamSpec(f"{DEC}/calculate_pgen/Linear/Matrix", (A + 2 * H + E, 1), "glorot"),
              ParamSpec(f"{DEC}/calculate_pgen/Linear/Bias", (1,), "zeros")]
    s += [
        ParamSpec(f"{DEC}/Attention/Linear/Matrix", (2 * H, A), "glorot"),
        ParamSpec(f"{DEC}/Attention/Linear/Bias", (A,), "zeros"),
        ParamSpec(f"{DEC}/lstm_cell/kernel", (E + H, 4 * H), "unif"),
        ParamSpec(f"{DEC}/lstm_cell/bias", (4 * H,), "zeros"),
        ParamSpec(f"{DEC}/Linear/Matrix", (E + A, E), "glorot"),
        ParamSpec(f"{DEC}/Linear/Bias", (E,), "zeros"),
        ParamSpec(f"{DEC}/v", (A,), "glorot"),
    ]
    if hps.coverage:
        s.append(ParamSpec(f"{DEC}/coverage/w_c", (1, 1, 1, A), "glorot"))
    s += [
        ParamSpec(f"{DEC}/W_h", (1, 1, A, A), "glorot"),
        ParamSpec(f"{P}/reduce_final_st/w_reduce_c", (2 * H, H), "tnorm"),
        ParamSpec(f"{P}/reduce_final_st/w_reduce_h", (2 * H, H), "tnorm"),
        ParamSpec(f"{P}/reduce_final_st/bias_reduce_c", (H,), "tnorm"),
        ParamSpec(f"{P}/reduce_final_st/bias_reduce_h", (H,), "tnorm"),
    ]
    L = max(1, getattr(hps, "enc_layers", 1))
    for layer in reversed(range(L)):
        din = E if layer == 0 else 2 * H
        for d in ("fw", "bw"):
            s += [ParamSpec(f"{enc_prefix(layer)}/bidirectional_rnn/{d}/lstm_cell/kernel", (din + H, 4 * H), "unif"),
                  ParamSpec(f"{enc_prefix(layer)}/bidirectional_rnn/{d}/lstm_cell/bias", (4 * H,), "zeros")]
    s.append(ParamSpec(f"{P}/embedding/embedding", (vsize, E), "tnorm"))
    return s


def _glorot_limit(shape) -> float:
    if len(shape) == 1:
        fan_in = fan_out = shape[0]
    elif len(shape) == 2:
        fan_in, fan_out = shape
    else:
        rf = 1
        for d in shape[:-2]:
            rf *= d
        fan_in, fan_out = shape[-2] * rf, shape[-1] * rf
    return math.sqrt(6.0 / (fan_in + fan_out))


def init_tensor(spec: ParamSpec, hps, gen: torch.Generator) -> torch.Tensor:
    t = torch.empty(spec.shape, dtype=torch.float32)
    if spec.init == "zeros":
        t.zero_()
    elif spec.init == "unif":
        m = hps.rand_unif_init_mag
        t.uniform_(-m, m, generator=gen)
    elif spec.init == "tnorm":
        std = hps.trunc_norm_init_std
        t.normal_(0.0, std, generator=gen)
        # resample outside 2 std (tf.truncated_normal)
        for _ in range(8):
            bad = t.abs() > 2 * std
            if not bad.any():
                break
            t[bad] = torch.empty(int(bad.sum()), dtype=torch.float32).normal_(0.0, std, generator=gen)
        t.clamp_(-2 * std, 2 * std)
    elif spec.init == "glorot":
        lim = _glorot_limit(spec.shape)
        t.uniform_(-lim, lim, generator=gen)
    else:
        raise ValueError(spec.init)
    return t


class FlatParams:
    """Named views into one contiguous fp32 buffer (+ optional grad / Adagrad buffers)."""

    ALIGN = 64  # elements; keeps every view 256-B aligned for vector loads

    def __init__(self, specs: List[ParamSpec], device="cpu"):
        self.specs = specs
        self.offsets: Dict[str, Tuple[int, int]] = OrderedDict()
        off = 0
        for sp in specs:
            n = 1
            for d in sp.shape:
                n *= d
            self.offsets[sp.name] = (off, n)
            off += (n + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.numel_padded = off
        self.device = torch.device(device)
        self.flat = torch.zeros(off, dtype=torch.float32, device=self.device)
        self.grad = None
        self.accum = None

    @property
    def names(self) -> List[str]:
        return list(self.offsets.keys())

    def numel(self) -> int:
        return sum(n for _, n in self.offsets.values())

    def view(self, name: str, buf: torch.Tensor = None) -> torch.Tensor:
        buf = self.flat if buf is None else buf
        off, n = self.offsets[name]
        shape = next(sp.shape for sp in self.specs if sp.name == name)
        return buf[off:off + n].view(shape)

    def __getitem__(self, name):
        return self.view(name)

    def __contains__(self, name):
        return name in self.offsets

    def g(self, name: str) -> torch.Tensor:
        return self.view(name, self.grad)

    def items(self):
        for n in self.offsets:
            yield n, self.view(n)

    def init(self, hps, seed: int = 123):
        gen = torch.Generator().manual_seed(seed)
        for sp in self.specs:
            self.view(sp.name).copy_(init_tensor(sp, hps, gen))
        return self

    def enable_grad(self):
        self.grad = torch.zeros_like(self.flat)
        return self

    def enable_adagrad(self, init_acc: float):
        self.accum = torch.full_like(self.flat, init_acc)
        return self

    def to(self, device):
        device = torch.device(device)
        out = FlatParams(self.specs, device)
        out.flat.copy_(self.flat)
        if self.grad is not None:
            out.grad = self.grad.to(device)
        if self.accum is not None:
            out.accum = self.accum.to(device)
        return out

    def state_dict(self, with_adagrad=True) -> Dict[str, torch.Tensor]:
        sd = OrderedDict((n, t.detach().cpu().clone()) for n, t in self.items())
        if with_adagrad and self.accum is not None:
            for n in self.names:
                sd[n + "/Adagrad"] = self.view(n, self.accum).detach().cpu().clone()
        return sd

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True, load_adagrad=True) -> List[str]:
        missing = []
        for n in self.names:
            if n in sd:
                self.view(n).copy_(torch.as_tensor(sd[n]).reshape(self.view(n).shape))
            else:
                missing.append(n)
            if load_adagrad and self.accum is not None and (n + "/Adagrad") in sd:
                self.view(n, self.accum).copy_(torch.as_tensor(sd[n + "/Adagrad"]).reshape(self.view(n).shape))
        if strict and missing:
            raise KeyError(f"missing variables in checkpoint: {missing}")
        return missing


def build_params(hps, vsize: int, device="cpu", seed: int = 123) -> FlatParams:
    return FlatParams(param_specs(hps, vsize), device).init(hps, seed)
