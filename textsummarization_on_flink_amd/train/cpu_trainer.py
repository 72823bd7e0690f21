"""Host (CPU) training backend over the PyTorch oracle model.

The MI355X path is ``GraphTrainer`` (hipGraph-captured HIP kernels).  This backend runs the
same step -- forward, backward, all-reduce, global-norm clip, Adagrad -- on the oracle
(``models.reference``) with autograd, so that the CLI, the streaming API, DP over ``gloo``
and checkpoint/resume are exercised on machines without a GPU (the reference's own runs
pinned the model to ``/cpu:0``, ``model.py:313``).  Both trainers expose the same interface
(``step``, ``check_finite``, ``eval_step``, ``params``, ``global_step``) so every loop above
them is backend-agnostic.

Optimizer semantics follow ``model.py:288-305``: gradients of ``total_loss`` (or ``loss``
without coverage), ``tf.clip_by_global_norm(max_grad_norm)`` (scale = max / max(norm, max)),
``AdagradOptimizer(lr, initial_accumulator_value)``: acc += g^2; w -= lr g / sqrt(acc).
A non-finite global norm skips the update and raises (NaN guard, ``train.py:107-108``).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch

from ..models.params import FlatParams, build_params
from ..models.reference import ReferencePointerGenerator, batch_to_tensors
from ..parallel.dist import DistInfo, GradAllReducer, broadcast_params
from .trainer import NonFiniteLossError


class _Views:
    """name -> view of one flat leaf tensor (so autograd yields one flat gradient)."""

    def __init__(self, params: FlatParams, flat: torch.Tensor):
        self.p, self.flat = params, flat

    def __getitem__(self, name):
        return self.p.view(name, self.flat)


class CpuTrainer:
    def __init__(self, hps, vsize: int, info: Optional[DistInfo] = None, params: Optional[FlatParams] = None,
                 device="cpu", bucket_mb: float = 32.0):
        self.hps = hps
        self.info = info or DistInfo()
        self.device = torch.device(device)
        if params is None:
            params = build_params(hps, vsize, device=self.device, seed=hps.seed)
        self.params = params
        if params.grad is None:
            params.enable_grad()
        if params.accum is None:
            params.enable_adagrad(hps.adagrad_init_acc)
        broadcast_params(params.flat, self.info)
        if self.info.enabled:
            broadcast_params(params.accum, self.info)
        self.model = ReferencePointerGenerator(hps, vsize)
        self.reducer = GradAllReducer(params.grad, self.info, bucket_mb=bucket_mb)
        self.global_step = 0
        self.last_norm = 0.0
        self.skipped = False
        self.poison_next = False  # fault injection: NaN gradient on the next step

    def _forward(self, batch, need_grad: bool):
        flat = self.params.flat.detach().requires_grad_(need_grad)
        out = self.model.forward(_Views(self.params, flat), batch_to_tensors(batch, self.device))
        return flat, out

    def step(self, batch) -> Dict[str, torch.Tensor]:
        hps = self.hps
        flat, out = self._forward(batch, True)
        out["total_loss"].backward()
        g = self.params.grad
        g.copy_(flat.grad)
        if self.poison_next:
            g[0] = float("nan")
            self.poison_next = False
        self.reducer()
        norm = float(g.norm())
        self.last_norm = norm
        self.skipped = not math.isfinite(norm)
        if not self.skipped:
            g.mul_(hps.max_grad_norm / max(norm, hps.max_grad_norm))
            acc = self.params.accum
            acc.addcmul_(g, g)
            self.params.flat.addcdiv_(g, acc.sqrt(), value=-hps.lr)
        self.global_step += 1
        res = {"loss": out["loss"].detach(), "total_loss": out["total_loss"].detach()}
        if "coverage_loss" in out:
            res["coverage_loss"] = out["coverage_loss"].detach()
        return res

    def check_finite(self, out) -> Dict[str, float]:
        vals = {k: float(v) for k, v in out.items()}
        if self.skipped or not all(math.isfinite(v) for v in vals.values()):
            raise NonFiniteLossError("Loss is not finite. Stopping.")
        vals["global_norm"] = self.last_norm
        return vals

    def named_debug_tensors(self):
        """(name, tensor) of parameters and gradients (``--debug``)."""
        p = self.params
        for n in p.names:
            yield "param/" + n, p.view(n)
            yield "grad/" + n, p.view(n, p.grad)

    @torch.no_grad()
    def eval_step(self, batch) -> Dict[str, float]:
        _, out = self._forward(batch, False)
        res = {"loss": float(out["loss"]), "total_loss": float(out["total_loss"])}
        if "coverage_loss" in out:
            res["coverage_loss"] = float(out["coverage_loss"])
        return res
