"""``--debug``: find the tensors that hold NaN / Inf after a step.

The reference wraps the session in tfdbg's ``LocalCLIDebugWrapperSession`` with the
``has_inf_or_nan`` filter (``run_summarization.py:216-218``), which stops at the first step
whose tensors contain a non-finite value.  Here the trainers expose their named device
buffers (``named_debug_tensors``: parameters, gradients and -- on the GPU engine -- every
activation buffer of the step), and ``NonFiniteWatch`` checks them all after each step
with one device reduction per tensor and a single host sync, then raises with a report
naming every offending tensor (element counts of NaN and Inf).
"""
from __future__ import annotations

import logging
from typing import Iterable, List, Tuple

import torch

log = logging.getLogger(__name__)


def nonfinite_report(named: Iterable[Tuple[str, torch.Tensor]]) -> List[Tuple[str, int, int]]:
    """[(name, n_nan, n_inf)] for every floating tensor that is not all finite."""
    names, counts = [], []
    for name, t in named:
        if t is None or not torch.is_floating_point(t) or t.numel() == 0:
            continue
        names.append(name)
        counts.append(torch.stack([torch.isnan(t).sum(), torch.isinf(t).sum()]))
    if not counts:
        return []
    c = torch.stack(counts).cpu().tolist()  # one sync for all tensors
    return [(n, int(a), int(b)) for n, (a, b) in zip(names, c) if a or b]


class NonFiniteWatch:
    """Checks ``trainer.named_debug_tensors()`` after every step (``hps.debug``)."""

    def __init__(self, trainer):
        self.trainer = trainer

    def check(self, step: int) -> List[Tuple[str, int, int]]:
        rep = nonfinite_report(self.trainer.named_debug_tensors())
        if rep:
            lines = ", ".join(f"{n} (nan={a}, inf={b})" for n, a, b in rep[:32])
            log.error("has_inf_or_nan at step %d: %d tensor(s): %s%s", step, len(rep), lines,
                      " ..." if len(rep) > 32 else "")
        return rep
