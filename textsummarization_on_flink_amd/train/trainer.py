"""Training engine: hipGraph-captured train step + synchronous DP over RCCL.

Replaces ``FlinkTrainer`` / ``run_training`` (``train.py:57-125``,
``run_summarization.py:181-244``):

  * the whole forward+backward is captured ONCE into a hipGraph (``torch.cuda.graph``)
    and replayed each step: ~1600 kernel launches per step cost one host call;
  * the flat gradient is all-reduced over RCCL between the two graphs (bucketed), then
    the optimizer graph (grad average, fused clip+Adagrad, bf16 repack) replays;
  * ``nan_guard``: a non-finite gradient norm skips the update on device (flag word);
    the training loop reads the flag and the loss every ``hps.check_every`` steps
    (``check_finite``) and raises like the reference ("Loss is not finite. Stopping.",
    ``train.py:107-108``); between checks the host never waits on the GPU;
  * persistent-LSTM safety under DP: the hand-off kernels need all their workgroups
    resident.  When the launch grid leaves fewer than ``LSTM_RCCL_RESERVE_CUS`` CUs free
    and gradients are all-reduced, the encoder-backward graph is ordered behind the
    in-flight bucket all-reduces (a device-side stream wait), so no RCCL kernel shares the
    GPU with the persistent launch; a hand-off timeout anyway sets the sticky ``lstm_err``
    word, which poisons the last gradient bucket before its all-reduce (``poison_where``):
    every rank's optimizer kernel skips that update and every rank's ``check_finite`` raises
    at the same check;
  * eval mode is the same engine with forward only.
"""
from __future__ import annotations

import logging
import math
import time
import weakref
from typing import Callable, Dict, Optional

import torch

from ..models.params import FlatParams, build_params
from ..models.pointer_generator import VOCAB_DW_SIDE, HipPointerGenerator, LstmHandoffError  # noqa: F401
from ..parallel.dist import DistInfo, GradAllReducer, broadcast_params, rccl_cu_reserve
from ..utils.graphs import capture_guard

log = logging.getLogger(__name__)


class NonFiniteLossError(RuntimeError):
    pass


# CUs kept free of persistent-LSTM workgroups before RCCL kernels may overlap the launch: RCCL's
# channel cap (parallel/dist.py RCCL_MAX_CHANNELS, applied to every rank's environment)
LSTM_RCCL_RESERVE_CUS = 64


def check_lstm_err(engine) -> None:
    engine.check_lstm_err()


# phase graphs of a step: 0 forward + vocab backward, 1 decoder backward, 2 encoder backward
# (+ the joined deferred decoder weight gradients), 3 embedding gradient; gradient buckets
# (HipPointerGenerator.phase_bounds): 0 output projection, 1 decoder + attention, 2 reduce_states
# + encoder, 3 embedding
BPTT_PHASE = 2


def issue_plan(defer_wgrad: bool, dw_side: bool = False):
    """Buckets whose all-reduce is issued after each phase graph (the last bucket, the embedding,
    is issued by the reducer call after the last graph).  With the decoder weight gradients
    deferred beside the encoder BPTT, bucket 1 completes with phase 2.  With the vocab dW beside
    the decoder backward loop (dw_side), phase 1 issues bucket 0 itself, from the side stream
    (GraphTrainer._Phase1)."""
    return [[] if dw_side else [0], [] if defer_wgrad else [1], [1, 2] if defer_wgrad else [2], []]


def replay_phases(graphs, reducer, plan, bptt_phase: int, lstm_exclusive: bool, ev=None):
    """Replay the phase graphs, issuing each bucket's all-reduce as soon as its phase has been
    queued (RCCL runs it on its own stream behind that work) -- overlapped with the later phases.
    ``lstm_exclusive``: the persistent BPTT fills the chip, so the device waits for the issued
    all-reduces before that phase (no RCCL kernel shares the GPU with it)."""
    for i, g in enumerate(graphs):
        if i == bptt_phase and lstm_exclusive:
            reducer.wait_issued()
        g.replay()
        if ev:
            ev[i + 1].record()
        for b in plan[i]:
            reducer.bucket_ready(b)


class GraphTrainer:
    def __init__(self, hps, vsize: int, B: int, T: int, device="cuda", info: Optional[DistInfo] = None,
                 params: Optional[FlatParams] = None, use_graph: bool = True, bucket_mb: float = 32.0):
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
        self.engine = HipPointerGenerator(hps, vsize, params, B=B, T=T)
        # buckets = backward phases: output_projection | decoder+attention | encoder | embedding;
        # each is all-reduced while the following phase computes (RCCL over xGMI); the
        # 1/world average happens inside the optimizer kernel
        self.reducer = GradAllReducer(params.grad, self.info, bucket_mb=bucket_mb,
                                      bounds=self.engine.phase_bounds(), average=False,
                                      compress=getattr(hps, "grad_compress", "none"))
        self.engine.grad_scale = 1.0 / self.info.world
        self.engine.poison_on_lstm_err = self.info.enabled  # a hand-off timeout skips the step on every rank
        eng = self.engine
        self.lstm_exclusive = False
        if self.info.enabled and eng.persistent_lstm:
            grid = int(eng.k.lstm_persistent_grid(eng.H, eng.B))
            cap = int(eng.k.lstm_persistent_capacity(eng.H))
            self.lstm_exclusive = grid > cap - max(LSTM_RCCL_RESERVE_CUS, rccl_cu_reserve())
        self.use_graph = use_graph
        self.g_fb = None
        self.g_opt = None
        self.out = None
        self.global_step = 0
        self.host_sync_free = True  # step() never waits on the GPU; loops check every hps.check_every steps
        self.poison_next = False  # fault injection: NaN gradient on the next step (exercises the NaN guard)
        self.timing = False       # per-phase HIP-event timing (phase_ms)
        self._ev = None
        # the vocab dW on a side stream beside the decoder backward loop (VOCAB_DW_SIDE): graph mode,
        # padded fused vocab head only (the other heads compute dW and dX in one call)
        self.dw_side = bool(use_graph and VOCAB_DW_SIDE and eng.fused_vocab and eng.Vp != eng.V)
        eng.split_vocab_dw = self.dw_side
        self.g_dw = {}

    # ------------------------------------------------------------------ capture
    def _fb(self):
        out = self._fwd_head()
        self.engine.backward_mid()
        self.engine.backward_tail()
        return out

    def _fwd_head(self):
        out = self.engine.forward(need_grad=True)
        self.engine.backward_head()
        self.engine.backward_head_dw()
        return out

    class _Phase0:
        """Phase graph 0 = the forward graph + the vocab-gradient graph of the batch's live-block
        bucket (HipPointerGenerator.compact_vocab: one head graph per block count)."""

        def __init__(self, trainer):
            self.t = weakref.proxy(trainer)  # no trainer <-> phase cycle: trainers free by refcount

        def replay(self):
            self.t.g_fwd.replay()
            self.t.g_head[self.t.engine.nbk].replay()

    class _Phase1:
        """Phase graph 1 = the decoder backward graph; with dw_side, the batch bucket's vocab-dW graph
        replayed on a side stream beside it (forked after phase 0, joined at the end), and bucket 0's
        all-reduce issued from that stream as soon as the dW is queued (it overlaps the decoder loop
        as before)."""

        def __init__(self, trainer):
            self.t = weakref.proxy(trainer)

        def replay(self):
            t = self.t
            if not t.g_dw:
                t.g_mid.replay()
                return
            cur = torch.cuda.current_stream()
            side = t._dw_stream
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                t.g_dw[t.engine.nbk].replay()
                t.reducer.bucket_ready(0)
            t.g_mid.replay()
            cur.wait_stream(side)

    def _opt(self):
        self.engine.optimizer_step()

    def capture(self):
        """Warm up on a side stream, then capture forward+backward and the optimizer."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        snap = (self.params.flat.clone(), self.params.accum.clone())
        eng = self.engine
        buckets = eng.vocab_buckets if eng.compact_vocab else [eng.nbk]
        with torch.cuda.stream(s):
            for _ in range(2):
                self._fb()
                self._opt()
            nbk = eng.nbk
            for b in buckets:  # every head variant once before its capture
                eng.nbk = b
                eng.backward_head()
                eng.backward_head_dw()
            eng.nbk = nbk
        torch.cuda.current_stream().wait_stream(s)
        # undo the warm-up updates so capture does not change the model
        self.params.flat.copy_(snap[0])
        self.params.accum.copy_(snap[1])
        self.engine.pack()
        torch.cuda.synchronize()
        with capture_guard():  # no cyclic GC (and its HIP-calling destructors) inside the captures
            pool = torch.cuda.graph_pool_handle()
            # four graphs (forward + vocab backward | decoder backward | encoder backward |
            # embedding gradient) so each gradient bucket's all-reduce overlaps the next phase
            self.g_fb = [self._Phase0(self), self._Phase1(self)] + [torch.cuda.CUDAGraph() for _ in range(2)]
            self.g_fwd = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_fwd, pool=pool):
                self.out = self.engine.forward(need_grad=True)
            nbk = eng.nbk
            self.g_head = {}
            self.g_dw = {}
            # the dW graphs replay beside g_mid: a pool of their own, so none of their private
            # allocations can alias one of g_mid's
            dw_pool = torch.cuda.graph_pool_handle() if self.dw_side else None
            for b in buckets:
                eng.nbk = b
                self.g_head[b] = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.g_head[b], pool=pool):
                    eng.backward_head()
                if self.dw_side:
                    self.g_dw[b] = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(self.g_dw[b], pool=dw_pool):
                        eng.backward_head_dw()
            eng.nbk = nbk
            if self.dw_side:
                self._dw_stream = torch.cuda.Stream(self.device)
            self.g_mid = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_mid, pool=pool):
                self.engine.backward_mid()
            with torch.cuda.graph(self.g_fb[2], pool=pool):
                eng.backward_tail_enc()
            with torch.cuda.graph(self.g_fb[3], pool=pool):
                eng.backward_tail_emb()
            self.g_opt = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_opt, pool=pool):
                self._opt()
        torch.cuda.synchronize()

    # ------------------------------------------------------------------ step
    def step(self, batch) -> Dict[str, torch.Tensor]:
        self.engine.set_batch(batch)
        if self.use_graph:
            if self.g_fb is None:
                self.capture()
            ev = self._events() if self.timing else None
            if ev:
                ev[0].record()
            ng = len(self.g_fb)
            replay_phases(self.g_fb, self.reducer, issue_plan(self.engine.defer_wgrad, bool(self.g_dw)), BPTT_PHASE,
                          self.lstm_exclusive, ev)
            self._maybe_poison()
            self.reducer()
            if ev:
                ev[ng + 1].record()
            self.g_opt.replay()
            if ev:
                ev[ng + 2].record()
            out = self.out
        else:
            out = self._fb()
            self._maybe_poison()
            self.reducer()
            self._opt()
        self.global_step += 1
        return out

    def _events(self):
        if self._ev is None:
            self._ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(self.g_fb) + 3)]
        return self._ev

    def phase_ms(self) -> Dict[str, float]:
        """Time of each phase of the last step (host-synchronising): forward + vocab backward,
        decoder backward, encoder backward, embedding gradient, exposed all-reduce wait, optimizer."""
        if not self._ev:
            return {}
        self._ev[-1].synchronize()
        names = ("ms_fwd_head", "ms_bwd_dec", "ms_bwd_enc", "ms_bwd_emb", "ms_allreduce", "ms_optimizer")
        return {n: self._ev[i].elapsed_time(self._ev[i + 1]) for i, n in enumerate(names)}

    def _maybe_poison(self):
        if self.poison_next:  # last element: its bucket's all-reduce has not been issued yet
            self.params.grad[-1] = float("nan")
            self.poison_next = False

    def check_finite(self, out) -> Dict[str, float]:
        """Host sync: raise on a persistent-LSTM hand-off error, a non-finite loss or an
        update skipped by the NaN guard (the flags are sticky, so a check every
        ``check_every`` steps sees every earlier step)."""
        vals = {k: float(v) for k, v in out.items()}
        check_lstm_err(self.engine)
        if not all(math.isfinite(v) for v in vals.values()) or (int(self.engine.w["nan_flag"].item()) & 1):
            raise NonFiniteLossError("Loss is not finite. Stopping.")
        vals["global_norm"] = float(self.engine.w["gnorm"].item())
        return vals

    def named_debug_tensors(self):
        """(name, tensor) of parameters, gradients and every activation buffer (``--debug``)."""
        p = self.params
        for n in p.names:
            yield "param/" + n, p.view(n)
            if p.grad is not None:
                yield "grad/" + n, p.view(n, p.grad)
        for n, t in self.engine.w.items():
            if isinstance(t, torch.Tensor):
                yield "act/" + n, t

    def eval_step(self, batch) -> Dict[str, float]:
        self.engine.set_batch(batch)
        out = self.engine.forward(need_grad=False)
        vals = {k: float(v) for k, v in out.items()}
        check_lstm_err(self.engine)  # never report (or save as bestmodel) a loss from a failed launch
        return vals
