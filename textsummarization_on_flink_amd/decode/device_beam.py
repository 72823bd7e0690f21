"""Batched, device-resident beam search on MI355X (SURVEY PAR3, K17/K20/K25/K26, 7.5-3).

The reference decodes ONE article at a time with beam_size rows and a host round trip per
step (``beam_search.py:82-168``, one ``sess.run`` + numpy state packing per step).  Here
``n_articles x beam`` rows decode together and the whole step stays on the GPU:

  gather-by-parent (c, h, ctx*, a*, cov)  ->  cov' = cov + a*  ->  XG / x from per-token
  tables  ->  dec_cell_fwd  ->  dec_sproj  ->  attn_score / attn_softmax_ctx  ->  p_gen,
  output projection, vocab GEMM  ->  final_topk (pointer mixture + top-2k)  ->  beam_step

The step reads its index t from a device counter and the decoder state ping-pongs between
two buffer sets, so ONE captured hipGraph of two steps
is replayed up to max_dec_steps times (host checks the all-done flag every ``chunk``
replays, the only host sync).

The reference's decode-mode attention runs twice per step (initial_state_attention):
the first attention of step t recomputes attention(state_{t-1}, cov'_{t-1}), which is
exactly the parent's post-cell attention of step t-1 -- same inputs -- so it is gathered
instead of recomputed (only step 0 runs it, in the prologue).  Coverage semantics are
unchanged: cov'_t = cov'_{t-1}[parent] + a_{t-1}[parent].
"""
from __future__ import annotations


import os
from typing import List
from dataclasses import replace

import numpy as np
import torch

from ..data.vocab import START_DECODING, STOP_DECODING, UNKNOWN_TOKEN
from ..models.pointer_generator import (ATT_B, CELL_B, CELL_K, EMB, LIN_B, LIN_M, OUT_B, OV, PG_B, PG_M,
                                        HipPointerGenerator, mmf)
from ..models.engine_config import EngineConfig
from ..utils.graphs import capture_guard
from .beam_search import Hypothesis

BF = torch.bfloat16
F32 = torch.float32


class DeviceBeamDecoder:
    def __init__(self, hps, vocab, params, n_articles: int, T: int, use_graph: bool = True, chunk: int = 10,
                 keep_attn: bool = True):
        self.hps, self.vocab, self.p = hps, vocab, params
        self.Na, self.beam = n_articles, hps.beam_size
        self.R = self.Na * self.beam
        # rows per encoder-feature row in the attention kernels (1, 2 or 4); other beam
        # sizes fall back to replicating E/F per hypothesis
        self.rep = self.beam if self.beam in (1, 2, 4) else 1
        self.K = 2 * self.beam
        self.T = T
        self.V = vocab.size()
        self.maxD = hps.max_dec_steps
        self.use_graph, self.chunk, self.keep_attn = use_graph, chunk, keep_attn
        # decode steps per captured graph: a whole early-exit chunk when it is even (one graph
        # launch per chunk instead of one per step pair), else 2
        self.gsteps = chunk if chunk % 2 == 0 else 2
        # the encoder side of the engine only (the projected-context G of the training loop is not used)
        self.eng = HipPointerGenerator(hps, self.V, params, B=self.Na, T=T, D=1,
                                       cfg=replace(EngineConfig.from_env(), proj_attn=False))
        # attention per step: the row-resident kernel (score + softmax + context in one launch,
        # one workgroup per hypothesis reading its article's F/E rows) when the shape allows
        # it, else the multi-block kernels over the transposed features (EngineConfig.decode_row_attn)
        self.k = self.eng.k
        self.row_attn = self.eng.cfg.decode_row_attn and bool(self.k.attn_row_ok(self.eng.A, T))
        self.eng.keep_ft = not self.row_attn  # the multi-block score kernel reads transposed features
        self.dev = self.eng.dev
        # decode_batches: up to ``group_enc`` queued plain batches are encoded as ONE
        # group_enc * n_articles-row encoder pass (the persistent LSTM's step time does not grow
        # with the rows, so the group costs about one batch's encoder); the later batches' outputs
        # wait in that engine's buffers for their turn (TSAMD_DEC_GROUP_ENC, 1 = off): headline
        # decode 6273 -> 6792-6877, config #5 decode 2838-2855 (the side-stream overlap below)
        # -> 3154-3167 summaries/s (profiles/r6/decode_pair_encoder.md)
        g = int(os.environ.get("TSAMD_DEC_GROUP_ENC", "8"))
        self.group_enc = g if (g > 1 and self.dev.type == "cuda") else 1
        # without grouping: run batch n + 1's encoder on a side stream beside batch n's decode
        # steps when the encoder is long enough to pay for the CUs its persistent LSTM holds
        # (bench, 64 articles: hidden 512 / 2 layers / T = 800 2263 -> 2550 summaries/s; hidden
        # 256 / 1 layer / T = 400, a 1.1 ms encoder: 6016 -> 5817, so off); TSAMD_DEC_OVERLAP_ENC
        # 0 / 1 forces it
        ov = os.environ.get("TSAMD_DEC_OVERLAP_ENC", "auto")
        self.overlap_encoder = ((self.eng.L > 1 or self.eng.H >= 512) and self.group_enc == 1) if ov == "auto" \
            else ov != "0"
        self.eng2 = None
        if self.group_enc > 1 and not self.overlap_encoder:
            self._group_engine()  # built up front: its construction must not land in a decode
        self._alloc()
        self.refresh_weights()
        self.graph = None
        self._captured_now = False

    # ------------------------------------------------------------------ setup
    def _alloc(self):
        R, T, H, A, E, V, K, Na, D = self.R, self.T, self.eng.H, self.eng.A, self.eng.E, self.V, self.K, self.Na, \
            self.maxD
        z = lambda *s, dt=F32: torch.zeros(*s, dtype=dt, device=self.dev)
        self._done_dev = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self._done_flags = [torch.zeros(1, dtype=torch.int32, pin_memory=True) for _ in range(2)]
        b = {}
        for name, shape, dt in [
            ("Ft" if not self.row_attn else "F", (R // self.rep, A, T) if not self.row_attn else (R // self.rep, T, A),
             BF), ("E", (R // self.rep, T, A), BF),
            ("lens_att", (R // self.rep,), torch.int32),
            ("c", (R, H), F32), ("h", (R, H), BF), ("ctxs", (R, A), F32), ("ctxs_bf", (R, A), BF),
            ("x", (R, E), F32), ("Cb2", (R, H), BF), ("XG", (R, 4 * H), F32), ("act", (R, 4 * H), F32),
            ("s", (R, A), F32), ("e", (R, T), F32),
            ("ctx_bf", (R, A), BF), ("PG", (R,), F32), ("outb", (R, H), BF), ("logits", (R, V), F32),
            ("top_ids", (R, K), torch.int32), ("top_lp", (R, K), F32), ("lp_sum", (R,), F32),
            ("latest", (R,), torch.int32), ("gidx", (R,), torch.int32), ("tok_hist", (D, R), torch.int32),
            ("par_hist", (D, R), torch.int32), ("done", (Na,), torch.int32), ("res_count", (Na,), torch.int32),
            ("res_score", (R,), F32), ("res_len", (R,), torch.int32), ("res_step", (R,), torch.int32),
            ("res_par", (R,), torch.int32), ("step", (1,), torch.int32), ("step_ctr", (1,), torch.int32),
            ("ext", (Na, T), torch.int32),
            ("lens", (Na,), torch.int32),
            ("part_ms", (R, int(self.k.topk_parts(V)), 2), F32), ("part_v", (R, int(self.k.topk_parts(V)), K), F32),
            ("part_i", (R, int(self.k.topk_parts(V)), K), torch.int32),
        ]:
            b[name] = z(*shape, dt=dt)
        # fused vocab head (vocab_topk.hip) partials; EngineConfig.fused_vocab_decode = False
        # selects the materialised-logits path (GEMM + final_topk) instead
        self.fused_vocab = self.eng.cfg.fused_vocab_decode and self.K <= 8 and (self.eng.H <= 256 or self.eng.H == 512)
        if self.fused_vocab:
            b["vpart_ms"] = z(R, int(self.k.vocab_topk_parts(V, H)), 2)
        # fused step (5 + 1 launches): the parent / token gathers inside the cell, x-merge and
        # attention kernels, the beam bookkeeping in the vocab select kernel's tail
        self.fused_step = self.fused_vocab and self.row_attn and self.beam * self.K <= 64
        b["art_ctr"] = z(Na, dt=torch.int32)
        b["gran"] = z(R, K, dt=torch.long)  # tagged candidate granules of the fused beam tail
        b["tail_err"] = z(1, dt=torch.int32)
        # ping-pong decoder state: step t reads set t%2 and writes set (t+1)%2, so a
        # captured 2-step graph needs no copies between steps
        self.st = [{"C": z(R, H), "H": z(R, H, dt=BF), "CTX": z(R, A), "CTXb": z(R, A, dt=BF), "ATT": z(R, T),
                    "COV": z(R, T)} for _ in range(2)]
        if self.keep_attn:
            b["ATT_hist"] = z(D, R, T)
            b["PG_hist"] = z(D, R)
        self.b = b

    def refresh_weights(self):
        """Per-token tables for the current weights (call after loading a checkpoint):
        Xtab = emb . W_in[:E] + b_in  and  XGtab = Xtab . W_cell[:E] + b_cell."""
        self.eng.pack()
        if getattr(self, "eng2", None) is not None:
            self.eng2.pack()
        p, E = self.p, self.eng.E
        emb = p[EMB]
        self.Xtab = (emb @ p[LIN_M][:E] + p[LIN_B]).contiguous()
        self.XGtab = (self.Xtab @ p[CELL_K][:E] + p[CELL_B]).contiguous()
        self.pg_w = p[PG_M][:, 0].contiguous() if self.hps.pointer_gen else None
        self.owT = self.eng.pk["ow"].t().contiguous() if self.fused_vocab else None  # [V][H] for the fused head
        self.graph = None

    # ------------------------------------------------------------------ per-chunk phases
    def _encode(self, batch):
        self.eng.set_batch(batch)
        self.eng._encoder_forward(need_grad=False)
        self._encode_copy()

    def _encode_launch(self, batch):
        """The encoder forward of ``batch`` into the engine's own buffers, queued on a side
        stream behind everything the current stream has queued so far (in particular the
        previous batch's ``_encode_copy`` out of those buffers).  The decode steps touch none
        of them, so the next batch's encoder runs beside the current batch's decode steps
        (``decode_batches``); ``_encode_copy`` after waiting on ``self._enc_ev`` picks it up."""
        if not hasattr(self, "_enc_stream"):
            self._enc_stream = torch.cuda.Stream(self.dev)
        s = self._enc_stream
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self.eng.set_batch(batch)
            self.eng._encoder_forward(need_grad=False)
        self._enc_ev = torch.cuda.Event()
        self._enc_ev.record(s)

    def _encode_copy(self, src=None):
        """Encoder outputs (engine buffers) -> the decoder's feature and initial-state buffers.
        ``src`` = (engine, first row): rows first .. first + n_articles of another engine's
        encoder outputs (the paired encoder), else this decoder's own engine."""
        eng, lo = src if src is not None else (self.eng, 0)
        hi = lo + self.Na
        b, beam = self.b, self.beam
        w = eng.w
        # encoder features stay one row per article: the attention kernels read them once for
        # all ``beam`` hypotheses of the article (rep = beam)
        r = beam // self.rep
        rep = (lambda x: x.repeat_interleave(r, 0)) if r > 1 else (lambda x: x)
        b["E"].copy_(rep(eng.enc[-1]["out"][lo:hi]))
        fk = "F" if self.row_attn else "Ft"
        b[fk].copy_(rep(w[fk][lo:hi]))
        b["lens_att"].copy_(rep(w["enc_lens"][lo:hi]))
        b["lens"].copy_(w["enc_lens"][lo:hi])
        b["ext"].copy_(w["ext"][lo:hi])
        X = self.st[0]
        X["C"].copy_(w["Cst"][0][lo:hi].repeat_interleave(beam, 0))
        X["H"].copy_(w["Hb"][0][lo:hi].repeat_interleave(beam, 0))

    def _group_engine(self):
        if self.eng2 is None:
            n = self.group_enc * self.Na
            self.eng2 = HipPointerGenerator(self.hps.replace(batch_size=n), self.V, self.p, B=n, T=self.T, D=1,
                                            cfg=replace(EngineConfig.from_env(), proj_attn=False))
            self.eng2.keep_ft = self.eng.keep_ft
        return self.eng2

    @staticmethod
    def _groupable(a, b) -> bool:
        return (b is not None and b is not DeviceBeamDecoder.FLUSH and getattr(a, "host_pack", None) is None
                and getattr(b, "host_pack", None) is None and a.enc_batch.shape == b.enc_batch.shape)

    def _encode_group(self, grp):
        """One encoder pass over the batches of ``grp`` (at most the engine's rows / n_articles; the
        rest of its rows repeat the last batch): batch j's outputs are rows j n_articles .. of the
        group engine's buffers."""
        from types import SimpleNamespace
        e2 = self._group_engine()
        full = list(grp) + [grp[-1]] * (e2.B // self.Na - len(grp))
        cat = lambda n: np.concatenate([getattr(b, n) for b in full], 0)  # noqa: E731
        merged = SimpleNamespace(**{n: cat(n) for n in ("enc_batch", "enc_lens", "enc_batch_extend_vocab", "dec_batch",
                                                         "dec_padding_mask", "target_batch", "valid")})
        e2.set_batch(merged)
        e2._encoder_forward(need_grad=False)

    def _prologue(self):
        """Step-0 initial-state attention into state set 0, beam state reset."""
        k, b, hps, eng = self.k, self.b, self.hps, self.eng
        R, T, H, A = self.R, self.T, eng.H, eng.A
        X = self.st[0]
        b["Cb2"].copy_(X["C"])
        k.dec_sproj(b["Cb2"], X["H"], eng.pk["WsT"], self.p[ATT_B], b["s"], R, H, A, None, 0)
        self._attention(None, X["ATT"], X["CTX"], X["CTXb"])
        X["COV"].zero_()
        b["gidx"].copy_(torch.arange(R, dtype=torch.int32, device=self.dev))
        b["latest"].fill_(self.vocab.word2id(START_DECODING))
        b["lp_sum"].zero_()
        for n in ("done", "res_count", "step", "step_ctr", "tok_hist", "par_hist", "res_len", "res_step", "res_par",
                  "art_ctr", "gran"):
            b[n].zero_()
        b["res_score"].fill_(-float("inf"))

    def _attention(self, cov, att_out, ctx_out, ctx_bf):
        """a_t = softmax(e_t), ctx_t = sum_i a_ti E_i for all R hypotheses (coverage, if any,
        was already accumulated into ``cov`` by beam_gather)."""
        k, b, eng = self.k, self.b, self.eng
        R, T, A = self.R, self.T, eng.A
        if self.row_attn:
            k.attn_fwd_row(b["F"], b["E"], b["s"], eng.f32["v"], eng.f32["wc"], cov, b["lens_att"], att_out, None,
                           None, ctx_out, ctx_bf, R, T, A, self.rep)
            return
        k.attn_score(b["Ft"], b["s"], eng.f32["v"], eng.f32["wc"], cov, b["lens_att"], b["e"], R, T, A, self.rep)
        k.attn_softmax_ctx(b["e"], b["E"], b["lens_att"], None, att_out, None, None, ctx_out, ctx_bf, R, T, A,
                           self.rep)

    def _step(self, parity: int):
        if self.fused_step:
            return self._step_fused(parity)
        k, b, hps, eng, p = self.k, self.b, self.hps, self.eng, self.p
        R, T, H, A, E, V, K = self.R, self.T, eng.H, eng.A, eng.E, self.V, self.K
        X, Y = self.st[parity], self.st[1 - parity]
        cov = hps.coverage
        k.beam_gather(b["gidx"], b["latest"], X["C"], X["H"], X["CTX"], X["ATT"], X["COV"] if cov else None,
                      self.XGtab, self.Xtab, b["c"], b["h"], b["ctxs"], b["ctxs_bf"], Y["COV"] if cov else None,
                      b["XG"], b["x"], R, H, A, T, E, V, self.vocab.word2id(UNKNOWN_TOKEN), b["step"])
        k.dec_cell_fwd(b["XG"], b["ctxs_bf"], b["h"], b["c"], eng.pk["WcT2"], Y["C"], b["Cb2"], Y["H"], b["act"],
                       R, H, A, None, 0)
        if hps.pointer_gen:
            # one launch: attention query s = [c, h] . W_s + b, and the x-merge for p_gen,
            # x = x0 + ctx*_{t-1} . W_in[E:] (x0 = emb . W_in[:E] + b_in gathered per token)
            k.linear2_pair(b["Cb2"], H, Y["H"], H, eng.pk["WsT"], p[ATT_B], None, b["s"], None, A,
                           b["ctxs_bf"], A, None, 0, eng.pk["WicT"], None, b["x"], b["x"], None, E, R)
        else:
            k.dec_sproj(b["Cb2"], Y["H"], eng.pk["WsT"], p[ATT_B], b["s"], R, H, A, None, 0)
        self._attention(Y["COV"] if cov else None, Y["ATT"], Y["CTX"], b["ctx_bf"])
        pg = b["PG"] if hps.pointer_gen else None
        if hps.pointer_gen and not self.fused_vocab:
            k.pgen(Y["CTX"], Y["C"], Y["H"], b["x"], self.pg_w, p[PG_B], b["PG"], R, A, H, E)
        k.linear2(Y["H"], H, b["ctx_bf"], A, eng.pk["OUTmT"], p[OUT_B], None, None, b["outb"], R, H)
        if self.fused_vocab and hps.pointer_gen:
            # p_gen is computed inside the select kernel (into b["PG"] for the histories)
            k.vocab_topk_pg(b["outb"], self.owT, p[OV], Y["CTX"], Y["C"], Y["H"], b["x"], self.pg_w, p[PG_B], b["PG"],
                            Y["ATT"], b["ext"], b["lens"], b["top_ids"], b["top_lp"], b["logits"], b["vpart_ms"], R,
                            V, H, T, K, self.beam, A, E)
        elif self.fused_vocab:
            k.vocab_topk(b["outb"], self.owT, p[OV], None, None, b["ext"], b["lens"], b["top_ids"], b["top_lp"],
                         b["logits"], b["vpart_ms"], R, V, H, T, K, self.beam)
        else:
            torch.mm(b["outb"], eng.pk["ow"], out_dtype=F32, out=b["logits"])
            k.final_topk(b["logits"], p[OV], pg, Y["ATT"] if hps.pointer_gen else None, b["ext"], b["lens"],
                         b["top_ids"], b["top_lp"], b["part_ms"], b["part_v"], b["part_i"], R, V, T, K, self.beam)
        # beam bookkeeping; also appends a_t / p_gen to the histories (b["step"] was advanced by
        # this step's beam_gather: no grid-wide counter here)
        hist = self.keep_attn
        k.beam_step(b["top_ids"], b["top_lp"], b["lp_sum"], b["latest"], b["gidx"], b["tok_hist"], b["par_hist"],
                    b["done"], b["res_count"], b["res_score"], b["res_len"], b["res_step"], b["res_par"], b["step"],
                    None, Y["ATT"] if hist else None, b["ATT_hist"] if hist else None,
                    pg if (hist and pg is not None) else None, b["PG_hist"] if (hist and pg is not None) else None,
                    T, self.Na, self.beam, K, self.vocab.word2id(STOP_DECODING), hps.min_dec_steps, self.maxD)

    def _step_fused(self, parity: int):
        """One decode step in 6 launches (reference model.py:367-443 decode_onestep + the beam
        update of beam_search.py:110-156): cell with the parent / token gathers (and the step
        counter), attention query + x-merge, row attention with the coverage gather, output
        projection, vocab logits, vocab select + p_gen + per-article beam bookkeeping."""
        k, b, hps, eng, p = self.k, self.b, self.hps, self.eng, self.p
        R, T, H, A, E, V, K = self.R, self.T, eng.H, eng.A, eng.E, self.V, self.K
        X, Y = self.st[parity], self.st[1 - parity]
        cov = hps.coverage
        unk = self.vocab.word2id(UNKNOWN_TOKEN)
        k.dec_cell_fwd_beam(b["gidx"], b["latest"], self.XGtab, X["CTXb"], X["H"], X["C"], eng.pk["WcT2"], Y["C"],
                            b["Cb2"], Y["H"], b["step"], R, H, A, V, unk)
        if hps.pointer_gen:
            k.beam_sproj_xmerge(b["Cb2"], Y["H"], eng.pk["WsT"], p[ATT_B], b["s"], X["CTXb"], eng.pk["WicT"],
                                self.Xtab, b["gidx"], b["latest"], b["x"], R, H, A, E, V, unk)
        else:
            k.dec_sproj(b["Cb2"], Y["H"], eng.pk["WsT"], p[ATT_B], b["s"], R, H, A, None, 0)
        k.attn_fwd_row_beam(b["F"], b["E"], b["s"], eng.f32["v"], eng.f32["wc"], X["COV"] if cov else None,
                            X["ATT"] if cov else None, Y["COV"] if cov else None, b["gidx"], b["lens_att"],
                            Y["ATT"], Y["CTX"], Y["CTXb"], R, T, A, self.rep)
        k.linear2(Y["H"], H, Y["CTXb"], A, eng.pk["OUTmT"], p[OUT_B], None, None, b["outb"], R, H)
        ptr, hist = hps.pointer_gen, self.keep_attn
        k.vocab_topk_beam(b["outb"], self.owT, p[OV], Y["CTX"] if ptr else None, Y["C"] if ptr else None,
                          Y["H"] if ptr else None, b["x"] if ptr else None, self.pg_w if ptr else None,
                          p[PG_B] if ptr else None, b["PG"] if ptr else None, Y["ATT"] if (ptr or hist) else None,
                          b["ext"], b["lens"], b["top_ids"], b["top_lp"], b["logits"], b["vpart_ms"], b["lp_sum"],
                          b["latest"], b["gidx"], b["tok_hist"], b["par_hist"], b["done"], b["res_count"],
                          b["res_score"], b["res_len"], b["res_step"], b["res_par"], b["step"], b["art_ctr"],
                          b["gran"], b["tail_err"],
                          b["ATT_hist"] if hist else None, b["PG_hist"] if (hist and ptr) else None, R, V, H, T, K,
                          self.beam, A, E, self.vocab.word2id(STOP_DECODING), hps.min_dec_steps, self.maxD)

    @staticmethod
    def _check_tail(err: int) -> None:
        if err:
            raise RuntimeError("beam decode: a fused beam-tail poll timed out (candidates of an article never "
                               "arrived); results discarded -- set TSAMD_DEC_ROW_ATTN=0 for the unfused step")

    def _graph_steps(self):
        for i in range(self.gsteps):  # parity alternates: gsteps is even
            self._step(i % 2)

    def _capture(self):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._graph_steps()  # warm-up (state discarded: the prologue re-runs before decoding)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with capture_guard(), torch.cuda.graph(self.graph):
            self._graph_steps()
        torch.cuda.synchronize()
        self._captured_now = True  # the warm-up consumed the encoded state: re-encode once

    # ------------------------------------------------------------------ driver
    def run(self, batch) -> None:
        """Decode one engine batch (n_articles rows) fully on the device."""
        for _ in self.run_chunks(batch):
            pass

    def run_chunks(self, batch, pre_encoded: bool = False, next_batch=None, enc_src=None):
        """Generator form of ``run``: each iteration queues one early-exit chunk of decode steps
        on the current stream and yields (``decode_batches`` does host work in between).
        ``pre_encoded``: ``batch``'s encoder was queued by ``_encode_launch``; ``next_batch``:
        queue its encoder (side stream) once this batch's encoder outputs are copied out;
        ``enc_src``: (engine, first row) holding ``batch``'s encoder outputs (the paired encoder)."""
        if pre_encoded:
            torch.cuda.current_stream().wait_event(self._enc_ev)
        if self.use_graph and self.graph is None:
            if enc_src is not None:
                self._encode_copy(enc_src)
            else:
                self._encode(batch)
            self._prologue()
            self._capture()
        if enc_src is not None:
            self._encode_copy(enc_src)  # (the source engine's buffers are intact after a capture too)
        elif pre_encoded and not self._captured_now:
            self._encode_copy()
        else:
            self._encode(batch)
        self._captured_now = False
        if next_batch is not None:
            self._encode_launch(next_batch)
        self._prologue()
        # early exit when every article is done, checked one chunk late: the all-done flag of
        # chunk c is copied to pinned memory behind an event and read once chunk c+1 is queued,
        # so the GPU never idles on the host round trip (steps after done are no-ops per article)
        t = 0
        pend = []
        chunk = 0
        while t < self.maxD:
            n = min(self.chunk, self.maxD - t)
            i = 0
            while i < n:
                if self.use_graph and n - i >= self.gsteps and (t + i) % 2 == 0:
                    self.graph.replay()  # steps t+i .. t+i+gsteps-1 (parity 0, 1, 0, ...)
                    i += self.gsteps
                else:
                    self._step((t + i) % 2)
                    i += 1
            t += n
            flag = self._done_flags[chunk % 2]  # reused by chunk + 2, queued after this one is read
            chunk += 1
            torch.amin(self.b["done"], 0, keepdim=True, out=self._done_dev)
            flag.copy_(self._done_dev, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            pend.append((ev, flag))
            self.steps_run = t
            yield
            if len(pend) == 2:
                ev0, f0 = pend.pop(0)
                ev0.synchronize()
                if int(f0[0]) == 1:
                    break
        self.steps_run = t

    def _fetch(self, names):
        """Device buffers -> numpy: every copy queued into pinned memory, one synchronisation."""
        if not self.b[names[0]].is_cuda:
            return {k: self.b[k].numpy() for k in names}
        if not hasattr(self, "_pinned"):
            self._pinned = {}
        for k in names:
            src = self.b[k]
            h = self._pinned.get(k)
            if h is None or h.shape != src.shape or h.dtype != src.dtype:
                h = self._pinned[k] = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
            h.copy_(src, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        return {k: self._pinned[k].numpy() for k in names}

    def _result_names(self):
        names = ["res_count", "res_score", "res_step", "res_par", "lp_sum", "tok_hist", "par_hist", "step"]
        return names + (["ATT_hist", "PG_hist"] if self.keep_attn else [])

    def results(self, n_valid: int = None) -> List[Hypothesis]:
        """Best hypothesis per article (host).  The winner is picked from the device scores
        first and only the winners are backtracked, vectorised over articles (one numpy
        gather per step instead of a Python walk per candidate)."""
        return self._backtrack(self._fetch(self._result_names()), n_valid)

    def _snapshot(self, slot: int):
        """Queue device -> pinned copies of the result buffers into pinned set ``slot`` (0/1)
        on the current stream and return (arrays, event): the next batch's prologue, queued
        after these copies, may then reset the device buffers."""
        if not hasattr(self, "_snap"):
            self._snap = [{}, {}]
        pin = self._snap[slot]
        srcs = {k: self.b[k] for k in self._result_names()}
        srcs["lstm_err"] = self.eng.w["lstm_err"]  # checked with the results, one batch late
        srcs["tail_err"] = self.b["tail_err"]
        for k, src in srcs.items():
            h = pin.get(k)
            if h is None or h.shape != src.shape or h.dtype != src.dtype:
                h = pin[k] = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
            h.copy_(src, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return {k: v.numpy() for k, v in pin.items()}, ev

    FLUSH = object()  # a ``decode_batches`` input item: "no batch ready now, finish the pending one"

    def _rows_ok(self, bt):
        if bt.enc_batch.shape[0] != self.Na:
            raise ValueError(f"batch has {bt.enc_batch.shape[0]} rows, engine expects {self.Na}")
        return bt

    @staticmethod
    def _n_valid(bt) -> int:
        nv = getattr(bt, "n_valid", None)  # a PackedBatch from a packer process
        return int(nv) if nv is not None else int(bt.valid.sum())

    def decode_batches(self, batches):
        """Decode a sequence of Batches, yielding each batch's hypotheses, with the host work
        pipelined behind the GPU: a batch's result buffers are snapshotted into pinned memory
        (double-buffered) before the next batch's prologue, and backtracked on the host while
        the next batch's encoder and first decode chunk run.  Same results as ``decode`` per
        batch; the last batch is finished after the loop.

        ``batches`` may yield ``FLUSH`` (a streaming source with nothing queued): the pending
        batch is finished and yielded at once instead of waiting for the next batch (a result
        must not lag behind the next request, Issue-6)."""
        from collections import deque
        pending, slot = None, 0
        it = iter(batches)
        ov = self.overlap_encoder
        group = self.group_enc > 1 and not ov
        batch, pre, src = None, False, None
        # group_enc: the batches read ahead with the current one, each with its encoder rows
        # (engine, first row), then the item that ended the read-ahead (a FLUSH, the end None, or a
        # batch that cannot join), in source order; taken where the loop would otherwise read the
        # next item during the current batch's last chunk
        ahead = deque()
        done_src = False  # the source ended while prefetching

        def take():  # the next item: read ahead first, else the source
            return ahead.popleft() if ahead else (next(it, None), None)

        while True:
            if batch is None:
                batch, src = take()
                if batch is self.FLUSH:
                    batch = None
                    if pending is not None:
                        yield self._finish(pending)
                        pending = None
                    continue
                if batch is None:
                    break
                self._rows_ok(batch)
                pre = False
                if ov:
                    self._encode_launch(batch)
                    pre = True
            if group and src is None and not ahead:
                grp = [batch]
                while len(grp) < self.group_enc:
                    nb = next(it, None)
                    if not self._groupable(batch, nb):
                        ahead.append((nb, None))
                        break
                    self._rows_ok(nb)
                    grp.append(nb)
                if len(grp) > 1:
                    self._encode_group(grp)
                    src = (self.eng2, 0)
                    for j, nb in enumerate(grp[1:], 1):
                        ahead.insert(j - 1, (nb, (self.eng2, j * self.Na)))
            # overlap_encoder: batch n + 1's encoder runs on a side stream beside batch n's decode steps
            nxt = next(it, None) if ov else None
            flushed = nxt is self.FLUSH
            if flushed:
                nxt = None  # nothing ready: polled again while this batch's last chunk runs
            elif nxt is not None:
                self._rows_ok(nxt)
            nxt_pre = nxt is not None  # run_chunks launches its encoder beside this batch's steps
            nxt_src = None
            first, fetched = True, ov and not flushed
            for _ in self.run_chunks(batch, pre_encoded=pre, next_batch=nxt, enc_src=src):
                if first and pending is not None:  # the GPU has this batch's work queued
                    yield self._finish(pending)
                    pending = None
                first = False
                if not fetched and self.steps_run >= self.maxD:
                    # the last chunk is queued (and the one before it may still run): take the next
                    # batch now, so forming and packing it overlaps the GPU instead of following it
                    # (a streaming source forms it from the requests that arrived meanwhile)
                    fetched = True
                    nxt, nxt_src = take()
                    nxt_pre = False
                    if nxt is self.FLUSH:
                        nxt, nxt_src = None, None  # nothing ready: polled again once this batch is done
                    elif nxt is not None:
                        self._rows_ok(nxt)
                    else:
                        done_src = True
            if not fetched and ahead:  # an early exit before the last chunk: the read-ahead is next
                nxt, nxt_src = ahead.popleft()
                nxt_pre = False
                if nxt is self.FLUSH:
                    nxt, nxt_src = None, None
                elif nxt is None:
                    done_src = True
            arrays, ev = self._snapshot(slot)
            slot ^= 1
            pending = (arrays, ev, self._n_valid(batch), self.steps_run)
            batch, pre, src = nxt, (nxt is not None and nxt_pre), nxt_src
            if batch is None and done_src:
                break
        if pending is not None:
            yield self._finish(pending)

    def _finish(self, pending) -> List[Hypothesis]:
        arrays, ev, nv, self.finished_steps = pending
        ev.synchronize()
        if int(arrays["lstm_err"][0]):  # never emit garbage summaries (see check_lstm_err)
            self.eng.check_lstm_err()
        self._check_tail(int(arrays["tail_err"][0]))
        return self._backtrack(arrays, nv)

    def _backtrack(self, b, n_valid: int = None) -> List[Hypothesis]:
        beam, start, stop = self.beam, self.vocab.word2id(START_DECODING), self.vocab.word2id(STOP_DECODING)
        nsteps = int(min(b["step"][0], self.maxD))
        na = n_valid if n_valid is not None else self.Na
        ar = np.arange(na)
        base = ar * beam
        nres = b["res_count"][:na].astype(np.int64)
        fin = nres > 0
        # winners: the finished hypotheses by final score, else the live beams by average
        # log-prob including [START]; argmax keeps the first of equal maxima, as the stable
        # sort of sort_hyps does
        rs = b["res_score"][:na * beam].reshape(na, beam).astype(np.float64)
        rs = np.where(np.arange(beam)[None, :] < nres[:, None], rs, -np.inf)
        q_fin = rs.argmax(1) if na else np.zeros(0, np.int64)
        live = b["lp_sum"][:na * beam].reshape(na, beam).astype(np.float64) / (nsteps + 1)
        q_live = live.argmax(1) if na else np.zeros(0, np.int64)
        score = np.where(fin, rs[ar, q_fin], live[ar, q_live])
        t_fin = b["res_step"][base + q_fin].astype(np.int64)
        tl0 = np.where(fin, t_fin - 1, nsteps - 1)
        slot = np.where(fin, b["res_par"][base + q_fin], q_live).astype(np.int64)
        L = int(tl0.max()) + 1 if na else 0
        toks = np.zeros((na, max(L, 1)), dtype=np.int64)
        arow = np.zeros((na, max(L, 1)), dtype=np.int64)  # attention / p_gen history rows (base + parent)
        for tl in range(L - 1, -1, -1):
            act = tl <= tl0
            rows = base + slot
            par = b["par_hist"][tl, rows].astype(np.int64)
            toks[act, tl] = b["tok_hist"][tl, rows][act]
            arow[act, tl] = (base + par)[act]
            slot = np.where(act, par, slot)
        out = []
        for a in range(na):
            n = int(tl0[a]) + 1
            tokens = [start] + toks[a, :n].tolist() + ([stop] if fin[a] else [])
            atts, pgs = [], []
            if self.keep_attn:
                # copies: b's arrays are views of pinned buffers that the next batch reuses
                atts = [b["ATT_hist"][tl, arow[a, tl]].copy() for tl in range(n)]
                pgs = [float(b["PG_hist"][tl, arow[a, tl]]) if self.hps.pointer_gen else None for tl in range(n)]
                if fin[a]:
                    t, par = int(t_fin[a]), int(b["res_par"][base[a] + q_fin[a]])
                    atts.append(b["ATT_hist"][t, base[a] + par].copy())
                    pgs.append(float(b["PG_hist"][t, base[a] + par]) if self.hps.pointer_gen else None)
            sc = float(score[a])
            out.append(Hypothesis(tokens, [sc * len(tokens)] + [0.0] * (len(tokens) - 1), None, atts, pgs, None))
        return out

    def _results_walk(self, n_valid: int = None) -> List[Hypothesis]:
        """Per-candidate Python walk (the original form of ``results``; kept as the test oracle)."""
        b = {k: v.cpu().numpy() for k, v in self.b.items() if k in (
            "res_count", "res_score", "res_len", "res_step", "res_par", "lp_sum", "tok_hist", "par_hist", "step",
            "ATT_hist", "PG_hist", "done")}
        beam, start, stop = self.beam, self.vocab.word2id(START_DECODING), self.vocab.word2id(STOP_DECODING)
        nsteps = int(min(b["step"][0], self.maxD))
        out = []
        for a in range(n_valid if n_valid is not None else self.Na):
            base = a * beam

            def path(tl, slot):
                toks, atts, pgs = [], [], []
                while tl >= 0:
                    toks.append(int(b["tok_hist"][tl, base + slot]))
                    par = int(b["par_hist"][tl, base + slot])
                    if self.keep_attn:
                        atts.append(b["ATT_hist"][tl, base + par])
                        pgs.append(float(b["PG_hist"][tl, base + par]) if self.hps.pointer_gen else None)
                    slot = par
                    tl -= 1
                return toks[::-1], atts[::-1], pgs[::-1]

            cands = []
            nres = int(b["res_count"][a])
            if nres > 0:
                for q in range(nres):
                    t, par = int(b["res_step"][base + q]), int(b["res_par"][base + q])
                    toks, atts, pgs = path(t - 1, par)
                    if self.keep_attn:
                        atts = atts + [b["ATT_hist"][t, base + par]]
                        pgs = pgs + [float(b["PG_hist"][t, base + par]) if self.hps.pointer_gen else None]
                    cands.append((float(b["res_score"][base + q]), [start] + toks + [stop], atts, pgs))
            else:
                tl = nsteps - 1
                for slot in range(beam):
                    toks, atts, pgs = path(tl, slot)
                    cands.append((float(b["lp_sum"][base + slot]) / (tl + 2), [start] + toks, atts, pgs))
            best = sorted(cands, key=lambda c: c[0], reverse=True)[0]  # stable, like sort_hyps
            h = Hypothesis(best[1], [best[0] * len(best[1])] + [0.0] * (len(best[1]) - 1), None,
                           list(best[2]), list(best[3]), None)
            out.append(h)
        return out

    def decode(self, batch) -> List[Hypothesis]:
        """Decode a Batch of up to n_articles examples; best hypothesis per valid row."""
        if batch.enc_batch.shape[0] != self.Na:
            raise ValueError(f"batch has {batch.enc_batch.shape[0]} rows, engine expects {self.Na}")
        if self.eng2 is not None and not getattr(self, "_group_warm", False) and self._groupable(batch, batch):
            # the first call (a warm-up) also runs the group encoder once: its first-shape library
            # picks and kernel loads then happen here, not inside a timed decode_batches
            self._encode_group([batch])
            self._group_warm = True
        self.run(batch)
        hyps = self.results(self._n_valid(batch))  # synchronises
        self.eng.check_lstm_err()  # the encoder ran the persistent LSTM: never emit garbage summaries
        self._check_tail(int(self.b["tail_err"].item()))
        return hyps
