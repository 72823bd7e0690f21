"""MI355X production path of the pointer-generator network (train / eval).

The step is written as an explicit forward + hand-derived backward over preallocated
buffers (no autograd graph, no per-step allocation), so ``train_step`` is a fixed
sequence of launches on one stream that ``torch.cuda.graph`` captures once and replays
(hipGraph): per step ~8 kernels x D decoder steps and 2 kernels x T encoder steps, each
paying only the ~1.5 us dependent-kernel boundary instead of ~10 us of Python dispatch.

Where the work goes:
  * recurrences (encoder bi-LSTM, decoder cell, attention) -> hand-written gfx950 kernels
    (``csrc/kernels/{lstm,decoder,attention}.hip``), one launch per time step;
  * vocab distribution + pointer mixture + NLL -> fused kernel (``loss.hip``) that never
    materialises the [N, V+O] final distribution;
  * every hoistable GEMM (input projections for all T, W_h features, p_gen / output
    projections for all D, vocab projection, all weight gradients) -> one big bf16 GEMM
    each (hipBLASLt, the fastest candidate per shape: ``gemm`` / csrc/blt_gemm.cpp; fp32
    accumulate/output);
  * clip + Adagrad -> fused kernel over the flat parameter buffer (``optim.hip``).

Reference semantics: ``model.py:76-305``, ``attention_decoder.py:27-180``.
"""
from __future__ import annotations


import os
from typing import Dict, List, Optional

import numpy as np
import torch

from ..ops import ops as _ops
from .engine_config import EngineConfig
from .params import DEC, P, FlatParams, enc_prefix

BF = torch.bfloat16
F32 = torch.float32

EMB = f"{P}/embedding/embedding"
RC, RH = f"{P}/reduce_final_st/w_reduce_c", f"{P}/reduce_final_st/w_reduce_h"
BRC, BRH = f"{P}/reduce_final_st/bias_reduce_c", f"{P}/reduce_final_st/bias_reduce_h"
WH, VATT, WCOV = f"{DEC}/W_h", f"{DEC}/v", f"{DEC}/coverage/w_c"
LIN_M, LIN_B = f"{DEC}/Linear/Matrix", f"{DEC}/Linear/Bias"
CELL_K, CELL_B = f"{DEC}/lstm_cell/kernel", f"{DEC}/lstm_cell/bias"
ATT_M, ATT_B = f"{DEC}/Attention/Linear/Matrix", f"{DEC}/Attention/Linear/Bias"
PG_M, PG_B = f"{DEC}/calculate_pgen/Linear/Matrix", f"{DEC}/calculate_pgen/Linear/Bias"
OUT_M, OUT_B = f"{DEC}/AttnOutputProjection/Linear/Matrix", f"{DEC}/AttnOutputProjection/Linear/Bias"
OW, OV = f"{P}/output_projection/w", f"{P}/output_projection/v"


class LstmHandoffError(RuntimeError):
    """A persistent-LSTM launch timed out in a hand-off (a workgroup was not co-resident)."""


def enc_k(layer, d):
    return f"{enc_prefix(layer)}/bidirectional_rnn/{d}/lstm_cell/kernel"


def enc_b(layer, d):
    return f"{enc_prefix(layer)}/bidirectional_rnn/{d}/lstm_cell/bias"


# TSAMD_BLT=0: library GEMMs through torch.mm (hipBLASLt's first heuristic pick) instead of
# blt_mm (csrc/blt_gemm.cpp: hipBLASLt called directly, the fastest of its candidates per shape)
BLT = os.environ.get("TSAMD_BLT", "1") != "0"
# the long-K weight gradients (encoder, vocab dW) through blt_mm too (default: split-K batched GEMM)
BLT_WGRAD = BLT and os.environ.get("TSAMD_BLT_WGRAD", "0") == "1"
BLT_VDW = BLT and os.environ.get("TSAMD_BLT_VOCAB_DW", "0") == "1"
# TSAMD_VOCAB_PAD (default 1, fused vocab head): dlogits rows and the bf16 output-projection weight
# padded to Vp = 128-aligned columns (the pad columns stay zero: allocated zeroed, never written), so
# the two vocab-gradient GEMMs run at an aligned K / N -- dX = dlogits . W^T on the split-K
# hand-written GEMM (headline: 566 -> 426 us) or the library (config #5: 7.88 -> 6.76 ms),
# dW = X^T . dlogits on the library into a [H][Vp] scratch (653 -> 502 us with the copy)
# (tools/vocab_grad_micro.py, profiles/r6/vocab_grad.md)
VOCAB_PAD = os.environ.get("TSAMD_VOCAB_PAD", "1") != "0"
# TSAMD_CTX_NATIVE (default 1): the three batched attention-context GEMMs (ctx = a . enc_out, its
# gradients dA = dctx . enc_out^T and dE = a^T . dctx) on the hand-written ctx_bmm.hip kernels
# (step-major outputs, no tr01 pass) instead of torch.bmm + tr01
CTX_NATIVE = os.environ.get("TSAMD_CTX_NATIVE", "1") != "0"
# TSAMD_DE_BF16 (default 1; with the native context kernels and the persistent BPTT): the encoder-
# output gradient dE = a^T . dctx + dF . W_h^T kept in bf16 -- ctx_de writes a^T . dctx in bf16, the
# W_h GEMM adds into it (beta = 1, bf16 in and out), the top layer's BPTT reads it -- instead of an
# fp32 [B][T][A] buffer written, re-read and rewritten, and read again (profiles/r6/de_bf16.md)
DE_BF16 = os.environ.get("TSAMD_DE_BF16", "1") != "0"
# K.M.N above which the vocab dW keeps the 4-way split-K batched GEMM (config #5: 8.2 ms against
# 9.5 ms for the library at the padded N)
VOCAB_DW_SPLIT_MIN = 1e12
# TSAMD_VOCAB_DW_SIDE=1 (graph trainer; default 0): the vocab weight gradient dW = X^T . dlogits
# leaves the vocab-backward graph for a graph of its own, replayed on a side stream beside the
# decoder backward loop (train/trainer.py _Phase1).  Measured at the headline: phase 0 -0.4 ms,
# phase 1 +0.4 ms -- the loop's step kernels wait behind the GEMM's workgroups and share its HBM
# stream; CU-masked and low-priority side streams were slower still (profiles/r6/vocab_dw_side.md)
VOCAB_DW_SIDE = os.environ.get("TSAMD_VOCAB_DW_SIDE", "0") == "1"


# TSAMD_GEMM_BT: the hand-written MFMA GEMM (csrc/kernels/gemm_mfma.hip) for the activation GEMMs
# whose weight operand has a [N][K] twin.  "table" (default): a fixed per-shape rule from the
# recorded head-to-head timings (``_bt_rule``; profiles/r5/gemm_micro_v3.jsonl,
# profiles/r6/gemm_dispatch.md) -- the same pick on every run, box and rank; "auto" times it
# against blt_mm once per shape on the first eager call and keeps the faster (the round-5 default:
# picks could differ between runs); "1" always where eligible (deterministic mode too); "0" never
GEMM_BT = os.environ.get("TSAMD_GEMM_BT", "table")
_BT_PICK: Dict[tuple, bool] = {}
_BT_TIMES: Dict[tuple, tuple] = {}
# TSAMD_DX_MERGE=0: the input gradients of an upper encoder layer as two per-direction GEMMs +
# step_frame_hop (default: one hand-written GEMM per output direction over [dz_fw | dz_bw], rows
# gathered through the reversed index, written straight into the lower layer's step frame --
# gemm_mfma.hip AMODE 2).  Config #5 at batch 2048: same step time (391.8 vs 391.9 ms), 14 GB less
# memory (no per-direction dxs).  Layer 0 keeps the library GEMMs + from_step_frame: its merged
# GEMM (N = E = 128, one 128-column tile) measured 0.1 ms slower at batch 256
# (profiles/r5/dx_merge.md).
DX_MERGE = os.environ.get("TSAMD_DX_MERGE", "1") != "0"
# TSAMD_LSTM_FX=0: encoder layer 0's input projection x.W_x as a GEMM writing gx (fp32
# [2][T][B][4H]) before the persistent recurrence.  Default: inside the recurrence
# (lstm_persistent.hip FX): the step-frame inputs (bf16, E = 128) are gathered once and each
# step's x MFMAs run in the shadow of the hand-off wait -- no gx GEMM, no gx buffer.
LSTM_FX = os.environ.get("TSAMD_LSTM_FX", "1") != "0"
# 2 log2(e): the attention features F = enc_out . W_h are stored multiplied by it (the kernels'
# tanh argument is 2^(K u); attn_common.h fadd_bf2)
K2LOG2E = 2.8853900817779268
# the step-frame gather path replaces to_step_frame + the GEMM: kept while the gather GEMM is at
# most this much slower than the library GEMM alone (the layout pass it saves costs ~25-40 % of it)
FRAME_SLACK = 1.25


def _aligned(t: torch.Tensor) -> bool:
    return t.stride(-1) == 1 and (t.dim() < 2 or t.stride(0) % 8 == 0) and t.data_ptr() % 16 == 0


def _bt_ok(out, sa, ta, Bt, beta, bias) -> bool:
    return (GEMM_BT != "0" and Bt is not None and not ta and Bt.dtype == BF and out.is_cuda and _aligned(sa)
            and _aligned(Bt) and _aligned(out) and beta in (0.0, 1.0) and not (beta and out.dtype == BF)
            and (bias is None or (bias.dtype == F32 and bias.is_contiguous()))
            and bool(_ops().gemm_bt_ok(out.shape[0], out.shape[1], Bt.shape[1])) and sa.shape[1] == Bt.shape[1])


def _deterministic() -> bool:
    return os.environ.get("TSAMD_DETERMINISTIC", "0") not in ("", "0")


def _time_us(fn, reps: int = 3) -> float:
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def _bt_timed(out, sa, Bt, beta, bias, sb, tb):
    """(gemm_bt us, blt_mm us) of this shape on a row subset (<= 131072 rows) into scratch."""
    key = (tuple(out.shape), out.dtype, sa.shape[1], beta != 0.0, bias is not None, sa.stride(0), Bt.stride(0))
    if key not in _BT_TIMES:
        m = min(out.shape[0], 131072)
        a, o = sa[:m], torch.empty(m, out.shape[1], dtype=out.dtype, device=out.device)
        k = _ops()
        t_bt = _time_us(lambda: k.gemm_bt(a, Bt, o, float(beta), bias, None, None, 0, 0, 0, None))
        t_blt = _time_us(lambda: k.blt_mm(a, sb, o, False, tb, float(beta), bias))
        _BT_TIMES[key] = (t_bt, t_blt)
    return _BT_TIMES[key]


def _bt_rule(K: int, out_bf16: bool, slack: float) -> bool:
    """The fixed dispatch (TSAMD_GEMM_BT=table), from the head-to-head records
    (profiles/r5/gemm_micro_v3.jsonl and the round-6 timed picks, profiles/r6/gemm_dispatch.md):
    the hand-written GEMM wins every K <= 256 shape (b256_gx 104 vs 112 us, c5_gx_l0 1340 vs 1443,
    25600 x 128 x 128 8.1 vs 16.2), the bf16-out shapes up to K = 1024 (25600 x 512 x 512 22.2 vs
    29.1, c5_F 1694 vs 1707; b256_F measured both ways across runs) and loses the fp32-out
    K >= 512 shapes (25600 x 256 x 512 28.1 vs 20.4, 102400 x 512 x 512 154 vs 117, c5_dx_l1 3380
    vs 3010) -- within FRAME_SLACK where it also saves the step-frame layout pass."""
    return slack > 1.0 or K <= 256 or (out_bf16 and K <= 1024)


def _use_bt(out, sa, ta, Bt, beta, bias, sb, tb, slack: float = 1.0) -> bool:
    if not _bt_ok(out, sa, ta, Bt, beta, bias):
        return False
    if GEMM_BT == "1" or _deterministic():
        return True
    key = (tuple(out.shape), out.dtype, sa.shape[1], beta != 0.0, bias is not None, sa.stride(0), Bt.stride(0), slack)
    if key not in _BT_PICK:
        if GEMM_BT != "auto":
            _BT_PICK[key] = _bt_rule(sa.shape[1], out.dtype == BF, slack)
        elif torch.cuda.is_current_stream_capturing():
            return False  # first seen inside a capture: no timing possible, keep the library GEMM
        else:
            t_bt, t_blt = _bt_timed(out, sa, Bt, beta, bias, sb, tb)
            _BT_PICK[key] = t_bt <= slack * t_blt
    return _BT_PICK[key]


def gemm_bt_stats() -> Dict[str, object]:
    """The hand-written-GEMM dispatch: mode, every shape seen (M x N x K, out dtype, frame
    gather) with the kernel it got, and (mode "auto") the timings behind the picks."""
    picks = {f"{k[0][0]}x{k[0][1]}x{k[2]}{'_bf16' if k[1] == BF else ''}{'_frame' if k[7] > 1.0 else ''}":
             ("gemm_bt" if v else "hipblaslt") for k, v in _BT_PICK.items()}
    return {"mode": "deterministic" if _deterministic() else GEMM_BT, "shapes": len(_BT_PICK),
            "gemm_bt": int(sum(_BT_PICK.values())), "picks": picks,
            "timed_us": {f"{k[0][0]}x{k[0][1]}x{k[2]}": [round(v[0], 1), round(v[1], 1)] for k, v in _BT_TIMES.items()}}


def _stored(x: torch.Tensor):
    """(row-contiguous tensor holding x's elements, whether x is its transpose)."""
    if x.stride(-1) == 1:
        return x, False
    if x.dim() == 2 and x.stride(0) == 1:
        return x.t(), True
    return x.contiguous(), False


def gemm(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor, beta: float = 0.0,
         bias: Optional[torch.Tensor] = None, bt: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = beta * out + a . b (+ bias[N]): bf16 operands, fp32 accumulate, fp32 or bf16 ``out``
    written in place (row slices of bigger buffers included).  Transposed views of stored
    operands are passed as (storage, transpose flag), never copied.  ``bt``: a row-major [N][K]
    twin of ``b`` (a packed weight layout) -- with it, or when ``b`` is itself the transpose of a
    row-major [N][K] matrix, the hand-written MFMA GEMM is eligible (TSAMD_GEMM_BT)."""
    if BLT and out.is_cuda and a.dtype == BF and b.dtype == BF:
        sa, ta = _stored(a)
        sb, tb = _stored(b)
        Bt = sb if tb else bt
        if _use_bt(out, sa, ta, Bt, beta, bias, sb, tb):
            _ops().gemm_bt(sa, Bt, out, float(beta), bias, None, None, 0, 0, 0, None)
            return out
        _ops().blt_mm(sa, sb, out, ta, tb, float(beta), bias)
        return out
    if beta != 0.0:
        assert bias is None
        if out.dtype == F32 and a.dtype == BF:
            return torch.addmm(out, a, b, out_dtype=F32, out=out)
        return out.addmm_(a, b, beta=beta)
    if out.dtype == F32 and a.dtype == BF:
        if bias is None:
            return torch.mm(a, b, out_dtype=F32, out=out)
        return torch.addmm(bias, a, b, out_dtype=F32, out=out)
    if bias is None:
        return torch.mm(a, b, out=out)
    return torch.addmm(bias.to(out.dtype), a, b, out=out)


def mm_into(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor, bias: Optional[torch.Tensor] = None,
            bt: Optional[torch.Tensor] = None):
    """out = a . b (+ bias), fp32 accumulate, written straight into ``out`` (fp32 or bf16)
    -- no temporary, no separate bias pass (GEMM bias epilogue)."""
    return gemm(out, a, b, 0.0, bias, bt)


def wgrad_into(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor):
    """out[M,N] = a[K,M]^T . b[K,N] for weight gradients: K (= rows: tokens or decoder steps
    x batch) is long and M x N is a handful of output tiles.  blt_mm picks among hipBLASLt's
    stream-K / split-K solutions per shape.  The torch path (TSAMD_BLT=0) splits K into S
    chunks as one batched GEMM (S x the tiles, fp32 partials) and sums the partials: 3-5x
    faster than torch.mm's pick for K = 25.6k-102k (tools/wgrad_micro.py)."""
    K = a.shape[0]
    if a.is_cuda and BLT_WGRAD and a.dtype == BF:
        return gemm(out, a.t(), b)
    if a.is_cuda:
        for S in ((32, 16, 8) if K >= 65536 else (16, 8)):
            if K % S == 0 and K // S >= 256:
                parts = torch.bmm(a.reshape(S, K // S, a.shape[1]).transpose(1, 2), b.reshape(S, K // S, b.shape[1]),
                                  out_dtype=F32)
                return torch.sum(parts, 0, out=out)
    return out.copy_(mmf(a.t(), b))


WGRAD_TT = os.environ.get("TSAMD_WGRAD_TT", "1") != "0"
WGRAD_TT_MIN = float(os.environ.get("TSAMD_WGRAD_TT_MIN", 1e11))
_WG_WS: Dict[object, torch.Tensor] = {}
_WG_WS_OLD: List[torch.Tensor] = []


def wgrad_enc_into(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor):
    """Long-K weight gradients out = a^T . b: the encoder's x^T.dz / h^T.dz (K = T.B tokens:
    102k at the headline, 1.6M at config #5) and the inline decoder-side ones (K = D.B): the
    hand-written deterministic split-K GEMM (wgrad.hip ``wgrad_tt``: fp32 slabs summed in split
    order, no atomics, no torch.sum pass) where the shape fits it and is large, else
    ``wgrad_into``.  Its slab workspace is one buffer per device, grown outside graph capture
    (the trainer's eager warm-up) and reused by the captured graphs: these calls run one after
    another on the backward stream (model.py:290-297 / 89-93 gradients)."""
    # large shapes only (config #5: K.M.N >= 3e11); at the headline's K = 102k the split-K bmm is
    # as fast or faster (profiles/r6/wgrad_tt.md)
    if (WGRAD_TT and a.is_cuda and a.dtype == BF and b.dtype == BF and out.dtype == F32
            and a.shape[0] * a.shape[1] * b.shape[1] >= WGRAD_TT_MIN):
        k = _ops()
        n = int(k.wgrad_tt_ws(a.shape[1], b.shape[1], a.shape[0]))
        if n > 0:
            key = out.device
            ws = _WG_WS.get(key)
            if ws is None or ws.numel() < n:
                if torch.cuda.is_current_stream_capturing():
                    return wgrad_into(out, a, b)  # first seen inside a capture: no allocation there
                if ws is not None:  # graphs captured earlier may hold the old buffer: never freed
                    _WG_WS_OLD.append(ws)
                ws = _WG_WS[key] = torch.empty(n, device=out.device, dtype=F32)
            if k.wgrad_tt(a, b, out, ws, False):
                return out
    return wgrad_into(out, a, b)


def mmf(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """bf16 x bf16 -> fp32 GEMM (fp32 accumulate), hipBLASLt."""
    if BLT and a.is_cuda:
        return gemm(torch.empty(a.shape[0], b.shape[1], device=a.device, dtype=F32), a, b)
    if not a.is_cuda:  # (the out_dtype matmul is GPU-only)
        return a.float() @ b.float()
    return torch.mm(a, b, out_dtype=F32)


def host_inputs(batch, hps, D: int, sort_rows: bool = False, need_grad: bool = True) -> Dict[str, np.ndarray]:
    """The engine's per-batch inputs as host arrays (pure numpy: runs in loader worker
    processes too): token ids, lengths, the reversed-index map of the backward LSTM
    direction, extended-vocab ids, step-major decoder inputs / targets and the per-(step,
    row) loss weights of the reference's loss averaging (``model.py:252-268``).

    ``sort_rows``: the engine's rows are the batch's rows ordered by live decoder steps, longest
    first (stable), so the steps a row skips past its summary form a suffix of the rows at every
    decoder step and whole 16-row tiles of the decoder kernels go idle together.  The loss is a
    sum over rows; ``row_src[b]`` is the batch row of engine row b.

    ``need_grad`` False (decode / eval packs): the embedding-gradient id order is not computed
    (zeros; no backward reads it) -- the largest host cost of a serving batch."""
    T = batch.enc_batch.shape[1]
    lens = batch.enc_lens.astype(np.int64)
    if lens.min() < 1:
        raise ValueError("empty article in batch")
    t = np.arange(T)[None, :]
    rev = np.where(t < lens[:, None], lens[:, None] - 1 - t, t)
    valid = batch.valid.astype(np.float64)
    nvalid = valid.sum()
    if batch.dec_batch.shape[1] < D:
        raise ValueError(f"batch has {batch.dec_batch.shape[1]} decoder steps, engine needs {D}")
    dm = batch.dec_padding_mask[:, :D].astype(np.float64)
    dec_lens = dm.sum(1)
    if hps.pointer_gen:
        rowg = dm * (valid / (np.maximum(dec_lens, 1) * nvalid))[:, None]
    else:  # sequence_loss: sum(mask*CE)/sum(mask)
        wm = dm * valid[:, None]
        rowg = wm / wm.sum()
    gcl = hps.cov_loss_wt * dm * (valid / (np.maximum(dec_lens, 1) * nvalid))[:, None]
    # live decoder steps per row: 1 + the last step with a nonzero loss weight (0: none).  Steps
    # past it reach only masked loss terms (model.py:252-268), so their forward values and
    # gradients need not be computed (EngineConfig.skip_pad_steps)
    live = (rowg != 0) | (gcl != 0)  # [B, D]
    dlen = np.where(live.any(1), D - np.argmax(live[:, ::-1], 1), 0)
    src = np.argsort(-dlen, kind="stable") if sort_rows else np.arange(len(dlen))
    enc_batch, ext, rev = batch.enc_batch[src], batch.enc_batch_extend_vocab[src], rev[src]
    enc_lens, rowg, gcl, dlen = batch.enc_lens[src], rowg[src], gcl[src], dlen[src]
    dec_t = np.ascontiguousarray(batch.dec_batch[src, :D].T).astype(np.int64)
    if need_grad:
        sid, perm = emb_sort(enc_batch, dec_t)
    else:
        sid = perm = np.zeros(enc_batch.size + dec_t.size, dtype=np.int32)
    # the fused vocab head's 32-row blocks of the t-major [D * B] rows that hold a live row, listed
    # first (vblk, vblk_n of them); vlive per block (the blocks pass 2 must keep zeroed)
    nb = (D * len(dlen) + 31) // 32
    lr = np.zeros(nb * 32, dtype=bool)
    lr[:D * len(dlen)] = (np.arange(D)[:, None] < dlen[None, :]).reshape(-1)
    vlive = lr.reshape(nb, 32).any(1)
    vblk = np.full(nb, nb, dtype=np.int32)  # past vblk_n: the dummy (all-zero) block nb of the compacted head
    live_ids = np.nonzero(vlive)[0]
    vblk[:len(live_ids)] = live_ids
    return {
        "enc_batch": enc_batch.astype(np.int64),
        "enc_lens": enc_lens.astype(np.int32),
        "rev_idx": rev.astype(np.int64),
        "ext": ext.astype(np.int32),
        "dec_batch_t": dec_t,
        "target_t": np.ascontiguousarray(batch.target_batch[src, :D].T).astype(np.int32),
        "rowg": np.ascontiguousarray(rowg.T).astype(np.float32),
        "gcl": np.ascontiguousarray(gcl.T).astype(np.float32),
        "emb_sid": sid,
        "emb_perm": perm,
        "dlen": dlen.astype(np.int32),
        "row_src": src.astype(np.int32),
        "vlive": vlive.astype(np.int32),
        "vblk": vblk,
        "vblk_n": np.array([len(live_ids)], dtype=np.int32),
    }


def emb_sort(enc_batch: np.ndarray, dec_t: np.ndarray):
    """Stable id order of the step's embedding-gradient rows: the encoder tokens (row b*T + t)
    then the decoder inputs (row B*T + t*B + b).  Returns (sorted ids, row permutation), int32.

    Computed on the host with the batch (a loader worker process when one is used) instead of
    a device sort inside the captured backward: torch.sort of more than ~1M keys (rocprim's
    onesweep radix sort) faulted the GPU on the second replay of the captured graph at config #5
    batch 2048 (memory-aperture violation at that kernel, three runs; the same step eager and
    kernel-serialised ran clean: profiles/r3/b2048_fault.md).  The stable order also makes the
    gradient's per-id summation order a function of the batch alone (deterministic mode)."""
    ids = np.concatenate([np.asarray(enc_batch).reshape(-1), np.asarray(dec_t).reshape(-1)])
    if ids.size and (ids.min() < 0 or ids.max() >= 2 ** 31):
        raise ValueError("token ids out of range")
    # numpy's stable sort is a radix sort for 16-bit keys: ~5 ms for 230k ids, 28 ms for 1.8M
    key = ids.astype(np.uint16) if ids.size == 0 or ids.max() < 65536 else ids.astype(np.int32)
    perm = np.argsort(key, kind="stable").astype(np.int32)
    return ids[perm].astype(np.int32), perm


_NP = {torch.long: np.int64, torch.int32: np.int32, F32: np.float32}


def input_layout(B: int, T: int, D: int):
    """Byte layout of the engine's input pack: [(name, offset, shape, torch dtype, nbytes)],
    total size (every array 256-byte aligned); the device copy is one buffer with views."""
    shapes = {"BT": (B, T), "B": (B,), "DB": (D, B), "R": (B * T + D * B,), "VB": ((D * B + 31) // 32,), "1": (1,)}
    layout, off = [], 0
    for name, sk, dt in (("enc_batch", "BT", torch.long), ("enc_lens", "B", torch.int32),
                         ("rev_idx", "BT", torch.long), ("ext", "BT", torch.int32),
                         ("dec_batch_t", "DB", torch.long), ("target_t", "DB", torch.int32),
                         ("rowg", "DB", F32), ("gcl", "DB", F32),
                         ("emb_sid", "R", torch.int32), ("emb_perm", "R", torch.int32), ("dlen", "B", torch.int32),
                         ("row_src", "B", torch.int32), ("vlive", "VB", torch.int32), ("vblk", "VB", torch.int32),
                         ("vblk_n", "1", torch.int32)):
        shp = shapes[sk]
        nb = int(np.prod(shp)) * np.dtype(_NP[dt]).itemsize
        layout.append((name, off, shp, dt, nb))
        off += (nb + 255) // 256 * 256
    return layout, off


def pack_host_inputs(host: Dict[str, np.ndarray], layout, out: Optional[np.ndarray] = None) -> np.ndarray:
    """host_inputs arrays -> one uint8 buffer in ``layout`` order (``out`` if given)."""
    if out is None:
        out = np.zeros(layout[-1][1] + (layout[-1][4] + 255) // 256 * 256, dtype=np.uint8)
    for name, o, shp, dt, nb in layout:
        a = np.ascontiguousarray(host[name], dtype=_NP[dt])
        if a.shape != tuple(shp):
            raise ValueError(f"input {name}: shape {a.shape} != {tuple(shp)}")
        out[o:o + nb] = a.reshape(-1).view(np.uint8)
    return out


class HipPointerGenerator:
    """Fixed-shape (B rows, T encoder steps, D decoder steps) train/eval engine."""

    def __init__(self, hps, vsize: int, params: FlatParams, B: int, T: int, D: Optional[int] = None,
                 cfg: Optional[EngineConfig] = None):
        self.hps = hps
        self.cfg = cfg = cfg or EngineConfig.from_env()
        self.V, self.E, self.H = vsize, hps.emb_dim, hps.hidden_dim
        self.A = 2 * self.H
        self.B, self.T, self.D = B, T, D or hps.max_dec_steps
        self.L = max(1, getattr(hps, "enc_layers", 1))
        self.p = params
        self.dev = params.flat.device
        if self.dev.type != "cuda":
            raise RuntimeError("HipPointerGenerator runs on the GPU; use ReferencePointerGenerator on CPU")
        if self.E % 32 or self.H % 32:
            raise ValueError("emb_dim and hidden_dim must be multiples of 32 for the MFMA kernels")
        if T > 2048:
            raise ValueError("max_enc_steps > 2048 not supported by the attention kernels")
        # Row counts (tokens B*T, decoder rows D*B) are int32 kernel arguments; every element
        # offset is 64-bit (config #5 at batch 2048 runs 3.4G-element gate buffers and 10G-element
        # dlogits: tools/big_batch_steps.py, tests/test_gpu_production.py).
        if B * T >= 2 ** 31 or self.D * B * max(self.V, 4 * self.H) >= 2 ** 62:
            raise ValueError(f"batch {B} x enc {T} exceeds the kernels' 32-bit row counts")
        self.k = _ops()
        self.grad_scale = 1.0  # set to 1/world by a data-parallel trainer (see optimizer_step)
        # set by a data-parallel trainer: a persistent-LSTM timeout poisons the last gradient
        # element before its bucket's all-reduce, so every rank skips that update (poison_where)
        self.poison_on_lstm_err = False
        self.nchunk = int(self.k.attn_chunks(T))
        # The decoder recurrences (forward: cell -> s-projection -> score -> softmax/context;
        # backward: attention step -> cell backward -> dz backward) are independent across
        # batch rows.  With ``split`` > 1 the rows are cut into that many groups, each group's
        # chain of per-step launches runs on its own stream (forked from and joined to the
        # current stream, so a captured hipGraph holds parallel branches): one group's small
        # latency-bound cell kernels run beside another group's bandwidth-bound attention
        # kernels instead of serialising behind them.  cfg.split overrides (1 = one chain).
        # Default: 2 groups from B = 128, 4 from B = 256 (config #5, H = 512: B = 512 161.6 -> 156.9 ms
        # per step, B = 1024 309.0 -> 301.1-301.9 ms; 8 groups 303.2 (profiles/r2/ab/split_groups.jsonl);
        # B = 256 since the LDS-parameter row backward: 4 groups 19.35 / 19.49 ms, 2 groups 20.21 /
        # 19.99, 8 groups 27.2, 1 group 20.75 (profiles/r3/ab/split_b256.txt))
        # With the projected attention and the rows sorted by live steps (B = 256: 2 groups 16.65-16.75 ms,
        # 1 group 16.77, 3 groups 16.99, 4 groups 17.37-17.44; config #5 batch 1024: 2 = 4 = 204.4 ms, 8 206.6;
        # profiles/r3/ab/split_sorted.txt)
        # B = 128: 1 group 13.67 vs 2 groups 13.86 ms (profiles/r3/ab/small_batch.txt)
        # Deterministic mode runs the same row groups: each row's arithmetic is the same on any
        # stream, and test_deterministic_mode_bit_identical requires split 1 / 2 / 4 to give the
        # single chain's bits (profiles/r4/det_streams.md: the round-3 one-chain override is gone)
        # Round 5 (projected attention with dot2 scores, FX encoder): 4 groups from B = 1024 --
        # config #5 batch 2048 366.2-367.7 ms vs 368.9-369.7 with 2 groups (8: 368.3; 8 forward / 4
        # backward 366.4), batch 1024 188.7 vs 191.0 ms (profiles/r5/runs/r5t*)
        sp = cfg.split or (4 if B >= 1024 and B % 64 == 0 else 2 if B >= 256 and B % 32 == 0 else 1)
        self.split = sp if (sp > 1 and B % (16 * sp) == 0) else 1
        # cfg.split_bwd: the decoder backward loop's own group count (default: split; B = 256 with
        # 4 forward groups: 4 backward groups 19.48 ms per step, 2 groups 19.79)
        spb = cfg.split_bwd or self.split
        self.split_bwd = spb if (spb > 1 and B % (16 * spb) == 0) else 1
        ns = max(self.split, self.split_bwd)
        self._streams = [torch.cuda.Stream(self.dev) for _ in range(ns)] if ns > 1 else []
        self._alloc()
        self.pack()

    # ------------------------------------------------------------------ buffers
    def _alloc(self):
        B, T, D, E, H, A, V, L = self.B, self.T, self.D, self.E, self.H, self.A, self.V, self.L
        z = lambda *s, dt=F32: torch.zeros(*s, dtype=dt, device=self.dev)
        w: Dict[str, torch.Tensor] = {}
        # inputs (static, copied into before every replay): views of ONE device buffer, so a
        # batch arrives with one H2D copy from a pinned host pack instead of eight (each
        # in-stream copy costs ~15 us of DMA latency ahead of the step)
        layout, off = input_layout(B, T, D)
        self._in_layout = layout
        self._in_off = {name: o for name, o, _, _, _ in layout}
        self._in_pack = torch.zeros(off, dtype=torch.uint8, device=self.dev)
        for name, o, shp, dt, nb in layout:
            w[name] = self._in_pack[o:o + nb].view(dt).view(shp)
        w["enc_lens"].fill_(1)
        # double-buffered pinned host packs and device staging copies: the H2D copy of the next
        # batch runs on a copy stream while the current step computes; the step itself only
        # pays a device-to-device copy staging -> inputs (~4 MB at B = 256: a few us instead of
        # ~0.2 ms of PCIe latency + transfer in the step's stream)
        self._in_host = [torch.zeros(off, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        self._in_stage = [torch.zeros(off, dtype=torch.uint8, device=self.dev) for _ in range(2)]
        self._in_ev = [None, None]     # host pack i free again (its H2D copy finished)
        self._in_used = [None, None]   # staging copy i consumed (its D2D copy into the inputs finished)
        self._copy_stream = torch.cuda.Stream(self.dev)
        self._in_i = 0
        # upper encoder layers' input gradients through the merged hand-written GEMM (no dxs)
        self.dx_merge = (DX_MERGE and L > 1 and BLT and GEMM_BT != "0" and self.dev.type == "cuda"
                         and hasattr(self.k, "gemm_bt_merge") and bool(self.k.gemm_bt_ok(T * B, H, 8 * H)))
        # layer 0's input projection inside the persistent recurrence (no gx)
        self.lstm_fx = (LSTM_FX and self.cfg.persistent_lstm and self.dev.type == "cuda"
                        and hasattr(self.k, "lstm_persistent_fx_ok") and bool(self.k.lstm_persistent_fx_ok(H, B, E)))
        # encoder, per layer
        self.enc = []
        for layer in range(L):
            din = E if layer == 0 else A
            self.enc.append({
                "din": din,
                "x_sf": z(2, T, B, din, dt=BF),          # step-frame inputs (bw reversed)
                "gx": None if (self.lstm_fx and layer == 0) else z(2, T, B, 4 * H),  # [2][T][B][H][4 gates]
                "hs": z(2, T + 1, B, H, dt=BF),
                "cs": z(2, T + 1, B, H),
                "acts": z(2, T, B, 4 * H),               # [2][T][B][H][4 gates]
                "out": z(B, T, A, dt=BF),
                "dz": z(2, T, B, 4 * H, dt=BF),
                "dout": z(B, T, A),
                "dh_fin": z(2, B, H),
                "dc_carry": z(2, B, H),
                "dxs": None if (self.dx_merge and layer > 0) else z(2, T * B, din),
                # batch-frame input gradient: the embedding gradient's source (layer 0 only; above it
                # step_frame_hop feeds the layer below directly)
                "dx": z(B, T, din) if layer == 0 else None,
            })
        # persistent weight-resident recurrence (lstm_persistent.hip) when the shape allows
        # it; cfg.persistent_lstm = False forces the per-step kernels
        cfg = self.cfg
        self.persistent_lstm = cfg.persistent_lstm and int(self.k.lstm_persistent_grid(H, B)) > 0
        if self.persistent_lstm:
            w["lstm_xf"] = z(int(self.k.lstm_persistent_xbuf(H, B, False)), dt=torch.long)
            w["lstm_xb"] = z(int(self.k.lstm_persistent_xbuf(H, B, True)), dt=torch.long)
            w["lstm_db"] = z(2, 4 * H)  # gate-bias gradients [fw; bw] accumulated by the BPTT kernel
        w["lstm_err"] = z(1, dt=torch.int32)
        # decoder-side weight gradients that nothing later in the step reads (output projection,
        # cell, input merge, attention query, W_h) run on a side stream beside the encoder BPTT,
        # which leaves half the CUs idle at B <= 256 (forked and joined inside backward_tail);
        # not when the persistent BPTT grid fills the chip.  Only custom kernels run on that
        # stream (wgrad.hip, cast_colsum, reductions): the library GEMMs are stream-K kernels
        # (hipBLASLt SK3: a tile owner spins on flags of higher-numbered workgroups), and two
        # such kernels -- or one beside the persistent BPTT, which spins on its own peers -- can
        # each hold CUs the other's waiting workgroups need (two concurrent library GEMMs in the
        # vocab backward hung on MI355X).  cfg.defer_wgrad = False: inline.
        self._late = []
        # Measured (bench A/B): +0.6-1.3% at B = 256; at B = 64 / 128 the BPTT it runs beside
        # slows more (its hand-offs are latency-bound) than the moved work saves, so B >= 256.
        # deterministic mode (cfg.deterministic): no fp32 atomics anywhere in the step -- fixed-order
        # reductions for the embedding, bias and attention-parameter gradients, the row-resident
        # attention backward (no atomics over position blocks), the weight gradients inline
        self.det = cfg.deterministic
        self.defer_wgrad = (not self.det and cfg.defer_wgrad and B >= 256 and E % 128 == 0
                            and H % 128 == 0 and (
            not self.persistent_lstm or
            int(self.k.lstm_persistent_grid(H, B)) <= int(self.k.lstm_persistent_capacity(H)) - 64))
        self._late_stream = torch.cuda.Stream(self.dev) if self.defer_wgrad else None
        # reduce_states: pre-activations [c; h], bf16 [fw, bw] inputs and bf16 dp (wgrad operands)
        w["rs_pre"] = z(2, B, H)
        w["rs_cat"] = z(2, B, 2 * H, dt=BF)
        w["rs_dp"] = z(2, B, H, dt=BF)
        # row-resident attention (attention_row.hip: one workgroup per row and step, forward
        # score + softmax + context in one launch) from batch 64 (with the projected context and the
        # skipped dead steps B = 64 12.02 -> 11.77 ms against the multi-block kernels); else the
        # multi-block-per-row kernels of attention.hip.  cfg.row_attn forces it on / off.
        self.row_attn = bool(self.k.attn_row_ok(A, T)) and (
            cfg.row_attn if cfg.row_attn is not None else (B >= 64 or self.det))
        # backward: the row kernel too (its per-feature parameters in LDS: at A = 1024, 256 rows,
        # T = 800 it streams E and F at 5.2 TB/s, 162 us vs 206 us for the multi-block
        # attn_bwd_step -- tools/attn_micro_c5.py)
        self.row_attn_bwd = self.row_attn
        # projected context (attention_row.hip, attn_*_rowp): the recurrence streams F and
        # G = enc_out . W_in[E:] ([B, T, E]) instead of F and enc_out; ctx of all steps is one batched
        # GEMM after the loop, the output-projection / p_gen part of dctx . E_i one before the backward
        self.proj_attn = self.row_attn and cfg.proj_attn and bool(self.k.attn_rowp_ok(A, T, E))
        if self.proj_attn:
            w["Genc"] = z(B, T, E, dt=BF)
            w["GV"] = z(D, B, E)         # g_t = sum_i a_ti G_i = ctx_t . W_in[E:]
            w["GVb"] = z(D, B, E, dt=BF)
            w["bd_tmp"] = z(B * D * max(A, T))  # [B, D, A] ctx / [B, D, T] da_dir GEMM outputs
            w["DXb"] = z(D, B, E, dt=BF)
        # (row, step) pairs past the row's last loss-weighted step are skipped by the projected
        # kernels (their outputs are written as zeros; loss and gradients are unchanged)
        self.skip_pad = self.proj_attn and cfg.skip_pad_steps
        self.compact_vocab = self.skip_pad and cfg.fused_vocab_train and cfg.compact_vocab_grad and not cfg.deterministic \
            and H in (128, 256, 512) and (D * B) % 32 == 0
        w["F"] = z(B, T, A, dt=BF)
        # transposed copy for the lanes-over-positions score kernel (not needed by the row
        # kernels; the beam decoder sets keep_ft to get it from _encoder_forward)
        self.keep_ft = not self.row_attn
        w["Ft"] = z(B, A, T, dt=BF) if self.keep_ft else None
        w["XG"] = z(D, B, 4 * H)
        # decoder forward state
        w["xe"] = z(D, B, E)
        w["X"] = z(D, B, E)
        w["Xb"] = z(D, B, E, dt=BF)
        w["Cst"] = z(D + 1, B, H)
        w["Cb"] = z(D + 1, B, H, dt=BF)
        w["Hb"] = z(D + 1, B, H, dt=BF)
        w["ACT"] = z(D, B, 4 * H)
        w["S"] = z(D, B, A)
        w["COV"] = z(D + 1, B, T)
        w["ATT"] = z(D, B, T)
        w["CTX"] = z(D, B, A)
        w["CTXb"] = z(D, B, A, dt=BF)
        w["e"] = z(B, T)
        w["covloss"] = z(D, B)
        # [outb | 1 | 0...]: the ones column makes the output-projection weight-gradient GEMM
        # also produce the bias gradient (one read of dlogits instead of two).  One extra all-zero
        # 32-row block after the D * B rows: the dummy block the compacted vocab head gathers for
        # its padding (see backward_head)
        nblk = (D * B + 31) // 32
        w["outb_blk"] = z(nblk * 32 + 32, H + 8, dt=BF)
        w["outb_ext"] = w["outb_blk"][:D * B]
        w["outb_ext"][:, H] = 1.0
        w["outb"] = w["outb_ext"][:, :H]
        w["pg"] = z(D, B)
        w["loss_row"] = z(D, B)
        # fused vocab head (vocab_train.hip): logits live only in MFMA accumulators, the
        # [N, V] buffer receives dlogits; cfg.fused_vocab_train = False selects the library GEMM
        # (bf16 logits, bias in the epilogue) + ptr_loss, which rewrites them in place
        self.fused_vocab = cfg.fused_vocab_train and H in (128, 256, 512)
        if self.fused_vocab:
            N = D * B
            w["vpart"] = z(int(self.k.vocab_train_tiles(V, H)) * N * 2)
            for n in ("zg", "lse", "pv", "alpha"):
                w[n] = z(N)
            w["dbias"] = z(V)  # output_projection/v gradient, column sums taken inside pass 2
            w["vstate"] = z((N + 31) // 32, dt=torch.int32)  # dlogits blocks written by the last pass 2
        # the fused head's dlogits rows: Vp columns (TSAMD_VOCAB_PAD; the columns past V stay zero)
        self.Vp = -(-V // 128) * 128 if (self.fused_vocab and VOCAB_PAD) else V
        self.ctx_native = CTX_NATIVE and self.dev.type == "cuda" and bool(self.k.ctx_bmm_ok(B, T, D, A))
        w["logits"] = z(D * B, self.Vp, dt=BF)
        if self.Vp != V and self.det:
            w["dbias_p"] = z(self.Vp)  # deterministic column sums over the padded rows
        # backward
        w["dlogits"] = w["logits"]
        # compacted vocab head (skip_pad with the fused head, not deterministic mode): pass 2 writes the
        # live 32-row blocks' dlogits to consecutive rows, and the two gradient GEMMs run over the
        # live rows only, rounded up to one of a few block counts (one captured graph each)
        self.vocab_buckets = sorted({max(1, -(-nblk * f // 8)) for f in (4, 5, 6, 7, 8)})
        self.nbk = self.vocab_buckets[-1]
        w["dpre"] = z(D, B)
        w["dA"] = z(D, B, T)
        w["DCTX"] = z(D, B, A)
        w["DX"] = z(D, B, E)
        w["DZ"] = z(D, B, 4 * H, dt=BF)
        w["DS"] = z(D, B, A)
        w["d_emb_dec"] = z(D * B, E)  # decoder-input embedding gradient rows
        w["out_f32"] = z(D * B, H)  # output projection [h, ctx] . W_o + b (fp32, before the bf16 copy)
        if self.hps.pointer_gen:  # p_gen direct terms of the decoder backward (pgen_dirs)
            w["dC_dir"] = z(D, B, H)
            w["dX_dir"] = z(D, B, E)
        w["DE"] = z(D, B, T)
        w["dcov"] = z(2, B, T)
        w["dh_rec"] = z(B, H)
        w["dc_carry"] = z(B, H)
        w["dF"] = z(B, T, A, dt=BF)  # written whole (zeros past len) by attn_bwd_feat, in bf16
        w["ATTb"] = z(D, B, T, dt=BF)
        w["DCTXb"] = z(D, B, A, dt=BF)
        self.de_bf16 = DE_BF16 and self.ctx_native and self.persistent_lstm
        self._dE = z(B, T, A, dt=BF if self.de_bf16 else F32)
        self.split_vocab_dw = False  # see _dw_job (the graph trainer sets it with TSAMD_VOCAB_DW_SIDE)
        self._pending_dw = None
        # attn_bwd_feat partial rows (spread the atomics), summed after; deterministic mode: one
        # row per workgroup (a single writer per slot)
        nfeat = ((T + 15) // 16) * B
        nslot = 1 << (nfeat - 1).bit_length() if self.det else 32
        w["dv"] = z(nslot, A)
        w["dwc"] = z(nslot, A)
        if self.det:  # embedding-gradient chunk partials (emb_grad_det)
            nc = int(self.k.emb_grad_det_chunks(B * T + D * B))
            w["emb_pf"] = z(nc, E)
            w["emb_pl"] = z(nc, E)
        # optimizer
        w["opt_part"] = z(int(self.k.opt_parts()))
        w["gnorm"] = z(1)
        w["nan_flag"] = z(1, dt=torch.int32)
        self.w = w

    def check_lstm_err(self) -> None:
        """Host sync: raise if a persistent-LSTM hand-off timed out in any launch since the
        engine was built.  The word is sticky: those results were garbage, the optimizer
        kernel skipped the update, and eval / decode must not report them."""
        if int(self.w["lstm_err"].item()):
            raise LstmHandoffError("persistent LSTM hand-off timed out (a workgroup was not co-resident); "
                                   "results of that launch were discarded -- set TSAMD_LSTM_PERSISTENT=0 "
                                   "(EngineConfig.persistent_lstm)")

    # ------------------------------------------------------------------ weights
    def pack(self):
        """fp32 master -> bf16 kernel layouts (recomputed after every optimizer step).  The
        first call allocates the layouts through torch ops; later calls (the optimizer graph)
        recompute W_comb with one GEMM and refresh every layout with ONE pack_cast launch over a
        job table (pack.hip) instead of ~50 cast / copy / cat launches."""
        jobs = getattr(self, "_pack_jobs", None)
        if jobs is not None:
            E = self.E
            torch.mm(self.p[LIN_M][E:], self.p[CELL_K][:E], out=self._wcomb)
            self.k.pack_cast(jobs, self._pack_total)
            return
        self._pack_torch()
        if self.p.flat.is_cuda:
            self._build_pack_jobs()

    def _pack_job_pairs(self):
        """(destination view, fp32 source view[, scale]) of every layout pack() maintains."""
        p, E, H, A, pk, f32 = self.p, self.E, self.H, self.A, self.pk, self.f32
        M, K, W = p[LIN_M], p[CELL_K], self._wcomb
        pairs = [(pk["emb"], p[EMB])]
        for layer in range(self.L):
            din = E if layer == 0 else A
            for di, d in enumerate(("fw", "bw")):
                Kd = p[enc_k(layer, d)]
                pairs += [(pk[f"enc{layer}_Kx{di}"], Kd[:din]),
                          (pk[f"enc{layer}_Kxi{di}"].view(din, H, 4), Kd[:din].view(din, 4, H).permute(0, 2, 1)),
                          (pk[f"enc{layer}_KxiT{di}"].view(H, 4, din), Kd[:din].view(din, 4, H).permute(2, 1, 0)),
                          (pk[f"enc{layer}_Wn"][di], Kd[din:]), (pk[f"enc{layer}_Wt"][di], Kd[din:].t()),
                          (f32[f"enc{layer}_b"][di], p[enc_b(layer, d)])]
                if layer > 0:
                    pairs.append((pk[f"enc{layer}_Kx01"][:, di * 4 * H:(di + 1) * 4 * H], Kd[:din]))
        pairs += [(pk["Wh"], p[WH].reshape(A, A)),
                  (pk["WhK"], p[WH].reshape(A, A), K2LOG2E), (pk["WhKT"], p[WH].reshape(A, A).t(), K2LOG2E),
                  (pk["lin_embT"], M[:E].t()),
                  (pk["RC"], p[RC]), (pk["RH"], p[RH]), (pk["RCt"], p[RC].t()),
                  (pk["RHt"], p[RH].t()), (pk["lin_emb"], M[:E]), (pk["Wic"], M[E:]), (pk["WicT"], M[E:].t()),
                  (pk["cell_x"], K[:E]), (pk["KcT"], K.t()), (pk["WcT2"][:, :A], W.t()), (pk["WcT2"][:, A:], K[E:].t()),
                  (pk["Wbig"][:E + H], K), (pk["Wbig"][E + H:], W), (pk["Ws"], p[ATT_M]), (pk["WsT"], p[ATT_M].t()),
                  (pk["OUTm"], p[OUT_M]), (pk["OUTmT"], p[OUT_M].t()), (pk["ow"], p[OW]), (pk["ovb"], p[OV])]
        if "owT" in pk:
            pairs.append((pk["owT"], p[OW].t()))
        return pairs

    def _build_pack_jobs(self):
        """The pack_cast job table (pack.hip): per layout its kind -- contiguous copy (2048
        elements per workgroup), transpose of a contiguous matrix (64 x 64 tiles) or generic
        strided (256) -- and its first workgroup."""
        E = self.E
        self._wcomb = torch.mm(self.p[LIN_M][E:], self.p[CELL_K][:E])
        rows, blk = [], 0
        for dst, src, *scale in self._pack_job_pairs():
            assert dst.shape == src.shape and src.dtype == F32 and dst.dtype in (BF, F32) and dst.dim() <= 3, \
                (dst.shape, src.shape)
            shape = [1] * (3 - dst.dim()) + list(dst.shape)
            ss = [0] * (3 - src.dim()) + list(src.stride())
            ts = [0] * (3 - dst.dim()) + list(dst.stride())
            n = dst.numel()
            if dst.is_contiguous() and src.is_contiguous() and src.data_ptr() % 32 == 0 and dst.data_ptr() % 16 == 0:
                kind, nblk = 1, -(-n // 2048)
            elif (dst.dim() == 2 and dst.is_contiguous() and src.stride() == (1, src.shape[0])):
                R, C = dst.shape  # src = the transpose view of a contiguous [C][R] matrix
                kind, nblk = 2, -(-R // 64) * -(-C // 64)
            elif (dst.dim() == 2 and dst.stride(1) == 1 and src.stride(1) == 1 and dst.shape[1] % 8 == 0
                  and dst.stride(0) % 8 == 0 and src.stride(0) % 4 == 0 and src.data_ptr() % 16 == 0
                  and dst.data_ptr() % 16 == 0):
                kind, nblk = 3, -(-n // 2048)  # row-strided rows (e.g. the [H][Vp] padded W): 8 per thread
            else:
                kind, nblk = 0, -(-n // 256)
            sc = int(np.array(scale[0], dtype=np.float32).view(np.int32)) if scale else 0  # fp32 bits, 0 = 1.0
            rows.append([src.data_ptr(), dst.data_ptr(), *shape, *ss, *ts, blk, kind, int(dst.dtype == F32), n, sc])
            blk += nblk
        if len(rows) > int(self.k.pack_max_jobs()) or len(rows[0]) != int(self.k.pack_job_cols()):
            return  # keep the torch path
        self._pack_jobs = torch.tensor(rows, dtype=torch.long, device=self.dev)
        self._pack_total = blk

    def _pack_torch(self):
        p, E, H, A = self.p, self.E, self.H, self.A
        pk = getattr(self, "pk", None) or {}

        def put(name, t):
            t = t.to(BF)
            if name in pk and pk[name].shape == t.shape:
                pk[name].copy_(t)
            else:
                pk[name] = t.contiguous()

        put("emb", p[EMB])
        for layer in range(self.L):
            din = E if layer == 0 else A
            for di, d in enumerate(("fw", "bw")):
                K = p[enc_k(layer, d)]
                put(f"enc{layer}_Kx{di}", K[:din])
                # forward copy with gate-interleaved columns (u*4 + g): the x.W_x GEMM then
                # writes gx as [T][B][H][4], one 16-byte load per (row, unit) in the recurrence
                put(f"enc{layer}_Kxi{di}", K[:din].reshape(din, 4, self.H).transpose(1, 2).reshape(din, 4 * self.H))
                # its [4H][din] twin: the "Bt" operand of the hand-written gather GEMM (gemm_mfma.hip)
                put(f"enc{layer}_KxiT{di}", K[:din].reshape(din, 4, self.H).permute(2, 1, 0).reshape(4 * self.H, din))
            if layer > 0:  # [Kx_fw | Kx_bw] ([din][8H]): the "Bt" operand of the merged input-gradient GEMM
                put(f"enc{layer}_Kx01", torch.cat([p[enc_k(layer, d)][:din] for d in ("fw", "bw")], 1))
            Kh = torch.stack([p[enc_k(layer, d)][din:] for d in ("fw", "bw")])  # [2][H][4H]
            put(f"enc{layer}_Wn", Kh)
            put(f"enc{layer}_Wt", Kh.transpose(1, 2))
        put("Wh", p[WH].reshape(A, A))
        # W_h * 2 log2(e): the F GEMM's operand -- F is stored pre-scaled for the attention
        # kernels' score arguments (attn_common.h fadd_bf2); Wh / WhT stay for dE = dF . W_h^T
        put("WhK", p[WH].reshape(A, A) * K2LOG2E)
        put("WhKT", p[WH].reshape(A, A).t() * K2LOG2E)
        put("RC", p[RC])
        put("RH", p[RH])
        put("RCt", p[RC].t())  # [H][2H]: "Bt" operand of the fused reduce_states forward
        put("RHt", p[RH].t())
        M = p[LIN_M]
        put("lin_emb", M[:E])
        put("lin_embT", M[:E].t())
        put("Wic", M[E:])
        put("WicT", M[E:].t())
        K = p[CELL_K]
        Wcomb = M[E:] @ K[:E]                      # [A][4H]: ctx_{t-1} -> z through x_t
        put("cell_x", K[:E])
        put("KcT", K.t())  # [4H][E+H]: the cell weights of the projected-context recurrence
        put("WcT2", torch.cat([Wcomb, K[E:]], 0).t())  # [4H][A+H]
        put("Wbig", torch.cat([K, Wcomb], 0))          # [E+H+A][4H]
        put("Ws", p[ATT_M])
        put("WsT", p[ATT_M].t())
        put("OUTm", p[OUT_M])
        put("OUTmT", p[OUT_M].t())  # [H][H+A] for the per-step linear2 kernel (decode)
        if getattr(self, "Vp", self.V) != self.V and "owP" not in pk:
            # [H][Vp], zero past V: the K operand of the padded dX GEMM; "ow" is its [:, :V] view
            pk["owP"] = torch.zeros(H, self.Vp, dtype=BF, device=p[OW].device)
            pk["ow"] = pk["owP"][:, :self.V]
        put("ow", p[OW])
        put("ovb", p[OV])  # bias of the bf16 logits GEMM epilogue
        if getattr(self, "fused_vocab", False):
            put("owT", p[OW].t())  # [V][H] B operand of the fused vocab head
        self.pk = pk
        f32 = getattr(self, "f32", None) or {}
        f32["v"] = p[VATT].reshape(A).contiguous()
        f32["wc"] = p[WCOV].reshape(A).contiguous() if self.hps.coverage else None
        # encoder gate biases [fw; bw] (added inside the LSTM kernels; the x.W_x GEMM is
        # bias-free): persistent buffers refreshed in place, captured graphs keep their address
        for layer in range(self.L):
            bb = torch.stack([p[enc_b(layer, d)] for d in ("fw", "bw")])
            key = f"enc{layer}_b"
            if key in f32:
                f32[key].copy_(bb)
            else:
                f32[key] = bb
        self.f32 = f32

    # ------------------------------------------------------------------ inputs
    def set_batch(self, batch) -> None:
        """Host batch -> static device buffers: one H2D copy of a pinned pack.  A batch from
        the multi-process loader (data/loader.py) arrives with ``host_pack`` already built
        by a worker process; otherwise it is built here."""
        B, T = self.B, self.T
        if batch.enc_batch.shape != (B, T):
            raise ValueError(f"batch enc shape {batch.enc_batch.shape} != engine shape {(B, T)}")
        packed = getattr(batch, "host_pack", None)  # bytes in input_layout order, or None
        i = self._in_i
        if self._in_ev[i] is not None:
            self._in_ev[i].synchronize()  # the copy out of this pack (two batches ago) is done
        hn = self._in_host[i].numpy()
        if packed is not None:
            if len(packed) != hn.nbytes:
                raise ValueError(f"host pack of {len(packed)} bytes, engine expects {hn.nbytes}")
            hn[:] = np.frombuffer(packed, dtype=np.uint8)
        else:
            pack_host_inputs(host_inputs(batch, self.hps, self.D, sort_rows=self.skip_pad,
                                         need_grad=getattr(self.hps, "mode", "train") != "decode"), self._in_layout, hn)
        if self.compact_vocab:  # this batch's live vocab-head blocks -> the head's block-count bucket
            o = self._in_off["vblk_n"]
            nlive = int(np.frombuffer(hn, dtype=np.int32, count=1, offset=o)[0])
            self.nbk = next(b for b in self.vocab_buckets if b >= nlive)
        cur = torch.cuda.current_stream()
        cs = self._copy_stream
        with torch.cuda.stream(cs):
            if self._in_used[i] is not None:
                cs.wait_event(self._in_used[i])  # staging i was copied into the inputs two batches ago
            self._in_stage[i].copy_(self._in_host[i], non_blocking=True)
            h2d = torch.cuda.Event()
            h2d.record(cs)
        self._in_ev[i] = h2d
        cur.wait_event(h2d)
        self._in_pack.copy_(self._in_stage[i], non_blocking=True)
        used = torch.cuda.Event()
        used.record(cur)
        self._in_used[i] = used
        self._in_i = i ^ 1

    # ------------------------------------------------------------------ forward
    def _frame_gemm_bt(self, layer: int) -> bool:
        """The input projection of encoder layer ``layer`` through the hand-written gather GEMM
        (its A rows read through the step frame: no to_step_frame pass) -- by TSAMD_GEMM_BT, timed
        once per shape against the library GEMM alone (``FRAME_SLACK``: the gather path also saves
        the layout pass)."""
        st = self.enc[layer]
        din, TB, G = st["din"], self.T * self.B, 4 * self.H
        Bt, xs = self.pk[f"enc{layer}_KxiT0"], st["x_sf"][0].view(TB, din)
        return _use_bt(st["gx"][0].view(TB, G), xs, False, Bt, 0.0, None, self.pk[f"enc{layer}_Kxi0"], False,
                       slack=FRAME_SLACK)

    def _encoder_forward(self, need_grad: bool = True):
        k, w, B, T, H, A = self.k, self.w, self.B, self.T, self.H, self.A
        lens, rev = w["enc_lens"], w["rev_idx"]
        x = None
        for layer, st in enumerate(self.enc):
            din = st["din"]
            xs = st["x_sf"]
            if self.lstm_fx and layer == 0:
                # x.W_x inside the recurrence: only the step-frame gather of the embeddings here
                k.to_step_frame(self.pk["emb"], w["enc_batch"], rev, xs, B, T, din, 0)
                st["hs"][:, 0].zero_()
                st["cs"][:, 0].zero_()
                w["lstm_xf"].zero_()  # hand-off tags must start at 0 every launch
                k.lstm_fwd_persistent_fx(xs, self.pk["enc0_KxiT0"], self.pk["enc0_KxiT1"], self.f32["enc0_b"],
                                         self.pk["enc0_Wt"], st["hs"], st["cs"], st["acts"], st["out"], lens,
                                         w["lstm_xf"], w["lstm_err"], T, B, H)
                x = st["out"]
                continue
            if self._frame_gemm_bt(layer):
                # x.W_x with the A rows gathered through the step frame inside the GEMM (layer 0
                # straight from the embedding table by token id); the gathered rows are also
                # stored to x_sf for the weight gradient (need_grad only)
                src = self.pk["emb"] if x is None else x.view(B * T, din)
                ids = w["enc_batch"] if x is None else None
                for di in range(2):
                    k.gemm_bt(src, self.pk[f"enc{layer}_KxiT{di}"], st["gx"][di].view(T * B, 4 * H), 0.0, None, ids,
                              rev, B, T, di, xs[di].view(T * B, din) if need_grad else None)
            else:
                # step-frame inputs [2][T][B][din] (bw reversed within each length) in one gather
                # launch: layer 0 straight from the embedding table by token id (frames.hip)
                if x is None:
                    k.to_step_frame(self.pk["emb"], w["enc_batch"], rev, xs, B, T, din, 0)
                else:
                    k.to_step_frame(x, None, rev, xs, B, T, din, 0)
                for di in range(2):  # x.W_x, bias added in the recurrence kernel
                    mm_into(st["gx"][di].view(T * B, 4 * H), xs[di].view(T * B, din), self.pk[f"enc{layer}_Kxi{di}"])
            st["hs"][:, 0].zero_()
            st["cs"][:, 0].zero_()
            if not self.persistent_lstm:  # (the persistent kernels write zeros past each length)
                st["out"].zero_()
            if self.persistent_lstm:
                w["lstm_xf"].zero_()  # hand-off tags must start at 0 every launch
                k.lstm_fwd_persistent(st["gx"], self.f32[f"enc{layer}_b"], self.pk[f"enc{layer}_Wt"], st["hs"], st["cs"], st["acts"], st["out"],
                                      lens, w["lstm_xf"], w["lstm_err"], T, B, H)
            else:
                for s in range(T):
                    k.lstm_enc_fwd_step(st["gx"], self.f32[f"enc{layer}_b"], self.pk[f"enc{layer}_Wt"], st["hs"], st["cs"], st["acts"],
                                        st["out"], lens, s, T, B, H)
            x = st["out"]
        top = self.enc[-1]
        # reduce_states: [c_fw, c_bw] / [h_fw, h_bw] -> relu(. W + b) -> the decoder's initial
        # state, one launch (reduce_states.hip) reading the encoder's final states in place
        k.rs_fwd(top["cs"], top["hs"], T, self.pk["RCt"], self.pk["RHt"], self.p[BRC], self.p[BRH], w["rs_pre"][0],
                 w["rs_pre"][1], w["Cst"][0], w["Cb"][0], w["Hb"][0], w["rs_cat"][0], w["rs_cat"][1], B, H)
        # F = enc_out . W_h * 2 log2(e) (stored pre-scaled: attn_common.h)
        mm_into(w["F"].view(B * T, A), top["out"].view(B * T, A), self.pk["WhK"], bt=self.pk["WhKT"])
        if self.proj_attn:
            mm_into(w["Genc"].view(B * T, self.E), top["out"].view(B * T, A), self.pk["Wic"], bt=self.pk["WicT"])
        if self.keep_ft:
            if w["Ft"] is None:
                w["Ft"] = torch.empty(B, A, T, dtype=BF, device=self.dev)
            k.transpose_bta(w["F"], w["Ft"], B, T, A)

    def _decoder_forward(self):
        k, w, hps = self.k, self.w, self.hps
        B, T, D, E, H, A = self.B, self.T, self.D, self.E, self.H, self.A
        cov = hps.coverage
        emb_dec = self.pk["emb"][w["dec_batch_t"]].view(D * B, E)
        xe = w["xe"].view(D * B, E)
        mm_into(xe, emb_dec, self.pk["lin_emb"], self.p[LIN_B], bt=self.pk["lin_embT"])
        mm_into(w["XG"].view(D * B, 4 * H), xe.to(BF), self.pk["cell_x"], self.p[CELL_B], bt=self.pk["KcT"][:, :E])
        self._emb_dec = emb_dec
        enc_out, lens, Ft, F = self.enc[-1]["out"], w["enc_lens"], w["Ft"], w["F"]
        v, wc = self.f32["v"], self.f32["wc"]

        if self.proj_attn:
            return self._decoder_forward_proj()

        def chain(r0, r1):
            Bg, rs = r1 - r0, slice(r0, r1)
            for t in range(D):
                k.dec_cell_fwd(w["XG"][t][rs], w["CTXb"][t - 1][rs] if t > 0 else None, w["Hb"][t][rs],
                               w["Cst"][t][rs], self.pk["WcT2"], w["Cst"][t + 1][rs], w["Cb"][t + 1][rs],
                               w["Hb"][t + 1][rs], w["ACT"][t][rs], Bg, H, A, None, 0)
                cov_in = w["COV"][t][rs] if (cov and t > 0) else None
                k.dec_sproj(w["Cb"][t + 1][rs], w["Hb"][t + 1][rs], self.pk["WsT"], self.p[ATT_B], w["S"][t][rs], Bg,
                            H, A, None, 0)
                if self.row_attn:
                    k.attn_fwd_row(F[rs], enc_out[rs], w["S"][t][rs], v, wc, cov_in, lens[rs], w["ATT"][t][rs],
                                   w["COV"][t + 1][rs] if cov else None, w["covloss"][t][rs] if cov else None,
                                   w["CTX"][t][rs], w["CTXb"][t][rs], Bg, T, A, 1)
                    continue
                k.attn_score(Ft[rs], w["S"][t][rs], v, wc, cov_in, lens[rs], w["e"][rs], Bg, T, A, 1)
                k.attn_softmax_ctx(w["e"][rs], enc_out[rs], lens[rs], cov_in, w["ATT"][t][rs],
                                   w["COV"][t + 1][rs] if cov else None, w["covloss"][t][rs] if cov else None,
                                   w["CTX"][t][rs], w["CTXb"][t][rs], Bg, T, A, 1)

        self._row_groups(chain)
        # x_t = xe_t + ctx_{t-1} . W_in[E:]  (rebuilt after the loop, one GEMM)
        w["X"].copy_(w["xe"])
        if D > 1:
            w["X"][1:].view((D - 1) * B, E).add_(mmf(w["CTXb"][:D - 1].reshape((D - 1) * B, A), self.pk["Wic"]))
        w["Xb"].copy_(w["X"])

    def _decoder_forward_proj(self):
        """Decoder forward loop with the projected context: per step the cell (its ctx input is
        g_{t-1}, E wide, against W_cell^T), the s-projection and attn_fwd_rowp (F and G); then
        x_t = xe_t + g_{t-1} and ctx_t = a_t . enc_out for all steps as one batched GEMM."""
        k, w, hps = self.k, self.w, self.hps
        B, T, D, E, H, A = self.B, self.T, self.D, self.E, self.H, self.A
        cov = hps.coverage
        enc_out, lens, F, G = self.enc[-1]["out"], w["enc_lens"], w["F"], w["Genc"]
        v, wc = self.f32["v"], self.f32["wc"]
        dlen = w["dlen"] if self.skip_pad else None

        def chain(r0, r1):
            Bg, rs = r1 - r0, slice(r0, r1)
            dl = dlen[rs] if dlen is not None else None
            for t in range(D):
                k.dec_cell_fwd(w["XG"][t][rs], w["GVb"][t - 1][rs] if t > 0 else None, w["Hb"][t][rs],
                               w["Cst"][t][rs], self.pk["KcT"], w["Cst"][t + 1][rs], w["Cb"][t + 1][rs],
                               w["Hb"][t + 1][rs], w["ACT"][t][rs], Bg, H, E, dl, t)
                k.dec_sproj(w["Cb"][t + 1][rs], w["Hb"][t + 1][rs], self.pk["WsT"], self.p[ATT_B], w["S"][t][rs], Bg,
                            H, A, dl, t)
                k.attn_fwd_rowp(F[rs], G[rs], w["S"][t][rs], v, wc, w["COV"][t][rs] if (cov and t > 0) else None,
                                lens[rs], w["ATT"][t][rs], w["COV"][t + 1][rs] if cov else None,
                                w["covloss"][t][rs] if cov else None, w["GV"][t][rs], w["GVb"][t][rs], Bg, T, A,
                                dl, t, w["ATTb"][t][rs])

        self._row_groups(chain)
        w["X"][0].copy_(w["xe"][0])
        if D > 1:
            torch.add(w["xe"][1:], w["GV"][:D - 1], out=w["X"][1:])
        w["Xb"].copy_(w["X"])
        # ctx_t = a_t . enc_out for every step: [B][D, T] x [B][T, A] (bf16 a -- written by the
        # attention kernel next to the fp32 a -- fp32 accumulate) into the step-major CTX [D][B][A]
        # and its bf16 twin: one ctx_bmm.hip launch, or torch.bmm + the tr01 layout pass
        if self.ctx_native:
            self.k.ctx_fwd(w["ATTb"], enc_out, w["CTX"], w["CTXb"], B, T, D, A)
            return
        ctx = w["bd_tmp"][:B * D * A].view(B, D, A)
        torch.bmm(w["ATTb"].permute(1, 0, 2), enc_out, out_dtype=F32, out=ctx)
        self.k.tr01(ctx, w["CTX"], w["CTXb"], B, D, A, False)

    def _head_forward(self, need_grad: bool):
        w, hps, p = self.w, self.hps, self.p
        B, T, D, E, H, A, V = self.B, self.T, self.D, self.E, self.H, self.A, self.V
        N = D * B
        Hn = w["Hb"][1:].reshape(N, H)
        ctxb = w["CTXb"].view(N, A)
        # out = [h, ctx] . W_o + b: bias-epilogue GEMM, second GEMM accumulating (beta = 1)
        out = w["out_f32"]
        gemm(out, Hn, self.pk["OUTm"][:H], 0.0, p[OUT_B], bt=self.pk["OUTmT"][:, :H])
        gemm(out, ctxb, self.pk["OUTm"][H:], 1.0, bt=self.pk["OUTmT"][:, H:])
        w["outb"].copy_(out)
        pg = None
        if hps.pointer_gen:
            # p_gen = sigmoid([ctx, c, h, x] . w + b) for all D*B rows, one wave per row (decoder.hip)
            self.k.pgen(w["CTX"].view(N, A), w["Cst"][1:].reshape(N, H), Hn, w["X"].view(N, E), p[PG_M].view(-1),
                        p[PG_B], w["pg"].view(N), N, A, H, E)
            pg = w["pg"]
        if self.fused_vocab:
            k, ldx = self.k, H + 8  # outb is the first H columns of outb_ext
            # skip_pad: only the 32-row blocks holding a live row are enumerated (host-built list)
            vb, vn = (w["vblk"], w["vblk_n"]) if self.skip_pad else (None, None)
            k.vocab_train_fwd(w["outb_ext"], self.pk["owT"], p[OV], w["target_t"], w["vpart"], w["zg"], w["lse"],
                              w["pv"], N, V, H, ldx, vb, vn)
            k.ptr_rowfin(w["pv"], w["target_t"], w["rowg"], pg, w["ATT"] if hps.pointer_gen else None, w["ext"],
                         w["enc_lens"], w["loss_row"], w["alpha"] if need_grad else None,
                         w["dpre"] if (need_grad and hps.pointer_gen) else None,
                         w["dA"] if (need_grad and hps.pointer_gen) else None, N, B, T)
            if need_grad:
                w["dbias"].zero_()
                inplace = vb is not None and not self.compact_vocab  # else compacted (or every block)
                k.vocab_train_bwd(w["outb_ext"], self.pk["owT"], p[OV], w["target_t"], w["lse"], w["alpha"],
                                  w["dlogits"], None if self.det else w["dbias"], N, V, H, ldx, vb, vn,
                                  w["vlive"] if inplace else None, w["vstate"] if inplace else None)
                if self.det:  # column sums of the bf16 dlogits in a fixed order
                    if self.Vp != V:
                        k.colsum(w["dlogits"], w["dbias_p"], N, self.Vp, False)
                        w["dbias"].copy_(w["dbias_p"][:V])
                    else:
                        k.colsum(w["dlogits"], w["dbias"], N, V, False)
            return
        gemm(w["logits"], w["outb"], self.pk["ow"], 0.0, self.pk["ovb"])
        self.k.ptr_loss(w["logits"], None, w["target_t"], w["rowg"], pg, w["ATT"] if hps.pointer_gen else None,
                        w["ext"], w["enc_lens"], w["loss_row"], w["dlogits"] if need_grad else None,
                        w["dpre"] if (need_grad and hps.pointer_gen) else None,
                        w["dA"] if (need_grad and hps.pointer_gen) else None, N, B, T, V)

    def _row_groups(self, chain, split=None):
        """Run ``chain(r0, r1)`` for every row group (``split`` groups, default self.split):
        inline when split == 1, else each group on its own stream, forked from and joined back
        to the current stream."""
        n = self.split if split is None else split
        if n == 1:
            return chain(0, self.B)
        cur = torch.cuda.current_stream()
        rows = [(self.B * g // n, self.B * (g + 1) // n) for g in range(n)]
        for st, (r0, r1) in zip(self._streams, rows):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                chain(r0, r1)
        for st in self._streams[:n]:
            cur.wait_stream(st)

    def forward(self, need_grad: bool = False):
        self._encoder_forward(need_grad)
        self._decoder_forward()
        self._head_forward(need_grad)
        return self.losses()

    def losses(self):
        w, hps = self.w, self.hps
        loss = (w["loss_row"] * w["rowg"]).sum()
        out = {"loss": loss}
        if hps.coverage:
            covl = (w["covloss"] * w["gcl"]).sum() / hps.cov_loss_wt if hps.cov_loss_wt else w["covloss"].sum() * 0
            out["coverage_loss"] = covl
            out["total_loss"] = loss + hps.cov_loss_wt * covl
        else:
            out["total_loss"] = loss
        return out

    # ------------------------------------------------------------------ backward
    # The backward runs in four phases so a data-parallel trainer can all-reduce each
    # phase's gradient bucket while the next phase computes (the flat gradient is laid out
    # in this order: output_projection | decoder + attention | reduce_states + encoder | emb).
    # The embedding (25.6 MB at V = 50k) is its own last bucket, so the only all-reduce left
    # after the last kernel is the embedding's.
    PHASE_FIRST_PARAM = (f"{DEC}/AttnOutputProjection/Linear/Matrix", f"{P}/reduce_final_st/w_reduce_c", EMB)

    def phase_bounds(self):
        return [self.p.offsets[n][0] for n in self.PHASE_FIRST_PARAM]

    def backward(self):
        self.backward_head()
        self.backward_head_dw()
        self.backward_mid()
        self.backward_tail()

    def backward_tail(self):
        """reduce_states, encoder BPTT, encoder weights (bucket 2), embedding (bucket 3)."""
        self.backward_tail_enc()
        self.backward_tail_emb()

    def backward_head(self):
        """Vocab projection gradients (the 51 MB output_projection bucket)."""
        w, p = self.w, self.p
        g = p.g
        p.grad.zero_()
        dl = w["dlogits"]
        H, V = self.H, self.V
        if self.fused_vocab:
            # the bias gradient came out of the fused kernel; the weight GEMM keeps M = H (an
            # M = H + 1 problem runs twice the output tiles on hipBLASLt's 256-row tiles)
            m, dst = H, g(OW)
            g(OV).copy_(w["dbias"])
        else:
            # [W | b] gradient in one GEMM: output_projection/w and /v are adjacent in the flat
            # buffer, and row H of outb_ext is all ones
            assert p.offsets[OV][0] == p.offsets[OW][0] + H * V
            o = p.offsets[OW][0]
            m, dst = H + 1, p.grad[o:o + (H + 1) * V].view(H + 1, V)
        N = self.D * self.B
        if self.compact_vocab:
            return self._backward_head_compact(g, dl, H, V, N)
        if self.Vp != V:  # padded dlogits rows (fused head, m == H)
            self._dw_job(lambda: self._vocab_dw(dst, w["outb_ext"][:, :H], dl))
            self._dout = self._vocab_dx(dl)
            return

        def dw():
            Sw = 4
            # keep the batched operand's batch stride (N / Sw rows of dlogits) below 2^31
            # elements: the library's strided-batched path is not trusted past 32-bit strides
            while Sw > 1 and (N // Sw) * V >= 2 ** 31 and N % (2 * Sw) == 0:
                Sw *= 2
            if not BLT_VDW and m == H and Sw > 1 and N % Sw == 0 and (N // Sw) * V < 2 ** 31:
                # split K = N in Sw = 4 (one batched GEMM + a sum): 0.82 -> 0.74 ms at B = 256
                xe = w["outb_ext"].view(Sw, N // Sw, H + 8)[:, :, :H]
                parts = torch.bmm(xe.transpose(1, 2), dl.view(Sw, N // Sw, V), out_dtype=F32)
                torch.sum(parts, 0, out=dst)
            else:
                gemm(dst, w["outb_ext"][:, :m].t(), dl)
        dw()
        # dX = dlogits . W^T unsplit (split-K over vocab chunks measured slower at B = 256:
        # profiles/r2/ab/vocab_grad_split.jsonl)
        self._dout = mmf(dl, self.pk["ow"].t())  # [N,H]

    def _backward_head_compact(self, g, dl, H, V, N):
        """Vocab gradients over the live rows only: pass 2 wrote live block j's dlogits to rows
        32 j .. 32 j + 31; the GEMMs run over nbk blocks (the batch's bucket, >= its live block count;
        the padding gathers the all-zero dummy block nb of outb_ext, so the stale dlogits rows past the
        live ones contribute exact zeros to dW) and dX is scattered back to the t-major rows (dead
        rows: dlogits 0, so dX 0).  Same sums as the full GEMMs up to the split-K order."""
        w = self.w
        nbk, M = self.nbk, self.nbk * 32
        nb = (N + 31) // 32
        idx = w["vblk"][:nbk].long()
        ob = w["outb_blk"].view(nb + 1, 32, H + 8)
        if not hasattr(self, "_outb_c"):
            self._outb_c = torch.zeros(nb * 32, H + 8, dtype=BF, device=self.dev)
            self._dout_ext = torch.zeros(nb + 1, 32, H, dtype=F32, device=self.dev)
        xc = self._outb_c[:M]
        torch.index_select(ob, 0, idx, out=xc.view(nbk, 32, H + 8))
        dlc = dl[:M]
        g(OV).copy_(w["dbias"])
        dst = g(OW)
        if self.Vp != V:
            self._dw_job(lambda: self._vocab_dw(dst, xc[:, :H], dlc))
            dxc = self._vocab_dx(dlc)
        else:
            dxc = self._vocab_grads_unpadded(dst, xc, dlc, H, V, M)
        de = self._dout_ext
        de.zero_()
        de.index_copy_(0, idx, dxc.view(nbk, 32, H))  # padding entries land in the dummy block nb
        self._dout = de[:nb].view(nb * 32, H)[:N]

    def _vocab_grads_unpadded(self, dst, xc, dlc, H, V, M):
        Sw = 4 if not BLT_VDW and M % 4 == 0 and (M // 4) * V < 2 ** 31 else 1
        if Sw > 1:  # split K = M in 4 (one batched GEMM + a sum), as the full head
            parts = torch.bmm(xc.view(Sw, M // Sw, H + 8)[:, :, :H].transpose(1, 2), dlc.view(Sw, M // Sw, V),
                              out_dtype=F32)
            torch.sum(parts, 0, out=dst)
        else:
            gemm(dst, xc[:, :H].t(), dlc)
        return mmf(dlc, self.pk["ow"].t())  # [M, H]

    def _dw_job(self, f):
        """Run the vocab dW now, or -- split_vocab_dw, set by the graph trainer -- keep it for
        backward_head_dw (its own graph, replayed beside the decoder backward loop)."""
        if self.split_vocab_dw:
            self._pending_dw = f
        else:
            f()

    def backward_head_dw(self):
        """The vocab dW left pending by the last backward_head (split_vocab_dw); else nothing."""
        f, self._pending_dw = self._pending_dw, None
        if f is not None:
            f()

    def _vocab_dw(self, dst, x, dl):
        """dst[H][V] = x^T . dl[:, :V] (output-projection weight gradient, model.py:290-297 over
        model.py:229-236) from the padded dlogits rows dl [K][Vp]: the library GEMM at the aligned
        N into a [H][Vp] scratch, then the first V columns; above VOCAB_DW_SPLIT_MIN the 4-way
        split-K batched GEMM (+ ordered torch.sum) as before."""
        K, H, V, Vp = dl.shape[0], self.H, self.V, self.Vp
        if not BLT_VDW and K * H * V >= VOCAB_DW_SPLIT_MIN and K % 4 == 0 and (K // 4) * Vp < 2 ** 31:
            parts = torch.bmm(x.unflatten(0, (4, K // 4)).transpose(1, 2), dl.view(4, K // 4, Vp), out_dtype=F32)
            torch.sum(parts[:, :, :V], 0, out=dst)
            return
        if getattr(self, "_dWp", None) is None:
            self._dWp = torch.empty(H, Vp, dtype=F32, device=self.dev)
        gemm(self._dWp, x.t(), dl)
        dst.copy_(self._dWp[:, :V])

    def _vocab_dx(self, dl):
        """dlogits . W^T [K][H] fp32 (the output-projection input gradient) from the padded dlogits
        rows and the padded bf16 W [H][Vp]: the hand-written split-K GEMM (gemm_bt + ordered slab
        sum: deterministic) where the output is a few tiles, else the library GEMM."""
        K, H, Vp = dl.shape[0], self.H, self.Vp
        out = torch.empty(K, H, dtype=F32, device=self.dev)
        ow = self.pk["owP"]
        if dl.is_cuda and GEMM_BT != "0":
            k = self.k
            n = int(k.gemm_bt_splitk_ws(K, H, Vp))
            if n > 0:
                ws = getattr(self, "_vdx_ws", None)
                if ws is None or ws.numel() < n:
                    if torch.cuda.is_current_stream_capturing():
                        ws = None  # first seen inside a capture: no allocation there
                    else:
                        old = getattr(self, "_vdx_ws_old", [])
                        if ws is not None:
                            old.append(ws)  # graphs captured earlier may hold it
                        self._vdx_ws_old = old
                        ws = self._vdx_ws = torch.empty(n, dtype=F32, device=self.dev)
                if ws is not None and k.gemm_bt_splitk(dl, ow, out, ws, False):
                    return out
        return gemm(out, dl, ow.t())

    def _cast_colsum(self, x, bias_grad):
        """bf16 copy of x [N, C] plus bias_grad += its column sums in one read of x (the
        cast_colsum kernel; bias_grad lies in the gradient buffer, zeroed by backward_head)."""
        N, C = x.shape
        xb = torch.empty(N, C, dtype=BF, device=x.device)
        if C % 4 == 0 and C // 4 <= 256 and 256 % (C // 4) == 0:
            self.k.cast_colsum(x, xb, bias_grad, N, C)
        else:
            xb.copy_(x)
            self.k.colsum(x, bias_grad, N, C, False)
        return xb

    def backward_mid(self):
        """Output projection, p_gen, decoder reverse loop, decoder/attention weight grads."""
        k, w, hps, p = self.k, self.w, self.hps, self.p
        B, T, D, E, H, A, V = self.B, self.T, self.D, self.E, self.H, self.A, self.V
        N = D * B
        g = p.g
        cov = hps.coverage
        dout = self._dout
        # ---- output projection [h, ctx]
        Hn = w["Hb"][1:].reshape(N, H)
        ctxb = w["CTXb"].view(N, A)
        doutb = self._cast_colsum(dout, g(OUT_B))
        late = self._late = []  # deferred weight gradients (see defer_wgrad)
        run = late.append if self.defer_wgrad else (lambda f: f())
        # the deferred ones go through wgrad_tn (wgrad.hip: no inter-workgroup waits) into the
        # zeroed gradient slices; inline, the library split-K path
        # inline (config #5's batch 2048, deterministic mode): the large shapes on wgrad_tt
        wg = (lambda out, a, b: k.wgrad_tn(a, b, out)) if self.defer_wgrad else wgrad_enc_into

        def out_proj_wgrad():
            wg(g(OUT_M)[:H], Hn, doutb)
            wg(g(OUT_M)[H:], ctxb, doutb)
        run(out_proj_wgrad)
        dH_dir = mmf(doutb, self.pk["OUTm"][:H].t()).view(D, B, H)
        if self.proj_attn:  # DCTX itself: the loop adds nothing per step, the post-loop GEMM accumulates into it
            mm_into(w["DCTX"].view(N, A), doutb, self.pk["OUTm"][H:].t())
            dCTX_dir = w["DCTX"]
        else:
            dCTX_dir = mmf(doutb, self.pk["OUTm"][H:].t()).view(D, B, A)
        dC_dir = None
        dX_dir = None
        if hps.pointer_gen:
            dpre = w["dpre"].view(N)
            pm = p[PG_M].view(-1)
            # one fused column-reduction kernel for the four p_gen weight slices (gw zeroed above)
            k.pgen_bwd(w["CTX"].view(N, A), w["Cst"][1:].reshape(N, H), Hn, w["X"].view(N, E), dpre,
                       g(PG_M).view(-1), N, A, H, E, self.det)
            # direct terms dCTX/dH += dp w_ctx/h, dC/dX = dp w_c/x and the bias gradient, one launch
            dC_dir, dX_dir = w["dC_dir"], w["dX_dir"]
            # the p_gen bias gradient sum(dp) by colsum in both modes: pgen_dirs' one same-address atomic per
            # workgroup (6400 at B = 256) serialised at L2 (95 us for a ~40 us kernel, round-3 kernel stats)
            k.pgen_dirs(dpre, pm, dCTX_dir, dC_dir, dH_dir, dX_dir, None, N, A, H, E)
            k.colsum(dpre, g(PG_B).view(1), N, 1, False)
        if self.proj_attn:
            return self._backward_mid_proj(dCTX_dir, dH_dir, dC_dir, dX_dir, Hn, wg, run)
        if dX_dir is not None and D > 1:  # p_gen path into ctx_{t-1} through x_t (hoisted out of the loop)
            gemm(dCTX_dir[:D - 1].view((D - 1) * B, A), dX_dir[1:].view((D - 1) * B, E), p[LIN_M][E:].t(), 1.0)
        # ---- decoder reverse loop
        enc_out, lens, F = self.enc[-1]["out"], w["enc_lens"], w["F"]
        v, wc = self.f32["v"], self.f32["wc"]
        w["DCTX"][D - 1].copy_(dCTX_dir[D - 1])
        w["dh_rec"].zero_()
        w["dc_carry"].zero_()
        dcov = w["dcov"]
        if not self.row_attn_bwd:
            w["DS"].zero_()  # accumulated with atomics by the multi-block kernels (the row kernel stores)
        Ga = w["dA"] if hps.pointer_gen else None
        def chain(r0, r1):
            Bg, rs = r1 - r0, slice(r0, r1)
            for t in reversed(range(D)):
                dcov_next = dcov[(t + 1) % 2][rs] if (cov and t < D - 1) else None
                cov_t = w["COV"][t][rs] if (cov and t > 0) else None
                gcl_t = w["gcl"][t][rs] if cov else None
                ga_t = Ga[t][rs] if Ga is not None else None
                if self.row_attn_bwd:
                    k.attn_bwd_row(enc_out[rs], F[rs], w["S"][t][rs], v, wc, cov_t, w["ATT"][t][rs], w["DCTX"][t][rs],
                                   w["CTX"][t][rs], ga_t, dcov_next, gcl_t, lens[rs], w["DE"][t][rs], w["DS"][t][rs],
                                   dcov[t % 2][rs] if cov else None, Bg, T, A)
                else:
                    k.attn_bwd_step(enc_out[rs], F[rs], w["S"][t][rs], v, wc, cov_t, w["ATT"][t][rs], w["DCTX"][t][rs],
                                    w["CTX"][t][rs], ga_t, dcov_next, gcl_t, lens[rs], w["DE"][t][rs], w["DS"][t][rs],
                                    dcov[t % 2][rs] if cov else None, Bg, T, A)
                k.dec_bwd_cell(w["DS"][t][rs], self.pk["Ws"], dC_dir[t][rs] if dC_dir is not None else None,
                               dH_dir[t][rs], w["dh_rec"][rs], w["dc_carry"][rs], w["ACT"][t][rs], w["Cst"][t + 1][rs],
                               w["Cst"][t][rs], w["DZ"][t][rs], Bg, H, A, None, 0)
                k.dec_bwd_dz(w["DZ"][t][rs], self.pk["Wbig"], dX_dir[t][rs] if dX_dir is not None else None,
                             dCTX_dir[t - 1][rs] if t > 0 else None, w["DX"][t][rs],
                             w["DCTX"][t - 1][rs] if t > 0 else None, w["dh_rec"][rs], Bg, E, H, A, None, 0)

        self._row_groups(chain, self.split_bwd)
        self._backward_mid_rest(Hn, wg, run)

    def _backward_mid_proj(self, dCTX_dir, dH_dir, dC_dir, dX_dir, Hn, wg, run):
        """Decoder reverse loop with the projected context.  Before it, the part of
        da_ti = dctx_t . E_i that does not wait on the recurrence (output projection + p_gen:
        dCTX_dir) as one batched GEMM, added to the pointer-path gradient dA; in it, attn_bwd_rowp
        adds dx_{t+1} . G_i and dec_bwd_dz produces dx_t (no dctx output); after it,
        dctx_t = dCTX_dir_t + dx_{t+1} . W_in[E:]^T for the dE GEMM."""
        k, w, hps = self.k, self.w, self.hps
        B, T, D, E, H, A = self.B, self.T, self.D, self.E, self.H, self.A
        N = D * B
        cov = hps.coverage
        enc_out, lens, F, G = self.enc[-1]["out"], w["enc_lens"], w["F"], w["Genc"]
        v, wc = self.f32["v"], self.f32["wc"]
        w["DCTXb"].copy_(dCTX_dir)
        Ga = w["dA"]  # [D][B][T] (+)= da^T
        if self.ctx_native:  # step-major straight from the kernel (accumulated with pointer_gen)
            k.ctx_da(w["DCTXb"], enc_out, Ga, B, T, D, A, bool(hps.pointer_gen))
        else:
            da = w["bd_tmp"][:B * D * T].view(B, D, T)
            torch.bmm(w["DCTXb"].permute(1, 0, 2), enc_out.transpose(1, 2), out_dtype=F32, out=da)
            if T % 4 == 0:  # one vectorised pass (tr01; T % 4 == 0)
                k.tr01(da, Ga, None, B, D, T, bool(hps.pointer_gen))
            elif hps.pointer_gen:
                Ga.add_(da.transpose(0, 1))
            else:
                Ga.copy_(da.transpose(0, 1))
        w["dh_rec"].zero_()
        w["dc_carry"].zero_()
        dcov = w["dcov"]
        Kc = self.pk["Wbig"][:E + H]  # W_cell: [dx | dh] = dz . W_cell^T
        dlen = w["dlen"] if self.skip_pad else None
        # dec_bwd_dz produces dx_t and dh_rec = dz_t . W_cell[E:]^T at the end of every step (the
        # 2-launch variant with dx in the attention backward's prologue measured slower:
        # profiles/r4/ab/dec_bwd_two_launch.md)

        def chain(r0, r1):
            Bg, rs = r1 - r0, slice(r0, r1)
            dl = dlen[rs] if dlen is not None else None
            for t in reversed(range(D)):
                nxt = t < D - 1
                k.attn_bwd_rowp(G[rs], F[rs], w["S"][t][rs], v, wc, w["COV"][t][rs] if (cov and t > 0) else None,
                                w["ATT"][t][rs], w["DX"][t + 1][rs] if nxt else None, w["GV"][t][rs],
                                Ga[t][rs], dcov[(t + 1) % 2][rs] if (cov and nxt) else None,
                                w["gcl"][t][rs] if cov else None, lens[rs], w["DE"][t][rs], w["DS"][t][rs],
                                dcov[t % 2][rs] if cov else None, Bg, T, A, dl, t)
                k.dec_bwd_cell(w["DS"][t][rs], self.pk["Ws"], dC_dir[t][rs] if dC_dir is not None else None,
                               dH_dir[t][rs], w["dh_rec"][rs], w["dc_carry"][rs], w["ACT"][t][rs], w["Cst"][t + 1][rs],
                               w["Cst"][t][rs], w["DZ"][t][rs], Bg, H, A, dl, t)
                k.dec_bwd_dz(w["DZ"][t][rs], Kc, dX_dir[t][rs] if dX_dir is not None else None, None,
                             w["DX"][t][rs], None, w["dh_rec"][rs], Bg, E, H, 0, dl, t)

        self._row_groups(chain, self.split_bwd)
        if dCTX_dir is not w["DCTX"]:
            w["DCTX"].copy_(dCTX_dir)
        if D > 1:
            dctx = w["DCTX"][:D - 1].view((D - 1) * B, A)
            dxb = w["DXb"][1:].view((D - 1) * B, E)
            dxb.copy_(w["DX"][1:].view((D - 1) * B, E))
            gemm(dctx, dxb, self.pk["WicT"], 1.0, bt=self.pk["Wic"])
        self._backward_mid_rest(Hn, wg, run)

    def _backward_mid_rest(self, Hn, wg, run):
        """Decoder / attention weight gradients, attention feature gradient and dE after the
        decoder reverse loop."""
        k, w, hps, p = self.k, self.w, self.hps, self.p
        B, T, D, E, H, A = self.B, self.T, self.D, self.E, self.H, self.A
        N = D * B
        g = p.g
        cov = hps.coverage
        v, wc = self.f32["v"], self.f32["wc"]
        lens, F = w["enc_lens"], w["F"]
        # ---- decoder weight gradients (one GEMM each over all D*B rows)
        emb_dec = self._emb_dec

        DXb = self._cast_colsum(w["DX"].view(N, E), g(LIN_B))
        gemm(w["d_emb_dec"], DXb, self.pk["lin_emb"].t())  # [N,E] (embedding gradient)

        def dec_wgrad():
            DZ = w["DZ"].view(N, 4 * H)
            gk = g(CELL_K)
            wg(gk[:E], w["Xb"].view(N, E), DZ)
            wg(gk[E:], w["Hb"][:D].reshape(N, H), DZ)
            k.colsum(DZ, g(CELL_B), N, 4 * H, False)
            gl = g(LIN_M)
            wg(gl[:E], emb_dec, DXb)
            gl[E:].zero_()
            if D > 1:
                wg(gl[E:], w["CTXb"][:D - 1].reshape((D - 1) * B, A), DXb[B:])
            DSb = self._cast_colsum(w["DS"].view(N, A), g(ATT_B))
            gs = g(ATT_M)
            wg(gs[:H], w["Cb"][1:].reshape(N, H), DSb)
            wg(gs[H:], Hn, DSb)
        run(dec_wgrad)
        # ---- attention feature gradients (tanh recomputed once over all steps)
        w["dv"].zero_()
        w["dwc"].zero_()
        k.attn_bwd_feat(F, w["S"], v, wc, w["COV"][:D] if cov else None, w["DE"], lens, w["dF"], w["dv"],
                        w["dwc"] if cov else None, D, B, T, A, w["dlen"] if self.skip_pad else None)
        k.colsum(w["dv"], g(VATT).view(A), w["dv"].shape[0], A, False)
        if cov:
            k.colsum(w["dwc"], g(WCOV).view(A), w["dwc"].shape[0], A, False)
        dFb = w["dF"].view(B * T, A)
        top = self.enc[-1]
        run(lambda: wg(g(WH).view(A, A), top["out"].view(B * T, A), dFb))
        dE = self._dE
        # dE = a^T . dctx (bf16 batched GEMM, fp32 out) + dF . W_h^T (accumulated in place)
        if not self.proj_attn:  # (the projected-context forward made ATTb already)
            w["ATTb"].copy_(w["ATT"])
        w["DCTXb"].copy_(w["DCTX"])
        if self.de_bf16:  # bf16 dE: a^T . dctx stored bf16, then += dF . W_h^T (library GEMM, beta = 1)
            k.ctx_de(w["ATTb"], w["DCTXb"], dE, B, T, D, A)
            _ops().blt_mm(dFb, self.pk["Wh"], dE.view(B * T, A), False, True, 1.0, None)
            return
        if self.ctx_native:
            k.ctx_de(w["ATTb"], w["DCTXb"], dE, B, T, D, A)
        else:
            torch.bmm(w["ATTb"].permute(1, 2, 0), w["DCTXb"].permute(1, 0, 2), out_dtype=F32, out=dE)
        dE2 = dE.view(B * T, A)
        gemm(dE2, dFb, self.pk["Wh"].t(), 1.0)

    def backward_tail_enc(self):
        """reduce_states, encoder BPTT and weight gradients; joins the deferred decoder weight
        gradients (buckets 1 and 2 are complete when this phase ends)."""
        k, w, p = self.k, self.w, self.p
        B, T, H = self.B, self.T, self.H
        g = p.g
        dE = self._dE
        lens = w["enc_lens"]
        late, self._late = self._late, []
        if late:  # the deferred decoder weight gradients, beside the encoder BPTT
            side = self._late_stream
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for f in late:
                    f()
        # ---- reduce_states (reduce_states.hip): dp = g [pre > 0], bias gradients, and
        # d[c_fw, c_bw] / d[h_fw, h_bw] written straight into the top layer's BPTT seeds
        top = self.enc[-1]
        k.rs_bwd(w["dc_carry"], w["dh_rec"], w["rs_pre"][0], w["rs_pre"][1], self.pk["RC"], self.pk["RH"],
                 w["rs_dp"][0], w["rs_dp"][1], None if self.det else g(BRC), None if self.det else g(BRH),
                 top["dc_carry"], top["dh_fin"], B, H)
        if self.det:  # bias gradients: relu'-masked row sums in a fixed order
            for pre, gsrc, dst in ((w["rs_pre"][0], w["dc_carry"], g(BRC)), (w["rs_pre"][1], w["dh_rec"], g(BRH))):
                k.colsum(torch.where(pre > 0, gsrc, torch.zeros_like(gsrc)), dst, B, H, False)
        gemm(g(RC), w["rs_cat"][0].t(), w["rs_dp"][0])
        gemm(g(RH), w["rs_cat"][1].t(), w["rs_dp"][1])
        # ---- encoder BPTT, top layer down
        d_in = dE
        for layer in reversed(range(self.L)):
            st = self.enc[layer]
            din = st["din"]
            # dL/dh_out in step frame: fw as is, bw reversed within each length (below the top layer
            # the previous iteration's step_frame_hop wrote it straight from the upper layer's dxs)
            # (the persistent BPTT reads the top layer's gradient in the batch frame itself: no pass)
            top_bf = layer == self.L - 1 and self.persistent_lstm
            if layer == self.L - 1 and not top_bf:
                k.to_step_frame(d_in, None, w["rev_idx"], st["dout"], B, T, H, H)
            if layer != self.L - 1:  # the top layer's seeds came from rs_bwd
                st["dh_fin"].zero_()
                st["dc_carry"].zero_()
            if self.persistent_lstm:
                w["lstm_xb"].zero_()
                w["lstm_db"].zero_()
                k.lstm_bwd_persistent(st["dz"], self.pk[f"enc{layer}_Wn"], d_in if top_bf else st["dout"], st["dh_fin"],
                                      st["dc_carry"], st["acts"], st["cs"], lens, w["lstm_xb"], w["lstm_err"],
                                      None if self.det else w["lstm_db"], T, B, H, top_bf)
            else:
                for s in reversed(range(T)):
                    k.lstm_enc_bwd_step(st["dz"], self.pk[f"enc{layer}_Wn"], st["dout"], st["dh_fin"],
                                        st["dc_carry"], st["acts"], st["cs"], lens, s, T, B, H)
            dxs = st["dxs"]  # [2][T*B][din]: both directions' input gradients, step frame
            rev = w["rev_idx"]
            merge = self.dx_merge and layer > 0
            for di, d in enumerate(("fw", "bw")):
                dzd = st["dz"][di].view(T * B, 4 * H)
                gkd = g(enc_k(layer, d))
                wgrad_enc_into(gkd[:din], st["x_sf"][di].view(T * B, din), dzd)
                wgrad_enc_into(gkd[din:], st["hs"][di, :T].reshape(T * B, H), dzd)
                if self.persistent_lstm and not self.det:
                    g(enc_b(layer, d)).copy_(w["lstm_db"][di])
                else:
                    k.colsum(dzd, g(enc_b(layer, d)), T * B, 4 * H, False)
                if not merge:
                    gemm(dxs[di], dzd, self.pk[f"enc{layer}_Kx{di}"].t())
            if layer > 0:  # the layer below's output-gradient step frame, without the batch-frame dx
                lo = self.enc[layer - 1]["dout"].view(2, T * B, H)
                if merge:  # fw units: [dz_fw(t) | dz_bw(rev)]; bw units: [dz_fw(rev) | dz_bw(t)]
                    Km = self.pk[f"enc{layer}_Kx01"]
                    k.gemm_bt_merge(st["dz"], Km[:H], lo[0], rev, B, T, 2)
                    k.gemm_bt_merge(st["dz"], Km[H:], lo[1], rev, B, T, 1)
                else:
                    k.step_frame_hop(dxs, rev, lo, B, T, H)
                continue
            dx = st["dx"]
            k.from_step_frame(dxs, rev, dx, B, T, din)  # fw + reversed bw, batch frame
            d_in = dx
        self._d_in = d_in
        if late:
            torch.cuda.current_stream().wait_stream(self._late_stream)  # the deferred weight gradients

    def backward_tail_emb(self):
        """Embedding gradient of the encoder and decoder token rows (the last bucket)."""
        k, w, p = self.k, self.w, self.p
        B, T = self.B, self.T
        gemb, d_in = p.g(EMB), self._d_in
        # encoder + decoder token rows in id order (the order is sorted on the host with the
        # batch, emb_sort; one launch, embedding.hip): atomics only where the id changes, so
        # Zipf-hot tokens do not serialise
        if self.det:
            k.emb_grad_det(gemb, w["emb_sid"], w["emb_perm"], d_in.reshape(B * T, self.E), w["d_emb_dec"],
                           w["emb_pf"], w["emb_pl"])
        else:
            k.emb_grad_sorted(gemb, w["emb_sid"], w["emb_perm"], d_in.reshape(B * T, self.E), w["d_emb_dec"])
        if self.poison_on_lstm_err:
            from ..parallel.dist import poison_where
            poison_where(w["lstm_err"], p.grad[-1:])

    # ------------------------------------------------------------------ optimizer
    def optimizer_step(self):
        """Fused clip + Adagrad over the flat buffers, then the bf16 repack.  ``grad_scale``
        (1/world under data parallelism) averages the all-reduced gradient sum inside the
        optimizer kernel; a set ``lstm_err`` word (sticky) skips the update on device."""
        hps, p, w = self.hps, self.p, self.w
        self.k.clip_adagrad(p.flat, p.accum, p.grad, w["opt_part"], hps.lr, hps.max_grad_norm, self.grad_scale,
                            w["gnorm"], w["nan_flag"], w["lstm_err"])
        self.pack()

    def train_step(self, allreduce=None):
        """forward + backward (+ optional grad all-reduce hook) + clip/Adagrad + repack."""
        out = self.forward(need_grad=True)
        self.backward()
        if allreduce is not None:
            allreduce(self.p.grad)
        self.optimizer_step()
        return out
