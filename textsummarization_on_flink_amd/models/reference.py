"""Pure-PyTorch oracle of the pointer-generator network with coverage.

Written line-by-line from the reference graph (``model.py:76-285,446-480``,
``attention_decoder.py:27-228``) with plain autograd.  It is

  * the numerics reference every HIP kernel is tested against (fp32/fp64 on CPU),
  * the CPU execution path for plumbing tests and BASELINE config #1 (tiny model),
  * the decode-step oracle reproducing the decode-mode quirks:
    initial-state attention updates coverage once, the post-cell attention reuses it
    without updating.

On a GPU device the production path is ``models.pointer_generator.HipPointerGenerator``;
this module never silently stands in for it there.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as Fn

from .params import DEC, P, enc_prefix


def lstm_cell(x, c, h, kernel, bias):
    """TF LSTMCell: z = [x, h] K + b, gates i, j, f, o; forget_bias = 1.0."""
    z = torch.cat([x, h], dim=-1) @ kernel + bias
    i, j, f, o = z.chunk(4, dim=-1)
    c2 = torch.sigmoid(f + 1.0) * c + torch.sigmoid(i) * torch.tanh(j)
    h2 = torch.sigmoid(o) * torch.tanh(c2)
    return c2, h2


def reverse_within_length(x, lens):
    """TF ReverseSequence along time (dim 1) per row length; padding stays in place."""
    B, T = x.shape[:2]
    t = torch.arange(T, device=x.device)[None, :]
    L = lens[:, None].to(t.dtype)
    idx = torch.where(t < L, L - 1 - t, t)
    return x.gather(1, idx[..., None].expand(-1, -1, x.shape[2]) if x.dim() == 3 else idx)


def dynamic_lstm(x, lens, kernel, bias, H):
    """dynamic_rnn with sequence_length: outputs zero past len, final state at len."""
    B, T, _ = x.shape
    c = x.new_zeros(B, H)
    h = x.new_zeros(B, H)
    outs = []
    for s in range(T):
        c2, h2 = lstm_cell(x[:, s], c, h, kernel, bias)
        act = (s < lens).to(x.dtype)[:, None]
        c = act * c2 + (1 - act) * c
        h = act * h2 + (1 - act) * h
        outs.append(act * h2)
    return torch.stack(outs, 1), c, h


def bidirectional_lstm(x, lens, kf, bf, kb, bb, H):
    of, cf, hf = dynamic_lstm(x, lens, kf, bf, H)
    xr = reverse_within_length(x, lens)
    orv, cb, hb = dynamic_lstm(xr, lens, kb, bb, H)
    ob = reverse_within_length(orv, lens)
    return torch.cat([of, ob], dim=2), (cf, hf), (cb, hb)


def masked_softmax(e, mask):
    """softmax(e) * mask, renormalised (attention_decoder.py:96-101)."""
    a = torch.softmax(e, dim=-1) * mask
    return a / a.sum(dim=-1, keepdim=True)


class ReferencePointerGenerator:
    """Functional oracle: all weights come from a name -> tensor mapping (FlatParams views)."""

    def __init__(self, hps, vsize: int):
        self.hps = hps
        self.V = vsize
        self.E, self.H = hps.emb_dim, hps.hidden_dim
        self.A = 2 * self.H

    # ------------------------------------------------------------------ pieces
    def encode(self, W, enc_batch, enc_lens):
        hps, H = self.hps, self.H
        x = W[f"{P}/embedding/embedding"][enc_batch]
        L = max(1, getattr(hps, "enc_layers", 1))
        fw = bw = None
        for layer in range(L):
            pre = f"{enc_prefix(layer)}/bidirectional_rnn"
            x, fw, bw = bidirectional_lstm(x, enc_lens, W[f"{pre}/fw/lstm_cell/kernel"], W[f"{pre}/fw/lstm_cell/bias"],
                                           W[f"{pre}/bw/lstm_cell/kernel"], W[f"{pre}/bw/lstm_cell/bias"], H)
        enc_out = x
        old_c = torch.cat([fw[0], bw[0]], 1)
        old_h = torch.cat([fw[1], bw[1]], 1)
        c0 = torch.relu(old_c @ W[f"{P}/reduce_final_st/w_reduce_c"] + W[f"{P}/reduce_final_st/bias_reduce_c"])
        h0 = torch.relu(old_h @ W[f"{P}/reduce_final_st/w_reduce_h"] + W[f"{P}/reduce_final_st/bias_reduce_h"])
        F = enc_out @ W[f"{DEC}/W_h"].reshape(self.A, self.A)
        return enc_out, F, (c0, h0)

    def attention(self, W, enc_out, F, mask, c, h, coverage):
        """Returns (ctx, attn, new_coverage) following attention_decoder.py:79-129."""
        dec_feat = torch.cat([c, h], 1) @ W[f"{DEC}/Attention/Linear/Matrix"] + W[f"{DEC}/Attention/Linear/Bias"]
        u = F + dec_feat[:, None, :]
        if self.hps.coverage and coverage is not None:
            u = u + coverage[..., None] * W[f"{DEC}/coverage/w_c"].reshape(1, 1, self.A)
            e = (W[f"{DEC}/v"] * torch.tanh(u)).sum(-1)
            a = masked_softmax(e, mask)
            coverage = coverage + a
        else:
            e = (W[f"{DEC}/v"] * torch.tanh(u)).sum(-1)
            a = masked_softmax(e, mask)
            if self.hps.coverage:
                coverage = a
        ctx = (a[..., None] * enc_out).sum(1)
        return ctx, a, coverage

    def post_cell(self, W, ctx, c, h, x):
        p_gen = None
        if self.hps.pointer_gen:
            p_gen = torch.sigmoid(torch.cat([ctx, c, h, x], 1) @ W[f"{DEC}/calculate_pgen/Linear/Matrix"]
                                  + W[f"{DEC}/calculate_pgen/Linear/Bias"])[:, 0]
        out = torch.cat([h, ctx], 1) @ W[f"{DEC}/AttnOutputProjection/Linear/Matrix"] + \
            W[f"{DEC}/AttnOutputProjection/Linear/Bias"]
        return p_gen, out

    def vocab_logits(self, W, out):
        return out @ W[f"{P}/output_projection/w"] + W[f"{P}/output_projection/v"]

    def final_dist(self, vocab_dist, attn, p_gen, ext_ids, max_oovs):
        """p_gen * [P_vocab, 0_oov] + scatter((1-p_gen) a) (model.py:146-183)."""
        R = vocab_dist.shape[0]
        ext = torch.cat([p_gen[:, None] * vocab_dist, vocab_dist.new_zeros(R, max_oovs)], 1)
        return ext.scatter_add(1, ext_ids.long(), (1 - p_gen[:, None]) * attn)

    # ------------------------------------------------------------------ train / eval
    def forward(self, W, batch: Dict[str, torch.Tensor]):
        """Returns dict(loss, coverage_loss, total_loss, attn_dists [D,B,T], p_gens [D,B])."""
        hps = self.hps
        enc_batch, lens = batch["enc_batch"], batch["enc_lens"]
        mask_enc = batch["enc_padding_mask"]
        enc_out, F, (c, h) = self.encode(W, enc_batch, lens)
        emb = W[f"{P}/embedding/embedding"]
        dec_batch = batch["dec_batch"]
        B, D = dec_batch.shape
        ctx = enc_out.new_zeros(B, self.A)
        coverage = None
        attn_dists, p_gens, outs = [], [], []
        for t in range(D):
            x = torch.cat([emb[dec_batch[:, t]], ctx], 1) @ W[f"{DEC}/Linear/Matrix"] + W[f"{DEC}/Linear/Bias"]
            c, h = lstm_cell(x, c, h, W[f"{DEC}/lstm_cell/kernel"], W[f"{DEC}/lstm_cell/bias"])
            ctx, a, coverage = self.attention(W, enc_out, F, mask_enc, c, h, coverage)
            attn_dists.append(a)
            p_gen, out = self.post_cell(W, ctx, c, h, x)
            p_gens.append(p_gen)
            outs.append(out)
        logits = self.vocab_logits(W, torch.stack(outs, 0))  # [D,B,V]
        target = batch["target_batch"].t()                   # [D,B]
        dec_mask = batch["dec_padding_mask"]                 # [B,D]
        valid = batch.get("valid")
        if valid is None:
            valid = dec_mask.new_ones(B)
        attn = torch.stack(attn_dists, 0)
        if hps.pointer_gen:
            pg = torch.stack(p_gens, 0)
            vocab_dist = torch.softmax(logits, -1)
            max_oovs = int(batch.get("max_art_oovs", 0))
            ext = batch["enc_batch_extend_vocab"]
            losses = []
            for t in range(D):
                fd = self.final_dist(vocab_dist[t], attn[t], pg[t], ext, max_oovs)
                gold = fd.gather(1, target[t][:, None].long())[:, 0]
                losses.append(-torch.log(gold))
            loss = mask_and_avg(torch.stack(losses, 0), dec_mask, valid)
        else:
            pg = None
            ce = Fn.cross_entropy(logits.reshape(D * B, -1), target.reshape(-1).long(), reduction="none").view(D, B)
            w = dec_mask.t() * valid[None, :]
            loss = (ce * w).sum() / w.sum()  # tf.contrib.seq2seq.sequence_loss
        out = {"loss": loss, "attn_dists": attn, "p_gens": pg}
        if hps.coverage:
            covl = coverage_loss(attn, dec_mask, valid)
            out["coverage_loss"] = covl
            out["total_loss"] = loss + hps.cov_loss_wt * covl
        else:
            out["total_loss"] = loss
        return out

    # ------------------------------------------------------------------ decode
    def decode_onestep(self, W, enc_out, F, mask, ext_ids, max_oovs, tokens, c, h, prev_cov, k2: int):
        """One beam step exactly as the decode graph (max_dec_steps=1,
        initial_state_attention=True).  Returns topk ids/log-probs (top 2*beam),
        new (c, h), attn, p_gen, coverage."""
        hps = self.hps
        cov = prev_cov if hps.coverage else None
        ctx, _, cov = self.attention(W, enc_out, F, mask, c, h, cov)
        emb = W[f"{P}/embedding/embedding"][tokens]
        x = torch.cat([emb, ctx], 1) @ W[f"{DEC}/Linear/Matrix"] + W[f"{DEC}/Linear/Bias"]
        c, h = lstm_cell(x, c, h, W[f"{DEC}/lstm_cell/kernel"], W[f"{DEC}/lstm_cell/bias"])
        ctx, a, _ = self.attention(W, enc_out, F, mask, c, h, cov)
        p_gen, out = self.post_cell(W, ctx, c, h, x)
        vd = torch.softmax(self.vocab_logits(W, out), -1)
        if hps.pointer_gen:
            fd = self.final_dist(vd, a, p_gen, ext_ids, max_oovs)
        else:
            fd = vd
        probs, ids = torch.topk(fd, k2, dim=1)
        return ids, torch.log(probs), c, h, a, p_gen, cov


def mask_and_avg(values, dec_mask, valid):
    """values [D,B]; per-example masked mean over dec_len, then mean over (valid) batch."""
    dec_lens = dec_mask.sum(1)
    per_ex = (values * dec_mask.t()).sum(0) / dec_lens
    return (per_ex * valid).sum() / valid.sum()


def coverage_loss(attn, dec_mask, valid):
    """sum_i min(a_t, cov_t) with cov starting at zero (model.py:463-480)."""
    cov = torch.zeros_like(attn[0])
    losses = []
    for t in range(attn.shape[0]):
        losses.append(torch.minimum(attn[t], cov).sum(1))
        cov = cov + attn[t]
    return mask_and_avg(torch.stack(losses, 0), dec_mask, valid)


def batch_to_tensors(batch, device="cpu") -> Dict[str, torch.Tensor]:
    d = {
        "enc_batch": torch.as_tensor(batch.enc_batch, dtype=torch.long),
        "enc_lens": torch.as_tensor(batch.enc_lens, dtype=torch.long),
        "enc_padding_mask": torch.as_tensor(batch.enc_padding_mask),
        "enc_batch_extend_vocab": torch.as_tensor(batch.enc_batch_extend_vocab, dtype=torch.long),
        "dec_batch": torch.as_tensor(batch.dec_batch, dtype=torch.long),
        "target_batch": torch.as_tensor(batch.target_batch, dtype=torch.long),
        "dec_padding_mask": torch.as_tensor(batch.dec_padding_mask),
        "valid": torch.as_tensor(batch.valid),
    }
    d = {k: v.to(device) for k, v in d.items()}
    d["max_art_oovs"] = int(batch.max_art_oovs)
    return d
