"""Host beam search with the reference's exact semantics (``beam_search.py:26-173``).

Reproduced quirks:
  * all beam_size hypotheses start as copies of [START]; on step 0 only hypothesis 0 is
    expanded (``beam_search.py:127-128``);
  * each live hypothesis is extended with its top 2*beam candidates; all candidates are
    sorted by average log-prob (sum / len(tokens), len INCLUDING [START] with log-prob 0);
  * a [STOP] candidate goes to results only if steps >= min_dec_steps, otherwise it is
    discarded; collection stops at beam_size live hyps or beam_size results;
  * the loop runs while steps < max_dec_steps and len(results) < beam_size; if no result
    finished, the live hyps are used; the best by average log-prob is returned.
  * in-article OOV ids (>= vocab size) are fed back as [UNK].

The step model is pluggable (``StepModel``): the PyTorch oracle on CPU, or the gfx950
decode step on GPU.  The batched device-resident version (many articles per launch,
hipGraph-captured) lives in ``decode.device_beam``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch

from ..data.vocab import START_DECODING, STOP_DECODING, UNKNOWN_TOKEN


@dataclass
class Hypothesis:
    tokens: List[int]
    log_probs: List[float]
    state: tuple
    attn_dists: List[np.ndarray] = field(default_factory=list)
    p_gens: List[Optional[float]] = field(default_factory=list)
    coverage: Optional[np.ndarray] = None

    def extend(self, token, log_prob, state, attn_dist, p_gen, coverage) -> "Hypothesis":
        return Hypothesis(self.tokens + [token], self.log_probs + [log_prob], state, self.attn_dists + [attn_dist],
                          self.p_gens + [p_gen], coverage)

    @property
    def latest_token(self) -> int:
        return self.tokens[-1]

    @property
    def log_prob(self) -> float:
        return sum(self.log_probs)

    @property
    def avg_log_prob(self) -> float:
        return self.log_prob / len(self.tokens)


def sort_hyps(hyps: List[Hypothesis]) -> List[Hypothesis]:
    return sorted(hyps, key=lambda h: h.avg_log_prob, reverse=True)


class OracleStepModel:
    """run_encoder / decode_onestep over ReferencePointerGenerator (model.py:347-443)."""

    def __init__(self, ref, W, hps, device="cpu"):
        self.ref, self.W, self.hps, self.device = ref, W, hps, torch.device(device)

    @torch.no_grad()
    def run_encoder(self, batch):
        enc_batch = torch.as_tensor(batch.enc_batch[:1], dtype=torch.long, device=self.device)
        lens = torch.as_tensor(batch.enc_lens[:1], dtype=torch.long, device=self.device)
        enc_out, F, (c0, h0) = self.ref.encode(self.W, enc_batch, lens)
        mask = torch.as_tensor(batch.enc_padding_mask[:1], device=self.device)
        ext = torch.as_tensor(batch.enc_batch_extend_vocab[:1], dtype=torch.long, device=self.device)
        return {"enc_out": enc_out, "F": F, "mask": mask, "ext": ext, "max_oovs": int(batch.max_art_oovs)}, \
            (c0[0], h0[0])

    @torch.no_grad()
    def decode_onestep(self, enc, latest_tokens, states, prev_coverage, k2):
        k = len(states)
        c = torch.stack([s[0] for s in states])
        h = torch.stack([s[1] for s in states])
        tok = torch.as_tensor(latest_tokens, dtype=torch.long, device=self.device)
        rep = lambda x: x.expand(k, *x.shape[1:])
        cov = torch.as_tensor(np.stack(prev_coverage), dtype=c.dtype, device=self.device) \
            if prev_coverage[0] is not None else None
        ids, lp, c2, h2, a, pg, cov2 = self.ref.decode_onestep(
            self.W, rep(enc["enc_out"]), rep(enc["F"]), rep(enc["mask"]), rep(enc["ext"]), enc["max_oovs"], tok, c, h,
            cov, k2)
        new_states = [(c2[i], h2[i]) for i in range(k)]
        attn = [a[i].cpu().numpy() for i in range(k)]
        pgens = [float(pg[i]) for i in range(k)] if pg is not None else [None] * k
        covs = [cov2[i].cpu().numpy() for i in range(k)] if cov2 is not None else [None] * k
        return ids.cpu().numpy(), lp.cpu().numpy(), new_states, attn, pgens, covs


def run_beam_search(model, vocab, batch, hps) -> Hypothesis:
    enc, dec_in_state = model.run_encoder(batch)
    T = batch.enc_batch.shape[1]
    start, stop, unk = vocab.word2id(START_DECODING), vocab.word2id(STOP_DECODING), vocab.word2id(UNKNOWN_TOKEN)
    V = vocab.size()
    hyps = [Hypothesis([start], [0.0], dec_in_state, [], [], np.zeros([T], np.float32)) for _ in range(hps.beam_size)]
    results: List[Hypothesis] = []
    steps = 0
    while steps < hps.max_dec_steps and len(results) < hps.beam_size:
        latest = [h.latest_token if h.latest_token < V else unk for h in hyps]
        ids, lps, new_states, attn, pgens, covs = model.decode_onestep(
            enc, latest, [h.state for h in hyps], [h.coverage if hps.coverage else None for h in hyps],
            2 * hps.beam_size)
        all_hyps = []
        num_orig = 1 if steps == 0 else len(hyps)
        for i in range(num_orig):
            for j in range(2 * hps.beam_size):
                all_hyps.append(hyps[i].extend(int(ids[i, j]), float(lps[i, j]), new_states[i], attn[i], pgens[i],
                                               covs[i]))
        hyps = []
        for h in sort_hyps(all_hyps):
            if h.latest_token == stop:
                if steps >= hps.min_dec_steps:
                    results.append(h)
            else:
                hyps.append(h)
            if len(hyps) == hps.beam_size or len(results) == hps.beam_size:
                break
        steps += 1
    if not results:
        results = hyps
    return sort_hyps(results)[0]
