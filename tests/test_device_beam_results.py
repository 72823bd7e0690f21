"""Device beam search, host side: the vectorised winner-first backtracking of
``DeviceBeamDecoder.results`` == the per-candidate walk it replaced (``_results_walk``), on
randomised beam histories with finished and live articles, score ties and short articles.
CPU only: the decoder's device buffers are replaced by CPU tensors."""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from textsummarization_on_flink_amd.data.vocab import Vocab
from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder


def _fake(seed, keep_attn, pointer_gen=True, Na=9, beam=4, D=12, T=5, steps=None):
    rng = np.random.default_rng(seed)
    R = Na * beam
    dec = object.__new__(DeviceBeamDecoder)
    dec.beam, dec.Na, dec.maxD, dec.keep_attn = beam, Na, D, keep_attn
    dec.hps = SimpleNamespace(pointer_gen=pointer_gen)
    dec.vocab = Vocab(words=[f"w{i}" for i in range(40)])
    res_count = rng.integers(0, beam + 1, Na)
    res_count[0], res_count[1] = 0, beam
    res_score = rng.normal(size=R).astype(np.float32)
    res_score[beam * 1 + 2] = res_score[beam * 1 + 0]  # tie among finished: first one wins
    lp_sum = rng.normal(size=R).astype(np.float32) * 5
    lp_sum[1] = lp_sum[3]                               # tie among live beams of article 0
    b = {
        "res_count": torch.tensor(res_count, dtype=torch.int32),
        "res_score": torch.tensor(res_score),
        "res_len": torch.zeros(R, dtype=torch.int32),
        "res_step": torch.tensor(rng.integers(1, D, R), dtype=torch.int32),
        "res_par": torch.tensor(rng.integers(0, beam, R), dtype=torch.int32),
        "lp_sum": torch.tensor(lp_sum),
        "tok_hist": torch.tensor(rng.integers(4, 40, (D, R)), dtype=torch.int32),
        "par_hist": torch.tensor(rng.integers(0, beam, (D, R)), dtype=torch.int32),
        "step": torch.tensor([D if steps is None else steps], dtype=torch.int32),
        "done": torch.zeros(Na, dtype=torch.int32),
    }
    if keep_attn:
        b["ATT_hist"] = torch.tensor(rng.random((D, R, T)), dtype=torch.float32)
        b["PG_hist"] = torch.tensor(rng.random((D, R)), dtype=torch.float32)
    dec.b = b
    return dec


@pytest.mark.parametrize("seed,keep_attn,pointer_gen,steps,n_valid", [
    (0, False, True, None, None), (1, True, True, None, None), (2, True, False, None, 7),
    (3, True, True, 5, None), (4, False, True, 1, 3)])
def test_vectorised_results_match_per_candidate_walk(seed, keep_attn, pointer_gen, steps, n_valid):
    dec = _fake(seed, keep_attn, pointer_gen, steps=steps)
    got, ref = dec.results(n_valid), dec._results_walk(n_valid)
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        assert g.tokens == r.tokens
        np.testing.assert_allclose(g.log_probs, r.log_probs, rtol=1e-12)
        assert len(g.attn_dists) == len(r.attn_dists)
        for x, y in zip(g.attn_dists, r.attn_dists):
            np.testing.assert_array_equal(x, y)
        assert g.p_gens == r.p_gens
