"""Host beam search reproduces the reference's quirks (SURVEY 2.9 items 7-8;
``beam_search.py:82-173``), checked with a scripted step model so every candidate list,
log-prob and STOP position is chosen by the test."""
from types import SimpleNamespace

import numpy as np
import pytest

from textsummarization_on_flink_amd.config import HParams
from textsummarization_on_flink_amd.data.vocab import Vocab
from textsummarization_on_flink_amd.decode.beam_search import Hypothesis, run_beam_search, sort_hyps

WORDS = [f"w{i}" for i in range(20)]


@pytest.fixture
def vocab():
    return Vocab(words=WORDS)  # ids: 0-3 specials, w0 = 4 ... w19 = 23; V = 24


class Scripted:
    """decode_onestep returns, for hypothesis row i at step s, ``script(s, i, latest_token)``:
    a list of (id, log_prob) pairs (2 * beam of them)."""

    def __init__(self, script):
        self.script = script
        self.step = 0
        self.calls = []

    def run_encoder(self, batch):
        return {}, ("c0", "h0")

    def decode_onestep(self, enc, latest, states, prev_cov, k2):
        self.calls.append(list(latest))
        ids, lps = [], []
        for i, tok in enumerate(latest):
            pairs = self.script(self.step, i, tok)
            assert len(pairs) == k2
            ids.append([p[0] for p in pairs])
            lps.append([p[1] for p in pairs])
        self.step += 1
        n = len(latest)
        return (np.array(ids), np.array(lps, dtype=np.float64), [("c", "h")] * n, [np.zeros(3)] * n, [0.5] * n,
                [np.zeros(3)] * n)


def _batch():
    return SimpleNamespace(enc_batch=np.zeros((2, 3), np.int64))


def _hps(**kw):
    base = dict(beam_size=2, max_dec_steps=6, min_dec_steps=2, coverage=False)
    base.update(kw)
    return HParams(**base)


def test_avg_log_prob_counts_start_token():
    h = Hypothesis([2, 7, 3], [0.0, -1.0, -2.0], None)
    assert h.log_prob == pytest.approx(-3.0)
    assert h.avg_log_prob == pytest.approx(-1.0)  # / len(tokens), [START] included
    a = Hypothesis([2, 5], [0.0, -1.0], None)     # avg -0.5
    b = Hypothesis([2, 5, 6], [0.0, -0.6, -0.6], None)  # avg -0.4
    assert sort_hyps([a, b])[0] is b


def test_step0_expands_only_first_hypothesis(vocab):
    # row i proposes ids 4 + 10*i + j; if row 1 were expanded at step 0, its (better-scored)
    # candidates would win
    def script(s, i, tok):
        return [(4 + 10 * i + j, -1.0 + 0.5 * i - 0.1 * j) for j in range(4)]

    m = Scripted(script)
    best = run_beam_search(m, vocab, _batch(), _hps(max_dec_steps=1))
    assert m.calls[0] == [2, 2]  # both hypotheses start as [START]
    assert best.tokens == [2, 4]


def test_stop_before_min_dec_steps_is_discarded(vocab):
    stop = vocab.word2id("[STOP]")

    # the best candidate is always [STOP]; below min_dec_steps it must be dropped
    def script(s, i, tok):
        return [(stop, -0.01), (4 + s, -1.0), (5 + s, -1.5), (6 + s, -2.0)]

    best = run_beam_search(Scripted(script), vocab, _batch(), _hps(min_dec_steps=2, max_dec_steps=6))
    assert best.tokens[-1] == stop
    # steps 0 and 1 are below min_dec_steps: the first accepted STOP comes at step 2
    assert len(best.tokens) == 4  # [START] w w [STOP]


def test_no_result_falls_back_to_live_hyps(vocab):
    def script(s, i, tok):
        return [(4, -0.5), (5, -0.7), (6, -0.9), (7, -1.1)]

    best = run_beam_search(Scripted(script), vocab, _batch(), _hps(max_dec_steps=3))
    assert vocab.word2id("[STOP]") not in best.tokens
    assert best.tokens == [2, 4, 4, 4]


def test_oov_ids_fed_back_as_unk(vocab):
    V = vocab.size()

    def script(s, i, tok):
        return [(V + 1, -0.1), (4, -0.5), (5, -0.6), (6, -0.7)]  # an in-article OOV wins every step

    m = Scripted(script)
    best = run_beam_search(m, vocab, _batch(), _hps(max_dec_steps=3))
    assert best.tokens[1] == V + 1                   # the hypothesis keeps the extended id
    assert m.calls[1][0] == vocab.word2id("[UNK]")   # ... but the decoder is fed [UNK]


def test_stops_when_beam_size_results(vocab):
    stop = vocab.word2id("[STOP]")

    def script(s, i, tok):
        return [(stop, -0.1), (stop, -0.2), (4, -3.0), (5, -3.5)]

    m = Scripted(script)
    best = run_beam_search(m, vocab, _batch(), _hps(min_dec_steps=0, max_dec_steps=10))
    assert m.step == 1  # two STOP results at step 0 fill the beam
    assert best.tokens == [2, stop]
