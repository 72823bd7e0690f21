"""Synthetic CNN/DailyMail-shaped data (there is no network for the real corpus).

Shapes follow the public CNN/DM statistics the reference pipeline sees after
``make_datafiles.py``: articles ~780 PTB tokens (so ~85% are truncated at
``max_enc_steps=400``), highlights of 3-4 sentences totalling ~56 tokens, Zipfian word
frequencies over a 200k-word raw vocabulary of which the model keeps the top
``vocab_size`` (so in-article OOVs exist and some are copied into the abstract, which
exercises the pointer/extended-vocab path exactly like the real data).
"""
from __future__ import annotations

from typing import Iterator, List, Optional, Tuple

import numpy as np

from .vocab import SENTENCE_END, SENTENCE_START, Vocab


class SyntheticCorpus:
    def __init__(self, vocab_size: int = 50000, raw_vocab: int = 200000, seed: int = 0,
                 art_mean: float = 780.0, art_sd: float = 380.0, abs_sents: Tuple[int, int] = (3, 4),
                 sent_mean: float = 15.0, copy_frac: float = 0.6):
        self.rng = np.random.default_rng(seed)
        self.raw_vocab = raw_vocab
        self.words = [f"w{i}" for i in range(raw_vocab)]
        ranks = np.arange(1, raw_vocab + 1, dtype=np.float64)
        p = 1.0 / ranks ** 1.07
        self.p = p / p.sum()
        self.cdf = np.cumsum(self.p)
        self.vocab_size = vocab_size
        self.art_mean, self.art_sd = art_mean, art_sd
        self.abs_sents = abs_sents
        self.sent_mean = sent_mean
        self.copy_frac = copy_frac

    def vocab(self, max_size: Optional[int] = None) -> Vocab:
        n = (max_size or self.vocab_size) - 4
        return Vocab(words=self.words[:n], max_size=max_size or self.vocab_size)

    def _draw(self, n: int) -> np.ndarray:
        return np.minimum(np.searchsorted(self.cdf, self.rng.random(n)), self.raw_vocab - 1)

    def sample(self) -> Tuple[str, str]:
        """Return (article, abstract) in the .bin text format (abstract is <s> tagged)."""
        n = int(np.clip(self.rng.normal(self.art_mean, self.art_sd), 40, 2000))
        art_ids = self._draw(n)
        art = [self.words[i] for i in art_ids]
        ns = int(self.rng.integers(self.abs_sents[0], self.abs_sents[1] + 1))
        sents = []
        for _ in range(ns):
            L = int(np.clip(self.rng.normal(self.sent_mean, 5.0), 4, 40))
            ncopy = int(round(L * self.copy_frac))
            copied = [art[j] for j in self.rng.integers(0, min(n, 400), ncopy)]
            fresh = [self.words[i] for i in self._draw(L - ncopy)]
            toks = copied + fresh
            self.rng.shuffle(toks)
            sents.append(" ".join(toks) + " .")
        abstract = " ".join(f"{SENTENCE_START} {s} {SENTENCE_END}" for s in sents)
        return " ".join(art), abstract

    def examples(self, n: int) -> List[Tuple[str, str]]:
        return [self.sample() for _ in range(n)]

    def stream(self) -> Iterator[Tuple[str, str]]:
        while True:
            yield self.sample()

    def rows(self, n: int, prefix: str = "uuid") -> List[dict]:
        """Streaming rows {uuid, article, summary, reference} (App.java:92, Message.java)."""
        from .vocab import abstract2sents
        out = []
        for i in range(n):
            a, s = self.sample()
            out.append({"uuid": f"{prefix}-{i}", "article": a, "summary": "",
                        "reference": " ".join(x.strip() for x in abstract2sents(s))})
        return out


def make_batches(hps, vocab: Vocab, corpus: SyntheticCorpus, n_batches: int, pad_enc_to=None):
    from .batch import Batch, Example
    from .vocab import abstract2sents
    out = []
    for _ in range(n_batches):
        exs = []
        for _ in range(hps.batch_size):
            a, s = corpus.sample()
            exs.append(Example(a, [x.strip() for x in abstract2sents(s)], vocab, hps))
        out.append(Batch(exs, hps, vocab, pad_enc_to=pad_enc_to))
    return out
