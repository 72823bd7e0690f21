"""Example / Batch construction (reference ``batcher.py:33-219, 398-410``).

Semantics reproduced exactly: whitespace tokenisation, truncation to ``max_enc_steps``,
``[START]``-prefixed decoder input and ``[STOP]``-terminated target (no STOP when
truncated), extended-vocab OOV ids for the pointer, PAD id 1 padding and float masks.

MI355X-side additions:
  * ``uuid`` is carried for the streaming path (``FlinkExample``/``FlinkBatch``);
  * masks are built vectorised;
  * optional static encoder padding to ``max_enc_steps`` so every batch has one shape
    and the whole train step replays from one hipGraph (padding is masked, so this is
    numerically identical to dynamic padding);
  * a short final batch is padded with copies of a real row marked ``valid = 0``
    (Issue-5 / SURVEY 2.9 item 3: the reference indexed past the end and hung); the
    loss averages over valid rows only, which equals the reference for full batches.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np

from .vocab import (PAD_TOKEN, START_DECODING, STOP_DECODING, Vocab, abstract2ids, article2ids)


class Example:
    def __init__(self, article: str, abstract_sentences: Sequence[str], vocab: Vocab, hps, uuid: Optional[str] = None):
        self.hps = hps
        self.uuid = uuid
        start_decoding = vocab.word2id(START_DECODING)
        stop_decoding = vocab.word2id(STOP_DECODING)
        article_words = article.split(None, hps.max_enc_steps)  # stops after the kept words
        if len(article_words) > hps.max_enc_steps:
            article_words = article_words[:hps.max_enc_steps]
        self.enc_len = len(article_words)
        self.enc_input = vocab.ids(article_words)
        abstract = " ".join(abstract_sentences)
        abstract_words = abstract.split()
        abs_ids = vocab.ids(abstract_words)
        self.dec_input, self.target = self.get_dec_inp_targ_seqs(abs_ids, hps.max_dec_steps, start_decoding,
                                                                 stop_decoding)
        self.dec_len = len(self.dec_input)
        if hps.pointer_gen:
            self.enc_input_extend_vocab, self.article_oovs = article2ids(article_words, vocab, self.enc_input)
            abs_ids_extend_vocab = abstract2ids(abstract_words, vocab, self.article_oovs, abs_ids)
            _, self.target = self.get_dec_inp_targ_seqs(abs_ids_extend_vocab, hps.max_dec_steps, start_decoding,
                                                        stop_decoding)
        else:
            self.enc_input_extend_vocab, self.article_oovs = list(self.enc_input), []
        self.original_article = article
        self.original_abstract = abstract
        self.original_abstract_sents = list(abstract_sentences)

    @staticmethod
    def get_dec_inp_targ_seqs(sequence, max_len, start_id, stop_id):
        inp = [start_id] + list(sequence)
        target = list(sequence)
        if len(inp) > max_len:
            inp = inp[:max_len]
            target = target[:max_len]
        else:
            target.append(stop_id)
        assert len(inp) == len(target)
        return inp, target


FlinkExample = Example  # the uuid-carrying variant (batcher.py:398-401) is the same class here


class Batch:
    def __init__(self, example_list: List[Example], hps, vocab: Vocab, pad_enc_to: Optional[int] = None):
        if not example_list:
            raise ValueError("empty batch")
        self.pad_id = vocab.word2id(PAD_TOKEN)
        bs = hps.batch_size
        if len(example_list) > bs:
            raise ValueError(f"{len(example_list)} examples for batch_size {bs}")
        n_real = len(example_list)
        exs = list(example_list) + [example_list[-1]] * (bs - n_real)
        self.valid = np.zeros(bs, np.float32)
        self.valid[:n_real] = 1.0
        self.init_encoder_seq(exs, hps, pad_enc_to)
        self.init_decoder_seq(exs, hps)
        self.store_orig_strings(exs)

    def init_encoder_seq(self, exs, hps, pad_enc_to):
        bs = len(exs)
        L = max(ex.enc_len for ex in exs)
        if pad_enc_to:
            L = max(L, pad_enc_to)
        self.enc_lens = np.array([ex.enc_len for ex in exs], dtype=np.int32)
        self.enc_batch = np.full((bs, L), self.pad_id, dtype=np.int32)
        self.enc_batch_extend_vocab = np.full((bs, L), self.pad_id, dtype=np.int32)
        for i, ex in enumerate(exs):
            self.enc_batch[i, :ex.enc_len] = ex.enc_input
            self.enc_batch_extend_vocab[i, :ex.enc_len] = ex.enc_input_extend_vocab
        self.enc_padding_mask = (np.arange(L)[None, :] < self.enc_lens[:, None]).astype(np.float32)
        self.max_art_oovs = max(len(ex.article_oovs) for ex in exs)
        self.art_oovs = [ex.article_oovs for ex in exs]

    def init_decoder_seq(self, exs, hps):
        bs, D = len(exs), hps.max_dec_steps
        self.dec_batch = np.full((bs, D), self.pad_id, dtype=np.int32)
        self.target_batch = np.full((bs, D), self.pad_id, dtype=np.int32)
        for i, ex in enumerate(exs):
            self.dec_batch[i, :ex.dec_len] = ex.dec_input
            self.target_batch[i, :len(ex.target)] = ex.target
        self.dec_lens = np.array([ex.dec_len for ex in exs], dtype=np.int32)
        self.dec_padding_mask = (np.arange(D)[None, :] < self.dec_lens[:, None]).astype(np.float32)

    def store_orig_strings(self, exs):
        self.original_articles = [ex.original_article for ex in exs]
        self.original_abstracts = [ex.original_abstract for ex in exs]
        self.original_abstracts_sents = [ex.original_abstract_sents for ex in exs]
        self.uuids = [ex.uuid for ex in exs]

    # ------------------------------------------------------------------ accounting
    @property
    def batch_size(self) -> int:
        return self.enc_batch.shape[0]

    def num_tokens(self) -> int:
        """Non-pad encoder + decoder tokens of the valid rows (BASELINE.md definition)."""
        v = self.valid > 0
        return int(self.enc_lens[v].sum() + self.dec_padding_mask[v].sum())

    def padded_tokens(self) -> int:
        return int(self.valid.sum() * (self.enc_batch.shape[1] + self.dec_batch.shape[1]))


FlinkBatch = Batch
