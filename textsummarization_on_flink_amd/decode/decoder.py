"""BeamSearchDecoder: decode loop, outputs and result sinks (reference ``decode.py:39-313``).

Per example: beam search -> ids -> words (in-article OOVs restored) -> cut at the first
[STOP] -> one of
  * ``write_for_flink``: sentences split at "." joined with two spaces, handed to the
    result writer as ``(uuid, article, summary, reference)`` (streaming serving);
  * ``write_for_rouge``: ``decoded/%06d_decoded.txt`` + ``reference/%06d_reference.txt``,
    one sentence per line, then ROUGE at the end of a single pass;
  * ``write_for_attnvis``: ``attn_vis_data.json`` for the attention visualiser.
``make_html_safe`` reproduces the reference's no-op by default (its ``str.replace``
results are discarded); ``html_escape=True`` fixes it.

Two engines plug in: the host beam search over a step model (CPU oracle, or any
``StepModel``) and the batched device beam search (``decode.device_beam``), which decodes
many articles per hipGraph replay and returns the same Hypothesis objects.
"""
from __future__ import annotations

import json
import logging
import os
import shutil
import time
from typing import List, Optional

from ..data import vocab as V
from . import rouge
from .beam_search import run_beam_search

log = logging.getLogger(__name__)
SECS_UNTIL_NEW_CKPT = 60


def make_html_safe(s: str, escape: bool = False) -> str:
    if escape:
        return s.replace("<", "&lt;").replace(">", "&gt;")
    s.replace("<", "&lt;")  # reference behaviour: results discarded (decode.py:261-265)
    s.replace(">", "&gt;")
    return s


def split_sentences(decoded_words: List[str]) -> List[str]:
    """Cut the decoded word list into sentences ending in "." (decode.py:166-174)."""
    sents, words = [], list(decoded_words)
    while words:
        try:
            idx = words.index(".")
        except ValueError:
            idx = len(words)
        sents.append(" ".join(words[:idx + 1]))
        words = words[idx + 1:]
    return sents


def decoded_words(ids: List[int], vocab, article_oovs) -> List[str]:
    """Token ids after [START] -> words (in-article OOVs restored), cut at the first [STOP]."""
    words = V.outputids2words([int(t) for t in ids], vocab, article_oovs)
    if V.STOP_DECODING in words:
        words = words[:words.index(V.STOP_DECODING)]
    return words


def flink_summary(ids: List[int], vocab, article_oovs, reference_sents, html_escape: bool = False):
    """(summary, reference) of a result row (decode.py:159-185): sentences of the decoded words
    joined with two spaces, reference sentences joined with one."""
    dec = [make_html_safe(s, html_escape) for s in split_sentences(decoded_words(ids, vocab, article_oovs))]
    refs = [make_html_safe(s, html_escape) for s in reference_sents]
    return "  ".join(dec), " ".join(refs)


def get_decode_dir_name(hps, ckpt_name: Optional[str]) -> str:
    dp = hps.data_path
    if "train" in dp:
        dataset = "train"
    elif "val" in dp:
        dataset = "val"
    elif "test" in dp:
        dataset = "test"
    else:
        raise ValueError("FLAGS.data_path %s should contain one of train, val or test" % dp)
    name = "decode_%s_%imaxenc_%ibeam_%imindec_%imaxdec" % (dataset, hps.max_enc_steps, hps.beam_size,
                                                             hps.min_dec_steps, hps.max_dec_steps)
    if ckpt_name is not None:
        name += "_%s" % ckpt_name
    return name


class NullWriter:
    """AbstractWriter (flink_writer.py:6-14): used when not serving into a stream."""

    def write_result(self, uuid, article, summary, reference):
        return

    def close(self):
        return


class BeamSearchDecoder:
    def __init__(self, step_model, batcher, vocab, hps, writer=None, decode_dir: Optional[str] = None,
                 ckpt_name: Optional[str] = None, html_escape: bool = False, device_beam=None, reload_fn=None):
        self.model = step_model
        self.batcher = batcher
        self.vocab = vocab
        self.hps = hps
        self.writer = writer or NullWriter()
        self.device_beam = device_beam
        self.html_escape = html_escape
        self.reload_fn = reload_fn
        self.counter = 0
        self.decode_dir = decode_dir
        if decode_dir is None and hps.log_root:
            if hps.single_pass:
                self.decode_dir = os.path.join(hps.log_root, get_decode_dir_name(hps, ckpt_name))
                if os.path.exists(self.decode_dir):
                    shutil.rmtree(self.decode_dir)
            else:
                self.decode_dir = os.path.join(hps.log_root, "decode")
        if self.decode_dir:
            os.makedirs(self.decode_dir, exist_ok=True)
            self.rouge_ref_dir = os.path.join(self.decode_dir, "reference")
            self.rouge_dec_dir = os.path.join(self.decode_dir, "decoded")
            if hps.single_pass:
                os.makedirs(self.rouge_ref_dir, exist_ok=True)
                os.makedirs(self.rouge_dec_dir, exist_ok=True)

    # ------------------------------------------------------------------ per example
    def hyp_to_words(self, best, batch, row: int = 0) -> List[str]:
        return decoded_words(best.tokens[1:], self.vocab, batch.art_oovs[row] if self.hps.pointer_gen else None)

    def handle(self, best, batch, row: int = 0, mode: str = "auto"):
        words = self.hyp_to_words(best, batch, row)
        article = batch.original_articles[row]
        abstract = batch.original_abstracts[row]
        abstract_sents = batch.original_abstracts_sents[row]
        uuid = batch.uuids[row] if batch.uuids[row] is not None else "uuid-%d" % self.counter
        if mode == "auto":
            mode = "flink" if not isinstance(self.writer, NullWriter) else ("rouge" if self.hps.single_pass else "vis")
        if mode == "flink":
            self.write_for_flink(uuid, article, words, abstract_sents)
        elif mode == "rouge":
            self.write_for_rouge(abstract_sents, words, self.counter)
        else:
            art_unk = V.show_art_oovs(article, self.vocab)
            abs_unk = V.show_abs_oovs(abstract, self.vocab, batch.art_oovs[row] if self.hps.pointer_gen else None)
            log.info("ARTICLE:  %s", art_unk)
            log.info("REFERENCE SUMMARY: %s", abs_unk)
            log.info("GENERATED SUMMARY: %s", " ".join(words))
            if self.decode_dir:
                self.write_for_attnvis(art_unk, abs_unk, words, best.attn_dists, best.p_gens)
        self.counter += 1
        return words

    def decode_one_batch(self, batch, mode="auto"):
        best = run_beam_search(self.model, self.vocab, batch, self.hps)
        return self.handle(best, batch, 0, mode)

    # ------------------------------------------------------------------ loops
    def decode(self, with_rouge: bool = True, max_examples: Optional[int] = None):
        t0 = time.time()
        self.counter = 0
        if self.device_beam is not None and self.hps.single_pass and isinstance(self.writer, NullWriter):
            # pipelined device decode: batch i's summaries are written while batch i+1 runs on
            # the GPU.  Offline single pass only: no checkpoint reload falls between batches,
            # and batch i's results wait for batch i+1 to be fetched -- a streaming source
            # (flink writer) must emit each batch as soon as it is decoded (Issue-6 analogue)
            self._decode_pipelined(max_examples)
            return self._finish_decode(with_rouge)
        while max_examples is None or self.counter < max_examples:
            if self.device_beam is not None:
                batch = self.batcher.next_batch()  # n_articles distinct examples per batch
                if batch is None:
                    break
                for row, best in enumerate(self.device_beam.decode(batch)):
                    self.handle(best, batch, row)
            else:
                batch = self.batcher.next_batch()
                if batch is None:
                    break
                self.decode_one_batch(batch)
            if not self.hps.single_pass and self.reload_fn and time.time() - t0 > SECS_UNTIL_NEW_CKPT:
                self.reload_fn()
                t0 = time.time()
        return self._finish_decode(with_rouge)

    def _decode_pipelined(self, max_examples: Optional[int]):
        queued = []

        def batches():
            n = 0
            while max_examples is None or n < max_examples:
                batch = self.batcher.next_batch()  # n_articles distinct examples per batch
                if batch is None:
                    return
                n += int(batch.valid.sum())
                queued.append(batch)
                yield batch

        for hyps in self.device_beam.decode_batches(batches()):
            batch = queued.pop(0)
            for row, best in enumerate(hyps):
                self.handle(best, batch, row)

    def _finish_decode(self, with_rouge: bool):
        if self.hps.single_pass and with_rouge and isinstance(self.writer, NullWriter) and self.decode_dir:
            res = rouge.rouge_eval(self.rouge_ref_dir, self.rouge_dec_dir)
            log.info(rouge.rouge_log(res, self.decode_dir))
            return res
        return None

    # ------------------------------------------------------------------ writers
    def write_for_flink(self, uuid, article, words, reference_sents):
        dec = [make_html_safe(s, self.html_escape) for s in split_sentences(words)]
        refs = [make_html_safe(s, self.html_escape) for s in reference_sents]
        self.writer.write_result(uuid, article, "  ".join(dec), " ".join(refs))

    def write_for_rouge(self, reference_sents, decoded_words, ex_index):
        dec = [make_html_safe(s, self.html_escape) for s in split_sentences(decoded_words)]
        refs = [make_html_safe(s, self.html_escape) for s in reference_sents]
        with open(os.path.join(self.rouge_ref_dir, "%06d_reference.txt" % ex_index), "w") as f:
            f.write("\n".join(refs))
        with open(os.path.join(self.rouge_dec_dir, "%06d_decoded.txt" % ex_index), "w") as f:
            f.write("\n".join(dec))

    def write_for_attnvis(self, article, abstract, decoded_words, attn_dists, p_gens):
        to_write = {
            "article_lst": [make_html_safe(t, self.html_escape) for t in article.split()],
            "decoded_lst": [make_html_safe(t, self.html_escape) for t in decoded_words],
            "abstract_str": make_html_safe(abstract, self.html_escape),
            "attn_dists": [[float(x) for x in a] for a in attn_dists],
        }
        if self.hps.pointer_gen:
            to_write["p_gens"] = [float(p) if p is not None else None for p in p_gens]
        path = os.path.join(self.decode_dir, "attn_vis_data.json")
        with open(path, "w") as f:
            json.dump(to_write, f)
        return path
