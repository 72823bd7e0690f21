"""Vocabulary and OOV helpers (reference ``data.py:25-276``).

Ids 0-3 are reserved for ``[UNK] [PAD] [START] [STOP]`` (``data.py:50-54``); the vocab file
holds ``word count`` lines sorted by frequency and is read up to ``max_size`` ids
*including* the four specials (``data.py:71``).
"""
from __future__ import annotations

import csv
import logging
from typing import Iterable, List, Optional, Sequence, Tuple

log = logging.getLogger(__name__)

SENTENCE_START = "<s>"
SENTENCE_END = "</s>"
PAD_TOKEN = "[PAD]"
UNKNOWN_TOKEN = "[UNK]"
START_DECODING = "[START]"
STOP_DECODING = "[STOP]"
SPECIALS = [UNKNOWN_TOKEN, PAD_TOKEN, START_DECODING, STOP_DECODING]


class Vocab:
    def __init__(self, vocab_file: Optional[str] = None, max_size: int = 0, words: Optional[Iterable[str]] = None):
        self._word_to_id = {}
        self._id_to_word = []
        for w in SPECIALS:
            self._add(w)
        src = words
        if vocab_file is not None:
            src = self._read(vocab_file)
        for w in src or ():
            if w in (SENTENCE_START, SENTENCE_END, *SPECIALS):
                raise ValueError(f"<s>, </s>, [UNK], [PAD], [START] and [STOP] shouldn't be in the vocab file, but {w} is")
            if w in self._word_to_id:
                raise ValueError(f"Duplicated word in vocabulary file: {w}")
            self._add(w)
            if max_size != 0 and len(self._id_to_word) >= max_size:
                break

    @staticmethod
    def _read(path):
        with open(path, "r", encoding="utf-8") as f:
            for line in f:
                pieces = line.split()
                if len(pieces) != 2:
                    log.warning("incorrectly formatted line in vocabulary file: %r", line)
                    continue
                yield pieces[0]

    def _add(self, w):
        self._word_to_id[w] = len(self._id_to_word)
        self._id_to_word.append(w)

    def word2id(self, word: str) -> int:
        return self._word_to_id.get(word, 0)

    def ids(self, words: Sequence[str]) -> List[int]:
        """word2id over a token list (one bound dict lookup per token: the host loader's
        hot loop)."""
        get = self._word_to_id.get
        return [get(w, 0) for w in words]

    def id2word(self, word_id: int) -> str:
        if not 0 <= word_id < len(self._id_to_word):
            raise ValueError(f"Id not found in vocab: {word_id}")
        return self._id_to_word[word_id]

    def size(self) -> int:
        return len(self._id_to_word)

    def __len__(self):
        return self.size()

    @property
    def words(self) -> List[str]:
        return list(self._id_to_word)

    def write_metadata(self, fpath: str) -> None:
        """TensorBoard embedding-projector metadata (``data.py:93-105``)."""
        with open(fpath, "w", encoding="utf-8", newline="") as f:
            w = csv.DictWriter(f, delimiter="\t", fieldnames=["word"])
            for i in range(self.size()):
                w.writerow({"word": self._id_to_word[i]})

    def save(self, fpath: str, counts: Optional[Sequence[int]] = None) -> None:
        with open(fpath, "w", encoding="utf-8") as f:
            for i, w in enumerate(self._id_to_word[4:]):
                f.write(f"{w} {counts[i] if counts else 1}\n")


def article2ids(article_words: Sequence[str], vocab: Vocab,
                ids: Optional[Sequence[int]] = None) -> Tuple[List[int], List[str]]:
    """In-article OOVs get temporary ids vocab.size()+k (``data.py:144-168``).  ``ids``:
    the words' plain vocab ids if already computed (only the [UNK] positions are revisited)."""
    out = list(vocab.ids(article_words) if ids is None else ids)
    oovs: List[str] = []
    if 0 not in out:
        return out, oovs
    index = {}
    V = vocab.size()
    for k, i in enumerate(out):
        if i == 0:
            w = article_words[k]
            if w not in index:
                index[w] = len(oovs)
                oovs.append(w)
            out[k] = V + index[w]
    return out, oovs


def abstract2ids(abstract_words: Sequence[str], vocab: Vocab, article_oovs: Sequence[str],
                 ids: Optional[Sequence[int]] = None) -> List[int]:
    """In-article OOVs -> temporary id; other OOVs -> [UNK] (``data.py:171-193``)."""
    out = list(vocab.ids(abstract_words) if ids is None else ids)
    if not article_oovs or 0 not in out:
        return out
    index = {w: k for k, w in reversed(list(enumerate(article_oovs)))}
    V = vocab.size()
    for k, i in enumerate(out):
        if i == 0:
            w = abstract_words[k]
            out[k] = V + index[w] if w in index else 0
    return out


def outputids2words(id_list: Sequence[int], vocab: Vocab, article_oovs: Optional[Sequence[str]]) -> List[str]:
    """Map ids (incl. temporary OOV ids) back to words (``data.py:196-219``)."""
    words = []
    V = vocab.size()
    table = vocab._id_to_word
    for i in id_list:
        i = int(i)
        if 0 <= i < V:
            words.append(table[i])
        elif i < 0:
            raise ValueError(f"Id not found in vocab: {i}")
        else:
            if article_oovs is None:
                raise ValueError("model produced a word ID that isn't in the vocabulary (baseline mode)")
            k = i - V
            if k >= len(article_oovs):
                raise ValueError(f"model produced word ID {i} which corresponds to article OOV {k} but this example "
                                 f"only has {len(article_oovs)} article OOVs")
            words.append(article_oovs[k])
    return words


def abstract2sents(abstract: str) -> List[str]:
    """Split ``<s> ... </s>`` tagged abstract text into sentences (``data.py:222-239``)."""
    cur, sents = 0, []
    while True:
        try:
            start_p = abstract.index(SENTENCE_START, cur)
            end_p = abstract.index(SENTENCE_END, start_p + 1)
        except ValueError:
            return sents
        cur = end_p + len(SENTENCE_END)
        sents.append(abstract[start_p + len(SENTENCE_START):end_p])


def show_art_oovs(article: str, vocab: Vocab) -> str:
    """Highlight article OOVs as __w__ (``data.py:242-248``)."""
    return " ".join(("__%s__" % w) if vocab.word2id(w) == 0 else w for w in article.split(" "))


def show_abs_oovs(abstract: str, vocab: Vocab, article_oovs: Optional[Sequence[str]]) -> str:
    """Highlight abstract OOVs; non-article OOVs as !!__w__!! (``data.py:251-276``)."""
    out = []
    for w in abstract.split(" "):
        if vocab.word2id(w) == 0:
            if article_oovs is None or w in article_oovs:
                out.append("__%s__" % w)
            else:
                out.append("!!__%s__!!" % w)
        else:
            out.append(w)
    return " ".join(out)
