"""Data layer parity: Vocab, OOV maps, tf.Example codec, .bin chunks, Example/Batch."""
import os

import numpy as np
import pytest

from textsummarization_on_flink_amd.config import HParams
from textsummarization_on_flink_amd.data import binfmt
from textsummarization_on_flink_amd.data.batch import Batch, Example
from textsummarization_on_flink_amd.data.example_proto import decode_example, encode_example, get_text
from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus
from textsummarization_on_flink_amd.data.tokenize import sent_tokenize, word_tokenize
from textsummarization_on_flink_amd.data.vocab import (Vocab, abstract2ids, abstract2sents, article2ids,
                                                       outputids2words, show_abs_oovs, show_art_oovs)


@pytest.fixture
def vocab(tmp_path):
    p = tmp_path / "vocab"
    p.write_text("the 100\ncat 50\nsat 40\non 30\nmat 20\n.  10\nbadline\n")
    return Vocab(str(p), 0)


def test_vocab_reserved_ids_and_limits(vocab, tmp_path):
    assert [vocab.word2id(w) for w in ["[UNK]", "[PAD]", "[START]", "[STOP]"]] == [0, 1, 2, 3]
    assert vocab.word2id("the") == 4 and vocab.word2id("zzz") == 0
    assert vocab.size() == 10  # 4 specials + 6 words (malformed line skipped)
    p = tmp_path / "v2"
    p.write_text("\n".join(f"w{i} 1" for i in range(10)))
    assert Vocab(str(p), 7).size() == 7  # max_size counts the specials (data.py:71)
    with pytest.raises(ValueError):
        Vocab(words=["a", "a"])
    with pytest.raises(ValueError):
        Vocab(words=["<s>"])
    with pytest.raises(ValueError):
        vocab.id2word(99)


def test_oov_maps(vocab):
    ids, oovs = article2ids("the dog sat on the fox dog".split(), vocab)
    V = vocab.size()
    assert oovs == ["dog", "fox"]
    assert ids == [4, V, 6, 7, 4, V + 1, V]
    assert abstract2ids("dog cow the".split(), vocab, oovs) == [V, 0, 4]
    assert outputids2words([4, V + 1, 3], vocab, oovs) == ["the", "fox", "[STOP]"]
    with pytest.raises(ValueError):
        outputids2words([V + 5], vocab, oovs)
    assert show_art_oovs("the dog", vocab) == "the __dog__"
    assert show_abs_oovs("dog cow", vocab, ["dog"]) == "__dog__ !!__cow__!!"


def test_abstract2sents():
    assert abstract2sents("<s> a b . </s> <s> c . </s>") == [" a b . ", " c . "]
    assert abstract2sents("no tags") == []


def test_example_proto_roundtrip():
    ex = {"article": "a b c", "abstract": b"<s> x </s>", "n": [1, -2, 3], "f": [0.5, 1.5]}
    d = decode_example(encode_example(ex))
    assert get_text(d, "article") == "a b c" and d["abstract"] == [b"<s> x </s>"]
    assert d["n"] == [1, -2, 3] and d["f"] == [0.5, 1.5]


def test_bin_roundtrip_and_chunk(tmp_path):
    exs = [{"article": f"art {i}", "abstract": f"<s> abs {i} </s>"} for i in range(25)]
    p = tmp_path / "all.bin"
    assert binfmt.write_bin(str(p), exs) == 25
    chunks = binfmt.chunk_file(str(p), str(tmp_path / "chunked"), "train", chunk_size=10)
    assert [os.path.basename(c) for c in chunks] == ["train_000.bin", "train_001.bin", "train_002.bin"]
    got = list(binfmt.text_generator(binfmt.example_generator(str(tmp_path / "chunked" / "train_*"), True)))
    assert got[0] == ("art 0", "<s> abs 0 </s>") and len(got) == 25
    n = binfmt.bin2txt(str(tmp_path / "chunked" / "train_*"), str(tmp_path / "json"))
    assert n == 25
    import json
    line = open(tmp_path / "json" / "train_000.txt").readline()
    msg = json.loads(line)
    assert list(msg) == ["uuid", "article", "summary", "reference"] and msg["uuid"] == "uuid-0"


def test_example_semantics(vocab):
    hps = HParams(max_enc_steps=4, max_dec_steps=5, batch_size=2)
    ex = Example("the cat sat on the mat", ["the dog sat ."], vocab, hps)
    assert ex.enc_len == 4 and ex.enc_input == [4, 5, 6, 7]
    assert ex.dec_input == [2, 4, 0, 6, 9]  # [START] the [UNK] sat .
    assert ex.target == [4, 0, 6, 9, 3]       # ... [STOP]
    ex2 = Example("the dog sat", ["dog sat the cat the the ."], vocab, hps)
    V = vocab.size()
    assert ex2.article_oovs == ["dog"]
    assert ex2.target == [V, 6, 4, 5, 4]      # truncated: no [STOP]; in-article OOV -> V
    assert ex2.dec_input == [2, 0, 6, 4, 5]


def test_batch_padding_masks_and_short_batch(vocab):
    hps = HParams(max_enc_steps=6, max_dec_steps=5, batch_size=3)
    exs = [Example("the cat", ["cat ."], vocab, hps), Example("the cat sat on", ["sat"], vocab, hps)]
    b = Batch(exs, hps, vocab)
    assert b.enc_batch.shape == (3, 4)
    np.testing.assert_array_equal(b.enc_lens, [2, 4, 4])
    np.testing.assert_array_equal(b.enc_padding_mask[0], [1, 1, 0, 0])
    np.testing.assert_array_equal(b.enc_batch[0], [4, 5, 1, 1])
    np.testing.assert_array_equal(b.valid, [1, 1, 0])
    np.testing.assert_array_equal(b.dec_padding_mask[0], [1, 1, 1, 0, 0])
    assert b.target_batch[0].tolist() == [5, 9, 3, 1, 1]
    b2 = Batch(exs, hps, vocab, pad_enc_to=6)
    assert b2.enc_batch.shape == (3, 6)
    assert b.num_tokens() == 2 + 4 + 3 + 2


def test_tokenizers():
    assert word_tokenize("He said \"don't go\" (now).") == ["He", "said", "``", "do", "n't", "go", "''", "(", "now",
                                                          ")", "."]
    assert sent_tokenize("Mr. Smith went. Then he left! OK") == ["Mr. Smith went.", "Then he left!", "OK"]


def test_synthetic_shapes():
    c = SyntheticCorpus(vocab_size=1000, raw_vocab=5000, seed=3)
    lens = [len(c.sample()[0].split()) for _ in range(200)]
    assert 500 < np.mean(lens) < 1000
    art, abs_ = c.sample()
    assert abs_.startswith("<s>") and len(abstract2sents(abs_)) >= 3
