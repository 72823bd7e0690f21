"""CNN/DM preprocessing pipeline (make_datafiles.py parity) on a handful of fake stories."""
import os

from textsummarization_on_flink_amd.data import binfmt
from textsummarization_on_flink_amd.data import make_datafiles as M
from textsummarization_on_flink_amd.data.example_proto import get_text
from textsummarization_on_flink_amd.data.vocab import Vocab


def _story(i):
    return (f"(CNN) -- Story number {i} says \"hello\" to the world\n\nIt was great. Wasn't it\n\n"
            f"@highlight\n\nFirst highlight {i}\n\n@highlight\n\nSecond one!\n")


def test_pipeline(tmp_path):
    cnn, dm, urls, out = tmp_path / "cnn", tmp_path / "dm", tmp_path / "url_lists", tmp_path / "finished"
    for d in (cnn, dm, urls):
        d.mkdir()
    split_urls = {"train": [], "val": [], "test": []}
    for i in range(9):
        url = f"http://example.com/story{i}"
        src = cnn if i % 2 else dm
        (src / (M.hashhex(url) + ".story")).write_text(_story(i))
        split_urls[["train", "val", "test"][i % 3]].append(url)
    for k, v in split_urls.items():
        (urls / f"all_{k}.txt").write_text("\n".join(v) + "\n")
    assert M.main([str(cnn), str(dm), "--url-lists", str(urls), "--out", str(out), "--tokenized-root",
                   str(tmp_path), "--workers", "2"]) == 0
    exs = list(binfmt.example_generator(str(out / "train.bin"), single_pass=True))
    assert len(exs) == 3
    art, abs_ = get_text(exs[0], "article"), get_text(exs[0], "abstract")
    assert art.startswith("-lrb- cnn -rrb- -- story number 0 says `` hello '' to the world .")
    assert "was n't it ." in art  # contraction split, missing period fixed
    assert abs_ == "<s> first highlight 0 . </s> <s> second one ! </s>"
    v = Vocab(str(out / "vocab"), 0)
    assert v.word2id("story") > 3 and v.word2id("<s>") == 0
    assert os.path.exists(out / "chunked" / "train_000.bin") and os.path.exists(out / "chunked" / "test_000.bin")
