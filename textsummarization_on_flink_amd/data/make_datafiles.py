"""CNN / DailyMail preprocessing: ``.story`` files -> tokenized stories -> ``{train,val,test}.bin``
+ vocab + 1000-example chunks (reference ``data/cnn-dailymail/make_datafiles.py``).

Same output format and rules as the reference: lower-cased PTB tokens, a period appended to
lines that lack an end token, ``@highlight`` lines become ``<s> ... </s>`` abstract sentences,
splits chosen by the SHA1 of each story URL (``url_lists/all_{train,val,test}.txt``), vocab =
the 200k most frequent tokens of the training split (``word count`` lines).  Differences:
no Java / Stanford CoreNLP (the built-in PTB-style tokenizer), no TensorFlow (the
``tf.Example`` codec is ``example_proto``), tokenization runs in a process pool, and the story
counts are checked only when ``--check-counts`` is given (any subset works).

    python -m textsummarization_on_flink_amd.data.make_datafiles CNN_STORIES DM_STORIES \\
        --url-lists url_lists --out finished_files [--workers 8] [--check-counts]
"""
from __future__ import annotations

import argparse
import collections
import hashlib
import logging
import os
from concurrent.futures import ProcessPoolExecutor
from typing import Iterable, List, Optional, Sequence, Tuple

from .binfmt import CHUNK_SIZE, chunk_file, write_bin
from .tokenize import word_tokenize
from .vocab import SENTENCE_END, SENTENCE_START

log = logging.getLogger(__name__)
DM_SINGLE_CLOSE_QUOTE = "’"
DM_DOUBLE_CLOSE_QUOTE = "”"
END_TOKENS = [".", "!", "?", "...", "'", "`", '"', DM_SINGLE_CLOSE_QUOTE, DM_DOUBLE_CLOSE_QUOTE, ")"]
NUM_EXPECTED_CNN_STORIES = 92579
NUM_EXPECTED_DM_STORIES = 219506
VOCAB_SIZE = 200000


def _tokenize_line(line: str) -> str:
    if line.strip().startswith("@highlight"):  # CoreNLP leaves the marker intact
        return line.strip()
    return " ".join(word_tokenize(line, ptb_brackets=True))


def _tokenize_file(args: Tuple[str, str]) -> None:
    src, dst = args
    with open(src, encoding="utf-8", errors="replace") as f:
        lines = f.read().split("\n")
    with open(dst, "w", encoding="utf-8") as f:  # -preserveLines: one output line per input line
        f.write("\n".join(_tokenize_line(x) for x in lines))


def tokenize_stories(stories_dir: str, tokenized_dir: str, workers: int = 8) -> int:
    os.makedirs(tokenized_dir, exist_ok=True)
    stories = sorted(os.listdir(stories_dir))
    jobs = [(os.path.join(stories_dir, s), os.path.join(tokenized_dir, s)) for s in stories]
    if workers > 1 and len(jobs) > 1:
        with ProcessPoolExecutor(max_workers=workers) as ex:
            list(ex.map(_tokenize_file, jobs, chunksize=64))
    else:
        for j in jobs:
            _tokenize_file(j)
    n_tok = len(os.listdir(tokenized_dir))
    if n_tok != len(stories):
        raise RuntimeError(f"The tokenized stories directory {tokenized_dir} contains {n_tok} files, but it should "
                           f"contain the same number as {stories_dir} (which has {len(stories)} files).")
    return n_tok


def read_text_file(path: str) -> List[str]:
    with open(path, encoding="utf-8", errors="replace") as f:
        return [line.strip() for line in f]


def hashhex(s: str) -> str:
    return hashlib.sha1(s.encode("utf-8")).hexdigest()


def get_url_hashes(url_list: Sequence[str]) -> List[str]:
    return [hashhex(u) for u in url_list]


def fix_missing_period(line: str) -> str:
    if "@highlight" in line or line == "":
        return line
    if line[-1] in END_TOKENS or any(line.endswith(t) for t in END_TOKENS):
        return line
    return line + " ."


def get_art_abs(story_file: str) -> Tuple[str, str]:
    lines = [fix_missing_period(x.lower()) for x in read_text_file(story_file)]
    article_lines, highlights = [], []
    next_is_highlight = False
    for line in lines:
        if line == "":
            continue
        if line.startswith("@highlight"):
            next_is_highlight = True
        elif next_is_highlight:
            highlights.append(line)
        else:
            article_lines.append(line)
    article = " ".join(article_lines)
    abstract = " ".join(f"{SENTENCE_START} {s} {SENTENCE_END}" for s in highlights)
    return article, abstract


def write_to_bin(url_file: str, out_file: str, tokenized_dirs: Sequence[str], vocab_out: Optional[str] = None,
                 vocab_size: int = VOCAB_SIZE) -> int:
    url_hashes = get_url_hashes(read_text_file(url_file))
    counter = collections.Counter() if vocab_out else None

    def examples():
        for h in url_hashes:
            name = h + ".story"
            path = next((os.path.join(d, name) for d in tokenized_dirs if os.path.isfile(os.path.join(d, name))), None)
            if path is None:
                raise FileNotFoundError(f"Couldn't find tokenized story file {name} in {list(tokenized_dirs)}")
            article, abstract = get_art_abs(path)
            if counter is not None:
                toks = article.split(" ") + [t for t in abstract.split(" ") if t not in (SENTENCE_START, SENTENCE_END)]
                counter.update(t.strip() for t in toks if t.strip())
            yield {"article": article, "abstract": abstract}

    n = write_bin(out_file, examples())
    if counter is not None:
        with open(vocab_out, "w", encoding="utf-8") as f:
            for w, c in counter.most_common(vocab_size):
                f.write(f"{w} {c}\n")
    log.info("wrote %d examples to %s", n, out_file)
    return n


def chunk_all(finished_dir: str, splits: Iterable[str] = ("train", "val", "test"), chunk_size: int = CHUNK_SIZE):
    out = os.path.join(finished_dir, "chunked")
    return {s: chunk_file(os.path.join(finished_dir, f"{s}.bin"), out, s, chunk_size) for s in splits
            if os.path.exists(os.path.join(finished_dir, f"{s}.bin"))}


def check_num_stories(stories_dir: str, num_expected: int) -> None:
    n = len(os.listdir(stories_dir))
    if n != num_expected:
        raise RuntimeError(f"stories directory {stories_dir} contains {n} files but should contain {num_expected}")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("cnn_stories_dir")
    ap.add_argument("dm_stories_dir")
    ap.add_argument("--url-lists", default="url_lists")
    ap.add_argument("--out", default="finished_files")
    ap.add_argument("--tokenized-root", default=".")
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--check-counts", action="store_true")
    ap.add_argument("--vocab-size", type=int, default=VOCAB_SIZE)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    if a.check_counts:
        check_num_stories(a.cnn_stories_dir, NUM_EXPECTED_CNN_STORIES)
        check_num_stories(a.dm_stories_dir, NUM_EXPECTED_DM_STORIES)
    cnn_tok = os.path.join(a.tokenized_root, "cnn_stories_tokenized")
    dm_tok = os.path.join(a.tokenized_root, "dm_stories_tokenized")
    os.makedirs(a.out, exist_ok=True)
    tokenize_stories(a.cnn_stories_dir, cnn_tok, a.workers)
    tokenize_stories(a.dm_stories_dir, dm_tok, a.workers)
    dirs = [cnn_tok, dm_tok]
    write_to_bin(os.path.join(a.url_lists, "all_test.txt"), os.path.join(a.out, "test.bin"), dirs)
    write_to_bin(os.path.join(a.url_lists, "all_val.txt"), os.path.join(a.out, "val.bin"), dirs)
    write_to_bin(os.path.join(a.url_lists, "all_train.txt"), os.path.join(a.out, "train.bin"), dirs,
                 vocab_out=os.path.join(a.out, "vocab"), vocab_size=a.vocab_size)
    chunk_all(a.out)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
