"""CNN/DailyMail ``.bin`` chunk format (reference ``data.py:108-141``,
``make_datafiles.py:36-64,183-189``, ``util.py:44-99``).

A file is a sequence of ``<int64 native-endian length><serialized tf.Example>`` records,
1000 examples per chunk.  ``example_generator`` mirrors the reference's infinite shuffled
/ single-pass ordered reader.
"""
from __future__ import annotations

import glob
import json
import logging
import os
import random
import struct
from collections import OrderedDict
from typing import Dict, Iterator, List, Optional, Tuple

from .example_proto import decode_example, encode_example, get_text
from .vocab import abstract2sents

log = logging.getLogger(__name__)
CHUNK_SIZE = 1000  # make_datafiles.py:33


def write_bin(path: str, examples) -> int:
    """Write ``examples`` (dicts of features, or pre-serialized bytes) as a .bin file."""
    n = 0
    with open(path, "wb") as f:
        for ex in examples:
            s = ex if isinstance(ex, (bytes, bytearray)) else encode_example(ex)
            f.write(struct.pack("q", len(s)))
            f.write(s)
            n += 1
    return n


def read_bin(path: str) -> Iterator[bytes]:
    with open(path, "rb") as f:
        while True:
            lb = f.read(8)
            if not lb:
                return
            if len(lb) < 8:
                raise ValueError(f"truncated length prefix in {path}")
            (n,) = struct.unpack("q", lb)
            s = f.read(n)
            if len(s) != n:
                raise ValueError(f"truncated record in {path}")
            yield s


def example_generator(data_path: str, single_pass: bool, rng: Optional[random.Random] = None,
                      decode: bool = True, shard: Tuple[int, int] = (0, 1)) -> Iterator[Dict[str, List]]:
    """Yield decoded tf.Examples (raw records with ``decode=False``); forever in shuffled
    file order unless single_pass.

    ``shard = (index, count)``: only the records k of each pass with k % count == index (k
    counts records in the pass's file order).  Readers that share ``rng``'s seed walk the same
    file order, so ``count`` of them with distinct indices see disjoint records that together
    cover every record once per pass -- the data-parallel split of the reference's Flink
    job, where each of ``worker_num`` flatMap instances receives its own share of the row
    stream (``doc/deprecated/About StreamExeEnv in AI-Extended Issue.md:68-74``)."""
    rng = rng or random.Random()
    index, count = shard
    if not 0 <= index < count:
        raise ValueError(f"bad shard {shard}")
    while True:
        filelist = glob.glob(data_path)
        if not filelist:
            raise FileNotFoundError(f"Error: Empty filelist at {data_path}")
        if single_pass:
            filelist = sorted(filelist)
        else:
            rng.shuffle(filelist)
        k = 0
        for fn in filelist:
            for rec in read_bin(fn):
                mine = k % count == index
                k += 1
                if mine:
                    yield decode_example(rec) if decode else rec
        if single_pass:
            log.info("example_generator completed reading all datafiles. No more data.")
            return


def text_generator(examples: Iterator[Dict[str, List]]) -> Iterator[Tuple[str, str]]:
    """(article, abstract) text pairs; empty articles skipped (``batcher.py:363-379``)."""
    for e in examples:
        if "article" not in e or "abstract" not in e:
            log.error("Failed to get article or abstract from example")
            continue
        art, abs_ = get_text(e, "article"), get_text(e, "abstract")
        if len(art) == 0:
            log.warning("Found an example with empty article text. Skipping it.")
            continue
        yield art, abs_


def chunk_file(in_file: str, out_dir: str, set_name: str, chunk_size: int = CHUNK_SIZE) -> List[str]:
    """Split one big .bin into ``{set}_{idx:03d}.bin`` chunks (``make_datafiles.py:36-53``)."""
    os.makedirs(out_dir, exist_ok=True)
    out, buf, idx = [], [], 0
    for rec in read_bin(in_file):
        buf.append(rec)
        if len(buf) == chunk_size:
            p = os.path.join(out_dir, "%s_%03d.bin" % (set_name, idx))
            write_bin(p, buf)
            out.append(p)
            buf, idx = [], idx + 1
    if buf:
        p = os.path.join(out_dir, "%s_%03d.bin" % (set_name, idx))
        write_bin(p, buf)
        out.append(p)
    return out


def bin2txt(data_path: str, finished_dir: str, sent_tokenize=None, word_tokenize=None) -> int:
    """Convert .bin chunks to JSONL ``{uuid, article, summary, reference}`` messages for the
    streaming source (``util.py:44-99``).  The reference is re-tokenized like the reference
    does with nltk (sentence split + word tokenize)."""
    from .tokenize import sent_tokenize as st, word_tokenize as wt
    sent_tokenize = sent_tokenize or st
    word_tokenize = word_tokenize or wt
    os.makedirs(finished_dir, exist_ok=True)
    counter = 0
    for fn in sorted(glob.glob(data_path)):
        outp = os.path.join(finished_dir, os.path.basename(fn).replace(".bin", ".txt"))
        with open(outp, "w", encoding="utf-8") as w:
            for art, abs_ in text_generator(decode_example(r) for r in read_bin(fn)):
                sents = [s.strip() for s in abstract2sents(abs_)]
                abstract = " ".join(sents)
                ref = " ".join(" ".join(word_tokenize(s)) for s in sent_tokenize(abstract))
                w.write(json.dumps(OrderedDict([("uuid", "uuid-%i" % counter), ("article", art), ("summary", ""),
                                                ("reference", ref)])))
                w.write("\n")
                counter += 1
    return counter
