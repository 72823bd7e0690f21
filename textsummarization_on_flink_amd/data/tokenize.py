"""Dependency-free tokenizers replacing Stanford CoreNLP PTBTokenizer
(``make_datafiles.py:67-87``) and nltk ``punkt`` sent/word tokenization
(``batcher.py:389,462,579,643``; ``util.py:88``) -- SURVEY N6/N8.

PTB-style rules: split punctuation, quotes -> `` '' , contractions ('s n't 're 've 'll
'd 'm) split off, brackets -> -LRB- -RRB- -LSB- -RSB- -LCB- -RCB- (CoreNLP's defaults,
which is what the CNN/DM vocab was built with) and lower-casing is done by the caller
(``make_datafiles.py:121``).  Sentence splitting breaks after . ! ? (optionally followed
by closing quotes/brackets) when the next token starts a new sentence, with a small
abbreviation list, which is what punkt does on news text in practice.
"""
from __future__ import annotations

import re
from typing import List

_BRACKETS = {"(": "-LRB-", ")": "-RRB-", "[": "-LSB-", "]": "-RSB-", "{": "-LCB-", "}": "-RCB-"}
_ABBREV = {"mr", "mrs", "ms", "dr", "prof", "sr", "jr", "st", "vs", "etc", "inc", "ltd", "co", "corp", "jan", "feb",
           "mar", "apr", "jun", "jul", "aug", "sep", "sept", "oct", "nov", "dec", "u.s", "u.k", "no", "gen", "gov",
           "sen", "rep", "lt", "col", "sgt", "capt", "rev", "mt", "ft", "a.m", "p.m", "e.g", "i.e"}

_TOKEN_RE = re.compile(
    r"""(?x)
    (?:[A-Za-z]\.){2,}(?=\s|$)            # acronyms u.s.
  | \$?\d+(?:[.,:]\d+)*%?                  # numbers, money, times
  | [A-Za-z0-9]+(?:[-'][A-Za-z0-9]+)*(?:n't)?   # words incl. hyphens (contractions split below)
  | \.\.\.|--
  | ``|''
  | [^\sA-Za-z0-9]                         # any other single symbol
    """)
_CONTRACTION = re.compile(r"(?i)^(.+?)(n't|'s|'re|'ve|'ll|'d|'m)$")


def word_tokenize(text: str, ptb_brackets: bool = False) -> List[str]:
    text = re.sub(r'^"', "`` ", text)
    text = re.sub(r'(?<=[\s(\[{<])"', " `` ", text)
    text = text.replace('"', " '' ")
    out: List[str] = []
    append = out.append
    for tok in _TOKEN_RE.findall(text):
        if "'" in tok:  # every contraction suffix holds an apostrophe: the regex only runs on those
            low = tok.lower()
            m = _CONTRACTION.match(tok)
            if m and len(m.group(1)) > 0 and low != "can't":
                out.extend([m.group(1), m.group(2)])
            elif low == "can't":
                out.extend([tok[:2], tok[2:]])
            elif ptb_brackets and tok in _BRACKETS:
                append(_BRACKETS[tok])
            else:
                append(tok)
        elif ptb_brackets and tok in _BRACKETS:
            append(_BRACKETS[tok])
        else:
            append(tok)
    return out


def sent_tokenize(text: str) -> List[str]:
    sents, cur = [], []
    toks = text.split()
    for i, tok in enumerate(toks):
        cur.append(tok)
        core = tok.rstrip("\"')]}'")
        if core.endswith(("!", "?")) or (core.endswith(".") and core[:-1].lower().rstrip(".") not in _ABBREV
                                          and not re.fullmatch(r"(?:[A-Za-z]\.)+", core)):
            nxt = toks[i + 1] if i + 1 < len(toks) else None
            if nxt is None or nxt[:1].isupper() or nxt[:1] in "\"'`(" or nxt[:1].isdigit():
                sents.append(" ".join(cur))
                cur = []
    if cur:
        sents.append(" ".join(cur))
    return sents


def ptb_tokenize_lower(text: str) -> str:
    """What make_datafiles produces per line: PTB tokens, lower-cased, space-joined."""
    return " ".join(word_tokenize(text, ptb_brackets=True)).lower()
