"""Pure-Python ROUGE-1/2/L (replaces ROUGE-1.5.5 via pyrouge, ``decode.py:268-301``).

Follows ROUGE-1.5.5's conventions where they matter for the reported numbers:
tokens are lower-cased alphanumeric runs (``-U``-style non-alphanumerics removed),
ROUGE-N counts clipped n-gram overlap over all summary sentences, ROUGE-L is the
summary-level union-LCS over sentences, per-document P/R/F (F with alpha = 0.5) are
macro-averaged, and 95% confidence intervals come from 1000 bootstrap resamples
(``-c 95 -r 1000``).  An optional stemmer hook replaces Porter stemming (``-m``);
exact agreement with the Perl implementation is "parity unpinned" (no pyrouge/Perl in
this environment to compare against).
"""
from __future__ import annotations

import glob
import os
import re
from collections import Counter
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np

_TOK = re.compile(r"[a-z0-9]+")


def tokenize(s: str, stem: Optional[Callable[[str], str]] = None) -> List[str]:
    toks = _TOK.findall(s.lower())
    return [stem(t) for t in toks] if stem else toks


def _ngrams(toks, n):
    return Counter(tuple(toks[i:i + n]) for i in range(len(toks) - n + 1))


def _prf(hit, ref_total, sys_total, alpha=0.5):
    r = hit / ref_total if ref_total else 0.0
    p = hit / sys_total if sys_total else 0.0
    f = (p * r / ((1 - alpha) * p + alpha * r)) if p > 0 and r > 0 else 0.0
    return p, r, f


def rouge_n(sys_sents: Sequence[str], ref_sents: Sequence[str], n: int, stem=None):
    s = _ngrams(tokenize(" ".join(sys_sents), stem), n)
    r = _ngrams(tokenize(" ".join(ref_sents), stem), n)
    hit = sum(min(c, s[g]) for g, c in r.items())
    return _prf(hit, sum(r.values()), sum(s.values()))


def _lcs_table(a, b):
    m, n = len(a), len(b)
    t = np.zeros((m + 1, n + 1), np.int32)
    for i in range(m):
        ai = a[i]
        for j in range(n):
            t[i + 1, j + 1] = t[i, j] + 1 if ai == b[j] else max(t[i, j + 1], t[i + 1, j])
    return t


def _lcs_positions(a, b):
    t = _lcs_table(a, b)
    i, j, pos = len(a), len(b), set()
    while i > 0 and j > 0:
        if a[i - 1] == b[j - 1]:
            pos.add(i - 1)
            i -= 1
            j -= 1
        elif t[i - 1, j] >= t[i, j - 1]:
            i -= 1
        else:
            j -= 1
    return pos


def rouge_l(sys_sents: Sequence[str], ref_sents: Sequence[str], stem=None):
    """Summary-level union LCS (ROUGE-1.5.5 ROUGE-L)."""
    sys_t = [tokenize(s, stem) for s in sys_sents]
    ref_t = [tokenize(s, stem) for s in ref_sents]
    sys_count = Counter(w for s in sys_t for w in s)
    ref_count = Counter(w for s in ref_t for w in s)
    hit = 0
    for r in ref_t:
        union = set()
        for s_i, s in enumerate(sys_t):
            union |= {(s_i, p) for p in _lcs_positions(s, r)}
        # clip by token budgets like ROUGE-1.5.5
        for (s_i, p) in sorted(union):
            w = sys_t[s_i][p]
            if sys_count[w] > 0 and ref_count[w] > 0:
                hit += 1
                sys_count[w] -= 1
                ref_count[w] -= 1
    return _prf(hit, sum(len(r) for r in ref_t), sum(len(s) for s in sys_t))


def score_pairs(pairs, stem=None, n_boot: int = 1000, seed: int = 0) -> Dict[str, float]:
    """pairs: list of (system_sentences, reference_sentences).  Returns pyrouge-style dict
    with rouge_{1,2,l}_{f_score,recall,precision}[_cb|_ce]."""
    per = {"1": [], "2": [], "l": []}
    for sys_s, ref_s in pairs:
        per["1"].append(rouge_n(sys_s, ref_s, 1, stem))
        per["2"].append(rouge_n(sys_s, ref_s, 2, stem))
        per["l"].append(rouge_l(sys_s, ref_s, stem))
    rng = np.random.default_rng(seed)
    out = {}
    for k, vals in per.items():
        arr = np.asarray(vals, dtype=np.float64).reshape(-1, 3)  # p, r, f
        for col, name in ((2, "f_score"), (1, "recall"), (0, "precision")):
            x = arr[:, col] if len(arr) else np.zeros(1)
            out[f"rouge_{k}_{name}"] = float(x.mean())
            if len(x) > 1 and n_boot:
                idx = rng.integers(0, len(x), size=(n_boot, len(x)))
                boots = np.sort(x[idx].mean(1))
                out[f"rouge_{k}_{name}_cb"] = float(boots[int(0.025 * n_boot)])
                out[f"rouge_{k}_{name}_ce"] = float(boots[min(n_boot - 1, int(0.975 * n_boot))])
            else:
                out[f"rouge_{k}_{name}_cb"] = out[f"rouge_{k}_{name}_ce"] = float(x.mean())
    return out


def rouge_eval(ref_dir: str, dec_dir: str, stem=None) -> Dict[str, float]:
    """Score ``%06d_decoded.txt`` against ``%06d_reference.txt`` (decode.py:268-277)."""
    pairs = []
    for dec in sorted(glob.glob(os.path.join(dec_dir, "*_decoded.txt"))):
        idx = os.path.basename(dec).split("_")[0]
        ref = os.path.join(ref_dir, f"{idx}_reference.txt")
        if not os.path.exists(ref):
            continue
        pairs.append((open(dec, encoding="utf-8").read().split("\n"), open(ref, encoding="utf-8").read().split("\n")))
    return score_pairs(pairs, stem)


def rouge_log(results: Dict[str, float], dir_to_write: Optional[str] = None) -> str:
    """Format like decode.py:280-301 and write ROUGE_results.txt."""
    s = ""
    for x in ["1", "2", "l"]:
        s += "\nROUGE-%s:\n" % x
        for y in ["f_score", "recall", "precision"]:
            key = "rouge_%s_%s" % (x, y)
            s += "%s: %.4f with confidence interval (%.4f, %.4f)\n" % (key, results[key], results[key + "_cb"],
                                                                       results[key + "_ce"])
    if dir_to_write:
        with open(os.path.join(dir_to_write, "ROUGE_results.txt"), "w") as f:
            f.write(s)
    return s
