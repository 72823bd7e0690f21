"""Shared fixtures: a tiny CNN/DM-shaped dataset on disk and tiny model flags."""
import os

from textsummarization_on_flink_amd.data import binfmt
from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus

TINY_FLAGS = ["--hidden_dim=16", "--emb_dim=8", "--vocab_size=200", "--max_enc_steps=30", "--max_dec_steps=8",
              "--min_dec_steps=2", "--batch_size=4", "--beam_size=2", "--save_model_secs=0"]


def tiny_corpus(seed=0):
    return SyntheticCorpus(vocab_size=200, raw_vocab=400, seed=seed, art_mean=30, art_sd=8, sent_mean=5)


GPU_FLAGS = ["--hidden_dim=64", "--emb_dim=64", "--vocab_size=600", "--max_enc_steps=48", "--max_dec_steps=12",
             "--min_dec_steps=3", "--batch_size=8", "--beam_size=4", "--decode_batch=8", "--save_model_secs=0"]


def gpu_corpus(seed=0):
    return SyntheticCorpus(vocab_size=600, raw_vocab=1800, seed=seed, art_mean=40, art_sd=10, sent_mean=4)


def make_dataset(root, n_files=2, per_file=12, seed=0, corpus=None):
    """Writes <root>/data/{train,val,test}_00k.bin + <root>/vocab; returns (data_dir, vocab_path, corpus)."""
    c = corpus or tiny_corpus(seed)
    d = os.path.join(root, "data")
    os.makedirs(d, exist_ok=True)
    for split in ("train", "val", "test"):
        for k in range(n_files):
            exs = [{"article": a, "abstract": s} for a, s in c.examples(per_file)]
            binfmt.write_bin(os.path.join(d, f"{split}_{k:03d}.bin"), exs)
    vp = os.path.join(root, "vocab")
    c.vocab().save(vp)
    return d, vp, c


def grad_mismatches(params, g_hip, g_ref, rel=5e-2, abs_frac=1e-3):
    """Per-parameter gradient check of an engine against the fp32 oracle.  A parameter whose
    reference gradient norm is >= 1e-6 must match at relative error < ``rel``; a smaller one
    (a near-zero gradient at init, where relative error is noise) must match absolutely, within
    ``abs_frac`` of the GLOBAL reference gradient norm -- never a looser relative bound.
    Returns [(name, rel_err, ref_norm, abs_err)] of the failures."""
    gnorm = float(g_ref.norm())
    bad = []
    for n in params.names:
        o, c = params.offsets[n]
        gr, gh = g_ref[o:o + c], g_hip[o:o + c]
        gn, d = float(gr.norm()), float((gh - gr).norm())
        ok = d <= abs_frac * gnorm if gn < 1e-6 else d < rel * gn
        if not ok:
            bad.append((n, round(d / (gn + 1e-12), 4), gn, d))
    return bad


def grad_rel(params, g_hip, g_ref):
    """{name: relative gradient error} against the oracle."""
    out = {}
    for n in params.names:
        o, c = params.offsets[n]
        gr = g_ref[o:o + c]
        out[n] = float((g_hip[o:o + c] - gr).norm() / (gr.norm() + 1e-12))
    return out
