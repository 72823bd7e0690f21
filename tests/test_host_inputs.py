"""Host-side engine inputs (models/pointer_generator.host_inputs), CPU only: the live decoder
steps per row, the row order sorted by them (every per-row array permuted consistently, the
loss weights unchanged as a multiset), and the fused vocab head's live-block list -- the inputs
the skipping kernels trust (EngineConfig.skip_pad_steps)."""
import numpy as np
import pytest

from textsummarization_on_flink_amd.config import HParams
from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
from textsummarization_on_flink_amd.models.pointer_generator import host_inputs, input_layout, pack_host_inputs


def _batch(B=24, T=60, D=30, pointer_gen=True, seed=3):
    hps = HParams(batch_size=B, max_enc_steps=T, max_dec_steps=D, vocab_size=2000, coverage=True,
                  pointer_gen=pointer_gen)
    corpus = SyntheticCorpus(vocab_size=2000, raw_vocab=8000, seed=seed, art_mean=50, art_sd=15, sent_mean=4)
    vocab = corpus.vocab(2000)
    return hps, make_batches(hps, vocab, corpus, 1, pad_enc_to=T)[0]


@pytest.mark.parametrize("pointer_gen", [True, False])
def test_dlen_is_last_loss_weighted_step(pointer_gen):
    hps, b = _batch(pointer_gen=pointer_gen)
    D = hps.max_dec_steps
    h = host_inputs(b, hps, D)
    dm = b.dec_padding_mask[:, :D] * b.valid[:, None]
    want = np.array([int(np.nonzero(r)[0].max()) + 1 if r.any() else 0 for r in dm])
    assert np.array_equal(h["dlen"], want)
    live = np.arange(D)[:, None] < h["dlen"][None, :]  # [D, B]
    assert not h["rowg"][~live].any() and not h["gcl"][~live].any()
    assert np.array_equal(h["row_src"], np.arange(hps.batch_size))


def test_sorted_rows_permute_every_row_array():
    hps, b = _batch()
    D, B = hps.max_dec_steps, hps.batch_size
    u = host_inputs(b, hps, D)
    s = host_inputs(b, hps, D, sort_rows=True)
    src = s["row_src"]
    assert sorted(src.tolist()) == list(range(B))
    assert (np.diff(s["dlen"]) <= 0).all(), "rows sorted by live steps, longest first"
    assert np.array_equal(s["dlen"], u["dlen"][src])
    for k in ("enc_batch", "enc_lens", "rev_idx", "ext"):
        assert np.array_equal(s[k], u[k][src]), k
    for k in ("dec_batch_t", "target_t", "rowg", "gcl"):  # step-major [D, B]
        assert np.array_equal(s[k], u[k][:, src]), k
    # the embedding-gradient order lists the same token ids
    assert np.array_equal(np.sort(s["emb_sid"]), np.sort(u["emb_sid"]))
    assert abs(float(s["rowg"].sum()) - float(u["rowg"].sum())) < 1e-6


def test_vocab_live_blocks():
    hps, b = _batch(B=24, D=30)  # D * B = 720 rows: 22.5 blocks of 32
    D, B = hps.max_dec_steps, hps.batch_size
    h = host_inputs(b, hps, D, sort_rows=True)
    nb = (D * B + 31) // 32
    live_rows = np.zeros(nb * 32, dtype=bool)
    live_rows[:D * B] = (np.arange(D)[:, None] < h["dlen"][None, :]).reshape(-1)  # t-major rows
    want = np.nonzero(live_rows.reshape(nb, 32).any(1))[0]
    n = int(h["vblk_n"][0])
    assert n == len(want) and np.array_equal(h["vblk"][:n], want)
    assert np.array_equal(h["vlive"].astype(bool), live_rows.reshape(nb, 32).any(1))
    assert 0 < n < nb  # the synthetic summaries leave dead blocks
    # every loss-weighted (step, row) lies in a listed block
    w = (h["rowg"] != 0) | (h["gcl"] != 0)
    assert h["vlive"][np.nonzero(w.reshape(-1))[0] // 32].all()
    layout, total = input_layout(B, hps.max_enc_steps, D)
    assert pack_host_inputs(h, layout).nbytes == total


def test_gemm_dispatch_table_is_fixed_by_shape():
    """The activation-GEMM dispatch (TSAMD_GEMM_BT=table, the default) depends only on the shape:
    the hand-written GEMM for step-frame gathers, K <= 256 and bf16-out K <= 1024; hipBLASLt for
    the fp32-out K >= 512 shapes -- the same pick on every run and rank (profiles/r6/gemm_dispatch.md)."""
    from textsummarization_on_flink_amd.models import pointer_generator as pg
    assert pg.GEMM_BT in ("table", "auto", "0", "1")
    rule = pg._bt_rule
    assert rule(128, False, 1.0) and rule(256, False, 1.0)
    assert not rule(512, False, 1.0) and not rule(1024, False, 1.0)
    assert rule(512, True, 1.0) and rule(1024, True, 1.0) and not rule(2048, True, 1.0)
    assert rule(2048, False, pg.FRAME_SLACK)  # the gather GEMMs save the layout pass
    assert all(rule(k, b, 1.0) == rule(k, b, 1.0) for k in (128, 512, 4096) for b in (False, True))


def test_encoder_wgrad_cpu_path_matches_matmul():
    """wgrad_enc_into on CPU tensors (the oracle backend) falls back to the plain matmul path."""
    import torch
    from textsummarization_on_flink_amd.models.pointer_generator import wgrad_enc_into
    g = torch.Generator().manual_seed(0)
    a, b = torch.randn(64, 16, generator=g), torch.randn(64, 24, generator=g)
    out = torch.empty(16, 24)
    wgrad_enc_into(out, a, b)
    assert torch.allclose(out, a.t() @ b, atol=1e-5)
