"""Device math of the attention kernels (attn_common.h): the tanh / sech^2 every score, score
gradient and feature gradient uses, against fp64 over [-20, 20] (reference semantics: the
Bahdanau score v . tanh(W_h h_i + W_s s_t + w_c c_i), attention_decoder.py:104-110)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _eval(mode, x):
    from textsummarization_on_flink_amd.ops import ops
    t, s2 = torch.empty_like(x), torch.empty_like(x)
    ops().tanh_eval(x, t, s2, mode)
    torch.cuda.synchronize()
    ref = torch.tanh(x.double())
    return float((t.double() - ref).abs().max()), float((s2.double() - (1 - ref * ref)).abs().max())


def test_attention_tanh_and_sech2_match_fp64():
    """The kernels' form: r = 1 / (1 + 2^(2 u log2 e)) (one exp2 + one rcp), tanh = 1 - 2r,
    sech^2 = 4 r (1 - r): within 3e-7 / 6e-7 absolute of fp64 everywhere."""
    x = torch.linspace(-20, 20, 4_000_001, device="cuda")
    et, es = _eval(0, x)
    assert et <= 3e-7, et
    assert es <= 6e-7, es


def test_rational_tanh_probe_is_the_documented_function():
    """The one-reciprocal rational alternative (probes.hip tanh_rat2, clamped at 7.905): a correct
    tanh to ~4e-7 (3 roundings near |t| = 1 keep it above the exp form's error).  Its issue cost
    against the exp form is measured by tools/tanh_probe.py (profiles/r5/tanh_probe.md)."""
    x = torch.linspace(-20, 20, 4_000_001, device="cuda")
    et, es = _eval(1, x)
    assert et <= 1e-6 and es <= 2e-6, (et, es)
