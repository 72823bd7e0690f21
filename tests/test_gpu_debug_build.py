"""Bounds-checked debug build of the kernel library (``_C_debug.so``: csrc/kernels/dcheck.h,
SURVEY 5.2 "HIP kernels get bounds-checked debug builds").  TSAMD_KERNEL_DEBUG=1 selects the
library at load time and one process cannot hold both libraries' op registrations, so the
checks run in a child process: a clean train step and beam decode must record nothing; an
out-of-vocabulary encoder token id and an encoder length past T must be reported by the
kernels that index with them (and clamped, so the run does not fault the GPU)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, torch
from textsummarization_on_flink_amd import ops
from textsummarization_on_flink_amd.config import HParams
from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
from textsummarization_on_flink_amd.models.params import build_params
from textsummarization_on_flink_amd.models.pointer_generator import HipPointerGenerator

k = ops.ops()
res = {"enabled": int(k.debug_enabled()), "lib": ops.library_path()}
V, T, B = 2000, 64, 16
hps = HParams(batch_size=B, max_enc_steps=T, max_dec_steps=8, min_dec_steps=2, vocab_size=V, coverage=True,
              beam_size=4)
corpus = SyntheticCorpus(vocab_size=V, raw_vocab=8000, seed=0, art_mean=50, art_sd=10, sent_mean=4)
vocab = corpus.vocab(V)
batch = make_batches(hps, vocab, corpus, 1, pad_enc_to=T)[0]
params = build_params(hps, vocab.size(), device="cuda").enable_grad().enable_adagrad(hps.adagrad_init_acc)
eng = HipPointerGenerator(hps, vocab.size(), params, B=B, T=T)

def status():
    torch.cuda.synchronize()
    s = [int(x) for x in k.debug_status().tolist()]
    k.debug_clear()
    return s

k.debug_clear()
eng.set_batch(batch)
eng.train_step()
res["clean_train"] = status()
dec = DeviceBeamDecoder(hps.replace(mode="decode"), vocab, params, n_articles=B, T=T, use_graph=False)
dec.decode(batch)
res["clean_decode"] = status()
eng.set_batch(batch)
eng.w["enc_batch"][3, 5] = V + 7          # token id past the embedding table
eng.forward(need_grad=True)
res["bad_id"] = status()
eng.set_batch(batch)
eng.w["enc_lens"][2] = T + 9              # encoder length past T
eng.forward(need_grad=True)
res["bad_len"] = status()
try:
    eng.set_batch(batch)
    eng.w["enc_batch"][0, 0] = -3
    eng.forward(need_grad=True)
    ops.debug_check()
    res["raised"] = ""
except ops.KernelBoundsError as e:
    res["raised"] = str(e)
print("RESULT " + json.dumps(res))
'''


@pytest.mark.gpu
def test_debug_build_reports_bad_indices():
    lib = os.path.join(REPO, "textsummarization_on_flink_amd", "_C_debug.so")
    assert os.path.exists(lib), "build the debug library first: python -m textsummarization_on_flink_amd._build"
    env = dict(os.environ, TSAMD_KERNEL_DEBUG="1", PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240, cwd=REPO)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert r.returncode == 0 and line, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    res = json.loads(line[0][7:])
    assert res["enabled"] == 1 and res["lib"].endswith("_C_debug.so")
    assert res["clean_train"] == [0, 0, 0, 0], res
    assert res["clean_decode"] == [0, 0, 0, 0], res
    assert res["bad_id"][0] == 1 and res["bad_id"][3] == 2000 + 7, res        # CHK_FRAME_ID, the bad value
    assert res["bad_len"][0] in (4, 5) and res["bad_len"][3] == 64 + 9, res   # attention / loss length check
    assert "to_step_frame row id" in res["raised"], res


def test_release_library_has_checks_compiled_out():
    """The release library reports the debug record as absent (CPU: no device needed)."""
    import subprocess as sp
    code = ("from textsummarization_on_flink_amd import ops; k = ops.load(build_if_missing=False); "
            "print(int(k.debug_enabled()), ops.library_path().endswith('_C.so'))")
    env = dict(os.environ, TSAMD_KERNEL_DEBUG="0", PYTHONPATH=REPO)
    r = sp.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240, cwd=REPO)
    if r.returncode != 0 and "not found" in r.stderr:
        pytest.skip("kernel library not built")
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split() == ["0", "True"]
