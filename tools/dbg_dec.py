import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
from test_gpu_decode import _peaked_setup
from textsummarization_on_flink_amd.decode.device_beam import DeviceBeamDecoder
for cov, pgen in [(True, True), (False, True), (False, False)]:
    hps, vocab, batch, params = _peaked_setup(cov, pointer_gen=pgen)
    res = {}
    for fv in ("0", "1"):
        os.environ["TSAMD_FUSED_VOCAB"] = fv
        d = DeviceBeamDecoder(hps, vocab, params, n_articles=hps.batch_size, T=hps.max_enc_steps, use_graph=False)
        res[fv] = [h.tokens for h in d.decode(batch)]
    print(cov, pgen, "fused==materialized:", res["0"] == res["1"], [a == b for a, b in zip(res["0"], res["1"])])
