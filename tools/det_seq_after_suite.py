"""Run the GPU test tier (minus the deterministic test), then -- in the same process, like
test_deterministic_mode_bit_identical -- train two deterministic-mode GraphTrainers one after the
other (the first deleted before the second is built) and print, per step, which engine buffers and
gradient slices differ (bit checksums).

  python tools/det_seq_after_suite.py [--no-suite]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import pytest  # noqa: E402


def sig(t):
    import torch
    x = t.detach().contiguous().reshape(-1)
    if x.dtype == torch.bfloat16:
        x = x.view(torch.int16).to(torch.int64)
    elif x.dtype == torch.float32:
        x = x.view(torch.int32).to(torch.int64)
    else:
        x = x.to(torch.int64)
    n = x.numel()
    w = torch.arange(1, n + 1, device=x.device, dtype=torch.int64) % 1000003
    return int((x * w).sum())


def main():
    if "--no-suite" not in sys.argv:
        rc = pytest.main(["tests", "-m", "gpu", "-q", "--timeout", "300", "--timeout-method", "thread",
                          "-k", os.environ.get("DSQ_K", "not deterministic")])
        print("suite rc", rc, flush=True)
    import torch
    os.environ["TSAMD_DETERMINISTIC"] = "1"
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer
    hps = HParams(batch_size=256, max_enc_steps=400, max_dec_steps=100, vocab_size=50000, coverage=True,
                  pointer_gen=True)
    corpus = SyntheticCorpus(vocab_size=50000, seed=17)
    vocab = corpus.vocab(50000)
    batches = make_batches(hps, vocab, corpus, 3, pad_enc_to=400)
    runs = []
    for r in range(2):
        tr = GraphTrainer(hps, vocab.size(), B=256, T=400, device="cuda:0")
        steps = []
        for i in range(5):
            tr.step(batches[i % 3])
            torch.cuda.synchronize()
            e = tr.engine
            d = {k: sig(v) for k, v in e.w.items() if torch.is_tensor(v)}
            for n, (o, c) in tr.params.offsets.items():
                d["grad:" + n] = sig(tr.params.grad[o:o + c])
                d["param:" + n] = sig(tr.params.flat[o:o + c])
            steps.append(d)
        runs.append(steps)
        del tr, e
        torch.cuda.empty_cache()
    for i in range(5):
        diff = sorted(k for k in runs[0][i] if runs[0][i][k] != runs[1][i].get(k))
        print(json.dumps({"step": i, "ndiff": len(diff), "diff": diff[:40]}), flush=True)


if __name__ == "__main__":
    main()
