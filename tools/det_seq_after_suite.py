"""Run the GPU test tier (minus the deterministic test), then -- in the same process, like
test_deterministic_mode_bit_identical -- train two deterministic-mode GraphTrainers one after the
other (the first deleted before the second is built) and print, per step, which engine buffers and
gradient slices differ (bit checksums).

  DSQ_SPLIT=4 python tools/det_seq_after_suite.py [--no-suite]
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


def profile(t):
    """(whole-tensor checksum, per-leading-index checksums, per-last-dim-index checksums) on the CPU:
    where two runs differ, the differing leading rows and last-dim columns are listed."""
    import torch
    x = t.detach().contiguous()
    if x.dtype == torch.bfloat16:
        x = x.view(torch.int16).to(torch.int64)
    elif x.dtype == torch.float32:
        x = x.view(torch.int32).to(torch.int64)
    else:
        x = x.to(torch.int64)
    if x.dim() < 2:
        x = x.reshape(1, -1)
    rows = x.reshape(x.shape[0], -1)
    wr = torch.arange(1, rows.shape[1] + 1, device=x.device, dtype=torch.int64) % 1000003
    cols = x.reshape(-1, x.shape[-1])
    wc = (torch.arange(1, cols.shape[0] + 1, device=x.device, dtype=torch.int64) % 999983).view(-1, 1)
    return sig(t), (rows * wr).sum(1).cpu(), (cols * wc).sum(0).cpu()


def where(a, b, lim=12):
    i = (a != b).nonzero().view(-1)
    return {"n": int(i.numel()), "first": i[:lim].tolist()}


def main():
    if "--no-suite" not in sys.argv:
        rc = pytest.main(["tests", "-m", "gpu", "-q", "--timeout", "300", "--timeout-method", "thread",
                          "-k", os.environ.get("DSQ_K", "not deterministic")])
        print("suite rc", rc, flush=True)
    import torch
    os.environ["TSAMD_DETERMINISTIC"] = "1"
    if os.environ.get("DSQ_SPLIT"):  # row groups of the two deterministic trainers only (not the suite's)
        os.environ["TSAMD_SPLIT"] = os.environ["DSQ_SPLIT"]
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
            d = {k: profile(v) for k, v in e.w.items() if torch.is_tensor(v) and v.numel()}
            for n, (o, c) in tr.params.offsets.items():
                d["grad:" + n] = profile(tr.params.grad[o:o + c])
                d["param:" + n] = profile(tr.params.flat[o:o + c])
            steps.append(d)
        runs.append(steps)
        del tr, e
        torch.cuda.empty_cache()
    for i in range(5):
        a, b = runs[0][i], runs[1][i]
        diff = sorted(k for k in a if k in b and a[k][0] != b[k][0])
        print(json.dumps({"step": i, "ndiff": len(diff), "diff": diff[:40]}), flush=True)
        if diff and i == min(j for j in range(5) if any(runs[0][j][k][0] != runs[1][j][k][0] for k in runs[0][j])):
            for k in diff[:24]:  # where, in the first step with a difference
                print(json.dumps({"step": i, "buf": k, "rows": where(a[k][1], b[k][1]),
                                  "cols": where(a[k][2], b[k][2])}), flush=True)


if __name__ == "__main__":
    main()
