"""Which torch ops (with shapes) make up the non-HIP-kernel time of a train step: one eager
step (use_graph=False) of the bench config under torch.profiler, top aten ops by device time.
Synthetic CNN/DM-shaped data, random-init weights."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.parallel import dist as D
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer
    info = D.init_from_env(backend="gloo")
    hps = HParams(batch_size=a.batch, max_enc_steps=400, max_dec_steps=100, vocab_size=50000, hidden_dim=256,
                  emb_dim=128, coverage=True, pointer_gen=True)
    corpus = SyntheticCorpus(vocab_size=50000, seed=1000)
    vocab = corpus.vocab(50000)
    batches = make_batches(hps, vocab, corpus, 2, pad_enc_to=400)
    tr = GraphTrainer(hps, vocab.size(), B=a.batch, T=400, device="cuda:0", info=info, use_graph=False)
    for i in range(2):
        tr.step(batches[i % 2])
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        tr.step(batches[0])
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=a.top,
                                                             max_name_column_width=40, max_shapes_column_width=70))


if __name__ == "__main__":
    main()
