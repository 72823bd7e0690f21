"""Probe: can the training vocab head run beside the decoder loop?  At the headline shape (B = 256,
T = 400, D = 100, V = 50k) times, with HIP events over 10 repetitions each:

  mid      the captured decoder-backward graph (phase 1: the reverse loop of two row groups)
  vocab    the fused vocab head's two passes (vocab_train_fwd + vocab_train_bwd) on the engine's buffers
  both     the two together: the vocab passes on a side stream, forked before and joined after the graph

If ``both`` is close to max(mid, vocab), the loop leaves room for the head (a chunked head inside the
forward loop would hide it); if it is close to mid + vocab, the loop's kernels and the head contend.
The passes overwrite buffers phase 1 does not read (partials, lse, dlogits), so the probe is timing
only: the trainer's state after it is not used.

  python tools/overlap_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.models.pointer_generator import OV
    from textsummarization_on_flink_amd.train.trainer import GraphTrainer

    B, T, D, V = 256, 400, 100, 50000
    hps = HParams(batch_size=B, max_enc_steps=T, max_dec_steps=D, vocab_size=V, coverage=True, pointer_gen=True)
    corpus = SyntheticCorpus(vocab_size=V, seed=5)
    vocab = corpus.vocab(V)
    batches = make_batches(hps, vocab, corpus, 3, pad_enc_to=T)
    tr = GraphTrainer(hps, vocab.size(), B=B, T=T, device="cuda:0")
    for i in range(3):
        tr.step(batches[i % 3])
    torch.cuda.synchronize()
    eng, k, w, p = tr.engine, tr.engine.k, tr.engine.w, tr.engine.p
    H, N = eng.H, eng.D * eng.B
    vb, vn = (w["vblk"], w["vblk_n"]) if eng.skip_pad else (None, None)
    inplace = vb is not None and not eng.compact_vocab

    def vocab_passes():
        k.vocab_train_fwd(w["outb_ext"], eng.pk["owT"], p[OV], w["target_t"], w["vpart"], w["zg"], w["lse"], w["pv"],
                          N, V, H, H + 8, vb, vn)
        k.vocab_train_bwd(w["outb_ext"], eng.pk["owT"], p[OV], w["target_t"], w["lse"], w["alpha"], w["dlogits"],
                          w["dbias"], N, V, H, H + 8, vb, vn, w["vlive"] if inplace else None,
                          w["vstate"] if inplace else None)

    side = torch.cuda.Stream()
    cur = torch.cuda.current_stream()

    def both():
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            vocab_passes()
        tr.g_mid.replay()
        cur.wait_stream(side)

    def timed(fn, it=10):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(it):
            fn()
        e.record()
        torch.cuda.synchronize()
        return round(s.elapsed_time(e) * 1e3 / it, 1)

    res = {"mid_us": timed(tr.g_mid.replay), "vocab_us": timed(vocab_passes), "both_us": timed(both)}
    res["mid_us_again"] = timed(tr.g_mid.replay)
    res["hidden_fraction"] = round((res["mid_us"] + res["vocab_us"] - res["both_us"]) / res["vocab_us"], 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
