"""Per-kernel timing of the B=256 training step's hot kernels, isolated (HIP events).

Builds the bench-shaped engine (pointer-gen + coverage, H=256, T=400, D=100, V=50k), runs one
forward + backward so every buffer holds realistic values, then re-launches single kernels
with the engine's own buffers at decoder step t=50.  Variants are chosen by the kernels'
engine switches (EngineConfig, TSAMD_*), so run one process per variant.
Prints one JSON line of microseconds per launch.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

F32, BF = torch.float32, torch.bfloat16


def timeit(fn, it=50):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) * 1e3 / it, 2)


def main():
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus, make_batches
    from textsummarization_on_flink_amd.models.params import build_params
    from textsummarization_on_flink_amd.models.pointer_generator import HipPointerGenerator

    B = int(os.environ.get("MICRO_B", "256"))
    T, D, V = 400, 100, 50000
    hps = HParams(batch_size=B, max_enc_steps=T, max_dec_steps=D, vocab_size=V, coverage=True, pointer_gen=True)
    corpus = SyntheticCorpus(vocab_size=V, seed=3)
    vocab = corpus.vocab(V)
    batch = make_batches(hps, vocab, corpus, 1, pad_enc_to=T)[0]
    params = build_params(hps, vocab.size(), device="cuda").enable_grad().enable_adagrad(hps.adagrad_init_acc)
    eng = HipPointerGenerator(hps, vocab.size(), params, B=B, T=T)
    eng.set_batch(batch)
    eng.forward(need_grad=True)
    eng.backward()
    torch.cuda.synchronize()
    k, w, A, H = eng.k, eng.w, eng.A, eng.H
    enc_out, lens, F, Ft = eng.enc[-1]["out"], w["enc_lens"], w["F"], w["Ft"]
    if Ft is None:  # row-attention engine: build the transposed copy for the multi-block kernels
        Ft = torch.empty(B, eng.A, T, dtype=BF, device="cuda")
        eng.k.transpose_bta(F, Ft, B, T, eng.A)
    v, wc = eng.f32["v"], eng.f32["wc"]
    t = 50
    res = {"B": B, "env": {x: os.environ[x] for x in os.environ if x.startswith("TSAMD_")}}
    if eng.k.attn_row_ok(eng.A, T):
        res["attn_fwd_row"] = timeit(lambda: eng.k.attn_fwd_row(F, enc_out, w["S"][t], v, wc, w["COV"][t], lens,
                                                                 w["ATT"][t], w["COV"][t + 1], w["covloss"][t],
                                                                 w["CTX"][t], w["CTXb"][t], B, T, eng.A, 1))
        res["attn_bwd_row"] = timeit(lambda: eng.k.attn_bwd_row(enc_out, F, w["S"][t], v, wc, w["COV"][t],
                                                                 w["ATT"][t], w["DCTX"][t], w["CTX"][t], w["dA"][t],
                                                                 w["dcov"][1], w["gcl"][t], lens, w["DE"][t],
                                                                 w["DS"][t], w["dcov"][0], B, T, eng.A))
    res["attn_score"] = timeit(lambda: k.attn_score(Ft, w["S"][t], v, wc, w["COV"][t], lens, w["e"], B, T, A, 1))
    res["attn_softmax_ctx"] = timeit(lambda: k.attn_softmax_ctx(w["e"], enc_out, lens, w["COV"][t], w["ATT"][t],
                                                                w["COV"][t + 1], w["covloss"][t], w["CTX"][t],
                                                                w["CTXb"][t], B, T, A, 1))
    dcov = w["dcov"]
    res["attn_bwd_step"] = timeit(lambda: k.attn_bwd_step(enc_out, F, w["S"][t], v, wc, w["COV"][t], w["ATT"][t],
                                                          w["DCTX"][t], w["CTX"][t], w["dA"][t], dcov[1], w["gcl"][t],
                                                          lens, w["DE"][t], w["DS"][t], dcov[0], B, T, A))
    res["attn_bwd_feat"] = timeit(lambda: k.attn_bwd_feat(F, w["S"], v, wc, w["COV"][:D], w["DE"], lens, w["dF"],
                                                          w["dv"], w["dwc"], D, B, T, A, None), it=5)
    # d out = dlogits . W^T (K = V): library GEMM vs split-K batched GEMM
    dl, ow = w["dlogits"], eng.pk["ow"]
    N = D * B
    res["dout_mm"] = timeit(lambda: torch.mm(dl, ow.t(), out_dtype=F32), it=10)
    ref = torch.mm(dl, ow.t(), out_dtype=F32)
    out = torch.empty(N, H, device="cuda")
    for S in (5, 10, 25, 50):
        if V % S:
            continue

        def f(S=S):
            p = torch.bmm(dl.view(N, S, V // S).transpose(0, 1), ow.view(H, S, V // S).permute(1, 2, 0), out_dtype=F32)
            torch.sum(p, 0, out=out)
        f()
        res[f"dout_split{S}"] = timeit(f, it=10)
        res[f"dout_split{S}_err"] = float((out - ref).abs().max() / ref.abs().max())
    # transposed problem: dout^T = W . dlogits^T (M = H, N = rows)
    res["dout_T"] = timeit(lambda: torch.mm(ow, dl.t(), out_dtype=F32), it=10)
    p, OV = eng.p, "seq2seq/output_projection/v"
    if eng.fused_vocab:
        ldx = H + 8
        res["vocab_fwd"] = timeit(lambda: k.vocab_train_fwd(w["outb_ext"], eng.pk["owT"], p[OV], w["target_t"],
                                                            w["vpart"], w["zg"], w["lse"], w["pv"], N, V, H, ldx, None, None),
                                  it=10)
        res["vocab_bwd"] = timeit(lambda: k.vocab_train_bwd(w["outb_ext"], eng.pk["owT"], p[OV], w["target_t"],
                                                            w["lse"], w["alpha"], w["dlogits"], w.get("dbias"), N, V,
                                                            H, ldx, None, None, None, None), it=10)
    # output-projection weight gradient (K = N rows): [W|b] (M = H+1) vs W only vs split-K
    xe = w["outb_ext"]
    dst = torch.empty(H + 1, V, device="cuda")
    res["dw_mm257"] = timeit(lambda: torch.mm(xe[:, :H + 1].t(), dl, out_dtype=F32, out=dst), it=10)
    res["dw_mm256"] = timeit(lambda: torch.mm(xe[:, :H].t(), dl, out_dtype=F32, out=dst[:H]), it=10)
    # transposed problem: dW^T = dlogits^T . X (M = V, N = H), then without / with the transpose back
    dstT = torch.empty(V, H, device="cuda")
    res["dw_T"] = timeit(lambda: torch.mm(dl.t(), xe[:, :H], out_dtype=F32, out=dstT), it=10)
    res["dw_T_transpose"] = timeit(lambda: dst[:H].copy_(dstT.t()), it=10)
    for S in (2, 4, 8):
        def g(S=S):
            p = torch.bmm(xe.view(S, N // S, H + 8)[:, :, :H].transpose(1, 2), dl.view(S, N // S, V),
                          out_dtype=F32)
            torch.sum(p, 0, out=dst[:H])
        res[f"dw_split{S}"] = timeit(g, it=10)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
