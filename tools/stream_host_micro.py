"""Host-side rate of the serving packer path without a GPU: coded rows -> StreamDecodePacker
(packer processes: row -> Example -> id arrays; the caller: batch gather + engine pack) ->
fake "decoded" token ids -> send_results -> result rows at the output ring.  The bench shape
(V = 50k, enc 400, 64 articles per batch); a summary of ``--sum-len`` tokens per article.

  python tools/stream_host_micro.py [--rows 6400] [--packers 6]

Prints one JSON line: rows/s end to end and the caller's per-batch host milliseconds (poll +
send_results), i.e. the host work the GPU process does per decode batch."""
import argparse
import json
import os
import sys
import time
import uuid

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=6400)
    ap.add_argument("--packers", type=int, default=6)
    ap.add_argument("--sum-len", type=int, default=60)
    ap.add_argument("--gpu-ms", type=float, default=0.0, help="simulated device time per batch (sleep)")
    a = ap.parse_args()
    import numpy as np
    import textsummarization_on_flink_amd.decode.decoder  # noqa: F401 -- as in a worker: the packers fork with it loaded
    from textsummarization_on_flink_amd.api.coding import ExampleCoding
    from textsummarization_on_flink_amd.api.types import DataTypes
    from textsummarization_on_flink_amd.config import HParams
    from textsummarization_on_flink_amd.data.stream_pack import StreamDecodePacker
    from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus
    from textsummarization_on_flink_amd.runtime.ring import RecordRing
    in_cols, out_cols = ["uuid", "article", "reference"], ["uuid", "article", "summary", "reference"]
    corpus = SyntheticCorpus(vocab_size=50000, seed=3)
    vocab = corpus.vocab(50000)
    T, Na = 400, 64
    hps = HParams(mode="decode", batch_size=4, beam_size=4, max_enc_steps=T, max_dec_steps=100, vocab_size=50000,
                  coverage=True)
    rows = corpus.rows(a.rows, "h")
    cin, cout = ExampleCoding(in_cols, [DataTypes.STRING] * 3), ExampleCoding(out_cols, [DataTypes.STRING] * 4)
    tag = uuid.uuid4().hex[:8]
    rin, rout = RecordRing.create(f"/tsamd_hm_in_{tag}", 512 << 20), RecordRing.create(f"/tsamd_hm_out_{tag}", 512 << 20)
    recs = [cin.encode({k: r[k] for k in in_cols}) for r in rows]
    pool = StreamDecodePacker(rin, rout, cin, cout, vocab, hps, packers=a.packers, n_articles=Na, T=T,
                              max_wait_s=0.0)
    rng = np.random.default_rng(0)
    t0 = time.perf_counter()
    for r in recs:
        rin.push(r)
    rin.close()
    host, n_b, n = 0.0, 0, 0
    while True:
        h0 = time.perf_counter()
        b = pool.poll(block=True)
        if b is None:
            break
        ids = [rng.integers(4, 50000, a.sum_len).tolist() for _ in range(b.n_valid)]
        h1 = time.perf_counter()
        pool.send_results(b, ids)
        host += time.perf_counter() - h1 + (h1 - h0 if b.n_valid else 0.0)
        if a.gpu_ms:
            time.sleep(a.gpu_ms / 1e3)
        n_b += 1
        n += b.n_valid
    pool.close()
    got = 0
    while got < n:
        rec = rout.pop(timeout_ms=20000)
        if rec is None:
            break
        got += 1
    el = time.perf_counter() - t0
    print(json.dumps({"metric": "stream_host_rows_per_sec", "value": round(got / el, 1), "rows": got,
                      "batches": n_b, "rows_per_batch": round(n / max(n_b, 1), 1), "gpu_ms": a.gpu_ms, "host_ms_per_batch": round(1e3 * host / max(n_b, 1), 3),
                      "packers": a.packers, "cpus": os.cpu_count()}), flush=True)
    pool.stop() if hasattr(pool, "stop") else None
    for r in (rin, rout):
        r.release()


if __name__ == "__main__":
    main()
