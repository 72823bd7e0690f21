"""Stream-fed pipelines at engine speed (data/stream_pack.py, the native ring pipes in
csrc/runtime/shm_ring.cpp): the packer processes must produce exactly the batches of the
serial stream batchers, and serving must answer every row through the fanin."""
import uuid

import numpy as np
import pytest

from textsummarization_on_flink_amd.api.coding import ExampleCoding
from textsummarization_on_flink_amd.api.types import DataTypes
from textsummarization_on_flink_amd.config import HParams
from textsummarization_on_flink_amd.data.batch import Batch
from textsummarization_on_flink_amd.data.batcher import FlinkTrainBatcher, IterRowReader, examples_from_rows
from textsummarization_on_flink_amd.data.stream_pack import StreamDecodePacker, StreamTrainPacker
from textsummarization_on_flink_amd.data.synthetic import SyntheticCorpus
from textsummarization_on_flink_amd.decode.decoder import flink_summary
from textsummarization_on_flink_amd.models.pointer_generator import host_inputs, input_layout, pack_host_inputs
from textsummarization_on_flink_amd.runtime.ring import RecordRing, RingPipe

IN_COLS = ["uuid", "article", "reference"]
OUT_COLS = ["uuid", "article", "summary", "reference"]


def _ring(tag, cap=8 << 20):
    return RecordRing.create(f"/tsamd_t_{tag}_{uuid.uuid4().hex[:8]}", cap)


def test_ring_fanout_groups_and_fanin():
    src = _ring("src")
    dsts = [_ring(f"d{i}") for i in range(3)]
    pipe = RingPipe.fanout(src, dsts, group=2)
    for k in range(13):
        src.push(b"r%d" % k)
    src.close()
    assert pipe.join() == 13
    got = [[x.decode() for x in d] for d in dsts]  # iteration ends at the fanout's close
    # record k -> destination (k // 2) % 3
    assert got == [["r0", "r1", "r6", "r7", "r12"], ["r2", "r3", "r8", "r9"], ["r4", "r5", "r10", "r11"]]
    # fanin: every record of every source, destination closed once all sources are
    srcs = [_ring(f"s{i}") for i in range(3)]
    out = _ring("out")
    fin = RingPipe.fanin(srcs, out, close_dst=True)
    for i, s in enumerate(srcs):
        for k in range(5):
            s.push(b"%d-%d" % (i, k))
        s.close()
    assert fin.join() == 15
    recs = [x.decode() for x in out]
    assert sorted(recs) == sorted("%d-%d" % (i, k) for i in range(3) for k in range(5))
    for i in range(3):  # per-source order is kept
        assert [r for r in recs if r.startswith(f"{i}-")] == [f"{i}-{k}" for k in range(5)]
    for r in [src, out, *dsts, *srcs]:
        r.release()


@pytest.mark.parametrize("n_rows,packers,drop_last", [(8 * 5 + 3, 3, False), (8 * 4, 2, False), (8 * 3 + 5, 2, True)])
def test_stream_train_packer_matches_serial_batcher(n_rows, packers, drop_last):
    corpus = SyntheticCorpus(vocab_size=2000, raw_vocab=6000, seed=3, art_mean=80, art_sd=30)
    vocab = corpus.vocab(2000)
    hps = HParams(batch_size=8, max_enc_steps=64, max_dec_steps=12, vocab_size=2000, coverage=True,
                  drop_last=drop_last)
    rows = corpus.rows(n_rows)
    coding = ExampleCoding(IN_COLS, [DataTypes.STRING] * 3)
    rin = _ring("in")
    sp = StreamTrainPacker(rin, coding, vocab, hps, packers, pad_enc_to=64)
    for r in rows:
        rin.push(coding.encode(r))
    rin.close()
    got = []
    while True:
        b = sp.next_batch()
        if b is None:
            break
        got.append(b)
    sp.stop()
    # the serial stream batcher over the same rows (decoded the same way)
    serial = FlinkTrainBatcher(IterRowReader([coding.decode_dict(coding.encode(r)) for r in rows]), vocab, hps,
                               pad_enc_to=64)
    layout, _ = input_layout(8, 64, 12)
    exp = []
    while True:
        b = serial.next_batch()
        if b is None:
            break
        exp.append(b)
    assert len(got) == len(exp) == (n_rows // 8 if drop_last else -(-n_rows // 8))
    for g, e in zip(got, exp):
        ref = pack_host_inputs(host_inputs(e, hps, 12, sort_rows=True), layout)
        assert bytes(g.host_pack) == ref.tobytes()
        assert g.num_tokens() == e.num_tokens() and g.padded_tokens() == e.padded_tokens()
        assert g.n_valid == int(e.valid.sum())
    rin.release()


def test_stream_decode_packer_answers_every_row():
    corpus = SyntheticCorpus(vocab_size=2000, raw_vocab=6000, seed=5, art_mean=60, art_sd=20)
    vocab = corpus.vocab(2000)
    T, Na = 48, 4
    hps = HParams(mode="decode", batch_size=4, beam_size=4, max_enc_steps=T, max_dec_steps=10, vocab_size=2000,
                  coverage=True)
    rows = corpus.rows(23, "q")
    rows[5]["uuid"] = ""  # an empty uuid is written back as is (the serial writer's rule)
    cin, cout = ExampleCoding(IN_COLS, [DataTypes.STRING] * 3), ExampleCoding(OUT_COLS, [DataTypes.STRING] * 4)
    rin, rout = _ring("din"), _ring("dout")
    pool = StreamDecodePacker(rin, rout, cin, cout, vocab, hps, packers=2, n_articles=Na, T=T, max_wait_s=0.0)
    for r in rows:
        rin.push(cin.encode({k: r[k] for k in IN_COLS}))
    rin.close()
    layout, _ = input_layout(Na, T, 1)
    enc_off = [x for x in layout if x[0] == "enc_batch"][0]
    stop = vocab.word2id("[STOP]")
    exs = {e.uuid: e for e in examples_from_rows(rows, vocab, hps)}
    by_ids = {tuple(e.enc_input): e for e in exs.values()}
    hb = hps.replace(batch_size=Na)
    n_batches = n_art = 0
    while True:
        b = pool.poll(block=True)
        if b is None:
            break
        assert b is not pool.NOT_READY
        n_batches += 1
        n_art += b.n_valid
        enc = np.frombuffer(bytes(b.host_pack)[enc_off[1]:enc_off[1] + enc_off[4]], dtype=np.int64).reshape(Na, T)
        # the pack is the one a Batch of these examples gives (padding rows, [START], first target)
        lens =[int(np.nonzero(enc[i] != 1)[0].max()) + 1 for i in range(b.n_valid)]
        mine = [by_ids[tuple(enc[i, :lens[i]].tolist())] for i in range(b.n_valid)]
        ref = pack_host_inputs(host_inputs(Batch(mine, hb, vocab, pad_enc_to=T), hb, 1, need_grad=False), layout)
        assert bytes(b.host_pack) == ref.tobytes()
        # "decoded" summary of article i: its first three tokens, then [STOP]
        pool.send_results(b, [enc[i, :3].tolist() + [stop, 5] for i in range(b.n_valid)])
    pool.close()
    rout.close()
    out = [cout.decode_dict(x) for x in rout]
    assert n_art == len(rows) == len(out)
    assert 1 <= n_batches <= len(rows)
    by_uuid = {o["uuid"]: o for o in out}
    for r in rows:
        o, ex = by_uuid[r["uuid"]], exs[r["uuid"]]
        summary, reference = flink_summary(ex.enc_input[:3] + [stop, 5], vocab, ex.article_oovs,
                                           ex.original_abstract_sents)
        assert o["summary"] == summary and o["reference"] == reference and o["article"] == r["article"]
    for x in (rin, rout):
        x.release()


def test_stream_train_packer_raises_when_its_feed_fails():
    """A row larger than a packer ring stops the native fanout, which closes every packer input:
    the consumer must see an error, not a normal end of stream on truncated input."""
    corpus = SyntheticCorpus(vocab_size=2000, raw_vocab=6000, seed=4, art_mean=80, art_sd=30)
    vocab = corpus.vocab(2000)
    hps = HParams(batch_size=8, max_enc_steps=64, max_dec_steps=12, vocab_size=2000, coverage=True)
    rows = corpus.rows(40)
    rows[20]["article"] = " ".join(["word"] * 40000)  # ~200 KB: does not fit a 64 KB packer ring
    coding = ExampleCoding(IN_COLS, [DataTypes.STRING] * 3)
    rin = _ring("in")
    sp = StreamTrainPacker(rin, coding, vocab, hps, 2, pad_enc_to=64, ring_bytes=1 << 16)
    for r in rows:
        rin.push(coding.encode(r))
    rin.close()
    n = 0
    with pytest.raises(RuntimeError, match="fanout"):
        while sp.next_batch() is not None:
            n += 1
    sp.stop()
    assert n <= 3  # the batches before the failed row at most
