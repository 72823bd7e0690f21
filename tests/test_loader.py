"""Multi-process input pipeline (data/loader.py) vs the threaded Batcher: same examples, each
read exactly once per pass, packs byte-identical to the engine's own host packing."""
import numpy as np
import pytest

from textsummarization_on_flink_amd.config import HParams
from textsummarization_on_flink_amd.data import binfmt
from textsummarization_on_flink_amd.data.batch import Batch, Example
from textsummarization_on_flink_amd.data.loader import ProcessBatcher
from textsummarization_on_flink_amd.data.vocab import Vocab, abstract2sents
from textsummarization_on_flink_amd.models.pointer_generator import host_inputs, input_layout, pack_host_inputs

from helpers import make_dataset


def _unpack(pb, layout):
    buf = np.frombuffer(pb.host_pack, dtype=np.uint8)
    out = {}
    for name, o, shp, dt, nb in layout:
        npdt = {"torch.int64": np.int64, "torch.int32": np.int32, "torch.float32": np.float32}[str(dt)]
        out[name] = buf[o:o + nb].view(npdt).reshape(shp)
    return out


@pytest.mark.parametrize("workers", [1, 3])
def test_single_pass_reads_every_example_once(tmp_path, workers):
    d, vp, _ = make_dataset(str(tmp_path), n_files=3, per_file=7)
    vocab = Vocab(vp, 500)
    T, D, B = 48, 12, 4
    hps = HParams(batch_size=B, max_enc_steps=T, max_dec_steps=D, vocab_size=500, pointer_gen=True, coverage=True)
    pattern = f"{d}/train_*.bin"
    ref = []
    for art, abs_ in binfmt.text_generator(binfmt.example_generator(pattern, True)):
        ex = Example(art, [s.strip() for s in abstract2sents(abs_)], vocab, hps)
        ref.append(tuple(ex.enc_input))
    pb_all = list(ProcessBatcher(pattern, vocab, hps, single_pass=True, workers=workers, seed=5, pad_enc_to=T))
    layout, total = input_layout(B, T, D)
    got, tokens = [], 0
    for pb in pb_all:
        assert pb.enc_batch.shape == (B, T) and len(pb.host_pack) == total
        h = _unpack(pb, layout)
        for r in range(pb.n_valid):
            got.append(tuple(int(x) for x in h["enc_batch"][r, :h["enc_lens"][r]]))
        tokens += pb.num_tokens()
        # padding rows of a short final batch carry zero loss weight
        assert np.all(h["rowg"][:, pb.n_valid:] == 0)
    assert sorted(got) == sorted(ref)  # every record exactly once
    assert tokens == sum(len(x) for x in ref) + sum(
        min(len(Example(a, [s.strip() for s in abstract2sents(b)], vocab, hps).dec_input), D)
        for a, b in binfmt.text_generator(binfmt.example_generator(pattern, True)))


def test_pack_matches_engine_host_packing(tmp_path):
    """A worker's bytes equal pack_host_inputs(host_inputs(Batch)) of the same examples."""
    d, vp, _ = make_dataset(str(tmp_path), n_files=1, per_file=4)
    vocab = Vocab(vp, 500)
    T, D, B = 40, 10, 4
    hps = HParams(batch_size=B, max_enc_steps=T, max_dec_steps=D, vocab_size=500, pointer_gen=True, coverage=True)
    pattern = f"{d}/val_*.bin"
    (pb,) = list(ProcessBatcher(pattern, vocab, hps, single_pass=True, workers=1, seed=0, pad_enc_to=T))
    exs = [Example(a, [s.strip() for s in abstract2sents(b)], vocab, hps)
           for a, b in binfmt.text_generator(binfmt.example_generator(pattern, True))]
    exs.sort(key=lambda e: e.enc_len)  # the worker's length bucketing
    ref = pack_host_inputs(host_inputs(Batch(exs, hps, vocab, pad_enc_to=T), hps, D, sort_rows=True),
                           input_layout(B, T, D)[0])
    assert bytes(pb.host_pack) == ref.tobytes()


def test_endless_mode_stops_promptly(tmp_path):
    d, vp, _ = make_dataset(str(tmp_path), n_files=2, per_file=5)
    vocab = Vocab(vp, 500)
    hps = HParams(batch_size=2, max_enc_steps=32, max_dec_steps=8, vocab_size=500)
    pb = ProcessBatcher(f"{d}/train_*.bin", vocab, hps, single_pass=False, workers=2, seed=1, pad_enc_to=32,
                        bucketing_cache_size=2, ring_bytes=1 << 20)
    for _ in range(25):  # more than one pass: the workers loop over the files
        assert pb.next_batch(timeout=30) is not None
    procs = list(pb.procs)
    pb.stop()
    assert all(not p.is_alive() for p in procs)


def _ref_inputs(pattern, vocab, hps):
    return [tuple(Example(a, [s.strip() for s in abstract2sents(b)], vocab, hps).enc_input)
            for a, b in binfmt.text_generator(binfmt.example_generator(pattern, True))]


def test_dp_ranks_read_disjoint_shares(tmp_path):
    """2 data-parallel ranks x 3 loader workers, single pass: every record is read exactly once
    over the whole job (record k -> rank k % world -> worker (k // world) % workers)."""
    d, vp, _ = make_dataset(str(tmp_path), n_files=3, per_file=7)
    vocab = Vocab(vp, 500)
    T, D, B = 48, 12, 2
    hps = HParams(batch_size=B, max_enc_steps=T, max_dec_steps=D, vocab_size=500, pointer_gen=True, coverage=True)
    pattern = f"{d}/train_*.bin"
    layout, _ = input_layout(B, T, D)
    per_rank = []
    for rank in range(2):
        got = []
        for pb in ProcessBatcher(pattern, vocab, hps, single_pass=True, workers=3, seed=5, pad_enc_to=T,
                                 rank=rank, world=2):
            h = _unpack(pb, layout)
            got += [tuple(int(x) for x in h["enc_batch"][r, :h["enc_lens"][r]]) for r in range(pb.n_valid)]
        per_rank.append(got)
    ref = _ref_inputs(pattern, vocab, hps)
    assert len(per_rank[0]) == 11 and len(per_rank[1]) == 10  # 21 records: k % 2
    assert sorted(per_rank[0] + per_rank[1]) == sorted(ref)


def test_dp_ranks_threaded_batcher_disjoint(tmp_path):
    from textsummarization_on_flink_amd.data.batcher import Batcher
    d, vp, _ = make_dataset(str(tmp_path), n_files=2, per_file=9)
    vocab = Vocab(vp, 500)
    hps = HParams(batch_size=3, max_enc_steps=48, max_dec_steps=12, vocab_size=500)
    pattern = f"{d}/train_*.bin"
    got = []
    for rank in range(3):
        bt = Batcher(pattern, vocab, hps, single_pass=True, seed=11, rank=rank, world=3)
        for b in bt:
            got += [tuple(int(x) for x in b.enc_batch[r, :b.enc_lens[r]]) for r in range(int(b.valid.sum()))]
        bt.stop()
    assert sorted(got) == sorted(_ref_inputs(pattern, vocab, hps))
    # without a shared seed each rank would shuffle the files differently: shards would overlap
    with pytest.raises(ValueError, match="seed"):
        Batcher(pattern, vocab, hps, single_pass=True, seed=None, rank=0, world=3)


def test_crashed_worker_is_not_end_of_data(tmp_path, monkeypatch):
    """A worker that dies without delivering its error record (exit code 1, ring closed) makes
    next_batch raise instead of silently dropping 1/n of the stream."""
    import json as _json

    import textsummarization_on_flink_amd.data.loader as L

    class _Json:
        loads = staticmethod(_json.loads)

        @staticmethod
        def dumps(obj, *a, **k):
            if isinstance(obj, dict) and "error" in obj:
                raise OSError("cannot report")
            return _json.dumps(obj, *a, **k)

    def boom(*a, **k):
        raise IOError("disk gone")
        yield  # noqa: unreachable -- generator

    d, vp, _ = make_dataset(str(tmp_path), n_files=1, per_file=4)
    monkeypatch.setattr(L, "json", _Json)
    monkeypatch.setattr(L.binfmt, "example_generator", boom)  # inherited by the forked workers
    hps = HParams(batch_size=2, max_enc_steps=32, max_dec_steps=8, vocab_size=500)
    pb = ProcessBatcher(f"{d}/train_*.bin", Vocab(vp, 500), hps, single_pass=False, workers=2, seed=1,
                        pad_enc_to=32, ring_bytes=1 << 20)
    try:
        with pytest.raises(RuntimeError, match="stopped|died"):
            pb.next_batch(timeout=30)
    finally:
        pb.stop()
