"""Native host runtime: crc32c, TF tensor-bundle codec (cross-checked by an independent
pure-Python SSTable parser), checkpoint manager, shared-memory SPSC ring."""
import multiprocessing as mp
import os
import struct
import time
import uuid

import numpy as np
import pytest
import torch

from textsummarization_on_flink_amd.config import HParams
from textsummarization_on_flink_amd.models.params import build_params
from textsummarization_on_flink_amd.runtime.native import crc32c
from textsummarization_on_flink_amd.runtime.ring import RecordRing, RingDrainer
from textsummarization_on_flink_amd.runtime.tf_bundle import list_bundle, load_bundle, save_bundle
from textsummarization_on_flink_amd.train import checkpoint as ck


def test_crc32c_known_vectors():
    assert crc32c(b"123456789") == 0xE3069283
    assert crc32c(b"") == 0
    m = crc32c(b"123456789", masked=True)
    assert m == ((((0xE3069283 >> 15) | (0xE3069283 << 17)) + 0xA282EAD8) & 0xFFFFFFFF)


def _varint(b, p):
    r = s = 0
    while True:
        x = b[p]; p += 1
        r |= (x & 0x7F) << s
        if not x & 0x80:
            return r, p
        s += 7


def _parse_block(f, off, size):
    blk = f[off:off + size]
    trailer = f[off + size:off + size + 5]
    assert trailer[0] == 0
    crc = struct.unpack("<I", trailer[1:])[0]
    c = crc32c(blk + b"\x00")
    assert crc == ((((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF)
    nrest = struct.unpack("<I", blk[-4:])[0]
    end = len(blk) - 4 - 4 * nrest
    p, key, out = 0, b"", []
    while p < end:
        sh, p = _varint(blk, p)
        ns, p = _varint(blk, p)
        vl, p = _varint(blk, p)
        key = key[:sh] + blk[p:p + ns]; p += ns
        out.append((key, blk[p:p + vl])); p += vl
    return out


def test_bundle_roundtrip_and_sstable_format(tmp_path):
    prefix = str(tmp_path / "model.ckpt-7")
    rng = np.random.default_rng(0)
    tensors = {f"v{i:03d}/w": rng.standard_normal((i + 1, 3)).astype(np.float32) for i in range(40)}
    tensors["global_step"] = np.array(7, np.int32)
    tensors["ids"] = np.arange(10, dtype=np.int64)
    save_bundle(prefix, tensors)
    back = load_bundle(prefix)
    assert list(back) == sorted(tensors)
    for k, v in tensors.items():
        np.testing.assert_array_equal(back[k], v)
    # independent parse of the .index SSTable
    f = open(prefix + ".index", "rb").read()
    assert struct.unpack("<Q", f[-8:])[0] == 0xDB4775248B80FB57
    p = len(f) - 48
    mo, p = _varint(f, p); ms, p = _varint(f, p); io, p = _varint(f, p); isz, p = _varint(f, p)
    idx = _parse_block(f, io, isz)
    keys = []
    for _, h in idx:
        bo, q = _varint(h, 0); bs, q = _varint(h, q)
        keys += [k for k, _ in _parse_block(f, bo, bs)]
    assert keys[0] == b"" and keys[1:] == sorted(k.encode() for k in tensors)
    assert list_bundle(prefix)["v005/w"][1] == (6, 3)
    # corrupt data -> crc error
    d = bytearray(open(prefix + ".data-00000-of-00001", "rb").read())
    d[5] ^= 0xFF
    open(prefix + ".data-00000-of-00001", "wb").write(bytes(d))
    with pytest.raises(OSError):
        load_bundle(prefix)


def test_saver_rotation_restore_and_inspect(tmp_path):
    hps = HParams(emb_dim=32, hidden_dim=32, coverage=True)
    p = build_params(hps, 300).enable_adagrad(0.1)
    s = ck.Saver(str(tmp_path / "train"), max_to_keep=2)
    for step in (1, 2, 3):
        s.save(p, step)
    latest = ck.latest_checkpoint(str(tmp_path / "train"))
    assert latest.endswith("model.ckpt-3")
    st = ck.read_state(str(tmp_path / "train"))
    assert [os.path.basename(x) for x in st[1]] == ["model.ckpt-2", "model.ckpt-3"]
    assert not os.path.exists(str(tmp_path / "train" / "model.ckpt-1.index"))
    names = list_bundle(latest)
    assert "seq2seq/decoder/attention_decoder/coverage/w_c" in names
    assert "seq2seq/embedding/embedding/Adagrad" in names and "global_step" in names
    q = build_params(hps, 300, seed=5).enable_adagrad(0.1)
    path, step = ck.load_ckpt(str(tmp_path), q, max_retries=0)
    assert step == 3 and torch.equal(q.flat, p.flat) and torch.equal(q.accum, p.accum)
    assert ck.inspect_checkpoint(latest)["some_infnan"] == []
    with pytest.raises(RuntimeError):
        ck.load_ckpt(str(tmp_path / "nowhere"), q, max_retries=1, sleep_s=0.01)


def test_convert_to_coverage_and_restore_best(tmp_path):
    hps = HParams(emb_dim=32, hidden_dim=32, coverage=False)
    p = build_params(hps, 300).enable_adagrad(0.1)
    ck.Saver(str(tmp_path / "train")).save(p, 11)
    hc = hps.replace(coverage=True)
    pc = build_params(hc, 300, seed=9).enable_adagrad(0.1)
    new = ck.convert_to_coverage_model(str(tmp_path), pc)
    assert new.endswith("model.ckpt-11_cov_init")
    t = load_bundle(new)
    np.testing.assert_array_equal(t["seq2seq/embedding/embedding"], p["seq2seq/embedding/embedding"].numpy())
    assert "seq2seq/decoder/attention_decoder/coverage/w_c" in t
    # eval best -> train
    ck.Saver(str(tmp_path / "eval"), prefix="bestmodel", latest_filename="checkpoint_best").save(p, 20)
    out = ck.restore_best_model(str(tmp_path), build_params(hps, 300).enable_adagrad(0.1))
    assert os.path.basename(out) == "model-20"


def _producer(name, n):
    r = RecordRing.open(name)
    for i in range(n):
        r.push(f"rec-{i}".encode() * (1 + i % 50))
    r.close()
    r.release(unlink=False)


def test_ring_cross_process_wraparound():
    name = "/tsamd_test_" + uuid.uuid4().hex[:8]
    ring = RecordRing.create(name, capacity=8192)
    try:
        ctx = mp.get_context("spawn")
        pr = ctx.Process(target=_producer, args=(name, 500))
        pr.start()
        got = list(ring)
        pr.join(60)
        assert pr.exitcode == 0
        assert got == [f"rec-{i}".encode() * (1 + i % 50) for i in range(500)]
        assert ring.stats()["in"] == ring.stats()["out"] == 500
    finally:
        ring.release()


def test_ring_drainer_emits_immediately():
    """Issue-6 regression: result k is observed before input k+1 is produced."""
    ring = RecordRing.create("/tsamd_drain_" + uuid.uuid4().hex[:8], capacity=1 << 16)
    seen = []
    d = RingDrainer(ring, lambda r: seen.append((r, time.monotonic())), poll_ms=5)
    d.start()
    try:
        for i in range(5):
            ring.push(b"r%d" % i)
            t0 = time.monotonic()
            while len(seen) < i + 1 and time.monotonic() - t0 < 5:
                time.sleep(0.001)
            assert len(seen) == i + 1, "record not emitted before the next one was produced"
        ring.close()
        d.join(5)
        assert not d.is_alive() and d.error is None and d.count == 5
    finally:
        ring.release()
