"""Binary HBM snapshots (swps_save / swps_restore, swps_w2v_save_state /
swps_w2v_restore_state) on the GPU.

The reference can only dump values as text at 6 significant digits and drops
the AdaGrad accumulators (SURVEY.md §5 'Checkpoint / resume': "training
cannot be resumed exactly").  The snapshot keeps every row element bit for
bit, and with the worker state (cache, batch cursor, both LCG streams) a run
stopped and resumed — at an epoch boundary or mid-epoch — ends bit-identical
to the uninterrupted run."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, zipf_corpus

pytestmark = pytest.mark.gpu


def _rows(t, keys):
    import torch
    kt = torch.as_tensor(np.asarray(keys, dtype=np.int64), device="cuda")
    return t.export(kt).cpu().numpy()


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_table_snapshot_roundtrip_bitexact(lib, gpu, tmp_path, dtype):
    import torch
    t = lib.Table("w2v", dim=24, capacity=5000, dtype=dtype, learning_rate=0.7, init="hash", seed=5)
    rng = np.random.default_rng(1)
    keys = rng.choice(2 ** 40, 3000, replace=False).astype(np.int64)
    kt = torch.as_tensor(keys, device="cuda")
    t.pull(kt)
    g = torch.as_tensor(rng.standard_normal((3000, 48)), device="cuda")
    t.push(kt, g)  # non-zero AdaGrad accumulators
    path = str(tmp_path / "t.snap")
    t.save(path)
    t2 = lib.Table("w2v", dim=24, capacity=5000, dtype=dtype, learning_rate=0.7, init="zero")
    t2.restore(path)
    assert t2.size() == 3000
    assert np.array_equal(np.sort(t2.keys()), np.sort(keys.astype(np.uint64)))
    a, b = _rows(t, keys), _rows(t2, keys)
    assert (a[:, 48:] != 0).any()
    assert np.array_equal(a, b)


def test_table_snapshot_hashfrag_filter(lib, gpu, tmp_path):
    """restore(node_id) keeps the keys BasicHashFrag gives that node
    (server.h:49-62): two nodes partition a one-node snapshot exactly."""
    import torch
    t = lib.Table("lr", capacity=10000, dtype="f32", learning_rate=0.05, init="hash", seed=2)
    keys = np.arange(1, 4001, dtype=np.int64) * 7919
    t.pull(torch.as_tensor(keys, device="cuda"))
    path = str(tmp_path / "lr.snap")
    t.save(path)
    frag = lib.hashfrag_table(1000, 2)
    owner = lib.to_node_id(keys.astype(np.uint64), 1000, frag)
    got = []
    for node in (1, 2):
        tn = lib.Table("lr", capacity=10000, dtype="f32", learning_rate=0.05, init="zero")
        tn.restore(path, frag_num=1000, world=2, node_id=node)
        kn = np.sort(tn.keys())
        assert np.array_equal(kn, np.sort(keys[owner == node].astype(np.uint64)))
        assert np.array_equal(_rows(tn, kn), _rows(t, kn))
        got.append(kn)
    assert len(got[0]) + len(got[1]) == len(keys)


def test_snapshot_rejects_corrupt_and_mismatched(lib, gpu, tmp_path):
    import torch
    t = lib.Table("w2v", dim=8, capacity=100, dtype="f32", init="hash", seed=1)
    t.pull(torch.arange(1, 51, dtype=torch.int64, device="cuda"))
    path = str(tmp_path / "a.snap")
    t.save(path)
    raw = bytearray(open(path, "rb").read())
    bad = str(tmp_path / "bad.snap")
    raw2 = bytearray(raw)
    raw2[len(raw2) // 2] ^= 0x40
    open(bad, "wb").write(bytes(raw2))
    with pytest.raises(lib.SwpsError, match="checksum"):
        lib.Table("w2v", dim=8, capacity=100, dtype="f32").restore(bad)
    open(bad, "wb").write(bytes(raw[:-20]))
    with pytest.raises(lib.SwpsError, match="truncated|checksum"):
        lib.Table("w2v", dim=8, capacity=100, dtype="f32").restore(bad)
    for kw in (dict(dim=16, dtype="f32"), dict(dim=8, dtype="f64")):
        with pytest.raises(lib.SwpsError, match="snapshot"):
            lib.Table("w2v", capacity=100, **kw).restore(path)
    with pytest.raises(lib.SwpsError):
        lib.Table("w2v", dim=8, capacity=10, dtype="f32").restore(path)  # 50 rows > capacity
    open(bad, "wb").write(b"not a snapshot at all")
    with pytest.raises(lib.SwpsError, match="snapshot"):
        lib.Table("w2v", dim=8, capacity=100, dtype="f32").restore(bad)


def _w2v(lib, path, dtype, init, **kw):
    t = lib.Table("w2v", dim=16, capacity=2000, dtype=dtype, learning_rate=0.7, init="hash", seed=3)
    w = lib.Word2Vec(t, init=init, **kw)
    w.load_text(path)
    return t, w


@pytest.mark.parametrize("dtype,fp64i,extra", [("f64", True, {}), ("f32", True, {}), ("f32", False, {}),
                                               ("f32", "bfp40", {}),
                                               ("f32", False, {"sampler": "alias"}),
                                               ("f64", True, {"minibatch_vocab": True, "key_mode": "atoi"})])
@pytest.mark.parametrize("stop", ["epoch", "mid"])
def test_w2v_resume_bitexact(lib, gpu, tmp_path, dtype, fp64i, extra, stop):
    """train E batches | save | fresh table + worker, restore | train the
    rest == the uninterrupted run, bit for bit (rows incl. AdaGrad sums, LCG
    states, counters)."""
    if extra.get("key_mode") == "atoi":
        from conftest import int_corpus
        path = int_corpus(str(tmp_path / "c.txt"), 150, 300, seed=21)
    else:
        path = zipf_corpus(str(tmp_path / "c.txt"), 150, 300, seed=21)
    kw = dict(window=3, negative=4, minibatch=11, sample=1e-3, unigram_size=10 ** 6, fp64_intermediates=fp64i,
              **extra)
    _, ref = _w2v(lib, path, dtype, "ref", **kw)
    ref.init()
    nb = ref.info()["batches"]
    total = 3 * nb
    ref.train_batches(total)
    ref.sync()
    first = nb if stop == "epoch" else nb + nb // 2 + 1
    ta, a = _w2v(lib, path, dtype, "ref", **kw)
    a.init()
    a.train_batches(first)
    prefix = str(tmp_path / "ck")
    a.save(prefix)
    a.train_batches(total - first)  # saving does not perturb the run
    a.sync()
    tb, b = _w2v(lib, path, dtype, "table", **kw)
    b.restore(prefix)
    b.train_batches(total - first)
    b.sync()
    for w in (a, b):
        sr, sw = ref.stats(), w.stats()
        for k in ("batches", "kept", "words", "pairs", "lstate", "fstate", "pulled", "pushed"):
            assert sw[k] == sr[k], k
        assert np.array_equal(w.get_params(), ref.get_params())


def test_w2v_restore_preconditions(lib, gpu, tmp_path):
    path = zipf_corpus(str(tmp_path / "c.txt"), 60, 200, seed=4)
    kw = dict(window=3, negative=4, minibatch=11, sample=1e-3, unigram_size=10 ** 6)
    _, a = _w2v(lib, path, "f32", "ref", **kw)
    a.init()
    a.train_batches(3)
    prefix = str(tmp_path / "ck")
    a.save(prefix)
    # worker state without its table: the vocab rows are missing
    t = lib.Table("w2v", dim=16, capacity=2000, dtype="f32")
    w = lib.Word2Vec(t, init="table", **kw)
    w.load_text(path)
    with pytest.raises(lib.SwpsError, match="table"):
        w.restore_state(prefix + ".w2v")
    # a different corpus or config
    other = zipf_corpus(str(tmp_path / "d.txt"), 61, 200, seed=5)
    for p, k in ((other, kw), (path, dict(kw, window=4))):
        t = lib.Table("w2v", dim=16, capacity=2000, dtype="f32")
        t.restore(prefix + ".table")
        w = lib.Word2Vec(t, init="table", **k)
        w.load_text(p)
        with pytest.raises(lib.SwpsError, match="corpus|config"):
            w.restore_state(prefix + ".w2v")
    # an already-initialised worker
    with pytest.raises(lib.SwpsError, match="fresh"):
        a.restore_state(prefix + ".w2v")
    # the table file of ANOTHER save (later step) with this worker state
    a.train_batches(2)
    a.save(prefix + "2")
    t = lib.Table("w2v", dim=16, capacity=2000, dtype="f32")
    t.restore(prefix + "2.table")
    w = lib.Word2Vec(t, init="table", **kw)
    w.load_text(path)
    with pytest.raises(lib.SwpsError, match="table snapshot"):
        w.restore_state(prefix + ".w2v")
    # a table whose push rule (server learning rate) differs from the snapshot's
    with pytest.raises(lib.SwpsError, match="push rule"):
        lib.Table("w2v", dim=16, capacity=2000, dtype="f32", learning_rate=0.5).restore(prefix + ".table")
    # saves are atomic: no temporary is left behind, and a failed write keeps the old file
    import glob
    assert not glob.glob(prefix + "*.tmp")


def test_lr_resume_from_table_snapshot(lib, gpu, tmp_path):
    """LR keeps no state beyond the table between epochs: 2 epochs | save |
    restore | 3 epochs == 5 epochs (weights, AdaGrad sums, epoch errors)."""
    data = os.path.join(GOLDEN, "lr_data.txt")
    t = lib.Table("lr", capacity=4096, dtype="f32", learning_rate=0.05)
    m = lib.LR(t, minibatch=200)
    m.load_text(data)
    m.init()
    e_all = m.train(5)
    t1 = lib.Table("lr", capacity=4096, dtype="f32", learning_rate=0.05)
    m1 = lib.LR(t1, minibatch=200)
    m1.load_text(data)
    m1.init()
    e_a = m1.train(2)
    snap = str(tmp_path / "lr.snap")
    t1.save(snap)
    t2 = lib.Table("lr", capacity=4096, dtype="f32", learning_rate=0.05, init="zero")
    t2.restore(snap)
    m2 = lib.LR(t2, minibatch=200, init_ref=False)
    m2.load_text(data)
    m2.init()
    e_b = m2.train(3)
    assert np.array_equal(np.concatenate([e_a, e_b]), e_all)
    k0, w0, g0 = m.params()
    k2, w2, g2 = m2.params()
    o0, o2 = np.argsort(k0), np.argsort(k2)
    assert np.array_equal(k0[o0], k2[o2])
    assert np.array_equal(w0[o0], w2[o2]) and np.array_equal(g0[o0], g2[o2])


def test_sharded_w2v_resume_world1(lib, gpu, gloo1, tmp_path):
    """The sharded lockstep driver saves each rank's shard + worker state and
    resumes bit-identically."""
    from swiftmpi_amd.dist import ShardedWord2Vec
    path = zipf_corpus(str(tmp_path / "c.txt"), 120, 300, seed=31)
    kw = dict(window=3, negative=4, minibatch=13, sample=1e-3, unigram_size=10 ** 6, fp64_intermediates=False)

    def make():
        t = lib.Table("w2v", dim=16, capacity=1000, dtype="f32", learning_rate=0.7, init="hash", seed=3)
        sh = ShardedWord2Vec(t, **kw)
        sh.load_text(path)
        return sh

    ref = make()
    ref.init()
    ref.train(3)
    a = make()
    a.init()
    a.train_steps(a.steps_per_epoch + 2)
    prefix = str(tmp_path / "sh")
    a.save(prefix)
    b = make()
    b.restore(prefix)
    b.train_steps(3 * b.steps_per_epoch - b.cursor)
    # a save without its commit marker (a crash between the ranks' files and the marker) is refused
    import os
    os.rename(prefix + ".commit", prefix + ".commit.bak")
    with pytest.raises(lib.SwpsError, match="commit"):
        make().restore(prefix)
    os.rename(prefix + ".commit.bak", prefix + ".commit")
    # a second save that dies after this rank's new shard + worker state but before its .json
    # (ADVICE r2): the old marker is gone, so the mixed files are never resumed
    import swiftmpi_amd.dist as sd
    real = sd._write_json_atomic

    def crash(path, obj):
        if path.endswith(".json"):
            raise OSError("killed between the table write and the json write")
        real(path, obj)
    sd._write_json_atomic = crash
    try:
        with pytest.raises(OSError):
            a.save(prefix)
    finally:
        sd._write_json_atomic = real
    with pytest.raises(lib.SwpsError, match="commit"):
        make().restore(prefix)
    b.sync()
    kr, rr = ref.shard_rows()
    kb, rb = b.shard_rows()
    o1, o2 = np.argsort(kr), np.argsort(kb)
    assert np.array_equal(kr[o1], kb[o2]) and np.array_equal(rr[o1], rb[o2])
    assert b.stats()["lstate"] == ref.stats()["lstate"]
