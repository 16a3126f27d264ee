"""Sparse LR on the GPU against the oracle and the reference binary's outputs."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DATA = os.path.join(GOLDEN, "lr_data.txt")


def run_gpu(lib, epochs, B=200, lr=0.05):
    t = lib.Table("lr", capacity=4096, dtype="f32", learning_rate=lr)
    m = lib.LR(t, minibatch=B)
    m.load_text(DATA)
    m.init()
    err = m.train(epochs)
    return t, m, err


@pytest.mark.parametrize("B", [200, 7, 1604])
def test_lr_matches_oracle(lib, oracle_mod, gpu, B):
    orc = oracle_mod.LR(DATA, B, 0.05)
    e_o = orc.train(5)
    _, m, e_g = run_gpu(lib, 5, B=B)
    ko, wo, go = orc.params()
    kg, wg, gg = m.params()
    assert np.array_equal(ko, kg)
    assert np.allclose(wg, wo, rtol=1e-5, atol=1e-6), np.abs(wg - wo).max()
    assert np.allclose(gg, go, rtol=1e-5, atol=1e-7)
    assert np.allclose(e_g, e_o, rtol=1e-5)


def test_lr_reference_quality(lib, oracle_mod, gpu):
    q = json.load(open(os.path.join(GOLDEN, "lr_reference_quality.json")))
    for ep, exp in q["epochs"].items():
        _, m, _ = run_gpu(lib, int(ep))
        p, t = m.predict()
        p6 = np.array([float("%g" % x) for x in p], dtype=np.float32)
        ll, acc = oracle_mod.logloss_accuracy(p6, t)
        assert abs(ll - exp["logloss"]) / exp["logloss"] < 0.01  # north star: log-loss within 1 %
        assert round(acc, 3) == exp["accuracy"]


def test_lr_dump_load_roundtrip(lib, gpu, tmp_path):
    t, m, _ = run_gpu(lib, 3)
    path = str(tmp_path / "param.txt")
    t.dump(path)
    lines = open(path).read().strip().split("\n")
    assert len(lines) == 113 and all(len(l.split("\t")) == 2 for l in lines)
    t2 = lib.Table("lr", capacity=4096, dtype="f32", learning_rate=0.05)
    t2.load(path)
    import torch
    keys = torch.tensor([int(l.split("\t")[0]) for l in lines], dtype=torch.int64, device="cuda")
    a = t.export(keys).cpu().numpy()
    b = t2.export(keys).cpu().numpy()
    assert np.allclose(a[:, 0], b[:, 0], rtol=1e-5) and (b[:, 1] == 0).all()


def _gen_float_draws(n):
    """LRPullAccessMethod::init_param's draws (lr.cpp:48-50 -> random.h gen_float):
    y = y * 4903917 + 11 from ULONG_MAX / 2, value (float)y / 2^64 (round to nearest even)."""
    out, y = np.zeros(n, dtype=np.float32), (2 ** 64 - 1) // 2
    for i in range(n):
        y = (y * 4903917 + 11) % 2 ** 64
        b = y.bit_length()
        q = y
        if b > 24:
            sh = b - 24
            q, r = y >> sh, y & ((1 << sh) - 1)
            if r > 1 << (sh - 1) or (r == 1 << (sh - 1) and q & 1):
                q += 1
            q <<= sh
        out[i] = np.float32(q / 2.0 ** 64)
    return out


def test_lr_init_after_partial_dump(lib, gpu, tmp_path):
    """Predict mode on data with features the dump never saw (lr.cpp:297-300 ->
    server.h:49-62, then the first pull): the dumped keys keep their values, the
    others get LRPullAccessMethod::init_param's gen_float() draws in first-pull
    order (lr.cpp:48-50) — the same draws a fresh table gives its first keys —
    and init does not fail on the misses."""
    t0 = lib.Table("lr", capacity=4096, dtype="f32", learning_rate=0.05)
    m0 = lib.LR(t0, minibatch=200)
    m0.load_text(DATA)
    m0.init()
    k0, w0, _ = m0.params()
    held = np.zeros(len(k0), dtype=bool)
    held[::3] = True
    vals = 0.25 + 1e-3 * np.arange(len(k0))
    path = str(tmp_path / "partial.txt")
    with open(path, "w") as f:
        for k, x in zip(k0[held], vals[held]):
            f.write("%d\t%g\n" % (k, x))
    t1 = lib.Table("lr", capacity=4096, dtype="f32", learning_rate=0.05)
    t1.load(path)
    m1 = lib.LR(t1, minibatch=200)
    m1.load_text(DATA)
    m1.init()
    k1, w1, g1 = m1.params()
    assert np.array_equal(k0, k1)
    assert np.array_equal(w1[held], np.array(["%g" % x for x in vals[held]], dtype=np.float32))
    # the fresh table's draws give each key's first-pull index (vid)
    seq = _gen_float_draws(len(k0))
    index = {float(x): i for i, x in enumerate(seq)}
    assert len(index) == len(seq)
    vid = np.array([index[float(x)] for x in w0])
    miss = np.flatnonzero(~held)
    miss = miss[np.argsort(vid[miss])]
    assert np.array_equal(w1[miss], seq[:len(miss)])
    assert (g1 == 0).all()
    m1.train(1)  # and the held keys train like any other
    assert np.isfinite(m1.params()[1]).all()


@pytest.mark.parametrize("B", [200, 13])
def test_sharded_lr_world1_equals_unsharded(lib, gpu, gloo1, B):
    """The sharded request / serve / step / push protocol (one rank, gloo)
    reproduces the single-GPU LR bit for bit: weights, AdaGrad sums, epoch
    errors and predictions."""
    from swiftmpi_amd.dist import ShardedLR
    t = lib.Table("lr", capacity=4096, dtype="f32", learning_rate=0.05, init="hash", seed=9)
    sh = ShardedLR(t, minibatch=B)
    sh.load_text(DATA)
    sh.init()
    e_s = sh.train(3)
    p_s, _ = sh.predict()
    t1 = lib.Table("lr", capacity=4096, dtype="f32", learning_rate=0.05, init="hash", seed=9)
    m = lib.LR(t1, minibatch=B, init_ref=False)
    m.load_text(DATA)
    m.init()
    e_1 = m.train(3)
    p_1, _ = m.predict()
    k1, w1, g1 = m.params()
    ks, ws, gs = sh.shard_weights()
    assert np.array_equal(ks.astype(np.uint32), k1)
    assert np.array_equal(ws, w1) and np.array_equal(gs, g1)
    assert np.array_equal(e_s, e_1) and np.array_equal(p_s, p_1)


def test_lr_criteo_shape_properties(lib, gpu):
    """Config-3-shaped data (39 hashed features per row, 2^24 key space) at a
    few batches: training is deterministic run to run, weights stay finite,
    and the training error falls from the first epoch to the third."""
    from swiftmpi_amd.synth import criteo
    y, off, f, v = criteo(20000, seed=3)
    errs, ws = [], []
    for _ in range(2):
        t = lib.Table("lr", capacity=1 << 20, dtype="f32", learning_rate=0.05, init="hash", seed=1)
        m = lib.LR(t, minibatch=4095, init_ref=False)
        m.load_csr(y, off, f, v)
        m.init()
        errs.append(m.train(3))
        ws.append(m.params()[1])
    assert np.array_equal(errs[0], errs[1]) and np.array_equal(ws[0], ws[1])
    assert np.isfinite(ws[0]).all() and errs[0][2] < errs[0][0]


@pytest.mark.parametrize("plan", ["step", "none"])
@pytest.mark.parametrize("B", [200, 1604])
def test_lr_fast_sums_within_1e5_of_oracle(lib, oracle_mod, gpu, B, plan):
    """Fast mode (fp64 per-key sums, long runs tree-reduced over a wave
    instead of the reference's sequential fp32 chain): weights and AdaGrad
    sums within 1e-5 relative of the oracle after 5 epochs, epoch errors
    within 1e-5, log-loss within 1 % of the reference binary's, and run to
    run bit-identical."""
    orc = oracle_mod.LR(DATA, B, 0.05)
    e_o = orc.train(5)
    ko, wo, go = orc.params()
    runs = []
    for _ in range(2):
        t = lib.Table("lr", capacity=4096, dtype="f32", learning_rate=0.05)
        m = lib.LR(t, minibatch=B, fast_sums=True, plan=plan)
        m.load_text(DATA)
        m.init()
        e = m.train(5)
        runs.append((e, m.params(), m.predict()))
    (e_g, (kg, wg, gg), (p, tgt)), (e_2, (_, w2, _), _) = runs
    assert np.array_equal(e_g, e_2) and np.array_equal(wg, w2)
    assert np.array_equal(ko, kg)
    assert np.allclose(wg, wo, rtol=1e-5, atol=1e-6), np.abs(wg - wo).max()
    assert np.allclose(gg, go, rtol=1e-5, atol=1e-7)
    assert np.allclose(e_g, e_o, rtol=1e-5)


def test_lr_fast_sums_reference_quality(lib, oracle_mod, gpu):
    q = json.load(open(os.path.join(GOLDEN, "lr_reference_quality.json")))
    for ep, exp in q["epochs"].items():
        t = lib.Table("lr", capacity=4096, dtype="f32", learning_rate=0.05)
        m = lib.LR(t, minibatch=200, fast_sums=True)
        m.load_text(DATA)
        m.init()
        m.train(int(ep))
        p, tg = m.predict()
        p6 = np.array([float("%g" % x) for x in p], dtype=np.float32)
        ll, acc = oracle_mod.logloss_accuracy(p6, tg)
        assert abs(ll - exp["logloss"]) / exp["logloss"] < 0.01


def test_lr_fast_sums_criteo_shape_close_to_exact(lib, gpu):
    """At the Criteo shape (hot categorical features: runs of thousands of
    records — the long-run path), fast sums stay within 1e-5 of the exact
    fp32-chain mode after 3 epochs, relative to the weights' scale (the fp32
    chain's own rounding over runs of thousands of records is ~1e-6 of it;
    the small-data bar against the oracle is element-wise)."""
    from swiftmpi_amd.synth import criteo
    y, off, f, v = criteo(20000, seed=3)
    ws = []
    for fast in (False, True):
        t = lib.Table("lr", capacity=1 << 20, dtype="f32", learning_rate=0.05, init="hash", seed=1)
        m = lib.LR(t, minibatch=4095, init_ref=False, fast_sums=fast)
        m.load_csr(y, off, f, v)
        m.init()
        m.train(3)
        ws.append(m.params()[1])
    assert np.abs(ws[1] - ws[0]).max() <= 1e-5 * np.abs(ws[0]).max(), (np.abs(ws[1] - ws[0]).max(),
                                                                       np.abs(ws[0]).max())


@pytest.mark.parametrize("fast", [False, True])
def test_lr_rows_per_wave_bit_identical(lib, gpu, monkeypatch, fast):
    """k_lr_forward_c (the default: whole rows in record-contiguous chunks) ==
    k_lr_forward_g / _r with the ordered sums through LDS (3 or 2 rows per
    wave by the batch's longest row) == the same with readlane chains == 2
    rows per wave == k_lr_forward_l (a lane per row) == one row per wave, bit
    for bit: Criteo-shaped rows (39 features: 3 per wave), the reference's
    data.txt (its own row lengths), ragged rows of 1-130 features (longer than
    one 40-feature chunk; one row per wave past 64) and 1-3-feature rows (over
    256 rows in one chunk)."""
    from swiftmpi_amd.synth import criteo
    y, off, f, v = criteo(9000, seed=5)
    res = []
    for pack, fc in (("1", "1"), ("0", "1"), ("1", "0"), ("2", "1"), ("3", "1"), ("4", "1")):
        monkeypatch.setenv("SWPS_LR_PACK", pack)
        monkeypatch.setenv("SWPS_LR_FWD_C", fc)
        t = lib.Table("lr", capacity=1 << 18, dtype="f32", learning_rate=0.05, init="hash", seed=1)
        m = lib.LR(t, minibatch=1000, init_ref=False, fast_sums=fast)
        m.load_csr(y, off, f, v)
        m.init()
        e = m.train(2)
        t2 = lib.Table("lr", capacity=4096, dtype="f32", learning_rate=0.05)
        m2 = lib.LR(t2, minibatch=200, fast_sums=fast)
        m2.load_text(DATA)
        m2.init()
        e2 = m2.train(2)
        # ragged rows of 1..130 features (several 40-feature chunks per lane)
        rng = np.random.default_rng(9)
        lens = rng.integers(1, 131, 3000)
        roff = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        feat = rng.integers(0, 5000, int(roff[-1])).astype(np.uint32)
        vals = rng.random(int(roff[-1])).astype(np.float32)
        yl = (rng.random(3000) < 0.5).astype(np.float32)
        t3 = lib.Table("lr", capacity=1 << 14, dtype="f32", learning_rate=0.05, init="hash", seed=2)
        m3 = lib.LR(t3, minibatch=500, init_ref=False, fast_sums=fast)
        m3.load_csr(yl, roff, feat, vals)
        m3.init()
        e3 = m3.train(2)
        # very short rows: a chunk holds more rows than a block has threads
        lens = rng.integers(1, 4, 6000)
        roff = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        feat = rng.integers(0, 3000, int(roff[-1])).astype(np.uint32)
        vals = rng.random(int(roff[-1])).astype(np.float32)
        t4 = lib.Table("lr", capacity=1 << 14, dtype="f32", learning_rate=0.05, init="hash", seed=3)
        m4 = lib.LR(t4, minibatch=2999, init_ref=False, fast_sums=fast)
        m4.load_csr((rng.random(6000) < 0.5).astype(np.float32), roff, feat, vals)
        m4.init()
        e4 = m4.train(2)
        res.append((e, m.params()[1], e2, m2.params()[1], e3, m3.params()[1], e4, m4.params()[1]))
    for r in res[1:]:
        for a, b in zip(res[0], r):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("fast", [False, True])
def test_lr_row_placement_bit_identical(lib, gpu, monkeypatch, fast):
    """The single-GPU init's row layout (keys' rows in first-appearance order by
    (batch, row tile, key): SWPS_LR_PLACE) and the XCD-aware block order of the
    row tiles (key octiles, SWPS_LR_XCD), both off by default (measured
    slower), change where rows live and which block runs where, never a
    result: errors and weights bit for bit with both off, one on, both on,
    and the (batch, key) layout — Criteo shape with 16 row tiles per batch,
    under the three init modes (reference gen_float draws in pull order, the
    table's SWPS_INIT_FLCG draws in call order, key hash)."""
    from swiftmpi_amd.synth import criteo
    y, off, f, v = criteo(12000, seed=11)
    monkeypatch.setenv("SWPS_LR_TILE_BITS", "8")  # 4,096-row batches: 16 tiles
    res = []
    for place, xcd in (("0", "0"), ("1", "1"), ("1", "0"), ("0", "1"), ("2", "0")):
        monkeypatch.setenv("SWPS_LR_PLACE", place)
        monkeypatch.setenv("SWPS_LR_XCD", xcd)
        out = []
        for init, ref in (("hash", False), ("flcg", False), ("hash", True)):
            t = lib.Table("lr", capacity=1 << 19, dtype="f32", learning_rate=0.05, init=init, seed=1)
            m = lib.LR(t, minibatch=4095, init_ref=ref, fast_sums=fast)
            m.load_csr(y, off, f, v)
            m.init()
            out.append(m.train(2))
            out.append(m.params()[1])
            m.close()
            t.close()
        res.append(out)
    for r in res[1:]:
        for a, b in zip(res[0], r):
            assert np.array_equal(a, b)


def test_lr_fused_reduce_bit_identical(lib, gpu, monkeypatch):
    """Fast sums: k_lr_reduce_fused (static long-run list, one launch) == the
    short / long pair with the runtime long list, bit for bit (Criteo shape
    with hot features: long runs present)."""
    from swiftmpi_amd.synth import criteo
    y, off, f, v = criteo(20000, seed=7)
    res = []
    monkeypatch.setenv("SWPS_LR_TILES", "0")  # the record path's two reduce forms
    for fused in ("0", "1"):
        monkeypatch.setenv("SWPS_LR_FUSED", fused)
        t = lib.Table("lr", capacity=1 << 18, dtype="f32", learning_rate=0.05, init="hash", seed=1)
        m = lib.LR(t, minibatch=4095, init_ref=False, fast_sums=True)
        m.load_csr(y, off, f, v)
        m.init()
        e = m.train(2)
        res.append((e, m.params()[1], m.params()[2]))
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b)


@pytest.fixture(scope="module")
def criteo_text(tmp_path_factory):
    """Three config-3 batches: 3 x 65,537 Criteo-shaped rows (a minibatch is
    the next B + nthreads valid lines, lr.cpp:308-354) over the 2^24 key
    space, as the reference's text format (parse_instance2, lr.cpp:103-131)."""
    from swiftmpi_amd.synth import criteo
    y, off, f, v = criteo(3 * 65537, seed=3)
    path = str(tmp_path_factory.mktemp("criteo") / "criteo.txt")
    fv = f.reshape(-1, 39)
    vv = v.reshape(-1, 39)
    with open(path, "w") as fh:
        for i in range(len(y)):
            fh.write("%d %s\n" % (int(y[i]), " ".join("%d:%.9g" % (a, b) for a, b in zip(fv[i], vv[i]))))
    return path


@pytest.mark.parametrize("fast", [False, True, "none"])
def test_lr_config3_batches_match_oracle(lib, oracle_mod, gpu, criteo_text, fast):
    """BASELINE config 3's per-GPU batch (65,537 rows, 39 features, keys
    < 2^24, AdaGrad lr 0.05) for 3 batches x 2 epochs against the oracle
    (lr.cpp:157-238,358-375): the batch shape where the 3-rows-per-wave
    forward and the long-run reduce (hot categorical keys: runs of tens of
    thousands of records) dominate.

    Exact mode (the reference's sequential fp32 chain): weights, AdaGrad sums
    and epoch errors within 1e-5 relative of the oracle.  fast_sums (fp64
    per-key sums): within 1e-5 of the oracle's fp64-sum variant (same
    definition, summation order aside); against the reference oracle every
    weight and AdaGrad sum within 1e-5 plus the reference's own fp32-chain
    rounding, measured as the distance between the two oracle modes (a hot
    key's mean of ~3e4 cancelling fp32 terms carries up to ~1e-4 relative
    rounding in the reference: 3e-6 absolute on a weight was seen)."""
    orc = oracle_mod.LR(criteo_text, 65536, 0.05)
    e_o = orc.train(2)
    ko, wo, go = orc.params()
    t = lib.Table("lr", capacity=1 << 22, dtype="f32", learning_rate=0.05)
    m = lib.LR(t, minibatch=65536, fast_sums=bool(fast), plan="none" if fast == "none" else "step")
    m.load_text(criteo_text)
    m.init()
    assert m.info()["batches"] >= 3
    e_g = m.train(2)
    kg, wg, gg = m.params()
    assert len(ko) > 100000 and np.array_equal(ko, kg)
    if not fast:
        assert np.allclose(wg, wo, rtol=1e-5, atol=1e-6), np.abs(wg - wo).max()
        assert np.allclose(gg, go, rtol=1e-5, atol=1e-7), np.abs(gg - go).max()
        assert np.allclose(e_g, e_o, rtol=1e-5)
        return
    o64 = oracle_mod.LR(criteo_text, 65536, 0.05, sum_f64=True)
    e_64 = o64.train(2)
    k64, w64, g64 = o64.params()
    assert np.array_equal(k64, kg)
    assert np.allclose(wg, w64, rtol=1e-5, atol=1e-6), np.abs(wg - w64).max()
    assert np.allclose(gg, g64, rtol=1e-5, atol=1e-7), np.abs(gg - g64).max()
    assert np.allclose(e_g, e_64, rtol=1e-5)
    for got, f64, ref, atol in ((wg, w64, wo, 1e-6), (gg, g64, go, 1e-7)):
        ref_round = np.abs(f64.astype(np.float64) - ref)  # the reference's own fp32-chain rounding
        assert (np.abs(got.astype(np.float64) - ref) <= ref_round + 1e-5 * np.abs(ref) + atol).all()
    assert np.allclose(e_g, e_o, rtol=1e-5)


@pytest.mark.parametrize("env,fast", [("SWPS_LR_FWD_RECORDS", False), ("SWPS_LR_FWD_RECORDS", True),
                                      ("SWPS_LR_INLINE", True)])
def test_lr_forward_records_bit_identical(lib, gpu, monkeypatch, env, fast):
    """Where the batch's gradient records e*x_i are formed — by k_lr_records
    after the forward (default), by the forward straight into their static
    key-sorted slots (SWPS_LR_FWD_RECORDS), or inside the fused fast-sums
    reduce (SWPS_LR_INLINE) — does not change a bit (Criteo shape: 3 rows per
    wave, hot long runs; ragged rows up to 60 features: 2 per wave)."""
    from swiftmpi_amd.synth import criteo
    y, off, f, v = criteo(20000, seed=7)
    rng = np.random.default_rng(4)
    lens = rng.integers(1, 61, 4000)
    roff = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    feat = rng.integers(0, 3000, int(roff[-1])).astype(np.uint32)
    vals = rng.random(int(roff[-1])).astype(np.float32)
    yl = (rng.random(4000) < 0.5).astype(np.float32)
    res = []
    monkeypatch.setenv("SWPS_LR_TILES", "0")  # the record path (fast sums default: row tiles)
    for on in ("0", "1"):
        monkeypatch.setenv(env, on)
        out = []
        for data, B in (((y, off, f, v), 4095), ((yl, roff, feat, vals), 700)):
            t = lib.Table("lr", capacity=1 << 18, dtype="f32", learning_rate=0.05, init="hash", seed=1)
            m = lib.LR(t, minibatch=B, init_ref=False, fast_sums=fast)
            m.load_csr(*data)
            m.init()
            out += [m.train(2), m.params()[1], m.params()[2]]
        res.append(out)
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("bits,chunk", [(None, None), ("6", None), ("4", None), (None, "512"), (None, "2048"),
                                        (None, "4096"), (None, "t512")])
def test_lr_tiles_match_record_path(lib, gpu, monkeypatch, bits, chunk):
    """Fast sums through row tiles (k_lr_tiles + k_lr_tiles_fin: e read from an LDS slice, a
    block-wide segmented scan over 1,024 records, one fp64 partial per piece = a key's records
    inside one block, a key's partials added in record order) against the record path
    (k_lr_records + k_lr_reduce_fused): the same fp32 products e*x_i, fp64 sums in another fixed
    order, so the means agree to fp64 rounding and the weights after 2 epochs within 1e-6 of
    their scale; run to run bit-identical.  Default tiles (4,096 rows: hot keys' runs cross
    block boundaries) and shrunken ones (64 / 16 rows: nearly every key in many pieces) on
    Criteo-shaped rows (hot keys) and ragged rows of 1-60 features."""
    from swiftmpi_amd.synth import criteo
    y, off, f, v = criteo(20000, seed=7)
    rng = np.random.default_rng(4)
    lens = rng.integers(1, 61, 4000)
    roff = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    feat = rng.integers(0, 3000, int(roff[-1])).astype(np.uint32)
    vals = rng.random(int(roff[-1])).astype(np.float32)
    yl = (rng.random(4000) < 0.5).astype(np.float32)
    if bits:
        monkeypatch.setenv("SWPS_LR_TILE_BITS", bits)
    if chunk == "t512":  # 512-thread blocks of 2,048 records
        monkeypatch.setenv("SWPS_LR_TILE_THREADS", "512")
    elif chunk:  # blocks of 512 / 2,048 / 4,096 records (2 / 8 / 16 per thread; default 1,024)
        monkeypatch.setenv("SWPS_LR_TILE_CHUNK", chunk)
    res = []
    for tiles in ("0", "1", "1"):
        monkeypatch.setenv("SWPS_LR_TILES", tiles)
        out = []
        for data, B in (((y, off, f, v), 4095), ((yl, roff, feat, vals), 700)):
            t = lib.Table("lr", capacity=1 << 18, dtype="f32", learning_rate=0.05, init="hash", seed=1)
            m = lib.LR(t, minibatch=B, init_ref=False, fast_sums=True)
            m.load_csr(*data)
            m.init()
            out += [m.train(2), m.params()[1], m.params()[2]]
        res.append(out)
    for a, b in zip(res[1], res[2]):
        assert np.array_equal(a, b)
    for a, b in zip(res[0], res[1]):
        a = np.asarray(a, dtype=np.float64)
        b = np.asarray(b, dtype=np.float64)
        assert np.abs(a - b).max() <= 1e-6 * np.abs(a).max(), (np.abs(a - b).max(), np.abs(a).max())


@pytest.mark.parametrize("fc", ["1", "0"])
def test_lr_hot_key_count_bit_identical(lib, gpu, monkeypatch, fc):
    """The forward's LDS copy of the batch's hottest keys' weights (SWPS_LR_NHOT = 1, 256, 512
    the default, 1024 the most: four loads per thread) == no LDS copy, bit for bit, in
    k_lr_forward_c and k_lr_forward_g: Criteo batches of 8,191 rows (over 1,024 keys with runs
    of >= 8 records), fast and exact sums."""
    from swiftmpi_amd.synth import criteo
    y, off, f, v = criteo(24000, seed=13)
    monkeypatch.setenv("SWPS_LR_FWD_C", fc)
    res = []
    for hot, nhot in (("0", "512"), ("1", "512"), ("1", "1"), ("1", "256"), ("1", "1024"), ("1", "700")):
        monkeypatch.setenv("SWPS_LR_HOT", hot)
        monkeypatch.setenv("SWPS_LR_NHOT", nhot)
        out = []
        for fast in (False, True):
            t = lib.Table("lr", capacity=1 << 20, dtype="f32", learning_rate=0.05, init="hash", seed=1)
            m = lib.LR(t, minibatch=8190, init_ref=False, fast_sums=fast)
            m.load_csr(y, off, f, v)
            m.init()
            out += [m.train(2), m.params()[1]]
            m.close()
            t.close()
        res.append(out)
    for r in res[1:]:
        for a, b in zip(res[0], r):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("groups,stage,hot", [("2", "0", "1"), ("4", "0", "1"), ("2", "1", "0"), ("2", "0", "0")])
def test_lr_forward_groups_bit_identical(lib, gpu, monkeypatch, groups, stage, hot):
    """k_lr_forward_g (2 / 4 groups of 3 rows per wave, every group's loads and gathers issued
    before the ordered sums; the batch's 256 hottest keys' weights from LDS, or the batch's
    weights staged densely by k_lr_stage, or the shard rows) == k_lr_forward_r<3> on the shard
    rows, bit for bit: Criteo-shaped rows (39 features), the reference's data.txt and ragged rows
    of 1-42 features, fast and exact sums."""
    monkeypatch.setenv("SWPS_LR_STAGE", stage)
    monkeypatch.setenv("SWPS_LR_HOT", hot)
    from swiftmpi_amd.synth import criteo
    y, off, f, v = criteo(9001, seed=5)
    rng = np.random.default_rng(6)
    lens = rng.integers(1, 43, 3001)
    roff = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    feat = rng.integers(0, 4000, int(roff[-1])).astype(np.uint32)
    vals = rng.random(int(roff[-1])).astype(np.float32)
    yl = (rng.random(3001) < 0.5).astype(np.float32)
    res = []
    for g in ("1", groups):
        monkeypatch.setenv("SWPS_LR_FWD_G", g)
        out = []
        for fast in (False, True):
            for data, B in (((y, off, f, v), 1000), ((yl, roff, feat, vals), 499)):
                t = lib.Table("lr", capacity=1 << 18, dtype="f32", learning_rate=0.05, init="hash", seed=1)
                m = lib.LR(t, minibatch=B, init_ref=False, fast_sums=fast)
                m.load_csr(*data)
                m.init()
                out += [m.train(2), m.params()[1]]
            t2 = lib.Table("lr", capacity=4096, dtype="f32", learning_rate=0.05)
            m2 = lib.LR(t2, minibatch=200, fast_sums=fast)
            m2.load_text(DATA)
            m2.init()
            out += [m2.train(2), m2.params()[1]]
        res.append(out)
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("env", [{}, {"SWPS_LR_TILE_BITS": "6"}, {"SWPS_LR_TILE_BITS": "4"},
                                 {"SWPS_LR_TILE_CHUNK": "512"}, {"SWPS_LR_TILE_CHUNK": "4096"},
                                 {"SWPS_LR_HOT": "0"}, {"SWPS_LR_NHOT": "1"}])
def test_lr_plan_step_equals_plan_load(lib, gpu, monkeypatch, env):
    """The per-step plan (each minibatch's key-sorted index, (tile, key) order, pieces, partial
    slots and hot keys built on the plan stream beside the previous step; lr.cpp:215-227) trains
    bit for bit like the index built once at load: errors, weights and AdaGrad sums after 2
    epochs, on Criteo-shaped rows (hot keys split across blocks) and ragged rows of 1-60
    features, with default, shrunken (64 / 16 rows) tiles, other block sizes and the hot-key LDS
    copy off or down to one key."""
    from swiftmpi_amd.synth import criteo
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    y, off, f, v = criteo(20000, seed=7)
    rng = np.random.default_rng(4)
    lens = rng.integers(1, 61, 4000)
    roff = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    feat = rng.integers(0, 3000, int(roff[-1])).astype(np.uint32)
    vals = rng.random(int(roff[-1])).astype(np.float32)
    yl = (rng.random(4000) < 0.5).astype(np.float32)
    res = []
    for plan in ("load", "step", "step"):
        out = []
        for data, B in (((y, off, f, v), 4095), ((yl, roff, feat, vals), 700)):
            t = lib.Table("lr", capacity=1 << 18, dtype="f32", learning_rate=0.05, init="hash", seed=1)
            m = lib.LR(t, minibatch=B, init_ref=False, fast_sums=True, plan=plan)
            m.load_csr(*data)
            m.init()
            out += [m.train(2), m.params()[1], m.params()[2]]
            m.close()
            t.close()
        res.append(out)
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b)
    for a, b in zip(res[1], res[2]):
        assert np.array_equal(a, b)


def test_lr_plan_step_config3_batch(lib, gpu):
    """At BASELINE config 3's per-GPU batch (65,537 Criteo-shaped rows over 2^24 keys, 3 batches,
    train_batches in uneven calls so plans are prefetched across calls): the per-step plan =
    the load-time index, bit for bit."""
    from swiftmpi_amd.synth import criteo
    y, off, f, v = criteo(3 * 65537, seed=3)
    res = []
    for plan in ("load", "step"):
        t = lib.Table("lr", capacity=1 << 22, dtype="f32", learning_rate=0.05, init="hash", seed=1)
        m = lib.LR(t, minibatch=65536, init_ref=False, fast_sums=True, plan=plan)
        m.load_csr(y, off, f, v)
        m.init()
        for n in (1, 3, 2):
            m.train_batches(n)
        m.sync()
        res.append(m.params())
        m.close()
        t.close()
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("hot", ["1", "0"])
def test_lr_fixed_point_step(lib, gpu, monkeypatch, hot):
    """The fixed-point step (plan="none": no index; each key's sum of e*x_i as a 64-bit integer
    at scale 2^s) is run-to-run bit-identical whatever order its adds land in, its bucketed form
    (k_lr_fxb_*: LDS sums per key bucket, hot keys' per-block partials) equals its per-record
    atomic form (SWPS_LR_FX_ATOMIC=1) and its form with gathered key codes instead of rows placed
    by fid (SWPS_LR_FX_AFFINE=0) bit for bit, and it is
    within 1e-6 of the sorted fp64 sums (plan="load") after 2 epochs, relative to the weights'
    scale, on Criteo-shaped rows (hot keys: LDS sums, one global add per block) and ragged rows of
    1-60 features; its per-batch errors equal the sorted path's for the first batch (same forward)."""
    from swiftmpi_amd.synth import criteo
    monkeypatch.setenv("SWPS_LR_HOT", hot)
    y, off, f, v = criteo(20000, seed=7)
    rng = np.random.default_rng(4)
    lens = rng.integers(1, 61, 4000)
    roff = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    feat = rng.integers(0, 3000, int(roff[-1])).astype(np.uint32)
    vals = rng.random(int(roff[-1])).astype(np.float32)
    yl = (rng.random(4000) < 0.5).astype(np.float32)
    res = []
    # variants (env over the default, the bucketed fixed-point step): the sorted fp64 sums (plan load);
    # run to run; the per-record atomic form; rows not placed by fid (gathered key codes); round 5's
    # per-chunk bucket segments (SWPS_LR_FXB_RES=0) with and without placement; one / two chunk
    # groups per bucket region; k_lr_fxb_step instead of the branch-free k_lr_fxr_step; the step's
    # weights from the rows instead of the dense copy by fid; the push prefetching no / every
    # bucket's rows; k_lr_fxr_step with 512 threads x 8 records
    base = dict(SWPS_LR_FX_ATOMIC="0", SWPS_LR_FX_AFFINE="1", SWPS_LR_FXB_RES="1", SWPS_LR_FXB_GBITS="3",
                SWPS_LR_FXR="1", SWPS_LR_FX_MIRROR="1", SWPS_LR_FX_PF="1", SWPS_LR_FX_NT="256")
    variants = [("load", {}), ("none", {}), ("none", {}), ("none", dict(SWPS_LR_FX_ATOMIC="1")),
                ("none", dict(SWPS_LR_FX_AFFINE="0")), ("none", dict(SWPS_LR_FXB_RES="0")),
                ("none", dict(SWPS_LR_FXB_RES="0", SWPS_LR_FX_AFFINE="0")), ("none", dict(SWPS_LR_FXB_GBITS="0")),
                ("none", dict(SWPS_LR_FXB_GBITS="1", SWPS_LR_FX_AFFINE="0")), ("none", dict(SWPS_LR_FXR="0")),
                ("none", dict(SWPS_LR_FX_MIRROR="0")), ("none", dict(SWPS_LR_FX_PF="0")),
                ("none", dict(SWPS_LR_FX_PF="2")), ("none", dict(SWPS_LR_FX_NT="512"))]
    for plan, env in variants:
        for k, val in dict(base, **env).items():
            monkeypatch.setenv(k, val)
        out = []
        for data, B in (((y, off, f, v), 4095), ((yl, roff, feat, vals), 700)):
            t = lib.Table("lr", capacity=1 << 18, dtype="f32", learning_rate=0.05, init="hash", seed=1)
            m = lib.LR(t, minibatch=B, init_ref=False, fast_sums=True, plan=plan)
            m.load_csr(*data)
            m.init()
            out += [m.train(2), m.params()[1], m.params()[2]]
            m.close()
            t.close()
        res.append(out)
    for a, *others in zip(*res[1:]):  # run to run; bucketed = atomic = gathered codes = segments
        for b in others:
            assert np.array_equal(a, b)
    for a, b in zip(res[0], res[1]):
        a = np.asarray(a, dtype=np.float64)
        b = np.asarray(b, dtype=np.float64)
        assert np.abs(a - b).max() <= 1e-6 * np.abs(a).max(), (np.abs(a - b).max(), np.abs(a).max())


def _libsvm_heavy_tailed(path, rows=4000, keys=3000, seed=12):
    """libsvm-style rows (lr.cpp:103-131's text format): 5-30 Zipf-drawn keys per row, values
    log-uniform over 1e-4 .. 1e6 (ten decades, as unscaled counts and amounts sit in real
    libsvm data), random labels."""
    rng = np.random.default_rng(seed)
    p = 1.0 / np.arange(1, keys + 1)
    p /= p.sum()
    with open(path, "w") as fh:
        for _ in range(rows):
            n = int(rng.integers(5, 31))
            fs = rng.choice(keys, n, p=p)
            vs = (10.0 ** rng.uniform(-4, 6, n)).astype(np.float32)
            fh.write("%d %s\n" % (int(rng.random() < 0.5), " ".join("%d:%.9g" % (a, b) for a, b in zip(fs, vs))))
    return path


def test_lr_heavy_tailed_values_fall_back_to_fp64_sums(lib, oracle_mod, gpu, tmp_path):
    """Verdict r05 item 4: the fixed-point step (plan none) sizes its scale 2^s so no sum can
    overflow (s = 62 - log2((max|y| + 1) * max|x_i| * batch records)); heavy-tailed x_i push s so
    low that small terms e * x_i would round away.  The load then switches to the fp64-sum path
    (plan step) and says so (swps_lr_plan_info), and training stays within 1e-5 of the oracle's
    fp64-sum variant after 2 epochs (weights, AdaGrad sums, epoch errors) — where forcing the fixed
    point on the same data (floor 0) does not."""
    path = _libsvm_heavy_tailed(str(tmp_path / "heavy.txt"))
    o64 = oracle_mod.LR(path, 999, 0.05, sum_f64=True)
    e_64 = o64.train(2)
    k64, w64, g64 = o64.params()
    t = lib.Table("lr", capacity=1 << 14, dtype="f32", learning_rate=0.05)
    m = lib.LR(t, minibatch=999, fast_sums=True, plan="none")
    m.load_text(path)
    pi = m.plan_info()
    assert pi["fallback"] and pi["plan"] == "step" and pi["plan_asked"] == "none", pi
    assert pi["fx_bits"] < pi["fx_floor"], pi
    m.init()
    e_g = m.train(2)
    kg, wg, gg = m.params()
    m.close()
    t.close()
    assert np.array_equal(k64, kg)
    assert np.allclose(wg, w64, rtol=1e-5, atol=1e-6), np.abs(wg - w64).max()
    assert np.allclose(gg, g64, rtol=1e-5, atol=1e-7), np.abs(gg - g64).max()
    assert np.allclose(e_g, e_64, rtol=1e-5)


def test_lr_criteo_keeps_the_fixed_point(lib, gpu):
    """The floor does not trip on the bench's Criteo shape (values in (0, 1]): plan none runs."""
    from swiftmpi_amd.synth import criteo
    y, off, f, v = criteo(20000, seed=7)
    t = lib.Table("lr", capacity=1 << 18, dtype="f32", learning_rate=0.05, init="hash", seed=1)
    m = lib.LR(t, minibatch=4095, init_ref=False, fast_sums=True, plan="none")
    m.load_csr(y, off, f, v)
    pi = m.plan_info()
    m.close()
    t.close()
    assert not pi["fallback"] and pi["plan"] == "none" and pi["fx_bits"] >= pi["fx_floor"], pi


@pytest.mark.parametrize("where", ["value_text", "value_csr", "label_csr"])
def test_lr_nonfinite_input_fails_loudly(lib, gpu, tmp_path, where):
    """A NaN / inf feature value or label is refused at load with SWPS_E_CFG naming where it is
    (the reference's parse_instance2 reads "nan" with %f and trains on it silently)."""
    t = lib.Table("lr", capacity=4096, dtype="f32", learning_rate=0.05)
    m = lib.LR(t, minibatch=10, fast_sums=True, plan="none")
    try:
        if where == "value_text":
            path = str(tmp_path / "nan.txt")
            with open(path, "w") as fh:
                fh.write("1 3:0.5 7:1\n0 3:nan 9:1\n1 2:1\n")
            with pytest.raises(lib.SwpsError) as ei:
                m.load_text(path)
            assert "record 2" in str(ei.value) and "row 1" in str(ei.value), str(ei.value)
        else:
            y = np.array([1, 0, 1], dtype=np.float32)
            off = np.array([0, 2, 4, 5], dtype=np.uint64)
            f = np.array([3, 7, 3, 9, 2], dtype=np.uint32)
            v = np.array([0.5, 1, 1, 1, 1], dtype=np.float32)
            if where == "value_csr":
                v[4] = np.inf
            else:
                y[2] = np.nan
            with pytest.raises(lib.SwpsError) as ei:
                m.load_csr(y, off, f, v)
            assert ei.value.code == -5, ei.value.code  # SWPS_E_CFG
            assert ("record 4" if where == "value_csr" else "label at row 2") in str(ei.value), str(ei.value)
    finally:
        m.close()
        t.close()


def test_lr_config3_full_rank_share(lib, gpu):
    """BASELINE config 3 at its full per-GPU share (45,840,617 Criteo-shaped rows / 8 GPUs =
    5.73M rows, 223M records, minibatches of 65,536 over a 2^24 hashed feature space): the
    fixed-point step (plan none) trains one epoch twice, bit-identical run to run, finite, every
    batch's examples counted."""
    from swiftmpi_amd.synth import criteo
    rows = 45_840_617 // 8
    y, off, f, v = criteo(rows, seed=3)
    outs = []
    for _ in range(2):
        t = lib.Table("lr", capacity=1 << 24, dtype="f32", learning_rate=0.05, init="hash", seed=1)
        m = lib.LR(t, minibatch=65536, init_ref=False, fast_sums=True, plan="none")
        m.load_csr(y, off, f, v)
        m.init()
        err = m.train(1)
        k, w, g2 = m.params()
        assert m.fx_bytes(0)["form"] == 1  # the bucketed fixed-point step ran
        assert m.info()["rows"] == rows and m.info()["batches"] == (rows + 65536) // 65537
        outs.append((err, w, g2, len(k)))
        m.close()
        t.close()
    assert outs[0][3] == outs[1][3] > 1_000_000
    for a, b in zip(outs[0][:3], outs[1][:3]):
        assert np.array_equal(a, b)
    assert np.isfinite(outs[0][1]).all() and np.isfinite(outs[0][0]).all()


@pytest.mark.parametrize("inplace", [1, 2, 0])
@pytest.mark.parametrize("B", [4095, 200])
def test_sharded_fixed_point_world1_equals_unsharded(lib, gpu, B, inplace, monkeypatch):
    """The sharded learner's fixed-point step (plan none, fast sums: swps_lr_step writes each
    key's mean of its integer sums as the push payload and the owner applies AdaGrad,
    k_lr_fxb_push<TO_GRADS>) through the library driver at world 1 (RCCL) == the single-GPU
    fixed-point step, bit for bit: weights, AdaGrad sums and epoch errors over 3 epochs, and the
    predictions after them.  inplace=1 (the default at world 1): the pull reads the shard rows and
    the push applies AdaGrad to them (no copy, payload or owner apply) — with the rows placed by
    fid, the single-GPU affine step itself; 2: in place through the install and a row-indexed push
    (SWPS_LR_W1_AFFINE=0); 0: the full protocol."""
    import torch
    monkeypatch.setenv("SWPS_PULL_IN_PLACE", str(min(inplace, 1)))
    monkeypatch.setenv("SWPS_LR_W1_AFFINE", "0" if inplace == 2 else "1")
    from conftest import free_port
    from swiftmpi_amd.comm import Comm
    from swiftmpi_amd.synth import criteo
    y, off, f, v = criteo(12 * B + 7, seed=21, bits=16)
    res = []
    for sharded in (False, True):
        t = lib.Table("lr", capacity=1 << 17, dtype="f32", learning_rate=0.05, init="hash", seed=4)
        m = lib.LR(t, minibatch=B, init_ref=False, fast_sums=True, plan="none")
        m.load_csr(y, off, f, v)
        comm = None
        if sharded:
            comm = Comm.rccl(0, 1, port=free_port())
            m.shard_comm(comm, frag_num=2000)
        m.init()
        e = m.train(3)
        p = m.predict()[0]  # sharded: a full pull refreshes the worker cache first
        k = np.sort(t.keys())
        rows = t.export(torch.as_tensor(k.astype(np.int64), device="cuda")).cpu().numpy()
        res.append((e, k, rows, p))
        m.close()
        t.close()
        if comm is not None:
            comm.close()
    assert np.array_equal(res[0][1], res[1][1])
    assert np.array_equal(res[0][2], res[1][2]), float(np.abs(res[0][2] - res[1][2]).max())
    assert np.array_equal(res[0][0], res[1][0]), (res[0][0], res[1][0])
    assert np.array_equal(res[0][3], res[1][3])
