"""The oracle (CPU restatement) against the reference's own outputs."""
import json
import os

import numpy as np

from conftest import GOLDEN, zipf_corpus


def test_lcg_matches_reference_random_h(oracle_mod):
    g = json.load(open(os.path.join(GOLDEN, "lcg_seed2008.json")))
    n = g["n"]
    lcg = oracle_mod.lcg_sequence(n, 2008)
    assert [str(x) for x in lcg] == g["lcg"]
    _, f = oracle_mod.float_lcg_sequence(n)
    assert f.view(np.uint32).tolist() == g["gen_float_bits"]


def test_lr_matches_reference_binary_quality(oracle_mod):
    """Pinned against the reference binary's own outputs."""
    q = json.load(open(os.path.join(GOLDEN, "lr_reference_quality.json")))
    data = os.path.join(GOLDEN, "lr_data.txt")
    for ep, exp in q["epochs"].items():
        m = oracle_mod.LR(data, q["minibatch"], q["lr"])
        m.train(int(ep))
        p, t = m.predict()
        # the reference predicts from its text dump (6 significant digits)
        p6 = np.array([float("%g" % x) for x in p], dtype=np.float32)
        ll, acc = oracle_mod.logloss_accuracy(p6, t)
        assert round(ll, 4) == exp["logloss"], (ep, ll)
        assert round(acc, 3) == exp["accuracy"], (ep, acc)


def test_lr_dataset_shape(oracle_mod):
    m = oracle_mod.LR(os.path.join(GOLDEN, "lr_data.txt"), 200, 0.05)
    m.train(1)
    keys, w, g2 = m.params()
    assert len(keys) == 113 and keys.max() == 119
    assert int(oracle_mod.lib().orc_lr_num_instances(m.h)) == 1605


def test_bkdr_signed_char_and_known_answers(oracle_mod):
    # h = h*13131 + (signed char)c (utils/string.h:130-137)
    def ref(b):
        h = 0
        for c in b:
            h = (h * 13131 + (c - 256 if c >= 128 else c)) % (1 << 64)
        return h
    for w in ["a", "b", "superjom", "而且", "2014年2月11日 ... 而且经过这么多年发展", "w12345"]:
        assert oracle_mod.bkdr(w) == ref(w.encode("utf-8"))
    assert oracle_mod.bkdr("a") == 97


def test_fmix64_and_hashfrag(oracle_mod):
    assert oracle_mod.fmix64(0) == 0
    t = oracle_mod.hashfrag_table(1000, 3)
    # int(1000/3) = 333 frags per node, the last node takes the remainder
    assert (t[:333] == 1).all() and (t[333:666] == 2).all() and (t[666:] == 3).all()
    t8 = oracle_mod.hashfrag_table(2000, 8)
    assert np.bincount(t8)[1:].tolist() == [250] * 8


def test_exptable(oracle_mod):
    e = oracle_mod.exptable()
    x = (np.arange(1000, dtype=np.float32) / np.float32(1000) * 2 - 1) * 6
    ed = np.exp(x.astype(np.float64)).astype(np.float32)
    assert np.array_equal(e, ed / (ed + np.float32(1)))


def test_unigram_table_run_length(oracle_mod, tmp_path):
    path = zipf_corpus(str(tmp_path / "c.txt"), 120, 300, seed=5)
    m = oracle_mod.W2V(path, 8, minibatch=20, table_size=10 ** 7)
    keys, counts = m.vocab()
    st = m.table_starts()
    assert st[0] == 0 and st[-1] == 10 ** 7 and (np.diff(st.astype(np.int64)) >= 1).all()
    # each run's share tracks count^0.75
    share = np.diff(st.astype(np.float64)) / 1e7
    w = counts.astype(np.float64) ** 0.75
    assert np.allclose(share, w / w.sum(), atol=2e-7)


def test_w2v_oracle_determinism(oracle_mod, tmp_path):
    path = zipf_corpus(str(tmp_path / "c.txt"), 90, 200, seed=7)
    outs = []
    for _ in range(2):
        m = oracle_mod.W2V(path, 8, window=3, negative=3, minibatch=20, sample=1e-3, table_size=10 ** 6)
        m.init_rand()
        m.train(2)
        outs.append((m.get_params(), m.stats()))
    assert np.array_equal(outs[0][0], outs[1][0]) and outs[0][1] == outs[1][1]
    st = outs[0][1]
    assert st["pushes"] > 0 and st["kept"] > 0


def test_oracle_lr_predict_mode(oracle_mod):
    """The oracle's lr.cpp predict mode (per-minibatch pulls) over a full dump of trained weights
    predicts exactly what orc_lr_predict does with those weights; over an empty dump every weight
    is a gen_float() draw, the first in the first minibatch's key-set order."""
    import os
    from conftest import GOLDEN
    data = os.path.join(GOLDEN, "lr_data.txt")
    a = oracle_mod.LR(data, 200, 0.05)
    a.train(2)
    k, w, _ = a.params()
    p_a, _ = a.predict()
    b = oracle_mod.LR(data, 200, 0.05)
    b.load(k, w)
    assert np.array_equal(b.predict_mode(), p_a)
    c = oracle_mod.LR(data, 200, 0.05)
    p = c.predict_mode()
    assert np.isfinite(p).all() and len(p) == len(p_a)
