"""The host iteration orders the reference's results depend on, against the
fixture recorded in the build container (tests/golden/make_order_fixture.py):
the word2vec vocabulary's vid order and counts, the unigram run starts, and
LR's first-pull (init) order.  CPU: the oracle on this box reproduces the
fixture.  GPU box: the library's own ingest does — so a C++ runtime that
iterates std::unordered_set differently fails here rather than passing
against a same-box oracle."""
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN

sys.path.insert(0, GOLDEN)
import make_order_fixture as mof  # noqa: E402

FIX = np.load(os.path.join(GOLDEN, "order_fixture.npz"))


def test_oracle_reproduces_order_fixture(oracle_mod, tmp_path):
    m = oracle_mod.W2V(mof.w2v_corpus(str(tmp_path / "c.txt")), 8, minibatch=100, table_size=int(1e8))
    k, c = m.vocab()
    assert np.array_equal(k, FIX["w2v_keys"]) and np.array_equal(c, FIX["w2v_counts"])
    assert np.array_equal(m.table_starts(), FIX["w2v_starts"])
    assert np.array_equal(oracle_mod.LR(os.path.join(GOLDEN, "lr_data.txt"), 200, 0.05).pull_order(),
                          FIX["lr_data_order"])
    assert np.array_equal(oracle_mod.LR(mof.lr_criteo_text(str(tmp_path / "lr.txt")), 255, 0.05).pull_order(),
                          FIX["lr_criteo_order"])


@pytest.mark.gpu
def test_library_ingest_matches_order_fixture(lib, gpu, tmp_path):
    t = lib.Table("w2v", dim=8, capacity=1 << 15, dtype="f32", learning_rate=0.7)
    w = lib.Word2Vec(t, minibatch=100)
    w.load_text(mof.w2v_corpus(str(tmp_path / "c.txt")))
    w.init()
    k, c = w.vocab()
    assert np.array_equal(k, FIX["w2v_keys"]) and np.array_equal(c, FIX["w2v_counts"])
    st = FIX["w2v_starts"].astype(np.int64)
    run = np.flatnonzero(st[1:] > st[:-1])
    assert len(run) > 1000
    assert np.array_equal(w.unigram_at(st[run].astype(np.uint64)), run.astype(np.uint32))
    assert np.array_equal(w.unigram_at((st[run + 1] - 1).astype(np.uint64)), run.astype(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["lr_data_order", "lr_criteo_order"])
def test_library_lr_init_order_matches_fixture(lib, gpu, tmp_path, which):
    """LR's init draws gen_float() per key in first-pull order (lr.cpp:48-50):
    each key's initial weight gives its position in that order."""
    from test_lr_gpu import _gen_float_draws
    path = (os.path.join(GOLDEN, "lr_data.txt") if which == "lr_data_order"
            else mof.lr_criteo_text(str(tmp_path / "lr.txt")))
    t = lib.Table("lr", capacity=1 << 16, dtype="f32", learning_rate=0.05)
    m = lib.LR(t, minibatch=200 if which == "lr_data_order" else 255)
    m.load_text(path)
    m.init()
    keys, w, _ = m.params()
    fix = FIX[which]
    assert np.array_equal(np.sort(fix), keys)
    # the key at position i of the fixture's order drew the i-th gen_float()
    expect = dict(zip(fix.tolist(), _gen_float_draws(len(fix)).tolist()))
    assert all(expect[int(k)] == float(x) for k, x in zip(keys, w))
