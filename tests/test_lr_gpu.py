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
