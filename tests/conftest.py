import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libswps.so on cuda:0)")


def zipf_corpus(path, nlines, vocab, seed, lo=10, hi=30, s=1.0, extra_lines=()):
    """Write a Zipf(s) corpus of `nlines` lines of lo..hi words named w<id>."""
    rng = np.random.default_rng(seed)
    p = 1.0 / np.arange(1, vocab + 1) ** s
    p /= p.sum()
    with open(path, "w") as f:
        for _ in range(nlines):
            n = int(rng.integers(lo, hi + 1))
            f.write(" ".join("w%d" % x for x in rng.choice(vocab, n, p=p)) + "\n")
        for ln in extra_lines:
            f.write(ln + "\n")
    return path


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def lib():
    import swiftmpi_amd
    from swiftmpi_amd import build
    build.build()
    return swiftmpi_amd


@pytest.fixture(scope="session")
def gpu(lib):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
