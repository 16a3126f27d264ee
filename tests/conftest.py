import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


_USED_PORTS = set()


def free_port():
    """A free TCP port P on 127.0.0.1 (P + 1 free too: the library bootstraps RCCL at
    MASTER_PORT + 1) not handed out before in this session nor adjacent to one, drawn
    below Linux's ephemeral range (32768-60999), where the kernel's own outgoing
    connections cannot take it between this probe and the bind that follows (a
    bind-to-0 probe hands out exactly such a port: EADDRINUSE on a busy box)."""
    import random
    import socket
    rng = random.Random()
    while True:
        p = rng.randrange(15000, 32000)
        if p in _USED_PORTS or p + 1 in _USED_PORTS or p - 1 in _USED_PORTS:
            continue
        socks = []
        try:
            for q in (p, p + 1):
                sk = socket.socket()
                socks.append(sk)
                sk.bind(("127.0.0.1", q))
        except OSError:
            continue
        finally:
            for sk in socks:
                sk.close()
        _USED_PORTS.add(p)
        return p


def init_gloo1():
    """A world-1 gloo process group rendezvousing through a fresh file (file://
    init): no port is probed or bound, so there is no probe-then-bind race."""
    import tempfile
    import torch.distributed as dist
    fd, path = tempfile.mkstemp(prefix="swps_gloo1_")
    os.close(fd)
    os.unlink(path)  # FileStore creates it; a stale file from an earlier group would be reused
    dist.init_process_group("gloo", init_method="file://" + path, rank=0, world_size=1)


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


def int_corpus(path, nlines, vocab, seed, lo=5, hi=25, s=1.0):
    """Zipf(s) corpus of integer tokens 1..vocab (word2vec.h's atoi keys;
    sent2vec / word2vec_local input)."""
    rng = np.random.default_rng(seed)
    p = 1.0 / np.arange(1, vocab + 1) ** s
    p /= p.sum()
    with open(path, "w") as f:
        for _ in range(nlines):
            n = int(rng.integers(lo, hi + 1))
            f.write(" ".join(str(x + 1) for x in rng.choice(vocab, n, p=p)) + "\n")
    return path


def word_dump(path, nwords, dim, seed, first=1):
    """A word2vec parameter dump in the reference's text format
    (sparsetable.h:63-70 + WParam operator<<: "key\\tv...\\th...") for keys
    first..first+nwords-1, values printed at ostream precision 6."""
    rng = np.random.default_rng(seed)
    with open(path, "w") as f:
        for k in rng.permutation(np.arange(first, first + nwords)):
            v = (rng.random(dim) - 0.5) / dim * 40
            h = (rng.random(dim) - 0.5) / dim * 40
            f.write("%d\t%s\t%s\n" % (k, " ".join("%g" % x for x in v), " ".join("%g" % x for x in h)))
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


@pytest.fixture
def gloo1():
    """A world-1 gloo process group for the sharded paths (torn down after
    the test if this fixture created it)."""
    import torch.distributed as dist
    own = not dist.is_initialized()
    if own:
        init_gloo1()
    yield dist
    if own:
        dist.destroy_process_group()
