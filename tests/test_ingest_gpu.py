"""Corpus ingest on the GPU (tokenize, BKDR / atoi,
vocab counts and order, the minibatch key sets) against the host
restatement (swps_w2v_cfg.host_ingest = 1, itself pinned to the oracle by
tests/test_w2v_gpu.py's vocab / unigram / training tests): every output
bit-identical — vocab keys in `_local_keys` order, counts, train_words,
every token's vid and line, every batch's lines and key set, and the
trained rows."""
import numpy as np
import pytest

from conftest import zipf_corpus

pytestmark = pytest.mark.gpu


def both(lib, load, **kw):
    out = []
    for host in (True, False):
        t = lib.Table("w2v", dim=16, capacity=1 << 16, dtype="f64", learning_rate=0.7)
        w = lib.Word2Vec(t, unigram_size=10 ** 6, host_ingest=host, **kw)
        load(w)
        out.append((t, w))
    return out


def assert_same_ingest(a, b):
    ka, ca = a.vocab()
    kb, cb = b.vocab()
    assert np.array_equal(ka, kb) and np.array_equal(ca, cb)
    ia, ib = a.info(), b.info()
    assert ia == ib, (ia, ib)
    va, la = a.corpus()
    vb, lb = b.corpus()
    assert np.array_equal(va, vb) and np.array_equal(la, lb)
    for bi in range(ia["batches"]):
        x, y = a.batch_keys(bi), b.batch_keys(bi)
        assert x[0] == y[0] and x[1] == y[1] and np.array_equal(x[2], y[2]), bi


EDGE_TEXT = ("w1 w2  w3 w1\n"            # double space
             "\n"                         # empty line
             "  w2 w4\tx w1 \n"           # leading / trailing spaces, a tab inside a word
             "w5 w6\r w1 w2\n"            # '\r' is part of a word
             "\xe9t\xe9 w1 w3 w2 w7\n"    # UTF-8 bytes >= 0x80 (BKDR adds them as signed char)
             "w2\n"                        # shorter than min_sentence_length 2
             "w1 w2 w3 w4 w5 w6 w7 w8 w9 w10 w11\n"
             "w8 w9 w1")                  # no trailing newline


@pytest.mark.parametrize("mb,msl", [(1, 1), (2, 2), (3, 1), (100, 2)])
def test_edge_text_gpu_equals_host(lib, gpu, tmp_path, mb, msl):
    p = tmp_path / "c.txt"
    p.write_bytes(EDGE_TEXT.encode("latin-1"))
    (ta, a), (tb, b) = both(lib, lambda w: w.load_text(str(p)), minibatch=mb, min_sentence_length=msl, window=2,
                            negative=2, sample=-1)
    assert_same_ingest(a, b)


def test_atoi_text_gpu_equals_host(lib, gpu, tmp_path):
    p = tmp_path / "i.txt"
    rng = np.random.default_rng(4)
    lines = []
    for _ in range(60):
        toks = [str(int(x)) for x in rng.integers(1, 400, rng.integers(3, 20))]
        toks += ["-17", "+23", "0042", "2147483648", "12abc"]  # sign, leading zeros, int truncation, trailing junk
        rng.shuffle(toks)
        lines.append(" ".join(toks))
    p.write_text("\n".join(lines) + "\n")
    (ta, a), (tb, b) = both(lib, lambda w: w.load_text(str(p)), key_mode="atoi", minibatch=7, window=3, negative=3)
    assert_same_ingest(a, b)


def test_word_only_in_short_lines_fails_both_ways(lib, gpu, tmp_path):
    from swiftmpi_amd import capi
    p = tmp_path / "c.txt"
    p.write_text("a b c d e f\nzz\na b c d e f g\n")
    for host in (True, False):
        t = lib.Table("w2v", dim=8, capacity=100, dtype="f64")
        w = lib.Word2Vec(t, min_sentence_length=2, unigram_size=10 ** 5, host_ingest=host)
        with pytest.raises(capi.SwpsError) as e:
            w.load_text(str(p))
        assert e.value.code == -7


@pytest.mark.parametrize("mb", [1, 13, 500])
def test_tokens_gpu_equals_host_and_trains_identically(lib, gpu, tmp_path, mb):
    path = zipf_corpus(str(tmp_path / "c.txt"), 400, 700, seed=77, lo=3, hi=40,
                       extra_lines=["w0 w1", "w2", "", "w3 w0 w5 w1"])  # short / empty lines: not gathered
    kw = dict(minibatch=mb, window=3, negative=4, sample=1e-3, min_sentence_length=3)
    (ta, a), (tb, b) = both(lib, lambda w: w.load_text(path), **kw)
    assert_same_ingest(a, b)
    for w in (a, b):
        w.init()
        w.train(2)
    assert np.array_equal(a.get_params(), b.get_params())
    assert a.stats()["lstate"] == b.stats()["lstate"]


def test_bench_scale_tokens_gpu_equals_host(lib, gpu):
    """The bench corpus shape (17M tokens of Zipf over 254k ids, 1000-token
    lines) through load_tokens: the GPU ingest equals the host's (vocab,
    counts, token vids, every batch's key set) and is timed beside it."""
    import time
    from swiftmpi_amd.synth import zipf_tokens
    ids, off = zipf_tokens(17005207, 253854, 1000, seed=8)
    keys = np.array([lib.bkdr("w%d" % i) for i in range(253854)], dtype=np.uint64)
    res = []
    for host in (True, False):
        t = lib.Table("w2v", dim=16, capacity=260000, dtype="f32")
        w = lib.Word2Vec(t, minibatch=5000, sample=1e-5, host_ingest=host)
        t0 = time.perf_counter()
        w.load_tokens(ids, off, keys)
        res.append((w, time.perf_counter() - t0, t))
    (a, da, _), (b, db, _) = res
    print("ingest 17M tokens: host %.2f s, GPU %.2f s" % (da, db))
    assert_same_ingest(a, b)
