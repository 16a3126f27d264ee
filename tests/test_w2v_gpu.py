"""word2vec CBOW-NS on the GPU (libswps.so) against the oracle, same inputs.

Bit-exact: vocab order and counts, unigram table, initial rows (glibc rand
emulation), negative draws, LCG / float-LCG end states, kept positions.
fp64 tables: updated rows within 1e-9 relative of the oracle (summation order
only).  fp32 tables: within 1e-5 relative of the oracle's fp32-storage mode
(the north star's fp32 single-batch tolerance), tested over whole epochs."""
import numpy as np
import pytest

from conftest import zipf_corpus

pytestmark = pytest.mark.gpu


def make(lib, oracle_mod, path, dtype, D=16, W=3, N=4, B=40, sample=1e-3, table=10 ** 6, min_len=1, key_mode=0,
         rand_offset=2, fp64_intermediates=True):
    orc = oracle_mod.W2V(path, D, window=W, negative=N, minibatch=B, sample=sample, table_size=table,
                         min_sentence_length=min_len, storage_f32=(dtype == "f32"), key_mode=key_mode)
    orc.init_rand(1, rand_offset)
    t = lib.Table("w2v", dim=D, capacity=orc.vocab_size + 16, dtype=dtype, learning_rate=0.7)
    w = lib.Word2Vec(t, window=W, negative=N, minibatch=B, sample=sample, unigram_size=table,
                     min_sentence_length=min_len, key_mode="atoi" if key_mode else "bkdr", init="ref",
                     rand_offset=rand_offset, fp64_intermediates=fp64_intermediates)
    w.load_text(path)
    w.init()
    return orc, t, w


def test_vocab_unigram_init_bitexact(lib, oracle_mod, gpu, tmp_path):
    path = zipf_corpus(str(tmp_path / "c.txt"), 301, 400, seed=3)
    orc, t, w = make(lib, oracle_mod, path, "f64", table=10 ** 8)
    k1, c1 = orc.vocab()
    k2, c2 = w.vocab()
    assert np.array_equal(k1, k2) and np.array_equal(c1, c2)
    assert w.info()["train_words"] == orc.train_words
    idx = np.random.default_rng(0).integers(0, 10 ** 8, 20000).astype(np.uint64)
    assert np.array_equal(w.unigram_at(idx), orc.table_at(idx))
    assert np.array_equal(w.get_params(), orc.get_params())


@pytest.mark.parametrize("sample,B,N,W", [(1e-3, 40, 4, 3), (-1.0, 25, 5, 5), (1e-2, 7, 2, 2), (1e-4, 1, 3, 4)])
def test_train_f64_matches_oracle(lib, oracle_mod, gpu, tmp_path, sample, B, N, W):
    path = zipf_corpus(str(tmp_path / "c.txt"), 203, 350, seed=11)
    orc, t, w = make(lib, oracle_mod, path, "f64", B=B, N=N, W=W, sample=sample)
    orc.trace_negatives(200000)
    w.trace_negatives(200000)
    orc.train(2)
    w.train(2)
    so, sg = orc.stats(), w.stats()
    assert sg["kept"] == so["kept"]
    assert sg["lstate"] == so["rng"] and sg["fstate"] == so["frng"]
    neg_o, neg_g = orc.negatives(200000), w.negatives(200000)
    assert len(neg_o) == len(neg_g) > 0 and np.array_equal(neg_o, neg_g)
    po, pg = orc.get_params(), w.get_params()
    assert np.allclose(pg, po, rtol=1e-9, atol=1e-12), np.abs(pg - po).max()


@pytest.mark.parametrize("combine", ["1", "0"])
def test_train_f64_matches_oracle_combine(lib, oracle_mod, gpu, tmp_path, monkeypatch, combine):
    """Hot runs' partials summed in groups by k_combine (forced on; the default
    only above 4M records per batch) or one by one in the push: both within the
    f64 tolerance of the oracle."""
    monkeypatch.setenv("SWPS_COMBINE", combine)
    path = zipf_corpus(str(tmp_path / "c.txt"), 203, 350, seed=11)
    orc, t, w = make(lib, oracle_mod, path, "f64", B=60, N=5, W=5, sample=-1.0)
    orc.train(2)
    w.train(2)
    po, pg = orc.get_params(), w.get_params()
    assert np.allclose(pg, po, rtol=1e-9, atol=1e-12), np.abs(pg - po).max()


def test_train_f32_matches_oracle_f32(lib, oracle_mod, gpu, tmp_path):
    path = zipf_corpus(str(tmp_path / "c.txt"), 251, 500, seed=13)
    orc, t, w = make(lib, oracle_mod, path, "f32", D=32, B=30, N=5, W=5, sample=1e-3)
    orc.train(2)
    w.train(2)
    po, pg = orc.get_params(), w.get_params()
    rel = np.abs(pg - po) / np.maximum(np.abs(po), 1e-3)
    assert rel.max() < 1e-5, rel.max()
    assert w.stats()["lstate"] == orc.stats()["rng"]


@pytest.mark.parametrize("fp64_intermediates", [True, False])
def test_single_batch_f32_vs_reference_f64(lib, oracle_mod, gpu, tmp_path, fp64_intermediates):
    """fp32 table after one deterministic minibatch vs the reference's fp64:
    rows within 1e-5 relative (the north star's fp32 tolerance), in the
    parity mode and in the fast mode the bench runs."""
    path = zipf_corpus(str(tmp_path / "c.txt"), 41, 300, seed=17)
    orc, _, _ = make(lib, oracle_mod, path, "f64", D=32, B=40, N=5, W=5, sample=1e-3)
    _, t, w = make(lib, oracle_mod, path, "f32", D=32, B=40, N=5, W=5, sample=1e-3,
                   fp64_intermediates=fp64_intermediates)
    orc.train(1)
    w.train(1)  # batch 0 = line 1 (dropped), batch 1 = lines 2..40, final push
    po, pg = orc.get_params(), w.get_params()
    rel = np.abs(pg - po) / np.maximum(np.abs(po), 1e-3)
    print("single batch fp32 (fp64 intermediates=%s) vs reference: frac<=1e-5 %.6f max %.3g"
          % (fp64_intermediates, np.mean(rel <= 1e-5), rel.max()))
    assert np.mean(rel <= 1e-5) > 0.999, np.mean(rel <= 1e-5)


def test_single_batch_bench_shape_f32_vs_f64(lib, gpu):
    """At bench shape (D=300, 1000-token lines, V=20k Zipf): one minibatch of
    the fp32 table (both modes) against the fp64 table from identical
    initial rows."""
    rng = np.random.default_rng(21)
    V, lines, L = 20000, 60, 1000
    p = 1.0 / np.arange(1, V + 1)
    ids = np.minimum(np.searchsorted(np.cumsum(p / p.sum()), rng.random(lines * L)), V - 1).astype(np.uint32)
    off = np.arange(0, lines * L + 1, L, dtype=np.uint64)
    keys = np.array([lib.bkdr("w%d" % i) for i in range(V)], dtype=np.uint64)
    outs = {}
    for name, dt, f64i in [("ref", "f64", True), ("parity", "f32", True), ("fast", "f32", False)]:
        t = lib.Table("w2v", dim=300, capacity=V, dtype=dt, learning_rate=0.7)
        w = lib.Word2Vec(t, window=5, negative=5, minibatch=59, sample=1e-5, init="ref", fp64_intermediates=f64i)
        w.load_tokens(ids, off, keys)
        w.init()
        w.train_batches(2)  # line-1 batch + one 59-line minibatch
        outs[name] = w.get_params()
    for name in ("parity", "fast"):
        rel = np.abs(outs[name] - outs["ref"]) / np.maximum(np.abs(outs["ref"]), 1e-3)
        print("%s: frac<=1e-5 %.6f max %.3g" % (name, np.mean(rel <= 1e-5), rel.max()))
        assert np.mean(rel <= 1e-5) > 0.999


def test_min_sentence_length_and_atoi(lib, oracle_mod, gpu, tmp_path):
    # short lines are trained but not gathered/counted (word2vec_global.h:617-618)
    rng = np.random.default_rng(2)
    path = str(tmp_path / "c.txt")
    with open(path, "w") as f:
        for i in range(150):
            n = int(rng.integers(2, 25))
            f.write(" ".join(str(x) for x in rng.integers(1, 120, n)) + "\n")
    orc, t, w = make(lib, oracle_mod, path, "f64", B=20, min_len=1, key_mode=1)
    orc.train(1)
    w.train(1)
    assert np.allclose(w.get_params(), orc.get_params(), rtol=1e-9, atol=1e-12)


def test_uneven_lines_and_empty_lines(lib, oracle_mod, gpu, tmp_path):
    path = zipf_corpus(str(tmp_path / "c.txt"), 120, 200, seed=23, lo=1, hi=60, extra_lines=["", "w1 w2", "", "w3"])
    orc, t, w = make(lib, oracle_mod, path, "f64", B=9, W=4, N=3)
    orc.train(3)
    w.train(3)
    assert w.stats()["lstate"] == orc.stats()["rng"]
    assert np.allclose(w.get_params(), orc.get_params(), rtol=1e-9, atol=1e-12)


def test_full_size_properties(lib, gpu):
    """At bench scale (no oracle): determinism run-to-run, finite rows, RNG
    bookkeeping consistent with the kept counts."""
    rng = np.random.default_rng(8)
    V, lines, L = 50000, 400, 1000
    p = 1.0 / np.arange(1, V + 1)
    p /= p.sum()
    ids = np.searchsorted(np.cumsum(p), rng.random(lines * L)).astype(np.uint32)
    ids = np.minimum(ids, V - 1)
    off = np.arange(0, lines * L + 1, L, dtype=np.uint64)
    keys = np.array([lib.bkdr("w%d" % i) for i in range(V)], dtype=np.uint64)
    outs = []
    for _ in range(2):
        t = lib.Table("w2v", dim=300, capacity=V, dtype="f32", learning_rate=0.7)
        w = lib.Word2Vec(t, window=5, negative=5, minibatch=100, sample=1e-5, init="ref")
        w.load_tokens(ids, off, keys)
        w.init()
        w.train(1)
        outs.append((w.get_params(), w.stats()))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.isfinite(outs[0][0]).all()
    st = outs[0][1]
    assert st["words"] == lines * L and 0 < st["kept"] < lines * L


def test_fast_mode_close_to_parity_mode(lib, oracle_mod, gpu, tmp_path):
    """fp32 intermediates (bench --fast) against fp64 intermediates: the mean
    gradients lose ~6e-8 * sum|terms|/|sum| to cancellation, so rows differ
    slightly more than fp32 storage alone; bounded here."""
    path = zipf_corpus(str(tmp_path / "c.txt"), 251, 500, seed=13)
    outs = []
    for fast in (False, True):
        t = lib.Table("w2v", dim=32, capacity=600, dtype="f32", learning_rate=0.7)
        w = lib.Word2Vec(t, window=5, negative=5, minibatch=30, sample=1e-3, unigram_size=10 ** 6,
                         fp64_intermediates=not fast)
        w.load_text(path)
        w.init()
        w.train(1)
        outs.append(w.get_params())
    rel = np.abs(outs[1] - outs[0]) / np.maximum(np.abs(outs[0]), 1e-3)
    print("fast-vs-parity rel: median %.3g p99 %.3g max %.3g" % (np.median(rel), np.quantile(rel, 0.99), rel.max()))
    assert np.median(rel) < 1e-5 and np.quantile(rel, 0.99) < 1e-2


@pytest.mark.parametrize("dtype,fp64i,overlap,D", [("f64", True, True, 16), ("f32", True, True, 16),
                                                  ("f32", False, True, 16), ("f32", False, False, 16),
                                                  ("f32", False, True, 300), ("f32", False, False, 300),
                                                  ("f32", "bfp40", True, 300), ("f32", "bfp40", True, 100)])
def test_sharded_world1_equals_unsharded(lib, gpu, tmp_path, dtype, fp64i, overlap, D):
    """The sharded request / serve / step / push path with one rank (gloo,
    world 1) reproduces the single-GPU path bit for bit — in fast mode too,
    where the push payload is fp32, and at D = 300, where the learner's mean
    gradients come from the fused k_push_thp<TO_GRADS> and the single GPU's
    update from the in-place k_push_thp."""
    import torch.distributed as dist
    from swiftmpi_amd.dist import ShardedWord2Vec
    path = zipf_corpus(str(tmp_path / "c.txt"), 120, 300, seed=31)
    kw = dict(window=3, negative=4, minibatch=13, sample=1e-3, unigram_size=10 ** 6, fp64_intermediates=fp64i)
    own = not dist.is_initialized()
    if own:
        from conftest import init_gloo1
        init_gloo1()
    try:
        t = lib.Table("w2v", dim=D, capacity=1000, dtype=dtype, learning_rate=0.7, init="hash", seed=3)
        sh = ShardedWord2Vec(t, overlap=overlap, **kw)
        sh.load_text(path)
        sh.init()
        sh.train(2)
        assert sh.stats()["lstate"] == w1_lstate(lib, path, dtype, kw)
        t1 = lib.Table("w2v", dim=D, capacity=1000, dtype=dtype, learning_rate=0.7, init="hash", seed=3)
        w1 = lib.Word2Vec(t1, init="table", **kw)
        w1.load_text(path)
        w1.init()
        w1.train(2)
        vk, _ = w1.vocab()
        keys, rows = sh.shard_rows()
        pos = {int(k): i for i, k in enumerate(keys)}
        got = np.stack([rows[pos[int(k)]] for k in vk])
        assert np.array_equal(got, w1.get_params())
    finally:
        if own:
            dist.destroy_process_group()


def w1_lstate(lib, path, dtype, kw):
    t = lib.Table("w2v", dim=16, capacity=1000, dtype=dtype, learning_rate=0.7, init="hash", seed=3)
    w = lib.Word2Vec(t, init="table", **kw)
    w.load_text(path)
    w.init()
    w.train(2)
    return w.stats()["lstate"]


def _sharded_run(lib, path, kw, pipeline, epochs=3, D=16, seed=3, lr=0.1):
    from swiftmpi_amd.dist import ShardedWord2Vec
    t = lib.Table("w2v", dim=D, capacity=4096, dtype="f32", learning_rate=lr, init="hash", seed=seed)
    sh = ShardedWord2Vec(t, pipeline=pipeline, **kw)
    sh.load_text(path)
    sh.init()
    for _ in range(epochs):  # uneven chunks: the prefetch makes results independent of chunking
        sh.train_steps(sh.steps_per_epoch // 2)
        sh.train_steps(sh.steps_per_epoch - sh.steps_per_epoch // 2)
    sh.sync()
    vk, cnt = sh.w.vocab()
    keys, rows = sh.shard_rows()
    pos = {int(k): i for i, k in enumerate(keys)}
    return (vk, cnt), np.stack([rows[pos[int(k)]] for k in vk]), t, sh


@pytest.mark.parametrize("fp64i", [True, False])
def test_pipelined_sharded_deterministic_and_close(lib, gpu, gloo1, tmp_path, fp64i):
    """The pipelined (bounded-staleness) sharded driver: bit-identical run to
    run, and its CBOW objective (swiftmpi_amd/evaluate.py) after 3 epochs
    within 2 % of the lockstep driver's, both clearly above the initial
    tables'."""
    from swiftmpi_amd.evaluate import cbow_objective, text_vid_lines
    path = zipf_corpus(str(tmp_path / "c.txt"), 3000, 300, seed=33)
    kw = dict(window=3, negative=4, minibatch=50, sample=1e-3, unigram_size=10 ** 6, fp64_intermediates=fp64i)
    (vk, cnt), p1, _, _ = _sharded_run(lib, path, kw, pipeline=True)
    _, p2, _, _ = _sharded_run(lib, path, kw, pipeline=True)
    assert np.array_equal(p1, p2)
    _, pl, _, _ = _sharded_run(lib, path, kw, pipeline=False)
    _, p0, _, _ = _sharded_run(lib, path, kw, pipeline=False, epochs=0)
    lines = text_vid_lines(path, vk, lib.bkdr)
    o1, ol, o0 = (cbow_objective(p, 16, lines, cnt, window=3, negatives=4) for p in (p1, pl, p0))
    print("objective: init %.4f lockstep %.4f pipelined %.4f" % (o0, ol, o1))
    assert not np.array_equal(p1, pl)
    assert abs(o1 - ol) <= 0.02 * abs(ol)
    assert ol > o0 + 0.1 and o1 > o0 + 0.1


# ---- word2vec.h's MiniBatch (w2v_local.cpp): per-minibatch vocab and table ----
def make_local(lib, oracle_mod, path, dtype, D=16, W=3, N=4, B=20, sample=1e-3, table=10 ** 6, min_len=1,
               fp64_intermediates=True):
    orc = oracle_mod.W2V(path, D, window=W, negative=N, minibatch=B, sample=sample, table_size=table,
                         min_sentence_length=min_len, storage_f32=(dtype == "f32"), key_mode=1,
                         minibatch_vocab=True)
    orc.init_rand(1, 2)
    t = lib.Table("w2v", dim=D, capacity=orc.vocab_size + 16, dtype=dtype, learning_rate=0.7)
    w = lib.Word2Vec(t, window=W, negative=N, minibatch=B, sample=sample, unigram_size=table,
                     min_sentence_length=min_len, key_mode="atoi", init="ref", rand_offset=2,
                     fp64_intermediates=fp64_intermediates, minibatch_vocab=True)
    w.load_text(path)
    w.init()
    return orc, t, w


@pytest.mark.parametrize("sample,B,N,W,extra", [(1e-3, 20, 4, 3, ()), (-1.0, 7, 5, 5, ()), (1e-2, 13, 2, 2, ("",) * 3),
                                                (1e-4, 1, 3, 4, ("1 2", "3"))])
def test_minibatch_vocab_f64_matches_oracle(lib, oracle_mod, gpu, tmp_path, sample, B, N, W, extra):
    """w2v_local.cpp semantics (word2vec.h MiniBatch): per-minibatch std::map
    vocab and unigram table, B+1-line gather/train windows, to_sample over the
    never-reset _num_words, a final short gather (< 5 keys) ending the epoch.
    Negative draws, kept positions, both RNG states bit-exact; fp64 rows
    within 1e-9."""
    from conftest import int_corpus
    path = int_corpus(str(tmp_path / "c.txt"), 160, 120, seed=41)
    with open(path, "a") as f:  # empty lines (trained, never gathered) and a short tail
        for ln in extra:
            f.write(ln + "\n")
    orc, t, w = make_local(lib, oracle_mod, path, "f64", W=W, N=N, B=B, sample=sample)
    orc.trace_negatives(100000)
    w.trace_negatives(100000)
    orc.train(3)
    w.train(3)
    so, sg = orc.stats(), w.stats()
    assert sg["lstate"] == so["rng"] and sg["fstate"] == so["frng"], (so, sg)
    assert sg["kept"] == so["kept"] and sg["words"] == 3 * so["actual_train_words"]  # oracle: last epoch
    assert np.array_equal(w.negatives(100000), orc.negatives(100000))
    po, pg = orc.get_params(), w.get_params()
    assert np.allclose(pg, po, rtol=1e-9, atol=1e-12), float(np.abs(pg - po).max())


def test_minibatch_vocab_f32_and_sharded(lib, oracle_mod, gpu, gloo1, tmp_path):
    """fp32 tables within 1e-5 of the oracle's fp32-storage mode; the sharded
    lockstep driver (world 1) equals the single-GPU run bit for bit."""
    from conftest import int_corpus
    from swiftmpi_amd.dist import ShardedWord2Vec
    path = int_corpus(str(tmp_path / "c.txt"), 200, 150, seed=42)
    orc, t, w = make_local(lib, oracle_mod, path, "f32", B=25)
    orc.train(2)
    w.train(2)
    po, pg = orc.get_params(), w.get_params()
    assert np.allclose(pg, po, rtol=1e-5, atol=1e-7), float(np.abs(pg - po).max())
    kw = dict(window=3, negative=4, minibatch=25, sample=1e-3, unigram_size=10 ** 6, key_mode="atoi",
              minibatch_vocab=True, fp64_intermediates=False)
    t1 = lib.Table("w2v", dim=16, capacity=1024, dtype="f32", learning_rate=0.7, init="hash", seed=2)
    w1 = lib.Word2Vec(t1, init="table", **kw)
    w1.load_text(path)
    w1.init()
    w1.train(2)
    t2 = lib.Table("w2v", dim=16, capacity=1024, dtype="f32", learning_rate=0.7, init="hash", seed=2)
    sh = ShardedWord2Vec(t2, **kw)
    sh.load_text(path)
    sh.init()
    sh.train(2)
    vk, _ = w1.vocab()
    keys, rows = sh.shard_rows()
    pos = {int(k): i for i, k in enumerate(keys)}
    assert np.array_equal(np.stack([rows[pos[int(k)]] for k in vk]), w1.get_params())


def test_alias_sampler_distribution(lib, gpu, tmp_path):
    """SWPS_SAMPLER_ALIAS draws negatives from count^0.75 / sum (the weights
    the reference's table discretises): empirical frequencies of the traced
    draws match within 5 sigma for every word, and the LCG stream advances
    exactly as with the table sampler (one draw per negative)."""
    path = zipf_corpus(str(tmp_path / "c.txt"), 300, 200, seed=51)
    kw = dict(window=3, negative=5, minibatch=40, sample=1e-3, unigram_size=10 ** 6)
    res = {}
    for sampler in ("table", "alias"):
        t = lib.Table("w2v", dim=16, capacity=512, dtype="f32", learning_rate=0.7)
        w = lib.Word2Vec(t, init="ref", sampler=sampler, **kw)
        w.load_text(path)
        w.init()
        w.trace_negatives(10 ** 7)
        w.train(20)
        res[sampler] = (w.negatives(10 ** 7), w.stats(), w.vocab()[1])
    (na, sa, cnt), (nt, st, _) = res["alias"], res["table"]
    assert sa["lstate"] == st["lstate"] and sa["kept"] == st["kept"]
    p = cnt.astype(np.float64) ** 0.75
    p /= p.sum()
    emp = np.bincount(na, minlength=len(cnt)) / len(na)
    sigma = np.sqrt(p * (1 - p) / len(na))
    assert len(na) > 100000
    assert (np.abs(emp - p) <= 5 * sigma + 1e-9).all(), float(np.max(np.abs(emp - p) / sigma))


@pytest.mark.parametrize("combine", ["1", "0"])
def test_fast_kernel_variants_bit_identical(lib, gpu, monkeypatch, combine):
    """k_push_t (compact-slice push) == k_push, k_push_tg (single-chunk runs
    summed inside the push, three variants) == k_gather_t + k_push_t, padded == D-strided neu1/neu1e
    rows, 128-B padded == D-strided worker-cache rows, and negatives from the
    coarse-indexed run-length unigram table == the
    1e8-slot table, bit for bit, at the bench's D = 300 (tail) shape in fast mode --
    with hot runs' partials pre-summed by k_combine (SWPS_COMBINE=1, the default
    for large batches) and read one by one by the push (0, small batches)."""
    monkeypatch.setenv("SWPS_COMBINE", combine)
    rng = np.random.default_rng(21)
    V, lines, L = 3000, 60, 400
    p = 1.0 / np.arange(1, V + 1)
    p /= p.sum()
    ids = np.minimum(np.searchsorted(np.cumsum(p), rng.random(lines * L)), V - 1).astype(np.uint32)
    off = np.arange(0, lines * L + 1, L, dtype=np.uint64)
    keys = np.array([lib.bkdr("w%d" % i) for i in range(V)], dtype=np.uint64)
    outs, negs = [], []
    variants = (("1", "1", "1", "1", "1", "0"), ("0", "1", "1", "1", "1", "0"), ("1", "0", "1", "1", "1", "0"),
                ("1", "1", "0", "1", "1", "0"), ("1", "1", "1", "0", "1", "0"), ("1", "1", "1", "1", "0", "0"),
                ("1", "1", "1", "1", "1", "1"), ("1", "1", "1", "1", "1", "2"), ("1", "1", "1", "1", "1", "3"), ("1", "1", "1", "1", "1", "4"), ("1", "1", "1", "1", "1", "5"),
                ("1", "1", "1", "1", "1", "sort"), ("1", "1", "1", "1", "1", "split"), ("1", "1", "1", "1", "1", "nosplit"),
                ("1", "1", "1", "1", "1", "nofull"))
    for push_t, pad, uidx, cpad, fused, tgv in variants:
        # "sort": the multi-chunk gather items in position order even for these small batches
        monkeypatch.setenv("SWPS_MULTI_SORT_MIN", "0" if tgv == "sort" else "65536")
        # split / nosplit: the multi-chunk gather beside the push on a side stream, or after it
        monkeypatch.setenv("SWPS_SPLIT_PUSH", {"split": "1", "nosplit": "0"}.get(tgv, "-1"))
        # nofull: neu1/neu1e and cache rows stored without their zero pad (partial last lines)
        monkeypatch.setenv("SWPS_FULL_LINES", "0" if tgv == "nofull" else "1")
        tgv = {"sort": "0", "split": "5", "nosplit": "5", "nofull": "5"}.get(tgv, tgv)
        monkeypatch.setenv("SWPS_PUSH_T", push_t)
        monkeypatch.setenv("SWPS_ROW_PAD", pad)
        monkeypatch.setenv("SWPS_UNI_INDEX", uidx)
        monkeypatch.setenv("SWPS_CACHE_PAD", cpad)
        monkeypatch.setenv("SWPS_FUSED_PUSH", fused)
        monkeypatch.setenv("SWPS_PUSH_TG", tgv)
        t = lib.Table("w2v", dim=300, capacity=V, dtype="f32", learning_rate=0.7)
        w = lib.Word2Vec(t, window=5, negative=5, minibatch=20, sample=1e-3, unigram_size=10 ** 8,
                         fp64_intermediates=False)
        w.load_tokens(ids, off, keys)
        w.init()
        w.trace_negatives(200000)
        w.train(1)
        outs.append(w.get_params())
        negs.append(w.negatives(200000))
    for k in range(1, len(variants)):
        assert np.array_equal(outs[0], outs[k]), k
        assert np.array_equal(negs[0], negs[k]), k
    assert len(negs[0]) > 1000


@pytest.mark.parametrize("dtype,fp64i", [("f32", False), ("f32", True), ("f64", True), ("f32", "bfp40")])
def test_overlapped_driver_bit_identical(lib, gpu, monkeypatch, dtype, fp64i):
    """prep(i+1) on a second stream into a second buffer set while learn(i)
    runs (SWPS_OVERLAP=1; =2: issued after learn(i), beside its gather and push) == the
    sequential loop, bit for bit,
    across epoch boundaries and uneven train_batches chunks; RNG states and
    counters equal too."""
    rng = np.random.default_rng(5)
    V, lines, L = 2000, 90, 300
    p = 1.0 / np.arange(1, V + 1)
    p /= p.sum()
    ids = np.minimum(np.searchsorted(np.cumsum(p), rng.random(lines * L)), V - 1).astype(np.uint32)
    off = np.arange(0, lines * L + 1, L, dtype=np.uint64)
    keys = np.array([lib.bkdr("w%d" % i) for i in range(V)], dtype=np.uint64)
    res = []
    for ov in ("0", "1", "2"):  # 2: prep(i+1) issued after learn(i), waiting for its forward
        monkeypatch.setenv("SWPS_OVERLAP", ov)
        t = lib.Table("w2v", dim=64 if dtype == "f64" else 300, capacity=V, dtype=dtype, learning_rate=0.7)
        w = lib.Word2Vec(t, window=5, negative=5, minibatch=20, sample=1e-3, unigram_size=10 ** 6,
                         fp64_intermediates=fp64i)
        w.load_tokens(ids, off, keys)
        w.init()
        nb = w.info()["batches"]
        for chunk in (1, 3, nb, 2 * nb + 1, 2):
            w.train_batches(chunk)
        w.sync()
        st = w.stats()
        res.append((w.get_params(), {k: st[k] for k in ("batches", "kept", "words", "lstate", "fstate",
                                                        "pulled", "pushed")}))
    for r in res[1:]:
        assert res[0][1] == r[1]
        assert np.array_equal(res[0][0], r[0])


def test_specialised_records_kernel_bit_identical(lib, gpu, tmp_path, monkeypatch):
    """k_records_t<5, 5> (the W = 5, N = 5 table-sampler path: independent
    loads batched, per-bit LCG jump constants) writes exactly what the
    generic k_records writes: same negatives, same trained rows."""
    path = zipf_corpus(str(tmp_path / "c.txt"), 150, 400, seed=23)
    outs = []
    for generic in ("1", "0"):
        monkeypatch.setenv("SWPS_REC_GENERIC", generic)
        t = lib.Table("w2v", dim=16, capacity=1000, dtype="f64", learning_rate=0.7)
        w = lib.Word2Vec(t, window=5, negative=5, minibatch=17, sample=1e-3, unigram_size=10 ** 6)
        w.load_text(path)
        w.init()
        w.trace_negatives(100000)
        w.train(2)
        outs.append((w.negatives(100000), w.get_params(), w.stats()["lstate"]))
    assert np.array_equal(outs[0][0], outs[1][0]) and len(outs[0][0]) > 0
    assert np.array_equal(outs[0][1], outs[1][1]) and outs[0][2] == outs[1][2]
