"""sent2vec on the GPU (libswps.so) against the oracle, same inputs
(apps/sent2vec/sent2vec.cpp on word2vec.h's MiniBatch, nthreads = 1).

Bit-exact: sentence ids, the LCG end state, the number of rand() calls, the
rows of keys the minibatch pulls insert.  fp64 word table: sentence vectors
within 1e-9 relative of the oracle (summation order of the dot products
only).  fp32 word table: within 1e-5 relative of the oracle's fp32-storage
mode."""
import numpy as np
import pytest

from conftest import int_corpus, word_dump

pytestmark = pytest.mark.gpu


def run_pair(lib, oracle_mod, tmp_path, dtype="f64", D=16, W=3, N=4, B=20, niters=2, min_len=1, extra=0,
             vocab=150, dump_vocab=120, nlines=130, table=10 ** 6, seed=5, lo=5, hi=25):
    corpus = int_corpus(str(tmp_path / "c.txt"), nlines, vocab, seed=seed, lo=lo, hi=hi)
    dump = word_dump(str(tmp_path / "w.txt"), dump_vocab, D, seed=seed + 1)
    orc = oracle_mod.S2V(corpus, D, window=W, negative=N, minibatch=B, niters=niters, min_sentence_length=min_len,
                         table_size=table, storage_f32=(dtype == "f32"), rand_offset=2, rand_insert_extra=extra)
    orc.load_words(dump)
    orc.train()
    t = lib.Table("w2v", dim=D, capacity=vocab + 64, dtype=dtype)
    s = lib.Sent2Vec(t, window=W, negative=N, minibatch=B, niters=niters, min_sentence_length=min_len,
                     unigram_size=table, rand_offset=2, rand_insert_extra=extra)
    s.load_word_vector(dump)
    s.load_text(corpus)
    s.train()
    return orc, t, s


@pytest.mark.parametrize("W,N,B,niters,extra", [(3, 4, 20, 2, 0), (5, 5, 7, 1, 32), (2, 3, 45, 3, 0),
                                                (4, 2, 1, 1, 0)])
def test_s2v_f64_matches_oracle(lib, oracle_mod, gpu, tmp_path, W, N, B, niters, extra):
    orc, t, s = run_pair(lib, oracle_mod, tmp_path, W=W, N=N, B=B, niters=niters, extra=extra)
    io, vo, eo = orc.docs()
    ig, vg, eg = s.docs()
    so, info = orc.stats(), s.info()
    assert len(io) == len(ig) > 0 and np.array_equal(io, ig)
    assert info["batches"] == so["batches"] and info["inserted"] == so["inserted"]
    assert info["lstate"] == so["rng"] and info["rand_calls"] == so["rand_calls"]
    assert np.allclose(vg, vo, rtol=1e-9, atol=1e-12), np.abs(vg - vo).max()
    assert np.allclose(eg, eo, rtol=1e-5, atol=1e-9)
    assert abs(s.error() - so["error_sum"] / len(io)) <= 1e-6 * max(1.0, abs(s.error()))
    # keys the pulls inserted carry the oracle's rand() rows
    keys = t.keys()
    import torch
    rows = t.export(torch.as_tensor(keys.astype(np.int64), device="cuda")).double().cpu().numpy()
    ref, ok = orc.word_rows(keys)
    assert ok
    assert np.array_equal(rows[:, :2 * t.dim], ref)


def test_s2v_f32_matches_oracle_f32(lib, oracle_mod, gpu, tmp_path):
    orc, t, s = run_pair(lib, oracle_mod, tmp_path, dtype="f32", D=32, W=5, N=5, B=15, niters=2)
    _, vo, _ = orc.docs()
    _, vg, _ = s.docs()
    rel = np.abs(vg - vo) / np.maximum(np.abs(vo), 1e-3)
    assert rel.max() < 1e-5, rel.max()


def test_s2v_short_lines_and_tail(lib, oracle_mod, gpu, tmp_path):
    """min_sentence_length > 1: short lines are read (they count toward the
    B+1 lines of a minibatch) but neither gathered nor trained; the run stops
    at the first minibatch with fewer than 5 keys (sent2vec.cpp:97)."""
    orc, t, s = run_pair(lib, oracle_mod, tmp_path, B=9, min_len=8, lo=1, hi=20, nlines=90, extra=32)
    io, vo, _ = orc.docs()
    ig, vg, _ = s.docs()
    assert np.array_equal(io, ig)
    assert np.allclose(vg, vo, rtol=1e-9, atol=1e-12)
    assert s.info()["lstate"] == orc.stats()["rng"]


def test_s2v_dump_format(lib, oracle_mod, gpu, tmp_path):
    orc, t, s = run_pair(lib, oracle_mod, tmp_path, B=30, niters=1)
    out = str(tmp_path / "sent.txt")
    s.dump(out)
    ids, vecs, _ = s.docs()
    lines = open(out).read().split("\n")
    assert lines[-1] == "" and len(lines) == len(ids) + 1
    for i in (0, len(ids) // 2, len(ids) - 1):  # Vec::operator<< (vec1.h:112-118)
        exp = "%d\tVec:\t" % ids[i] + "".join("%g " % x for x in vecs[i])
        assert lines[i] == exp


def test_s2v_rejects_key_zero(lib, gpu, tmp_path):
    """atoi of a non-numeric word is key 0; the reference redraws negatives
    that hit it (a data-dependent draw count): refused, not silently wrong."""
    p = tmp_path / "c.txt"
    p.write_text("1 2 3 4 5 6 x\n" * 10)
    dump = word_dump(str(tmp_path / "w.txt"), 10, 8, seed=1)
    t = lib.Table("w2v", dim=8, capacity=64, dtype="f64")
    s = lib.Sent2Vec(t, window=2, negative=2, minibatch=3, unigram_size=10 ** 5)
    s.load_word_vector(dump)
    with pytest.raises(lib.SwpsError, match="key 0"):
        s.load_text(str(p))


def test_s2v_bench_shape_properties(lib, gpu):
    """D=300, 10k sentences of 50-200 tokens (BASELINE config 5's shape at
    1/1000 scale): run-to-run bit-identical, finite, every position counted."""
    rng = np.random.default_rng(5)
    V, nd = 20000, 10000
    p = 1.0 / np.arange(1, V + 1)
    cdf = np.cumsum(p / p.sum())
    lens = rng.integers(50, 201, nd)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    toks = (np.minimum(np.searchsorted(cdf, rng.random(int(off[-1]))), V - 1) + 1).astype(np.uint64)
    ids = np.arange(1, nd + 1, dtype=np.uint64) * 2654435761
    outs = []
    for _ in range(2):
        t = lib.Table("w2v", dim=300, capacity=V + 16, dtype="f32", init="hash", seed=3)
        import torch
        keys = torch.arange(1, V + 1, dtype=torch.int64, device="cuda")
        t.pull(keys)  # the word table: hash-initialised rows for every word
        s = lib.Sent2Vec(t, window=5, negative=5, minibatch=4096, niters=1)
        s.load_tokens(toks, off, ids)
        s.train()
        outs.append((s.docs()[1], s.stats()))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.isfinite(outs[0][0]).all()
    st = outs[0][1]
    assert st["docs"] == nd and st["positions"] == int(off[-1])
    assert st["tgt_rows"] >= st["positions"]  # the positive target is never skipped


def test_s2v_doc_sharding_partitions_docs(lib, gpu, tmp_path):
    """Config 5's layout: with swps_s2v_shard every rank keeps exactly the
    sentences whose id BasicHashFrag maps to it — the ranks' outputs partition
    the corpus, and world 1 is the unsharded run bit for bit."""
    corpus = int_corpus(str(tmp_path / "c.txt"), 300, 150, seed=8)
    dump = word_dump(str(tmp_path / "w.txt"), 150, 16, seed=9)

    def run(rank, world):
        t = lib.Table("w2v", dim=16, capacity=256, dtype="f64")
        s = lib.Sent2Vec(t, window=3, negative=4, minibatch=20, niters=1, unigram_size=10 ** 6)
        s.load_word_vector(dump)
        if world:
            s.shard(rank, world, 1000)
        s.load_text(corpus)
        s.train()
        return s.docs()

    ids0, v0, _ = run(0, 0)
    ids1, v1, _ = run(0, 1)
    assert np.array_equal(ids0, ids1) and np.array_equal(v0, v1)
    world = 3
    fm = lib.hashfrag_table(1000, world)
    seen = []
    for r in range(world):
        ids, vecs, _ = run(r, world)
        assert len(ids) > 0 and np.isfinite(vecs).all()
        assert (lib.to_node_id(ids, 1000, fm) - 1 == r).all()
        seen.append(ids)
    allids = np.concatenate(seen)
    assert len(np.unique(allids)) == len(allids) == len(ids0)
    assert set(allids.tolist()) == set(ids0.tolist())


@pytest.mark.parametrize("dtype,D", [("f64", 300), ("f32", 300), ("f64", 100), ("f32", 100)])
def test_s2v_bench_dim_matches_oracle(lib, oracle_mod, gpu, tmp_path, dtype, D):
    """The benchmarked dimension (config 5: D = 300, W = N = 5, docs of 50-200
    tokens) against the oracle, the dump covering every word of the docs
    (sent2vec.cpp:119-179: neu1 = sent_vec + sum of context v, sent_vec +=
    alpha * neu1e).  D = 300 instantiates the scalar-tail docs kernels
    (k_s2v_docs<float, 1, true> fp32, <double, 2, true> fp64) that D = 16 / 32
    never reach; D = 100 the partial-chunk ones.  fp64 within 1e-9, fp32 within
    1e-5 of the oracle's fp32-storage mode (full array)."""
    orc, t, s = run_pair(lib, oracle_mod, tmp_path, dtype=dtype, D=D, W=5, N=5, B=40, niters=2, vocab=1500,
                         dump_vocab=1500, nlines=160, lo=50, hi=200, seed=11)
    io, vo, _ = orc.docs()
    ig, vg, _ = s.docs()
    assert len(io) == len(ig) > 100 and np.array_equal(io, ig)
    info, so = s.info(), orc.stats()
    assert info["lstate"] == so["rng"] and info["rand_calls"] == so["rand_calls"]
    if dtype == "f64":
        assert np.allclose(vg, vo, rtol=1e-9, atol=1e-12), np.abs(vg - vo).max()
    else:
        rel = np.abs(vg - vo) / np.maximum(np.abs(vo), 1e-3)
        assert rel.max() < 1e-5, rel.max()


def _tokens_of(lib, path):
    """(tok_keys, line_off, sent_ids) of a text corpus as the loaders parse it: split(" "), atoi
    keys (word2vec.h:206,212-224), sentence id = BKDR of the line (sent2vec.cpp:75)."""
    toks, off, ids = [], [0], []
    with open(path) as f:
        for line in f:
            line = line.rstrip("\n")
            ids.append(lib.bkdr(line))
            toks += [int(w) for w in line.split(" ") if w]
            off.append(len(toks))
    return (np.array(toks, dtype=np.uint64), np.array(off, dtype=np.uint64), np.array(ids, dtype=np.uint64))


@pytest.mark.parametrize("B,min_len,lo,hi,extra,nlines", [(20, 1, 5, 25, 0, 130), (9, 8, 1, 20, 32, 90),
                                                          (7, 1, 5, 25, 0, 300), (1, 1, 5, 25, 0, 40)])
def test_s2v_single_pass_equals_load_then_train(lib, oracle_mod, gpu, tmp_path, B, min_len, lo, hi, extra, nlines):
    """The reference's single pass (swps_s2v_run_tokens: each minibatch group planned on host threads
    while the GPU trains the groups before it) = load_tokens + train, bit for bit: sentence ids and
    vectors, errors, the rows the pulls inserted, the rand() call count and the LCG end state — with
    misses (keys the loaded word dump lacks), short lines and the tail stop; and = the oracle."""
    import torch
    D = 16
    corpus = int_corpus(str(tmp_path / "c.txt"), nlines, 150, seed=5, lo=lo, hi=hi)
    dump = word_dump(str(tmp_path / "w.txt"), 120, D, seed=6)
    toks, off, ids = _tokens_of(lib, corpus)
    res = []
    for single in (False, True):
        t = lib.Table("w2v", dim=D, capacity=214, dtype="f64")
        s = lib.Sent2Vec(t, window=3, negative=4, minibatch=B, niters=2, min_sentence_length=min_len,
                         unigram_size=10 ** 6, rand_offset=2, rand_insert_extra=extra)
        s.load_word_vector(dump)
        if single:
            s.run_tokens(toks, off, ids)
        else:
            s.load_tokens(toks, off, ids)
            s.train()
        keys = np.sort(t.keys())
        res.append((s.docs(), s.info(), s.stats(), keys,
                    t.export(torch.as_tensor(keys.astype(np.int64), device="cuda")).cpu().numpy()))
        del s
        t.close()
    (da, ia, sa, ka, ra), (db, ib, sb, kb, rb) = res
    for x, y in zip(da, db):
        assert np.array_equal(x, y)
    assert ia == ib and sa == sb, (ia, ib, sa, sb)
    assert np.array_equal(ka, kb) and np.array_equal(ra, rb)
    orc = oracle_mod.S2V(corpus, D, window=3, negative=4, minibatch=B, niters=2, min_sentence_length=min_len,
                         table_size=10 ** 6, rand_offset=2, rand_insert_extra=extra)
    orc.load_words(dump)
    orc.train()
    io, vo, _ = orc.docs()
    assert len(io) > 0 and np.array_equal(io, db[0])
    assert ib["lstate"] == orc.stats()["rng"] and ib["rand_calls"] == orc.stats()["rand_calls"]
    assert np.allclose(db[1], vo, rtol=1e-9, atol=1e-12), np.abs(db[1] - vo).max()


def _zipf_docs(rng, V, nd, lo=50, hi=200):
    p = 1.0 / np.arange(1, V + 1)
    cdf = np.cumsum(p / p.sum())
    lens = rng.integers(lo, hi + 1, nd)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    toks = (np.minimum(np.searchsorted(cdf, rng.random(int(off[-1]))), V - 1) + 1).astype(np.uint64)
    return toks, off


def test_s2v_config5_shape(lib, oracle_mod, gpu, tmp_path):
    """BASELINE config 5's per-rank shape: a hash-initialised 1M x 300 fp32
    word table (every word pulled once: the frozen word table), 60k docs of
    50-200 Zipf(1M) tokens in minibatches of 4096 — run to run bit-identical,
    finite, every position counted — and an oracle-sized slice of the same
    docs (the first 120) trained on the same word rows (a full-precision dump
    of the words they use, loaded by both) within 1e-5 of the oracle."""
    import torch
    rng = np.random.default_rng(5)
    V, nd, D = 1_000_000, 60_000, 300
    toks, off = _zipf_docs(rng, V, nd)
    ids = np.arange(1, nd + 1, dtype=np.uint64) * 2654435761
    t = lib.Table("w2v", dim=D, capacity=V + 16, dtype="f32", init="hash", seed=3)
    keys = torch.arange(1, V + 1, dtype=torch.int64, device="cuda")
    for k0 in range(0, V, 1 << 18):
        t.pull(keys[k0:k0 + (1 << 18)])
    outs = []
    for _ in range(2):
        s = lib.Sent2Vec(t, window=5, negative=5, minibatch=4096, niters=1)
        s.load_tokens(toks, off, ids)
        s.train()
        outs.append((s.docs()[1], s.stats()))
        del s
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.isfinite(outs[0][0]).all()
    st = outs[0][1]
    assert st["docs"] == nd and st["positions"] == int(off[-1])
    assert st["tgt_rows"] >= st["positions"]
    # the oracle slice: the first 120 docs as text, the rows of their words dumped at full precision
    ns = 120
    corpus = str(tmp_path / "slice.txt")
    with open(corpus, "w") as f:
        for i in range(ns):
            f.write(" ".join(str(int(x)) for x in toks[int(off[i]):int(off[i + 1])]) + "\n")
    words = np.unique(toks[:int(off[ns])])
    rows = t.export(torch.as_tensor(words.astype(np.int64), device="cuda")).cpu().numpy()
    dump = str(tmp_path / "words.txt")
    with open(dump, "w") as f:
        for k, r in zip(words, rows):  # WParam operator<< order: v then h (word2vec_global.h:102-111)
            f.write("%d\t%s\t%s\n" % (k, " ".join("%.9g" % x for x in r[D:2 * D]),
                                      " ".join("%.9g" % x for x in r[:D])))
    orc = oracle_mod.S2V(corpus, D, window=5, negative=5, minibatch=4096, niters=1, table_size=10 ** 8,
                         storage_f32=True, rand_offset=2)
    orc.load_words(dump)
    orc.train()
    t2 = lib.Table("w2v", dim=D, capacity=len(words) + 64, dtype="f32")
    s2 = lib.Sent2Vec(t2, window=5, negative=5, minibatch=4096, niters=1, rand_offset=2)
    s2.load_word_vector(dump)
    s2.load_text(corpus)
    s2.train()
    io, vo, _ = orc.docs()
    ig, vg, _ = s2.docs()
    assert len(io) == ns and np.array_equal(io, ig)
    assert np.array_equal(t2.export(torch.as_tensor(words.astype(np.int64), device="cuda")).cpu().numpy()[:, :2 * D],
                          rows[:, :2 * D])  # the word rows the slice trained on are the 1M table's
    rel = np.abs(vg - vo) / np.maximum(np.abs(vo), 1e-3)
    assert rel.max() < 1e-5, rel.max()


def test_s2v_config5_full_rank_share(lib, gpu):
    """BASELINE config 5 at its full per-GPU share (1e7 docs / 8 GPUs = 1.25M docs of 50-200
    Zipf(1M) tokens, 156M words, minibatches of 8192 against a 1M x 300 hash-initialised word
    table): loaded and trained, then run as the single pass (swps_s2v_run_tokens), the sentence
    vectors are bit-identical between the two and finite, every document and position is counted,
    and the load (the per-minibatch vocabularies on worker threads) finishes in seconds."""
    import time
    import torch
    from swiftmpi_amd.synth import zipf_tokens
    V, nd, D = 1_000_000, 1_250_000, 300
    rng = np.random.default_rng(7)
    lens = rng.integers(50, 201, nd)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    ids, _ = zipf_tokens(int(off[-1]), V, 100, seed=7)
    toks = ids.astype(np.uint64) + 1
    del ids
    sent = (np.arange(nd, dtype=np.uint64) + np.uint64(1)) * np.uint64(2654435761)
    t = lib.Table("w2v", dim=D, capacity=V + 1024, dtype="f32", init="hash", seed=3)
    t.pull(torch.arange(1, V + 1, dtype=torch.int64, device="cuda"))
    outs, loads = [], []
    for single in (False, True):  # load + train, then the single pass (swps_s2v_run_tokens)
        s = lib.Sent2Vec(t, window=5, negative=5, minibatch=8192, niters=1)
        t0 = time.perf_counter()
        if single:
            s.run_tokens(toks, off, sent)
        else:
            s.load_tokens(toks, off, sent)
        loads.append(time.perf_counter() - t0)
        if not single:
            s.train()
        outs.append((s.docs()[1], s.stats()))
        del s
    print("load s, single pass s", loads)
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.isfinite(outs[0][0]).all()
    st = outs[0][1]
    assert st["docs"] == nd and st["positions"] == int(off[-1])
    assert min(loads) < 30.0
