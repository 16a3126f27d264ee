import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import oracle, swiftmpi_amd as lib
from test_bench_shape_gpu import corpus, CFG, rel_err
for D in (300, 100):
    path = corpus('/tmp/c1.txt', lines=41, seed=83)
    c = dict(CFG, minibatch=40)
    orc = oracle.W2V(path, D, window=5, negative=5, minibatch=40, sample=1e-5, alpha=0.05, lr=0.7, table_size=10**8, storage_f32=True)
    orc.init_rand(1, 2); orc.train(1)
    po = orc.get_params()
    outs = {}
    for mode in ("parity", "fast"):
        t = lib.Table("w2v", dim=D, capacity=orc.vocab_size + 16, dtype="f32", learning_rate=0.7)
        w = lib.Word2Vec(t, window=5, negative=5, minibatch=40, sample=1e-5, alpha=0.05, unigram_size=10**8, init="ref", rand_offset=2, fp64_intermediates=(mode == "parity"))
        w.load_text(path); w.init(); w.train(1)
        outs[mode] = w.get_params()
    keys, cnt = orc.vocab()
    for mode in ("parity", "fast"):
        rel = rel_err(outs[mode], po)
        i, j = np.unravel_index(np.argmax(rel), rel.shape)
        print("D", D, mode, "max", rel.max(), "at row", i, "col", j, "block", j // D, "count", cnt[i], "oracle", po[i, j], "gpu", outs[mode][i, j],
              "h2/v2 at col", po[i, 2 * D + j % D], po[i, 3 * D + j % D])
        for blk in range(4):
            r = rel[:, blk * D:(blk + 1) * D]
            print("   block", blk, "max", r.max(), "p99.9", np.quantile(r, 0.999), "n>1e-5", int((r > 1e-5).sum()))
    rel = rel_err(outs["fast"], outs["parity"])
    print("fast vs parity max", rel.max())
