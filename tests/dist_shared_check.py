"""Multi-rank check of the key-sharded path with keys SHARED across ranks,
against the lockstep multi-rank oracle (oracle/swps_oracle.cpp W2VMulti /
LRMulti: one server, every rank's mean-gradient push its own AdaGrad step in
rank order — cluster/server.h:156-176, global_push_access.h:69-96).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29531 tests/dist_shared_check.py [--backend gloo|nccl]

Every rank trains its own corpus drawn from ONE Zipf vocabulary (w<id>), so
the hot keys are pulled and pushed by every rank in every step and their
owners apply several pushes per step.  Checked (rank 0, after gathering every
shard): the union of the shards has exactly the oracle's keys; rows within
1e-9 relative (f64 table) or 1e-5 (fp32 table, fp64 intermediates) of the
oracle's after two epochs, 1e-3 after three steps in fast mode; every rank's LCG
end states bit-exact.  LR (Criteo-shaped rows over one shared 2^14 feature
space): weights and AdaGrad sums within 1e-5 relative.  Ranks may share one
GPU (gloo, host staging)."""
import argparse
import os
import sys
import tempfile

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def w2v_corpus(path, rank):
    rng = np.random.default_rng(60 + rank)
    V = 400
    p = 1.0 / np.arange(1, V + 1)
    p /= p.sum()
    with open(path, "w") as f:
        for _ in range(140 + 30 * rank):
            f.write(" ".join("w%d" % x for x in rng.choice(V, int(rng.integers(5, 40)), p=p)) + "\n")
    return path


def gather(obj, world):
    objs = [None] * world
    dist.all_gather_object(objs, obj)
    return objs


def check_w2v(sw, rank, world, dev, tmp, mode, epochs):
    from swiftmpi_amd.dist import ShardedWord2Vec
    dtype, fp64i = {"f64": ("f64", True), "parity": ("f32", True), "fast": ("f32", False),
                    "fast300": ("f32", False), "bfp300": ("f32", "bfp40"),
                    "fp32str": ("f32", "fp32"), "bfp32str": ("f32", "bfp32")}[mode]
    paths = [w2v_corpus(os.path.join(tmp, "c%d.txt" % r), r) for r in range(world)]
    kw = dict(window=4, negative=4, minibatch=17, sample=1e-3, unigram_size=10 ** 6)
    # fast300: the bench's D = 300 kernels (k_push_thp<TO_GRADS> on the learner, the
    # register-pass k_push_w2v_multi_t on the owners, several sources per hot row)
    D, seed = (300 if mode.endswith("300") else 16), 9
    t = sw.Table("w2v", dim=D, capacity=4096, dtype=dtype, learning_rate=0.7, init="hash", seed=seed, device=dev)
    sh = ShardedWord2Vec(t, frag_num=1000, fp64_intermediates=fp64i, **kw)
    sh.load_text(paths[rank])
    sh.init()
    # fast mode (fp32 neu1/neu1e/partials/push payload): the first 3 lockstep
    # steps (each rank's line-1 batch + two minibatches) — over hundreds of
    # steps a tiny hot vocabulary turns fp32 rounding into exp-table bucket
    # flips (tests/test_bench_shape_gpu.py), which compare nothing about the
    # exchange; f64 / parity: whole epochs
    # "fp32str" = fast mode selected by name (its push payload must be fp32 like False's)
    fast = mode.startswith("fast") or mode in ("fp32str", "bfp32str")
    nsteps = 3 if fast else epochs * sh.steps_per_epoch
    sh.train_steps(nsteps)
    sh.sync()
    keys, rows = sh.shard_rows()
    st = sh.stats()
    objs = gather((keys.tolist(), rows.tolist(), st["lstate"], st["fstate"]), world)
    if rank != 0:
        return True
    import oracle
    orc = oracle.W2VMulti(paths, D, window=kw["window"], negative=kw["negative"], minibatch=kw["minibatch"],
                          sample=kw["sample"], table_size=kw["unigram_size"], storage_f32=(dtype == "f32"), seed=seed)
    orc.train_steps(nsteps)
    ok_keys, ok_rows = orc.params()
    owned = {}
    for k, r, _, _ in objs:
        for kk, rr in zip(k, r):
            assert kk not in owned, "key owned twice"
            owned[kk] = rr
    assert sorted(owned) == [int(k) for k in ok_keys], "key sets differ"
    got = np.array([owned[int(k)] for k in ok_keys])
    if not fast:  # at an epoch boundary (the library plans, and jumps its LCGs, a whole epoch ahead)
        for r in range(world):
            so = orc.rank_stats(r)
            assert (objs[r][2], objs[r][3]) == (so["rng"], so["frng"]), "rank %d RNG streams diverged" % r
    rel = np.abs(got - ok_rows) / np.maximum(np.abs(ok_rows), 1e-3)
    vocabs = [set(open(p).read().split()) for p in paths]
    shared = len(set.intersection(*vocabs))  # words every rank trains (their keys get world pushes per step)
    assert shared > 100
    print("w2v %s world=%d keys=%d shared by all ranks=%d max rel %.3g p99.9 %.3g"
          % (mode, world, len(ok_keys), shared, rel.max(), np.quantile(rel, 0.999)), flush=True)
    if mode == "f64":
        return bool(np.allclose(got, ok_rows, rtol=1e-9, atol=1e-12))
    if mode == "parity":
        return bool(rel.max() <= 1e-5)
    if mode == "bfp300":  # whole epochs: ~2^-40 intermediates (tests/test_bench_shape_gpu.py BFP_TOL_MAX)
        return bool(rel.max() <= 1e-3)
    return bool(rel.max() <= 1e-3)


def check_lr(sw, rank, world, dev, tmp, epochs):
    from swiftmpi_amd.dist import ShardedLR
    from swiftmpi_amd.synth import criteo
    paths = []
    for r in range(world):  # every rank writes every rank's file (rank 0 needs them all for the oracle)
        y, off, f, v = criteo(2500 + 600 * r, seed=70 + r, bits=14)
        p = os.path.join(tmp, "lr%d.txt" % r)
        with open(p, "w") as fh:
            for i in range(len(y)):
                a, b = int(off[i]), int(off[i + 1])
                fh.write("%g %s\n" % (y[i], " ".join("%d:%.9g" % (k, x) for k, x in zip(f[a:b], v[a:b]))))
        paths.append(p)
    B, seed = 255, 4
    t = sw.Table("lr", capacity=1 << 16, dtype="f32", learning_rate=0.05, init="hash", seed=seed, device=dev)
    m = ShardedLR(t, frag_num=2000, minibatch=B)
    m.load_text(paths[rank])
    m.init()
    m.train(epochs)
    keys, w, g2 = m.shard_weights()
    objs = gather((keys.tolist(), w.tolist(), g2.tolist()), world)
    if rank != 0:
        return True
    import oracle
    orc = oracle.LRMulti(paths, minibatch=B, lr=0.05, seed=seed)
    orc.train(epochs)
    ok, ow, og = orc.params()
    got = {}
    for k, ww, gg in objs:
        for a, b, c in zip(k, ww, gg):
            assert a not in got, "key owned twice"
            got[a] = (b, c)
    assert sorted(got) == [int(k) for k in ok], "LR key sets differ"
    gw = np.array([got[int(k)][0] for k in ok])
    gg = np.array([got[int(k)][1] for k in ok])
    rw = np.abs(gw - ow) / np.maximum(np.abs(ow), 1e-3)
    rg = np.abs(gg - og) / np.maximum(np.abs(og), 1e-6)
    print("lr world=%d keys=%d w max rel %.3g g2 max rel %.3g" % (world, len(ok), rw.max(), rg.max()), flush=True)
    return bool(rw.max() <= 1e-5 and rg.max() <= 1e-5)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--modes", default="f64,parity,fast,lr")
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ngpu = torch.cuda.device_count()
    dev = rank % max(ngpu, 1)
    torch.cuda.set_device(dev)
    dist.init_process_group(args.backend, rank=rank, world_size=world)
    import swiftmpi_amd as sw
    tmp = tempfile.mkdtemp()
    ok = True
    for mode in args.modes.split(","):
        res = check_lr(sw, rank, world, dev, tmp, args.epochs) if mode == "lr" else \
            check_w2v(sw, rank, world, dev, tmp, mode, args.epochs)
        if rank == 0 and not res:
            print("FAIL", mode, flush=True)
            ok = False
        dist.barrier()
    if rank == 0:
        print("SHARED OK" if ok else "SHARED FAIL", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
