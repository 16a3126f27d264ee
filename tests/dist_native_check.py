"""The library-driven sharded loop (swps_w2v_shard_comm / swps_lr_shard_comm,
src/swps_driver.cpp) against the Python driver (swiftmpi_amd/dist.py) on the
same inputs: both run the lockstep protocol of SURVEY.md §8(e), so every
rank's shard must come out bit-identical, with the same LCG end states.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29551 tests/dist_native_check.py --tcp-port 29561

The Python driver exchanges over gloo; the native one over the library's TCP
transport (swps_comm_create_tcp) — ranks share one GPU.  Corpora differ in
size per rank (so the short rank runs empty steps) and share one Zipf
vocabulary (owners apply several sources' pushes per key)."""
import argparse
import os
import sys
import tempfile

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def corpus(path, rank):
    rng = np.random.default_rng(70 + rank)
    V = 500
    p = 1.0 / np.arange(1, V + 1)
    p /= p.sum()
    with open(path, "w") as f:
        for _ in range(150 + 45 * rank):
            f.write(" ".join("w%d" % x for x in rng.choice(V, int(rng.integers(5, 40)), p=p)) + "\n")
    return path


def lr_data(path, rank):
    rng = np.random.default_rng(90 + rank)
    with open(path, "w") as f:
        for _ in range(600 + 200 * rank):
            feats = sorted(set(int(x) for x in rng.zipf(1.3, 12) % 3000))
            f.write("%d %s\n" % (int(rng.integers(0, 2)), " ".join("%d:%.3f" % (k, rng.random()) for k in feats)))
    return path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tcp-port", type=int, default=29561)
    a = ap.parse_args()
    os.environ["SWPS_SPLIT_PULL"] = "1"  # the native driver's early / late pulls (opt-in) from the third epoch
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import swiftmpi_amd as sw
    from swiftmpi_amd.comm import Comm
    from swiftmpi_amd.dist import ShardedLR, ShardedWord2Vec
    dev = 0
    torch.cuda.set_device(dev)
    comm = Comm.tcp(rank, world, dev, port=a.tcp_port)
    tmp = tempfile.mkdtemp()
    path = corpus(os.path.join(tmp, "c%d.txt" % rank), rank)
    kw = dict(window=4, negative=4, minibatch=19, sample=1e-3, unigram_size=10 ** 6)
    # fast300: the bench kernels (D = 300): the learner's mean gradients in two owner-half passes,
    # the native driver's gradient exchange in two halves (the first behind the second pass)
    # bfp300: the BFP-row kernels (bfp40) (fp64 push payload, two owner-half passes)
    for mode in ("f64", "parity", "fast", "fast300", "bfp300"):
        dtype, fp64i = {"f64": ("f64", True), "parity": ("f32", True), "fast": ("f32", False),
                        "fast300": ("f32", False), "bfp300": ("f32", "bfp40")}[mode]
        tk = dict(dim=300 if mode.endswith("300") else 16, capacity=4096, dtype=dtype, learning_rate=0.7, init="hash",
                  seed=3, device=dev)
        ta = sw.Table("w2v", **tk)
        py = ShardedWord2Vec(ta, frag_num=1000, fp64_intermediates=fp64i, **kw)
        py.load_text(path)
        py.init()
        steps = 3 * py.steps_per_epoch + 2  # the split pull runs from the third epoch on
        py.train_steps(steps)
        py.sync()
        tb = sw.Table("w2v", **tk)
        nat = sw.Word2Vec(tb, init="table", fp64_intermediates=fp64i, **kw)
        nat.load_text(path)
        nat.shard_comm(comm, frag_num=1000)
        nat.init()
        nat.train_batches(steps)
        nat.sync()
        ka = np.sort(ta.keys())
        assert np.array_equal(ka, np.sort(tb.keys())), (mode, "shard key sets differ")
        kt = torch.as_tensor(ka.astype(np.int64), device="cuda")
        ra, rb = ta.export(kt), tb.export(kt)
        assert torch.equal(ra, rb), (mode, rank, float((ra.double() - rb.double()).abs().max()))
        sa, sb = py.stats(), nat.stats()
        assert sa["lstate"] == sb["lstate"] and sa["fstate"] == sb["fstate"], (mode, sa, sb)
        print("rank %d w2v %s ok: %d keys, %d steps" % (rank, mode, len(ka), steps), flush=True)
        nat.close()
        py.w.close()
        ta.close()
        tb.close()
    # LR
    lpath = lr_data(os.path.join(tmp, "l%d.txt" % rank), rank)
    tk = dict(capacity=8192, dtype="f32", learning_rate=0.05, init="hash", seed=5, device=dev)
    ta = sw.Table("lr", **tk)
    py = ShardedLR(ta, frag_num=2000, minibatch=50)
    py.load_text(lpath)
    py.init()
    ea = py.train(3)
    pa = py.predict()
    tb = sw.Table("lr", **tk)
    nat = sw.LR(tb, minibatch=50, init_ref=False)
    nat.load_text(lpath)
    nat.shard_comm(comm, frag_num=2000)
    nat.init()
    eb = nat.train(3)
    pb = nat.predict()
    assert np.array_equal(ea, eb), (ea, eb)
    assert np.array_equal(pa[0], pb[0])
    ka = np.sort(ta.keys())
    kt = torch.as_tensor(ka.astype(np.int64), device="cuda")
    assert torch.equal(ta.export(kt), tb.export(kt))
    print("rank %d lr ok: %d keys" % (rank, len(ka)), flush=True)
    comm.close()
    dist.barrier()
    if rank == 0:
        print("NATIVE OK")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
