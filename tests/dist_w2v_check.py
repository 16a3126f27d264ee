"""Multi-rank check of the key-sharded path on GPU(s).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 tests/dist_w2v_check.py [--backend gloo|nccl] [--dtype f64|f32]

Rank r trains its own corpus whose words are disjoint from every other rank's
(w<r>_<id>), so negatives never cross ranks: the union of the shards after
sharded training must equal, key for key and bit for bit, each rank's own
single-GPU (unsharded) training with the same hash-initialised rows — while
the keys' owners are spread over all ranks (BasicHashFrag), exercising every
pull / push exchange.  Ranks may share one GPU (gloo, host staging)."""
import argparse
import os
import sys
import tempfile

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--fast", action="store_true", help="fp32 intermediates (fp32 push payload)")
    ap.add_argument("--pipeline", action="store_true",
                    help="pipelined driver: check run-to-run bit-identity instead of equality with lockstep")
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ngpu = torch.cuda.device_count()
    dev = rank % max(ngpu, 1)
    torch.cuda.set_device(dev)
    dist.init_process_group(args.backend, rank=rank, world_size=world)
    import swiftmpi_amd as sw
    from swiftmpi_amd.dist import ShardedWord2Vec

    rng = np.random.default_rng(40 + rank)
    V = 300 + 50 * rank
    p = 1.0 / np.arange(1, V + 1)
    p /= p.sum()
    tmp = tempfile.mkdtemp()
    path = os.path.join(tmp, "c%d.txt" % rank)
    with open(path, "w") as f:
        for _ in range(150 + 40 * rank):
            f.write(" ".join("w%d_%d" % (rank, x) for x in rng.choice(V, int(rng.integers(5, 40)), p=p)) + "\n")
    kw = dict(window=4, negative=4, minibatch=17, sample=1e-3, unigram_size=10 ** 6, fp64_intermediates=not args.fast)
    D = 16
    # sharded
    def sharded_run():
        t = sw.Table("w2v", dim=D, capacity=4096, dtype=args.dtype, learning_rate=0.7, init="hash", seed=7,
                     device=dev)
        sh = ShardedWord2Vec(t, frag_num=1000, pipeline=args.pipeline, **kw)
        sh.load_text(path)
        sh.init()
        sh.train(args.epochs)
        return sh, sh.shard_rows()

    sh, (keys, rows) = sharded_run()
    if args.pipeline:
        _, (k2, r2) = sharded_run()
        o1, o2 = np.argsort(keys), np.argsort(k2)  # row order = insertion order, which is racy
        assert np.array_equal(keys[o1], k2[o2]) and np.array_equal(rows[o1], r2[o2]), "pipelined run not reproducible"
        assert np.isfinite(rows).all()
        if rank == 0:
            print("DIST PIPELINE OK world=%d owned=%d steps/epoch=%d" % (world, len(keys), sh.steps_per_epoch))
        dist.barrier()
        dist.destroy_process_group()
        return
    # every rank's own single-GPU training
    t1 = sw.Table("w2v", dim=D, capacity=4096, dtype=args.dtype, learning_rate=0.7, init="hash", seed=7, device=dev)
    w1 = sw.Word2Vec(t1, init="table", **kw)
    w1.load_text(path)
    w1.init()
    w1.train(args.epochs)
    vk, _ = w1.vocab()
    ref = w1.get_params()
    # exchange: owners' shards and everyone's reference rows
    objs = [None] * world
    dist.all_gather_object(objs, (keys.tolist(), rows.tolist(), vk.tolist(), ref.tolist(),
                                  sh.stats()["lstate"], w1.stats()["lstate"]))
    if rank == 0:
        owned = {}
        for k, r, _, _, _, _ in objs:
            for kk, rr in zip(k, r):
                assert kk not in owned, "key owned twice"
                owned[kk] = np.array(rr)
        n = 0
        for _, _, vkeys, refrows, ls, lr in objs:
            assert ls == lr, "RNG streams diverged"
            for kk, rr in zip(vkeys, refrows):
                got = owned[kk]
                if not np.array_equal(got, np.array(rr)):
                    print("MISMATCH key", kk, np.abs(got - np.array(rr)).max())
                    sys.exit(1)
                n += 1
        owners = {}
        fm = sw.hashfrag_table(1000, world)
        for src, (k, _, _, _, _, _) in enumerate(objs):
            if len(k):
                assert (sw.to_node_id(np.array(k, dtype=np.uint64), 1000, fm) - 1 == src).all()
            owners[src] = len(k)
        print("DIST OK world=%d keys=%d per-owner=%s steps/epoch=%d" % (world, n, owners, sh.steps_per_epoch))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
