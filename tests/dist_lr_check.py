"""Multi-rank check of the key-sharded LR path on GPU(s).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29521 tests/dist_lr_check.py [--backend gloo|nccl]

Rank r trains its own Criteo-shaped rows whose feature keys are disjoint from
every other rank's (offset r << 20), so the union of the shards after sharded
training must equal, key for key and bit for bit, each rank's own single-GPU
training with the same hash-initialised weights — while the keys' owners are
spread over all ranks (BasicHashFrag, frag_num 2000), exercising every
exchange.  Ranks may share one GPU (gloo, host staging)."""
import argparse
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--epochs", type=int, default=2)
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ngpu = torch.cuda.device_count()
    dev = rank % max(ngpu, 1)
    torch.cuda.set_device(dev)
    dist.init_process_group(args.backend, rank=rank, world_size=world)
    import swiftmpi_amd as sw
    from swiftmpi_amd.dist import ShardedLR
    from swiftmpi_amd.synth import criteo

    y, off, f, v = criteo(3000 + 700 * rank, seed=50 + rank, bits=14)
    f = f + np.uint32(rank << 20)
    B = 255
    t = sw.Table("lr", capacity=1 << 16, dtype="f32", learning_rate=0.05, init="hash", seed=4, device=dev)
    sh = ShardedLR(t, frag_num=2000, minibatch=B)
    sh.load_csr(y, off, f, v)
    sh.init()
    e_s = sh.train(args.epochs)
    p_s, _ = sh.predict()
    keys, w, g2 = sh.shard_weights()
    t1 = sw.Table("lr", capacity=1 << 16, dtype="f32", learning_rate=0.05, init="hash", seed=4, device=dev)
    m = sw.LR(t1, minibatch=B, init_ref=False)
    m.load_csr(y, off, f, v)
    m.init()
    e_1 = m.train(args.epochs)
    p_1, _ = m.predict()
    k1, w1, g1 = m.params()
    assert np.array_equal(e_s, e_1), (e_s, e_1)
    assert np.array_equal(p_s, p_1)
    objs = [None] * world
    dist.all_gather_object(objs, (keys.tolist(), w.tolist(), g2.tolist(), k1.tolist(), w1.tolist(), g1.tolist()))
    if rank == 0:
        owned = {}
        for k, ww, gg, _, _, _ in objs:
            for a, b, c in zip(k, ww, gg):
                assert a not in owned, "key owned twice"
                owned[a] = (b, c)
        n = 0
        for _, _, _, kk, ww, gg in objs:
            for a, b, c in zip(kk, ww, gg):
                if owned[a] != (b, c):
                    print("MISMATCH key", a, owned[a], (b, c))
                    sys.exit(1)
                n += 1
        fm = sw.hashfrag_table(2000, world)
        per = {}
        for src, (k, _, _, _, _, _) in enumerate(objs):
            if len(k):
                assert (sw.to_node_id(np.array(k, dtype=np.uint64), 2000, fm) - 1 == src).all()
            per[src] = len(k)
        print("DIST LR OK world=%d keys=%d per-owner=%s steps/epoch=%d" % (world, n, per, sh.steps_per_epoch))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
