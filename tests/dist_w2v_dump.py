"""Reference side of test_compat.py's two-rank C++ app test: the Python
key-sharded driver (swiftmpi_amd/dist.py, gloo) trains each rank's own corpus
with the compat Word2VecApp's settings and dumps every rank's shard in the
reference's text format (`<out>.<rank>`).

    python -m torch.distributed.run --nproc-per-node 2 ... tests/dist_w2v_dump.py \\
        --data c0.txt,c1.txt --out py_param.txt --niters 2 --dim 16 ..."""
import argparse
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--data")
    ap.add_argument("--out")
    ap.add_argument("--niters", type=int, default=2)
    ap.add_argument("--dim", type=int, default=16)
    ap.add_argument("--window", type=int, default=3)
    ap.add_argument("--negative", type=int, default=4)
    ap.add_argument("--minibatch", type=int, default=20)
    ap.add_argument("--sample", type=float, default=1e-3)
    ap.add_argument("--alpha", type=float, default=0.05)
    ap.add_argument("--lr", type=float, default=0.7)
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    import swiftmpi_amd as sw
    from swiftmpi_amd.dist import ShardedWord2Vec
    torch.cuda.set_device(0)
    # Cluster's shard: fp32, hash init with seed 0, capacity 2^22; Word2VecApp: fp64 intermediates
    t = sw.Table("w2v", dim=a.dim, capacity=1 << 22, dtype="f32", learning_rate=a.lr, init="hash", seed=0)
    w = ShardedWord2Vec(t, frag_num=1000, window=a.window, negative=a.negative, minibatch=a.minibatch,
                        sample=a.sample, alpha=a.alpha, fp64_intermediates=True)
    w.load_text(a.data.split(",")[rank])
    w.init()
    w.train(a.niters)
    t.dump("%s.%d" % (a.out, rank))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
