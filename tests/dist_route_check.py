"""Multi-rank check of the library's own key-sharded table (swps_table_route:
the RPC path of GlobalPullAccess / GlobalPushAccess, global_pull_access.h:
46-107, global_push_access.h:48-96, served by the owners as in server.h:
129-176) over the host transport (gloo; ranks may share one GPU).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29541 tests/dist_route_check.py

Every rank pulls and pushes keys drawn from ONE Zipf key space (so hot keys
are pulled / pushed by every rank in every round and owners apply several
sources' pushes per key).  Rank 0 then gathers every shard and compares it
with ONE unrouted table driven through the same rounds: per round, the union
of the pulls, then every rank's push in rank order (the reference applies
each worker's push request as its own AdaGrad step).  Rows must be bit-exact,
pulled values bit-exact, and each key must live on its BasicHashFrag owner.
The last rank runs extra rounds after the others called swps_finish (they
keep serving).  Layouts: W2V (fp32 and fp64 tables, AdaGrad), LR (AdaGrad)
and W2V with the SGD push rule."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ROUNDS = 4
EXTRA = 2  # rounds the last rank runs alone (the others are in swps_finish)


def round_keys(rng, n, V=3000):
    p = 1.0 / np.arange(1, V + 1)
    p /= p.sum()
    k = np.unique(rng.choice(V, n, p=p)).astype(np.uint64) * np.uint64(7919) + np.uint64(11)
    rng.shuffle(k)
    return k


def plan(world, seed, layout, D):
    """[round][rank] -> (keys, grads) for every rank: the same on every rank."""
    out = []
    for r in range(ROUNDS + EXTRA):
        row = []
        for src in range(world):
            rng = np.random.default_rng(seed * 1000 + r * 31 + src)
            if r >= ROUNDS and src != world - 1:
                row.append(None)
                continue
            k = round_keys(rng, 200 + 40 * src)
            if layout == "w2v":
                g = rng.normal(0, 0.3, (len(k), 2 * D))
            else:
                g = rng.normal(0, 0.3, len(k)).astype(np.float32)
            row.append((k, g))
        out.append(row)
    return out


def run_case(sw, comm, rank, world, dev, layout, dtype, rule, seed):
    D = 12 if layout == "w2v" else 1
    tk = dict(dim=D, capacity=8192, dtype=dtype, learning_rate=0.7 if layout == "w2v" else 0.05, init="hash",
              seed=seed, device=dev, push_rule=rule)
    t = sw.Table(layout, **tk)
    t.route(comm, frag_num=997)
    P = plan(world, seed, layout, D)
    pulled = []
    for r, row in enumerate(P):
        if row[rank] is None:
            t.finish()
            break
        k, g = row[rank]
        pulled.append(t.pull_h(k))
        t.push_h(k, g)
    else:
        t.finish()
    stats = t.route_stats()
    keys = t.keys()
    rows = []
    if len(keys):
        kk = torch.as_tensor(keys.astype(np.int64), device="cuda:%d" % dev)
        rows = t.export(kk).double().cpu().numpy()
    objs = [None] * world
    dist.all_gather_object(objs, (keys, rows, pulled, stats))
    t.close()
    if rank != 0:
        return
    # the reference run: one unrouted table, same rounds, pushes in rank order
    ref = sw.Table(layout, **tk)
    ref_pulled = [[] for _ in range(world)]
    for r, row in enumerate(P):
        active = [s for s in range(world) if row[s] is not None]
        for s in active:
            k, _ = row[s]
            ref_pulled[s].append(ref.pull_h(k))
        for s in active:
            k, g = row[s]
            ref.push_h(k, g)
    frag = np.zeros(997, dtype=np.uint32)
    sw.capi.check(sw.capi.lib().swps_hashfrag_table(997, world, sw.capi.ptr(frag)))
    allk = []
    for src, (keys, rows, pulled, stats) in enumerate(objs):
        for a, b in zip(pulled, ref_pulled[src]):
            assert np.array_equal(a, b), (layout, dtype, rule, "pulled values differ", src)
        if len(keys):
            node = frag[[sw.capi.lib().swps_fmix64(int(x)) % 997 for x in keys]]
            assert np.all(node == src + 1), "key on the wrong owner"
            kk = torch.as_tensor(keys.astype(np.int64), device="cuda:%d" % dev)
            want = ref.export(kk).double().cpu().numpy()
            assert np.array_equal(rows, want), (layout, dtype, rule, src, float(np.abs(rows - want).max()))
        allk.extend(int(x) for x in keys)
        assert stats["rounds"] == 2 * (ROUNDS + EXTRA), stats  # a pull and a push per round
    assert sorted(allk) == sorted(int(x) for x in ref.keys()), "union of the shards != reference key set"
    print("case ok", layout, dtype, rule, "keys", len(allk), "remote keys sent by rank 0", objs[0][3]["keys_remote"])


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import swiftmpi_amd as sw
    from swiftmpi_amd.comm import Comm
    dev = 0
    torch.cuda.set_device(dev)
    comm = Comm.host(device=dev)
    if "--ipc" in sys.argv:  # payloads device to device through IPC-mapped inboxes (small slots: rounds)
        comm.enable_ipc(64 << 10)
        comm.set_timeout(60)
    for i, (layout, dtype, rule) in enumerate([("w2v", "f32", "adagrad"), ("w2v", "f64", "adagrad"),
                                               ("lr", "f32", "adagrad"), ("w2v", "f32", "sgd")]):
        run_case(sw, comm, rank, world, dev, layout, dtype, rule, seed=5 + i)
    info = comm.ipc_info()
    comm.close()
    dist.barrier()
    if rank == 0:
        print("ROUTE OK", "(ipc: %d exchanges)" % info["exchanges"] if "--ipc" in sys.argv else "")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
