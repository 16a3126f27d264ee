"""The N>1 exchange path on CPU: world_size-2 gloo, the same Exchanger the
GPU orchestrator (swiftmpi_amd/dist.py) uses, driving a key-sharded parameter
server protocol (owner = BasicHashFrag node - 1) against a dict model."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    from conftest import free_port
    return free_port()


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import swiftmpi_amd as sw
        from swiftmpi_amd.dist import Exchanger
        ex = Exchanger()
        frag = 1000
        fm = sw.hashfrag_table(frag, world)
        rng = np.random.default_rng(100 + rank)
        D = 3
        # each rank requests a distinct key set (keys shared across ranks too)
        keys = np.unique(np.concatenate([rng.integers(0, 50, 40), rng.integers(1000 + rank * 100, 1100 + rank * 100, 30)])).astype(np.uint64)
        owner = sw.to_node_id(keys, frag, fm) - 1
        order = np.argsort(owner, kind="stable")
        keys, owner = keys[order], owner[order]
        sc = np.bincount(owner, minlength=world).astype(np.int64)
        rc = ex.all_gather_matrix(sc[None, :])[:, 0, rank].copy()
        rkeys = ex.a2a(torch.as_tensor(keys.astype(np.int64)), sc, rc).numpy().astype(np.uint64)
        # the owner's shard: value of key k = [k, 2k, 3k]
        assert (sw.to_node_id(rkeys, frag, fm) - 1 == rank).all()
        vals = np.stack([rkeys * (i + 1) for i in range(D)], 1).astype(np.float64)
        back = ex.a2a(torch.as_tensor(vals.ravel()), rc, sc, D).numpy().reshape(-1, D)
        assert np.array_equal(back[:, 0], keys.astype(np.float64))
        # push: per-source updates applied in rank order by the owner
        grads = np.full((len(keys), D), rank + 1.0)
        rg = ex.a2a(torch.as_tensor(grads.ravel()), sc, rc, D).numpy().reshape(-1, D)
        table = {}
        off = 0
        for src in range(world):
            for i in range(rc[src]):
                k = int(rkeys[off + i])
                table[k] = table.get(k, 0.0) * 2 + rg[off + i, 0]  # order-sensitive update
            off += rc[src]
        q.put((rank, {k: v for k, v in table.items()}, [int(x) for x in keys]))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_sharded_exchange():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    req = {r: set(k) for r, _, k in res}
    owned = {}
    for r, tab, _ in res:
        for k, v in tab.items():
            assert k not in owned
            owned[k] = v
    # every requested key is served by exactly one owner; updates in rank order
    for k in set().union(*req.values()):
        srcs = [r for r in range(world) if k in req[r]]
        exp = 0.0
        for r in srcs:
            exp = exp * 2 + (r + 1.0)
        assert owned[k] == exp
