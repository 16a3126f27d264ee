"""The device-initiated IPC exchange (swps_comm_enable_ipc) against the library's TCP transport,
two ranks on one GPU (same-device IPC):

  1. swps_comm_alltoallv on seeded segments — empty, odd-sized (byte / 4-byte / 16-byte paths),
     several times a slot (segments stream through the two parities in rounds), from two streams
     in turn — must deliver exactly what the TCP transport delivers;
  2. the library-driven LR and CBOW loops (swps_lr_shard_comm / swps_w2v_shard_comm) over an
     IPC communicator must leave every rank's shard bit-identical to the same loops over TCP, and
     the sharded fixed-point LR step (plan none) on disjoint per-rank keys must equal each rank's
     single-GPU fixed-point training;
  3. the per-exchange latency of a small exchange (the LR step's size class) over both, printed
     as one JSON line ("IPC_LAT {...}");
  4. a lost peer: a lone exchange fails within its deadline, naming the peer, and the peer's next
     exchange fails at once; closing the communicator afterwards takes seconds on every rank.
  (2c: two ranks pushing the same keys to one owner in a step, fixed point vs fp64 sums; 3b: the
  bench's canary and its mismatch report, on an injected wrong byte.)

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29571 tests/dist_ipc_check.py --tcp-port 29581
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from dist_native_check import corpus, lr_data  # noqa: E402


def segments(call, world, rank, slot):
    """Byte counts [src][dst] for one call: every pattern from empty to 2.5 slots."""
    rng = np.random.default_rng(1000 + call)
    sizes = [0, 1, 7, 16, 4096, 4100, 65536, slot - 16, slot + 3, int(2.5 * slot), 12, 40000]
    m = np.array([[sizes[int(rng.integers(0, len(sizes)))] for _ in range(world)] for _ in range(world)])
    return m


def payload(call, src, dst, n):
    g = np.random.default_rng((call * 7919 + src * 131 + dst) & 0xFFFFFFFF)
    return g.integers(0, 256, n, dtype=np.uint8)


def raw_exchange(comm, rank, world, slot, calls, streams):
    out = []
    for call in range(calls):
        m = segments(call, world, rank, slot)
        send = np.concatenate([payload(call, rank, d, int(m[rank, d])) for d in range(world)] + [np.zeros(0, np.uint8)])
        st = streams[call % len(streams)]
        with torch.cuda.stream(st):
            ds = torch.as_tensor(send, device="cuda") if send.size else torch.zeros(1, dtype=torch.uint8, device="cuda")
            dr = torch.full((max(int(m[:, rank].sum()), 1),), 0xAB, dtype=torch.uint8, device="cuda")
            comm.alltoallv(ds, m[rank, :], dr, m[:, rank], stream=st)
            got = dr[:int(m[:, rank].sum())].cpu().numpy()
        want = np.concatenate([payload(call, s, rank, int(m[s, rank])) for s in range(world)] + [np.zeros(0, np.uint8)])
        assert np.array_equal(got, want), ("raw exchange differs", call, rank, m.tolist())
        out.append(got)
    return out


def latency(comm, world, nbytes, reps=200):
    send = torch.arange(nbytes * world, dtype=torch.int64, device="cuda").to(torch.uint8)
    recv = torch.empty_like(send)
    cnt = [nbytes] * world
    for _ in range(10):
        comm.alltoallv(send, cnt, recv, cnt)
    torch.cuda.synchronize()
    dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(reps):
        comm.alltoallv(send, cnt, recv, cnt)
    e1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps * 1e6
    return {"device_us": e0.elapsed_time(e1) / reps * 1e3, "wall_us": wall}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tcp-port", type=int, default=29581)
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import swiftmpi_amd as sw
    from swiftmpi_amd.comm import Comm
    torch.cuda.set_device(0)
    slot = 64 << 10  # small: 2.5-slot segments take several rounds per channel
    tcp = Comm.tcp(rank, world, 0, port=a.tcp_port)
    ipc = Comm.tcp(rank, world, 0, port=a.tcp_port + 1).enable_ipc(slot)
    ipc.set_timeout(60)
    info = ipc.ipc_info()
    assert info["enabled"] == 1 and info["slot_bytes"] == slot, info
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    # 1. raw exchanges
    rt = raw_exchange(tcp, rank, world, slot, 24, streams)
    ri = raw_exchange(ipc, rank, world, slot, 24, streams)
    assert all(np.array_equal(x, y) for x, y in zip(rt, ri))
    ipc.check()
    print("rank %d raw ok: %d exchanges" % (rank, len(ri)), flush=True)
    # 2. the library-driven loops, TCP vs IPC
    tmp = tempfile.mkdtemp()
    lpath = lr_data(os.path.join(tmp, "l%d.txt" % rank), rank)
    res = {}
    for name, comm in (("tcp", tcp), ("ipc", ipc)):
        t = sw.Table("lr", capacity=8192, dtype="f32", learning_rate=0.05, init="hash", seed=5, device=0)
        m = sw.LR(t, minibatch=50, init_ref=False)
        m.load_text(lpath)
        m.shard_comm(comm, frag_num=2000)
        m.init()
        err = m.train(3)
        pred = m.predict()
        k = np.sort(t.keys())
        res[name] = (err, pred[0], k, t.export(torch.as_tensor(k.astype(np.int64), device="cuda")).cpu())
        m.close()
        t.close()
    a_, b_ = res["tcp"], res["ipc"]
    assert np.array_equal(a_[0], b_[0]) and np.array_equal(a_[1], b_[1]) and np.array_equal(a_[2], b_[2])
    assert torch.equal(a_[3], b_[3])
    print("rank %d lr ok: %d keys" % (rank, len(a_[2])), flush=True)
    # 2b. the sharded fixed-point step (plan none, fast sums) at world 2: each rank's keys are
    # disjoint from the other's (offset rank << 20), so the union of the shards must equal each
    # rank's own single-GPU fixed-point training, key for key and bit for bit — over TCP and IPC
    from swiftmpi_amd.synth import criteo
    y, off, f, v = criteo(3000 + 700 * rank, seed=50 + rank, bits=14)
    f = f + np.uint32(rank << 20)
    lk = dict(capacity=1 << 16, dtype="f32", learning_rate=0.05, init="hash", seed=4, device=0)
    res = {}
    for name, comm in (("tcp", tcp), ("ipc", ipc), ("single", None)):
        t = sw.Table("lr", **lk)
        m = sw.LR(t, minibatch=255, init_ref=False, fast_sums=True, plan="none")
        m.load_csr(y, off, f, v)
        if comm is not None:
            m.shard_comm(comm, frag_num=2000)
        m.init()
        m.train(2)
        k = np.sort(t.keys())
        res[name] = (k, t.export(torch.as_tensor(k.astype(np.int64), device="cuda")).cpu().numpy())
        m.close()
        t.close()
    assert np.array_equal(res["tcp"][0], res["ipc"][0]) and np.array_equal(res["tcp"][1], res["ipc"][1])
    objs = [None] * world
    dist.all_gather_object(objs, (res["ipc"][0].tolist(), res["ipc"][1].tolist(), res["single"][0].tolist(),
                                  res["single"][1].tolist()))
    if rank == 0:
        owned = {}
        for k, r, _, _ in objs:
            for a, b in zip(k, r):
                assert a not in owned, "key owned twice"
                owned[a] = tuple(b)
        n = 0
        for _, _, k, r in objs:
            for a, b in zip(k, r):
                assert owned[a] == tuple(b), ("fixed-point shard differs", a, owned[a], b)
                n += 1
        assert n == len(owned), (n, len(owned))
        print("lr fixed point sharded ok: %d keys" % n, flush=True)
    # 2c. shared keys: both ranks' rows draw from one key space, so in one step two
    # learners push the same key to its owner (the N > 1 LR leg's case).  The sharded fixed-point
    # step (plan none) must equal itself over TCP and IPC bit for bit, and the sharded fp64-sum step
    # (plan load, fast sums) within 1e-6 relative — the single-GPU bar between the two sum forms
    y, off, f, v = criteo(3000 + 500 * rank, seed=70 + rank, bits=13)
    res = {}
    for name, comm, plan in (("tcp", tcp, "none"), ("ipc", ipc, "none"), ("load", ipc, "load")):
        t = sw.Table("lr", **lk)
        m = sw.LR(t, minibatch=255, init_ref=False, fast_sums=True, plan=plan)
        m.load_csr(y, off, f, v)
        m.shard_comm(comm, frag_num=2000)
        m.init()
        m.train(2)
        k = np.sort(t.keys())
        res[name] = (k, t.export(torch.as_tensor(k.astype(np.int64), device="cuda")).cpu().numpy())
        m.close()
        t.close()
    assert np.array_equal(res["tcp"][0], res["ipc"][0]) and np.array_equal(res["tcp"][1], res["ipc"][1])
    assert np.array_equal(res["ipc"][0], res["load"][0])
    a_, b_ = res["ipc"][1].astype(np.float64), res["load"][1].astype(np.float64)
    assert np.abs(a_ - b_).max() <= 1e-6 * np.abs(b_).max(), (np.abs(a_ - b_).max(), np.abs(b_).max())
    shared = [None] * world
    dist.all_gather_object(shared, set(np.unique(f).tolist()))
    print("rank %d lr shared keys ok: %d keys owned, %d keys in both ranks' data" %
          (rank, len(res["ipc"][0]), len(shared[0] & shared[1 % world])), flush=True)
    path = corpus(os.path.join(tmp, "c%d.txt" % rank), rank)
    kw = dict(window=4, negative=4, minibatch=19, sample=1e-3, unigram_size=10 ** 6, fp64_intermediates=False)
    res = {}
    for name, comm in (("tcp", tcp), ("ipc", ipc)):
        t = sw.Table("w2v", dim=300, capacity=4096, dtype="f32", learning_rate=0.7, init="hash", seed=3, device=0)
        w = sw.Word2Vec(t, init="table", **kw)
        w.load_text(path)
        w.shard_comm(comm, frag_num=1000)
        w.init()
        w.train_batches(2 * 9 + 1)
        w.sync()
        k = np.sort(t.keys())
        res[name] = (k, t.export(torch.as_tensor(k.astype(np.int64), device="cuda")).cpu(), w.stats())
        w.close()
        t.close()
    a_, b_ = res["tcp"], res["ipc"]
    assert np.array_equal(a_[0], b_[0]) and torch.equal(a_[1], b_[1])
    assert a_[2]["lstate"] == b_[2]["lstate"], (a_[2], b_[2])
    print("rank %d w2v ok: %d keys" % (rank, len(a_[0])), flush=True)
    # 3. latency of one exchange (8 KiB / 64 KiB per peer)
    lat = {}
    for nb in (8 << 10, 64 << 10):
        lat["tcp_%dKiB" % (nb >> 10)] = latency(tcp, world, nb, reps=100)
        lat["ipc_%dKiB" % (nb >> 10)] = latency(ipc, world, nb, reps=400)
    ipc.check()
    info = ipc.ipc_info()
    if rank == 0:
        print("IPC_LAT " + json.dumps({"world": world, "same_gpu": True, "slot_bytes": slot, "latency": lat,
                                       "ipc_exchanges": info["exchanges"], "ipc_bytes_remote": info["bytes_remote"]}),
              flush=True)
    # 3b. the canary (bench.py's gate for the IPC path) passes, and a wrong byte injected on rank
    # world - 1 at offset 5000 of the receive buffer (inside rank 0's segment, whose first part is
    # 1 KiB .. 2.5 slots) is reported with the peer, the channel / round and the offset
    ok, rep = ipc.canary()
    assert ok and not rep, rep
    os.environ["SWPS_IPC_DIAG_CORRUPT"] = "%d:%d" % (world - 1, 5000)
    ok, rep = ipc.canary()
    del os.environ["SWPS_IPC_DIAG_CORRUPT"]
    if rank == world - 1:
        assert not ok and len(rep) == 1, rep
        r0 = rep[0]
        assert r0["peer"] == 0 and r0["recv_offset"] == 5000 and r0["offset"] == 5000 and r0["bad_bytes"] == 1, r0
        assert r0["expected"] != r0["got"] and r0["channel"] >= 0 and r0["round"] >= 0, r0
        print("rank %d canary report ok: %s" % (rank, json.dumps(r0)), flush=True)
    else:
        assert ok and not rep, rep
    ipc.check()
    # 4. a lost peer: rank 0 exchanges alone (rank 1 never joins) and must fail within its 2-s
    # deadline; its give-up marks every rank dead, so rank 1's next exchange fails at once
    from swiftmpi_amd.capi import SwpsError
    dist.barrier()
    one = torch.ones(1024 * world, dtype=torch.uint8, device="cuda")
    got = torch.empty_like(one)
    if rank == 0:
        ipc.set_timeout(2)
        t0 = time.perf_counter()
        ipc.alltoallv(one, [1024] * world, got, [1024] * world)
        torch.cuda.synchronize()
        waited = time.perf_counter() - t0
        try:
            ipc.check()
            raise AssertionError("a lone exchange did not time out")
        except SwpsError as e:
            assert "IPC exchange" in str(e) and ("rank 1" in str(e) or world > 2), str(e)
        assert waited < 30, waited
        print("rank 0 lost peer detected after %.1f s: ok" % waited, flush=True)
    dist.barrier()
    if rank != 0:
        t0 = time.perf_counter()
        ipc.alltoallv(one, [1024] * world, got, [1024] * world)
        torch.cuda.synchronize()
        try:
            ipc.check()
            raise AssertionError("an exchange with a dead peer did not fail")
        except SwpsError as e:
            assert "IPC exchange" in str(e), str(e)
        assert time.perf_counter() - t0 < 10
        print("rank %d dead peer detected: ok" % rank, flush=True)
    dist.barrier()
    t0 = time.perf_counter()
    ipc.close()  # collective: every rank joins one bounded all-gather, also after a dead exchange
    assert time.perf_counter() - t0 < 15, time.perf_counter() - t0
    print("rank %d close after a dead exchange: %.2f s" % (rank, time.perf_counter() - t0), flush=True)
    tcp.close()
    dist.barrier()
    if rank == 0:
        print("IPC OK")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
