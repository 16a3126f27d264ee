"""The library's own key-sharded table (swps_table_route + swps_comm_*):
RCCL at world 1 through the full routed code path, two gloo ranks on one GPU
against one unrouted table (tests/dist_route_check.py), the SGD push rule,
the stream-ordered forms, and the app contexts refusing routed / non-AdaGrad
tables."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    from conftest import free_port
    return free_port()


def _keys(rng, n, V=5000):
    return (np.unique(rng.integers(0, V, n)).astype(np.uint64) * np.uint64(104729) + np.uint64(3))


@pytest.mark.parametrize("layout,dtype", [("w2v", "f32"), ("w2v", "f64"), ("lr", "f32")])
def test_rccl_world1_routed_equals_local(lib, gpu, layout, dtype):
    import swiftmpi_amd as sw
    from swiftmpi_amd.comm import Comm
    D = 20 if layout == "w2v" else 1
    kw = dict(dim=D, capacity=20000, dtype=dtype, learning_rate=0.7, init="hash", seed=4)
    comm = Comm.rccl(0, 1, port=_port())
    a, b = sw.Table(layout, **kw), sw.Table(layout, **kw)
    a.route(comm, frag_num=1000)
    rng = np.random.default_rng(2)
    for _ in range(5):
        k = _keys(rng, 3000)
        rng.shuffle(k)
        pa, pb = a.pull_h(k), b.pull_h(k)
        assert np.array_equal(pa, pb)
        g = rng.normal(0, 0.2, (len(k), a.push_elems)).astype(np.float64 if layout == "w2v" else np.float32)
        a.push_h(k, g)
        b.push_h(k, g)
    a.barrier()
    a.finish()
    st = a.route_stats()
    assert st["rounds"] == 10 and st["keys_remote"] == 0 and st["keys_sent"] == st["keys_served"]
    keys = np.sort(b.keys())
    assert np.array_equal(np.sort(a.keys()), keys)
    kk = torch.as_tensor(keys.astype(np.int64), device="cuda")
    assert torch.equal(a.export(kk), b.export(kk))
    a.close()
    b.close()
    comm.close()


@pytest.mark.parametrize("ipc", [False, True])
def test_routed_two_ranks_host_transport(lib, gpu, ipc):
    """ipc: the same rounds with the payloads through the device-initiated IPC exchange
    (swps_comm_enable_ipc; headers still over the host transport), incl. the rounds the last
    rank runs while the others serve from swps_finish."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dist_route_check.py")] + (["--ipc"] if ipc else [])
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    print(r.stdout[-6000:])
    print("\n".join(ln for ln in r.stderr.splitlines() if "rank0" in ln or "Error" in ln)[-6000:])
    assert r.returncode == 0 and "ROUTE OK" in r.stdout


def test_sgd_push_rule(lib, gpu):
    import swiftmpi_amd as sw
    rng = np.random.default_rng(3)
    k = _keys(rng, 500)
    for layout, dt in (("w2v", np.float64), ("lr", np.float32)):
        t = sw.Table(layout, dim=8, capacity=1000, dtype="f64" if layout == "w2v" else "f32", learning_rate=0.5,
                     init="hash", seed=1, push_rule="sgd")
        before = t.pull_h(k)
        g = rng.normal(0, 1, before.shape).astype(dt)
        t.push_h(k, g)
        after = t.pull_h(k)
        want = (before.astype(np.float64) + g.astype(np.float64) * np.float64(np.float32(0.5))).astype(dt)
        if layout == "w2v":
            assert np.array_equal(after, want)
            rows = t.export(torch.as_tensor(k.astype(np.int64), device="cuda")).cpu().numpy()
            assert not rows[:, 16:].any()  # the AdaGrad sums stay untouched
        else:
            want = (before + np.float32(0.5) * g).astype(np.float32)
            assert np.array_equal(after, want)
        t.close()


def test_async_forms_and_latched_errors(lib, gpu):
    import swiftmpi_amd as sw
    from swiftmpi_amd import capi
    t = sw.Table("w2v", dim=16, capacity=100, dtype="f32", init="hash", seed=2)
    s = torch.cuda.Stream()
    k = torch.arange(1, 51, dtype=torch.int64, device="cuda")
    out = torch.empty((50, 32), dtype=torch.float32, device="cuda")
    capi.check(capi.lib().swps_pull_async(t.h, capi.ptr(k), 50, capi.ptr(out), ctypes_stream(s)))
    g = torch.full((50, 32), 0.1, dtype=torch.float64, device="cuda")
    capi.check(capi.lib().swps_push_async(t.h, capi.ptr(k), 50, capi.ptr(g), ctypes_stream(s)))
    t.barrier()
    ref = sw.Table("w2v", dim=16, capacity=100, dtype="f32", init="hash", seed=2)
    want = ref.pull(k)
    assert torch.equal(out, want)
    ref.push(k, g)
    assert torch.equal(t.export(k), ref.export(k))
    # a push of unknown keys is latched and reported by the next sync
    bad = torch.arange(1000, 1010, dtype=torch.int64, device="cuda")
    capi.check(capi.lib().swps_push_async(t.h, capi.ptr(bad), 10, capi.ptr(g), ctypes_stream(s)))
    with pytest.raises(capi.SwpsError) as e:
        t.barrier()
    assert e.value.code == -2
    t.close()
    ref.close()


def ctypes_stream(s):
    import ctypes
    return ctypes.c_void_p(s.cuda_stream)


def test_app_contexts_refuse_routed_or_sgd_tables(lib, gpu):
    import swiftmpi_amd as sw
    from swiftmpi_amd import capi
    t = sw.Table("w2v", dim=16, capacity=100, push_rule="sgd")
    with pytest.raises(capi.SwpsError) as e:
        sw.Word2Vec(t)
    assert e.value.code == -7
    t.close()
    t = sw.Table("lr", capacity=100, push_rule="sgd")
    with pytest.raises(capi.SwpsError):
        sw.LR(t)
    t.close()


def test_native_sharded_driver_equals_python_driver(lib, gpu):
    """swps_w2v_shard_comm / swps_lr_shard_comm (the library runs the
    exchange over its TCP transport) == the Python driver over gloo, bit for
    bit, two ranks on one GPU (tests/dist_native_check.py)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dist_native_check.py"), "--tcp-port", str(_port())]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    print(r.stdout[-6000:])
    print("\n".join(ln for ln in r.stderr.splitlines() if "rank0" in ln or "Error" in ln)[-6000:])
    assert r.returncode == 0 and "NATIVE OK" in r.stdout


@pytest.mark.parametrize("ranks", [2, 4])
def test_ipc_exchange_equals_tcp(lib, gpu, ranks):
    """The device-initiated IPC exchange (swps_comm_enable_ipc) == the TCP transport, bit for bit:
    raw all-to-all-v calls (empty / odd / multi-slot segments, two streams) and the library-driven
    LR and CBOW loops, 2 and 4 ranks on one GPU (tests/dist_ipc_check.py); prints the per-exchange
    latency of both, and a lost peer fails every rank's next exchange."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(ranks),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "dist_ipc_check.py"), "--tcp-port", str(_port())]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    print(r.stdout[-6000:])
    print("\n".join(ln for ln in r.stderr.splitlines() if "rank0" in ln or "Error" in ln)[-6000:])
    assert r.returncode == 0 and "IPC OK" in r.stdout


@pytest.mark.parametrize("split", ["0", "1"])
def test_native_sharded_driver_rccl_world1(lib, gpu, tmp_path, monkeypatch, split):
    """The library-driven loop over RCCL at world 1 == the unsharded context
    with the same hash init, over four epochs: without the split the owner's
    buffers are the learner's (no self-copy); with it, from the third epoch
    on, every slot's pull is split into the keys the previous slot did not
    touch (served during the previous step's learn) and the rest."""
    import swiftmpi_amd as sw
    from swiftmpi_amd.comm import Comm
    from conftest import zipf_corpus
    path = zipf_corpus(str(tmp_path / "c.txt"), 120, 300, seed=12)
    kw = dict(window=3, negative=4, minibatch=23, sample=1e-3, unigram_size=10 ** 6, fp64_intermediates=False)
    # split 1: the early / late pulls (opt-in); split 0: world 1's aliased exchange (no self-copy)
    monkeypatch.setenv("SWPS_SPLIT_PULL", split)
    comm = Comm.rccl(0, 1, port=_port())
    ta = sw.Table("w2v", dim=24, capacity=2048, dtype="f32", init="hash", seed=7)
    a = sw.Word2Vec(ta, init="table", **kw)
    a.load_text(path)
    a.shard_comm(comm, frag_num=1000)
    a.init()
    a.exchange_stats(on=1)
    a.train(4)  # epochs 3-4 pull each slot's keys in an early and a late part
    xs = a.exchange_stats()
    tb = sw.Table("w2v", dim=24, capacity=2048, dtype="f32", init="hash", seed=7)
    b = sw.Word2Vec(tb, init="table", **kw)
    b.load_text(path)
    b.init()
    b.train(4)
    vk, _ = b.vocab()
    kk = torch.as_tensor(vk.astype(np.int64), device="cuda")
    assert torch.equal(ta.export(kk), tb.export(kk))  # every key lives on the one rank
    assert a.stats()["lstate"] == b.stats()["lstate"]
    assert xs["bytes_remote"] == 0 and xs["bytes_total"] > 0 and xs["calls"] > 0
    a.close()
    b.close()
    comm.close()


def test_native_sharded_resume_rccl_world1(lib, gpu, tmp_path):
    """A library-driven sharded context (swps_w2v_shard_comm) saves at an epoch
    boundary and a fresh context resumes it bit for bit: restore_state sets the
    driver's lockstep cursor and serve stream.  A mid-epoch save
    and a second shard_comm are refused."""
    import swiftmpi_amd as sw
    from swiftmpi_amd.comm import Comm
    from conftest import zipf_corpus
    path = zipf_corpus(str(tmp_path / "c.txt"), 120, 300, seed=14)
    kw = dict(window=3, negative=4, minibatch=23, sample=1e-3, unigram_size=10 ** 6, fp64_intermediates="bfp40")
    comm = Comm.rccl(0, 1, port=_port())

    def make():
        t = sw.Table("w2v", dim=24, capacity=2048, dtype="f32", init="hash", seed=7)
        w = sw.Word2Vec(t, init="table", **kw)
        w.load_text(path)
        w.shard_comm(comm, frag_num=1000)
        return t, w
    ta, a = make()
    with pytest.raises(lib.SwpsError, match="already"):
        a.shard_comm(comm, frag_num=1000)
    a.init()
    a.train(3)
    tb, b = make()
    b.init()
    b.train(1)
    b.train_batches(1)
    with pytest.raises(lib.SwpsError, match="epoch"):
        b.save(str(tmp_path / "mid"))
    b.train_batches(b.info()["batches"] - 1)
    prefix = str(tmp_path / "ck")
    b.save(prefix)
    tc, c = make()
    c.restore(prefix)
    c.train(1)
    vk, _ = a.vocab()
    kk = torch.as_tensor(vk.astype(np.int64), device="cuda")
    assert torch.equal(ta.export(kk), tc.export(kk))
    assert a.stats()["lstate"] == c.stats()["lstate"]
    for w in (a, b, c):
        w.close()
    comm.close()


def test_native_sharded_world1_full_table_fails_loudly(lib, gpu, tmp_path):
    """A shard whose capacity is below the vocabulary: the first
    full pull reports the table-full error instead of the steps reading a
    missing row's index past the shard, and the context stays un-initialised
    (training is refused, not run on rows that do not exist)."""
    import swiftmpi_amd as sw
    from swiftmpi_amd.comm import Comm
    from conftest import zipf_corpus
    path = zipf_corpus(str(tmp_path / "c.txt"), 80, 300, seed=15)
    comm = Comm.rccl(0, 1, port=_port())
    t = sw.Table("w2v", dim=24, capacity=64, dtype="f32", init="hash", seed=7)
    w = sw.Word2Vec(t, init="table", window=3, negative=4, minibatch=23, sample=1e-3, unigram_size=10 ** 6,
                    fp64_intermediates="bfp32")
    w.load_text(path)
    assert w.info()["vocab"] > 64
    w.shard_comm(comm, frag_num=1000)
    with pytest.raises(lib.SwpsError, match="capacity"):
        w.init()
    with pytest.raises(lib.SwpsError):
        w.train(1)
    w.close()
    comm.close()
