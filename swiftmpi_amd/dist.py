"""Key-sharded multi-GPU word2vec and LR: one process per GPU, the reference's
worker+server-per-rank layout with the ZeroMQ request /
response path (transfer/transfer.h:86-241) replaced by three all-to-all-v
exchanges per minibatch over torch.distributed — RCCL over xGMI with the
"nccl" backend (device buffers, ordered on the library's HIP stream, no host
sync), gloo with host staging for CPU tests and several ranks sharing one GPU.

Per minibatch, every rank in lockstep:
  1. request    keys of its next batch, grouped by owner       (pull request)
  2. serve_pull owners look up rows of the keys they received  (pull response)
  3. step       install the pulled rows, learn, mean gradients (push request)
  4. serve_push owners apply AdaGrad once per source rank, in rank order
Key -> owner rank is BasicHashFrag (cluster/hashfrag.h:33-56) with S = world.
Per-(step, source, destination) key counts come from the static batch
schedules and are exchanged once, so no step needs a size handshake.
"""
import ctypes

import numpy as np
import torch
import torch.distributed as dist

from . import LR, Word2Vec, capi
from .capi import check, ptr


class Exchanger:
    """all-to-all-v of flat tensors among the ranks of a process group."""

    def __init__(self, group=None, device=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = dist.get_backend(group)
        self.device = device

    def a2a(self, send, send_counts, recv_counts, width=1):
        """send holds sum(send_counts)*width elements ordered by destination rank."""
        ss = [int(c) * width for c in send_counts]
        rs = [int(c) * width for c in recv_counts]
        if self.backend == "nccl":
            out = torch.empty(sum(rs), dtype=send.dtype, device=send.device)
            dist.all_to_all_single(out, send, rs, ss, group=self.group)
            return out
        out = torch.empty(sum(rs), dtype=send.dtype)
        dist.all_to_all_single(out, send.cpu(), rs, ss, group=self.group)
        if not send.is_cuda:
            return out
        out = out.to(send.device)
        torch.cuda.synchronize(send.device)  # the library reads it on its own stream
        return out

    def all_gather_matrix(self, mat):
        """[rows, world] int64 per rank -> [world(src), rows, world] on every rank."""
        t = torch.as_tensor(mat, dtype=torch.int64)
        if self.backend == "nccl":
            t = t.to(self.device)
        outs = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(outs, t, group=self.group)
        return torch.stack([o.cpu() for o in outs]).numpy()

    def max(self, x):
        t = torch.tensor([x], dtype=torch.int64, device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def min(self, x):
        return -self.max(-x)


def _write_json_atomic(path, obj):
    """<path>.tmp, fsync, rename over <path>, fsync the directory (a crash
    leaves the old file or the new one, never a torn one)."""
    import json
    import os
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)
    fd = os.open(os.path.dirname(os.path.abspath(path)), os.O_RDONLY)
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


class _ShardedApp:
    """Lockstep driver of a sharded app context (swps_<app>_request /
    serve_pull / step / serve_push).  Subclasses set the handle `self.h`,
    the C prefix `self.pfx`, the value width per key `self.width`, and the
    value / gradient tensor dtypes."""

    def _setup(self, table, group, frag_num):
        self.table = table
        self.dev = torch.device("cuda", table.device)
        self.ex = Exchanger(group, self.dev)
        self.rank, self.world = self.ex.rank, self.ex.world
        self.frag_num = frag_num
        self.cursor = 0
        self._ext = None
        self._xprof = None

    def _fn(self, name):
        return getattr(capi.lib(), "swps_%s_%s" % (self.pfx, name))

    def _shard(self, nb):
        check(self._fn("shard")(self.h, self.rank, self.world, self.frag_num))
        cnt = np.zeros(max(nb * self.world, 1), dtype=np.uint64)
        n = ctypes.c_uint64()
        check(self._fn("batch_counts")(self.h, ptr(cnt), len(cnt), ctypes.byref(n)))
        self.nb = nb
        self.steps_per_epoch = self.ex.max(nb)
        mat = np.zeros((self.steps_per_epoch, self.world), dtype=np.int64)
        mat[:nb] = cnt[:nb * self.world].reshape(nb, self.world).astype(np.int64)
        g = self.ex.all_gather_matrix(mat)  # [src][step][dst]
        self.send_counts = g[self.rank]                 # [step][dst]
        self.recv_counts = g[:, :, self.rank].T.copy()  # [step][src]

    def _cstream(self):
        """The library's compute stream as a torch stream."""
        if self._ext is None:
            self._ext = torch.cuda.ExternalStream(self._fn("stream")(self.h), device=self.dev)
        return self._ext

    def _a2a(self, stream, send, sc, rc, width):
        # RCCL (or gloo's host staging) ordered after / before the library's
        # kernels on `stream`
        with torch.cuda.stream(stream):
            if self._xprof is None:
                return self.ex.a2a(send, sc, rc, width)
            # exchange accounting (bench.py's xGMI roofline): bytes this rank
            # sends to other ranks, and the exchange's time on its stream
            es = send.element_size() * width
            remote = sum(int(c) for d, c in enumerate(sc) if d != self.rank) * es
            self._xprof["bytes_remote"] += remote
            self._xprof["bytes_total"] += int(sum(int(c) for c in sc)) * es
            self._xprof["calls"] += 1
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            out = self.ex.a2a(send, sc, rc, width)
            e1.record(stream)
            self._xprof["events"].append((e0, e1))
            return out

    def set_exchange_profile(self, on):
        """Count the bytes every all-to-all sends and time it with events on
        its stream (off: no events in the exchange path)."""
        self._xprof = {"bytes_remote": 0, "bytes_total": 0, "calls": 0, "events": [], "ms": 0.0} if on else None

    def exchange_stats(self):
        """{bytes_remote, bytes_total, calls, ms} since set_exchange_profile(True)."""
        if self._xprof is None:
            return None
        torch.cuda.synchronize(self.dev)
        x = self._xprof
        x["ms"] += sum(a.elapsed_time(b) for a, b in x["events"])
        x["events"] = []
        return {k: x[k] for k in ("bytes_remote", "bytes_total", "calls", "ms")}

    def _empty(self, stream, n, dtype):
        with torch.cuda.stream(stream):
            return torch.empty(n, dtype=dtype, device=self.dev)

    def full_pull(self):
        """Pull every key of the local data (the reference's first full pull)
        into the worker cache, inserting keys new to their owners."""
        C = self._cstream()
        counts = np.zeros(self.world, dtype=np.uint64)
        n = ctypes.c_uint64()
        check(self._fn("request")(self.h, 1, ptr(counts), None, ctypes.byref(n)))
        keys = self._empty(C, n.value, torch.int64)
        check(self._fn("request")(self.h, 1, ptr(counts), ptr(keys), ctypes.byref(n)))
        sc = counts.astype(np.int64)
        rc = self.ex.all_gather_matrix(sc[None, :])[:, 0, self.rank].copy()  # [src]
        rkeys = self._a2a(C, keys, sc, rc, 1)
        vals = self._empty(C, int(rc.sum()) * self.width, self.val_dtype)
        rcu = rc.astype(np.uint64)
        check(self._fn("serve_pull")(self.h, ptr(rkeys), ptr(rcu), 1, ptr(vals)))
        mine = self._a2a(C, vals, rc, sc, self.width)
        check(self._fn(self.install_fn)(self.h, ptr(mine)))
        check(self._fn("sync")(self.h))

    # -- the two halves of a minibatch's exchange ------------------------------
    def _pull_phase(self, s, S):
        """Request keys of step s, owners serve them, values back (on S)."""
        sc, rc = self.send_counts[s], self.recv_counts[s]
        nsend = int(sc.sum())
        keys = self._empty(S, nsend, torch.int64)
        if s < self.nb and nsend:
            counts = np.zeros(self.world, dtype=np.uint64)
            n = ctypes.c_uint64()
            check(self._fn("request")(self.h, 0, ptr(counts), ptr(keys), ctypes.byref(n)))
        rkeys = self._a2a(S, keys, sc, rc, 1)
        vals = self._empty(S, int(rc.sum()) * self.width, self.val_dtype)
        rcu = rc.astype(np.uint64)
        check(self._fn("serve_pull")(self.h, ptr(rkeys), ptr(rcu), 0, ptr(vals)))
        my_vals = self._a2a(S, vals, rc, sc, self.width)
        return my_vals, rkeys

    def _push_phase(self, s, grads, rkeys, S):
        """Mean gradients of step s to the owners, AdaGrad per source (on S)."""
        sc, rc = self.send_counts[s], self.recv_counts[s]
        rgrads = self._a2a(S, grads, sc, rc, self.width)
        rcu = rc.astype(np.uint64)
        check(self._fn("serve_push")(self.h, ptr(rkeys), ptr(rgrads), ptr(rcu)))

    def _learn(self, s, my_vals, stream):
        nsend = int(self.send_counts[s].sum())
        grads = self._empty(stream, nsend * self.width, self.grad_dtype)
        if s < self.nb:
            check(self._fn("step")(self.h, ptr(my_vals) if nsend else None, ptr(grads) if nsend else None))
        return grads

    def step(self):
        """One lockstep minibatch on every rank: pull, learn, push, in order
        (every pull sees every earlier push — the reference's semantics for
        one worker)."""
        C = self._cstream()
        s = self.cursor % self.steps_per_epoch
        my_vals, rkeys = self._pull_phase(s, C)
        grads = self._learn(s, my_vals, C)
        self._push_phase(s, grads, rkeys, C)
        self.cursor += 1

    def train_steps(self, n):
        for _ in range(n):
            self.step()

    train_batches = train_steps

    def sync(self):
        check(self._fn("sync")(self.h))
        torch.cuda.synchronize(self.dev)


class ShardedWord2Vec(_ShardedApp):
    """Word2Vec over key-sharded HBM tables on several GPUs (one per rank).

    The table passed in is this rank's shard (create it with init="hash":
    owners initialise keys on their first pull)."""

    pfx = "w2v"
    install_fn = "install_init"

    def __init__(self, table, group=None, frag_num=1000, pipeline=False, overlap=True, **kw):
        kw.setdefault("init", "table")
        self.w = Word2Vec(table, **kw)
        self.h = self.w.h
        self._setup(table, group, frag_num)
        self.D = table.dim
        self.width = 2 * self.D
        self.val_dtype = table.torch_dtype
        # push payload: fp64 (the reference's wire format) unless fast mode (fp32 table, fp32 intermediates)
        from . import INTERMEDIATES
        fast = table.dtype == "f32" and INTERMEDIATES[kw.get("fp64_intermediates", True)] == 0
        self.grad_dtype = torch.float32 if fast else torch.float64
        self.pipeline = pipeline
        self.overlap = overlap
        self._S = None
        self._next = None

    def step(self, prep_next=True):
        if self.pipeline:
            return self._step_pipelined()
        if self.overlap:
            return self._step_overlapped(prep_next)
        return super().step()

    def train_steps(self, n):
        for k in range(n):
            self.step(prep_next=k + 1 < n)

    train_batches = train_steps

    def _serve_stream(self):
        if self._S is None:
            self._S = torch.cuda.Stream(device=self.dev)
            self._S.wait_stream(self._cstream())  # after init's full pull
            check(capi.lib().swps_w2v_set_serve_stream(self.h, ctypes.c_void_p(self._S.cuda_stream)))
        return self._S

    def _step_overlapped(self, prep_next):
        """Lockstep minibatch (exact: every pull sees every earlier push) with
        the exchanges on a serve stream S, and the next minibatch's
        parameter-independent half (swps_w2v_prep: records, sort, index)
        issued on the compute stream C right after this one's learn — so it
        runs while this push and the next pull cross the fabric:

            S:  pull(i) ......... wait learn(i) -> push(i) -> pull(i+1) ...
            C:  wait pull(i) -> learn(i) -> prep(i+1) -> wait pull(i+1) -> ...
        """
        C, S = self._cstream(), self._serve_stream()
        s = self.cursor % self.steps_per_epoch
        my_vals, rkeys = self._pull_phase(s, S)
        C.wait_event(self._record(S))
        my_vals.record_stream(C)            # produced on S before the event
        grads = self._learn(s, my_vals, C)  # allocated on C, its first writer
        eg = self._record(C)
        nxt = (self.cursor + 1) % self.steps_per_epoch
        if prep_next and nxt < self.nb:
            check(capi.lib().swps_w2v_prep(self.h))
        S.wait_event(eg)
        grads.record_stream(S)
        self._push_phase(s, grads, rkeys, S)
        self.cursor += 1

    def _step_pipelined(self):
        """Bounded-staleness minibatch (overlap minibatch
        i+1's pull with step i).  The serve stream S runs the exchanges and the
        owners' serve kernels while the compute stream C learns:

            C:  learn(i) ------------------------------> learn(i+1) ...
            S:  pull(i+1) [sees pushes <= i-1] -> wait learn(i) -> push(i)

        so minibatch i+1 reads rows that lack only step i's updates (every
        rank's).  Deterministic: the order on each stream is fixed, and the
        prefetch is issued whatever the caller's chunking of steps."""
        C, S = self._cstream(), self._serve_stream()
        s = self.cursor % self.steps_per_epoch
        if self._next is None:  # prologue: nothing prefetched yet
            S.wait_stream(C)
            self._next = self._pull_phase(s, S) + (self._record(S),)
        my_vals, rkeys, ev = self._next
        C.wait_event(ev)
        my_vals.record_stream(C)            # produced on S before ev
        grads = self._learn(s, my_vals, C)  # allocated on C, its first writer
        eg = self._record(C)
        nvals, nkeys = self._pull_phase((self.cursor + 1) % self.steps_per_epoch, S)
        ev_next = self._record(S)           # learn(i+1) waits for the pull only
        S.wait_event(eg)
        grads.record_stream(S)
        self._push_phase(s, grads, rkeys, S)
        self._next = (nvals, nkeys, ev_next)
        self.cursor += 1

    @staticmethod
    def _record(stream):
        e = torch.cuda.Event()
        e.record(stream)
        return e

    # -- setup -----------------------------------------------------------------
    def load_text(self, path):
        self.w.load_text(path)
        self._shard(self.w.info()["batches"])

    def load_tokens(self, word_ids, line_off, word_keys):
        self.w.load_tokens(word_ids, line_off, word_keys)
        self._shard(self.w.info()["batches"])

    def init(self):
        """The first full pull (word2vec_global.h:557-562)."""
        self.full_pull()

    def train(self, niters=1):
        self.train_steps(niters * self.steps_per_epoch)
        self.sync()

    def stats(self):
        return self.w.stats()

    def kernel_times(self, reset=False):
        return self.w.kernel_times(reset)

    def info(self):
        return self.w.info()

    def set_profile(self, on):
        self.w.set_profile(on)

    def save(self, prefix):
        """Per-rank checkpoint <prefix>.rank<r>.{table,w2v,json}: this rank's
        shard, its worker state (tied to that shard file by its checksum) and
        the driver's step cursor, all tagged with one generation id; after
        every rank has written its files, rank 0 writes <prefix>.commit —
        a save without a commit marker (a crash mid-save) is never resumed;
        rank 0 removes the previous marker before any rank writes.
        Lockstep drivers only (a pipelined driver holds a prefetched pull that
        lacks the last push)."""
        import os
        if self._next is not None:
            raise capi.SwpsError(-6, "save: the pipelined driver holds a prefetched pull")
        self.sync()
        gen = self.ex.max(int.from_bytes(os.urandom(7), "little") if self.rank == 0 else 0)
        # an earlier save's marker must not vouch for files this save is about to replace: a crash
        # between a rank's new shard and its new .json would otherwise resume mixed generations
        if self.rank == 0 and os.path.exists(prefix + ".commit"):
            os.remove(prefix + ".commit")
        self.ex.max(0)  # barrier: no rank writes while the old marker exists
        base = "%s.rank%d" % (prefix, self.rank)
        self.w.save(base)
        _write_json_atomic(base + ".json", {"cursor": self.cursor, "world": self.world, "frag_num": self.frag_num,
                                            "generation": gen})
        self.ex.max(0)  # barrier: every rank's files are durable
        if self.rank == 0:
            _write_json_atomic(prefix + ".commit", {"generation": gen, "world": self.world, "cursor": self.cursor})
        self.ex.max(0)

    def restore(self, prefix):
        """Resume after load_text/load_tokens (instead of init).  Every rank
        must find the committed generation in its own files and all ranks the
        same cursor (mismatched counts would desynchronise the all-to-alls)."""
        import json
        import os
        base = "%s.rank%d" % (prefix, self.rank)
        if not os.path.exists(prefix + ".commit"):
            raise capi.SwpsError(-8, "no commit marker %s.commit: the save did not complete" % prefix)
        with open(prefix + ".commit") as f:
            commit = json.load(f)
        with open(base + ".json") as f:
            meta = json.load(f)
        if meta["world"] != self.world or meta["frag_num"] != self.frag_num or commit["world"] != self.world:
            raise capi.SwpsError(-5, "checkpoint of world %d / frag_num %d" % (meta["world"], meta["frag_num"]))
        if meta.get("generation") != commit["generation"]:
            raise capi.SwpsError(-5, "rank %d files belong to another save than %s.commit" % (self.rank, prefix))
        lo, hi = self.ex.min(meta["cursor"]), self.ex.max(meta["cursor"])
        if lo != hi or hi != commit["cursor"]:
            raise capi.SwpsError(-5, "ranks resume at different cursors (%d..%d, commit %d)" % (lo, hi,
                                                                                           commit["cursor"]))
        self.w.restore(base)
        self.cursor = meta["cursor"]

    def shard_rows(self):
        """(keys, rows [n][4D] fp64) of the keys this rank owns."""
        keys = self.table.keys()
        if len(keys) == 0:
            return keys, np.zeros((0, 4 * self.D))
        kt = torch.as_tensor(keys.astype(np.int64), device=self.dev)
        return keys, self.table.export(kt).double().cpu().numpy()


class ShardedLR(_ShardedApp):
    """Sparse LR over key-sharded HBM tables (BASELINE config 3): one fp32
    weight per feature key, owners apply AdaGrad per source rank in rank
    order (lr.cpp:58-81).  The table must be created with init="hash"."""

    pfx = "lr"
    install_fn = "install"
    width = 1
    val_dtype = torch.float32
    grad_dtype = torch.float32

    def __init__(self, table, group=None, frag_num=2000, minibatch=200, profile=False, fast_sums=False):
        self.m = LR(table, minibatch=minibatch, init_ref=False, profile=profile, fast_sums=fast_sums)
        self.h = self.m.h
        self._setup(table, group, frag_num)

    def load_text(self, path):
        self.m.load_text(path)
        self._shard(self.m.info()["batches"])

    def load_csr(self, labels, row_off, feat, vals):
        self.m.load_csr(labels, row_off, feat, vals)
        self._shard(self.m.info()["batches"])

    def init(self):
        """The first full pull of every local feature (lr.cpp:161-166)."""
        self.full_pull()

    def train(self, niters=1):
        """niters epochs in lockstep; per-epoch mean squared error of the
        local rows (lr.cpp:231)."""
        err = np.zeros(niters)
        for it in range(niters):
            self.train_steps(self.steps_per_epoch)
            e = ctypes.c_double()
            check(capi.lib().swps_lr_epoch_error(self.h, ctypes.byref(e)))
            err[it] = e.value
        self.sync()
        return err

    def predict(self):
        """Refresh the worker cache with a full pull, then predict the local rows."""
        self.full_pull()
        return self.m.predict()

    def info(self):
        return self.m.info()

    def kernel_times(self, reset=False):
        return self.m.kernel_times(reset)

    def set_profile(self, on):
        self.m.set_profile(on)

    def shard_weights(self):
        """(keys, w, g2) of the feature keys this rank owns, sorted by key."""
        keys = np.sort(self.table.keys())
        if len(keys) == 0:
            return keys, np.zeros(0, np.float32), np.zeros(0, np.float32)
        kt = torch.as_tensor(keys.astype(np.int64), device=self.dev)
        rows = self.table.export(kt).cpu().numpy().reshape(len(keys), 2)
        return keys, rows[:, 0].copy(), rows[:, 1].copy()


class NativeShardedWord2Vec:
    """The library-driven sharded loop (swps_w2v_shard_comm, src/swps_driver.cpp)
    behind ShardedWord2Vec's interface (what bench.py --driver native uses):
    the library issues the three all-to-all-v per minibatch itself over its
    own communicator — RCCL when every rank has its own GPU, its TCP
    transport when ranks share one."""

    def __init__(self, table, comm, frag_num=1000, **kw):
        kw.setdefault("init", "table")
        self.w = Word2Vec(table, **kw)
        self.table, self.comm, self.frag_num = table, comm, frag_num

    def load_tokens(self, word_ids, line_off, word_keys):
        self.w.load_tokens(word_ids, line_off, word_keys)
        self.w.shard_comm(self.comm, self.frag_num)

    def load_text(self, path):
        self.w.load_text(path)
        self.w.shard_comm(self.comm, self.frag_num)

    def init(self):
        self.w.init()

    def train_batches(self, n):
        self.w.train_batches(n)

    train_steps = train_batches

    def sync(self):
        self.w.sync()

    def stats(self):
        return self.w.stats()

    def info(self):
        return self.w.info()

    def kernel_times(self, reset=False):
        return self.w.kernel_times(reset)

    def set_profile(self, on):
        self.w.set_profile(on)

    def set_exchange_profile(self, on):
        self.w.exchange_stats(on=1 if on else 0)

    def exchange_stats(self):
        return self.w.exchange_stats()
