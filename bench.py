"""Headline benchmark: CBOW negative-sampling word2vec trained words/sec on a
synthetic text8-shaped corpus, D=300, table in one HBM shard per GPU
(BASELINE.json configs[1]).

A "step" is one reference minibatch: pull of the gathered key set, training of
`--minibatch` lines (learn_instance for every kept position), push of the mean
gradients with AdaGrad — all on the GPU through libswps.so.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

N > 1: every rank trains its own corpus of the same size (the reference's
per-rank local data) and serves the keys BasicHashFrag assigns to it; each
minibatch pulls rows from and pushes mean gradients to the owning GPUs with
RCCL all-to-all-v issued by the library itself (swps_w2v_shard_comm; its RCCL
id bootstrapped over TCP at MASTER_ADDR:MASTER_PORT+1), or with
--driver python by swiftmpi_amd/dist.py over torch.distributed.  Weak
scaling.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
XGMI_PEAK_GBS = 7 * 153.0  # per GPU: 7 xGMI links x ~153 GB/s


LR_TILE_CHUNK = int(os.environ.get("SWPS_LR_TILE_CHUNK", "1536"))  # swps_lr.hip kTileChunk (records per block)


def lr_tile_pieces(f, off, r0, r1, tile_bits=12, chunk=None):
    """The LR row-tile path's pieces and partials for batch rows [r0, r1): records ordered by
    (tile, key) (stable: row order inside), cut into blocks of `chunk` records per tile; a piece
    is a key's records inside one block, a partial a piece of a key with several
    (swps_lr.hip lr_tile_index)."""
    chunk = chunk or LR_TILE_CHUNK
    n = np.diff(off[r0:r1 + 1].astype(np.int64))
    tile = np.repeat((np.arange(r1 - r0) >> tile_bits), n)
    feat = f[off[r0]:off[r1]].astype(np.int64)
    o = np.lexsort((feat, tile))
    t, k = tile[o], feat[o]
    start = np.searchsorted(t, t, side="left")  # each tile's first sorted position
    blk = (np.arange(len(t)) - start) // chunk
    head = np.ones(len(t), dtype=bool)
    head[1:] = (t[1:] != t[:-1]) | (blk[1:] != blk[:-1]) | (k[1:] != k[:-1])
    pk = k[head]
    _, inv, cnt = np.unique(pk, return_inverse=True, return_counts=True)
    return int(head.sum()), int((cnt[inv] > 1).sum())


def pmc_traffic(config, groups):
    """HBM bytes per launch of kernel groups (one launch of each kernel per
    step), from the committed PMC summary of this exact workload
    (profiles/rNN_pmc_*.json, written by scripts/pmc_summary.py from separate
    rocprofv3 --pmc passes of the same command; read requests counted by size
    + WRITE_SIZE).  groups: name -> kernel base names (template arguments
    dropped).  Returns ({name: bytes or None}, source or None)."""
    import glob
    # the newest round's summaries first (profiles/rNN_pmc_<leg>.json)
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc_*.json")),
                       key=lambda q: (-int(os.path.basename(q)[1:3]), q)):
        try:
            prof = json.load(open(path))
        except (OSError, ValueError):
            continue
        if {k: prof.get("config", {}).get(k) for k in config} != config:
            continue
        res = {}
        for name, bases in groups.items():
            vals = [v["hbm_bytes"] for k, v in prof["kernels"].items()
                    if k.split("<")[0] in bases and v.get("hbm_bytes") is not None]
            res[name] = sum(vals) if vals else None
        src = "profiles/%s (32/64/128-B read requests + WRITE_SIZE per launch)" % os.path.basename(path)
        return res, src
    return {name: None for name in groups}, None


def make_corpus(tokens, vocab, line_len, seed):
    """Zipf(s=1) over `vocab` word ids, `tokens` tokens in lines of `line_len`
    (the synthetic text8 stand-in)."""
    from swiftmpi_amd.synth import zipf_tokens
    return zipf_tokens(tokens, vocab, line_len, seed, progress=tokens > (1 << 26))


def word_keys(lib, vocab):
    return np.array([lib.bkdr("w%d" % i) for i in range(vocab)], dtype=np.uint64)


_W2V_CPU_WORKER = r"""
import json, sys, time
sys.path.insert(0, sys.argv[1])
import oracle
path, dim, window, negative, minibatch, sample, alpha, lr = sys.argv[2:10]
m = oracle.W2V(path, int(dim), window=int(window), negative=int(negative), minibatch=int(minibatch),
               sample=float(sample), alpha=float(alpha), lr=float(lr), table_size=int(1e8))
m.init_rand(1, 2)
t0 = time.perf_counter()
m.train(1)
dt = time.perf_counter() - t0
print(json.dumps({"words": m.stats()["actual_train_words"], "dt": dt}))
"""


def cpu_baseline(ids, off, keys, args, lines):
    """The oracle (C++ port of the reference algorithm, fp64 like the
    reference, nthreads = 1 semantics) as `--cpu-procs` independent processes,
    one per host core, each on its own `lines`-line slice of the same corpus:
    the reference's MPI ranks each train their own file (apps/word2vec/
    README.md:37-46); the ranks' ZeroMQ parameter exchange is left out, so
    this is an upper bound on the reference's multi-core throughput.  Started
    as child processes (fresh interpreters), never forked from this GPU
    process."""
    import subprocess
    import oracle
    oracle.build()
    procs = max(1, args.cpu_procs)
    nl = len(off) - 1
    per = max(1, min(lines, nl // procs))
    with tempfile.TemporaryDirectory() as d:
        runs = []
        for r in range(procs):
            path = os.path.join(d, "sample%d.txt" % r)
            with open(path, "w") as f:
                for l in range(r * per, (r + 1) * per):
                    a, b = int(off[l]), int(off[l + 1])
                    f.write(" ".join("w%d" % x for x in ids[a:b]) + "\n")
            runs.append(path)
        env = dict(os.environ, OMP_NUM_THREADS="1")
        t0 = time.perf_counter()
        ps = [subprocess.Popen([sys.executable, "-c", _W2V_CPU_WORKER, ROOT, path, str(args.dim), str(args.window),
                                str(args.negative), str(args.minibatch), str(args.sample), str(args.alpha),
                                str(args.lr)], stdout=subprocess.PIPE, env=env) for path in runs]
        res = [json.loads(p.communicate()[0].decode().strip().splitlines()[-1]) for p in ps]
        wall = time.perf_counter() - t0
        if any(p.returncode for p in ps):
            raise RuntimeError("cpu baseline worker failed")
    words = sum(r["words"] for r in res)
    slowest = max(r["dt"] for r in res)
    return {"value": words / slowest, "unit": "words/s", "cores": procs, "kind": "port",
            "sample": "oracle/swps_oracle.cpp (fp64, nthreads=1 semantics) as %d concurrent processes, each on its "
                      "own %d-line slice (%d words in all) of the same corpus, 1 epoch, D=%d, no parameter "
                      "exchange between them; slowest process %.1f s (wall %.1f s incl. setup); single-process "
                      "rate %.3g words/s" % (procs, per, words, args.dim, slowest, wall,
                                               res[0]["words"] / res[0]["dt"])}


_W2V_MULTI_WORKER = r"""
import json, sys, time
sys.path.insert(0, sys.argv[1])
import oracle
paths = sys.argv[2].split(",")
dim, window, negative, minibatch, sample, alpha, lr = sys.argv[3:10]
m = oracle.W2VMulti(paths, int(dim), window=int(window), negative=int(negative), minibatch=int(minibatch),
                    sample=float(sample), alpha=float(alpha), lr=float(lr), table_size=int(1e8))
t0 = time.perf_counter()
m.train(1)
dt = time.perf_counter() - t0
print(json.dumps({"words": sum(m.rank_stats(r)["actual_train_words"] for r in range(len(paths))), "dt": dt}))
"""


def cpu_baseline_config1(ids, off, args, lines):
    """BASELINE config 1 on the CPU: 2 ranks, D = 100, minibatch 100 lines, in
    the oracle's lockstep multi-rank restatement (W2VMulti: each rank trains
    its own `lines`-line slice, pulls from and pushes to one key-sharded
    server state, every rank's push its own AdaGrad step in rank order — the
    exchange of apps/word2vec/cluster_run.sh:2 done in memory), one process,
    one core.  Child process (fresh interpreter), never forked from this GPU
    process."""
    import subprocess
    import oracle
    oracle.build()
    with tempfile.TemporaryDirectory() as d:
        paths = []
        for r in range(2):
            path = os.path.join(d, "rank%d.txt" % r)
            with open(path, "w") as f:
                for l in range(r * lines, (r + 1) * lines):
                    a, b = int(off[l]), int(off[l + 1])
                    f.write(" ".join("w%d" % x for x in ids[a:b]) + "\n")
            paths.append(path)
        env = dict(os.environ, OMP_NUM_THREADS="1")
        r = subprocess.run([sys.executable, "-c", _W2V_MULTI_WORKER, ROOT, ",".join(paths), "100", str(args.window),
                            str(args.negative), "100", str(args.sample), str(args.alpha), str(args.lr)],
                           capture_output=True, text=True, env=env)
        if r.returncode:
            raise RuntimeError("config-1 cpu worker failed: " + r.stderr[-2000:])
        res = json.loads(r.stdout.strip().splitlines()[-1])
    return {"value": res["words"] / res["dt"], "unit": "words/s", "cores": 1, "kind": "port",
            "sample": "oracle/swps_oracle.cpp W2VMulti (fp64, nthreads=1 semantics): 2 ranks in lockstep, each on its "
                      "own %d-line slice of the same corpus (%d words in all), D=100, minibatch 100, 1 epoch, one "
                      "process; %.1f s" % (lines, res["words"], res["dt"])}


def cpu_baseline_lr(y, off, f, v, minibatch, lr, rows):
    """The oracle's LR (lr.cpp semantics, nthreads = 1, fp32) on the first
    `rows` rows of the same synthetic Criteo-shaped data, one epoch (the rows
    handed over as arrays: the parse is not part of the timed training)."""
    import oracle
    oracle.build()
    rows = min(rows, len(y))
    n = int(off[rows])
    m = oracle.LR.from_csr(y[:rows], off[:rows + 1], f[:n], v[:n], minibatch=minibatch, lr=lr)
    t0 = time.perf_counter()
    m.train(1)
    dt = time.perf_counter() - t0
    return {"value": rows / dt, "unit": "examples/s", "cores": 1, "kind": "port",
            "sample": "oracle/swps_oracle.cpp LR (fp32, nthreads=1 semantics) on the first %d rows (%d features) "
                      "of the same data, minibatch %d, 1 epoch; %.1f s" % (rows, n, minibatch, dt)}


def cpu_baseline_s2v(toks, off, args, docs):
    """The oracle's sent2vec (sent2vec.cpp on word2vec.h's MiniBatch,
    nthreads = 1, fp64) on the first `docs` documents, word vectors for their
    vocabulary in the reference's dump format."""
    import oracle
    oracle.build()
    docs = min(docs, len(off) - 1)
    n = int(off[docs])
    words = np.unique(toks[:n])
    rng = np.random.default_rng(11)
    with tempfile.TemporaryDirectory() as d:
        cpath, wpath = os.path.join(d, "docs.txt"), os.path.join(d, "words.txt")
        with open(cpath, "w") as fh:
            for i in range(docs):
                fh.write(" ".join(str(int(x)) for x in toks[int(off[i]):int(off[i + 1])]) + "\n")
        # values (U(-0.5,0.5)/D, the reference's init scale) from a pool of 4096 fixed-width
        # strings so the dump of ~1e5 words x 2D values is written in seconds
        pool = np.array([b"% .6f " % x for x in (rng.random(4096) - 0.5) / args.dim], dtype="S10")
        body = pool[rng.integers(0, 4096, (len(words), 2 * args.dim))].view(np.uint8).reshape(len(words), -1).copy()
        body[:, 10 * args.dim - 1] = ord("\t")
        body[:, -1] = ord("\n")
        with open(wpath, "wb") as fh:
            for k, row in zip(words, body):
                fh.write(b"%d\t" % int(k) + row.tobytes())
        m = oracle.S2V(cpath, args.dim, window=args.window, negative=args.negative, minibatch=args.s2v_docs,
                       niters=1, alpha=args.alpha)
        m.load_words(wpath)
        t0 = time.perf_counter()
        m.train()
        dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "words/s", "cores": 1, "kind": "port",
            "sample": "oracle/swps_oracle.cpp sent2vec (fp64, nthreads=1 semantics) on the first %d docs (%d words) "
                      "of the same corpus, word vectors for their %d distinct words; %.1f s"
                      % (docs, n, len(words), dt)}


MODE_DESC = {"parity": "fp64 neu1/neu1e + gradient partials (reference-parity mode)",
             "bfp40": "block-fp neu1/neu1e, int32 + int8 mantissas per row exponent, fp64 sums (5 B/element)",
             "bfp32": "block-fp neu1/neu1e, int32 mantissas per row exponent, fp64 sums (4 B/element)",
             "fast": "fp32 neu1/neu1e + partials (fast mode: outside the 1e-5 single-batch bar)"}
INTER = {"bfp40": "bfp40", "bfp32": "bfp32", "fast": False, "parity": True}

# ---- per-rank deadline, phases and fault injection ---------------------------------------------
# A rank that waits on a lost or stuck peer must not hang the job until the driver's own timeout:
# the library's RCCL guard aborts a communicator whose exchange does not retire in
# SWPS_COMM_TIMEOUT_S (include/swps.h), torch.distributed's barriers get the same timeout, and
# every rank arms an overall deadline (SWPS_BENCH_DEADLINE_S) that ends the process with rc 124
# naming the phase it was in.  SWPS_BENCH_FAULT=<rank>:<phase> makes that rank kill itself
# (SIGKILL) when it enters the phase: the test of those paths (tests/test_bench_gpu.py).
_PHASE = {"name": "start", "rank": 0}


def set_phase(name):
    _PHASE["name"] = name
    f = os.environ.get("SWPS_BENCH_FAULT")
    if f and f.split(":")[0] == str(_PHASE["rank"]) and f.split(":", 1)[1] == name:
        import signal
        print("bench.py: rank %d: SWPS_BENCH_FAULT: killed entering phase %s" % (_PHASE["rank"], name),
              file=sys.stderr, flush=True)
        os.kill(os.getpid(), signal.SIGKILL)


def arm_deadline(rank):
    import threading
    _PHASE["rank"] = rank
    limit = float(os.environ.get("SWPS_BENCH_DEADLINE_S", "1500"))

    def expire():
        print("bench.py: rank %d: deadline of %g s exceeded in phase %s; exiting" % (rank, limit, _PHASE["name"]),
              file=sys.stderr, flush=True)
        os._exit(124)
    t = threading.Timer(limit, expire)
    t.daemon = True
    t.start()


def comm_timeout_s():
    return float(os.environ.get("SWPS_COMM_TIMEOUT_S", "120"))


class Ctx:
    """One process per GPU: rank / world / device, torch.distributed (for the bench's own
    barrier and max-over-ranks timing) and the library's communicator, made once and shared by
    every sharded leg (RCCL when each rank has its own GPU, the library's TCP transport when
    ranks share one)."""

    def __init__(self, sharded):
        import torch
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        ngpu = torch.cuda.device_count()
        self.local = int(os.environ.get("LOCAL_RANK", "0")) % max(ngpu, 1)
        torch.cuda.set_device(self.local)
        self.dist, self.backend, self._comm, self._ipc = None, None, [], None
        self.exchange = os.environ.get("SWPS_BENCH_EXCHANGE", "auto")  # main() sets --exchange
        self.sharded = self.world > 1 or sharded
        if self.sharded:
            import datetime
            import torch.distributed as dist
            self.dist = dist
            if "MASTER_ADDR" not in os.environ:
                os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", RANK="0", WORLD_SIZE="1")
            to = datetime.timedelta(seconds=comm_timeout_s())
            if ngpu >= self.world:  # one GPU per rank: RCCL over xGMI
                self.backend = "nccl"
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local), timeout=to)
            else:                    # functional check with ranks sharing a GPU
                self.backend = "gloo"
                dist.init_process_group("gloo", timeout=to)

    def tuple(self):
        return (self.rank, self.world, self.local, self.dist, self.backend)

    def barrier(self):
        import torch
        torch.cuda.synchronize()
        if self.dist is not None:
            self.dist.barrier()

    def comm(self):
        """The library's communicator (None if it could not be made on every rank)."""
        if not self._comm and self.dist is not None:
            import torch
            from swiftmpi_amd.comm import Comm
            port = int(os.environ.get("MASTER_PORT", "29533")) + 1
            addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
            set_phase("communicator")
            try:
                c = (Comm.rccl(self.rank, self.world, self.local, addr=addr, port=port)
                     if self.backend == "nccl" else Comm.tcp(self.rank, self.world, self.local, addr=addr, port=port))
                ok = 1
            except Exception as e:  # noqa: BLE001 — reported, and every rank falls back together
                print("native communicator failed on rank %d: %s" % (self.rank, e), file=sys.stderr, flush=True)
                c, ok = None, 0
            t = torch.tensor([ok], dtype=torch.int32, device="cuda")
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
            self._comm.append(c if int(t.item()) else None)
        return self._comm[0] if self._comm else None

    def transport(self):
        c = self._comm[0] if self._comm else None
        return c.transport() if c is not None else None

    def close(self):
        """Every rank at the same point: the IPC communicator's teardown is collective (peers store
        into this rank's inboxes until their last exchange retires)."""
        c = getattr(self, "_ipc_made", None)
        if c is not None:
            c.close()
        self._ipc, self._ipc_made = [None], None

    def ipc_comm(self):
        """A second library communicator whose exchanges run device to device through IPC-mapped
        peer inboxes (swps_comm_enable_ipc), for the latency-bound LR leg.  A canary exchange
        (segments of 1 KiB to 2.5 inbox slots, every byte checked on the device) must come out
        exact on every rank, within a 30-s deadline; otherwise every rank falls back to comm()
        together.  None at world 1 or when --exchange base."""
        if self._ipc is None:
            self._ipc = [None]
            if self.dist is not None and 1 < self.world <= 8 and self.exchange != "base":
                import torch
                from swiftmpi_amd.comm import Comm
                port = int(os.environ.get("MASTER_PORT", "29533")) + 3
                addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
                set_phase("ipc communicator")
                c, ok = None, 0
                try:
                    c = (Comm.rccl(self.rank, self.world, self.local, addr=addr, port=port)
                         if self.backend == "nccl" else Comm.tcp(self.rank, self.world, self.local, addr=addr, port=port))
                    c.set_timeout(min(30.0, comm_timeout_s()))
                    c.enable_ipc()
                    ok, report = c.canary()
                    ok = int(ok)
                    for rec in report:  # where the first wrong byte of each peer's segment came in
                        print("IPC canary mismatch: %s" % json.dumps(rec), file=sys.stderr, flush=True)
                    c.set_timeout(comm_timeout_s())
                except Exception as e:  # noqa: BLE001 — reported; every rank falls back together
                    print("IPC exchange unavailable on rank %d: %s" % (self.rank, e), file=sys.stderr, flush=True)
                    ok = 0
                t = torch.tensor([ok], dtype=torch.int32, device="cuda")
                self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
                self._ipc_made = c  # closed by close() on every rank at once (its teardown is collective)
                if int(t.item()):
                    self._ipc = [c]
                else:
                    print("rank %d: IPC canary failed somewhere; LR exchanges stay on the base transport"
                          % self.rank, file=sys.stderr, flush=True)
        return self._ipc[0]

    def max_sum(self, dt, units):
        """(max over ranks of dt, sum over ranks of units)."""
        if self.dist is None:
            return dt, float(units)
        import torch
        tt = torch.tensor([dt, float(units)], dtype=torch.float64, device="cuda")
        mx = tt.clone()
        self.dist.all_reduce(mx, op=self.dist.ReduceOp.MAX)
        self.dist.all_reduce(tt, op=self.dist.ReduceOp.SUM)
        return float(mx[0]), float(tt[1])


def exchange_block(xs, steps, step_s, world, note):
    """xGMI accounting of a sharded leg: bytes this rank sent to other ranks per step, over the
    exchanges' event time on their stream (profiled pass), against 7 links x 153 GB/s."""
    if xs is None:
        return None
    xg = xs["bytes_remote"] / (xs["ms"] * 1e-3) / 1e9 if xs["ms"] > 0 else 0.0
    return {"bytes_remote_per_step": xs["bytes_remote"] / steps, "bytes_total_per_step": xs["bytes_total"] / steps,
            "a2a_per_step": xs["calls"] / steps, "ms_per_step": xs["ms"] / steps,
            "share_of_step": xs["ms"] / (step_s * 1e3) if step_s > 0 else None,
            "GBps": xg, "peak": XGMI_PEAK_GBS, "frac": xg / XGMI_PEAK_GBS, "world": world, "note": note}


def w2v_leg(sw, ctx, args, ids, off, keys, prec, minibatch, dim, frag_num, steps, warmup, tokens, vocab,
            profile=True, setup_s=None):
    """Build a CBOW-NS context on this rank's corpus (key-sharded over ctx's communicator when
    ctx.sharded, else one HBM shard), warm up, time `steps` minibatches (barrier + sync on both
    sides, max over ranks), then a second, profiled pass for the per-kernel roofline.  Returns
    the leg's raw measurements."""
    kw = dict(window=args.window, negative=args.negative, minibatch=minibatch, sample=args.sample, alpha=args.alpha,
              profile=False, fp64_intermediates=INTER[prec], sampler=args.sampler)
    t = sw.Table("w2v", dim=dim, capacity=vocab, dtype=args.dtype, learning_rate=args.lr, device=ctx.local,
                 init="hash", seed=1)
    comm = ctx.comm() if ctx.sharded and args.driver == "native" else None
    if comm is not None and cbow_ipc(ctx, args):
        comm = ctx.ipc_comm()  # opt-in: the CBOW legs' exchanges through the IPC path too
    if comm is not None:  # the library's own exchange
        from swiftmpi_amd.dist import NativeShardedWord2Vec
        w = NativeShardedWord2Vec(t, comm, frag_num=frag_num, **kw)
    elif ctx.sharded:     # key-sharded over the ranks (BasicHashFrag), all-to-all per minibatch
        from swiftmpi_amd.dist import ShardedWord2Vec
        w = ShardedWord2Vec(t, frag_num=frag_num, pipeline=ctx.sharded and args.pipeline, **kw)
    else:
        w = sw.Word2Vec(t, init="ref", **kw)
    t0 = time.perf_counter()
    w.load_tokens(ids, off, keys)
    t1 = time.perf_counter()
    w.init()
    if setup_s is not None:
        setup_s.update(ingest=t1 - t0, first_pull=time.perf_counter() - t1)
    info = w.info()
    w.train_batches(warmup)
    w.sync()

    def timed(n):
        s0 = w.stats()
        ctx.barrier()
        a = time.perf_counter()
        w.train_batches(n)
        w.sync()
        ctx.barrier()
        dt = time.perf_counter() - a
        s1 = w.stats()
        return dt, {k: s1[k] - s0[k] for k in s1 if k not in ("lstate", "fstate")}

    dt, d = timed(steps)                    # the measured region: no event timing inside
    res = {"dt": dt, "d": d, "info": info, "steps": steps, "warmup": warmup}
    if profile:
        w.set_profile(True)                 # a second, profiled pass for the per-kernel roofline
        w.kernel_times(reset=True)
        gw = getattr(w, "w", w)             # the per-rank Word2Vec (sharded: its learner)
        g0 = gw.sum_stats()
        if ctx.sharded:
            w.set_exchange_profile(True)
        dpt, dp = timed(steps)
        res.update(dpt=dpt, dp=dp, kt=w.kernel_times(), g0=g0, g1=gw.sum_stats(),
                   xs=w.exchange_stats() if ctx.sharded else None)
        w.set_profile(False)
        if ctx.sharded:
            w.set_exchange_profile(False)
    del w
    t.close()
    return res


def w2v_roofline(r, args, prec, minibatch, dim, tokens, vocab, world, sharded):
    """Roofline of the dominant kernel group of a w2v leg (the segmented gradient sums + fused
    push), its PMC traffic from the committed passes of the same workload, the
    forward's PMC rate and the whole step's §8(d) bytes."""
    D, es = dim, (8 if args.dtype == "f64" else 4)
    parity_main = prec == "parity"
    bfp_main = prec.startswith("bfp") and args.dtype == "f32"
    rb = 1 if prec == "bfp40" else 0
    ea = 8 if (parity_main or args.dtype == "f64") else 4   # neu1/neu1e element size
    # BFP modes: a record reads its position's mantissas (4 B, + the int8 residual in bfp40) per
    # element and the row scale (4 B); partials and the mean-gradient payload are fp64
    rec_row = D * (4 + rb) + 4 if bfp_main else D * ea
    pa = 8 if bfp_main else ea
    d, dp, kt, g0, g1 = r["d"], r["dp"], r["kt"], r["g0"], r["g1"]
    dt = r["dt"]
    # SURVEY.md §8(d) algorithmic bytes of k_forward: every context/target row occurrence read
    # (4·D per row in fp32) + neu1, neu1e written per position
    fwd_ms, fwd_n = kt["forward"]
    fwd_bytes = es * D * (dp["ctx_rows"] + dp["tgt_rows"]) + 2 * rec_row * dp["kept"]
    fwd_gbs = fwd_bytes / (fwd_ms * 1e-3) / 1e9 if fwd_ms > 0 else 0.0
    # the dominant kernel by time: the segmented gradient sums + AdaGrad push.  Each gradient
    # record reads its source row (neu1 or neu1e of its position) and its 4-B record index; each
    # item (chunk of <= 128 records of one key) that goes through a partial writes it (+ a 16-B
    # descriptor) and the push reads it back; each pushed key reads h,v,h2,v2 (4·D·es), writes
    # them (4·D·es) and its pre-update h,v to the worker cache (2·D·es) + 8 B of bounds.
    g_rec, g_items = g1["records"] - g0["records"], g1["items"] - g0["items"]
    g_mitems = g1["multi_items"] - g0["multi_items"]
    nbat = g1["batches"] - g0["batches"]
    fused = nbat > 0 and g1["fused"] - g0["fused"] == nbat
    fused_g = nbat > 0 and g1.get("fused_grads", 0) - g0.get("fused_grads", 0) == nbat
    # small batches run the multi-chunk gather on a side stream beside the push: the push timer
    # then spans the whole group
    split = nbat > 0 and g1.get("split", 0) - g0.get("split", 0) == nbat
    gat_ms, gat_n = kt["gather"]
    push_ms, push_n = kt.get("push", (0.0, 0))
    kn = ("k_gather_b", "k_combine_b", "k_push_b") if bfp_main else ("k_gather_t", "k_combine", "k_push_thp")
    if fused_g:  # sharded learner: the fused push stops at the mean gradients (2·D·pa written per key)
        sum_kernel = "%s + %s + %s<TO_GRADS> (segmented gradient sums + fused mean gradients of the push payload)" % kn
        gat_bytes = g_rec * (rec_row + 4) + g_mitems * (2 * D * pa + 16) + dp["pushed"] * (2 * D * pa + 8)
        sum_ms = push_ms if split else gat_ms + push_ms
    elif fused:
        sum_kernel = "%s + %s + %s (segmented gradient sums + fused AdaGrad push)" % kn
        gat_bytes = g_rec * (rec_row + 4) + g_mitems * (2 * D * pa + 16) + dp["pushed"] * (10 * es * D + 8)
        sum_ms = push_ms if split else gat_ms + push_ms
    else:
        sum_kernel = ("k_gather + k_combine" if (parity_main or args.dtype == "f64") else "k_gather_t + k_combine") + \
            " (segmented gradient sums)"
        gat_bytes = g_rec * (D * ea + 4) + g_items * (D * ea + 16)
        sum_ms = gat_ms
    gat_gbs = gat_bytes / (sum_ms * 1e-3) / 1e9 if sum_ms > 0 else 0.0
    # whole step (§8(d) full formula): rows read + gradients written + pull 16D/key + push (40D+8)/key
    step_bytes = (2 * es * D * (dp["ctx_rows"] + dp["tgt_rows"]) + d["pulled"] * 4 * es * D +
                  d["pushed"] * (10 * es * D + 8))
    step_gbs = step_bytes / dt / 1e9
    # the metric's "sparse push/pull HBM GB/s".  Single GPU: the pull is no kernel of its own —
    # the forward reads the batch's keys straight from the table rows (counted in
    # roofline.forward) and the push leaves their pre-update h, v in the worker cache
    pp = {}
    for name, nbytes in (("pull", dp["pulled"] * 4 * es * D), ("push", dp["pushed"] * (12 * es * D + 8))):
        ms, n = kt.get(name, (0.0, 0))
        if ms > 0 and not sharded and not ((fused or fused_g) and name == "push"):
            gbs = nbytes / (ms * 1e-3) / 1e9
            pp[name] = {"GBps": gbs, "frac": gbs / HBM_PEAK_GBS, "bytes_per_launch": nbytes / max(n, 1),
                        "avg_launch_ms": ms / max(n, 1)}
    if not sharded and "pull" not in pp:
        pp["pull"] = "fused: k_forward reads the pulled keys' table rows directly; k_push writes their cache rows"
    # HBM traffic of the same kernels from the committed PMC passes of this exact workload
    # (scripts/gpu_profile.sh -> scripts/pmc_summary.py); null otherwise
    mine = dict(app="w2v", minibatch=minibatch, dim=dim, dtype=args.dtype, mode=prec, world=world, tokens=tokens,
                vocab=vocab, line_len=args.line_len, sharded=bool(sharded), sampler=args.sampler)
    if bfp_main:
        grp = ("k_gather_b", "k_combine_b", "k_push_b")
    elif parity_main or args.dtype == "f64":
        grp = ("k_gather", "k_combine") + (("k_push_thp", "k_push_tg") if (fused or fused_g) else ())
    else:
        grp = ("k_gather_t", "k_combine") + (("k_push_thp", "k_push_tg") if (fused or fused_g) else ())
    tr, traffic_src = pmc_traffic(mine, {"sum": grp, "forward": ("k_forward_t", "k_forward_b", "k_forward_b8",
                                                                  "k_forward")})
    fwd_traffic = tr["forward"]
    return {"bound": "hbm", "kernel": sum_kernel, "achieved": gat_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": gat_gbs / HBM_PEAK_GBS, "traffic": tr["sum"], "traffic_source": traffic_src,
            "bytes_per_launch": gat_bytes / max(gat_n, 1), "avg_launch_ms": sum_ms / max(gat_n, 1),
            "launches": gat_n, "records_per_launch": g_rec / max(gat_n, 1),
            "items_per_launch": g_items / max(gat_n, 1),
            "partial_items_per_launch": (g_mitems if fused else g_items) / max(gat_n, 1),
            "gather_ms_per_launch": gat_ms / max(gat_n, 1), "push_ms_per_launch": push_ms / max(push_n, 1),
            # k_forward: its row-occurrence bytes count every context/target row read, most of them
            # L2 / Infinity-Cache hits (hot Zipf rows), so they are no roofline quantity
            # (row_bytes_GBps); its roofline fraction is the PMC-measured memory-side traffic of the
            # same launches over their time
            "forward": {"kernel": "k_forward_b" if bfp_main else "k_forward_t",
                        "row_bytes_GBps": fwd_gbs, "row_bytes_per_launch": fwd_bytes / max(fwd_n, 1),
                        "avg_launch_ms": fwd_ms / max(fwd_n, 1), "launches": fwd_n, "traffic": fwd_traffic,
                        "hbm_GBps": (fwd_traffic / (fwd_ms / max(fwd_n, 1) * 1e-3) / 1e9
                                     if fwd_traffic and fwd_ms > 0 else None),
                        "frac": (fwd_traffic / (fwd_ms / max(fwd_n, 1) * 1e-3) / 1e9 / HBM_PEAK_GBS
                                 if fwd_traffic and fwd_ms > 0 else None)},
            "step_GBps": step_gbs, "step_frac": step_gbs / HBM_PEAK_GBS, "pull_push": pp or None}


def parallelism(ctx, args, frag_num):
    if not ctx.sharded:
        return "1 GPU, one HBM shard"
    tr = ctx.transport()
    via = (("library-issued RCCL" if tr[0] == "rccl" else "library TCP transport") if tr is not None and
           args.driver == "native" else ("RCCL" if ctx.backend == "nccl" else "gloo"))
    return ("key-sharded PS over %d GPU(s) (BasicHashFrag frag_num %d), %s all-to-all-v, %s"
            % (ctx.world, frag_num, via, "pipelined: pull(i+1)/push(i) overlap learn(i), staleness 1"
               if args.pipeline else "lockstep pull/learn/push"))


def with_transport(out, ctx, ipc=False):
    tr = ctx.transport()
    if tr is not None:  # the library's own communicator: what its transport reports
        out["transport"] = tr[0] + ("+ipc" if ipc else "")
        out["rccl_ranks" if tr[0] == "rccl" else "transport_ranks"] = tr[1]
    return out


def cbow_ipc(ctx, args):
    """--exchange ipc-all: the CBOW legs' exchanges go through the IPC communicator."""
    return (ctx.sharded and args.driver == "native" and args.exchange == "ipc-all" and ctx.dist is not None
            and ctx.ipc_comm() is not None)


def config4_leg(sw, ctx, args):
    """BASELINE config 4 as weak scaling: each rank trains its own 1e9/8-token share (125M
    tokens, Zipf over V = 1M, 1000-token lines, seed 4 + rank), D = 300, W = N = 5, minibatch
    5000 lines, keys hash-sharded over the ranks with frag_num 8000 — at N = 8 the job is
    config 4's whole 1e9-token corpus; at N = 1 the same per-rank workload on one HBM shard."""
    set_phase("config4")
    tokens, vocab = args.config4_tokens, 1000000
    ids, off = make_corpus(tokens, vocab, args.line_len, seed=4 + ctx.rank)
    import swiftmpi_amd as sw_
    keys = word_keys(sw_, vocab)
    setup_s = {}
    r = w2v_leg(sw, ctx, args, ids, off, keys, args.precision, args.minibatch, 300, 8000, args.config4_steps, 3,
                tokens, vocab, setup_s=setup_s)
    del ids, off
    dt, total = ctx.max_sum(r["dt"], r["d"]["words"])
    roof = w2v_roofline(r, args, args.precision, args.minibatch, 300, tokens, vocab, ctx.world, ctx.sharded)
    out = {"metric": "SGNS trained words/sec (BASELINE config 4: Zipf V=1M, D=300, 1e9 tokens over 8 GPUs)",
           "value": total / dt, "unit": "words/s", "n_gpus": ctx.world, "steps": r["steps"], "warmup": r["warmup"],
           "ms_per_step": dt * 1e3 / r["steps"], "higher_is_better": True, "scaling": "weak",
           "config": {"workload": "word2vec CBOW-NS, per rank %d tokens (1e9/8: config 4's per-GPU share) of Zipf(s=1) "
                                  "over V=%d, dim 300, window %d, negative %d, sample %g, minibatch %d lines of %d "
                                  "tokens; %d tokens over all ranks"
                                  % (tokens, vocab, args.window, args.negative, args.sample, args.minibatch,
                                     args.line_len, tokens * ctx.world),
                      "parallelism": parallelism(ctx, args, 8000), "mode": args.precision,
                      "vocab_per_rank": r["info"]["vocab"], "batches_per_epoch": r["info"]["batches"],
                      "kept_positions_per_s": r["d"]["kept"] * ctx.world / dt,
                      "pulled_keys_per_step": r["d"]["pulled"] / r["steps"], "setup_s": setup_s},
           "roofline": roof,
           "exchange": exchange_block(r.get("xs"), r["steps"], r.get("dpt", 0.0), ctx.world,
                                      "remote bytes (keys 8 B, rows 2*D*4 B, grads 2*D*8 B per remote key) / "
                                      "all-to-all time (events on the exchange stream, profiled pass)")}
    return with_transport(out, ctx, cbow_ipc(ctx, args))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--cpu-procs", type=int, default=8,
                    help="concurrent single-threaded oracle processes for the w2v cpu_baseline (host cores used)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dim", type=int, default=300)
    ap.add_argument("--window", type=int, default=5)
    ap.add_argument("--negative", type=int, default=5)
    ap.add_argument("--sample", type=float, default=1e-5)
    ap.add_argument("--alpha", type=float, default=0.05)
    ap.add_argument("--lr", type=float, default=0.7)
    ap.add_argument("--minibatch", type=int, default=5000,
                    help="worker.minibatch in lines (the reference demo: apps/word2vec/demo.conf:11)")
    ap.add_argument("--tokens", type=int, default=17005207)
    ap.add_argument("--vocab", type=int, default=253854)
    ap.add_argument("--line-len", type=int, default=1000)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--frag-num", type=int, default=1000)
    ap.add_argument("--sharded", action="store_true", help="use the key-sharded multi-GPU path even at N=1")
    ap.add_argument("--driver", default="native", choices=["python", "native"],
                    help="sharded exchange: swiftmpi_amd/dist.py over torch.distributed, or the library's own "
                         "(swps_w2v_shard_comm over RCCL / its TCP transport)")
    ap.add_argument("--exchange", default="auto", choices=["auto", "base", "ipc-all"],
                    help="N > 1 LR leg: auto = the device-initiated IPC exchange (swps_comm_enable_ipc) when its "
                         "canary passes on every rank, else the base transport; base = RCCL / TCP only; ipc-all = "
                         "the CBOW legs (headline, config 4) through it too (opt-in: unmeasured against RCCL at N = 8)")
    ap.add_argument("--pipeline", action="store_true",
                    help="sharded path: the bounded-staleness driver (pull(i+1)/push(i) overlap learn(i)) instead "
                         "of the default lockstep pull/learn/push order (exact reference semantics)")
    ap.add_argument("--cpu-lines", type=int, default=2500)
    ap.add_argument("--cpu-rows", type=int, default=1000000, help="LR CPU baseline sample (rows)")
    ap.add_argument("--cpu-docs", type=int, default=3000, help="sent2vec CPU baseline sample (documents)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--precision", default="bfp32", choices=["bfp40", "bfp32", "fast", "parity"],
                    help="fp32-table intermediates: bfp32 (block-floating-point neu1/neu1e, int32 mantissas per "
                         "row exponent, fp64 sums and mean: within the north star's 1e-5 single-batch bar at fp32's "
                         "4 B per element; the default), bfp40 (+ an int8 residual: 1e-5 after two batches too), "
                         "fast (fp32), parity (fp64)")
    ap.add_argument("--parity", action="store_true", help="= --precision parity")
    ap.add_argument("--no-parity-leg", action="store_true",
                    help="skip the extra parity- and fast-mode timings reported beside the headline")
    ap.add_argument("--b100-steps", type=int, default=200,
                    help="minibatches of the extra B = 100 leg (SURVEY.md §8(d) config 1's minibatch); 0 = skip")
    ap.add_argument("--config1-steps", type=int, default=200,
                    help="minibatches of the BASELINE config-1 leg (D = 100, minibatch 100) on the GPU; 0 = skip")
    ap.add_argument("--config1-cpu-lines", type=int, default=600,
                    help="lines per rank of the config-1 CPU leg (2 ranks in lockstep, oracle W2VMulti)")
    ap.add_argument("--config4-tokens", type=int, default=125000000,
                    help="tokens per rank of the config-4 leg (1e9 / 8: config 4's per-GPU share); 0 = skip the leg")
    ap.add_argument("--config4-steps", type=int, default=10, help="timed minibatches of the config-4 leg")
    ap.add_argument("--sampler", default="table", choices=["table", "alias"],
                    help="negative sampler: the reference's unigram table (bit-exact draws) or an alias table")
    ap.add_argument("--app", default="w2v", choices=["w2v", "lr", "s2v"],
                    help="w2v: the headline (config 2); lr: config 3 shape; s2v: config 5 shape")
    ap.add_argument("--lr-batch", type=int, default=65536, help="LR rows per GPU per minibatch (config 3)")
    ap.add_argument("--lr-plan", default="none", choices=["step", "load", "none"],
                    help="LR: none = the fixed-point step (no per-minibatch index: each step groups its "
                         "minibatch's keys itself, as the reference gathers per minibatch, lr.cpp:215-227); "
                         "step = a sorted index per minibatch built beside the previous step; load = every "
                         "minibatch's sorted index built once at load")
    ap.add_argument("--lr-exact", action="store_true",
                    help="LR: the reference's sequential fp32 per-key sums (bit-exact) instead of fast fp64 sums")
    ap.add_argument("--s2v-docs", type=int, default=8192, help="sent2vec documents per minibatch")
    ap.add_argument("--no-lr-sharded-base", action="store_true",
                    help="skip the lr leg's world-1 sharded base point (lr.sharded_world1) at N = 1")
    ap.add_argument("--no-app-legs", action="store_true",
                    help="skip the config-4, LR (config 3) and sent2vec (config 5) legs of the default line")
    ap.add_argument("--app-steps", type=int, default=20, help="timed LR minibatches of the default line's lr leg")
    args = ap.parse_args()
    os.environ["SWPS_BENCH_EXCHANGE"] = args.exchange  # read by Ctx (the LR leg's IPC communicator)
    if args.parity:
        args.precision = "parity"
    arm_deadline(int(os.environ.get("RANK", "0")))
    if args.app != "w2v":
        return bench_other(args)

    import swiftmpi_amd as sw
    set_phase("init")
    ctx = Ctx(args.sharded)
    rank, world = ctx.rank, ctx.world

    set_phase("headline")
    ids, off = make_corpus(args.tokens, args.vocab, args.line_len, seed=8 + rank)
    print("corpus: %d tokens" % len(ids), file=sys.stderr, flush=True)
    keys = word_keys(sw, args.vocab)
    prec = args.precision
    setup_s = {}
    r = w2v_leg(sw, ctx, args, ids, off, keys, prec, args.minibatch, args.dim, args.frag_num, args.steps,
                args.warmup, args.tokens, args.vocab, setup_s=setup_s)
    dt, total_words = ctx.max_sum(r["dt"], r["d"]["words"])
    roof = w2v_roofline(r, args, prec, args.minibatch, args.dim, args.tokens, args.vocab, world, ctx.sharded)
    d, info = r["d"], r["info"]
    one = rank == 0 and world == 1 and not ctx.sharded

    # the other precision modes on the same workload, timed the same way
    other_modes = {}
    if one and not args.no_parity_leg and args.dtype == "f32":
        set_phase("other_modes")
        for m in ("parity", "bfp40", "bfp32", "fast"):
            if m != prec:
                q = w2v_leg(sw, ctx, args, ids, off, keys, m, args.minibatch, args.dim, args.frag_num, args.steps,
                            args.warmup, args.tokens, args.vocab, profile=False)
                other_modes[m] = {"value": q["d"]["words"] / q["dt"], "ms_per_step": q["dt"] * 1e3 / args.steps,
                                  "mode": MODE_DESC[m]}
    # SURVEY.md §8(d) config 1's minibatch (B = 100 lines of the same 1000-token lines), same mode as
    # the headline, timed the same way over --b100-steps minibatches (the small-batch number)
    b100_leg = None
    if one and args.b100_steps > 0 and args.minibatch != 100:
        set_phase("minibatch_100")
        q = w2v_leg(sw, ctx, args, ids, off, keys, prec, 100, args.dim, args.frag_num, args.b100_steps, 10,
                    args.tokens, args.vocab, profile=False)
        b100_leg = {"value": q["d"]["words"] / q["dt"], "unit": "words/s", "minibatch": 100,
                    "steps": args.b100_steps, "warmup": 10, "ms_per_step": q["dt"] * 1e3 / args.b100_steps,
                    "kept_positions_per_s": q["d"]["kept"] / q["dt"],
                    "pulled_keys_per_step": q["d"]["pulled"] / args.b100_steps}
    # BASELINE config 1 (D = 100, minibatch 100 lines) on this GPU, same mode, beside its CPU run
    # (2 ranks in lockstep, cpu_baseline_config1)
    config1 = None
    if one and args.config1_steps > 0:
        set_phase("config1")
        q = w2v_leg(sw, ctx, args, ids, off, keys, prec, 100, 100, args.frag_num, args.config1_steps, 10,
                    args.tokens, args.vocab, profile=False)
        config1 = {"gpu": {"value": q["d"]["words"] / q["dt"], "unit": "words/s", "n_gpus": 1, "dim": 100,
                           "minibatch": 100, "steps": args.config1_steps,
                           "ms_per_step": q["dt"] * 1e3 / args.config1_steps},
                   "note": "BASELINE config 1 (D=100, window 5, negative 5, minibatch 100): the GPU on one rank's "
                           "corpus; the reference's 2-rank CPU plumbing as cpu_2rank"}
        if not args.no_cpu_baseline:
            config1["cpu_2rank"] = cpu_baseline_config1(ids, off, args, args.config1_cpu_lines)

    D = args.dim
    out = {
        "metric": "SGNS trained words/sec at 1/8 GPUs; sparse push/pull HBM GB/s vs peak",
        "value": total_words / dt,
        "unit": "words/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": {"parity": "f32 table, f64 intermediates + accumulate",
                  "bfp40": "f32 table, block-fp intermediates (int32+int8 mantissas/row exponent), f64 accumulate",
                  "bfp32": "f32 table, block-fp intermediates (int32 mantissas/row exponent), f64 accumulate",
                  "fast": "f32 table, f32 intermediates, f64 accumulate"}[prec] if args.dtype == "f32" else "f64",
        "data": "synthetic Zipf(s=1) text8 stand-in, random-init (reference glibc-rand) params",
        "config": {"mode": {"parity": "parity (fp64 intermediates)",
                            "bfp40": "bfp40 (block-fp neu1/neu1e: int32 + int8 mantissas, one exponent per row; "
                                     "fp64 sums and mean)",
                            "bfp32": "bfp32 (block-fp neu1/neu1e: int32 mantissas, one exponent per row; "
                                     "fp64 sums and mean)",
                            "fast": "fast (fp32 intermediates)"}[prec] +
                           (", alias sampler" if args.sampler == "alias" else ""),
                   "workload": "word2vec CBOW-NS (the reference's 'SGNS' app) text8-shaped corpus %d tokens, "
                               "vocab %d, dim %d, window %d, negative %d, sample %g, minibatch %d lines of %d "
                               "tokens, %s" % (args.tokens, info["vocab"], D, args.window, args.negative, args.sample,
                                               args.minibatch, args.line_len,
                                               "table in one HBM shard" if not ctx.sharded else
                                               "per rank (weak scaling: each rank its own corpus)"),
                   "global_batch": args.minibatch * world,
                   "parallelism": parallelism(ctx, args, args.frag_num),
                   "kept_positions_per_s": d["kept"] * world / dt, "batches_per_epoch": info["batches"],
                   "pulled_keys_per_step": d["pulled"] / args.steps,
                   "setup_s": dict(setup_s)},
        "roofline": roof,
        "kernel_ms": {k: v[0] for k, v in r["kt"].items()},
        "other_modes": other_modes or None,
        "minibatch_100": b100_leg,
        "config1": config1,
        "exchange": exchange_block(r.get("xs"), args.steps, r.get("dpt", 0.0), world,
                                   "remote bytes (keys 8 B, rows and grads %d B per remote key) / all-to-all time "
                                   "(events on the exchange stream, profiled pass); world %d"
                                   % (2 * D * (8 if args.dtype == "f64" else 4), world)),
    }
    with_transport(out, ctx, cbow_ipc(ctx, args))
    if one and not args.no_cpu_baseline:
        set_phase("cpu_baseline")
        out["cpu_baseline"] = cpu_baseline(ids, off, keys, args, args.cpu_lines)
    del ids, off
    # BASELINE configs 4, 3 and 5 at their per-GPU shapes beside the headline, at every N (each
    # rank its own share: weak scaling; the same legs at N = 1 give each curve its base point),
    # each with its own roofline, exchange block and (N = 1) CPU baseline
    if not args.no_app_legs:
        if args.config4_tokens > 0 and args.config4_steps > 0:
            out["config4"] = config4_leg(sw, ctx, args)
        la = argparse.Namespace(**vars(args))
        la.steps, la.warmup = args.app_steps, 3
        set_phase("lr")
        out["lr"] = bench_lr(la, ctx, corpus_batches=10, cpu_rows=10 * (args.lr_batch + 1))
        if os.environ.get("BENCH_ORDER") != "s2v_first":
            lr_sharded_base(out, ctx, args, la)
        sa = argparse.Namespace(**vars(args))
        sa.steps, sa.warmup = 31, 31  # one launch of 31 minibatches (swps_s2v group_docs) per pass
        set_phase("s2v")
        out["s2v"] = bench_s2v(sa, ctx, corpus_batches=31)
        if os.environ.get("BENCH_ORDER") == "s2v_first":
            lr_sharded_base(out, ctx, args, la)
    set_phase("report")
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if ctx.dist is not None:
        ctx.dist.destroy_process_group()


def lr_sharded_base(out, ctx, args, la):
    """lr.sharded_world1 (N = 1 only): the lr leg's workload through the key-sharded protocol."""
    if ctx.world != 1 or ctx.sharded or args.no_lr_sharded_base:
        return
    # the N > 1 LR leg runs the key-sharded protocol (owner pull, exchange, install, the step,
    # the mean-gradient push, owner AdaGrad); its world-1 run is the like-for-like base point
    # of the scaling curve (lr.value above is the unsharded single-GPU step)
    set_phase("lr_sharded_world1")
    sctx = Ctx(True)
    lb = argparse.Namespace(**vars(la))
    lb.no_cpu_baseline = True
    # two forms: the full protocol (SWPS_PULL_IN_PLACE=0: owner copy, install, step, payload, owner
    # AdaGrad — what every rank runs at N > 1, less the remote bytes) and world 1's own in-place form
    # (the install reads the shard rows, the push applies AdaGrad to them)
    q = {}
    prev = os.environ.get("SWPS_PULL_IN_PLACE")
    try:
        for form, env in (("protocol", "0"), ("in_place", "1")):
            os.environ["SWPS_PULL_IN_PLACE"] = env
            q[form] = bench_lr(lb, sctx, corpus_batches=10)
    finally:
        if prev is None:
            os.environ.pop("SWPS_PULL_IN_PLACE", None)
        else:
            os.environ["SWPS_PULL_IN_PLACE"] = prev
    p, i = q["protocol"], q["in_place"]
    out["lr"]["sharded_world1"] = {
        "value": p["value"], "unit": p["unit"], "ms_per_step": p["ms_per_step"], "kernel_ms": p["kernel_ms"],
        "parallelism": p["config"]["parallelism"],
        "note": "the same workload through the key-sharded protocol at world 1 (no remote bytes, SWPS_PULL_IN_PLACE=0):"
                " the like-for-like base point for the N > 1 lr legs, which run this protocol",
        "in_place": {"value": i["value"], "ms_per_step": i["ms_per_step"], "kernel_ms": i["kernel_ms"],
                     "note": "the library driver's default at world 1: the step's install reads the shard rows the "
                             "owner looked up and its push applies AdaGrad to them (no owner copy, payload or owner "
                             "apply)"}}
    sctx.close()
    if sctx.dist is not None:
        sctx.dist.destroy_process_group()


def bench_other(args):
    """Config 3 (sparse LR, Criteo shape, key-sharded over the GPUs) and
    config 5 (sent2vec, doc-sharded, word table replicated) — one JSON line
    each, same timing contract as the headline."""
    set_phase("init")
    ctx = Ctx(args.sharded)
    set_phase(args.app)
    out = bench_lr(args, ctx) if args.app == "lr" else bench_s2v(args, ctx)
    if ctx.rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if ctx.dist is not None:
        ctx.dist.destroy_process_group()


def bench_lr(args, ctx, corpus_batches=None, cpu_rows=None):
    """BASELINE config 3's per-GPU shape: one result dict (the JSON line of
    --app lr, or the default line's `lr` object).  corpus_batches: minibatches
    of synthetic data (default warmup + 2 x steps: every pass trains new rows;
    fewer wrap around, like further epochs)."""
    import swiftmpi_amd as sw
    from swiftmpi_amd.synth import criteo
    rank, world, local, dist = ctx.rank, ctx.world, ctx.local, ctx.dist
    steps, warm = args.steps, args.warmup
    B1 = args.lr_batch + 1
    nb = corpus_batches or (2 * steps + warm)
    y, off, f, v = criteo(B1 * nb, seed=3 + rank)
    lr_rate = args.lr if args.lr != 0.7 else 0.05
    t = sw.Table("lr", capacity=1 << 23, dtype="f32", learning_rate=lr_rate, init="hash", seed=1, device=local)
    comm = ctx.comm() if dist is not None and args.driver == "native" else None  # the library issues the exchange
    ipc = ctx.ipc_comm() if comm is not None else None
    if ipc is not None:  # the latency-bound exchange: device to device through IPC-mapped inboxes
        comm = ipc
    # end to end: load (the CSR rows to the GPU, the per-batch key-sorted index, the first full
    # pull) and the first epoch over the nb minibatches, to its last push (lr.cpp:157-238 rebuilds
    # that index per minibatch; here it is built once at load)
    ctx.barrier()
    t0 = time.perf_counter()
    if comm is not None:
        m = sw.LR(t, minibatch=args.lr_batch, init_ref=False, profile=False, fast_sums=not args.lr_exact,
                  plan=args.lr_plan)
        m.load_csr(y, off, f, v)
        m.shard_comm(comm, frag_num=2000)
        t1 = time.perf_counter()
        m.init()
        run = m.train_batches
    elif dist is not None:
        from swiftmpi_amd.dist import ShardedLR
        m = ShardedLR(t, frag_num=2000, minibatch=args.lr_batch, profile=False, fast_sums=not args.lr_exact)
        m.load_csr(y, off, f, v)
        t1 = time.perf_counter()
        m.init()
        run = m.train_steps
    else:
        m = sw.LR(t, minibatch=args.lr_batch, init_ref=False, profile=False, fast_sums=not args.lr_exact,
                  plan=args.lr_plan)
        m.load_csr(y, off, f, v)
        t1 = time.perf_counter()
        m.init()
        run = m.train_batches
    m.sync()
    t2 = time.perf_counter()
    run(nb)                                # the first epoch
    m.sync()
    ctx.barrier()
    e2e = time.perf_counter() - t0
    setup_s = {"load": t1 - t0, "first_pull": t2 - t1, "first_epoch": time.perf_counter() - t2}
    run(warm)
    m.sync()

    def run_timed(n):
        ctx.barrier()
        a = time.perf_counter()
        run(n)
        m.sync()
        ctx.barrier()
        return time.perf_counter() - a

    dt = run_timed(steps)                  # the measured region: no event timing inside
    m.set_profile(True)                    # a second, profiled pass for the per-kernel roofline
    m.kernel_times(reset=True)
    if comm is not None:
        m.exchange_stats(on=1)
    dpt = run_timed(steps)
    kt = m.kernel_times()
    xs = m.exchange_stats(on=0) if comm is not None else None
    m.set_profile(False)
    pbat = [(warm + steps + k) % nb for k in range(steps)]  # the profiled pass's batches
    # the fixed-point step runs unsharded and on the library driver's sharded learner (plan none)
    fxb = [m.fx_bytes(b) for b in pbat] if args.lr_plan == "none" and (comm is not None or dist is None) else []
    fx = bool(fxb) and all(d["form"] == 1 for d in fxb)
    m.close()
    t.close()
    e2e, e2e_rows = ctx.max_sum(e2e, nb * B1)
    dt, total = ctx.max_sum(dt, steps * B1)
    # SURVEY.md §8(d) LR bytes, over the profiled pass's batches (warm + steps + k) mod nb:
    # k_lr_forward: per feature its shard row index, x_i and weight (4 B each); per example 20 B
    # (row offset, label, e, e^2).  Push (k_lr_records + k_lr_reduce_*, the push timer): per
    # feature the sorted (row, x_i), the gathered e and the record written then read back (20 B);
    # per unique key its run (key, count, offset, shard row: 16 B) + the [w | g2] row read and
    # written (16 B).
    nnz = sum(int(off[(b + 1) * B1] - off[b * B1]) for b in pbat)
    uniq = sum(len(np.unique(f[off[b * B1]:off[(b + 1) * B1]])) for b in pbat)
    fwd_ms, fwd_n = kt["forward"]
    fwd_bytes = 12 * nnz + 20 * steps * B1
    tiles = not args.lr_exact and os.environ.get("SWPS_LR_TILES", "1") != "0" and not fx
    if fx:  # the fixed-point step's own model (swps_lr_fx_bytes)
        fwd_bytes = sum(d["step"] for d in fxb)
    fwd_gbs = fwd_bytes / (fwd_ms * 1e-3) / 1e9 if fwd_ms > 0 else 0.0
    push_ms, push_n = kt.get("push", (0.0, 0))
    if fx:
        push_bytes = sum(d["push"] for d in fxb)
    elif tiles:  # row tiles: per feature its (row, x_i) (6 B); per piece its run and slot (8 B), per
        # partial its fp64 write + read (16 B); per unique key its run (16 B) + the row RMW (16 B)
        pieces = partials = 0
        for b in pbat:
            pc, pa = lr_tile_pieces(f, off, b * B1, (b + 1) * B1)
            pieces += pc
            partials += pa
        push_bytes = 6 * nnz + 8 * pieces + 16 * partials + 32 * uniq
    else:
        push_bytes = 20 * nnz + 32 * uniq
    push_gbs = push_bytes / (push_ms * 1e-3) / 1e9 if push_ms > 0 else 0.0
    step_gbs = (fwd_bytes + push_bytes) * world / dt / 1e9
    kf = {"kernel": "k_lr_fxr_step (forward + per-chunk bucket sort into the bucket regions + hot-key partials)" if fx
          else "k_lr_forward_c" if os.environ.get("SWPS_LR_FWD_C", "1") != "0" else "k_lr_forward_g",
          "achieved": fwd_gbs, "frac": fwd_gbs / HBM_PEAK_GBS,
          "bytes_per_launch": fwd_bytes / max(fwd_n, 1), "avg_launch_ms": fwd_ms / max(fwd_n, 1), "launches": fwd_n}
    kp = {"kernel": ("k_lr_records + k_lr_reduce_short + k_lr_reduce_long" if args.lr_exact
                     else "k_lr_fxb_push (bucket LDS sums, hot-key column sums)" if fx
                     else "k_lr_tiles + k_lr_tiles_fin" if tiles
                     else "k_lr_records + k_lr_reduce_fused") + " (per-key mean + AdaGrad push)",
          "achieved": push_gbs, "frac": push_gbs / HBM_PEAK_GBS,
          "bytes_per_launch": push_bytes / max(push_n, 1), "avg_launch_ms": push_ms / max(push_n, 1),
          "launches": push_n}
    tr, tsrc = pmc_traffic(dict(app="lr", lr_batch=args.lr_batch, exact=bool(args.lr_exact), world=world,
                                sharded=dist is not None, plan=args.lr_plan),
                           {"forward": ("k_lr_forward_c", "k_lr_forward_r", "k_lr_forward", "k_lr_forward_g",
                                        "k_lr_fxb_step", "k_lr_fxr_step", "k_lr_fx_step"),
                            "push": ("k_lr_records", "k_lr_reduce_fused", "k_lr_reduce_short", "k_lr_reduce_long",
                                     "k_lr_reduce_long_fast", "k_lr_tiles", "k_lr_tiles_fin", "k_lr_fxb_push",
                                     "k_lr_fx_apply")})
    for kd, name in ((kf, "forward"), (kp, "push")):
        kd["traffic"] = tr[name]
        kd["traffic_source"] = tsrc
        if tr[name] and kd["avg_launch_ms"] > 0:
            kd["hbm_GBps"] = tr[name] / (kd["avg_launch_ms"] * 1e-3) / 1e9
            kd["hbm_frac"] = kd["hbm_GBps"] / HBM_PEAK_GBS
    dom, other = (kp, kf) if push_ms >= fwd_ms else (kf, kp)
    out = {"metric": "sparse LR trained examples/sec (AdaGrad, key-sharded PS)", "value": total / dt,
           "unit": "examples/s", "n_gpus": world, "steps": steps, "warmup": warm,
           "ms_per_step": dt * 1e3 / steps, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "f32", "data": "synthetic Criteo-shape hashed features (swiftmpi_amd/synth.py criteo)",
           "config": {"workload": "sparse logistic regression (BASELINE config 3 shape), 39 features/row, "
                                  "2^24 hashed feature space, %d rows per GPU per minibatch, AdaGrad lr %g, "
                                  "%d minibatches of data" % (B1, lr_rate, nb),
                      "parallelism": ("key-sharded PS over %d GPU(s) (BasicHashFrag frag_num 2000), %s all-to-all-v%s"
                                      % (world, "device-initiated IPC" if ipc is not None else ctx.backend,
                                         ", library-issued" if comm is not None else ""))
                      if dist is not None else "1 GPU, one HBM shard",
                      "mode": "exact (sequential fp32 per-key sums, bit-exact with the reference)" if args.lr_exact
                      else ("fixed point (each key's sum of e*x_i as an exact 64-bit integer at scale 2^s "
                            "fixed at load: order-free, deterministic; no per-batch index, every minibatch's "
                            "key grouping done inside its step; within 1e-6 of the fp64 sums)"
                            if fx else "fast (fp64 per-key sums%s; within 1e-5 of the oracle)"
                            % (" through row tiles" if tiles else ", wave tree-reduced")),
                      "plan": args.lr_plan,
                      "features_per_s": total * nnz / max(steps * B1, 1) / dt,
                      "unique_keys_per_step": uniq / steps, "setup_s": setup_s,
                      "end_to_end": {"value": e2e_rows / e2e, "unit": "examples/s", "s": e2e, "minibatches": nb,
                                     "note": ("load (CSR to the GPU, the vocabulary, the first full pull) + the "
                                              "first epoch to its last push, max over ranks; no per-batch index "
                                              "exists (plan none)" if fx else
                                              "load (CSR to the GPU, the per-batch key-sorted index built once for "
                                              "the corpus, the first full pull) + the first epoch to its last push, "
                                              "max over ranks") + "; `value` is the steady state of later epochs"}},
           "roofline": dict(dom, bound="hbm", peak=HBM_PEAK_GBS, unit="GB/s",
                            step_GBps=step_gbs, step_frac=step_gbs / HBM_PEAK_GBS, other=other),
           "kernel_ms": {k: v[0] for k, v in kt.items() if v[1]},
           "exchange": exchange_block(xs, steps, dpt, world, "remote bytes (keys 8 B, weights 4 B, mean gradients 4 B "
                                                             "per remote key) / all-to-all time (events on the "
                                                             "exchange stream, profiled pass)")}
    if comm is not None:
        with_transport(out, ctx)
        if ipc is not None:
            out["transport"] += "+ipc"
            out["ipc"] = ipc.ipc_info()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_lr(y, off, f, v, args.lr_batch, lr_rate,
                                              cpu_rows if cpu_rows is not None else args.cpu_rows)
    return out


def bench_s2v(args, ctx, corpus_batches=None):
    """BASELINE config 5's per-GPU share: one result dict (the JSON line of
    --app s2v, or the default line's `s2v` object).  corpus_batches: minibatches
    of synthetic documents (default warmup + steps; fewer wrap around)."""
    import torch
    import swiftmpi_amd as sw
    from swiftmpi_amd.synth import zipf_tokens
    rank, world, local = ctx.rank, ctx.world, ctx.local
    steps, warm = args.steps, args.warmup
    V, D = 1000000, args.dim
    # a minibatch is the next B + 1 documents (sent2vec.cpp on word2vec.h's MiniBatch); the
    # passes wrap to the corpus start
    nd = (args.s2v_docs + 1) * (corpus_batches or (steps + warm))
    rng = np.random.default_rng(5 + rank)
    lens = rng.integers(50, 201, nd)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    ids, _ = zipf_tokens(int(off[-1]), V, 100, seed=5 + rank, progress=True)
    toks = ids.astype(np.uint64) + 1
    sent = (np.arange(nd, dtype=np.uint64) + np.uint64(nd * rank + 1)) * np.uint64(2654435761)
    t = sw.Table("w2v", dim=D, capacity=V + 1024, dtype="f32", init="hash", seed=3, device=local)
    keys = torch.arange(1, V + 1, dtype=torch.int64, device="cuda")
    t.pull(keys)  # the frozen word table (replicated on every GPU)
    del keys
    # `value`: the reference's sent2vec is ONE pass over its documents (sent2vec.cpp:95-103: per
    # minibatch gather_keys, pull, the unigram table, train), so the measured step is that pass,
    # load included — swps_s2v_run_tokens, the host's per-minibatch plan overlapped with the GPU's
    # training — timed from the caller's token arrays to the last sentence trained.  One untimed
    # pass on a throwaway object first (the warm-up); each rank its own docs (doc-sharded by
    # construction, no exchange)
    def fresh():
        return sw.Sent2Vec(t, window=args.window, negative=args.negative, minibatch=args.s2v_docs, niters=1,
                           alpha=args.alpha)
    s2 = fresh()
    s2.run_tokens(toks, off, sent)
    passes_b = s2.info()["batches"]
    s2.close()
    ctx.barrier()
    t0 = time.perf_counter()
    s2 = fresh()
    s2.run_tokens(toks, off, sent)
    s2.sync()
    ctx.barrier()
    e2e = time.perf_counter() - t0
    st0 = s2.stats()
    setup_s = {"single_pass": e2e, "minibatches": passes_b}

    def run_timed(n):
        ctx.barrier()
        a = time.perf_counter()
        s2.train_batches(n)
        s2.sync()
        ctx.barrier()
        return time.perf_counter() - a

    dt = run_timed(steps)
    st1 = s2.stats()
    s2.set_profile(True)
    s2.kernel_times(reset=True)
    run_timed(steps)
    st2 = s2.stats()
    kt = s2.kernel_times()
    s2.set_profile(False)
    s2.close()
    t.close()
    e2e, e2e_words = ctx.max_sum(e2e, st0["positions"])
    dt, total = ctx.max_sum(dt, st1["positions"] - st0["positions"])
    steady = {"value": total / dt, "unit": "words/s", "ms_per_minibatch": dt * 1e3 / steps, "minibatches": steps,
              "note": "the same documents trained again after the single pass (train_batches: every "
                      "minibatch's plan already on the device) — not the reference's workload, which is one "
                      "pass; kept as the kernels' steady state"}
    # SURVEY.md §8(d) sent2vec bytes of the docs kernel: 4*D per word row read (contexts + targets)
    # + 8*D per document (its row read and written)
    rows_read = (st2["ctx_rows"] - st1["ctx_rows"]) + (st2["tgt_rows"] - st1["tgt_rows"])
    ndocs = st2["docs"] - st1["docs"]
    doc_ms, doc_n = kt["docs"]
    doc_bytes = 4 * D * rows_read + 8 * D * ndocs
    doc_gbs = doc_bytes / (doc_ms * 1e-3) / 1e9 if doc_ms > 0 else 0.0
    tr, tsrc = pmc_traffic(dict(app="s2v", s2v_docs=args.s2v_docs, dim=D, world=world), {"docs": ("k_s2v_docs",)})
    out = {"metric": "sent2vec trained words/sec (frozen word table, doc-sharded)", "value": e2e_words / e2e,
           "unit": "words/s", "n_gpus": world, "steps": passes_b, "warmup": passes_b,
           "ms_per_step": e2e * 1e3 / max(passes_b, 1),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32 table, f64 math",
           "data": "synthetic Zipf(s=1) docs of 50-200 tokens over V=1M, hash-initialised word table",
           "config": {"workload": "sent2vec (BASELINE config 5 shape), D=%d, window %d, negative %d, %d docs "
                                  "per minibatch, word table 1M x %d, %d documents"
                                  % (D, args.window, args.negative, args.s2v_docs, D, nd),
                      "parallelism": "doc-sharded over %d GPU(s), no exchange (replicas only)" % world,
                      "setup_s": setup_s,
                      "step": "one minibatch of the single pass (load included): value = words of the pass / "
                              "its wall time, max over ranks; warmup = one untimed pass on a throwaway object",
                      "end_to_end": {"value": e2e_words / e2e, "unit": "words/s", "s": e2e,
                                     "note": "= value: load + the single pass over this leg's %d documents per "
                                             "rank (the reference's sent2vec is one pass), max over ranks" % nd},
                      "steady_state": steady},
           "roofline": {"bound": "hbm", "kernel": "k_s2v_docs", "achieved": doc_gbs, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": doc_gbs / HBM_PEAK_GBS, "traffic": tr["docs"],
                        "traffic_source": tsrc,
                        "hbm_GBps": (tr["docs"] / (doc_ms / max(doc_n, 1) * 1e-3) / 1e9
                                     if tr["docs"] and doc_ms > 0 else None),
                        "bytes_per_launch": doc_bytes / max(doc_n, 1), "avg_launch_ms": doc_ms / max(doc_n, 1),
                        "launches": doc_n},
           "kernel_ms": {k: v[0] for k, v in kt.items()}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_s2v(toks, off, args, args.cpu_docs)
    return out


def _free_port_pair():
    """A port P on 127.0.0.1 with P and P + 1 both free (torch.distributed's
    store at MASTER_PORT, the library's bootstrap at MASTER_PORT + 1), below Linux's
    ephemeral range (32768-60999) so no outgoing connection takes it meanwhile."""
    import random
    import socket
    rng = random.Random()
    while True:
        p = rng.randrange(15000, 32000)
        socks = []
        try:
            for q in (p, p + 1):
                sk = socket.socket()
                socks.append(sk)
                sk.bind(("127.0.0.1", q))
            return p
        except OSError:
            continue
        finally:
            for sk in socks:
                sk.close()


def launch_ranks(n, argv):
    """`bench.py --gpus N` without a launcher (no WORLD_SIZE in the environment):
    start N rank processes of this script — one per GPU, RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR / MASTER_PORT set as torch.distributed.run would —
    and wait for them.  This process never touches the GPU (child processes,
    no exec).  Rank 0 prints the JSON line.  If any rank fails, the others are
    stopped (SIGTERM, then SIGKILL after 10 s) and the first failing exit code is
    returned; past the overall deadline (SWPS_BENCH_DEADLINE_S + 60 s) every rank
    is killed and 124 returned."""
    import subprocess
    port = _free_port_pair()
    deadline = time.time() + float(os.environ.get("SWPS_BENCH_DEADLINE_S", "1500")) + 60
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc, stop_at = 0, None
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c  # a signal: 128 + its number, as a shell reports it
                print("bench.py: rank %d exited with %d; stopping the other ranks" % (procs.index(p), c),
                      file=sys.stderr, flush=True)
                for q in live:  # the others would wait in a collective until their own deadlines
                    q.terminate()
                stop_at = time.time() + 10
        if live and ((stop_at and time.time() > stop_at) or time.time() > deadline):
            if not stop_at:
                print("bench.py: overall deadline exceeded; killing every rank", file=sys.stderr, flush=True)
                rc = rc or 124
            for q in live:
                q.kill()
            for q in live:
                q.wait()
            live = []
        time.sleep(0.2)
    return rc


def _launcher():
    """Resolve --gpus against the environment before anything imports torch."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    a, _ = ap.parse_known_args()
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None and int(ws) != a.gpus:
        print("bench.py: WORLD_SIZE=%s but --gpus %d: launch one rank per GPU with --gpus equal to the world size"
              % (ws, a.gpus), file=sys.stderr, flush=True)
        return 2
    if ws is None and a.gpus > 1:
        return launch_ranks(a.gpus, sys.argv[1:])
    return None


if __name__ == "__main__":
    _rc = _launcher()
    if _rc is not None:
        sys.exit(_rc)
    try:
        main()
    except BaseException as _e:  # noqa: BLE001 — name the rank and phase, and do not hang in teardown
        import traceback
        traceback.print_exc()
        print("bench.py: rank %s failed in phase %s: %s" % (os.environ.get("RANK", "0"), _PHASE["name"], _e),
              file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(1)
