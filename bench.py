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
    ap.add_argument("--sampler", default="table", choices=["table", "alias"],
                    help="negative sampler: the reference's unigram table (bit-exact draws) or an alias table")
    ap.add_argument("--app", default="w2v", choices=["w2v", "lr", "s2v"],
                    help="w2v: the headline (config 2); lr: config 3 shape; s2v: config 5 shape")
    ap.add_argument("--lr-batch", type=int, default=65536, help="LR rows per GPU per minibatch (config 3)")
    ap.add_argument("--lr-exact", action="store_true",
                    help="LR: the reference's sequential fp32 per-key sums (bit-exact) instead of fast fp64 sums")
    ap.add_argument("--s2v-docs", type=int, default=8192, help="sent2vec documents per minibatch")
    ap.add_argument("--no-app-legs", action="store_true",
                    help="skip the LR (config 3) and sent2vec (config 5) legs of the default line")
    ap.add_argument("--app-steps", type=int, default=20, help="timed LR minibatches of the default line's lr leg")
    args = ap.parse_args()
    if args.app != "w2v":
        return bench_other(args)

    import torch
    import swiftmpi_amd as sw

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    ngpu = torch.cuda.device_count()
    sharded = world > 1 or args.sharded
    backend = None
    if sharded:
        import torch.distributed as dist
        local = local % max(ngpu, 1)
        torch.cuda.set_device(local)
        if "MASTER_ADDR" not in os.environ:
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", RANK="0", WORLD_SIZE="1")
        if ngpu >= world:  # one GPU per rank: RCCL over xGMI
            backend = "nccl"
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:               # functional check with ranks sharing a GPU
            backend = "gloo"
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)

    ids, off = make_corpus(args.tokens, args.vocab, args.line_len, seed=8 + rank)
    print("corpus: %d tokens" % len(ids), file=sys.stderr, flush=True)
    keys = word_keys(sw, args.vocab)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    setup_s = {}
    _comm = []

    def native_comm():  # one communicator per process, reused by every leg
        if not _comm:
            from swiftmpi_amd.comm import Comm
            port = int(os.environ.get("MASTER_PORT", "29533")) + 1
            addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
            try:
                c = (Comm.rccl(rank, world, local, addr=addr, port=port) if backend == "nccl"
                     else Comm.tcp(rank, world, local, addr=addr, port=port))
                ok = 1
            except Exception as e:  # noqa: BLE001 — reported, and every rank falls back together
                print("native communicator failed on rank %d: %s" % (rank, e), file=sys.stderr, flush=True)
                c, ok = None, 0
            t = torch.tensor([ok], dtype=torch.int32, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            _comm.append(c if int(t.item()) else None)
        return _comm[0]

    def build(fp64_intermediates, minibatch=None, dim=None):
        kw = dict(window=args.window, negative=args.negative, minibatch=minibatch or args.minibatch, sample=args.sample,
                  alpha=args.alpha, profile=False, fp64_intermediates=fp64_intermediates, sampler=args.sampler)
        t = sw.Table("w2v", dim=dim or args.dim, capacity=args.vocab, dtype=args.dtype, learning_rate=args.lr,
                     device=local, init="hash", seed=1)
        if sharded and args.driver == "native" and native_comm() is not None:  # the library's own exchange
            from swiftmpi_amd.dist import NativeShardedWord2Vec
            w = NativeShardedWord2Vec(t, native_comm(), frag_num=args.frag_num, **kw)
        elif sharded:  # key-sharded over the ranks (BasicHashFrag), RCCL all-to-all per minibatch
            from swiftmpi_amd.dist import ShardedWord2Vec
            w = ShardedWord2Vec(t, frag_num=args.frag_num, pipeline=pipelined, **kw)
        else:
            w = sw.Word2Vec(t, init="ref", **kw)
        t0 = time.perf_counter()
        w.load_tokens(ids, off, keys)
        t1 = time.perf_counter()
        w.init()
        setup_s.update(ingest=t1 - t0, first_pull=time.perf_counter() - t1)
        return t, w

    def timed(w, steps):
        s0 = w.stats()
        barrier()
        t0 = time.perf_counter()
        w.train_batches(steps)
        w.sync()
        barrier()
        dt = time.perf_counter() - t0
        s1 = w.stats()
        return dt, {k: s1[k] - s0[k] for k in s1 if k not in ("lstate", "fstate")}

    if args.parity:
        args.precision = "parity"
    prec = args.precision
    parity_main = prec == "parity"
    bfp_main = prec.startswith("bfp") and args.dtype == "f32"
    rb = 1 if prec == "bfp40" else 0  # BFP residual bytes per element
    INTER = {"bfp40": "bfp40", "bfp32": "bfp32", "fast": False, "parity": True}
    pipelined = sharded and args.pipeline
    t, w = build(fp64_intermediates=INTER[prec])
    info = w.info()
    w.train_batches(args.warmup)
    w.sync()
    dt, d = timed(w, args.steps)           # the measured region: no event timing inside
    words = d["words"]
    w.set_profile(True)                     # a second, profiled pass for the per-kernel roofline
    w.kernel_times(reset=True)
    gw = getattr(w, "w", w)                 # the per-rank Word2Vec (sharded: its learner)
    g0 = gw.sum_stats()
    if sharded:
        w.set_exchange_profile(True)
    dpt, dp = timed(w, args.steps)
    kt = w.kernel_times()
    g1 = gw.sum_stats()
    xs = w.exchange_stats() if sharded else None
    w.set_profile(False)
    if sharded:
        w.set_exchange_profile(False)
    del w, t
    if dist is not None:
        tt = torch.tensor([dt, float(words)], dtype=torch.float64, device="cuda")
        mx = tt.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        dt, total_words = float(mx[0]), float(tt[1])
    else:
        total_words = float(words)

    D, es = args.dim, (8 if args.dtype == "f64" else 4)
    ea = 8 if (parity_main or args.dtype == "f64") else 4   # neu1/neu1e element size
    # BFP modes: a record reads its position's mantissas (4 B, + the int8 residual in bfp40) per
    # element and the row scale (4 B); partials and the mean-gradient payload are fp64
    rec_row = D * (4 + rb) + 4 if bfp_main else D * ea
    pa = 8 if bfp_main else ea
    kept = d["kept"]
    # SURVEY.md §8(d) algorithmic bytes of k_forward: every context/target row
    # occurrence read (4·D per row in fp32) + neu1, neu1e written (2·D·ea per position)
    ctx_rows, tgt_rows = dp["ctx_rows"], dp["tgt_rows"]
    fwd_ms, fwd_n = kt["forward"]
    fwd_bytes = es * D * (ctx_rows + tgt_rows) + 2 * rec_row * dp["kept"]
    fwd_gbs = fwd_bytes / (fwd_ms * 1e-3) / 1e9 if fwd_ms > 0 else 0.0
    # the dominant kernel by time: the segmented gradient sums + AdaGrad push.
    # Algorithmic bytes: each gradient record reads its source row (neu1 or neu1e of its
    # position, D·ea) and its 4-B record index; each item (chunk of <= 128 records of one
    # key) that goes through a partial writes it (D·ea + a 16-B descriptor read) and the
    # push reads it back (D·ea); each pushed key reads h,v,h2,v2 (4·D·es), writes them
    # (4·D·es) and its pre-update h,v to the worker cache (2·D·es) + 8 B of bounds.
    # Fused push (k_push_thp, the fast-mode default): k_gather_t + k_combine sum only the
    # multi-chunk runs, k_push_thp sums the single-chunk runs itself -> the group is
    # k_gather_t + k_combine + k_push_thp, timed by the gather and push timers.
    # Otherwise the group is k_gather_t + k_combine alone (the push is reported below).
    g_rec, g_items = g1["records"] - g0["records"], g1["items"] - g0["items"]
    g_mrec, g_mitems = g1["multi_records"] - g0["multi_records"], g1["multi_items"] - g0["multi_items"]
    nbat = g1["batches"] - g0["batches"]
    fused = nbat > 0 and g1["fused"] - g0["fused"] == nbat
    fused_g = nbat > 0 and g1.get("fused_grads", 0) - g0.get("fused_grads", 0) == nbat
    # small batches run the multi-chunk gather on a side stream beside the push: the push timer
    # (push start .. the multi-chunk halves' push end) then spans the whole group
    split = nbat > 0 and g1.get("split", 0) - g0.get("split", 0) == nbat
    gat_ms, gat_n = kt["gather"]
    push_ms, push_n = kt.get("push", (0.0, 0))
    kn = ("k_gather_b", "k_combine_b", "k_push_b") if bfp_main else ("k_gather_t", "k_combine", "k_push_thp")
    if fused_g:  # sharded learner: the fused push stops at the mean gradients (2·D·pa written per key)
        sum_kernel = ("%s + %s + %s<TO_GRADS> (segmented gradient sums + fused mean "
                      "gradients of the push payload)" % kn)
        gat_bytes = g_rec * (rec_row + 4) + g_mitems * (2 * D * pa + 16) + dp["pushed"] * (2 * D * pa + 8)
        sum_ms = push_ms if split else gat_ms + push_ms
    elif fused:
        sum_kernel = "%s + %s + %s (segmented gradient sums + fused AdaGrad push)" % kn
        gat_bytes = (g_rec * (rec_row + 4) + g_mitems * (2 * D * pa + 16) +
                     dp["pushed"] * (10 * es * D + 8))
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
    # the metric's "sparse push/pull HBM GB/s".  Single GPU: the pull is no
    # kernel of its own — the forward reads the batch's keys straight from the
    # table rows (counted in roofline.forward) and the push leaves their
    # pre-update h, v in the worker cache.  Push (§8(d) + that cache write):
    # mean grads 2·D, read h,v,h2,v2 4·D, write 4·D, cache h,v 2·D elements
    # + the count per key, over the push kernel's event time in the profiled
    # pass (sharded mode: the owner-side install / serve kernels are not in
    # these timers, so the fields are omitted)
    pp = {}
    for name, nbytes in (("pull", dp["pulled"] * 4 * es * D), ("push", dp["pushed"] * (12 * es * D + 8))):
        ms, n = kt.get(name, (0.0, 0))
        if ms > 0 and not sharded and not ((fused or fused_g) and name == "push"):
            gbs = nbytes / (ms * 1e-3) / 1e9
            pp[name] = {"GBps": gbs, "frac": gbs / HBM_PEAK_GBS, "bytes_per_launch": nbytes / max(n, 1),
                        "avg_launch_ms": ms / max(n, 1)}
    if not sharded and "pull" not in pp:
        pp["pull"] = "fused: k_forward reads the pulled keys' table rows directly; k_push writes their cache rows"
    # xGMI: bytes this rank's all-to-alls sent to other ranks per step, over the
    # exchanges' event time on their stream, against 7 links x 153 GB/s
    exchange = None
    if xs is not None:
        xg = xs["bytes_remote"] / (xs["ms"] * 1e-3) / 1e9 if xs["ms"] > 0 else 0.0
        exchange = {"bytes_remote_per_step": xs["bytes_remote"] / args.steps,
                    "bytes_total_per_step": xs["bytes_total"] / args.steps,
                    "a2a_per_step": xs["calls"] / args.steps, "ms_per_step": xs["ms"] / args.steps,
                    "share_of_step": xs["ms"] / (dpt * 1e3) if dpt > 0 else None,
                    "GBps": xg, "peak": XGMI_PEAK_GBS, "frac": xg / XGMI_PEAK_GBS,
                    "note": "remote bytes (keys 8 B, rows and grads %d B per remote key) / all-to-all time "
                            "(events on the exchange stream, profiled pass); world %d" % (2 * D * es, world)}
    # HBM traffic of the same kernel from the committed PMC passes of this exact
    # command (scripts/gpu_profile.sh -> scripts/pmc_summary.py); null otherwise
    # (per-launch bytes do not depend on --steps / --warmup: only the workload
    # keys must match)
    mine = dict(app="w2v", minibatch=args.minibatch, dim=args.dim, dtype=args.dtype, mode=prec, world=world,
                tokens=args.tokens, vocab=args.vocab, line_len=args.line_len, sharded=bool(sharded),
                sampler=args.sampler)
    if bfp_main:
        grp = ("k_gather_b", "k_combine_b", "k_push_b")
    elif parity_main or args.dtype == "f64":
        grp = ("k_gather", "k_combine") + (("k_push_thp", "k_push_tg") if (fused or fused_g) else ())
    else:
        grp = ("k_gather_t", "k_combine") + (("k_push_thp", "k_push_tg") if (fused or fused_g) else ())
    tr, traffic_src = pmc_traffic(mine, {"sum": grp, "forward": ("k_forward_t", "k_forward_b", "k_forward_b8",
                                                                  "k_forward")})
    traffic, fwd_traffic = tr["sum"], tr["forward"]

    # the other precision modes on the same workload, timed the same way
    MODE_DESC = {"parity": "fp64 neu1/neu1e + gradient partials (reference-parity mode)",
                 "bfp40": "block-fp neu1/neu1e, int32 + int8 mantissas per row exponent, fp64 sums (5 B/element)",
                 "bfp32": "block-fp neu1/neu1e, int32 mantissas per row exponent, fp64 sums (4 B/element)",
                 "fast": "fp32 neu1/neu1e + partials (fast mode: outside the 1e-5 single-batch bar)"}
    other_modes = {}
    if rank == 0 and world == 1 and not args.no_parity_leg and args.dtype == "f32":
        for m in ("parity", "bfp40", "bfp32", "fast"):
            if m == prec:
                continue
            t2, w2 = build(fp64_intermediates=INTER[m])
            w2.train_batches(args.warmup)
            w2.sync()
            pdt, pd = timed(w2, args.steps)
            other_modes[m] = {"value": pd["words"] / pdt, "ms_per_step": pdt * 1e3 / args.steps,
                              "mode": MODE_DESC[m]}
            del w2, t2
    # SURVEY.md §8(d) config 1's minibatch (B = 100 lines of the same
    # 1000-token lines), same mode as the headline, timed the same way over
    # --b100-steps minibatches (the driver-visible small-batch number)
    b100_leg = None
    if rank == 0 and world == 1 and not sharded and args.b100_steps > 0 and args.minibatch != 100:
        t3, w3 = build(fp64_intermediates=INTER[prec], minibatch=100)
        w3.train_batches(10)
        w3.sync()
        bdt, bd = timed(w3, args.b100_steps)
        b100_leg = {"value": bd["words"] / bdt, "unit": "words/s", "minibatch": 100, "steps": args.b100_steps,
                    "warmup": 10, "ms_per_step": bdt * 1e3 / args.b100_steps,
                    "kept_positions_per_s": bd["kept"] / bdt, "pulled_keys_per_step": bd["pulled"] / args.b100_steps}
        del w3, t3

    # BASELINE config 1 (D = 100, minibatch 100 lines) on this GPU, same mode, beside its CPU
    # run (2 ranks in lockstep, cpu_baseline_config1)
    config1 = None
    if rank == 0 and world == 1 and not sharded and args.config1_steps > 0:
        t4, w4 = build(fp64_intermediates=INTER[prec], minibatch=100, dim=100)
        w4.train_batches(10)
        w4.sync()
        cdt, cd = timed(w4, args.config1_steps)
        config1 = {"gpu": {"value": cd["words"] / cdt, "unit": "words/s", "n_gpus": 1, "dim": 100, "minibatch": 100,
                           "steps": args.config1_steps, "ms_per_step": cdt * 1e3 / args.config1_steps},
                   "note": "BASELINE config 1 (D=100, window 5, negative 5, minibatch 100): the GPU on one rank's "
                           "corpus; the reference's 2-rank CPU plumbing as cpu_2rank"}
        del w4, t4
        if not args.no_cpu_baseline:
            config1["cpu_2rank"] = cpu_baseline_config1(ids, off, args, args.config1_cpu_lines)

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
                               "tokens, table in one HBM shard" % (args.tokens, info["vocab"], D, args.window,
                                                                  args.negative, args.sample, args.minibatch,
                                                                  args.line_len),
                   "global_batch": args.minibatch * world,
                   "parallelism": ("key-sharded PS over %d GPU(s) (BasicHashFrag frag_num %d), %s all-to-all-v, %s"
                                   % (world, args.frag_num,
                                      ("library-issued RCCL" if backend == "nccl" else "library TCP transport")
                                      if args.driver == "native" and _comm and _comm[0] is not None
                                      else ("RCCL" if backend == "nccl" else "gloo"),
                                      "pipelined: pull(i+1)/push(i) overlap learn(i), staleness 1" if pipelined
                                      else "lockstep pull/learn/push"))
                   if sharded else "1 GPU, one HBM shard",
                   "kept_positions_per_s": kept * world / dt, "batches_per_epoch": info["batches"],
                   "pulled_keys_per_step": d["pulled"] / args.steps,
                   "setup_s": dict(setup_s)},
        "roofline": {"bound": "hbm", "kernel": sum_kernel,
                     "achieved": gat_gbs, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": gat_gbs / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_src,
                     "bytes_per_launch": gat_bytes / max(gat_n, 1), "avg_launch_ms": sum_ms / max(gat_n, 1),
                     "launches": gat_n, "records_per_launch": g_rec / max(gat_n, 1),
                     "items_per_launch": g_items / max(gat_n, 1),
                     "partial_items_per_launch": (g_mitems if fused else g_items) / max(gat_n, 1),
                     "gather_ms_per_launch": gat_ms / max(gat_n, 1),
                     "push_ms_per_launch": push_ms / max(push_n, 1),
                     # k_forward: its row-occurrence bytes count every context/target row read,
                     # most of them L2 / Infinity-Cache hits (hot Zipf rows), so they are no
                     # roofline quantity (row_bytes_GBps); its roofline fraction is the
                     # PMC-measured memory-side traffic of the same launches over their time
                     "forward": {"kernel": "k_forward_b" if bfp_main else "k_forward_t",
                                 "row_bytes_GBps": fwd_gbs, "row_bytes_per_launch": fwd_bytes / max(fwd_n, 1),
                                 "avg_launch_ms": fwd_ms / max(fwd_n, 1), "launches": fwd_n,
                                 "traffic": fwd_traffic,
                                 "hbm_GBps": (fwd_traffic / (fwd_ms / max(fwd_n, 1) * 1e-3) / 1e9
                                              if fwd_traffic and fwd_ms > 0 else None),
                                 "frac": (fwd_traffic / (fwd_ms / max(fwd_n, 1) * 1e-3) / 1e9 / HBM_PEAK_GBS
                                          if fwd_traffic and fwd_ms > 0 else None)},
                     "step_GBps": step_gbs, "step_frac": step_gbs / HBM_PEAK_GBS,
                     "pull_push": pp or None},
        "kernel_ms": {k: v[0] for k, v in kt.items()},
        "other_modes": other_modes or None,
        "minibatch_100": b100_leg,
        "config1": config1,
        "exchange": exchange,
    }
    if _comm and _comm[0] is not None:  # the library's own communicator: what its transport reports
        kind, nranks = _comm[0].transport()
        out["transport"] = kind
        out["rccl_ranks" if kind == "rccl" else "transport_ranks"] = nranks
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(ids, off, keys, args, args.cpu_lines)
    # BASELINE configs 3 and 5 at their per-GPU shapes beside the headline (each with its own
    # roofline and CPU baseline): the driver's default line carries every app of the hot path
    if rank == 0 and world == 1 and not sharded and not args.no_app_legs:
        del ids, off
        one = (0, 1, local, None, None)
        la = argparse.Namespace(**vars(args))
        la.steps, la.warmup = args.app_steps, 3
        out["lr"] = bench_lr(la, one, corpus_batches=10, cpu_rows=10 * (args.lr_batch + 1))
        sa = argparse.Namespace(**vars(args))
        sa.steps, sa.warmup = 31, 31  # one launch of 31 minibatches (swps_s2v group_docs) per pass
        out["s2v"] = bench_s2v(sa, one, corpus_batches=31)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def _dist_init(args):
    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dist, backend = None, None
    if world > 1 or args.sharded:
        import torch.distributed as dist
        if "MASTER_ADDR" not in os.environ:
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", RANK="0", WORLD_SIZE="1")
        if torch.cuda.device_count() >= world:
            backend = "nccl"
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            backend = "gloo"
            dist.init_process_group("gloo")
    return rank, world, local, dist, backend


def bench_other(args):
    """Config 3 (sparse LR, Criteo shape, key-sharded over the GPUs) and
    config 5 (sent2vec, doc-sharded, word table replicated) — one JSON line
    each, same timing contract as the headline."""
    ctx = _dist_init(args)
    rank, dist = ctx[0], ctx[3]
    out = bench_lr(args, ctx) if args.app == "lr" else bench_s2v(args, ctx)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def _other_helpers(ctx):
    import torch
    dist = ctx[3]

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    def finish(dt, units):
        if dist is not None:
            tt = torch.tensor([dt, float(units)], dtype=torch.float64, device="cuda")
            mx = tt.clone()
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            dist.all_reduce(tt, op=dist.ReduceOp.SUM)
            return float(mx[0]), float(tt[1])
        return dt, float(units)

    def run_timed(run, sync, n):
        barrier()
        t0 = time.perf_counter()
        run(n)
        sync()
        barrier()
        return time.perf_counter() - t0
    return finish, run_timed


def bench_lr(args, ctx, corpus_batches=None, cpu_rows=None):
    """BASELINE config 3's per-GPU shape: one result dict (the JSON line of
    --app lr, or the default line's `lr` object).  corpus_batches: minibatches
    of synthetic data (default warmup + 2 x steps: every pass trains new rows;
    fewer wrap around, like further epochs)."""
    import swiftmpi_amd as sw
    from swiftmpi_amd.synth import criteo
    rank, world, local, dist, backend = ctx
    finish, run_timed = _other_helpers(ctx)
    steps, warm = args.steps, args.warmup
    B1 = args.lr_batch + 1
    nb = corpus_batches or (2 * steps + warm)
    y, off, f, v = criteo(B1 * nb, seed=3 + rank)
    lr_rate = args.lr if args.lr != 0.7 else 0.05
    t = sw.Table("lr", capacity=1 << 23, dtype="f32", learning_rate=lr_rate, init="hash", seed=1, device=local)
    comm = None
    if dist is not None and args.driver == "native":  # the library issues the exchange
        from swiftmpi_amd.comm import Comm
        import torch
        port = int(os.environ.get("MASTER_PORT", "29533")) + 1
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        try:
            comm = (Comm.rccl(rank, world, local, addr=addr, port=port) if backend == "nccl"
                    else Comm.tcp(rank, world, local, addr=addr, port=port))
        except Exception as e:  # noqa: BLE001 — every rank falls back to the Python driver together
            print("native communicator failed on rank %d: %s" % (rank, e), file=sys.stderr, flush=True)
        ok = torch.tensor([int(comm is not None)], dtype=torch.int32, device="cuda")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if not int(ok.item()):
            comm = None
    if comm is not None:
        m = sw.LR(t, minibatch=args.lr_batch, init_ref=False, profile=False, fast_sums=not args.lr_exact)
        m.load_csr(y, off, f, v)
        m.shard_comm(comm, frag_num=2000)
        m.init()
        run = m.train_batches
    elif dist is not None:
        from swiftmpi_amd.dist import ShardedLR
        m = ShardedLR(t, frag_num=2000, minibatch=args.lr_batch, profile=False, fast_sums=not args.lr_exact)
        m.load_csr(y, off, f, v)
        m.init()
        run = m.train_steps
    else:
        m = sw.LR(t, minibatch=args.lr_batch, init_ref=False, profile=False, fast_sums=not args.lr_exact)
        m.load_csr(y, off, f, v)
        m.init()
        run = m.train_batches
    run(warm)
    m.sync()
    dt = run_timed(run, m.sync, steps)     # the measured region: no event timing inside
    m.set_profile(True)                    # a second, profiled pass for the per-kernel roofline
    m.kernel_times(reset=True)
    run_timed(run, m.sync, steps)
    kt = m.kernel_times()
    m.set_profile(False)
    xport = comm.transport() if comm is not None else None
    m.close()
    t.close()
    if comm is not None:
        comm.close()
    dt, total = finish(dt, steps * B1)
    # SURVEY.md §8(d) LR bytes, over the profiled pass's batches (warm + steps + k) mod nb:
    # k_lr_forward: per feature its shard row index, x_i and weight (4 B each); per example 20 B
    # (row offset, label, e, e^2).  Push (k_lr_records + k_lr_reduce_*, the push timer): per
    # feature the sorted (row, x_i), the gathered e and the record written then read back (20 B);
    # per unique key its run (key, count, offset, shard row: 16 B) + the [w | g2] row read and
    # written (16 B).
    pbat = [(warm + steps + k) % nb for k in range(steps)]
    nnz = sum(int(off[(b + 1) * B1] - off[b * B1]) for b in pbat)
    uniq = sum(len(np.unique(f[off[b * B1]:off[(b + 1) * B1]])) for b in pbat)
    fwd_ms, fwd_n = kt["forward"]
    fwd_bytes = 12 * nnz + 20 * steps * B1
    tiles = not args.lr_exact and os.environ.get("SWPS_LR_TILES", "1") != "0"
    fwd_gbs = fwd_bytes / (fwd_ms * 1e-3) / 1e9 if fwd_ms > 0 else 0.0
    push_ms, push_n = kt.get("push", (0.0, 0))
    if tiles:  # row tiles: per feature its (row, x_i) (6 B); per piece its run and slot (8 B), per
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
    kf = {"kernel": "k_lr_forward_c" if os.environ.get("SWPS_LR_FWD_C", "1") != "0" else "k_lr_forward_g",
          "achieved": fwd_gbs, "frac": fwd_gbs / HBM_PEAK_GBS,
          "bytes_per_launch": fwd_bytes / max(fwd_n, 1), "avg_launch_ms": fwd_ms / max(fwd_n, 1), "launches": fwd_n}
    kp = {"kernel": ("k_lr_records + k_lr_reduce_short + k_lr_reduce_long" if args.lr_exact
                     else "k_lr_tiles + k_lr_tiles_fin" if tiles
                     else "k_lr_records + k_lr_reduce_fused") + " (per-key mean + AdaGrad push)",
          "achieved": push_gbs, "frac": push_gbs / HBM_PEAK_GBS,
          "bytes_per_launch": push_bytes / max(push_n, 1), "avg_launch_ms": push_ms / max(push_n, 1),
          "launches": push_n}
    tr, tsrc = pmc_traffic(dict(app="lr", lr_batch=args.lr_batch, exact=bool(args.lr_exact), world=world,
                                sharded=dist is not None),
                           {"forward": ("k_lr_forward_c", "k_lr_forward_r", "k_lr_forward", "k_lr_forward_g"),
                            "push": ("k_lr_records", "k_lr_reduce_fused", "k_lr_reduce_short", "k_lr_reduce_long",
                                     "k_lr_reduce_long_fast", "k_lr_tiles", "k_lr_tiles_fin")})
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
                      "parallelism": ("key-sharded PS over %d GPU(s), %s all-to-all-v%s"
                                      % (world, backend, ", library-issued" if comm is not None else ""))
                      if dist is not None else "1 GPU, one HBM shard",
                      "mode": "exact (sequential fp32 per-key sums, bit-exact with the reference)" if args.lr_exact
                      else "fast (fp64 per-key sums%s; within 1e-5 of the oracle)"
                      % (" through row tiles" if tiles else ", wave tree-reduced"),
                      "features_per_s": total * nnz / max(steps * B1, 1) / dt,
                      "unique_keys_per_step": uniq / steps},
           "roofline": dict(dom, bound="hbm", peak=HBM_PEAK_GBS, unit="GB/s",
                            step_GBps=step_gbs, step_frac=step_gbs / HBM_PEAK_GBS, other=other),
           "kernel_ms": {k: v[0] for k, v in kt.items() if v[1]}}
    if xport is not None:
        out["rccl_ranks" if xport[0] == "rccl" else "transport_ranks"] = xport[1]
        out["transport"] = xport[0]
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
    rank, world, local, dist, backend = ctx
    finish, run_timed = _other_helpers(ctx)
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
    s2 = sw.Sent2Vec(t, window=args.window, negative=args.negative, minibatch=args.s2v_docs, niters=1,
                     alpha=args.alpha)
    s2.load_tokens(toks, off, sent)  # each rank generated its own docs: doc-sharded by construction
    s2.train_batches(warm)
    s2.sync()
    st0 = s2.stats()
    dt = run_timed(s2.train_batches, s2.sync, steps)
    st1 = s2.stats()
    s2.set_profile(True)
    s2.kernel_times(reset=True)
    run_timed(s2.train_batches, s2.sync, steps)
    st2 = s2.stats()
    kt = s2.kernel_times()
    s2.set_profile(False)
    s2.close()
    t.close()
    dt, total = finish(dt, st1["positions"] - st0["positions"])
    # SURVEY.md §8(d) sent2vec bytes of the docs kernel: 4*D per word row read (contexts + targets)
    # + 8*D per document (its row read and written)
    rows_read = (st2["ctx_rows"] - st1["ctx_rows"]) + (st2["tgt_rows"] - st1["tgt_rows"])
    ndocs = st2["docs"] - st1["docs"]
    doc_ms, doc_n = kt["docs"]
    doc_bytes = 4 * D * rows_read + 8 * D * ndocs
    doc_gbs = doc_bytes / (doc_ms * 1e-3) / 1e9 if doc_ms > 0 else 0.0
    tr, tsrc = pmc_traffic(dict(app="s2v", s2v_docs=args.s2v_docs, dim=D, world=world), {"docs": ("k_s2v_docs",)})
    out = {"metric": "sent2vec trained words/sec (frozen word table, doc-sharded)", "value": total / dt,
           "unit": "words/s", "n_gpus": world, "steps": steps, "warmup": warm, "ms_per_step": dt * 1e3 / steps,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32 table, f64 math",
           "data": "synthetic Zipf(s=1) docs of 50-200 tokens over V=1M, hash-initialised word table",
           "config": {"workload": "sent2vec (BASELINE config 5 shape), D=%d, window %d, negative %d, %d docs "
                                  "per minibatch, word table 1M x %d, %d documents"
                                  % (D, args.window, args.negative, args.s2v_docs, D, nd),
                      "parallelism": "doc-sharded over %d GPU(s), no exchange (replicas only)" % world},
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
    no exec).  Rank 0 prints the JSON line; if any rank fails the others are
    stopped and the first failing exit code is returned."""
    import subprocess
    port = _free_port_pair()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    while procs:
        for p in list(procs):
            c = p.poll()
            if c is None:
                continue
            procs.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in procs:  # the others would wait forever in a collective
                    q.terminate()
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
    main()
