"""swiftmpi_amd — MI355X-native rebuild of SwiftMPI's data-parallel hot path.

The pull -> gradient -> push loop of SwiftMPI's sparse parameter server
(word2vec CBOW negative sampling, sparse logistic regression) runs as HIP
kernels over HBM-resident key-hash-sharded tables (libswps.so, C ABI in
include/swps.h).  This package is the Python mirror of the reference's app
interfaces over that ABI:

    Table     <- parameter/sparsetable.h + cluster/server.h pull/push handlers
    Word2Vec  <- apps/word2vec/word2vec_global.h  (Word2Vec<MiniBatch>)
    Sent2Vec  <- apps/sent2vec/sent2vec.cpp       (Sent2Vec)
    LR        <- apps/logistic/lr.cpp             (LR)
    Config    <- utils/ConfigParser.h

Every compute call goes through libswps.so; if it is missing the import of the
classes below raises (no CPU fallback).
"""
import ctypes
import weakref

import numpy as np

from . import capi
from .capi import SwpsError, check, ptr

__all__ = ["Table", "Word2Vec", "Sent2Vec", "LR", "Config", "SwpsError", "bkdr", "fmix64", "hashfrag_table",
           "to_node_id", "load_library"]


def load_library():
    return capi.lib()


def bkdr(word):
    """BKDRHash<size_t>(word, 13131) (utils/string.h:130-137)."""
    if isinstance(word, str):
        word = word.encode("utf-8")
    return int(capi.lib().swps_bkdr(word))


def fmix64(x):
    return int(capi.lib().swps_fmix64(x))


def hashfrag_table(frag_num, num_nodes):
    out = np.zeros(frag_num, dtype=np.uint32)
    check(capi.lib().swps_hashfrag_table(frag_num, num_nodes, ptr(out)))
    return out


def to_node_id(keys, frag_num, table):
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    out = np.zeros(len(keys), dtype=np.int32)
    check(capi.lib().swps_to_node_id(ptr(keys), len(keys), frag_num, ptr(table), ptr(out)))
    return out


def unigram_starts(keys, counts, table_size=int(1e8)):
    """Run-length form of gen_unigram_table (host helper of libswps)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    counts = np.ascontiguousarray(counts, dtype=np.int32)
    out = np.zeros(len(keys) + 1, dtype=np.uint64)
    check(capi.lib().swps_unigram_starts(ptr(keys), ptr(counts), len(keys), table_size, ptr(out)))
    return out


def glibc_rand(n, seed=1, skip=0):
    out = np.zeros(n, dtype=np.int32)
    check(capi.lib().swps_glibc_rand(seed, skip, n, ptr(out)))
    return out


class Config:
    """The reference's INI-like config (utils/ConfigParser.h:84-115):
    ``[section]`` headers, ``key: value`` lines, ``#`` comments, ``import path``.
    ``get(section, key)`` raises KeyError like the reference's CHECK."""

    def __init__(self, path=None):
        self.sections = {}
        if path:
            self.parse(path)

    def parse(self, path):
        cur = ""
        with open(path) as f:
            for line in f:
                line = line.strip(" \t\n\r")
                if not line or line.startswith("#"):
                    continue
                if line.startswith("import"):
                    sub = line.split(" ", 1)[1].strip()
                    if sub == path:
                        raise ValueError("recursive import")
                    self.parse(sub)
                    continue
                if line[0] == "[" and line[-1] == "]":
                    cur = line[1:-1].strip()
                    if not cur:
                        raise ValueError("empty section")
                    continue
                if ":" not in line:
                    raise ValueError(f"bad config line: {line}")
                k, v = line.split(":", 1)
                self.sections.setdefault(cur, {}).setdefault(k.strip(), v.strip())
        return self

    def get(self, section, key):
        try:
            return self.sections[section][key]
        except KeyError:
            raise KeyError(f"no such key:\t[{section}]\t{key}")

    def get_int(self, section, key):
        return int(self.get(section, key))

    def get_float(self, section, key):
        return float(self.get(section, key))


class Table:
    """One HBM parameter shard (SparseTable + server access methods)."""

    def __init__(self, layout="w2v", dim=100, capacity=1 << 20, dtype="f32", learning_rate=0.7, fudge=1e-6,
                 init="hash", seed=0, device=0, push_rule="adagrad"):
        inits = {"hash": capi.INIT_HASH, "zero": capi.INIT_ZERO, "flcg": capi.INIT_FLCG}
        rules = {"adagrad": capi.PUSH_ADAGRAD, "sgd": capi.PUSH_SGD}
        layouts = {"w2v": capi.LAYOUT_W2V, "lr": capi.LAYOUT_LR}
        dtypes = {"f32": capi.F32, "f64": capi.F64}
        for name, val, known in (("init", init, inits), ("push_rule", push_rule, rules), ("layout", layout, layouts),
                                 ("dtype", dtype, dtypes)):
            if val not in known:
                raise ValueError("unknown %s %r (one of %s)" % (name, val, ", ".join(sorted(known))))
        cfg = capi.TableCfg(device, layouts[layout], dtypes[dtype], dim, capacity, learning_rate, fudge,
                            inits[init], seed, rules[push_rule])
        h = ctypes.c_void_p()
        check(capi.lib().swps_table_create(ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h
        self.layout, self.dim, self.dtype, self.device = layout, dim, dtype, device
        r, p, q = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        capi.lib().swps_table_row_elems(self.h, ctypes.byref(r), ctypes.byref(p), ctypes.byref(q))
        self.row_elems, self.pull_elems, self.push_elems = r.value, p.value, q.value
        self._deps = weakref.WeakSet()  # app contexts bound to this shard: closed first

    def close(self):
        if getattr(self, "h", None):
            for d in list(getattr(self, "_deps", ())):
                d.close()
            capi.lib().swps_table_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except (AttributeError, TypeError):  # interpreter shutdown: modules already torn down
            pass

    @property
    def torch_dtype(self):
        import torch
        return torch.float64 if self.dtype == "f64" else torch.float32

    def size(self):
        n = ctypes.c_uint64()
        check(capi.lib().swps_table_size(self.h, ctypes.byref(n)))
        return n.value

    def pull(self, keys):
        """keys: int64/uint64 CUDA tensor of distinct keys -> [n, pull_elems] tensor."""
        import torch
        out = torch.empty((keys.numel(), self.pull_elems), dtype=self.torch_dtype, device=keys.device)
        check(capi.lib().swps_pull(self.h, ptr(keys), keys.numel(), ptr(out)))
        return out

    def push(self, keys, grads):
        """grads: [n, push_elems] CUDA tensor, fp64 (w2v) or fp32 (lr) — the reference wire types."""
        check(capi.lib().swps_push(self.h, ptr(keys), keys.numel(), ptr(grads)))
        capi.lib().swps_table_sync(self.h)

    def assign(self, keys, rows):
        check(capi.lib().swps_assign(self.h, ptr(keys), keys.numel(), ptr(rows)))

    def export(self, keys):
        import torch
        out = torch.empty((keys.numel(), self.row_elems), dtype=self.torch_dtype, device=keys.device)
        check(capi.lib().swps_export(self.h, ptr(keys), keys.numel(), ptr(out)))
        return out

    def keys(self):
        n = self.size()
        out = np.zeros(max(n, 1), dtype=np.uint64)
        m = ctypes.c_uint64()
        check(capi.lib().swps_table_keys(self.h, ptr(out), len(out), ctypes.byref(m)))
        return out[:m.value]

    def dump(self, path):
        check(capi.lib().swps_dump(self.h, path.encode()))

    def load(self, path, frag_num=1000, world=1, node_id=0):
        check(capi.lib().swps_load(self.h, path.encode(), frag_num, world, node_id))

    def save(self, path):
        """Binary snapshot of every key and row, bit for bit (swps_save)."""
        check(capi.lib().swps_save(self.h, path.encode()))

    def restore(self, path, frag_num=1000, world=1, node_id=0):
        """Assign the rows of a swps_save snapshot (node_id's keys only when
        world > 1, as `load`); the file is verified before any row changes."""
        check(capi.lib().swps_restore(self.h, path.encode(), frag_num, world, node_id))

    # ---- key-sharded mode (swps_table_route): pull / push become collective ----
    def route(self, comm, frag_num=1000):
        check(capi.lib().swps_table_route(self.h, comm.h, frag_num))
        self._comm = comm  # the communicator must outlive the routed table

    def finish(self):
        check(capi.lib().swps_finish(self.h))

    def barrier(self):
        check(capi.lib().swps_barrier(self.h))

    def route_stats(self):
        out = np.zeros(6, dtype=np.uint64)
        check(capi.lib().swps_route_stats(self.h, ptr(out)))
        return dict(zip(["rounds", "keys_sent", "keys_remote", "bytes_sent", "bytes_remote", "keys_served"],
                        (int(x) for x in out)))

    def pull_h(self, keys):
        """Host keys (uint64) -> host pull values in the wire type (W2V fp64, LR fp32)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        out = np.zeros((len(keys), self.pull_elems), dtype=np.float64 if self.layout == "w2v" else np.float32)
        check(capi.lib().swps_pull_h(self.h, ptr(keys), len(keys), ptr(out)))
        return out

    def push_h(self, keys, grads):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        grads = np.ascontiguousarray(grads, dtype=np.float64 if self.layout == "w2v" else np.float32)
        check(capi.lib().swps_push_h(self.h, ptr(keys), len(keys), ptr(grads)))


KT_NAMES = ["plan", "forward", "sort", "gather", "push", "pull", "records"]


INTERMEDIATES = {False: 0, True: 1, "fp32": 0, "fp64": 1, "bfp40": 2, "bfp32": 3, 0: 0, 1: 1, 2: 2, 3: 3}


class Word2Vec:
    """CBOW negative-sampling word2vec (Word2Vec<MiniBatch>, word2vec_global.h:541-748).

    fp64_intermediates (fp32 tables): True / "fp64" = parity mode (neu1/neu1e and
    sums in fp64), False / "fp32" = fast mode (fp32 intermediates), "bfp40" /
    "bfp32" = block-floating-point neu1/neu1e rows (int32 + int8 / int32
    mantissas, one exponent per row) with fp64 sums (swps_w2v_bfp.h)."""

    def __init__(self, table, window=5, negative=5, min_sentence_length=1, minibatch=100, sample=1e-5, alpha=0.05,
                 unigram_size=int(1e8), key_mode="bkdr", init="ref", rand_seed=1, rand_offset=2, profile=False,
                 fp64_intermediates=True, minibatch_vocab=False, sampler="table", host_ingest=False):
        assert table.layout == "w2v"
        cfg = capi.W2VCfg(window, negative, min_sentence_length, minibatch, sample, alpha, unigram_size,
                          capi.KEY_ATOI if key_mode == "atoi" else capi.KEY_BKDR,
                          capi.W2V_INIT_REF if init == "ref" else capi.W2V_INIT_TABLE, rand_seed, rand_offset,
                          INTERMEDIATES[fp64_intermediates], int(profile), int(minibatch_vocab),
                          {"table": 0, "alias": 1}[sampler], int(host_ingest))
        h = ctypes.c_void_p()
        check(capi.lib().swps_w2v_create(table.h, ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h
        table._deps.add(self)
        self.table = table
        self.dim = table.dim

    def shard_comm(self, comm, frag_num=1000):
        """Library-driven key-sharded mode (swps_w2v_shard_comm): after load_*,
        init() is the first full pull and train_batches / train run lockstep
        minibatches over `comm` (collective).  The table must use init="hash"
        and this context init="table"."""
        check(capi.lib().swps_w2v_shard_comm(self.h, comm.h, frag_num))
        self._comm = comm

    def exchange_stats(self, on=-1):
        out = np.zeros(4)
        check(capi.lib().swps_w2v_exchange_stats(self.h, on, ptr(out)))
        return dict(zip(["bytes_remote", "bytes_total", "calls", "ms"], out.tolist()))

    @classmethod
    def from_config(cls, config, table_kwargs=None, **kw):
        """Build a Table + Word2Vec from the reference's demo.conf keys."""
        c = config if isinstance(config, Config) else Config(config)
        dim = c.get_int("word2vec", "len_vec")
        tk = dict(layout="w2v", dim=dim, learning_rate=c.get_float("server", "initial_learning_rate"))
        tk.update(table_kwargs or {})
        t = Table(**tk)
        args = dict(window=c.get_int("word2vec", "window"), negative=c.get_int("word2vec", "negative"),
                    min_sentence_length=c.get_int("word2vec", "min_sentence_length"),
                    minibatch=c.get_int("worker", "minibatch"), sample=c.get_float("word2vec", "sample"),
                    alpha=c.get_float("word2vec", "learning_rate"))
        args.update(kw)
        return cls(t, **args)

    def close(self):
        if getattr(self, "h", None):
            capi.lib().swps_w2v_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except (AttributeError, TypeError):  # interpreter shutdown: modules already torn down
            pass

    def load_text(self, path):
        check(capi.lib().swps_w2v_load_text(self.h, path.encode()))

    def load_tokens(self, word_ids, line_off, word_keys):
        word_ids = np.ascontiguousarray(word_ids, dtype=np.uint32)
        line_off = np.ascontiguousarray(line_off, dtype=np.uint64)
        word_keys = np.ascontiguousarray(word_keys, dtype=np.uint64)
        check(capi.lib().swps_w2v_load_tokens(self.h, ptr(word_ids), len(word_ids), ptr(line_off),
                                               len(line_off) - 1, ptr(word_keys), len(word_keys)))

    def info(self):
        o = np.zeros(8, dtype=np.uint64)
        check(capi.lib().swps_w2v_info(self.h, ptr(o)))
        return dict(zip(["vocab", "train_words", "lines", "tokens", "batches", "max_batch_tokens", "lstate",
                         "fstate"], [int(x) for x in o]))

    def vocab(self):
        V = self.info()["vocab"]
        keys = np.zeros(V, dtype=np.uint64)
        counts = np.zeros(V, dtype=np.int32)
        n = ctypes.c_uint64()
        check(capi.lib().swps_w2v_vocab(self.h, ptr(keys), ptr(counts), V, ctypes.byref(n)))
        return keys, counts

    def corpus(self):
        """(vid per token, line per token) — introspection for the ingest tests."""
        n = self.info()["tokens"]
        vid = np.zeros(max(n, 1), dtype=np.int32)
        line = np.zeros(max(n, 1), dtype=np.int32)
        check(capi.lib().swps_w2v_corpus(self.h, ptr(vid), ptr(line), len(vid)))
        return vid[:n], line[:n]

    def batch_keys(self, b):
        """(l0, l1, sorted vids of the gathered key set) of schedule batch b."""
        n = ctypes.c_uint64()
        lines = np.zeros(2, dtype=np.uint64)
        capi.lib().swps_w2v_batch_keys(self.h, b, None, 0, ctypes.byref(n), ptr(lines))
        out = np.zeros(max(n.value, 1), dtype=np.int32)
        check(capi.lib().swps_w2v_batch_keys(self.h, b, ptr(out), len(out), ctypes.byref(n), ptr(lines)))
        return int(lines[0]), int(lines[1]), out[:n.value]

    def init(self):
        check(capi.lib().swps_w2v_init(self.h))

    def train_batches(self, count):
        check(capi.lib().swps_w2v_train_batches(self.h, count))

    def train(self, niters=1):
        check(capi.lib().swps_w2v_train_epochs(self.h, niters))

    def sync(self):
        check(capi.lib().swps_w2v_sync(self.h))

    def stats(self):
        o = np.zeros(10, dtype=np.uint64)
        check(capi.lib().swps_w2v_stats(self.h, ptr(o)))
        return dict(zip(["batches", "kept", "words", "pairs", "lstate", "fstate", "pulled", "pushed", "ctx_rows",
                         "tgt_rows"], [int(x) for x in o]))

    def gather_stats(self):
        """Cumulative gather work: gradient records summed and gather items (chunks)."""
        o = np.zeros(2, dtype=np.uint64)
        check(capi.lib().swps_w2v_gather_stats(self.h, ptr(o)))
        return {"records": int(o[0]), "items": int(o[1])}

    def sum_stats(self):
        """Cumulative gradient-sum work split by kernel: all records / items, the
        multi-chunk runs' records / items (k_gather_t's share when the push is fused),
        fused pushes and batches with sums."""
        o = np.zeros(8, dtype=np.uint64)
        check(capi.lib().swps_w2v_sum_stats(self.h, ptr(o)))
        return dict(zip(["records", "items", "multi_records", "multi_items", "fused", "batches", "fused_grads",
                         "split"], [int(x) for x in o]))

    def get_params(self):
        V = self.info()["vocab"]
        out = np.zeros((V, 4 * self.dim), dtype=np.float64)
        check(capi.lib().swps_w2v_get_params(self.h, ptr(out)))
        return out

    def set_params(self, hv):
        hv = np.ascontiguousarray(hv, dtype=np.float64)
        check(capi.lib().swps_w2v_set_params(self.h, ptr(hv)))

    def unigram_at(self, idx):
        idx = np.ascontiguousarray(idx, dtype=np.uint64)
        out = np.zeros(len(idx), dtype=np.uint32)
        check(capi.lib().swps_w2v_unigram_at(self.h, ptr(idx), len(idx), ptr(out)))
        return out

    def trace_negatives(self, cap):
        check(capi.lib().swps_w2v_trace_negatives(self.h, cap))

    def negatives(self, cap):
        out = np.zeros(max(cap, 1), dtype=np.int64)
        n = ctypes.c_uint64()
        check(capi.lib().swps_w2v_negatives(self.h, ptr(out), cap, ctypes.byref(n)))
        return out[:n.value]

    def kernel_times(self, reset=False):
        o = np.zeros(2 * len(KT_NAMES), dtype=np.float64)
        check(capi.lib().swps_w2v_kernel_times(self.h, ptr(o), int(reset)))
        return {k: (o[2 * i], int(o[2 * i + 1])) for i, k in enumerate(KT_NAMES)}

    def set_profile(self, on):
        check(capi.lib().swps_w2v_set_profile(self.h, int(on)))

    def stream(self):
        return capi.lib().swps_w2v_stream(self.h)

    def save_state(self, path):
        """Worker checkpoint: batch cursor, RNG streams, counters, cache."""
        check(capi.lib().swps_w2v_save_state(self.h, path.encode()))

    def restore_state(self, path):
        """Resume a fresh context (corpus loaded, not initialised) whose table
        already holds the vocab rows."""
        check(capi.lib().swps_w2v_restore_state(self.h, path.encode()))

    def save(self, prefix):
        """Exact resume point: <prefix>.table (the shard) + <prefix>.w2v."""
        self.sync()
        self.table.save(prefix + ".table")
        self.save_state(prefix + ".w2v")

    def restore(self, prefix):
        self.table.restore(prefix + ".table")
        self.restore_state(prefix + ".w2v")


class Sent2Vec:
    """Sentence vectors against frozen word vectors (Sent2Vec, sent2vec.cpp:14-195,
    on word2vec.h's MiniBatch: per-minibatch vocab and unigram table).

    glibc rand() bookkeeping (the sentence vectors and the rows of keys a pull
    misses come from it): ``rand_offset`` = calls before load_word_vector (the
    two port binds by default); ``rand_insert_extra`` = extra calls per key the
    server inserts — 0 for a map that does not construct a value on insert,
    2*dim for sparsehash's dense_hash_map::operator[] (then also add 2*dim per
    SparseTable shard to ``rand_offset`` for set_empty_key)."""

    def __init__(self, table, window=5, negative=5, min_sentence_length=1, minibatch=100, niters=1, alpha=0.05,
                 unigram_size=int(1e8), rand_seed=1, rand_offset=2, rand_insert_extra=0, profile=False):
        assert table.layout == "w2v"
        self.table = table
        self.dim = table.dim
        self.kw = dict(window=window, negative=negative, min_sentence_length=min_sentence_length,
                       minibatch=minibatch, niters=niters, alpha=alpha, unigram_size=unigram_size,
                       rand_seed=rand_seed, rand_insert_extra=rand_insert_extra, profile=int(profile))
        self.rand_offset = rand_offset
        self.h = None

    @classmethod
    def from_config(cls, config, table, niters, **kw):
        c = config if isinstance(config, Config) else Config(config)
        args = dict(window=c.get_int("word2vec", "window"), negative=c.get_int("word2vec", "negative"),
                    min_sentence_length=c.get_int("word2vec", "min_sentence_length"),
                    minibatch=c.get_int("worker", "minibatch"), alpha=c.get_float("word2vec", "learning_rate"),
                    niters=niters)
        args.update(kw)
        return cls(table, **args)

    def load_word_vector(self, path, frag_num=1000, world=1, node_id=0):
        """ClusterServer::load (server.h:49-62): one WParam (2*dim rand()) is
        constructed first, then every owned key of the dump is assigned."""
        before = self.table.size()
        self.table.load(path, frag_num, world, node_id)
        inserted = self.table.size() - before
        self.rand_offset += 2 * self.dim + self.kw["rand_insert_extra"] * inserted

    def _create(self):
        if self.h is None:
            k = self.kw
            cfg = capi.S2VCfg(k["window"], k["negative"], k["min_sentence_length"], k["minibatch"], k["niters"],
                              k["alpha"], k["unigram_size"], k["rand_seed"], self.rand_offset,
                              k["rand_insert_extra"], k["profile"])
            h = ctypes.c_void_p()
            check(capi.lib().swps_s2v_create(self.table.h, ctypes.byref(cfg), ctypes.byref(h)))
            self.h = h
            self.table._deps.add(self)
            if getattr(self, "_shard", None):
                check(capi.lib().swps_s2v_shard(self.h, *self._shard))

    def close(self):
        if getattr(self, "h", None):
            capi.lib().swps_s2v_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except (AttributeError, TypeError):  # interpreter shutdown: modules already torn down
            pass

    def load_text(self, path):
        self._create()
        check(capi.lib().swps_s2v_load_text(self.h, path.encode()))

    def load_tokens(self, tok_keys, line_off, sent_ids):
        self._create()
        tok_keys = np.ascontiguousarray(tok_keys, dtype=np.uint64)
        line_off = np.ascontiguousarray(line_off, dtype=np.uint64)
        sent_ids = np.ascontiguousarray(sent_ids, dtype=np.uint64)
        assert len(sent_ids) == len(line_off) - 1
        check(capi.lib().swps_s2v_load_tokens(self.h, ptr(tok_keys), len(tok_keys), ptr(line_off),
                                               len(line_off) - 1, ptr(sent_ids)))

    def run_tokens(self, tok_keys, line_off, sent_ids):
        """The reference's single pass (Sent2Vec::train, sent2vec.cpp:95-103): load and train every
        minibatch once, the host's per-minibatch work overlapped with the GPU's training
        (swps_s2v_run_tokens; = load_tokens + train bit for bit)."""
        self._create()
        tok_keys = np.ascontiguousarray(tok_keys, dtype=np.uint64)
        line_off = np.ascontiguousarray(line_off, dtype=np.uint64)
        sent_ids = np.ascontiguousarray(sent_ids, dtype=np.uint64)
        assert len(sent_ids) == len(line_off) - 1
        check(capi.lib().swps_s2v_run_tokens(self.h, ptr(tok_keys), len(tok_keys), ptr(line_off),
                                              len(line_off) - 1, ptr(sent_ids)))

    def shard(self, rank, world, frag_num=1000):
        """Keep only the documents BasicHashFrag assigns to `rank` (call before
        loading; config 5's doc-sharded layout, no exchange)."""
        self._shard = (rank, world, frag_num)

    def info(self):
        o = np.zeros(9, dtype=np.uint64)
        check(capi.lib().swps_s2v_info(self.h, ptr(o)))
        return dict(zip(["lines", "docs", "batches", "tokens", "inserted", "max_batch_docs", "max_batch_records",
                         "rand_calls", "lstate"], [int(x) for x in o]))

    def train(self):
        check(capi.lib().swps_s2v_train(self.h))

    def train_batches(self, count):
        check(capi.lib().swps_s2v_train_batches(self.h, count))

    def sync(self):
        check(capi.lib().swps_s2v_sync(self.h))

    def docs(self):
        """(sentence ids, vectors [n, dim] fp64, per-sentence g*g of the last pass)."""
        n = self.info()["docs"]
        ids = np.zeros(max(n, 1), dtype=np.uint64)
        vecs = np.zeros((max(n, 1), self.dim), dtype=np.float64)
        errs = np.zeros(max(n, 1), dtype=np.float32)
        m = ctypes.c_uint64()
        check(capi.lib().swps_s2v_docs(self.h, ptr(ids), ptr(vecs), ptr(errs), len(ids), ctypes.byref(m)))
        return ids[:n], vecs[:n], errs[:n]

    def error(self):
        """Error::norm() of the run (sent2vec.cpp:80,105): float mean of g*g."""
        _, _, errs = self.docs()
        acc = np.float32(0)
        for e in errs:
            acc = np.float32(acc + e)
        return float(acc / np.float32(len(errs))) if len(errs) else float("nan")

    def dump(self, path):
        check(capi.lib().swps_s2v_dump(self.h, path.encode()))

    def stats(self):
        o = np.zeros(5, dtype=np.uint64)
        check(capi.lib().swps_s2v_stats(self.h, ptr(o)))
        return dict(zip(["batches", "docs", "positions", "ctx_rows", "tgt_rows"], [int(x) for x in o]))

    def set_profile(self, on):
        check(capi.lib().swps_s2v_set_profile(self.h, int(on)))

    def kernel_times(self, reset=False):
        o = np.zeros(4, dtype=np.float64)
        check(capi.lib().swps_s2v_kernel_times(self.h, ptr(o), int(reset)))
        return {k: (o[2 * i], int(o[2 * i + 1])) for i, k in enumerate(["records", "docs"])}

    def stream(self):
        return capi.lib().swps_s2v_stream(self.h)


class LR:
    """Sparse logistic regression with server-side AdaGrad (lr.cpp:133-411)."""

    def __init__(self, table, minibatch=200, init_ref=True, profile=False, fast_sums=False, plan="step"):
        """plan: "step" builds each minibatch's index inside its step (beside the previous step,
        lr.cpp:215-227's per-minibatch gather; single GPU with fast_sums), "load" every
        minibatch's index once at load (reused each epoch).  Same results."""
        assert table.layout == "lr"
        plans = {"step": capi.LR_PLAN_STEP, "load": capi.LR_PLAN_LOAD, "none": capi.LR_PLAN_NONE}
        if plan not in plans:
            raise ValueError("unknown plan %r (step, load or none)" % (plan,))
        cfg = capi.LRCfg(minibatch, int(init_ref), int(profile), int(fast_sums), plans[plan])
        h = ctypes.c_void_p()
        check(capi.lib().swps_lr_create(table.h, ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h
        table._deps.add(self)
        self.table = table

    def shard_comm(self, comm, frag_num=2000):
        """Library-driven key-sharded LR (swps_lr_shard_comm): init / train /
        train_batches / predict become collective over `comm`."""
        check(capi.lib().swps_lr_shard_comm(self.h, comm.h, frag_num))
        self._comm = comm

    def exchange_stats(self, on=-1):
        """As Word2Vec.exchange_stats (swps_lr_exchange_stats)."""
        out = np.zeros(4)
        check(capi.lib().swps_lr_exchange_stats(self.h, on, ptr(out)))
        return dict(zip(["bytes_remote", "bytes_total", "calls", "ms"], out.tolist()))

    def plan_info(self):
        """swps_lr_plan_info: the plan the step runs and the fixed point's scale against its floor
        (fallback True: plan "none" was asked for, heavy-tailed x_i put the scale below the floor,
        and the load switched to plan "step", fp64 sums)."""
        o = np.zeros(5, dtype=np.int32)
        check(capi.lib().swps_lr_plan_info(self.h, ptr(o)))
        names = {0: "step", 1: "load", 2: "none"}
        return {"plan": names.get(int(o[0]), int(o[0])), "plan_asked": names.get(int(o[1]), int(o[1])),
                "fx_bits": int(o[2]), "fx_floor": int(o[3]), "fallback": bool(o[4])}

    def fx_bytes(self, batch):
        """The fixed-point step's algorithmic bytes on `batch` (swps_lr_fx_bytes): a dict with
        step / push bytes, form (1 bucketed, 2 atomic, 0 other plan), hot, buckets, blocks,
        nonhot records, distinct nonhot keys."""
        out = np.zeros(8, dtype=np.uint64)
        check(capi.lib().swps_lr_fx_bytes(self.h, batch, ptr(out)))
        return dict(zip(["step", "push", "form", "hot", "buckets", "blocks", "nonhot", "uniq"],
                        [int(x) for x in out]))

    def close(self):
        if getattr(self, "h", None):
            capi.lib().swps_lr_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except (AttributeError, TypeError):  # interpreter shutdown: modules already torn down
            pass

    def load_text(self, path):
        check(capi.lib().swps_lr_load_text(self.h, path.encode()))

    def load_csr(self, labels, row_off, feat, vals):
        labels = np.ascontiguousarray(labels, dtype=np.float32)
        row_off = np.ascontiguousarray(row_off, dtype=np.uint64)
        feat = np.ascontiguousarray(feat, dtype=np.uint32)
        vals = np.ascontiguousarray(vals, dtype=np.float32)
        check(capi.lib().swps_lr_load_csr(self.h, ptr(labels), len(labels), ptr(row_off), ptr(feat), ptr(vals)))

    def init(self):
        check(capi.lib().swps_lr_init(self.h))

    def train(self, niters):
        err = np.zeros(niters, dtype=np.float64)
        check(capi.lib().swps_lr_train(self.h, niters, ptr(err)))
        return err

    def train_batches(self, count):
        check(capi.lib().swps_lr_train_batches(self.h, count))

    def sync(self):
        check(capi.lib().swps_lr_sync(self.h))

    def info(self):
        o = np.zeros(4, dtype=np.uint64)
        check(capi.lib().swps_lr_info(self.h, ptr(o)))
        return dict(zip(["rows", "keys", "batches", "nnz"], [int(x) for x in o]))

    def predict(self):
        n = self.info()["rows"]
        p = np.zeros(n, dtype=np.float32)
        t = np.zeros(n, dtype=np.float32)
        check(capi.lib().swps_lr_predict(self.h, ptr(p), ptr(t), n))
        return p, t

    def params(self):
        n = self.info()["keys"]
        keys = np.zeros(max(n, 1), dtype=np.uint32)
        w = np.zeros(max(n, 1), dtype=np.float32)
        g2 = np.zeros(max(n, 1), dtype=np.float32)
        m = ctypes.c_uint64()
        check(capi.lib().swps_lr_params(self.h, ptr(keys), ptr(w), ptr(g2), len(keys), ctypes.byref(m)))
        return keys[:m.value], w[:m.value], g2[:m.value]

    def set_profile(self, on):
        check(capi.lib().swps_lr_set_profile(self.h, int(on)))

    def kernel_times(self, reset=False):
        o = np.zeros(8, dtype=np.float64)
        check(capi.lib().swps_lr_kernel_times(self.h, ptr(o), int(reset)))
        return {k: (o[2 * i], int(o[2 * i + 1])) for i, k in enumerate(["forward", "sort", "gather", "push"])}
