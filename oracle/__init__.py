"""ORACLE — test infrastructure only.

ctypes bindings to oracle/libswps_oracle.so, the CPU restatement of SwiftMPI's
hot path (see swps_oracle.cpp's header for what is pinned and how).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module; the product package `swiftmpi_amd` never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libswps_oracle.so")
REF_KAT = os.path.join(HERE, "_ref", "random_kat")

_u64 = ctypes.c_uint64
_p = ctypes.c_void_p


def build(ref=False):
    targets = ["all"] + (["ref"] if ref else [])
    subprocess.check_call(["make", "-s", "-C", HERE] + targets)


class W2VCfg(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int32), ("window", ctypes.c_int32), ("negative", ctypes.c_int32),
                ("min_sentence_length", ctypes.c_int32), ("minibatch", ctypes.c_int32),
                ("storage_f32", ctypes.c_int32), ("sample", ctypes.c_float), ("alpha", ctypes.c_float),
                ("lr", ctypes.c_float), ("table_size", ctypes.c_uint64), ("key_mode", ctypes.c_int32),
                ("minibatch_vocab", ctypes.c_int32)]


class S2VCfg(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int32), ("window", ctypes.c_int32), ("negative", ctypes.c_int32),
                ("min_sentence_length", ctypes.c_int32), ("minibatch", ctypes.c_int32), ("niters", ctypes.c_int32),
                ("storage_f32", ctypes.c_int32), ("alpha", ctypes.c_float), ("table_size", ctypes.c_uint64),
                ("rand_seed", ctypes.c_uint32), ("rand_offset", ctypes.c_uint64),
                ("rand_insert_extra", ctypes.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(
                os.path.join(HERE, "swps_oracle.cpp")):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_bkdr.restype = _u64
        L.orc_bkdr.argtypes = [ctypes.c_char_p]
        L.orc_fmix64.restype = _u64
        L.orc_fmix64.argtypes = [_u64]
        L.orc_hashfrag_table.argtypes = [ctypes.c_int, ctypes.c_int, _p]
        L.orc_to_node_id.argtypes = [_u64, ctypes.c_int, _p]
        L.orc_shard_id.argtypes = [_u64, ctypes.c_int]
        L.orc_lcg_sequence.argtypes = [_u64, _u64, _p]
        L.orc_float_lcg_sequence.argtypes = [_u64, _p, _p]
        L.orc_exptable.argtypes = [_p]
        L.orc_libc_rand_sequence.argtypes = [ctypes.c_uint, _u64, _u64, _p]
        L.orc_last_error.restype = ctypes.c_char_p
        L.orc_w2v_create.restype = _p
        L.orc_w2v_create.argtypes = [ctypes.c_char_p, ctypes.POINTER(W2VCfg)]
        L.orc_w2v_destroy.argtypes = [_p]
        L.orc_set_diag_round.argtypes = [ctypes.c_int]
        for n in ("orc_w2v_vocab_size", "orc_w2v_train_words"):
            getattr(L, n).restype = _u64
            getattr(L, n).argtypes = [_p]
        L.orc_w2v_vocab.argtypes = [_p, _p, _p]
        L.orc_w2v_table_at.argtypes = [_p, _p, _u64, _p]
        L.orc_w2v_table_starts.argtypes = [_p, _p]
        L.orc_w2v_init_rand.argtypes = [_p, ctypes.c_uint, _u64]
        L.orc_w2v_set_params.argtypes = [_p, _p]
        L.orc_w2v_get_params.argtypes = [_p, _p]
        L.orc_w2v_trace_negatives.argtypes = [_p, _u64]
        L.orc_w2v_negatives.restype = _u64
        L.orc_w2v_negatives.argtypes = [_p, _p, _u64]
        L.orc_w2v_train.argtypes = [_p, ctypes.c_int]
        L.orc_w2v_stats.argtypes = [_p, _p]
        L.orc_lr_create.restype = _p
        L.orc_lr_create.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_float]
        L.orc_lr_create_csr.restype = _p
        L.orc_lr_create_csr.argtypes = [_p, _u64, _p, _p, _p, ctypes.c_int, ctypes.c_float]
        L.orc_lr_destroy.argtypes = [_p]
        L.orc_lr_set_sum_f64.argtypes = [_p, ctypes.c_int]
        L.orc_lr_num_instances.restype = _u64
        L.orc_lr_num_instances.argtypes = [_p]
        L.orc_lr_train.argtypes = [_p, ctypes.c_int, _p]
        L.orc_lr_num_keys.restype = _u64
        L.orc_lr_num_keys.argtypes = [_p]
        L.orc_lr_params.argtypes = [_p, _p, _p, _p]
        L.orc_lr_predict.argtypes = [_p, _p, _p]
        L.orc_lr_load.argtypes = [_p, _p, _p, ctypes.c_uint64]
        L.orc_lr_predict_mode.argtypes = [_p, _p]
        L.orc_lr_pull_order.restype = _u64
        L.orc_lr_pull_order.argtypes = [_p, _p, _u64]
        L.orc_s2v_create.restype = _p
        L.orc_s2v_create.argtypes = [ctypes.c_char_p, ctypes.POINTER(S2VCfg)]
        L.orc_s2v_destroy.argtypes = [_p]
        L.orc_s2v_load_words.argtypes = [_p, ctypes.c_char_p]
        L.orc_s2v_train.argtypes = [_p]
        L.orc_s2v_num_docs.restype = _u64
        L.orc_s2v_num_docs.argtypes = [_p]
        L.orc_s2v_docs.argtypes = [_p, _p, _p, _p]
        L.orc_s2v_stats.argtypes = [_p, _p]
        L.orc_s2v_word_rows.argtypes = [_p, _p, _u64, _p]
        L.orc_w2vm_create.restype = _p
        L.orc_w2vm_create.argtypes = [_p, ctypes.c_int, ctypes.POINTER(W2VCfg), _u64]
        L.orc_w2vm_destroy.argtypes = [_p]
        L.orc_w2vm_train.argtypes = [_p, ctypes.c_int]
        L.orc_w2vm_train_steps.argtypes = [_p, _u64]
        L.orc_w2vm_num_keys.restype = _u64
        L.orc_w2vm_num_keys.argtypes = [_p]
        L.orc_w2vm_params.argtypes = [_p, _p, _p]
        L.orc_w2vm_rank_stats.argtypes = [_p, ctypes.c_int, _p]
        L.orc_lrm_create.restype = _p
        L.orc_lrm_create.argtypes = [_p, ctypes.c_int, ctypes.c_int, ctypes.c_float, _u64]
        L.orc_lrm_destroy.argtypes = [_p]
        L.orc_lrm_train.argtypes = [_p, ctypes.c_int]
        L.orc_lrm_num_keys.restype = _u64
        L.orc_lrm_num_keys.argtypes = [_p]
        L.orc_lrm_params.argtypes = [_p, _p, _p, _p]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def bkdr(word):
    if isinstance(word, str):
        word = word.encode("utf-8")
    return int(lib().orc_bkdr(word))


def fmix64(x):
    return int(lib().orc_fmix64(x))


def hashfrag_table(frag_num, num_nodes):
    out = np.zeros(frag_num, dtype=np.uint32)
    if lib().orc_hashfrag_table(frag_num, num_nodes, _ptr(out)) != 0:
        raise ValueError("frag_num < num_nodes")
    return out


def to_node_id(key, frag_num, table):
    return int(lib().orc_to_node_id(key, frag_num, _ptr(table)))


def lcg_sequence(n, seed=2008):
    out = np.zeros(n, dtype=np.uint64)
    lib().orc_lcg_sequence(seed, n, _ptr(out))
    return out


def float_lcg_sequence(n):
    st = np.zeros(n, dtype=np.uint64)
    out = np.zeros(n, dtype=np.float32)
    lib().orc_float_lcg_sequence(n, _ptr(st), _ptr(out))
    return st, out


def exptable():
    out = np.zeros(1000, dtype=np.float32)
    lib().orc_exptable(_ptr(out))
    return out


def libc_rand(n, seed=1, skip=0):
    out = np.zeros(n, dtype=np.int32)
    lib().orc_libc_rand_sequence(seed, skip, n, _ptr(out))
    return out


class W2V:
    """Reference-semantics CBOW-NS trainer (word2vec_global.h, nthreads = 1);
    minibatch_vocab=True: word2vec.h's MiniBatch (w2v_local.cpp) — per-minibatch
    vocab and unigram table."""

    def __init__(self, corpus_path, dim, window=5, negative=5, min_sentence_length=1, minibatch=100,
                 sample=1e-5, alpha=0.05, lr=0.7, table_size=int(1e8), storage_f32=False, key_mode=0,
                 minibatch_vocab=False):
        c = W2VCfg(dim, window, negative, min_sentence_length, minibatch, int(storage_f32), sample, alpha, lr,
                   table_size, key_mode, int(minibatch_vocab))
        self.dim = dim
        self.h = lib().orc_w2v_create(corpus_path.encode(), ctypes.byref(c))
        if not self.h:
            raise RuntimeError(lib().orc_last_error().decode())

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_w2v_destroy(self.h)
            self.h = None

    @property
    def vocab_size(self):
        return int(lib().orc_w2v_vocab_size(self.h))

    @property
    def train_words(self):
        return int(lib().orc_w2v_train_words(self.h))

    def vocab(self):
        V = self.vocab_size
        keys = np.zeros(V, dtype=np.uint64)
        counts = np.zeros(V, dtype=np.int32)
        lib().orc_w2v_vocab(self.h, _ptr(keys), _ptr(counts))
        return keys, counts

    def table_at(self, idx):
        idx = np.ascontiguousarray(idx, dtype=np.uint64)
        out = np.zeros(len(idx), dtype=np.uint32)
        lib().orc_w2v_table_at(self.h, _ptr(idx), len(idx), _ptr(out))
        return out

    def table_starts(self):
        out = np.zeros(self.vocab_size + 1, dtype=np.uint64)
        if lib().orc_w2v_table_starts(self.h, _ptr(out)) != 0:
            raise RuntimeError("unigram table is not run-length ordered")
        return out

    def init_rand(self, seed=1, rand_offset=2):
        if lib().orc_w2v_init_rand(self.h, seed, rand_offset) != 0:
            raise RuntimeError(lib().orc_last_error().decode())

    def set_params(self, hv):
        hv = np.ascontiguousarray(hv, dtype=np.float64)
        assert hv.shape == (self.vocab_size, 2 * self.dim)
        lib().orc_w2v_set_params(self.h, _ptr(hv))

    def get_params(self):
        out = np.zeros((self.vocab_size, 4 * self.dim), dtype=np.float64)
        lib().orc_w2v_get_params(self.h, _ptr(out))
        return out

    def trace_negatives(self, cap):
        lib().orc_w2v_trace_negatives(self.h, cap)

    def negatives(self, cap):
        out = np.zeros(cap, dtype=np.int64)
        n = lib().orc_w2v_negatives(self.h, _ptr(out), cap)
        return out[:n]

    def train(self, niters=1):
        if lib().orc_w2v_train(self.h, niters) != 0:
            raise RuntimeError(lib().orc_last_error().decode())

    def stats(self):
        out = np.zeros(6, dtype=np.uint64)
        lib().orc_w2v_stats(self.h, _ptr(out))
        return dict(zip(["kept", "pushes", "pulls", "actual_train_words", "rng", "frng"], [int(x) for x in out]))


class LR:
    """Reference-semantics sparse logistic regression (lr.cpp, nthreads = 1)."""

    def __init__(self, path, minibatch=200, lr=0.05, sum_f64=False):
        """sum_f64: NOT the reference — each key's gradient terms summed in
        fp64 (mean = float(sum/count)), the definition the rebuild's
        fast_sums mode implements; its distance from the default mode is the
        reference's own fp32-chain rounding."""
        self.h = lib().orc_lr_create(path.encode(), minibatch, lr)
        if not self.h:
            raise RuntimeError(lib().orc_last_error().decode())
        lib().orc_lr_set_sum_f64(self.h, int(sum_f64))

    @classmethod
    def from_csr(cls, labels, row_off, feat, vals, minibatch=200, lr=0.05):
        """The same instances from CSR arrays (labels f32, row_off u64, feat u32, vals f32)."""
        self = cls.__new__(cls)
        a = [np.ascontiguousarray(x, dtype=t) for x, t in
             ((labels, np.float32), (row_off, np.uint64), (feat, np.uint32), (vals, np.float32))]
        self.h = lib().orc_lr_create_csr(_ptr(a[0]), len(a[0]), _ptr(a[1]), _ptr(a[2]), _ptr(a[3]), minibatch, lr)
        if not self.h:
            raise RuntimeError(lib().orc_last_error().decode())
        return self

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_lr_destroy(self.h)
            self.h = None

    def train(self, niters):
        err = np.zeros(niters, dtype=np.float64)
        if lib().orc_lr_train(self.h, niters, _ptr(err)) != 0:
            raise RuntimeError(lib().orc_last_error().decode())
        return err

    def params(self):
        n = int(lib().orc_lr_num_keys(self.h))
        keys = np.zeros(n, dtype=np.uint32)
        w = np.zeros(n, dtype=np.float32)
        g2 = np.zeros(n, dtype=np.float32)
        lib().orc_lr_params(self.h, _ptr(keys), _ptr(w), _ptr(g2))
        return keys, w, g2

    def predict(self):
        n = int(lib().orc_lr_num_instances(self.h))
        p = np.zeros(n, dtype=np.float32)
        t = np.zeros(n, dtype=np.float32)
        lib().orc_lr_predict(self.h, _ptr(p), _ptr(t))
        return p, t

    def load(self, keys, vals):
        """ClusterServer::load of an LR dump: assign, draw nothing (server.h:49-62)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        vals = np.ascontiguousarray(vals, dtype=np.float32)
        lib().orc_lr_load(self.h, _ptr(keys), _ptr(vals), len(keys))

    def predict_mode(self):
        """lr.cpp:240-295: per-minibatch pulls (misses drawn in key-set order), then predictions."""
        p = np.zeros(int(lib().orc_lr_num_instances(self.h)), dtype=np.float32)
        lib().orc_lr_predict_mode(self.h, _ptr(p))
        return p

    def pull_order(self):
        cap = 1 << 26
        n = int(lib().orc_lr_num_keys(self.h)) or 4096
        out = np.zeros(max(n, 1 << 16), dtype=np.uint32)
        m = lib().orc_lr_pull_order(self.h, _ptr(out), len(out))
        return out[:m]


class S2V:
    """Reference-semantics sent2vec (sent2vec.cpp on word2vec.h's MiniBatch,
    nthreads = 1).  rand_offset = rand() calls before load_words."""

    def __init__(self, corpus_path, dim, window=5, negative=5, min_sentence_length=1, minibatch=100, niters=1,
                 alpha=0.05, table_size=int(1e8), storage_f32=False, rand_seed=1, rand_offset=2,
                 rand_insert_extra=0):
        c = S2VCfg(dim, window, negative, min_sentence_length, minibatch, niters, int(storage_f32), alpha,
                   table_size, rand_seed, rand_offset, rand_insert_extra)
        self.dim = dim
        self.h = lib().orc_s2v_create(corpus_path.encode(), ctypes.byref(c))
        if not self.h:
            raise RuntimeError(lib().orc_last_error().decode())

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_s2v_destroy(self.h)
            self.h = None

    def load_words(self, path):
        if lib().orc_s2v_load_words(self.h, path.encode()) != 0:
            raise RuntimeError(lib().orc_last_error().decode())

    def train(self):
        if lib().orc_s2v_train(self.h) != 0:
            raise RuntimeError(lib().orc_last_error().decode())

    def docs(self):
        n = int(lib().orc_s2v_num_docs(self.h))
        ids = np.zeros(max(n, 1), dtype=np.uint64)
        vecs = np.zeros((max(n, 1), self.dim), dtype=np.float64)
        errs = np.zeros(max(n, 1), dtype=np.float32)
        lib().orc_s2v_docs(self.h, _ptr(ids), _ptr(vecs), _ptr(errs))
        return ids[:n], vecs[:n], errs[:n]

    def stats(self):
        out = np.zeros(8, dtype=np.uint64)
        lib().orc_s2v_stats(self.h, _ptr(out))
        d = dict(zip(["batches", "pulled", "inserted", "rand_calls", "draws", "rng", "server_keys", "err_bits"],
                     [int(x) for x in out]))
        d["error_sum"] = float(np.array([d.pop("err_bits")], dtype=np.uint32).view(np.float32)[0])
        return d

    def word_rows(self, keys):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        out = np.zeros((len(keys), 2 * self.dim), dtype=np.float64)
        rc = lib().orc_s2v_word_rows(self.h, _ptr(keys), len(keys), _ptr(out))
        return out, rc == 0


def _cstrings(paths):
    arr = (ctypes.c_char_p * len(paths))(*[p.encode() for p in paths])
    return ctypes.cast(arr, ctypes.c_void_p), arr


class W2VMulti:
    """Lockstep multi-rank word2vec (swps_oracle.cpp W2VMulti): one worker per
    corpus path, one server map, hash-initialised keys (the sharded tables'
    SWPS_INIT_HASH with `seed`), every rank's push its own AdaGrad step in
    rank order."""

    def __init__(self, paths, dim, window=5, negative=5, min_sentence_length=1, minibatch=100, sample=1e-5,
                 alpha=0.05, lr=0.7, table_size=int(1e8), storage_f32=False, seed=0):
        c = W2VCfg(dim, window, negative, min_sentence_length, minibatch, int(storage_f32), sample, alpha, lr,
                   table_size, 0, 0)
        self.dim = dim
        pp, self._keep = _cstrings(paths)
        self.h = lib().orc_w2vm_create(pp, len(paths), ctypes.byref(c), seed)
        if not self.h:
            raise RuntimeError(lib().orc_last_error().decode())
        self.R = len(paths)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_w2vm_destroy(self.h)
            self.h = None

    def train(self, niters=1):
        if lib().orc_w2vm_train(self.h, niters) != 0:
            raise RuntimeError(lib().orc_last_error().decode())

    def train_steps(self, n):
        """The next n lockstep steps (one minibatch per rank each; epochs wrap)."""
        if lib().orc_w2vm_train_steps(self.h, n) != 0:
            raise RuntimeError(lib().orc_last_error().decode())

    def params(self):
        """(keys ascending, rows [n][4D] = h | v | h2sum | v2sum)"""
        n = int(lib().orc_w2vm_num_keys(self.h))
        keys = np.zeros(n, dtype=np.uint64)
        rows = np.zeros((n, 4 * self.dim), dtype=np.float64)
        lib().orc_w2vm_params(self.h, _ptr(keys), _ptr(rows))
        return keys, rows

    def rank_stats(self, r):
        out = np.zeros(6, dtype=np.uint64)
        lib().orc_w2vm_rank_stats(self.h, r, _ptr(out))
        return dict(zip(["kept", "pushes", "pulls", "actual_train_words", "rng", "frng"], [int(x) for x in out]))


class LRMulti:
    """Lockstep multi-rank sparse LR (swps_oracle.cpp LRMulti)."""

    def __init__(self, paths, minibatch=200, lr=0.05, seed=0):
        pp, self._keep = _cstrings(paths)
        self.h = lib().orc_lrm_create(pp, len(paths), minibatch, lr, seed)
        if not self.h:
            raise RuntimeError(lib().orc_last_error().decode())

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_lrm_destroy(self.h)
            self.h = None

    def train(self, niters):
        if lib().orc_lrm_train(self.h, niters) != 0:
            raise RuntimeError(lib().orc_last_error().decode())

    def params(self):
        n = int(lib().orc_lrm_num_keys(self.h))
        keys = np.zeros(n, dtype=np.uint32)
        w = np.zeros(n, dtype=np.float32)
        g2 = np.zeros(n, dtype=np.float32)
        lib().orc_lrm_params(self.h, _ptr(keys), _ptr(w), _ptr(g2))
        return keys, w, g2


def logloss_accuracy(p, y, eps=1e-15):
    p = np.clip(np.asarray(p, dtype=np.float64), eps, 1 - eps)
    y = np.asarray(y, dtype=np.float64)
    ll = -np.mean(y * np.log(p) + (1 - y) * np.log(1 - p))
    acc = np.mean((p > 0.5) == (y > 0.5))
    return float(ll), float(acc)
