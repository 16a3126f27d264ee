"""ctypes binding of include/swps.h (libswps.so).

The product's compute path is the HIP library; this module only loads it and
declares the C ABI.  It fails loudly when the library is missing — there is no
CPU fallback anywhere in the package.
"""
import ctypes
import os

from . import build as _build

LIB_PATH = os.environ.get("SWPS_LIB", _build.LIB)  # SWPS_LIB: A/B timing of another in-tree build

SWPS_OK = 0
ERRORS = {-1: "SWPS_E_OOM", -2: "SWPS_E_BADKEY", -3: "SWPS_E_HIP", -4: "SWPS_E_RCCL", -5: "SWPS_E_CFG",
          -6: "SWPS_E_STATE", -7: "SWPS_E_UNSUPPORTED", -8: "SWPS_E_IO"}
LAYOUT_W2V, LAYOUT_LR = 0, 1
F32, F64 = 0, 1
INIT_ZERO, INIT_HASH, INIT_FLCG = 0, 1, 2
KEY_BKDR, KEY_ATOI = 0, 1
W2V_INIT_REF, W2V_INIT_TABLE = 0, 1
PUSH_ADAGRAD, PUSH_SGD = 0, 1
LR_PLAN_STEP, LR_PLAN_LOAD, LR_PLAN_NONE = 0, 1, 2
COMM_ID_BYTES = 128

# swps_transport callbacks (host all-gather / all-to-all-v)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)
ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64))

_p = ctypes.c_void_p
_u64 = ctypes.c_uint64
_i32 = ctypes.c_int32


class SwpsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class TableCfg(ctypes.Structure):
    _fields_ = [("device", _i32), ("layout", _i32), ("dtype", _i32), ("dim", _i32), ("capacity", _u64),
                ("learning_rate", ctypes.c_float), ("fudge", ctypes.c_float), ("init_mode", _i32), ("seed", _u64),
                ("push_rule", _i32)]


class Transport(ctypes.Structure):
    _fields_ = [("ctx", ctypes.c_void_p), ("allgather", ALLGATHER_FN), ("alltoallv", ALLTOALLV_FN)]


class W2VCfg(ctypes.Structure):
    _fields_ = [("window", _i32), ("negative", _i32), ("min_sentence_length", _i32), ("minibatch", _i32),
                ("sample", ctypes.c_float), ("alpha", ctypes.c_float), ("unigram_size", _u64), ("key_mode", _i32),
                ("init_mode", _i32), ("rand_seed", ctypes.c_uint32), ("rand_offset", _u64),
                ("fp64_intermediates", _i32), ("profile", _i32), ("minibatch_vocab", _i32), ("sampler", _i32),
                ("host_ingest", _i32)]


class LRCfg(ctypes.Structure):
    _fields_ = [("minibatch", _i32), ("init_ref", _i32), ("profile", _i32), ("fast_sums", _i32), ("plan", _i32)]


class S2VCfg(ctypes.Structure):
    _fields_ = [("window", _i32), ("negative", _i32), ("min_sentence_length", _i32), ("minibatch", _i32),
                ("niters", _i32), ("alpha", ctypes.c_float), ("unigram_size", _u64), ("rand_seed", ctypes.c_uint32),
                ("rand_offset", _u64), ("rand_insert_extra", _u64), ("profile", _i32)]


# name -> (restype, argtypes); every symbol declared in include/swps.h
PROTOS = {
    "swps_last_error": (ctypes.c_char_p, []),
    "swps_version": (ctypes.c_int, []),
    "swps_build_hash": (ctypes.c_char_p, []),
    "swps_table_create": (ctypes.c_int, [ctypes.POINTER(TableCfg), ctypes.POINTER(_p)]),
    "swps_table_destroy": (ctypes.c_int, [_p]),
    "swps_table_size": (ctypes.c_int, [_p, ctypes.POINTER(_u64)]),
    "swps_table_sync": (ctypes.c_int, [_p]),
    "swps_table_row_elems": (ctypes.c_int, [_p, ctypes.POINTER(_i32), ctypes.POINTER(_i32), ctypes.POINTER(_i32)]),
    "swps_pull": (ctypes.c_int, [_p, _p, _u64, _p]),
    "swps_push": (ctypes.c_int, [_p, _p, _u64, _p]),
    "swps_pull_h": (ctypes.c_int, [_p, _p, _u64, _p]),
    "swps_pull_async": (ctypes.c_int, [_p, _p, _u64, _p, _p]),
    "swps_push_async": (ctypes.c_int, [_p, _p, _u64, _p, _p]),
    "swps_comm_unique_id": (ctypes.c_int, [_p]),
    "swps_comm_bootstrap_tcp": (ctypes.c_int, [ctypes.c_char_p, _i32, _i32, _i32, _i32, _p]),
    "swps_comm_create_rccl": (ctypes.c_int, [_p, _i32, _i32, _i32, ctypes.POINTER(_p)]),
    "swps_comm_create_host": (ctypes.c_int, [ctypes.POINTER(Transport), _i32, _i32, _i32, ctypes.POINTER(_p)]),
    "swps_comm_create_tcp": (ctypes.c_int, [ctypes.c_char_p, _i32, _i32, _i32, _i32, _i32, ctypes.POINTER(_p)]),
    "swps_comm_destroy": (ctypes.c_int, [_p]),
    "swps_comm_info": (ctypes.c_int, [_p, ctypes.POINTER(_i32), ctypes.POINTER(_i32)]),
    "swps_comm_transport": (ctypes.c_int, [_p, ctypes.POINTER(_i32), ctypes.POINTER(_i32)]),
    "swps_comm_set_timeout": (ctypes.c_int, [_p, ctypes.c_double]),
    "swps_comm_check": (ctypes.c_int, [_p]),
    "swps_comm_abort": (ctypes.c_int, [_p, ctypes.c_char_p]),
    "swps_comm_enable_ipc": (ctypes.c_int, [_p, ctypes.c_uint64]),
    "swps_comm_ipc_info": (ctypes.c_int, [_p, _p]),
    "swps_comm_alltoallv": (ctypes.c_int, [_p, _p, _p, _p, _p, _p]),
    "swps_table_route": (ctypes.c_int, [_p, _p, _i32]),
    "swps_finish": (ctypes.c_int, [_p]),
    "swps_barrier": (ctypes.c_int, [_p]),
    "swps_route_stats": (ctypes.c_int, [_p, _p]),
    "swps_push_h": (ctypes.c_int, [_p, _p, _u64, _p]),
    "swps_table_find_h": (ctypes.c_int, [_p, _p, _u64, _p]),
    "swps_assign_h": (ctypes.c_int, [_p, _p, _u64, _p]),
    "swps_assign": (ctypes.c_int, [_p, _p, _u64, _p]),
    "swps_export": (ctypes.c_int, [_p, _p, _u64, _p]),
    "swps_table_keys": (ctypes.c_int, [_p, _p, _u64, ctypes.POINTER(_u64)]),
    "swps_dump": (ctypes.c_int, [_p, ctypes.c_char_p]),
    "swps_load": (ctypes.c_int, [_p, ctypes.c_char_p, _i32, _i32, _i32]),
    "swps_save": (ctypes.c_int, [_p, ctypes.c_char_p]),
    "swps_restore": (ctypes.c_int, [_p, ctypes.c_char_p, _i32, _i32, _i32]),
    "swps_fmix64": (_u64, [_u64]),
    "swps_bkdr": (_u64, [ctypes.c_char_p]),
    "swps_hashfrag_table": (ctypes.c_int, [_i32, _i32, _p]),
    "swps_to_node_id": (ctypes.c_int, [_p, _u64, _i32, _p, _p]),
    "swps_w2v_create": (ctypes.c_int, [_p, ctypes.POINTER(W2VCfg), ctypes.POINTER(_p)]),
    "swps_w2v_destroy": (ctypes.c_int, [_p]),
    "swps_w2v_load_text": (ctypes.c_int, [_p, ctypes.c_char_p]),
    "swps_w2v_load_tokens": (ctypes.c_int, [_p, _p, _u64, _p, _u64, _p, _u64]),
    "swps_w2v_vocab": (ctypes.c_int, [_p, _p, _p, _u64, ctypes.POINTER(_u64)]),
    "swps_w2v_info": (ctypes.c_int, [_p, _p]),
    "swps_w2v_corpus": (ctypes.c_int, [_p, _p, _p, _u64]),
    "swps_w2v_batch_keys": (ctypes.c_int, [_p, _u64, _p, _u64, ctypes.POINTER(_u64), _p]),
    "swps_w2v_init": (ctypes.c_int, [_p]),
    "swps_w2v_train_batches": (ctypes.c_int, [_p, _u64]),
    "swps_w2v_train_epochs": (ctypes.c_int, [_p, _i32]),
    "swps_w2v_sync": (ctypes.c_int, [_p]),
    "swps_w2v_stats": (ctypes.c_int, [_p, _p]),
    "swps_w2v_gather_stats": (ctypes.c_int, [_p, _p]),
    "swps_w2v_sum_stats": (ctypes.c_int, [_p, _p]),
    "swps_w2v_get_params": (ctypes.c_int, [_p, _p]),
    "swps_w2v_set_params": (ctypes.c_int, [_p, _p]),
    "swps_w2v_unigram_at": (ctypes.c_int, [_p, _p, _u64, _p]),
    "swps_w2v_trace_negatives": (ctypes.c_int, [_p, _u64]),
    "swps_w2v_negatives": (ctypes.c_int, [_p, _p, _u64, ctypes.POINTER(_u64)]),
    "swps_w2v_kernel_times": (ctypes.c_int, [_p, _p, _i32]),
    "swps_w2v_set_profile": (ctypes.c_int, [_p, _i32]),
    "swps_w2v_stream": (_p, [_p]),
    "swps_w2v_save_state": (ctypes.c_int, [_p, ctypes.c_char_p]),
    "swps_w2v_restore_state": (ctypes.c_int, [_p, ctypes.c_char_p]),
    "swps_w2v_shard": (ctypes.c_int, [_p, _i32, _i32, _i32]),
    "swps_w2v_batch_counts": (ctypes.c_int, [_p, _p, _u64, ctypes.POINTER(_u64)]),
    "swps_w2v_request": (ctypes.c_int, [_p, _i32, _p, _p, ctypes.POINTER(_u64)]),
    "swps_w2v_serve_pull": (ctypes.c_int, [_p, _p, _p, _i32, _p]),
    "swps_w2v_install_init": (ctypes.c_int, [_p, _p]),
    "swps_w2v_step": (ctypes.c_int, [_p, _p, _p]),
    "swps_w2v_serve_push": (ctypes.c_int, [_p, _p, _p, _p]),
    "swps_w2v_set_serve_stream": (ctypes.c_int, [_p, _p]),
    "swps_w2v_prep": (ctypes.c_int, [_p]),
    "swps_w2v_shard_comm": (ctypes.c_int, [_p, _p, _i32]),
    "swps_w2v_exchange_stats": (ctypes.c_int, [_p, _i32, _p]),
    "swps_lr_shard_comm": (ctypes.c_int, [_p, _p, _i32]),
    "swps_lr_exchange_stats": (ctypes.c_int, [_p, _i32, _p]),
    "swps_lr_fx_bytes": (ctypes.c_int, [_p, _u64, _p]),
    "swps_unigram_starts": (ctypes.c_int, [_p, _p, _u64, _u64, _p]),
    "swps_glibc_rand": (ctypes.c_int, [ctypes.c_uint32, _u64, _u64, _p]),
    "swps_s2v_create": (ctypes.c_int, [_p, ctypes.POINTER(S2VCfg), ctypes.POINTER(_p)]),
    "swps_s2v_destroy": (ctypes.c_int, [_p]),
    "swps_s2v_load_text": (ctypes.c_int, [_p, ctypes.c_char_p]),
    "swps_s2v_shard": (ctypes.c_int, [_p, _i32, _i32, _i32]),
    "swps_s2v_load_tokens": (ctypes.c_int, [_p, _p, _u64, _p, _u64, _p]),
    "swps_s2v_run_tokens": (ctypes.c_int, [_p, _p, _u64, _p, _u64, _p]),
    "swps_s2v_info": (ctypes.c_int, [_p, _p]),
    "swps_s2v_train_batches": (ctypes.c_int, [_p, _u64]),
    "swps_s2v_train": (ctypes.c_int, [_p]),
    "swps_s2v_sync": (ctypes.c_int, [_p]),
    "swps_s2v_docs": (ctypes.c_int, [_p, _p, _p, _p, _u64, ctypes.POINTER(_u64)]),
    "swps_s2v_dump": (ctypes.c_int, [_p, ctypes.c_char_p]),
    "swps_s2v_stats": (ctypes.c_int, [_p, _p]),
    "swps_s2v_set_profile": (ctypes.c_int, [_p, _i32]),
    "swps_s2v_kernel_times": (ctypes.c_int, [_p, _p, _i32]),
    "swps_s2v_stream": (_p, [_p]),
    "swps_lr_create": (ctypes.c_int, [_p, ctypes.POINTER(LRCfg), ctypes.POINTER(_p)]),
    "swps_lr_destroy": (ctypes.c_int, [_p]),
    "swps_lr_load_text": (ctypes.c_int, [_p, ctypes.c_char_p]),
    "swps_lr_load_csr": (ctypes.c_int, [_p, _p, _u64, _p, _p, _p]),
    "swps_lr_init": (ctypes.c_int, [_p]),
    "swps_lr_train": (ctypes.c_int, [_p, _i32, _p]),
    "swps_lr_train_batches": (ctypes.c_int, [_p, _u64]),
    "swps_lr_predict": (ctypes.c_int, [_p, _p, _p, _u64]),
    "swps_lr_params": (ctypes.c_int, [_p, _p, _p, _p, _u64, ctypes.POINTER(_u64)]),
    "swps_lr_info": (ctypes.c_int, [_p, _p]),
    "swps_lr_plan_info": (ctypes.c_int, [_p, _p]),
    "swps_lr_sync": (ctypes.c_int, [_p]),
    "swps_lr_kernel_times": (ctypes.c_int, [_p, _p, _i32]),
    "swps_lr_set_profile": (ctypes.c_int, [_p, _i32]),
    "swps_lr_epoch_error": (ctypes.c_int, [_p, ctypes.POINTER(ctypes.c_double)]),
    "swps_lr_stream": (_p, [_p]),
    "swps_lr_shard": (ctypes.c_int, [_p, _i32, _i32, _i32]),
    "swps_lr_batch_counts": (ctypes.c_int, [_p, _p, _u64, ctypes.POINTER(_u64)]),
    "swps_lr_request": (ctypes.c_int, [_p, _i32, _p, _p, ctypes.POINTER(_u64)]),
    "swps_lr_serve_pull": (ctypes.c_int, [_p, _p, _p, _i32, _p]),
    "swps_lr_install": (ctypes.c_int, [_p, _p]),
    "swps_lr_step": (ctypes.c_int, [_p, _p, _p]),
    "swps_lr_serve_push": (ctypes.c_int, [_p, _p, _p, _p]),
}

_lib = None


def lib():
    """Load libswps.so (raises if it was never built — no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run `python -m swiftmpi_amd.build` (HIP extension required)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in PROTOS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != SWPS_OK:
        raise SwpsError(rc, lib().swps_last_error().decode(errors="replace"))
    return rc


def ptr(a):
    """Address of a numpy array or a torch tensor (device or host)."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return ctypes.c_void_p(a.data_ptr())
    return a.ctypes.data_as(ctypes.c_void_p)
