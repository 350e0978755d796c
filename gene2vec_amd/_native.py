"""ctypes binding of ``libg2v.so`` (C ABI in ``include/g2v.h``).

There is no fallback: if the library is missing or fails to load, every
entry point raises ``NativeLibraryError``.  Build it with
``python -m gene2vec_amd.build`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libg2v.so")

G2V_OK = 0
G2V_EINVAL = -1
G2V_EHIP = -2
G2V_ENOMEM = -3
G2V_ESTATE = -4
G2V_ERANGE = -5
G2V_ECOMM = -6
ABI_VERSION = 5

MODE_HOGWILD = 0
MODE_SEQUENTIAL = 1
MODE_MINIBATCH = 2
FLAG_TIMING = 0x100
FLAG_COMPUTE_LOSS = 0x200
MERGE_TOUCH = 0
MERGE_MEAN = 1
MERGE_ALIGN = 2
UNIQUE_ID_BYTES = 128
CORPUS_DEVICE = 0x1
OPT_HOT_ROWS = 1
OPT_CACHE_POLICY = 2
OPT_SEG_JOBS = 3
OPT_GRID = 4
OPT_TABLE_MEM = 5
OPT_DEBUG_WRITE = 6
OPT_STRIPE_ROWS = 7
OPT_STRIPE_COPIES = 8
OPT_ATOMIC_OVERLAP = 9
OPT_SAMPLE_OVERLAP = 10
OPT_MERGE_EVERY_JOBS = 11
OPT_MERGE_RULE = 12
OPT_STRIPE2_ROWS = 13
OPT_STRIPE2_COPIES = 14
OPT_ACTIVE_WAVES = 15
OPT_MERGE_BETA_MILLI = 16
OPT_MERGE_GAMMA_MILLI = 17
OPT_DEBUG_FAIL_MERGE = 18
OPT_TAIL_STORE = 21
COLL_SUM = 0
COLL_BCAST0 = 1
BATCH_WORDS = 10000
MAX_DIM = 512
TXT_MATRIX = 0
TXT_W2V = 1
SUPPORTED_NEGATIVE = tuple(range(1, 21))


class NativeLibraryError(RuntimeError):
    pass


class G2VError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"g2v error {code}: {msg}")
        self.code = code


class Stats(C.Structure):
    _fields_ = [("raw_words", C.c_int64), ("effective_words", C.c_int64),
                ("examples", C.c_int64), ("jobs", C.c_int64), ("launches", C.c_int64),
                ("sgns_kernel_ms", C.c_double), ("sample_kernel_ms", C.c_double),
                ("training_loss", C.c_double), ("sgns_grid", C.c_int64),
                ("stripe_rows", C.c_int64), ("stripe_copies", C.c_int64),
                ("stripe2_rows", C.c_int64), ("stripe2_copies", C.c_int64),
                ("sgns_waves", C.c_int64), ("tail_row_syn0", C.c_int64),
                ("tail_row_syn1neg", C.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_vp = C.c_void_p
_i32 = C.c_int32
_i64 = C.c_int64
_u32 = C.c_uint32
_f32 = C.c_float
_f64 = C.c_double
# g2v_collective_fn: int (*)(void *user, int op, float *buf, int64_t count)
COLLECTIVE_FN = C.CFUNCTYPE(C.c_int, _vp, C.c_int, C.POINTER(C.c_float), _i64)

# name -> (restype, argtypes); every symbol include/g2v.h declares
SIGNATURES = {
    "g2v_last_error": (C.c_char_p, []),
    "g2v_abi_version": (C.c_int, []),
    "g2v_create": (C.c_int, [C.c_int, _i32, _i32, _i32, _i32, C.POINTER(_vp)]),
    "g2v_destroy": (C.c_int, [_vp]),
    "g2v_set_stream": (C.c_int, [_vp, _vp]),
    "g2v_set_option": (C.c_int, [_vp, C.c_int, _i64]),
    "g2v_get_option": (C.c_int, [_vp, C.c_int, C.POINTER(_i64)]),
    "g2v_row_stride": (C.c_int, [_vp, C.POINTER(_i64)]),
    "g2v_set_vocab": (C.c_int, [_vp, _vp, _f64, _f64, _vp, _vp]),
    "g2v_bind_tables": (C.c_int, [_vp, _vp, _vp, _i64]),
    "g2v_set_weights": (C.c_int, [_vp, _vp, _vp, _vp]),
    "g2v_get_weights": (C.c_int, [_vp, _vp, _vp]),
    "g2v_set_corpus": (C.c_int, [_vp, _vp, _i64, _vp, _i64, _i64, _u32]),
    "g2v_plan_jobs": (C.c_int, [_vp, _i64, _i64, _i64, _vp, _i64, C.POINTER(_i64)]),
    "g2v_train": (C.c_int, [_vp, _vp, _vp, _vp, _i64, _u32]),
    "g2v_sgns_step_explicit": (C.c_int, [_vp, _vp, _vp, _vp, _i64, _f32, _u32]),
    "g2v_debug_sample": (C.c_int, [_vp, _vp, _vp, _i64, _vp, _i64, C.POINTER(_i64)]),
    "g2v_debug_stamps": (C.c_int, [_vp, _vp, _i64]),
    "g2v_reset_loss": (C.c_int, [_vp]),
    "g2v_sync": (C.c_int, [_vp]),
    "g2v_comm_unique_id": (C.c_int, [_vp, _i64]),
    "g2v_comm_init": (C.c_int, [_vp, _vp, C.c_int, C.c_int]),
    "g2v_average": (C.c_int, [_vp, C.c_int]),
    "g2v_merge_snapshot": (C.c_int, [_vp]),
    "g2v_average_local": (C.c_int, [C.POINTER(_vp), C.c_int, C.c_int]),
    "g2v_local_group_create": (C.c_int, [C.c_int, C.c_int, C.POINTER(_vp)]),
    "g2v_local_group_destroy": (C.c_int, [_vp]),
    "g2v_comm_init_local": (C.c_int, [_vp, _vp, C.c_int]),
    "g2v_comm_init_host": (C.c_int, [_vp, COLLECTIVE_FN, _vp, C.c_int, C.c_int]),
    "g2v_comm_abort": (C.c_int, [_vp]),
    "g2v_read_stats": (C.c_int, [_vp, C.POINTER(Stats)]),
    "g2v_cosine_pairs": (C.c_int, [C.c_int, _vp, _i64, _i32, _vp, _vp, _i64, _vp]),
    "g2v_permute_items8": (C.c_int, [C.c_int, _vp, _vp, _i64, _i64, _i64, C.c_uint64, _vp]),
    "g2v_first_occurrence_perm8": (C.c_int, [C.c_int, _vp, _i64, C.c_uint64, _i32, _vp, _vp]),
    "g2v_seeded_vectors": (C.c_int, [_vp, _i64, _i32, _vp]),
    "g2v_format_rows": (C.c_int, [_vp, _i64, _i32, _vp, _i64, _vp, _vp, _i32, _vp, _i64,
                                  C.POINTER(_i64)]),
    "g2v_format_f32": (C.c_int, [_vp, _i64, _vp, _i64, C.POINTER(_i64)]),
    "g2v_coexpr_pairs": (C.c_int, [C.c_int, _vp, _i64, _i64, _f64, _vp, _i64, C.POINTER(_i64)]),
    "g2v_coexpr_last_timing": (C.c_int, [C.POINTER(_f64), C.POINTER(_f64)]),
    "g2v_count_ids": (C.c_int, [_vp, _i64, _i32, _vp, _vp]),
    "g2v_corpus_read": (C.c_int, [C.POINTER(C.c_char_p), C.c_int, C.c_int, C.POINTER(_vp)]),
    "g2v_corpus_info": (C.c_int, [_vp, C.POINTER(_i64), C.POINTER(_i64), C.POINTER(_i64),
                                  C.POINTER(_i64)]),
    "g2v_corpus_export": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "g2v_corpus_sent_len": (C.c_int, [_vp, C.POINTER(_i64)]),
    "g2v_count_lines": (C.c_int, [_vp, C.c_int, C.c_int, C.POINTER(_i64)]),
    "g2v_corpus_free": (C.c_int, [_vp]),
    "g2v_csr_permute": (C.c_int, [_vp, _vp, _i64, _vp, _vp, _vp]),
    "g2v_pairs_permute": (C.c_int, [_vp, _i64, _vp, _vp]),
    "g2v_py_shuffle": (C.c_int, [_vp, _vp, _vp, _i64]),
    "g2v_py_shuffle_range": (C.c_int, [_vp, _vp, _vp, _i64]),
    "g2v_py_shuffle_skip": (C.c_int, [_vp, _vp, _i64]),
}

_lib = None


def use_library(path):
    """Load `path` (e.g. build.ABLATIONS_LIB, the -DG2V_ABLATIONS build the
    throughput-ablation scripts use) instead of libg2v.so; only before the
    first call into the library"""
    global LIB_PATH
    if _lib is not None and os.path.abspath(path) != LIB_PATH:
        raise NativeLibraryError(f"{LIB_PATH} is already loaded")
    LIB_PATH = os.path.abspath(path)


def lib():
    """Load libg2v.so once; raise loudly when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            f"{LIB_PATH} is missing: build it with `python -m gene2vec_amd.build` "
            "(the SGNS path has no CPU fallback)")
    # torch bundles its own HIP runtime under the same soname
    # (libamdhip64.so.7) as /opt/rocm's, which libg2v links.  Whichever loads
    # first serves the whole process; torch fails on the other one ("no
    # ROCm-capable device"), so torch's is loaded before libg2v and libg2v runs
    # on it (measured on MI355X: libg2v first -> torch.cuda init fails).
    # `import torch` itself, not just a dlopen of torch's libamdhip64: with the
    # dlopen alone the CLI's 10 training iterations took 19.4 s instead of
    # 7.3 s on MI355X (profiles/r01/r01_experiments/e2e_runtime_*.json), for the 1.5 s import.
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover - torch is plumbing, not required
        pass
    try:
        L = C.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the ROCm runtime
        raise NativeLibraryError(f"failed to load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.g2v_abi_version() != ABI_VERSION:
        raise NativeLibraryError("libg2v ABI version mismatch")
    _lib = L
    return L


def check(rc):
    if rc != G2V_OK:
        msg = lib().g2v_last_error()
        raise G2VError(rc, msg.decode() if msg else "")
    return rc


def ptr(a):
    """data pointer of a numpy array (or None)."""
    if a is None:
        return None
    return a.ctypes.data_as(C.c_void_p)
