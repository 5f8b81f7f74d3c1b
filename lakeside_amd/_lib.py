"""ctypes binding of include/lakeside_gpu.h (the C ABI the Scala worker binds over JNA).

The product path has no CPU fallback: if the HIP library is missing this module raises at import.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# LK_LIB_PATH: an alternative build of the same library (kernel A/B experiments only)
LIB_PATH = os.environ.get("LK_LIB_PATH") or os.path.join(_HERE, "liblakeside_gpu.so")
SYNTH_PATH = os.path.join(_HERE, "liblakeside_synth.so")

LK_OK = 0
LK_ERR_ARG = -1
LK_ERR_UNSUPPORTED = -2
LK_ERR_IO = -3
LK_ERR_DEVICE = -4
LK_ERR_EVICTED = -6
LK_ERR_MEMORY = -5
LK_PER_GLOB_ROWS = 1
LK_MERGED = 2
LK_PLAN_BYTES = 4
LK_UNIQUE_ID_BYTES = 128

# (name, restype, argtypes) of every symbol the header declares
_c = ctypes
_P = _c.c_void_p
SIGNATURES = [
    ("lk_engine_create", _c.c_int, [_c.c_char_p, _c.POINTER(_P)]),
    ("lk_engine_destroy", None, [_P]),
    ("lk_segment_put", _c.c_int, [_P, _c.c_char_p, _c.c_void_p, _c.c_size_t]),
    ("lk_segment_load", _c.c_int, [_P, _c.c_char_p]),
    ("lk_segment_evict", _c.c_int, [_P, _c.c_char_p]),
    ("lk_segment_count", _c.c_size_t, [_P]),
    ("lk_segment_bytes", _c.c_size_t, [_P]),
    ("lk_engine_stats", _c.c_char_p, [_P]),
    ("lk_engine_drop_caches", _c.c_int, [_P]),
    ("lk_eval_pushdown", _c.c_int, [_P, _c.c_char_p, _c.POINTER(_c.c_char_p), _c.c_size_t, _c.c_int, _c.c_uint,
                                    _c.POINTER(_P)]),
    ("lk_result_num_rows", _c.c_size_t, [_P]),
    ("lk_result_timestamps", _c.POINTER(_c.c_int64), [_P]),
    ("lk_result_values", _c.POINTER(_c.c_double), [_P]),
    ("lk_result_globs", _c.POINTER(_c.c_uint32), [_P]),
    ("lk_result_num_tag_columns", _c.c_size_t, [_P]),
    ("lk_result_tag_name", _c.c_char_p, [_P, _c.c_size_t]),
    ("lk_result_tag_value", _c.c_char_p, [_P, _c.c_size_t, _c.c_size_t]),
    ("lk_result_group_ids", _c.POINTER(_c.c_uint32), [_P]),
    ("lk_result_num_group_columns", _c.c_size_t, [_P]),
    ("lk_result_tag_dictionary", _c.POINTER(_c.c_void_p), [_P, _c.c_size_t, _c.POINTER(_c.c_uint64),
                                                           _c.POINTER(_c.c_uint64)]),
    ("lk_result_stats", _c.c_char_p, [_P]),
    ("lk_result_sketch", _c.POINTER(_c.c_uint8), [_P, _c.c_size_t, _c.POINTER(_c.c_size_t)]),
    ("lk_result_free", None, [_P]),
    ("lk_last_error", _c.c_char_p, []),
    ("lk_comm_unique_id", _c.c_int, [_c.c_void_p]),
    ("lk_comm_init", _c.c_int, [_P, _c.c_void_p, _c.c_int, _c.c_int]),
    ("lk_eval_pushdown_dist", _c.c_int, [_P, _c.c_char_p, _c.POINTER(_c.c_char_p), _c.c_size_t,
                                         _c.POINTER(_c.c_int32), _c.c_int, _c.POINTER(_P)]),
]

# int (*lk_allgather_fn)(void* user, const void* send, size_t bytes, void* recv)
ALLGATHER_FN = _c.CFUNCTYPE(_c.c_int, _c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_void_p)
SIGNATURES.append(("lk_comm_init_host", _c.c_int, [_P, _c.c_int, _c.c_int, ALLGATHER_FN, _c.c_void_p]))


class LakesideError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"lakeside_gpu error {code}: {msg}")
        self.code = code


_lib = None


def lib():
    """Load liblakeside_gpu.so (built by `make` / __graft_entry__.build()).  Raises if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make` (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            if os.environ.get("LK_LIB_PATH") and not hasattr(L, name):
                continue   # an A/B build from before this symbol existed (experiments only)
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != LK_OK:
        msg = lib().lk_last_error()
        raise LakesideError(rc, msg.decode() if msg else "")
    return rc
