"""ctypes binding of libtips_hip.so (the C-ABI declared in include/tips_hip.h).

This is the only way the Python surface reaches the device: there is no CPU
fallback. If the shared library is missing the first call raises
``TipsLibraryError`` — the product path fails loudly rather than silently
computing on the host (the oracle under ``oracle/`` is test infrastructure and
is never imported from here).
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TIPS_HIP_LIB", os.path.join(_HERE, "lib", "libtips_hip.so"))
# the development library (include/tips_hip_dev.h): tests, tuning sweeps and probes only
DEV_LIB_PATH = os.environ.get("TIPS_HIP_DEV_LIB", os.path.join(os.path.dirname(_HERE), "tools", "lib",
                                                                 "libtips_hip_dev.so"))

# dtype codes (include/tips_hip.h enum tips_dtype; 0-3 = collective_messages.fbs:17-23)
FLOAT32, FLOAT64, INT32, INT64, FLOAT16, BFLOAT16 = 0, 1, 2, 3, 4, 5
OP_SUM, OP_MAX, OP_MIN = 0, 1, 2
REQ_ALLREDUCE, REQ_ALLGATHER, REQ_BROADCAST = 0, 1, 2
MAX_DIMS = 8
REQUEST_WORDS = 3 + MAX_DIMS
ALGO_AUTO, ALGO_RING, ALGO_DIRECT, ALGO_RCCL, ALGO_ONESHOT, ALGO_PEER, ALGO_TUNE = -1, 0, 1, 2, 3, 4, 5

STATUS_NAMES = {
    0: "TIPS_OK",
    -1: "TIPS_ERR_INVALID_ARG",
    -2: "TIPS_ERR_NOT_INITIALIZED",
    -3: "TIPS_ERR_HIP",
    -4: "TIPS_ERR_RCCL",
    -5: "TIPS_ERR_UNSUPPORTED",
    -6: "TIPS_ERR_BOOTSTRAP",
    -7: "TIPS_ERR_MISMATCH",
}


class TipsLibraryError(RuntimeError):
    """libtips_hip.so could not be loaded (not built, or built for another arch)."""


class TipsError(RuntimeError):
    """A C-ABI call returned a negative status; carries tips_last_error()."""

    def __init__(self, func, code, message):
        self.func = func
        self.code = code
        super().__init__("%s -> %s (%d): %s" % (func, STATUS_NAMES.get(code, "?"), code, message))


_lock = threading.Lock()
_lib = None

_c_void_pp = ctypes.POINTER(ctypes.c_void_p)
_c_i64_p = ctypes.POINTER(ctypes.c_int64)
# tips_alloc_fn (include/tips_hip.h): void* (*)(void* ctx, int64_t bytes)
ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64)
# tips_done_fn: void (*)(void* ctx, int status, const char* message)
DONE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p)

# (name, restype, argtypes) — must match include/tips_hip.h
_SIGNATURES = [
    ("tips_init", None, []),
    ("tips_shutdown", None, []),
    ("tips_is_initialize", ctypes.c_bool, []),
    ("tips_size", ctypes.c_int, []),
    ("tips_rank", ctypes.c_int, []),
    ("tips_unique_id_bytes", ctypes.c_int, []),
    ("tips_get_unique_id", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    ("tips_init_rank", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64]),
    ("tips_last_error", ctypes.c_char_p, []),
    ("tips_version", ctypes.c_char_p, []),
    ("tips_bucket_sum", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]),
    ("tips_multi_sum", ctypes.c_int,
     [ctypes.c_void_p, _c_void_pp, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]),
    ("tips_allreduce", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("tips_check_requests", ctypes.c_int, [_c_i64_p, ctypes.c_int]),
    ("tips_allreduce_checked", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, _c_i64_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("tips_allgather_i64", ctypes.c_int, [_c_i64_p, ctypes.c_int, _c_i64_p]),
    ("tips_broadcast", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("tips_allgatherv", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, _c_i64_p, ctypes.c_int, ctypes.c_void_p]),
    ("tips_host_register", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    ("tips_host_unregister", ctypes.c_int, [ctypes.c_void_p]),
    ("tips_fused_allreduce", ctypes.c_int, [_c_void_pp, _c_i64_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("tips_fused_allreduce_oop", ctypes.c_int,
     [_c_void_pp, _c_void_pp, _c_i64_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("tips_fused_allreduce_cast", ctypes.c_int,
     [_c_void_pp, _c_void_pp, _c_i64_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("tips_fused_layout", ctypes.c_int64, [_c_i64_p, ctypes.c_int, ctypes.c_int, _c_i64_p]),
    ("tips_fused_allreduce_flat", ctypes.c_int,
     [_c_void_pp, _c_i64_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    ("tips_fusion_stats", ctypes.c_int, [_c_i64_p, _c_i64_p, _c_i64_p, _c_i64_p]),
    ("tips_fused_pack_bucket", ctypes.c_int64,
     [_c_void_pp, _c_i64_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    ("tips_fused_allreduce_host", ctypes.c_int, [_c_void_pp, _c_void_pp, _c_i64_p, ctypes.c_int, ctypes.c_int]),
    ("tips_fused_allreduce_host_flat", ctypes.c_int, [_c_void_pp, _c_i64_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("tips_enqueue_allreduce", ctypes.c_int64,
     [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]),
    ("tips_enqueue_allreduce_shaped", ctypes.c_int64,
     [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, _c_i64_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("tips_enqueue_allreduce_shaped_n", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_char_p), _c_void_pp, _c_void_pp, ctypes.POINTER(ctypes.c_int), _c_i64_p, ctypes.c_int,
      ctypes.c_int, ctypes.c_void_p, _c_i64_p]),
    ("tips_poll", ctypes.c_int, [ctypes.c_int64]),
    ("tips_enqueue_allreduce_n", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_char_p), _c_void_pp, _c_void_pp, _c_i64_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
      _c_i64_p]),
    ("tips_wait_n", ctypes.c_int, [_c_i64_p, ctypes.c_int]),
    ("tips_on_done", ctypes.c_int, [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    ("tips_enqueue_allreduce_cb", ctypes.c_int64,
     [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, _c_i64_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
      ctypes.c_void_p, ctypes.c_void_p]),
    ("tips_net_stats", ctypes.c_int, [_c_i64_p, _c_i64_p]),
    ("tips_debug_state", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int64]),
    ("tips_wait", ctypes.c_int, [ctypes.c_int64]),
    ("tips_enqueue_broadcast", ctypes.c_int64,
     [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, _c_i64_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
      ctypes.c_void_p]),
    ("tips_enqueue_allgather", ctypes.c_int64,
     [ctypes.c_char_p, ctypes.c_void_p, _c_i64_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
      ctypes.c_void_p, _c_i64_p]),
    ("tips_set_algorithm", ctypes.c_int, [ctypes.c_int]),
    ("tips_get_algorithm", ctypes.c_int, []),
    ("tips_resolve_algorithm", ctypes.c_int, [ctypes.c_int, ctypes.c_int64]),
    ("tips_tuned_choice", ctypes.c_int, [ctypes.c_int64, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    ("tips_tuned_schedule", ctypes.c_int, [ctypes.c_int64, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                           ctypes.POINTER(ctypes.c_int)]),
    ("tips_tuned_timings", ctypes.c_int,
     [ctypes.c_int64, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
      ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    ("tips_graph_stats", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    ("tips_replay_order_stats", ctypes.c_int, [_c_i64_p, _c_i64_p]),
    ("tips_schedule_shape", ctypes.c_int,
     [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int), _c_i64_p]),
    ("tips_chunk_bounds", ctypes.c_int,
     [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_i64_p, _c_i64_p]),
    ("tips_bootstrap_broadcast", ctypes.c_int,
     [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]),
]

# include/tips_hip_dev.h: libtips_hip_dev.so's entry points beyond the product C-ABI (tests, sweeps)
_DEV_SIGNATURES = [
    ("tips_fusion_tile_table", ctypes.c_int64,
     [_c_i64_p, ctypes.c_int, ctypes.c_int, _c_i64_p, _c_i64_p, _c_i64_p, ctypes.c_int64, _c_i64_p, _c_i64_p]),
    ("tips_host_pool_selftest", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    ("tips_negotiation_selftest", ctypes.c_int,
     [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int64]),
    ("tips_negotiation_stop_race_selftest", ctypes.c_int,
     [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]),
    ("tips_ring_simulate", ctypes.c_int,
     [_c_void_pp, _c_void_pp, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]),
    ("tips_oneshot_simulate", ctypes.c_int,
     [_c_void_pp, _c_void_pp, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]),
    ("tips_direct_simulate", ctypes.c_int,
     [_c_void_pp, _c_void_pp, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]),
    ("tips_set_sim_transport", ctypes.c_int, [ctypes.c_int]),
    ("tips_sum_variant", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
      ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("tips_multi_sum_variant", ctypes.c_int,
     [ctypes.c_void_p, _c_void_pp, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    ("tips_xfer", ctypes.c_int, [_c_void_pp, _c_void_pp, _c_i64_p, ctypes.c_int, ctypes.c_void_p]),
    ("tips_copy_tiles_variant", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p]),
    ("tips_schedule_plan", ctypes.c_int64,
     [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int, _c_i64_p, ctypes.c_int64]),
    ("tips_tune_candidates", ctypes.c_int,
     [ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
      ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
]


def _share_torch_runtime():
    """Import torch before dlopen-ing libtips_hip.so.

    torch-ROCm bundles its own libamdhip64 / libhsa-runtime64 / librccl with
    the same sonames as /opt/rocm's (libamdhip64.so.7, ...). If our library is
    loaded first, torch later maps a second HIP runtime into the process and
    torch's streams / allocations would be handed to a runtime that does not
    own them. Loaded after torch, our DT_NEEDED entries resolve to the copies
    torch already mapped, so the process has exactly one HIP runtime and one
    RCCL (tests/test_abi.py::test_single_hip_runtime checks /proc/self/maps).
    """
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover - standalone use: /opt/rocm's runtime
        pass


def lib():
    """Load (once) and return the ctypes handle; raises TipsLibraryError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    _share_torch_runtime()
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise TipsLibraryError(
                    "libtips_hip.so not found at %s — build it with `make` (or __graft_entry__.build()); "
                    "there is no CPU fallback" % LIB_PATH)
            try:
                handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            except OSError as e:
                raise TipsLibraryError("cannot load %s: %s" % (LIB_PATH, e)) from e
            for name, res, args in _SIGNATURES:
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
    return _lib


_dev = None


def dev():
    """The development library (include/tips_hip_dev.h: simulators, self-tests, tuning sweeps),
    loaded once beside the product library. It is a second, complete copy of the runtime with
    state of its own, loaded RTLD_LOCAL and linked -Bsymbolic, so nothing in it binds to the
    product library's symbols or they to it: tests call its extra entry points through it
    (dev_call), never a job's collectives."""
    global _dev
    if _dev is not None:
        return _dev
    _share_torch_runtime()
    with _lock:
        if _dev is None:
            if not os.path.exists(DEV_LIB_PATH):
                raise TipsLibraryError("libtips_hip_dev.so not found at %s — build it with `make`" % DEV_LIB_PATH)
            try:
                handle = ctypes.CDLL(DEV_LIB_PATH, mode=ctypes.RTLD_LOCAL)
            except OSError as e:
                raise TipsLibraryError("cannot load %s: %s" % (DEV_LIB_PATH, e)) from e
            for name, res, args in _SIGNATURES + _DEV_SIGNATURES:
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _dev = handle
    return _dev


def dev_call(name, *args):
    """Call development-library function `name` and raise on a negative status (its own last error)."""
    code = getattr(dev(), name)(*args)
    if code < 0:
        raise TipsError(name, code, dev().tips_last_error().decode(errors="replace"))
    return code


def last_error():
    return lib().tips_last_error().decode(errors="replace")


def check(func, code):
    """Raise TipsError for a negative status returned by C-ABI function `func`."""
    if code < 0:
        raise TipsError(func, code, last_error())
    return code


def call(name, *args):
    """Call C-ABI function `name` and raise on a negative status."""
    return check(name, getattr(lib(), name)(*args))


def ptr_array(ptrs):
    """(void** for ctypes, keep-alive). numpy-backed: ~10x faster than a ctypes array built
    element by element, which matters for gradient lists of 1000 tensors per step."""
    import numpy as np
    arr = np.asarray(ptrs, dtype=np.uint64).reshape(-1)
    return arr.ctypes.data_as(_c_void_pp), arr


def i64_array(vals):
    import numpy as np
    arr = np.asarray(vals, dtype=np.int64).reshape(-1)
    return arr.ctypes.data_as(_c_i64_p), arr
