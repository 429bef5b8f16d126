"""ctypes binding of oracle/build/liboracle.so — the CPU restatement (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this; the product (tips_amd/, libtips_hip.so) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "liboracle.so")

F32, F64, I32, I64, F16, BF16 = 0, 1, 2, 3, 4, 5
NP = {F32: np.float32, F64: np.float64, I32: np.int32, I64: np.int64, F16: np.float16, BF16: np.uint16}
CODE = {np.dtype(np.float32): F32, np.dtype(np.float64): F64, np.dtype(np.int32): I32, np.dtype(np.int64): I64,
        np.dtype(np.float16): F16}

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", ORACLE_DIR, "build/liboracle.so"], check=True, capture_output=True)
    L = ctypes.CDLL(ORACLE_SO)
    vp, vpp, i64 = ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int64
    L.oracle_sum2.argtypes = [ctypes.c_int, vp, vp, vp, i64]
    L.oracle_fold.argtypes = [ctypes.c_int, vp, vpp, ctypes.c_int, i64, ctypes.c_int]
    L.oracle_ring.argtypes = [ctypes.c_int, vpp, vpp, ctypes.c_int, i64, i64]
    L.oracle_chunk_bounds.argtypes = [i64, ctypes.c_int, i64, ctypes.c_int, ctypes.POINTER(i64), ctypes.POINTER(i64)]
    L.oracle_chunk_bounds.restype = None
    L.oracle_half_to_float.argtypes = [ctypes.c_uint16]
    L.oracle_half_to_float.restype = ctypes.c_float
    L.oracle_float_to_half.argtypes = [ctypes.c_float]
    L.oracle_float_to_half.restype = ctypes.c_uint16
    L.oracle_bf16_to_float.argtypes = [ctypes.c_uint16]
    L.oracle_bf16_to_float.restype = ctypes.c_float
    L.oracle_float_to_bf16.argtypes = [ctypes.c_float]
    L.oracle_float_to_bf16.restype = ctypes.c_uint16
    L.oracle_cast_to16.argtypes = [ctypes.c_int, vp, vp, i64]
    L.oracle_cast_from16.argtypes = [ctypes.c_int, vp, vp, i64]
    _lib = L
    return L


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def sum2(a, b, code=None):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    code = CODE[a.dtype] if code is None else code
    out = np.empty_like(a)
    assert load().oracle_sum2(code, out.ctypes.data, a.ctypes.data, b.ctypes.data, a.size) == 0
    return out


def fold(ins, code=None, wide_acc=False):
    ins = [np.ascontiguousarray(x) for x in ins]
    code = CODE[ins[0].dtype] if code is None else code
    out = np.empty_like(ins[0])
    assert load().oracle_fold(code, out.ctypes.data, _ptrs(ins), len(ins), ins[0].size, int(wide_acc)) == 0
    return out


def ring(ins, code=None, align_elems=None):
    """Ring RS+AG result every rank ends with (list of p identical arrays)."""
    ins = [np.ascontiguousarray(x) for x in ins]
    code = CODE[ins[0].dtype] if code is None else code
    if align_elems is None:
        align_elems = 256 // ins[0].itemsize
    outs = [np.empty_like(ins[0]) for _ in ins]
    assert load().oracle_ring(code, _ptrs(outs), _ptrs(ins), len(ins), ins[0].size, align_elems) == 0
    return outs


def chunk_bounds(n, p, align_elems, c):
    b, e = ctypes.c_int64(), ctypes.c_int64()
    load().oracle_chunk_bounds(n, p, align_elems, c, ctypes.byref(b), ctypes.byref(e))
    return b.value, e.value


def cast_to16(x, code):
    """float32 array -> uint16 bits of F16 / BF16 (RNE): Compression.fp16's compress (compression.py:49-66)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(x.shape, dtype=np.uint16)
    assert load().oracle_cast_to16(code, out.ctypes.data, x.ctypes.data, x.size) == 0
    return out


def cast_from16(h, code):
    """uint16 bits of F16 / BF16 -> float32 (exact): the decompress."""
    h = np.ascontiguousarray(h, dtype=np.uint16)
    out = np.empty(h.shape, dtype=np.float32)
    assert load().oracle_cast_from16(code, out.ctypes.data, h.ctypes.data, h.size) == 0
    return out


def compressed_fold(ins, code):
    """What Compression.fp16 (code F16) or a bf16 wire gives for an allreduce of f32 inputs under a
    rank-order schedule: each rank's tensor cast to the 16-bit type, folded in rank order in fp32
    and rounded once (the library's f16 / bf16 fold: oracle_fold wide_acc), cast back to f32."""
    folded = fold([cast_to16(x, code).view(np.float16 if code == F16 else np.uint16) for x in ins], code=code,
                  wide_acc=True)
    return cast_from16(folded.view(np.uint16), code)
