"""Op bindings — mirrors tips/tensorflow/ops.py:24-95 over the C-ABI.

`allreduce_op` is the MPIAllreduce op (ops.cc:79-136): an out-of-place SUM of
one tensor over all ranks, output of the input's shape and dtype. Device
(torch CUDA/HIP) tensors stay in HBM and are ordered on the caller's current
stream; host tensors (numpy / CPU torch) are staged through HBM and the call
returns when the result is in host memory, like the reference's CPU op.
"""
import re

from . import _lib
from . import basics
from . import tensors


def _normalize_name(name):
    """Normalizes operation name to TensorFlow rules (ops.py:33-35)."""
    return re.sub('[^a-zA-Z0-9_]', '_', name)


def size_op(name=None):
    """Number of ranks (ops.py:45-47; MPISize, ops.cc:21-48)."""
    return basics.size()


def rank_op(name=None):
    """This process's rank (ops.py:53-55; MPIRank, ops.cc:50-77)."""
    return basics.rank()


def allreduce_op(tensor, name=None):
    """Sum `tensor` over all ranks (ops.py:61-65 -> MPIAllreduce, ops.cc:86-115)."""
    basics.init()
    code = tensors.dtype_code(tensor)
    src = tensors.contiguous(tensor)
    out = tensors.empty_like(src)
    n = tensors.numel(src)
    if n:
        _lib.call("tips_allreduce", tensors.data_ptr(src), tensors.data_ptr(out), n, code, _lib.OP_SUM,
                  tensors.stream_of(src))
    return out


def fused_allreduce_(tensor_list):
    """In-place SUM of a list of same-dtype device tensors through fusion buckets.

    No reference counterpart (the reference issues one op per gradient,
    tips/tensorflow/__init__.py:212-222): the tensors are packed into buckets
    of at most TIPS_FUSION_THRESHOLD bytes (default 64 MiB), each bucket is
    allreduced once, and the sums are unpacked in place.
    """
    basics.init()
    if not tensor_list:
        return tensor_list
    code = tensors.dtype_code(tensor_list[0])
    for t in tensor_list:
        if not tensors.is_device(t):
            raise ValueError("fused_allreduce_ needs device tensors")
        if tensors.dtype_code(t) != code:
            raise TypeError("fused_allreduce_ needs one dtype per call")
        if not t.is_contiguous():
            raise ValueError("fused_allreduce_ needs contiguous tensors")
    pp, _keep1 = _lib.ptr_array([t.data_ptr() for t in tensor_list])
    cp, _keep2 = _lib.i64_array([t.numel() for t in tensor_list])
    _lib.call("tips_fused_allreduce", pp, cp, len(tensor_list), code, tensors.stream_of(tensor_list[0]))
    return tensor_list


def bucket_sum(a, b, out=None):
    """out = a + b on the device: the per-chunk reduction kernel on its own (tips_bucket_sum)."""
    if not (tensors.is_device(a) and tensors.is_device(b)):
        raise ValueError("bucket_sum needs device tensors")
    if a.shape != b.shape or a.dtype != b.dtype:
        raise ValueError("bucket_sum needs equal shapes and dtypes")
    a, b = a.contiguous(), b.contiguous()
    if out is None:
        out = tensors.empty_like(a)
    _lib.call("tips_bucket_sum", out.data_ptr(), a.data_ptr(), b.data_ptr(), a.numel(), tensors.dtype_code(a),
              tensors.stream_of(a))
    return out


def set_algorithm(algo):
    """Select 'auto', 'ring', 'direct' or 'rccl'; returns the previous selection's name."""
    names = {"auto": _lib.ALGO_AUTO, "ring": _lib.ALGO_RING, "direct": _lib.ALGO_DIRECT, "rccl": _lib.ALGO_RCCL}
    inv = {v: k for k, v in names.items()}
    prev = _lib.lib().tips_get_algorithm()
    _lib.call("tips_set_algorithm", names[algo])
    return inv.get(prev, str(prev))
