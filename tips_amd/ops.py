"""Op bindings — mirrors tips/tensorflow/ops.py:24-95 over the C-ABI.

`allreduce_op` is the MPIAllreduce op (ops.cc:79-136): an out-of-place SUM of
one tensor over all ranks, output of the input's shape and dtype. Device
(torch CUDA/HIP) tensors stay in HBM and are ordered on the caller's current
stream; host tensors (numpy / CPU torch) are staged through HBM and the call
returns when the result is in host memory, like the reference's CPU op.
"""
import os
import re
import threading

from . import _fast  # (built in-tree by `make`: tips_amd/_fast*.so; no Python fallback)
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


_check = os.environ.get("TIPS_CHECK_CONSISTENCY", "0") == "1"


def set_consistency_check(enabled):
    """Validate dtype/shape across ranks before every allreduce (the reference's rank-0
    negotiation, coordinator.cc:90-186): one small exchange per call. Off by default."""
    global _check
    _check = bool(enabled)


def _shape(t):
    return tuple(int(d) for d in t.shape)


def allreduce_op(tensor, name=None):
    """Sum `tensor` over all ranks (ops.py:61-65 -> MPIAllreduce, ops.cc:86-115). With a `name`,
    through the negotiation like the reference's op (rank 0 validates and orders it; the name
    normalised as ops.py:33-35 does), and returns when it has run; without one, stream-ordered."""
    if name is not None:
        return synchronize(allreduce_async(tensor, _normalize_name(name)))
    basics.init()
    code = tensors.dtype_code(tensor)
    src = tensors.contiguous(tensor)
    out = _HOST_OUT.take(src) if not tensors.is_device(src) else tensors.empty_like(src)
    n = tensors.numel(src)
    if _check:
        shape = _shape(src) or (1,)  # scalars travel as shape [1] (CreateNoEmptyTfShape, coordinator.cc:212-221)
        sp, _keep = _lib.i64_array(shape)
        _lib.call("tips_allreduce_checked", tensors.data_ptr(src), tensors.data_ptr(out), sp, len(shape), code,
                  _lib.OP_SUM, tensors.stream_of(src))
    elif n:
        _lib.call("tips_allreduce", tensors.data_ptr(src), tensors.data_ptr(out), n, code, _lib.OP_SUM,
                  tensors.stream_of(src))
    return out


class _HostOutPool(object):
    """Outputs of host allreduces of at least 1 MiB (the reference's op works on CPU tensors,
    ops.cc:118): kept page-locked (tips_host_register) and handed out again once the caller has
    released them - no Python reference left and, for torch, no other tensor on the storage (numpy
    views hold a reference to their base). A fresh numpy / torch array of that size is new pages every
    call, and the D2H into it pays their first-touch faults: one 97.6 MiB numpy buffer took 16.7 ms
    per allreduce that way (profiles/r03/p_numa_probe.jsonl). Up to PER_KEY outputs per (kind, dtype,
    shape), TIPS_HOST_OUT_POOL_MIB (4096) page-locked in all; past that, fresh outputs as before."""

    MIN_BYTES = 1 << 20
    PER_KEY = 2

    def __init__(self):
        self.sets = {}
        self.bytes = 0
        self.lock = threading.Lock()

    @staticmethod
    def _free(e):
        import sys
        a = e[0]
        if sys.getrefcount(a) > 3:  # (the entry, the local a, getrefcount's argument)
            return False
        if e[1] is not None:  # torch: no other tensor on the storage
            import torch
            return torch._C._storage_Use_Count(a.untyped_storage()._cdata) == e[1]
        return True

    def take(self, src):
        is_t = tensors.is_torch(src)
        nbytes = src.numel() * src.element_size() if is_t else src.nbytes
        if nbytes < self.MIN_BYTES:
            return tensors.empty_like(src)
        key = (is_t, str(src.dtype), tuple(src.shape))
        with self.lock:  # (the check and the hand-out together: another thread cannot get it too)
            lst = self.sets.setdefault(key, [])
            for e in lst:
                if self._free(e):
                    return e[0]
            out = tensors.empty_like(src)
            cap = int(os.environ.get("TIPS_HOST_OUT_POOL_MIB", "4096")) << 20
            if len(lst) < self.PER_KEY and self.bytes + nbytes <= cap:
                if _lib.lib().tips_host_register(tensors.data_ptr(out), nbytes) == 0:
                    use0 = None
                    if is_t:
                        import torch
                        use0 = torch._C._storage_Use_Count(out.untyped_storage()._cdata)
                    lst.append((out, use0))
                    self.bytes += nbytes
            return out


_HOST_OUT = _HostOutPool()


def allgather_op(tensor, name=None):
    """Concatenate `tensor` from all ranks along dimension 0 (ops.py:72-76 -> MPIAllgather,
    ops.cc:156-212; sizes exchanged as GatherFirstRankSizes does, coordinator.cc:40-88). With a
    `name`, through the negotiation (allgather_async), as allreduce_op."""
    if name is not None:
        return synchronize(allgather_async(tensor, _normalize_name(name)))
    basics.init()
    code = tensors.dtype_code(tensor)
    src = tensors.contiguous(tensor)
    shape = _shape(src)
    if not shape:
        raise ValueError("An empty tensor found")
    if _check:
        rec = [_lib.REQ_ALLGATHER, code, len(shape)] + list(shape) + [0] * (_lib.MAX_DIMS - len(shape))
        table = _gather_records(rec)
        _lib.call("tips_check_requests", _lib.i64_array(table)[0], len(table) // _lib.REQUEST_WORDS)
    firsts = _allgather_i64([shape[0]])
    row = 1
    for d in shape[1:]:
        row *= d
    counts = [int(f) * row for f in firsts]
    out_shape = (sum(int(f) for f in firsts),) + shape[1:]
    if tensors.is_torch(src):
        import torch
        out = torch.empty(out_shape, dtype=src.dtype, device=src.device)
    else:
        import numpy as np
        out = np.empty(out_shape, dtype=src.dtype)
    cp, _keep = _lib.i64_array(counts)
    _lib.call("tips_allgatherv", tensors.data_ptr(src), tensors.numel(src), tensors.data_ptr(out), cp, code,
              tensors.stream_of(src))
    return out


def _allgather_i64(values):
    """Every rank's int64 words, rank-major (tips_allgather_i64)."""
    import ctypes
    p = basics.size()
    vp, _keep = _lib.i64_array(values)
    out = (ctypes.c_int64 * (p * len(values)))()
    _lib.call("tips_allgather_i64", vp, len(values), out)
    return [int(v) for v in out]


def _gather_records(rec):
    """Every rank's request record (rank-major table for tips_check_requests)."""
    return _allgather_i64(rec)


def broadcast_op(tensor, root_rank=0, name=None):
    """`tensor` of rank `root_rank`, on every rank (ops.py:83-87 -> MPIBroadcast, ops.cc:214-286).
    With a `name`, through the negotiation (broadcast_async), as allreduce_op."""
    if name is not None:
        return synchronize(broadcast_async(tensor, root_rank, _normalize_name(name)))
    basics.init()
    code = tensors.dtype_code(tensor)
    src = tensors.contiguous(tensor)
    out = _HOST_OUT.take(src) if not tensors.is_device(src) else tensors.empty_like(src)
    n = tensors.numel(src)
    if n:
        _lib.call("tips_broadcast", tensors.data_ptr(src), tensors.data_ptr(out), n, code, int(root_rank),
                  tensors.stream_of(src))
    return out


def broadcast_variables(variables, root_rank=0):
    """Overwrite each tensor in place with root_rank's value (functions.py:36-46)."""
    for v in variables:
        b = broadcast_op(v, root_rank)
        if tensors.is_torch(v):
            v.copy_(b)
        else:
            v[...] = b
    return variables


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
    code = _check_fusable(tensor_list, "fused_allreduce_")
    pp, _keep1 = _lib.ptr_array([t.data_ptr() for t in tensor_list])
    cp, _keep2 = _lib.i64_array([t.numel() for t in tensor_list])
    _lib.call("tips_fused_allreduce", pp, cp, len(tensor_list), code, tensors.stream_of(tensor_list[0]))
    return tensor_list


def fused_allreduce(tensor_list, out_list=None):
    """Out-of-place SUM of a list of same-dtype device tensors through the fusion buckets
    (tips_fused_allreduce_oop): returns new tensors (or fills `out_list`), inputs unchanged.
    Pack reads each input once and unpack writes each output once: 4 x the bytes in HBM
    traffic, no extra copy."""
    basics.init()
    if not tensor_list:
        return []
    code = _check_fusable(tensor_list, "fused_allreduce")
    outs = [tensors.empty_like(t) for t in tensor_list] if out_list is None else list(out_list)
    if len(outs) != len(tensor_list) or any(o.shape != t.shape or o.dtype != t.dtype or not o.is_contiguous()
                                            for o, t in zip(outs, tensor_list)):
        raise ValueError("out_list must hold one contiguous tensor of each input's shape and dtype")
    pi, _keep1 = _lib.ptr_array([t.data_ptr() for t in tensor_list])
    po, _keep2 = _lib.ptr_array([o.data_ptr() for o in outs])
    cp, _keep3 = _lib.i64_array([t.numel() for t in tensor_list])
    _lib.call("tips_fused_allreduce_oop", pi, po, cp, len(tensor_list), code, tensors.stream_of(tensor_list[0]))
    return outs


_WIRE_CODES = {"float16": _lib.FLOAT16, "bfloat16": _lib.BFLOAT16}


def fused_allreduce_cast(tensor_list, wire="float16"):
    """SUM of a list of float32 device tensors reduced in a 16-bit wire type
    (tips_fused_allreduce_cast): each tensor is cast to `wire` (round to nearest even) as it is
    packed into a fusion bucket, every bucket is allreduced in the wire type, and the sums are cast
    back to float32 as they are unpacked - Compression.fp16's compress -> allreduce -> decompress
    (tips/tensorflow/compression.py:49-66) with one pack and one unpack launch per bucket instead of
    two casts per tensor. Returns float32 views of one flat buffer (reused, as fused_allreduce_flat's,
    once every view is released); inputs unchanged."""
    basics.init()
    if not tensor_list:
        return []
    code = _check_fusable(tensor_list, "fused_allreduce_cast")
    if code != _lib.FLOAT32:
        raise TypeError("fused_allreduce_cast: float32 tensors only (got dtype code %d)" % code)
    if wire not in _WIRE_CODES:
        raise ValueError("fused_allreduce_cast: wire must be one of %s" % sorted(_WIRE_CODES))
    res = _dev_list_cast(tensor_list, _WIRE_CODES[wire])  # (dense, contiguous, one device: C++ reads the list)
    if res is not None:
        return res
    fo = _flat_outputs(tensor_list, code)
    flat, views = fo.take()
    pi, _keep1 = _lib.ptr_array([t.data_ptr() for t in tensor_list])
    _lib.call("tips_fused_allreduce_cast", pi, _out_ptrs(fo, flat), fo.cp[0], len(tensor_list), code, _WIRE_CODES[wire],
              tensors.stream_of(tensor_list[0]))
    return views


class _FlatOutputs(object):
    """Output sets of fused_allreduce_flat for one list signature (dtype, device, shapes): the
    layout's byte offsets (tips_fused_layout: a function of the counts alone) and a few sets of
    {one flat buffer, one view of it per tensor}. A set is handed out again once every tensor of
    it has been released by the caller: no Python reference to any of its views, and no other
    tensor sharing its storage (derived views included). Allocating the buffer and 1000 views per
    call costs milliseconds of host time - more than the device work of the whole allreduce."""

    MAX_SETS = 4

    def __init__(self, shapes, numels, code, dtype, device):
        import torch
        self.numels = numels
        import ctypes
        cp, _keep = _lib.i64_array(numels)
        offs = (ctypes.c_int64 * len(numels))()
        self.total = _lib.check("tips_fused_layout", _lib.lib().tips_fused_layout(cp, len(numels), code, offs))
        self.es = torch.empty((), dtype=dtype).element_size()
        self.offs = [int(o) // self.es for o in offs]
        self.shapes, self.dtype, self.device = shapes, dtype, device
        self.sets = []
        self.lock = threading.Lock()  # (the free check and the hand-out together, as _HostOutPool)

    def _free(self, s):
        flat, views, use0, rc0 = s
        import torch
        if torch._C._storage_Use_Count(flat.untyped_storage()._cdata) != use0:
            return False
        return _fast.max_refcount(views) <= rc0

    def take(self):
        """(flat buffer, a new list of its views) for this call: a released set, or a new one. The
        list is made here, before the library call releases the GIL, so another thread's take()
        already sees the set's views referenced and does not hand it out twice."""
        import torch
        with self.lock:  # another thread's take() cannot see a set free between the check and the copy
            for s in self.sets:
                if self._free(s):
                    return s[0], list(s[1])
            flat = torch.empty(max(1, self.total // self.es), dtype=self.dtype, device=self.device)
            views = [flat[o:o + n].view(shp) for o, n, shp in zip(self.offs, self.numels, self.shapes)]
            if len(self.sets) < self.MAX_SETS:
                use0 = torch._C._storage_Use_Count(flat.untyped_storage()._cdata)
                rc0 = _fast.max_refcount(views)
                self.sets.append((flat, views, use0, rc0))
            return flat, list(views)


_FLAT_OUTPUTS = {}  # (dtype, device, shapes, layout settings) -> _FlatOutputs (small LRU)


def _layout_settings():
    """The settings a fusion layout depends on besides the counts (fusion.cc reads them per call):
    part of every flat-output cache key, so a changed setting never reuses offsets of another layout."""
    env = os.environ
    return (env.get("TIPS_FUSION_THRESHOLD"), env.get("TIPS_COPY_TILE_BYTES"), env.get("TIPS_FUSION_BALANCE"))


def fused_allreduce_flat(tensor_list):
    """Out-of-place SUM of a list of same-dtype device tensors (tips_fused_allreduce_flat): the
    outputs are views of ONE flat buffer laid out as the fusion buckets - each bucket packed straight
    into it and allreduced there in place, no slot and no unpack (2 x the bytes of HBM traffic). The
    flat buffer and views are reused for a later call of the same list signature once the caller has
    released every output (_FlatOutputs). Inputs unchanged."""
    basics.init()
    if not tensor_list:
        return []
    code = _check_fusable(tensor_list, "fused_allreduce_flat")
    return _flat_call(tensor_list, code, [t.data_ptr() for t in tensor_list])


def _flat_outputs(tensor_list, code):
    """The _FlatOutputs of this list's signature (dtype, device, shapes)."""
    t0 = tensor_list[0]
    shapes = tuple(t.shape for t in tensor_list)
    key = (t0.dtype, t0.device, shapes, _layout_settings())
    fo = _FLAT_OUTPUTS.get(key)
    if fo is None:
        if len(_FLAT_OUTPUTS) >= 16:
            _FLAT_OUTPUTS.pop(next(iter(_FLAT_OUTPUTS)))
        fo = _FLAT_OUTPUTS[key] = _FlatOutputs(shapes, [t.numel() for t in tensor_list], code, t0.dtype, t0.device)
        fo.cp = _lib.i64_array(fo.numels)
        fo.code = code
        fo.last = (None, None)  # (pointer list, its ptr_array) of the previous call
    return fo


def _flat_run(fo, tensor_list, ptrs):
    """tips_fused_allreduce_flat of `tensor_list` (whose data pointers are `ptrs`) into an output set
    of `fo`; returns the outputs."""
    last = fo.last  # (one read: another thread may replace it)
    if ptrs == last[0]:
        pp = last[1]
    else:
        pp = _lib.ptr_array(ptrs)
        fo.last = (ptrs, pp)
    flat, views = fo.take()
    t0 = tensor_list[0]
    _lib.call("tips_fused_allreduce_flat", pp[0], fo.cp[0], len(ptrs), fo.code, flat.data_ptr(),
              _torch_mod().cuda.current_stream(t0.device).cuda_stream)
    return views


def _torch_mod():
    import torch
    return torch


# c10::ScalarType -> tips dtype code (Float, Double, Int, Long, Half, BFloat16)
_ST_CODES = {6: _lib.FLOAT32, 7: _lib.FLOAT64, 3: _lib.INT32, 4: _lib.INT64, 5: _lib.FLOAT16, 15: _lib.BFLOAT16}
_LIST_BUFS = threading.local()  # .d: n -> (pointer array, count array, their addresses), per thread:
                                # the library call releases the GIL while it reads them
_FAST_FLAT = {}   # (scalar type, device, n, shape hash, layout settings) -> (_FlatOutputs, count bytes)
_CUR_STREAM = None


def _dev_list_flat(tensor_list):
    """fused_allreduce_flat of a list of dense, contiguous device tensors of one dtype on one
    device, with the per-tensor host work in C++ (_fast.dev_list: data pointers, counts, a hash of
    the shapes): the outputs, or None when the list is not such a list (the caller's general path
    then inspects it tensor by tensor). A training loop hands over fresh gradient tensors every
    step; this costs tens of nanoseconds per tensor where reading them through Python cost ~0.2 us."""
    global _CUR_STREAM
    n = len(tensor_list)
    mine = getattr(_LIST_BUFS, "d", None)
    if mine is None:
        mine = _LIST_BUFS.d = {}
    bufs = mine.get(n)
    if bufs is None:
        import ctypes
        pa, na = (ctypes.c_void_p * n)(), (ctypes.c_int64 * n)()
        if len(mine) >= 16:
            mine.pop(next(iter(mine)))
        bufs = mine[n] = (pa, na, ctypes.addressof(pa), ctypes.addressof(na))
    r = _fast.dev_list(tensor_list, bufs[2], bufs[3], 1, n)
    if r is None or r[0] not in _ST_CODES:
        return None
    import ctypes
    key = (r[0], r[1], n, r[2], _layout_settings())
    hit = _FAST_FLAT.get(key)
    counts = ctypes.string_at(bufs[3], 8 * n)
    if hit is None or hit[1] != counts:
        fo = _flat_outputs(tensor_list, _ST_CODES[r[0]])
        if len(_FAST_FLAT) >= 16:
            _FAST_FLAT.pop(next(iter(_FAST_FLAT)))
        _FAST_FLAT[key] = hit = (fo, counts)
    fo = hit[0]
    flat, views = fo.take()
    if _CUR_STREAM is None:
        import torch
        _CUR_STREAM = torch.cuda.current_stream
    _lib.call("tips_fused_allreduce_flat", bufs[0], fo.cp[0], n, fo.code, flat.data_ptr(),
              _CUR_STREAM(tensor_list[0].device).cuda_stream)
    return views


def _dev_list_cast(tensor_list, wire=_lib.FLOAT16):
    """fused_allreduce_cast of a list of dense, contiguous float32 device tensors on one device,
    with the per-tensor host work in C++ as _dev_list_flat's (Compression.fp16's fast path in
    allreduce_grads); the float32 outputs, or None when the list is not such a list."""
    global _CUR_STREAM
    n = len(tensor_list)
    mine = getattr(_LIST_BUFS, "d", None)
    if mine is None:
        mine = _LIST_BUFS.d = {}
    bufs = mine.get(n)
    if bufs is None:
        import ctypes
        pa, na = (ctypes.c_void_p * n)(), (ctypes.c_int64 * n)()
        if len(mine) >= 16:
            mine.pop(next(iter(mine)))
        bufs = mine[n] = (pa, na, ctypes.addressof(pa), ctypes.addressof(na))
    r = _fast.dev_list(tensor_list, bufs[2], bufs[3], 1, n)
    if r is None or _ST_CODES.get(r[0]) != _lib.FLOAT32:
        return None
    import ctypes
    key = (r[0], r[1], n, r[2], _layout_settings())
    hit = _FAST_FLAT.get(key)
    counts = ctypes.string_at(bufs[3], 8 * n)
    if hit is None or hit[1] != counts:
        fo = _flat_outputs(tensor_list, _lib.FLOAT32)
        if len(_FAST_FLAT) >= 16:
            _FAST_FLAT.pop(next(iter(_FAST_FLAT)))
        _FAST_FLAT[key] = hit = (fo, counts)
    fo = hit[0]
    flat, views = fo.take()
    if _CUR_STREAM is None:
        import torch
        _CUR_STREAM = torch.cuda.current_stream
    _lib.call("tips_fused_allreduce_cast", bufs[0], _out_ptrs(fo, flat), fo.cp[0], n, _lib.FLOAT32, wire,
              _CUR_STREAM(tensor_list[0].device).cuda_stream)
    return views


def _out_ptrs(fo, flat):
    """The data pointers of an output set's views (flat buffer + each view's offset), as a void**,
    cached per flat buffer."""
    cache = fo.__dict__.setdefault("out_ptrs", {})
    base = flat.data_ptr()
    hit = cache.get(base)
    if hit is None:
        import ctypes
        import numpy as np
        arr = np.asarray(fo.offs, dtype=np.uint64) * np.uint64(fo.es) + np.uint64(base)
        if len(cache) >= 2 * _FlatOutputs.MAX_SETS:
            cache.pop(next(iter(cache)))
        hit = cache[base] = (arr, ctypes.cast(arr.ctypes.data, ctypes.POINTER(ctypes.c_void_p)))
    return hit[1]


def _flat_call(tensor_list, code, ptrs):
    return _flat_run(_flat_outputs(tensor_list, code), tensor_list, ptrs)


def fused_allreduce_host(tensor_list, out_list=None):
    """Out-of-place SUM of a list of same-dtype HOST tensors (numpy / CPU torch) through
    tips_fused_allreduce_host: packed by the library's host threads into page-locked pieces,
    each piece H2D -> allreduce -> D2H pipelined, unpacked into the outputs. Returns when done."""
    basics.init()
    if not tensor_list:
        return []
    code = tensors.dtype_code(tensor_list[0])
    srcs = []
    for t in tensor_list:
        if tensors.is_device(t):
            raise ValueError("fused_allreduce_host needs host tensors")
        if tensors.dtype_code(t) != code:
            raise TypeError("fused_allreduce_host needs one dtype per call")
        srcs.append(tensors.contiguous(t))
    outs = [tensors.empty_like(s) for s in srcs] if out_list is None else list(out_list)
    pi, _k1 = _lib.ptr_array([tensors.data_ptr(s) for s in srcs])
    po, _k2 = _lib.ptr_array([tensors.data_ptr(o) for o in outs])
    cp, _k3 = _lib.i64_array([tensors.numel(s) for s in srcs])
    _lib.call("tips_fused_allreduce_host", pi, po, cp, len(srcs), code)
    return outs


class _HostFlatOutputs(object):
    """Output sets of fused_allreduce_host_flat for one host list signature (numpy, or CPU torch):
    one flat host buffer laid out as tips_fused_layout, page-locked once (tips_host_register) so
    the device writes the sums straight into it, and one view of it per tensor. A set is handed out
    again once every output of it has been released (as _FlatOutputs: no reference to a view, no
    other array or tensor on its memory)."""

    MAX_SETS = 4

    def __init__(self, shapes, numels, code, dtype, is_torch):
        import ctypes
        cp, _keep = _lib.i64_array(numels)
        offs = (ctypes.c_int64 * len(numels))()
        self.total = max(256, _lib.check("tips_fused_layout", _lib.lib().tips_fused_layout(cp, len(numels), code, offs)))
        self.cp = _lib.i64_array(numels)
        self.code, self.numels, self.shapes, self.dtype, self.is_torch = code, numels, shapes, dtype, is_torch
        self.es = _itemsize(dtype, is_torch)
        self.offs = [int(o) for o in offs]
        self.sets = []
        self.last = (None, None)  # (pointer list, its ptr_array) of the previous call
        self.lock = threading.Lock()

    def _refs(self, s):
        """(references to the flat buffer, most references to one view) of set s. Measured the same
        way when a set is made (its baseline) and when it is looked at again, so a set is free
        exactly when nothing beyond the set itself refers to it: a view held, or an array / tensor
        made from one (numpy collapses every view's .base to the owner; torch counts storage users)."""
        import sys
        if self.is_torch:
            import torch
            n = torch._C._storage_Use_Count(s[0].untyped_storage()._cdata)
        else:
            n = sys.getrefcount(s[0])
        return n, max(map(sys.getrefcount, s[1]), default=0)

    def take(self):
        """(flat buffer, a new list of its views): made before the library call releases the GIL,
        as _FlatOutputs.take, under the object's lock."""
        with self.lock:
            for s in self.sets:
                if self._refs(s) == s[2]:
                    return s[0], list(s[1])
            import numpy as np
            mem = np.empty(self.total, dtype=np.uint8)
            if self.is_torch:
                import torch
                flat = torch.from_numpy(mem)  # (the storage keeps `mem` alive: see _register_until_freed)
                views = [flat[o:o + n * self.es].view(self.dtype).view(shp)
                         for o, n, shp in zip(self.offs, self.numels, self.shapes)]
            else:
                flat = mem
                views = [flat[o:o + n * self.es].view(self.dtype).reshape(shp)
                         for o, n, shp in zip(self.offs, self.numels, self.shapes)]
            if len(self.sets) < self.MAX_SETS:
                # a kept set is page-locked while its memory lives (the device's D2H lands in it
                # directly); one past MAX_SETS is not (it is freed with its last output)
                _register_until_freed(mem, self.total)
                del mem
                st = [flat, views, None]
                del flat, views  # (the baseline counts the set's own references only)
                st[2] = self._refs(st)
                self.sets.append(st)
                return st[0], list(st[1])
            return flat, views


def _register_until_freed(mem, nbytes):
    """Page-lock a numpy host buffer (tips_host_register) and unregister it just before its memory
    is freed: numpy views hold their base, and a torch tensor made by torch.from_numpy holds the
    array from its storage, so the array dies with the last output that uses its memory. A set
    evicted from _HOST_FLAT is therefore unregistered once its last output is released - never while
    a call writes into it (the call holds the buffer) - and no later allocation at the same address
    finds a stale registration."""
    import weakref
    ptr = mem.ctypes.data
    _lib.call("tips_host_register", ptr, nbytes)
    weakref.finalize(mem, _unregister, ptr).atexit = False  # (at exit the process's pages go anyway)


def _unregister(ptr):
    try:
        _lib.lib().tips_host_unregister(ptr)
    except Exception:  # noqa: BLE001 - at interpreter exit the library may be gone
        pass


def _itemsize(dtype, is_torch):
    if is_torch:
        import torch
        return torch.empty((), dtype=dtype).element_size()
    import numpy as np
    return np.dtype(dtype).itemsize


_HOST_FLAT = {}  # (dtype, torch?, shapes, layout settings) -> _HostFlatOutputs


def fused_allreduce_host_flat(tensor_list):
    """Out-of-place SUM of a list of same-dtype HOST tensors (numpy / CPU torch), the outputs views
    of one page-locked flat host buffer (tips_fused_allreduce_host_flat): host threads pack the
    inputs into page-locked pieces, each piece H2D -> allreduce -> D2H straight into the output
    buffer - no unpack. The buffer and its views are reused by a later call of the same list
    signature once the caller has released every output. Returns when the outputs are written."""
    basics.init()
    if not tensor_list:
        return []
    code = tensors.dtype_code(tensor_list[0])
    srcs = []
    for t in tensor_list:
        if tensors.is_device(t):
            raise ValueError("fused_allreduce_host_flat needs host tensors")
        if tensors.dtype_code(t) != code:
            raise TypeError("fused_allreduce_host_flat needs one dtype per call")
        srcs.append(tensors.contiguous(t))
    return _host_flat_run(_host_flat_outputs(srcs), [tensors.data_ptr(s) for s in srcs])


def _host_flat_outputs(srcs):
    """The _HostFlatOutputs of this host list's signature (dtype, numpy or torch, shapes); srcs are
    contiguous host tensors of one dtype."""
    is_torch = tensors.is_torch(srcs[0])
    shapes = tuple(tuple(s.shape) for s in srcs)
    key = (str(srcs[0].dtype), is_torch, shapes, _layout_settings())
    fo = _HOST_FLAT.get(key)
    if fo is None:
        if len(_HOST_FLAT) >= 16:
            _HOST_FLAT.pop(next(iter(_HOST_FLAT)))
        fo = _HOST_FLAT[key] = _HostFlatOutputs(shapes, [tensors.numel(s) for s in srcs],
                                                tensors.dtype_code(srcs[0]), srcs[0].dtype, is_torch)
    return fo


def _host_flat_run(fo, ptrs):
    """tips_fused_allreduce_host_flat of the host tensors at `ptrs` into an output set of `fo`;
    returns the outputs (views of the set's flat buffer)."""
    last = fo.last  # (one read: another thread may replace it)
    if ptrs == last[0]:
        pp = last[1]
    else:
        pp = _lib.ptr_array(ptrs)
        fo.last = (ptrs, pp)
    flat, views = fo.take()
    _lib.call("tips_fused_allreduce_host_flat", pp[0], fo.cp[0], len(ptrs), fo.code, tensors.data_ptr(flat))
    return views


def fusion_stats():
    """{layouts_built, layout_hits, tables_built, table_hits} of this process's fusion caches
    (tips_fusion_stats): layouts depend on the counts only, tables on the pointers."""
    import ctypes
    v = [ctypes.c_int64() for _ in range(4)]
    _lib.call("tips_fusion_stats", *[ctypes.byref(x) for x in v])
    return dict(zip(("layouts_built", "layout_hits", "tables_built", "table_hits"), [x.value for x in v]))


class FusedList(object):
    """A list of device tensors reduced in place together, step after step (a model's gradients).

    fused_allreduce_ validates every tensor and rebuilds the pointer arrays on each call; for a
    list that keeps the same tensors (or a new tensor at the same address) that host work is
    repeated for nothing, and for 1000 gradients it costs more than the pack + unpack kernels
    themselves. This keeps the validated arrays and, per call, only re-reads the data pointers:
    when they are unchanged the cached arrays go straight to tips_fused_allreduce.

    `counts` fixes the element count of each position (a parameter's gradient always has the
    parameter's shape, which torch enforces on assignment); a list whose counts differ is refused."""

    def __init__(self, counts):
        self._counts = [int(c) for c in counts]
        self._ptrs = None
        self._arrays = None
        self._cp = _lib.i64_array(self._counts)
        self._count_bytes = self._cp[1].tobytes()  # (little-endian int64, as _fast.dev_list writes them)
        self._tls = threading.local()  # per-thread scratch: the library call releases the GIL

    def allreduce_(self, tensor_list):
        if not tensor_list:
            return tensor_list
        import ctypes
        n = len(tensor_list)
        sc = getattr(self._tls, "sc", None)
        if sc is None or len(sc[0]) != n:
            pa, na = (ctypes.c_void_p * n)(), (ctypes.c_int64 * n)()
            sc = self._tls.sc = (pa, na, ctypes.addressof(pa), ctypes.addressof(na))
        # pointers, counts and dtype read in C++ (_fast.dev_list); the Python checks below only when
        # the list is not one dtype of dense contiguous device tensors, or its pointers changed
        r = _fast.dev_list(tensor_list, sc[2], sc[3], 1, n)
        cur = ctypes.string_at(sc[2], 8 * n) if r is not None else None
        if r is None or cur != self._ptrs:
            code = _check_fusable(tensor_list, "fused_allreduce_")
            basics.init()
            if len(tensor_list) != len(self._counts) or (r is not None and ctypes.string_at(sc[3], 8 * n) != self._count_bytes) \
                    or (r is None and [t.numel() for t in tensor_list] != self._counts):
                raise ValueError("FusedList: the tensors' element counts changed")
            ptrs = [t.data_ptr() for t in tensor_list]
            self._ptrs, self._arrays = cur, (code,) + _lib.ptr_array(ptrs)
        code, pp = self._arrays[0], self._arrays[1]
        _lib.call("tips_fused_allreduce", pp, self._cp[0], n, code, tensors.stream_of(tensor_list[0]))
        return tensor_list


def _check_fusable(tensor_list, what):
    code = tensors.dtype_code(tensor_list[0])
    for t in tensor_list:
        if not tensors.is_device(t):
            raise ValueError("%s needs device tensors" % what)
        if tensors.dtype_code(t) != code:
            raise TypeError("%s needs one dtype per call" % what)
        if not t.is_contiguous():
            raise ValueError("%s needs contiguous tensors" % what)
    return code


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


_INFLIGHT = {}  # handle -> Handle: the buffers of every named request stay alive until it has run


class Handle(object):
    """An in-flight named request (tips_enqueue_allreduce / _broadcast / _allgather); see
    allreduce_async, broadcast_async, allgather_async. Until the request has run (synchronize /
    poll reports it, or it failed) the module holds it, with its input and output: the library
    reads and writes them when rank 0's order reaches the name, possibly after the caller dropped
    its own references (a freed host buffer would be written into; a freed device block could
    already belong to another tensor)."""

    def __init__(self, handle, output, name):
        self.handle = handle
        self.output = output
        self.name = name
        self.done = False
        self._finish = None  # allgather: builds the output once the request has run

    def _track(self):
        _INFLIGHT[self.handle] = self
        return self

    def _release(self):
        _INFLIGHT.pop(self.handle, None)

    def _complete(self):
        self._release()
        self.done = True
        if self._finish is not None:
            self.output = self._finish()
            self._finish = None


def allreduce_async(tensor, name):
    """Start a negotiated SUM of a device tensor under `name` and return a Handle.

    The reference's op path (MPIAllreduce -> EnqueueTensorCollective -> rank-0
    negotiation, ops.cc:86-115, coordinator.cc:223-513): ranks may call this in
    any order; each named tensor is reduced once every rank has enqueued it, in
    rank 0's order, with the reference's dtype/shape validation. `name` must be
    the same on every rank (the reference uses the TF node name). Device tensors are reduced
    stream-ordered; host tensors (numpy / CPU torch: the reference's op is a CPU op) on the
    negotiation thread, done when synchronize() returns."""
    basics.init()
    code = tensors.dtype_code(tensor)
    src = tensors.contiguous(tensor)
    out = tensors.empty_like(src)
    shape = _shape(src)  # validated across ranks with ConstructResponseMessage's rule (coordinator.cc:129-146)
    sp, _keep = _lib.i64_array(shape or [1])
    h = _lib.lib().tips_enqueue_allreduce_shaped(name.encode(), tensors.data_ptr(src), tensors.data_ptr(out), sp,
                                                 len(shape), code, tensors.stream_of(src))
    if h < 0:
        raise _lib.TipsError("tips_enqueue_allreduce", int(h), _lib.last_error())
    hd = Handle(int(h), out, name)
    hd._keep = src  # the input must stay alive until the reduction has run
    return hd._track()


def broadcast_async(tensor, root_rank, name):
    """Start a negotiated broadcast of a device tensor under `name` (MPIBroadcast, ops.cc:214-286 ->
    EnqueueTensorCollective(RequestType_BROADCAST)); the Handle's output is root_rank's tensor.
    Ranks may call it in any order; rank 0 checks dtype, shape and root on every rank. Device or
    host tensors, as allreduce_async."""
    basics.init()
    code = tensors.dtype_code(tensor)
    src = tensors.contiguous(tensor)
    out = tensors.empty_like(src)
    shape = _shape(src)
    sp, _keep = _lib.i64_array(shape or [1])
    h = _lib.lib().tips_enqueue_broadcast(name.encode(), tensors.data_ptr(src), tensors.data_ptr(out), sp, len(shape),
                                          code, int(root_rank), tensors.stream_of(src))
    if h < 0:
        raise _lib.TipsError("tips_enqueue_broadcast", int(h), _lib.last_error())
    hd = Handle(int(h), out, name)
    hd._keep = src
    return hd._track()


def allgather_async(tensor, name):
    """Start a negotiated allgather of a device tensor under `name` (MPIAllgather, ops.cc:156-212
    -> RequestType_ALLGATHER): every rank's tensor concatenated along dimension 0 in rank order.
    Rank 0 checks all but the first dimension (GatherFirstRankSizes, coordinator.cc:40-88) and
    sends every rank the first dimensions; the output is allocated then, on the negotiation
    thread, through a callback (as the reference's allocate_output in PerformCollectiveOp). Device
    or host tensors, as allreduce_async (a host tensor gets a host output)."""
    import ctypes
    import numpy as np
    basics.init()
    code = tensors.dtype_code(tensor)
    src = tensors.contiguous(tensor)
    shape = _shape(src)
    if not shape:
        raise ValueError("An empty tensor found")
    sp, _keep = _lib.i64_array(shape)
    rows = ctypes.c_int64(-1)
    hd = Handle(0, None, name)
    box = {}

    torch_src = tensors.is_torch(src)
    req_stream = None
    if torch_src and src.is_cuda:
        import torch
        req_stream = torch.cuda.current_stream(src.device)  # the stream the request runs on

    def alloc(_ctx, nbytes):
        if torch_src:
            import contextlib
            import torch
            # allocated on the negotiation thread, but the transfer writes it on the request's
            # stream: allocate under that stream, so the caching allocator ties the block to it
            with torch.cuda.stream(req_stream) if req_stream is not None else contextlib.nullcontext():
                buf = torch.empty(int(nbytes), dtype=torch.uint8, device=src.device)
        else:
            buf = np.empty(int(nbytes), dtype=np.uint8)
        box["buf"] = buf
        return tensors.data_ptr(buf)

    cb = _lib.ALLOC_FN(alloc)

    def finish():
        out_shape = (int(rows.value),) + tuple(shape[1:])
        if "buf" in box:
            return box.pop("buf").view(src.dtype).reshape(out_shape)
        if torch_src:
            import torch
            return torch.empty(out_shape, dtype=src.dtype, device=src.device)
        return np.empty(out_shape, dtype=src.dtype)

    h = _lib.lib().tips_enqueue_allgather(name.encode(), tensors.data_ptr(src), sp, len(shape), code,
                                          tensors.stream_of(src), ctypes.cast(cb, ctypes.c_void_p), None,
                                          ctypes.byref(rows))
    if h < 0:
        raise _lib.TipsError("tips_enqueue_allgather", int(h), _lib.last_error())
    hd.handle = int(h)
    hd._keep = (src, sp, rows, cb)  # alive until the request has run (the callback, the out-param)
    hd._finish = finish
    return hd._track()


def allreduce_async_many(tensor_list, names):
    """allreduce_async over a list in one library call (tips_enqueue_allreduce_n): what a
    gradient hook hands over at once. Same negotiation per name; returns one Handle each."""
    import ctypes
    basics.init()
    if len(tensor_list) != len(names):
        raise ValueError("one name per tensor")
    if not tensor_list:
        return []
    code = tensors.dtype_code(tensor_list[0])
    srcs, outs = [], []
    for t in tensor_list:
        if not tensors.is_device(t):
            raise ValueError("allreduce_async_many needs device tensors")
        if tensors.dtype_code(t) != code:
            raise ValueError("allreduce_async_many needs one dtype (call it once per dtype)")
        srcs.append(t.contiguous())
        outs.append(tensors.empty_like(srcs[-1]))
    n = len(srcs)
    nm = (ctypes.c_char_p * n)(*[x.encode() for x in names])
    pi, _k1 = _lib.ptr_array([x.data_ptr() for x in srcs])
    po, _k2 = _lib.ptr_array([x.data_ptr() for x in outs])
    shapes = [_shape(x) for x in srcs]
    nd = (ctypes.c_int * n)(*[len(s) for s in shapes])
    pd, _k3 = _lib.i64_array([d for s in shapes for d in s] or [0])
    hs = (ctypes.c_int64 * n)()
    _lib.call("tips_enqueue_allreduce_shaped_n", nm, pi, po, nd, pd, n, code, tensors.stream_of(srcs[0]), hs)
    out = []
    for h, o, x, name in zip(hs, outs, srcs, names):
        hd = Handle(int(h), o, name)
        hd._keep = x
        out.append(hd._track())
    return out


def synchronize_many(handles):
    """synchronize() over a list in one library call (tips_wait_n); returns the outputs."""
    import ctypes
    pend = [h for h in handles if not h.done]
    if pend:
        arr = (ctypes.c_int64 * len(pend))(*[h.handle for h in pend])
        try:
            _lib.call("tips_wait_n", arr, len(pend))
        except _lib.TipsError:
            for h in pend:  # every handle has been waited on (tips_wait_n waits for all of them)
                h._release()
            raise
        for h in pend:
            h._complete()
    return [h.output for h in handles]


def poll(handle):
    """True once the named allreduce has completed on the device."""
    if handle.done:
        return True
    try:
        rc = _lib.call("tips_poll", handle.handle)
    except _lib.TipsError:
        handle._release()
        raise
    if rc == 1:
        handle._complete()
    return handle.done


def synchronize(handle):
    """Wait for a Handle and return its output tensor (raises TipsError on a negotiation error)."""
    if not handle.done:
        try:
            _lib.call("tips_wait", handle.handle)
        except _lib.TipsError:
            handle._release()
            raise
        handle._complete()
    return handle.output


class registered_host_buffer(object):
    """Context manager: page-lock a long-lived host (numpy / CPU torch) buffer for the
    duration, so host-memory allreduces on it use asynchronous DMA (tips_host_register)."""

    def __init__(self, array):
        self.array = array

    def __enter__(self):
        basics.init()
        _lib.call("tips_host_register", tensors.data_ptr(self.array),
                  tensors.numel(self.array) * self.array.dtype.itemsize if not tensors.is_torch(self.array)
                  else self.array.numel() * self.array.element_size())
        return self.array

    def __exit__(self, *exc):
        _lib.call("tips_host_unregister", tensors.data_ptr(self.array))
        return False


def set_algorithm(algo):
    """Select 'auto', 'ring', 'direct', 'oneshot', 'peer' or 'rccl'; returns the previous selection's name."""
    names = {"auto": _lib.ALGO_AUTO, "ring": _lib.ALGO_RING, "direct": _lib.ALGO_DIRECT, "rccl": _lib.ALGO_RCCL,
             "oneshot": _lib.ALGO_ONESHOT, "peer": _lib.ALGO_PEER}
    inv = {v: k for k, v in names.items()}
    prev = _lib.lib().tips_get_algorithm()
    _lib.call("tips_set_algorithm", names[algo])
    return inv.get(prev, str(prev))
