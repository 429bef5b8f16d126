"""tips_amd — MI355X-native gradient-bucket reduction behind TiPS's allreduce API.

Drop-in surface of `tips.tensorflow` for the collective-allreduce path
(reference tips/tensorflow/__init__.py:20-103,189-227, ops.py, basics.py,
compression.py), over numpy arrays and torch tensors instead of TF tensors
(TensorFlow is not in this image). Everything below reaches the GPU through
libtips_hip.so (include/tips_hip.h); there is no CPU fallback.
"""
from .basics import TipsBasics, init, is_initialized, rank, shutdown, size
from .compression import Compression, Compressor, FP16Compressor, NoneCompressor
from .ops import (Handle, allgather_async, allgather_op, allreduce_async, broadcast_async, allreduce_async_many, synchronize_many, allreduce_op, broadcast_op, poll, synchronize, broadcast_variables, bucket_sum, fused_allreduce,
                  fused_allreduce_, rank_op, registered_host_buffer, set_algorithm, set_consistency_check, size_op)
from .ops import fused_allreduce_cast, fused_allreduce_flat, fused_allreduce_host, fused_allreduce_host_flat, fusion_stats
from ._lib import TipsError, TipsLibraryError
from . import ops as _ops
from . import tensors as _tensors

Average = 'Average'
Sum = 'Sum'


class IndexedSlices(object):
    """A sparse gradient: rows `values` of a dense tensor of `dense_shape`, at row `indices`
    (what tf.IndexedSlices carries, e.g. an embedding gradient). The represented tensor is the
    sum over repeated indices."""

    def __init__(self, values, indices, dense_shape=None):
        self.values = values
        self.indices = indices
        self.dense_shape = dense_shape

__all__ = [
    "allreduce", "IndexedSlices", "allreduce_async", "broadcast_async", "allgather_async", "allreduce_async_many", "synchronize_many", "poll", "synchronize", "Handle", "allreduce_grads", "allreduce_op", "allgather_op", "broadcast_op", "broadcast_variables",
    "set_consistency_check", "registered_host_buffer", "bucket_sum", "fused_allreduce", "fused_allreduce_", "init",
    "shutdown",
    "is_initialized", "size", "rank", "size_op", "rank_op", "set_algorithm", "Compression", "Compressor",
    "NoneCompressor", "FP16Compressor", "Average", "Sum", "TipsBasics", "TipsError", "TipsLibraryError",
    "DistributedOptimizer", "DistributedGradientTape", "fused_allreduce_cast", "fused_allreduce_flat", "fused_allreduce_host", "fused_allreduce_host_flat", "fusion_stats",
]


def allreduce(tensor,
              average=None,
              device_dense='',
              device_sparse='',
              compression=Compression.none,
              op=None,
              prescale_factor=1.0,
              postscale_factor=1.0,
              name=None):
    """Sum `tensor` over all ranks — mirrors tips.tensorflow.allreduce (__init__.py:20-91).

    Same arguments as the reference. As in the reference, `op`,
    `prescale_factor` and `postscale_factor` do not reach the reduction (they
    are commented out at the C++ boundary, __init__.py:82-87), so the result
    is the plain SUM for op=Average too — parity with the
    reference, not a recommendation. `average`, `device_dense` and
    `device_sparse` are accepted for signature compatibility.

    Sparse gradients take the reference's allgather branch (__init__.py:59-74).
    An `IndexedSlices` gets its values and indices allgathered, and they are
    divided by size() for op=Average, as the reference does there. A torch
    sparse COO tensor gets the same treatment on its nonzeros. The result
    represents the summed tensor.
    """
    if isinstance(tensor, IndexedSlices):
        values = allgather_op(tensor.values)
        indices = allgather_op(tensor.indices)
        new_values = (values / size()) if op == Average else values
        return IndexedSlices(new_values, indices, dense_shape=tensor.dense_shape)
    if _tensors.is_torch(tensor) and tensor.is_sparse:
        import torch
        idx = tensor._indices().t().contiguous()  # (nnz, ndim): rows concatenate along dim 0
        vals = tensor._values().contiguous()
        g_idx = allgather_op(idx).t()
        g_vals = allgather_op(vals)
        if op == Average:
            g_vals = g_vals / size()
        return torch.sparse_coo_tensor(g_idx, g_vals, tensor.shape)
    tensor_compressed, ctx = compression.compress(tensor)
    summed_tensor_compressed = allreduce_op(tensor_compressed, name=name)
    return compression.decompress(summed_tensor_compressed, ctx)


def _allreduce_cond(tensor, *args, **kwargs):
    """size() > 1 ? allreduce(tensor) : tensor  (__init__.py:94-103)."""
    if size() > 1:
        return allreduce(tensor, *args, **kwargs)
    return tensor


def _to_dense(g):
    """tf.convert_to_tensor of an IndexedSlices (rows summed over repeated indices), or a torch
    sparse tensor's dense form; anything else unchanged."""
    if isinstance(g, IndexedSlices):
        if g.dense_shape is None:
            raise ValueError("sparse_as_dense needs the IndexedSlices' dense_shape")
        if _tensors.is_torch(g.values):
            import torch
            dense = torch.zeros(tuple(int(d) for d in g.dense_shape), dtype=g.values.dtype, device=g.values.device)
            idx = g.indices if _tensors.is_torch(g.indices) else torch.as_tensor(g.indices)
            return dense.index_add_(0, idx.to(dense.device, torch.int64), g.values)
        import numpy as np
        dense = np.zeros(tuple(int(d) for d in g.dense_shape), dtype=np.asarray(g.values).dtype)
        np.add.at(dense, np.asarray(g.indices), np.asarray(g.values))
        return dense
    if _tensors.is_torch(g) and g.is_sparse:
        return g.to_dense()
    return g


def allreduce_grads(grads, compression=Compression.none, op=None, fused=True, sparse_as_dense=False):
    """Allreduce a list of gradients (None entries pass through).

    Mirrors the per-gradient loop of _make_cached_allreduce_grads_fn
    (__init__.py:203-222), including the size()==1 identity of
    _allreduce_cond and `sparse_as_dense` (__init__.py:205-210: sparse
    gradients are densified first and then take the dense path). With
    fused=True, device tensors are summed through the fusion buckets (one
    allreduce per <=64 MiB bucket instead of one per gradient); outputs are
    new tensors, inputs are left unchanged.
    """
    if sparse_as_dense:
        grads = [_to_dense(g) if g is not None else g for g in grads]
    if size() <= 1:
        return list(grads)
    return _reduce_grads(grads, compression, op, fused)


def _reduce_grads(grads, compression=Compression.none, op=None, fused=True):
    """What allreduce_grads runs at N > 1 (bench.py times it on one rank, where allreduce_grads
    itself is the identity). With fused=True:
      - dense device gradients, per dtype: fused_allreduce_flat - the outputs are views of one flat
        buffer laid out as the fusion buckets, each bucket packed into it and allreduced in place
        (a layout depends on the counts only, so fresh gradient tensors every step hit the caches);
      - dense host gradients (numpy / CPU torch: the reference's op is a CPU op, ops.cc:118), per
        dtype: fused_allreduce_host_flat - packed into page-locked pieces by host threads,
        pipelined H2D -> allreduce -> D2H straight into one page-locked flat host buffer, the
        outputs views of it (reused as the device flat outputs are);
      - the rest (sparse) one by one, through the reference's allgather branch."""
    none = compression is Compression.none
    global _DATA_PTR
    if _DATA_PTR is None:
        import torch
        _DATA_PTR = torch.Tensor.data_ptr
    if fused and grads and compression is FP16Compressor:  # (one list of dense f32 device tensors)
        res = _ops._dev_list_cast(grads)
        if res is not None:
            return res
    if fused and none and grads:
        res = _ops._dev_list_flat(grads)  # (one dtype of dense device tensors: the common case)
        if res is not None:
            return res
        plan = _find_plan(grads)
        if plan is not None:  # the same tensor objects as a recent call: no per-tensor inspection
            res = plan.run(grads)
            if res is not None:
                return res
            _PLANS.remove(plan)
    out = list(grads)
    dev, host, cast = {}, {}, {}
    simple = fused and none  # only dense, contiguous device tensors: the split can be remembered
    fp16 = fused and compression is FP16Compressor
    for i, g in enumerate(grads):
        if g is None:
            continue
        if not fused:
            out[i] = allreduce(g, compression=compression, op=op)
            continue
        kind = _kind(g)
        if kind is None:
            out[i] = allreduce(g, compression=compression, op=op)
            simple = False
            continue
        if fp16 and kind == "dev" and g.dtype == _torch().float32:
            # Compression.fp16 fused into the buckets: cast while packed, fp16 on the wire, cast back
            # while unpacked (tips_fused_allreduce_cast) - no per-tensor cast launches
            cast.setdefault(g.device, []).append((i, g if g.is_contiguous() else g.contiguous()))
            continue
        c, ctx = (g, None) if none else compression.compress(g)
        if kind == "dev":
            if not c.is_contiguous():
                c = c.contiguous()
                simple = False
            dev.setdefault((c.dtype, c.device), []).append((i, c, ctx))
        else:
            c = _tensors.contiguous(c)
            host.setdefault(str(c.dtype), []).append((i, c, ctx))
    plan_groups = []
    for members in dev.values():
        ts = [c for _, c, _ in members]
        fo = _ops._flat_outputs(ts, _tensors.dtype_code(ts[0]))
        sums = _ops._flat_run(fo, ts, list(map(_DATA_PTR, ts)))
        for (i, _, ctx), s in zip(members, sums):
            out[i] = s if none else compression.decompress(s, ctx)
        plan_groups.append(([i for i, _, _ in members], None, None))
    for members in cast.values():
        for (i, _), s in zip(members, _ops.fused_allreduce_cast([c for _, c in members], "float16")):
            out[i] = s
    for members in host.values():
        ts = [c for _, c, _ in members]
        sums = _ops.fused_allreduce_host_flat(ts)
        if simple:
            # a plan re-reads the pointers with the fast reader and re-checks shapes and dtypes:
            # only for lists of the inputs themselves (contiguous, not copies) that it reads right
            ok = all(c is grads[i] for i, c, _ in members) and \
                _tensors.host_data_ptrs(ts) == [_tensors.data_ptr(t) for t in ts]
            if ok:
                plan_groups.append(([i for i, _, _ in members], _ops._host_flat_outputs(ts),
                                    [(t.shape, t.dtype) for t in ts]))
            else:
                simple = False
        for (i, _, ctx), s in zip(members, sums):
            out[i] = s if none else compression.decompress(s, ctx)
    if simple:
        _remember_plan(grads, plan_groups)
    return out


_DATA_PTR = None  # torch.Tensor.data_ptr, bound on first use


def _torch():
    import torch
    return torch
_PLANS = []       # recent _GradPlans, most recent first


class _GradPlan(object):
    """How _reduce_grads split one list of dense gradients, kept for a later call with the SAME
    tensor objects (a training loop whose .grad tensors persist, or a set of gradient buffers used
    in turn): such a call is recognised through weak references and skips the per-tensor Python
    inspection (kind, dtype, contiguity, shape), which costs more host time for 1000 gradients than
    the fused allreduce's device work. A plan whose tensors one has died never matches again (a
    weak-reference callback marks it), and a position that was None must be None again: a dead
    gradient cannot pass for a None one. Tensors can still change in place (.data =, set_, resize_,
    a numpy array's shape), so every call re-reads each group through the checking readers: device
    groups through _ops._dev_list_flat (pointers, counts, dtype, contiguity in C++), host groups
    through their recorded shapes and dtypes; any difference plans again."""

    def __init__(self, grads, groups):
        import weakref
        self.dead = False

        def died(_ref, plan=weakref.ref(self)):
            p = plan()
            if p is not None:
                p.dead = True
        self.refs = [weakref.ref(g, died) if g is not None else _NONE_REF for g in grads]
        self.n = len(grads)
        # [(positions, None, None)] for device groups, [(positions, _HostFlatOutputs,
        # [(shape, dtype)])] for host groups
        self.groups = groups
        self.whole = len(groups) == 1 and groups[0][0] == list(range(self.n))

    def matches(self, grads):
        import operator
        import weakref
        if self.dead or len(grads) != self.n:
            return False
        # a live tensor's reference returns it; a None position's returns None (_NONE_REF)
        return all(map(operator.is_, map(weakref.ref.__call__, self.refs), grads))

    def run(self, grads):
        """The outputs, or None when a tensor changed in place (the caller plans again)."""
        out = list(grads)
        for pos, fo, meta in self.groups:
            ts = grads if self.whole else [grads[i] for i in pos]
            if meta is None:
                sums = _ops._dev_list_flat(ts)  # (None: not one dtype of dense contiguous device tensors now)
                if sums is None:
                    return None
            else:
                if any(t.shape != shp or t.dtype is not dt for t, (shp, dt) in zip(ts, meta)):
                    return None
                sums = _ops._host_flat_run(fo, _tensors.host_data_ptrs(ts))
            if self.whole:
                return sums
            for i, s in zip(pos, sums):
                out[i] = s
        return out


class _Gone(object):
    pass


def _dead():
    import weakref
    return weakref.ref(_Gone())  # (the object is gone at once: the reference reads None, as a None gradient)


_NONE_REF = _dead()  # the reference of a position that held None (only a plan's None positions use it)


def _find_plan(grads):
    for k, p in enumerate(_PLANS):
        if p.matches(grads):
            if k:
                _PLANS.insert(0, _PLANS.pop(k))
            return p
    return None


def _remember_plan(grads, groups):
    if not groups:
        return
    _PLANS.insert(0, _GradPlan(grads, groups))
    del _PLANS[8:]


def _kind(g):
    """'dev' for a dense device tensor, 'host' for a dense host tensor (numpy, CPU torch), None for
    anything reduced on its own (sparse)."""
    if _tensors.is_torch(g):
        if g.is_sparse:
            return None
        return "dev" if g.is_cuda else "host"
    if isinstance(g, IndexedSlices):
        return None
    return "host"


def _fusable(g):
    """Dense device tensors go through the fusion buckets; sparse and host ones are reduced one by one."""
    return g is not None and _tensors.is_device(g) and not g.is_sparse


from .optim import DistributedGradientTape, DistributedOptimizer  # noqa: E402  (uses allreduce_grads above)
