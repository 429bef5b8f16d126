"""The tips_amd Python surface on CPU: it mirrors tips.tensorflow's names and
signatures, maps dtypes like the reference (plus f16/bf16), and fails loudly
when the HIP library is missing (no CPU fallback)."""
import inspect
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO


def test_reference_names_exist():
    import tips_amd
    # tips/tensorflow/__init__.py:8,17-18 and ops.py/basics.py names used on the allreduce path
    for name in ("allreduce", "allreduce_op", "size", "rank", "shutdown", "size_op", "rank_op", "Compression",
                 "Average", "Sum", "TipsBasics"):
        assert hasattr(tips_amd, name), name
    assert tips_amd.Average == 'Average' and tips_amd.Sum == 'Sum'


def test_allreduce_signature_matches_reference():
    import tips_amd
    params = list(inspect.signature(tips_amd.allreduce).parameters)
    # tips/tensorflow/__init__.py:20-28
    assert params == ["tensor", "average", "device_dense", "device_sparse", "compression", "op", "prescale_factor",
                      "postscale_factor", "name"]
    assert list(inspect.signature(tips_amd.allreduce_op).parameters) == ["tensor", "name"]  # ops.py:61


def test_dtype_codes():
    import torch
    from tips_amd import tensors
    assert tensors.dtype_code(np.zeros(1, np.float32)) == 0
    assert tensors.dtype_code(np.zeros(1, np.float64)) == 1
    assert tensors.dtype_code(np.zeros(1, np.int32)) == 2
    assert tensors.dtype_code(np.zeros(1, np.int64)) == 3
    assert tensors.dtype_code(np.zeros(1, np.float16)) == 4
    assert tensors.dtype_code(torch.zeros(1, dtype=torch.bfloat16)) == 5
    assert tensors.dtype_code(torch.zeros(1, dtype=torch.float32)) == 0
    for bad in (np.zeros(1, np.uint8), torch.zeros(1, dtype=torch.bool), np.zeros(1, np.complex64)):
        with pytest.raises(TypeError, match="Not supported dtype found"):
            tensors.dtype_code(bad)


def test_compression_round_trip():
    import torch
    from tips_amd import Compression
    x = np.linspace(-3, 3, 17).astype(np.float32)
    c, ctx = Compression.fp16.compress(x)
    assert c.dtype == np.float16
    assert Compression.fp16.decompress(c, ctx).dtype == np.float32
    t = torch.linspace(-3, 3, 17)
    c, ctx = Compression.fp16.compress(t)
    assert c.dtype == torch.float16 and Compression.fp16.decompress(c, ctx).dtype == torch.float32
    i = np.arange(5, dtype=np.int32)
    c, ctx = Compression.fp16.compress(i)
    assert c is i  # integers are not compressed (compression.py:55-57)
    assert Compression.none.compress(x) == (x, None)


def test_missing_library_fails_loudly():
    code = ("import tips_amd, numpy as np\n"
            "try:\n"
            "    tips_amd.allreduce(np.ones(3, np.float32))\n"
            "except tips_amd.TipsLibraryError as e:\n"
            "    print('LOUD', e)\n")
    env = dict(os.environ, TIPS_HIP_LIB="/nonexistent/libtips_hip.so")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=REPO, env=env, timeout=300)
    assert "LOUD" in r.stdout and "no CPU fallback" in r.stdout, r.stdout + r.stderr


def test_allreduce_without_gpu_raises_not_computes():
    """On a host with no HIP device the op must raise (init fails), never return a host-computed sum."""
    code = ("import tips_amd, numpy as np\n"
            "try:\n"
            "    out = tips_amd.allreduce(np.ones(3, np.float32))\n"
            "    print('COMPUTED', out)\n"
            "except tips_amd.TipsError as e:\n"
            "    print('RAISED', e.code)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=REPO, timeout=300)
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    assert "RAISED" in r.stdout, r.stdout + r.stderr


def _fake_two_ranks(monkeypatch):
    """allgather over two ranks that hold the same tensor, without a GPU: the host logic of the sparse
    branch (__init__.py:59-74 of the reference) is what is under test here."""
    import torch
    import tips_amd

    def gather(t, name=None):
        return torch.cat([t, t]) if isinstance(t, torch.Tensor) else np.concatenate([t, t])

    monkeypatch.setattr(tips_amd, "allgather_op", gather)
    monkeypatch.setattr(tips_amd, "size", lambda: 2)
    # dense host gradients go through the fused host path at N > 1: here each through the (faked)
    # tips_amd.allreduce, so the tests below see one reduction per gradient
    monkeypatch.setattr(tips_amd._ops, "fused_allreduce_host_flat", lambda ts: [tips_amd.allreduce(t) for t in ts])
    # (a remembered plan calls the library directly: none here, so every call takes the fake)
    monkeypatch.setattr(tips_amd, "_remember_plan", lambda grads, groups: None)


def test_indexed_slices_take_the_allgather_branch(monkeypatch):
    import tips_amd
    _fake_two_ranks(monkeypatch)
    vals = np.arange(6, dtype=np.float32).reshape(3, 2)
    idx = np.array([4, 0, 4], dtype=np.int64)
    s = tips_amd.allreduce(tips_amd.IndexedSlices(vals, idx, dense_shape=(5, 2)))
    assert isinstance(s, tips_amd.IndexedSlices) and s.dense_shape == (5, 2)
    assert np.array_equal(s.values, np.concatenate([vals, vals])) and np.array_equal(s.indices, np.tile(idx, 2))
    a = tips_amd.allreduce(tips_amd.IndexedSlices(vals, idx, dense_shape=(5, 2)), op=tips_amd.Average)
    assert np.array_equal(a.values, np.concatenate([vals, vals]) / 2)  # the reference divides here


def test_torch_sparse_allreduce_represents_the_sum(monkeypatch):
    import torch
    import tips_amd
    _fake_two_ranks(monkeypatch)
    dense = torch.zeros(6, 3)
    dense[1, 2] = 1.5
    dense[4, 0] = -2.0
    sp = dense.to_sparse()
    out = tips_amd.allreduce(sp)
    assert out.is_sparse and out.shape == dense.shape
    assert torch.equal(out.to_dense(), 2 * dense)
    assert torch.equal(tips_amd.allreduce(sp, op=tips_amd.Average).to_dense(), dense)


def test_allreduce_grads_routes_sparse_to_allgather(monkeypatch):
    import torch
    import tips_amd
    _fake_two_ranks(monkeypatch)
    dense = torch.zeros(4, 2)
    dense[2, 1] = 3.0
    sl = tips_amd.IndexedSlices(np.ones((1, 2), np.float32), np.array([3]), dense_shape=(4, 2))
    out = tips_amd.allreduce_grads([None, dense.to_sparse(), sl])
    assert out[0] is None
    assert torch.equal(out[1].to_dense(), 2 * dense)
    assert np.array_equal(out[2].indices, [3, 3])


def test_allreduce_grads_sparse_as_dense(monkeypatch):
    """sparse_as_dense (reference __init__.py:205-210): IndexedSlices (numpy or torch) and torch sparse
    gradients are densified (repeated rows summed) and then take the dense allreduce."""
    import torch
    import tips_amd
    _fake_two_ranks(monkeypatch)
    monkeypatch.setattr(tips_amd, "allreduce", lambda t, **kw: t * 2)
    sl = tips_amd.IndexedSlices(np.ones((3, 2), np.float32), np.array([1, 3, 1]), dense_shape=(4, 2))
    tsl = tips_amd.IndexedSlices(torch.ones(2, 2), torch.tensor([0, 0]), dense_shape=(3, 2))
    dense = torch.zeros(4, 2)
    dense[2, 1] = 3.0
    out = tips_amd.allreduce_grads([sl, tsl, dense.to_sparse(), None], sparse_as_dense=True, fused=False)
    exp0 = np.zeros((4, 2), np.float32)
    exp0[1] = 2.0
    exp0[3] = 1.0
    assert isinstance(out[0], np.ndarray) and np.array_equal(out[0], 2 * exp0)
    assert torch.equal(out[1], 2 * torch.tensor([[2.0, 2.0], [0.0, 0.0], [0.0, 0.0]]))
    assert not out[2].is_sparse and torch.equal(out[2], 2 * dense)
    assert out[3] is None


def _toy_model():
    import torch
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.Tanh(), torch.nn.Linear(3, 2))


def test_distributed_optimizer_sums_gradients_before_step(monkeypatch):
    """DistributedOptimizer (reference __init__.py:252-456) over torch.optim: step() allreduces every
    .grad first; as in the reference the reduction is a SUM even for op=Average (two fake ranks
    holding the same gradient: the update is twice the local one)."""
    import torch
    import tips_amd
    _fake_two_ranks(monkeypatch)
    monkeypatch.setattr(tips_amd, "allreduce", lambda t, **kw: t * 2)
    ref, dist_m = _toy_model(), _toy_model()
    x = torch.randn(5, 4)
    for m in (ref, dist_m):
        m(x).pow(2).sum().backward()
    lr = 0.1
    opt = tips_amd.DistributedOptimizer(torch.optim.SGD(dist_m.parameters(), lr=lr))
    with torch.no_grad():
        exp = [p - lr * 2 * p.grad for p in ref.parameters()]
    opt.step()
    for p, e in zip(dist_m.parameters(), exp):
        assert torch.allclose(p, e, atol=1e-7)


def test_distributed_optimizer_backward_passes_and_validation(monkeypatch):
    import torch
    import tips_amd
    _fake_two_ranks(monkeypatch)
    calls = []
    monkeypatch.setattr(tips_amd, "allreduce", lambda t, **kw: calls.append(1) or t)
    m = _toy_model()
    x = torch.randn(5, 4)
    opt = tips_amd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1), backward_passes_per_step=2,
                                        average_aggregated_gradients=True)
    before = [p.detach().clone() for p in m.parameters()]
    m(x).sum().backward()
    g1 = [p.grad.clone() for p in m.parameters()]
    opt.step()  # first pass: accumulate only
    assert not calls and all(torch.equal(p, b) for p, b in zip(m.parameters(), before))
    m(x).sum().backward()  # .grad now holds both passes
    opt.step()
    assert len(calls) == len(before)
    for p, b, g in zip(m.parameters(), before, g1):  # averaged over the 2 passes: (g + g) / 2 = g
        assert torch.allclose(p, b - 0.1 * g, atol=1e-6)
    with pytest.raises(ValueError, match="gradient_predivide_factor not supported"):
        tips_amd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1), op="Sum", gradient_predivide_factor=2.0)
    with pytest.raises(ValueError, match="groups should be a non-negative integer"):
        tips_amd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1), groups=-1)
    with pytest.raises(ValueError, match="doesn't inherit"):
        tips_amd.DistributedOptimizer(object())


def test_distributed_optimizer_synchronize_then_step(monkeypatch):
    """step() skips its own reduction only after a synchronize() of this very pass with no backward
    after it (the clip-gradients pattern). A synchronize() followed by another backward without a
    step (evaluation), or one in an earlier accumulation pass, does not excuse step(): it reduces
    again, with a warning; a second synchronize() without a backward in between warns too."""
    import warnings
    import torch
    import tips_amd
    _fake_two_ranks(monkeypatch)
    calls = []
    monkeypatch.setattr(tips_amd, "allreduce", lambda t, **kw: calls.append(1) or t)
    m = _toy_model()
    x = torch.randn(5, 4)
    n = len(list(m.parameters()))
    opt = tips_amd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.0))
    m(x).sum().backward()
    opt.synchronize()
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        opt.step()  # the clip pattern: reduced once, in synchronize()
    assert len(calls) == n
    opt.zero_grad()
    m(x).sum().backward()
    opt.synchronize()  # e.g. an evaluation that never steps
    opt.zero_grad()
    m(x).sum().backward()
    with pytest.warns(UserWarning, match="before a later backward"):
        opt.step()
    assert len(calls) == 3 * n
    opt.synchronize()
    with pytest.warns(UserWarning, match="called again with no backward"):
        opt.synchronize()
    assert len(calls) == 5 * n
    calls.clear()
    acc = tips_amd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.0), backward_passes_per_step=2)
    opt.zero_grad()
    m(x).sum().backward()
    acc.synchronize()  # in the first (accumulation) pass
    acc.step()
    m(x).sum().backward()
    with pytest.warns(UserWarning, match="earlier accumulation pass"):
        acc.step()
    assert len(calls) == 2 * n


def test_distributed_gradient_tape(monkeypatch):
    """DistributedGradientTape (reference __init__.py:460-569): gradient() differentiates, then sums
    the gradients over the ranks (a SUM for op=Average too); an unused source stays None; a single
    source gives a single gradient; a wrapped tape object supplies the gradients; the reference's
    argument validation."""
    import torch
    import tips_amd
    _fake_two_ranks(monkeypatch)
    monkeypatch.setattr(tips_amd, "allreduce", lambda t, **kw: t * 2)
    w = torch.randn(3, requires_grad=True)
    unused = torch.randn(2, requires_grad=True)
    x = torch.randn(3)
    tape = tips_amd.DistributedGradientTape()
    gw, gu = tape.gradient((w * x).sum(), [w, unused])
    assert torch.equal(gw, 2 * x) and gu is None
    assert torch.equal(tape.gradient((w * w).sum(), w), 4 * w.detach())

    class Tape(object):
        def gradient(self, target, sources, output_gradients=None):
            return [torch.ones_like(s) for s in sources]
    assert torch.equal(tips_amd.DistributedGradientTape(Tape()).gradient(None, [w])[0], 2 * torch.ones(3))
    with pytest.raises(ValueError, match="gradient_predivide_factor not supported"):
        tips_amd.DistributedGradientTape(op="Sum", gradient_predivide_factor=2.0)
    with pytest.raises(ValueError, match="groups should be a non-negative integer"):
        tips_amd.DistributedGradientTape(groups=0)
    with pytest.warns(DeprecationWarning):
        tips_amd.DistributedGradientTape(num_groups=2)
    with pytest.raises(ValueError, match="gradient"):
        tips_amd.DistributedGradientTape(object())


def test_fast_list_helper_reads_pointers_counts_and_shapes():
    """tips_amd._fast (the list helper allreduce_grads' device path uses) on CPU tensors: data
    pointers and counts as torch reports them, one hash per shape list, None for a list it must not
    take (another dtype, a strided view, a non-tensor), and max_refcount as sys.getrefcount - 1."""
    import ctypes
    import sys
    import torch
    from tips_amd import _fast
    flat = torch.zeros(4096)
    ts = [flat[0:10].view(2, 5), flat[64:64 + 7], flat[128:128 + 300].view(3, 10, 10), torch.zeros(0)]
    n = len(ts)
    pa, na = (ctypes.c_int64 * n)(), (ctypes.c_int64 * n)()
    a, b = ctypes.addressof(pa), ctypes.addressof(na)
    st, dev, h = _fast.dev_list(ts, a, b, 0)
    assert st == 6 and dev == -1  # c10::ScalarType::Float, CPU
    assert list(pa) == [t.data_ptr() for t in ts] and list(na) == [t.numel() for t in ts]
    # the hash follows the shapes, not only the counts
    ts2 = [flat[0:10].view(5, 2)] + ts[1:]
    assert _fast.dev_list(ts2, a, b, 0)[2] != h
    assert _fast.dev_list(list(ts), a, b, 0)[2] == h
    # lists it leaves to the general path
    assert _fast.dev_list(ts, a, b, 1) is None                       # not device tensors
    assert _fast.dev_list(ts[:2] + [torch.zeros(3, dtype=torch.float64)], a, b, 0) is None
    assert _fast.dev_list([flat[::2]], a, b, 0) is None              # not contiguous
    assert _fast.dev_list([flat[:4], None], a, b, 0) is None
    assert _fast.dev_list([torch.zeros(3).to_sparse()], a, b, 0) is None
    assert _fast.dev_list([torch.empty(3, device="meta")], a, b, 0) is None  # neither CPU nor device
    # cap: the arrays hold n entries; a sequence of any other length is refused before any write
    pa[0] = na[0] = -7
    assert _fast.dev_list(ts + [flat[:1]], a, b, 0, n) is None
    assert pa[0] == -7 and na[0] == -7
    assert _fast.dev_list(ts, a, b, 0, n)[2] == h
    x = torch.zeros(3)
    assert _fast.max_refcount([x]) == sys.getrefcount(x) - 1
    keep = [x, x]
    assert _fast.max_refcount([x]) == sys.getrefcount(x) - 1 and len(keep) == 2
    assert _fast.max_refcount([]) == 0


def test_flat_output_sets_are_not_handed_out_twice():
    """_FlatOutputs.take (allreduce_grads' output sets) returns the views in a new list, made before
    the library call releases the GIL: while one call's outputs are referenced, a second take()
    gets another set; once they are dropped, the first set comes back. (CPU tensors stand in for
    device ones; tips_fused_layout is host-only.)"""
    import gc
    import torch
    from tips_amd import _lib
    from tips_amd.ops import _FlatOutputs
    shapes = (torch.Size([3, 5]), torch.Size([7]), torch.Size([2, 2, 2]))
    fo = _FlatOutputs(shapes, [15, 7, 8], _lib.FLOAT32, torch.float32, torch.device("cpu"))
    f1, v1 = fo.take()
    assert [v.shape for v in v1] == list(shapes)
    f2, v2 = fo.take()
    assert f2.data_ptr() != f1.data_ptr()  # set 1's views are still held
    p1 = f1.data_ptr()
    del v1, f1
    gc.collect()
    f3, v3 = fo.take()
    assert f3.data_ptr() == p1 and v3[0].data_ptr() == p1
    held = v3[1]
    del v3, f3
    f4, v4 = fo.take()
    assert f4.data_ptr() != p1  # one view of set 1 is still held by the caller
    del held


def test_host_output_pool_reuses_only_released_outputs(monkeypatch):
    """allreduce_op's host outputs of >= 1 MiB come from _HostOutPool: a released output is handed
    out again (page-locked once, no fresh pages per call); one still referenced - directly, through
    a numpy view, or through torch's .numpy() on its storage - is not; small outputs are fresh.
    (tips_host_register is stubbed: no GPU here.)"""
    import numpy as np
    import torch
    import tips_amd.ops as ops

    class Stub:
        def tips_host_register(self, p, n):
            return 0
    monkeypatch.setattr(ops._lib, "lib", lambda: Stub())
    pool = ops._HostOutPool()
    src = np.zeros(1 << 19, dtype=np.float32)  # 2 MiB
    a = pool.take(src)
    b = pool.take(src)
    assert a is not b and a.shape == src.shape and a.dtype == src.dtype
    pa = a.ctypes.data
    del a
    c = pool.take(src)
    assert c.ctypes.data == pa
    view = c[::2]
    del c
    assert pool.take(src).ctypes.data != pa and view.size == 1 << 18
    small = np.zeros(100, dtype=np.float32)
    pool.take(small)
    assert (False, "float32", (100,)) not in pool.sets  # (under 1 MiB: a fresh output, not pooled)
    t = torch.zeros(1 << 19)
    x = pool.take(t)
    px = x.data_ptr()
    del x
    y = pool.take(t)
    assert y.data_ptr() == px
    arr = y.numpy()
    del y
    assert pool.take(t).data_ptr() != px and arr.size == 1 << 19


def test_fused_list_refuses_host_tensors():
    """FusedList.allreduce_ reads pointers, counts and dtype in C++ (_fast.dev_list) and falls back
    to the Python checks, with their error text, for a list it does not take: host tensors here."""
    import torch
    from tips_amd.ops import FusedList
    fl = FusedList([3, 4])
    with pytest.raises(ValueError, match="needs device tensors"):
        fl.allreduce_([torch.zeros(3), torch.zeros(4)])
    assert fl.allreduce_([]) == []


def test_evicted_host_flat_sets_unregister_after_last_use(monkeypatch):
    """_HOST_FLAT keeps 16 host list signatures; a set evicted from it stays page-locked only while
    an output of it is alive, and is unregistered once the last one goes (numpy views and
    torch.from_numpy storages both hold the page-locked array). Cycles through 20 signatures.
    (tips_host_register / _unregister are stubbed: no GPU here.)"""
    import gc
    import torch
    import tips_amd.ops as ops

    live = {}

    class Stub:
        def tips_host_register(self, p, n):
            assert p not in live, "address registered twice"
            live[p] = n
            return 0

        def tips_host_unregister(self, p):
            assert p in live
            del live[p]
            return 0

        def tips_fused_layout(self, cp, n, code, offs):
            return ops._lib.lib().tips_fused_layout(cp, n, code, offs)
    real = ops._lib.lib
    monkeypatch.setattr(ops._lib, "lib", lambda: Stub())
    monkeypatch.setattr(ops._lib, "call", lambda name, *a: getattr(Stub(), name)(*a))
    monkeypatch.setattr(Stub, "tips_fused_layout", lambda self, *a: real().tips_fused_layout(*a))
    monkeypatch.setattr(ops, "_HOST_FLAT", {})
    held = []
    for k in range(20):
        srcs = [np.zeros(k + 3, np.float32), np.zeros(7, np.float32)] if k % 2 else \
            [torch.zeros(k + 3), torch.zeros(5)]
        fo = ops._host_flat_outputs(srcs)
        flat, views = fo.take()
        if k == 0:
            held.append(views[1])  # an output of the first (torch) set outlives its eviction
        del flat, views
    gc.collect()
    assert len(ops._HOST_FLAT) == 16
    kept = {tensors_ptr(s[0]) for fo in ops._HOST_FLAT.values() for s in fo.sets}
    # every registration still live belongs to a kept set, or to the output still held
    assert set(live) - kept == {held[0].untyped_storage().data_ptr()}
    del held[:]
    gc.collect()
    assert set(live) == kept


def tensors_ptr(x):
    from tips_amd import tensors
    return tensors.data_ptr(x)


def test_grad_plan_never_matches_a_dead_gradient_or_a_changed_tensor(monkeypatch):
    """_GradPlan (allreduce_grads' remembered split): a gradient that died does not pass for a
    None in the same position, and a None position must stay None; a plan's run() re-checks its
    device groups through the checking reader (here: _dev_list_flat refuses the changed list)."""
    import gc
    import torch
    import tips_amd
    a, b = torch.zeros(3), torch.zeros(4)
    plan = tips_amd._GradPlan([a, None, b], [([0, 2], None, None)])
    assert plan.matches([a, None, b])
    assert not plan.matches([a, b, b]) and not plan.matches([a, None])
    del a
    gc.collect()
    assert plan.dead and not plan.matches([None, None, b])
    c = torch.zeros(2)
    plan2 = tips_amd._GradPlan([c], [([0], None, None)])
    calls = []
    monkeypatch.setattr(tips_amd._ops, "_dev_list_flat", lambda ts: calls.append(ts) or None)
    assert plan2.run([c]) is None and calls == [[c]]


def test_flat_output_keys_follow_the_layout_settings(monkeypatch):
    """A fusion layout depends on TIPS_FUSION_THRESHOLD / TIPS_COPY_TILE_BYTES / TIPS_FUSION_BALANCE
    as well as the counts: the cached flat-output sets are keyed on them, so a changed setting gets
    offsets of its own layout."""
    import torch
    import tips_amd.ops as ops
    monkeypatch.setattr(ops, "_FLAT_OUTPUTS", {})
    ts = [torch.zeros(300 << 10), torch.zeros(300 << 10)]  # 1.2 MiB each
    fo1 = ops._flat_outputs(ts, ops._lib.FLOAT32)
    monkeypatch.setenv("TIPS_FUSION_THRESHOLD", str(1 << 20))
    fo2 = ops._flat_outputs(ts, ops._lib.FLOAT32)
    assert fo2 is not fo1
    monkeypatch.delenv("TIPS_FUSION_THRESHOLD")
    assert ops._flat_outputs(ts, ops._lib.FLOAT32) is fo1


def test_flat_output_take_is_exclusive_across_threads():
    """_FlatOutputs.take from many threads at once: no set is handed to two holders at a time (the
    free check and the hand-out run under the object's lock)."""
    import threading
    import torch
    from tips_amd import _lib
    from tips_amd.ops import _FlatOutputs
    fo = _FlatOutputs((torch.Size([8]), torch.Size([3])), [8, 3], _lib.FLOAT32, torch.float32, torch.device("cpu"))
    owners = {}
    bad = []
    lock = threading.Lock()

    def worker(k):
        for _ in range(300):
            flat, views = fo.take()
            p = flat.data_ptr()
            with lock:
                if owners.get(p) is not None:
                    bad.append((p, owners[p], k))
                owners[p] = k
            with lock:
                owners[p] = None
            del flat, views
    th = [threading.Thread(target=worker, args=(k,)) for k in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not bad


@pytest.mark.parametrize("warm", ["0", "1", "2"])
def test_overlap_trial_with_any_warmup(monkeypatch, warm):
    """TIPS_OVERLAP_TRIAL_WARMUP=0 made the last trial step read the end event of a step
    that was never recorded (KeyError inside step() on every rank). The warm-up is clamped to 1;
    the trial then runs to its choice. Events are faked on the CPU: 'during' steps take 5 ms,
    'after' steps 7 ms, so the choice is 'during'."""
    import torch
    import tips_amd.ops
    from tips_amd import basics
    from tips_amd.optim import _OverlapChoice
    monkeypatch.setenv("TIPS_OVERLAP_TRIAL_WARMUP", warm)
    monkeypatch.setenv("TIPS_OVERLAP_TRIAL_STEPS", "2")
    clock = [0.0]

    class Ev(object):
        def record(self, *a):
            self.t = clock[0]

        def synchronize(self):
            pass

        def elapsed_time(self, other):
            return other.t - self.t

    monkeypatch.setattr(torch.cuda, "Event", lambda enable_timing=True: Ev())
    monkeypatch.setattr(tips_amd.ops, "_allgather_i64", lambda v: list(v))
    monkeypatch.setattr(basics, "size", lambda: 1)
    oc = _OverlapChoice("auto")
    assert oc.warm >= 1
    s = 0
    while oc.chosen is None:
        clock[0] += 5.0 if oc.on(s) else 7.0
        oc.stepped(s)
        s += 1
        assert s < 20
    assert oc.chosen is True and oc.report["chosen"] == "during"
    assert s == oc.warm + 4
