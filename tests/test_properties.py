"""Property tests (hypothesis) on the CPU: the oracle's schedules and the C-ABI's partition.

* integer sums are order-independent (two's-complement add is associative), so the ring
  restatement and the rank-order fold must agree bit for bit for any p, n;
* fp32 ring vs fold differ only by reordering: |ring - fold| <= 2 (p-1) eps * sum_r |x_r|;
* the chunk / sub-chunk partition tiles [0, n) exactly, 256-B aligned, for every dtype;
* f16 sum2 equals numpy's correctly rounded half add on random bit patterns (finite results).
"""
import ctypes

import numpy as np
import pytest

hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402


@settings(max_examples=60, deadline=None)
@given(p=st.integers(1, 12), n=st.integers(0, 3000), seed=st.integers(0, 2**31 - 1),
       dt=st.sampled_from([np.int32, np.int64]))
def test_int_ring_equals_fold(oracle, p, n, seed, dt):
    rng = np.random.default_rng(seed)
    info = np.iinfo(dt)
    ins = [rng.integers(info.min, info.max, size=n, dtype=dt, endpoint=True) for _ in range(p)]
    ring = oracle.ring(ins, align_elems=int(rng.integers(1, 70)))
    fold = oracle.fold(ins)
    for r in ring:
        assert np.array_equal(r, fold)


@settings(max_examples=40, deadline=None)
@given(p=st.integers(2, 12), n=st.integers(1, 2000), seed=st.integers(0, 2**31 - 1))
def test_f32_ring_vs_fold_reorder_bound(oracle, p, n, seed):
    rng = np.random.default_rng(seed)
    ins = [(rng.standard_normal(n) * 10).astype(np.float32) for _ in range(p)]
    ring = oracle.ring(ins)[0].astype(np.float64)
    fold = oracle.fold(ins).astype(np.float64)
    bound = 2 * (p - 1) * np.finfo(np.float32).eps * np.sum(np.abs(np.stack(ins).astype(np.float64)), axis=0)
    assert np.all(np.abs(ring - fold) <= bound + 1e-30)


@settings(max_examples=80, deadline=None)
@given(n=st.integers(0, 10**9), p=st.integers(1, 64), dtype=st.sampled_from([0, 1, 2, 3, 4, 5]))
def test_abi_chunk_partition(n, p, dtype):
    from tips_amd import _lib
    L = _lib.lib()
    es = {0: 4, 1: 8, 2: 4, 3: 8, 4: 2, 5: 2}[dtype]
    b, e = ctypes.c_int64(), ctypes.c_int64()
    prev = 0
    for c in range(p):
        assert L.tips_chunk_bounds(n, p, dtype, c, ctypes.byref(b), ctypes.byref(e)) == 0
        assert b.value == prev and e.value >= b.value
        if e.value < n:
            assert (e.value * es) % 256 == 0
        prev = e.value
    assert prev == n
    d, sub = ctypes.c_int(), ctypes.c_int64()
    assert L.tips_schedule_shape(n, p, dtype, ctypes.byref(d), ctypes.byref(sub)) == 0
    assert 1 <= d.value <= 4 and 0 <= sub.value


@settings(max_examples=30, deadline=None)
@given(seed=st.integers(0, 2**31 - 1))
def test_f16_sum2_bit_patterns(oracle, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 65536, size=4096, dtype=np.uint32).astype(np.uint16).view(np.float16)
    b = rng.integers(0, 65536, size=4096, dtype=np.uint32).astype(np.uint16).view(np.float16)
    got = oracle.sum2(a, b)
    with np.errstate(all="ignore"):
        ref = (a.astype(np.float64) + b.astype(np.float64)).astype(np.float16)
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(got), nan)
    assert np.array_equal(got[~nan].view(np.uint16), ref[~nan].view(np.uint16))
