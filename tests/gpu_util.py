"""Helpers for the -m gpu parity tests: numpy <-> device buffers and C-ABI calls."""
import numpy as np

F32, F64, I32, I64, F16, BF16 = 0, 1, 2, 3, 4, 5
NPDT = {F32: np.float32, F64: np.float64, I32: np.int32, I64: np.int64, F16: np.float16, BF16: np.uint16}
ALL_DTYPES = [F32, F64, I32, I64, F16, BF16]


def rand(dtype, n, rng, kind="normal"):
    if dtype in (I32, I64):
        info = np.iinfo(NPDT[dtype])
        return rng.integers(info.min, info.max, size=n, dtype=NPDT[dtype], endpoint=True)
    if kind == "positive":
        x = 0.5 + rng.random(n)
    else:
        x = rng.standard_normal(n) * 3.0
    if dtype == BF16:
        import torch
        return torch.from_numpy(x.astype(np.float32)).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    return x.astype(NPDT[dtype])


def with_specials(a, dtype):
    a = a.copy()
    if dtype in (F32, F64, F16):
        sp = np.array([np.inf, -np.inf, np.nan, 0.0, -0.0], dtype=NPDT[dtype])
        a[:len(sp)] = sp[:len(a)]
        if len(a) > 8:
            tiny = np.array([1], dtype={F32: np.uint32, F64: np.uint64, F16: np.uint16}[dtype]).view(NPDT[dtype])[0]
            a[6] = tiny
            a[7] = np.finfo(NPDT[dtype]).max
    return a


def to_dev(a):
    import torch
    if a.dtype == np.uint16:
        return torch.from_numpy(a.view(np.int16).copy()).cuda()
    return torch.from_numpy(a.copy()).cuda()


def from_dev(t, dtype):
    return t.cpu().numpy().view(NPDT[dtype]).copy()


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[a.itemsize])


def same_bits(got, exp, dtype):
    """Bit-exact, except any NaN matches any NaN (payloads are not part of the contract)."""
    if dtype in (F32, F64, F16):
        gn, en = np.isnan(got), np.isnan(exp)
        if not np.array_equal(gn, en):
            return False
        return np.array_equal(bits(got)[~gn], bits(exp)[~en])
    if dtype == BF16:
        gf = (got.astype(np.uint32) << 16).view(np.float32)
        ef = (exp.astype(np.uint32) << 16).view(np.float32)
        gn, en = np.isnan(gf), np.isnan(ef)
        return np.array_equal(gn, en) and np.array_equal(got[~gn], exp[~en])
    return np.array_equal(got, exp)


def stream():
    import torch
    return torch.cuda.current_stream().cuda_stream


def simulate(kind, ins, dtype, inplace=False, transport=0):
    """p virtual ranks' plans on this one GPU through the development library's simulators
    (include/tips_hip_dev.h): the same plans, kernels and stream order as the RCCL executor."""
    import torch
    from tips_amd import _lib
    _lib.dev_call("tips_set_sim_transport", transport)
    devs = [to_dev(x) for x in ins]
    outs = devs if inplace else [torch.empty_like(d) for d in devs]
    pi, _k1 = _lib.ptr_array([d.data_ptr() for d in devs])
    po, _k2 = _lib.ptr_array([o.data_ptr() for o in outs])
    fn = {"ring": "tips_ring_simulate", "direct": "tips_direct_simulate", "oneshot": "tips_oneshot_simulate"}[kind]
    try:
        _lib.dev_call(fn, po, pi, len(ins), ins[0].size, dtype, stream())
        torch.cuda.synchronize()
    finally:
        _lib.dev_call("tips_set_sim_transport", 0)
    return [from_dev(o, dtype) for o in outs]
