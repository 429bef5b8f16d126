"""-m gpu: the gfx950 bucket-sum kernels against the oracle, through the C-ABI.

Bar (BASELINE.json north_star): bit-exact for integers; floats here are
bit-exact too, because one IEEE add per element is order-free (f16 =
correctly rounded half add, bf16 = fp32 add rounded to nearest-even).
"""
import numpy as np
import pytest

from gpu_util import (ALL_DTYPES, BF16, F16, F32, F64, I32, I64, NPDT, from_dev, rand, same_bits, stream, to_dev,
                      with_specials)

pytestmark = pytest.mark.gpu

SIZES = [1, 7, 8, 9, 63, 4099, 65539, 1 << 20]


@pytest.mark.parametrize("dtype", ALL_DTYPES)
@pytest.mark.parametrize("n", SIZES)
def test_bucket_sum_matches_oracle(gpu, oracle, dtype, n):
    import torch
    from tips_amd import _lib
    rng = np.random.default_rng(100 + n + dtype)
    a, b = with_specials(rand(dtype, n, rng), dtype), rand(dtype, n, rng)
    da, db = to_dev(a), to_dev(b)
    dc = torch.empty_like(da)
    _lib.call("tips_bucket_sum", dc.data_ptr(), da.data_ptr(), db.data_ptr(), n, dtype, stream())
    torch.cuda.synchronize()
    assert same_bits(from_dev(dc, dtype), oracle.sum2(a, b, code=dtype), dtype)


@pytest.mark.parametrize("dtype", ALL_DTYPES)
def test_bucket_sum_inplace_and_unaligned(gpu, oracle, dtype):
    import torch
    from tips_amd import _lib
    rng = np.random.default_rng(7)
    n = 100003
    a, b = rand(dtype, n, rng), rand(dtype, n, rng)
    da, db = to_dev(a), to_dev(b)
    _lib.call("tips_bucket_sum", da.data_ptr(), da.data_ptr(), db.data_ptr(), n, dtype, stream())  # a += b
    torch.cuda.synchronize()
    assert same_bits(from_dev(da, dtype), oracle.sum2(a, b, code=dtype), dtype)
    # views offset by one element: not 16-B aligned -> scalar path
    da, db = to_dev(a), to_dev(b)
    dc = torch.empty_like(da)
    _lib.call("tips_bucket_sum", dc[1:].data_ptr(), da[1:].data_ptr(), db[1:].data_ptr(), n - 1, dtype, stream())
    torch.cuda.synchronize()
    assert same_bits(from_dev(dc, dtype)[1:], oracle.sum2(a[1:], b[1:], code=dtype), dtype)


def test_int_wrap_on_device(gpu, oracle):
    import torch
    from tips_amd import _lib
    a = np.array([2**31 - 1] * 37, dtype=np.int32)
    b = np.array([1] * 37, dtype=np.int32)
    da, db = to_dev(a), to_dev(b)
    _lib.call("tips_bucket_sum", da.data_ptr(), da.data_ptr(), db.data_ptr(), 37, I32, stream())
    torch.cuda.synchronize()
    assert (from_dev(da, I32) == -2**31).all()


SWEEP_VARIANTS = ([(m, u, t, 256) for m in (0, 1) for u in (1, 2, 4, 8) for t in (0, 1)]
                  + [(1, 2, 2, 256), (1, 4, 2, 256), (1, 2, 3, 256), (1, 4, 3, 256), (1, 2, 1, 512), (1, 4, 1, 512),
                     (1, 8, 1, 512), (1, 1, 1, 1024), (1, 2, 1, 1024), (1, 4, 1, 1024), (1, 4, 2, 512),
                     (1, 4, 3, 512), (1, 16, 1, 256), (1, 16, 1, 128), (1, 8, 1, 128), (1, 4, 1, 128), (1, 8, 1, 64),
                     (1, 1, 2, 256), (1, 8, 2, 256), (1, 2, 2, 512), (1, 2, 2, 128), (1, 1, 2, 512), (0, 2, 2, 256),
                     (0, 4, 2, 256), (2, 1, 2, 256), (2, 2, 2, 256), (2, 1, 2, 512), (2, 4, 1, 256)]
                  + [(3, 1, i, 256) for i in range(14)]
                  + [(3, u, 1, t) for u, t in ((2, 256), (4, 256), (1, 512), (2, 128), (1, 1024), (1, 128), (2, 512))]
                  + [(3, 1, 7, 128), (3, 1, 7, 64), (3, 2, 7, 128)]  # the product default since round 6 (128 lanes, nt stores) and its neighbours
                  + [(4, u, 0, 256) for u in (1, 2, 4)]
                  + [(5, w, 0, 256) for w in (1, 2, 4, 8)]
                  + [(3, u, 7, t) for u, t in ((1, 512), (1, 1024), (2, 256), (4, 256), (2, 512))])


@pytest.mark.parametrize("mode,unroll,nt,threads", SWEEP_VARIANTS)
def test_every_sum_variant_is_exact(gpu, oracle, mode, unroll, nt, threads):
    import torch
    from tips_amd import _lib
    rng = np.random.default_rng(11)
    n = (1 << 20) + 5
    a, b = rand(F32, n, rng), rand(F32, n, rng)
    da, db = to_dev(a), to_dev(b)
    dc = torch.empty_like(da)
    _lib.dev_call("tips_sum_variant", dc.data_ptr(), da.data_ptr(), db.data_ptr(), n, F32, mode, unroll, nt, 512,
              threads, stream())
    torch.cuda.synchronize()
    assert same_bits(from_dev(dc, F32), oracle.sum2(a, b), F32)


@pytest.mark.parametrize("dtype", ALL_DTYPES)
@pytest.mark.parametrize("nsrc", [1, 2, 3, 5, 8, 16])
def test_multi_sum_matches_oracle_fold(gpu, oracle, dtype, nsrc):
    import torch
    from tips_amd import _lib
    rng = np.random.default_rng(200 + nsrc * 7 + dtype)
    n = 4099 * 3
    ins = [rand(dtype, n, rng) for _ in range(nsrc)]
    devs = [to_dev(x) for x in ins]
    out = torch.empty_like(devs[0])
    pp, _keep = _lib.ptr_array([d.data_ptr() for d in devs])
    _lib.call("tips_multi_sum", out.data_ptr(), pp, nsrc, n, dtype, stream())
    torch.cuda.synchronize()
    assert same_bits(from_dev(out, dtype), oracle.fold(ins, code=dtype, wide_acc=True), dtype)
    # in place into the last source, unaligned view
    pp, _keep = _lib.ptr_array([d[1:].data_ptr() for d in devs])
    _lib.call("tips_multi_sum", devs[-1][1:].data_ptr(), pp, nsrc, n - 1, dtype, stream())
    torch.cuda.synchronize()
    exp = oracle.fold([x[1:] for x in ins], code=dtype, wide_acc=True)
    assert same_bits(from_dev(devs[-1], dtype)[1:], exp, dtype)


@pytest.mark.slow
def test_config2_full_size(gpu, oracle):
    """BASELINE config 2: two 256 MiB fp32 buffers, U[-1,1), seeds 1 and 2; out-of-place and in-place."""
    import torch
    from tips_amd import _lib
    n = 67108864
    a = (np.random.default_rng(1).random(n) * 2 - 1).astype(np.float32)
    b = (np.random.default_rng(2).random(n) * 2 - 1).astype(np.float32)
    exp = oracle.sum2(a, b)
    da, db = to_dev(a), to_dev(b)
    dc = torch.empty_like(da)
    _lib.call("tips_bucket_sum", dc.data_ptr(), da.data_ptr(), db.data_ptr(), n, F32, stream())
    _lib.call("tips_bucket_sum", da.data_ptr(), da.data_ptr(), db.data_ptr(), n, F32, stream())
    torch.cuda.synchronize()
    assert np.array_equal(from_dev(dc, F32).view(np.uint32), exp.view(np.uint32))
    assert np.array_equal(from_dev(da, F32).view(np.uint32), exp.view(np.uint32))


def test_python_bucket_sum(gpu):
    import torch
    a = torch.randn(1000, device="cuda")
    b = torch.randn(1000, device="cuda")
    assert torch.equal(gpu.bucket_sum(a, b), a + b)


@pytest.mark.slow
def test_count_beyond_int32(gpu):
    """count > 2^31 elements (the reference passes an int count, utils.h:62; the C-ABI takes int64):
    2^31 + 13 fp16 elements (4 GiB per buffer), compared with torch's fp16 add (same correctly
    rounded result) on the device, including the scalar tail."""
    import torch
    from tips_amd import _lib
    n = (1 << 31) + 13
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    a = torch.empty(n, dtype=torch.float16, device="cuda").uniform_(-100, 100, generator=g)
    b = torch.empty(n, dtype=torch.float16, device="cuda").uniform_(-100, 100, generator=g)
    c = torch.empty_like(a)
    _lib.call("tips_bucket_sum", c.data_ptr(), a.data_ptr(), b.data_ptr(), n, F16, stream())
    torch.cuda.synchronize()
    assert torch.equal(c, a + b)
    assert torch.equal(c[-13:], a[-13:] + b[-13:])


@pytest.mark.parametrize("nseg", [1, 3, 7, 16])
@pytest.mark.parametrize("shift", [0, 1, 4, 16])
def test_xfer_segments(gpu, nseg, shift):
    """The peer schedule's transfer kernel: ragged segment sizes (0, < 16 B, tile multiples and
    not), 16-B-aligned and misaligned pointers; every byte copied, nothing written outside."""
    import torch
    from tips_amd import _lib
    rng = np.random.default_rng(nseg * 100 + shift)
    sizes = [int(x) for x in rng.choice([0, 1, 15, 16, 17, 4096, 16384, 16385, 65536 + 48, 1000003], size=nseg)]
    src = torch.from_numpy(rng.integers(0, 256, size=sum(sizes) + 64 * nseg + 64, dtype=np.uint8)).cuda()
    dst = torch.full((sum(sizes) + 64 * nseg + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    offs, o = [], shift
    for k in sizes:
        offs.append(o)
        o += k + 48 + shift
    pd, _k1 = _lib.ptr_array([dst.data_ptr() + x for x in offs])
    ps, _k2 = _lib.ptr_array([src.data_ptr() + x for x in offs])
    pb, _k3 = _lib.i64_array(sizes)
    _lib.dev_call("tips_xfer", pd, ps, pb, nseg, stream())
    torch.cuda.synchronize()
    d, s = dst.cpu().numpy(), src.cpu().numpy()
    mask = np.zeros(len(d), dtype=bool)
    for x, k in zip(offs, sizes):
        assert np.array_equal(d[x:x + k], s[x:x + k])
        mask[x:x + k] = True
    assert np.all(d[~mask] == 0xAB)
