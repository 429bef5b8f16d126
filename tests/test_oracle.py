"""Pin the CPU oracle (oracle/oracle.c) before trusting it.

Against: the reference's three KATs (their inputs, formulas and tolerances),
the MPICH golden vectors in tests/golden (the reference's exact
MPI_Allreduce(MPI_SUM) call), numpy/torch for the 16-bit conversions, and the
reference's own KAT binary compiled from its sources (oracle/_ref) when present.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import golden_cases, load_golden, REPO


# ---------------------------------------------------------------- reference KATs

def test_kat_utils_test(oracle):
    """utils_test.cc:12-37: p=5, x_r[i]=0.1*i*r -> 0.1*i*p(p-1)/2, abs tol 1e-5."""
    p, n = 5, 4
    ins = [np.array([i * 0.1 * r for i in range(n)], dtype=np.float64).astype(np.float32) for r in range(p)]
    for out in (oracle.fold(ins), oracle.ring(ins)[0]):
        for i in range(n):
            assert abs(out[i] - i * 0.1 * ((p - 1) * p / 2)) <= 1e-5


def test_kat_coordinator_test(oracle):
    """coordinator_test.cc:10-45: p=3, 2x4, x[i]=0.1*i -> x*p, tol 1e-4."""
    p = 3
    x = np.array([i * 0.1 for i in range(8)], dtype=np.float64).astype(np.float32)
    for out in (oracle.fold([x] * p), oracle.ring([x] * p)[0]):
        assert np.all(np.abs(x * p - out) <= 1e-4)


def test_kat_mpi_allreduce(oracle):
    """mpi_allreduce_test.cc:8-33: p=3, n=10, x[i]=0.1*i -> 0.1*i*p, tol 1e-5."""
    p = 3
    x = np.array([i * 0.1 for i in range(10)], dtype=np.float64).astype(np.float32)
    for out in (oracle.fold([x] * p), oracle.ring([x] * p)[0]):
        for i in range(10):
            assert abs(out[i] - i * 0.1 * p) <= 1e-5


# ---------------------------------------------------------------- golden vectors (MPICH)

CASES = golden_cases()


@pytest.mark.parametrize("name", sorted(CASES))
def test_golden(oracle, name):
    meta = CASES[name]
    ins, exp = load_golden(name)
    if name == "cfg1_f32_p2_1MiB":
        import hashlib
        assert hashlib.sha256(ins.tobytes()).hexdigest() == meta["inputs_sha256"]
    rows = [ins[r] for r in range(ins.shape[0])]
    for got in (oracle.fold(rows), oracle.ring(rows)[0]):
        assert got.dtype == exp.dtype and got.shape == exp.shape
        if exp.dtype.kind == "i":
            assert np.array_equal(got, exp), "integer sums must be bit-exact (wrap-around)"
        elif name.startswith("signed"):
            # norm-wise: |got - ref| <= 1e-6 * sum_r |x_r|
            bound = 1e-6 * np.sum(np.abs(ins.astype(np.float64)), axis=0)
            assert np.all(np.abs(got.astype(np.float64) - exp.astype(np.float64)) <= bound)
        elif name.startswith("kat"):
            assert np.allclose(got, exp, rtol=0, atol=1e-6)
        else:
            rel = np.abs(got.astype(np.float64) - exp.astype(np.float64)) / np.abs(exp.astype(np.float64))
            assert rel.max() <= 1e-6, rel.max()


def test_golden_manifest_hashes():
    import hashlib
    for name, meta in CASES.items():
        with open(os.path.join(REPO, "tests", "golden", name + ".npz"), "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == meta["sha256"], name


# ---------------------------------------------------------------- arithmetic details

def test_int_wraparound(oracle):
    a = np.array([2**31 - 1, -2**31, 5], dtype=np.int32)
    b = np.array([1, -1, -7], dtype=np.int32)
    assert oracle.sum2(a, b).tolist() == [-2**31, 2**31 - 1, -2]
    a = np.array([2**63 - 1], dtype=np.int64)
    assert oracle.sum2(a, np.array([1], dtype=np.int64)).tolist() == [-2**63]


def test_float_specials(oracle):
    tiny = np.array([1], dtype=np.uint32).view(np.float32)[0]  # smallest subnormal
    a = np.array([np.inf, -np.inf, np.nan, tiny, 3.0e38], dtype=np.float32)
    b = np.array([1.0, np.inf, 0.0, tiny, 3.0e38], dtype=np.float32)
    out = oracle.sum2(a, b)
    assert out[0] == np.inf and np.isnan(out[1]) and np.isnan(out[2])
    assert out[3:4].view(np.uint32)[0] == 2 and out[4] == np.inf  # denormals kept, overflow to inf


def test_half_conversions_exhaustive(oracle):
    L = oracle.load()
    allh = np.arange(65536, dtype=np.uint32).astype(np.uint16)
    f_np = allh.view(np.float16).astype(np.float32)
    f_or = np.array([L.oracle_half_to_float(int(h)) for h in allh], dtype=np.float32)
    nan = np.isnan(f_np)
    assert np.array_equal(np.isnan(f_or), nan)
    assert np.array_equal(f_or[~nan].view(np.uint32), f_np[~nan].view(np.uint32))
    rng = np.random.default_rng(3)
    xs = np.concatenate([rng.standard_normal(20000).astype(np.float32) * s for s in (1e-6, 1e-3, 1, 100, 6e4)])
    xs = np.concatenate([xs, np.array([65504, 65519.99, 65520, 6.1e-5, 5.96e-8, 2.98e-8, 2.99e-8], np.float32)])
    h_or = np.array([L.oracle_float_to_half(float(x)) for x in xs], dtype=np.uint16)
    assert np.array_equal(h_or, xs.astype(np.float16).view(np.uint16))


def test_bf16_conversion_matches_torch(oracle):
    torch = pytest.importorskip("torch")
    L = oracle.load()
    rng = np.random.default_rng(4)
    xs = np.concatenate([rng.standard_normal(20000).astype(np.float32) * s for s in (1e-30, 1, 1e30)])
    got = np.array([L.oracle_float_to_bf16(float(x)) for x in xs], dtype=np.uint16)
    ref = torch.from_numpy(xs).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    assert np.array_equal(got, ref)


def test_f16_sum_is_correctly_rounded(oracle):
    rng = np.random.default_rng(5)
    a = (rng.standard_normal(50000) * 100).astype(np.float16)
    b = (rng.standard_normal(50000) * 100).astype(np.float16)
    got = oracle.sum2(a, b)
    ref = (a.astype(np.float64) + b.astype(np.float64)).astype(np.float16)  # exact sum, one rounding
    assert np.array_equal(got.view(np.uint16), ref.view(np.uint16))


def test_ring_fold_order(oracle):
    """Ring chunk c is folded in[c], in[c+1], ...: check against a numpy restatement."""
    rng = np.random.default_rng(6)
    p, n = 5, 3001
    ins = [rng.standard_normal(n).astype(np.float32) for _ in range(p)]
    got = oracle.ring(ins, align_elems=64)
    for r in range(p):
        assert np.array_equal(got[r].view(np.uint32), got[0].view(np.uint32))
    exp = np.empty(n, np.float32)
    for c in range(p):
        b, e = oracle.chunk_bounds(n, p, 64, c)
        acc = ins[c][b:e].copy()
        for k in range(1, p):
            acc = ins[(c + k) % p][b:e] + acc
        exp[b:e] = acc
    assert np.array_equal(got[0].view(np.uint32), exp.view(np.uint32))


@pytest.mark.parametrize("n,p,align", [(0, 4, 64), (1, 8, 64), (63, 2, 64), (4099, 8, 64), (10**6 + 3, 7, 32)])
def test_chunk_bounds_partition(oracle, n, p, align):
    prev = 0
    for c in range(p):
        b, e = oracle.chunk_bounds(n, p, align, c)
        assert b == prev and e >= b
        if e < n:
            assert b % align == 0 and e % align == 0
        prev = e
    assert prev == n


def test_wide_fold_f16(oracle):
    rng = np.random.default_rng(8)
    ins = [(rng.standard_normal(4000)).astype(np.float16) for _ in range(8)]
    got = oracle.fold(ins, wide_acc=True)
    acc = ins[0].astype(np.float32)
    for x in ins[1:]:
        acc = acc + x.astype(np.float32)
    assert np.array_equal(got.view(np.uint16), acc.astype(np.float16).view(np.uint16))


# ---------------------------------------------------------------- reference's own KAT binary

@pytest.mark.skipif(not os.path.exists(os.path.join(REPO, "oracle", "_ref", "mpi_allreduce_test"))
                    or not shutil.which("mpirun", path="/opt/conda/bin"),
                    reason="reference KAT not built here (needs /root/reference + MPICH)")
def test_reference_kat_binary():
    exe = os.path.join(REPO, "oracle", "_ref", "mpi_allreduce_test")
    r = subprocess.run(["/opt/conda/bin/mpirun", "-np", "3", exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]


def test_compression_casts_match_numpy_and_rne():
    """The oracle's Compression.fp16 casts (oracle_cast_to16 / oracle_cast_from16, the checker of
    tips_fused_allreduce_cast): f32 -> f16 equals numpy's IEEE cast (RNE, subnormals, overflow to
    inf) on every value class; f32 -> bf16 -> f32 rounds to nearest even on the 16 dropped bits."""
    import numpy as np
    import oracle_bind as ob
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.standard_normal(200000).astype(np.float32),
                        (rng.standard_normal(20000) * 1e-6).astype(np.float32),   # f16 subnormals
                        (rng.standard_normal(20000) * 1e5).astype(np.float32),    # f16 overflow
                        np.array([0.0, -0.0, np.inf, -np.inf, 65504.0, 65520.0, 65519.99, 2 ** -24, 2 ** -25],
                                 dtype=np.float32)])
    h = ob.cast_to16(x, ob.F16)
    assert np.array_equal(h, x.astype(np.float16).view(np.uint16))
    assert np.array_equal(ob.cast_from16(h, ob.F16), x.astype(np.float16).astype(np.float32))
    b = ob.cast_to16(x, ob.BF16).astype(np.uint32)
    u = x.view(np.uint32).astype(np.uint64)
    exp = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint32)
    assert np.array_equal(b, exp)
    assert np.array_equal(ob.cast_from16(b.astype(np.uint16), ob.BF16).view(np.uint32), b << 16)
