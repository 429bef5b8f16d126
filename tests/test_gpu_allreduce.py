"""-m gpu: the allreduce schedules and the drop-in surface, through the C-ABI.

The ring and direct schedules are run for p virtual ranks on the one GPU of
the test box (tips_ring_simulate / tips_direct_simulate: same chunking,
sub-chunk pipeline, streams, events and sum kernels as the RCCL path; peer
transfers become device copies) and compared bit-exact with the oracle's
restatement of the same schedule; against the MPICH golden vectors they are
held to the reference's tolerance (fp32 <= 1e-6 relative, ints bit-exact).
The real RCCL exchange needs >1 GPU and is exercised by bench.py on the
8-GPU node.
"""
import numpy as np
import pytest

from conftest import golden_cases, load_golden
from gpu_util import ALL_DTYPES, BF16, F16, F32, F64, I32, I64, NPDT, from_dev, rand, same_bits, simulate, stream, to_dev

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", ALL_DTYPES)
@pytest.mark.parametrize("p", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("n", [1, 7, 4099, 262144, 1000003])
def test_ring_schedule_matches_oracle(gpu, oracle, dtype, p, n):
    rng = np.random.default_rng(1000 * p + n % 997 + dtype)
    ins = [rand(dtype, n, rng) for _ in range(p)]
    exp = oracle.ring(ins, code=dtype)[0]
    for got in simulate("ring", ins, dtype):
        assert same_bits(got, exp, dtype)


@pytest.mark.parametrize("dtype", ALL_DTYPES)
@pytest.mark.parametrize("p", [2, 3, 8, 16])
@pytest.mark.parametrize("n", [1, 4099, 1000003])
def test_direct_schedule_matches_oracle(gpu, oracle, dtype, p, n):
    rng = np.random.default_rng(2000 * p + n % 991 + dtype)
    ins = [rand(dtype, n, rng) for _ in range(p)]
    exp = oracle.fold(ins, code=dtype, wide_acc=True)
    for got in simulate("direct", ins, dtype):
        assert same_bits(got, exp, dtype)


@pytest.mark.parametrize("dtype", ALL_DTYPES)
@pytest.mark.parametrize("p", [2, 3, 8, 16])
@pytest.mark.parametrize("n", [1, 4099, 262147])
@pytest.mark.parametrize("transport", [0, 1])
def test_oneshot_schedule_matches_oracle(gpu, oracle, dtype, p, n, transport):
    rng = np.random.default_rng(3000 * p + n % 983 + dtype)
    ins = [rand(dtype, n, rng) for _ in range(p)]
    exp = oracle.fold(ins, code=dtype, wide_acc=True)
    for got in simulate("oneshot", ins, dtype, transport=transport):
        assert same_bits(got, exp, dtype)


@pytest.mark.parametrize("kind", ["ring", "direct"])
@pytest.mark.parametrize("dtype", [F32, I64, F16])
def test_pipelined_subchunks_inplace(gpu, oracle, monkeypatch, kind, dtype):
    """Force K=4 sub-chunks on small buckets, in place (in == out)."""
    monkeypatch.setenv("TIPS_MIN_SUBCHUNK_BYTES", "256")
    monkeypatch.setenv("TIPS_PIPELINE_DEPTH", "4")
    rng = np.random.default_rng(77)
    for p, n in [(4, 50001), (7, 131), (8, 262147)]:
        ins = [rand(dtype, n, rng) for _ in range(p)]
        exp = oracle.ring(ins, code=dtype)[0] if kind == "ring" else oracle.fold(ins, code=dtype, wide_acc=True)
        for got in simulate(kind, ins, dtype, inplace=True):
            assert same_bits(got, exp, dtype)


@pytest.mark.parametrize("kind", ["ring", "direct"])
@pytest.mark.parametrize("dtype", [F32, I32, BF16, F64])
@pytest.mark.parametrize("p,n", [(2, 4099), (4, 1000003), (8, 262147)])
def test_schedules_over_rccl_selfloop(gpu, oracle, monkeypatch, kind, dtype, p, n):
    """Same schedules with every peer transfer as a grouped ncclSend/ncclRecv (RCCL, rank to itself)."""
    monkeypatch.setenv("TIPS_MIN_SUBCHUNK_BYTES", "65536")
    rng = np.random.default_rng(31 * p + dtype)
    ins = [rand(dtype, n, rng) for _ in range(p)]
    exp = oracle.ring(ins, code=dtype)[0] if kind == "ring" else oracle.fold(ins, code=dtype, wide_acc=True)
    for got in simulate(kind, ins, dtype, transport=1):
        assert same_bits(got, exp, dtype)


CASES = golden_cases()


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("kind", ["ring", "direct", "oneshot"])
def test_golden_vectors(gpu, name, kind):
    ins, exp = load_golden(name)
    dtype = {"f32": F32, "f64": F64, "i32": I32, "i64": I64}[CASES[name]["dtype"]]
    outs = simulate(kind, [ins[r] for r in range(ins.shape[0])], dtype)
    for got in outs:
        assert np.array_equal(bits(got), bits(outs[0])), "every rank ends with the same bits"
        if exp.dtype.kind == "i":
            assert np.array_equal(got, exp)
        elif name.startswith("signed"):
            bound = 1e-6 * np.sum(np.abs(ins.astype(np.float64)), axis=0)
            assert np.all(np.abs(got.astype(np.float64) - exp) <= bound)
        elif name.startswith("kat"):
            # the reference KAT tolerances: utils_test 1e-5, coordinator_test 1e-4, mpi_allreduce_test 1e-5
            assert np.allclose(got, exp, rtol=0, atol=1e-6)
        else:
            assert (np.abs(got.astype(np.float64) - exp) / np.abs(exp)).max() <= 1e-6


def bits(a):
    return np.ascontiguousarray(a).view(np.uint8)


def test_reference_kats_formulas(gpu):
    """The three reference KATs through both device schedules, with their own formulas/tolerances."""
    p, n = 5, 4
    ins = [np.array([i * 0.1 * r for i in range(n)], np.float64).astype(np.float32) for r in range(p)]
    for kind in ("ring", "direct"):
        out = simulate(kind, ins, F32)[0]
        assert all(abs(out[i] - i * 0.1 * ((p - 1) * p / 2)) <= 1e-5 for i in range(n))
        x = np.array([i * 0.1 for i in range(8)], np.float64).astype(np.float32)
        out = simulate(kind, [x] * 3, F32)[0]
        assert np.all(np.abs(x * 3 - out) <= 1e-4)
        x = np.array([i * 0.1 for i in range(10)], np.float64).astype(np.float32)
        out = simulate(kind, [x] * 3, F32)[0]
        assert all(abs(out[i] - i * 0.1 * 3) <= 1e-5 for i in range(10))


def test_empty_and_single_rank(gpu, oracle):
    x = np.arange(10, dtype=np.float32)
    assert np.array_equal(simulate("ring", [x], F32)[0], x)
    assert np.array_equal(simulate("direct", [x], F32)[0], x)
    from tips_amd import _lib
    pp, _k = _lib.ptr_array([0, 0])
    assert _lib.dev().tips_ring_simulate(pp, pp, 2, 0, F32, None) == 0


@pytest.mark.slow
def test_ring_p8_256MiB_property(gpu, oracle):
    """8 virtual ranks x 256 MiB fp32 (config-3 shape at 1/4 size): ring == oracle ring, bitwise,
    every rank identical, and within 1e-6 relative of a float64 sum (positive data)."""
    p, n = 8, 67108864
    ins = [(0.5 + np.random.default_rng(3000 + r).random(n)).astype(np.float32) for r in range(p)]
    outs = simulate("ring", ins, F32, inplace=True)
    exp = oracle.ring(ins)[0]
    for got in outs:
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))
    ref = np.sum(np.stack(ins).astype(np.float64), axis=0)
    assert (np.abs(outs[0] - ref) / ref).max() <= 1e-6


# ------------------------------------------------------------------ drop-in surface (one rank)

def test_allreduce_single_rank_device_and_host(gpu):
    import torch
    assert gpu.size() == 1 and gpu.rank() == 0
    t = torch.randn(12345, device="cuda")
    assert torch.equal(gpu.allreduce(t), t)
    assert torch.equal(gpu.allreduce_op(t), t)
    h = np.random.default_rng(0).random(1001).astype(np.float64)
    assert np.array_equal(gpu.allreduce(h), h)
    c = torch.arange(77, dtype=torch.int64)
    assert torch.equal(gpu.allreduce(c), c)
    f = torch.randn(999, device="cuda")
    out = gpu.allreduce(f, compression=gpu.Compression.fp16)
    assert out.dtype == torch.float32 and torch.equal(out, f.half().float())
    with pytest.raises(TypeError, match="Not supported dtype"):
        gpu.allreduce(torch.zeros(3, dtype=torch.uint8, device="cuda"))


@pytest.mark.parametrize("n", [1, 3, 4, 5, 1023, 4099, (1 << 20) + 7, 3 << 21])
@pytest.mark.parametrize("dtype", [F32, F16, F64])
def test_single_rank_out_of_place_copy(gpu, n, dtype):
    """At one rank an out-of-place tips_allreduce / tips_broadcast is a copy (MPI_Allreduce returns the
    input): copy_buf_kernel for 16-B aligned pointers (vectors + a bytewise tail), hipMemcpyAsync
    otherwise. Every byte of out copied, nothing past it touched, for aligned and shifted views."""
    import torch
    from tips_amd import _lib
    tdt, idt = {F32: (torch.float32, torch.int32), F16: (torch.float16, torch.int16),
                F64: (torch.float64, torch.int64)}[dtype]
    s = torch.cuda.current_stream().cuda_stream
    for shift in (0, 1, 2):  # elements: shift * element size bytes off the allocation's aligned base
        src = torch.randn(n + 8, device="cuda").to(tdt)
        sentinel = torch.full((n + 8,), 7.0, device="cuda", dtype=tdt)
        i = src[shift:shift + n]
        for call in ("tips_allreduce", "tips_broadcast"):
            dst = sentinel.clone()
            o = dst[shift:shift + n]
            args = (_lib.OP_SUM,) if call == "tips_allreduce" else (0,)  # op / root
            assert _lib.call(call, i.data_ptr(), o.data_ptr(), n, dtype, *args, s) == 0
            torch.cuda.synchronize()
            assert torch.equal(o.view(idt), i.view(idt)), (call, shift)
            assert torch.equal(dst[:shift], sentinel[:shift]) and torch.equal(dst[shift + n:], sentinel[shift + n:])


def test_rccl_allreduce_single_rank(gpu):
    import torch
    prev = gpu.set_algorithm("rccl")
    try:
        t = torch.randn(4096, device="cuda")
        assert torch.equal(gpu.allreduce(t), t)
    finally:
        gpu.set_algorithm(prev)


@pytest.mark.parametrize("aligned", [False, True])
@pytest.mark.parametrize("wire", ["float16", "bfloat16"])
@pytest.mark.parametrize("threshold", [4096, 64 << 20])
def test_fused_cast_round_trip(gpu, monkeypatch, threshold, wire, aligned):
    """One rank: tips_fused_allreduce_cast is the round trip f32 -> wire -> f32 (the reference's
    compress -> allreduce -> decompress at one rank, compression.py:49-66), bit-exact against the
    oracle's casts (RNE): 300 odd-sized misaligned views (ragged ends: the kernel's per-element
    path), a tensor above the threshold at 4096 (the range-cast path through the scratch buffer),
    values that round to f16 subnormals and overflow to inf; out of place through
    tips_amd.fused_allreduce_cast and in place through the C-ABI; the inputs of the out-of-place
    call unchanged. aligned=True starts every view on 16 B (the kernels' quad path: 16 B of f32 and
    8 B of wire per lane, the odd sizes' last n % 4 elements one at a time)."""
    import torch
    import oracle_bind
    from tips_amd import _lib
    monkeypatch.setenv("TIPS_FUSION_THRESHOLD", str(threshold))
    code = oracle_bind.F16 if wire == "float16" else oracle_bind.BF16
    rng = np.random.default_rng(7)
    sizes = [int(round(2 ** rng.uniform(0, 14))) for _ in range(300)] + [5000, 1, 70001]
    vals = rng.standard_normal(sum(sizes) + 4 * len(sizes) + 4).astype(np.float32)
    vals[::97] *= 1e-6   # f16 subnormals
    vals[::211] *= 1e5   # beyond f16's range: inf
    base = torch.from_numpy(vals).cuda()
    views, off = [], 0 if aligned else 1  # offset 1: misaligned views (4-B aligned f32 sides), a gap after each
    for k in sizes:
        views.append(base[off:off + k])
        off += k + 1
        if aligned:
            off = (off + 3) // 4 * 4
    before = base.clone()
    exp = [oracle_bind.cast_from16(oracle_bind.cast_to16(v.cpu().numpy(), code), code) for v in views]
    for _ in range(2):  # (the second call finds the layout and the table)
        outs = gpu.fused_allreduce_cast(views, wire)
        torch.cuda.synchronize()
        for o, e in zip(outs, exp):
            assert o.dtype == torch.float32
            assert np.array_equal(o.cpu().numpy().view(np.uint32), e.view(np.uint32))
        del outs
    assert torch.equal(base, before)
    # in place through the C-ABI (in == out)
    pp, _k = _lib.ptr_array([v.data_ptr() for v in views])
    cp, _k2 = _lib.i64_array(sizes)
    wcode = _lib.FLOAT16 if wire == "float16" else _lib.BFLOAT16
    _lib.call("tips_fused_allreduce_cast", pp, pp, cp, len(sizes), _lib.FLOAT32, wcode,
              torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for v, e in zip(views, exp):
        assert np.array_equal(v.cpu().numpy().view(np.uint32), e.view(np.uint32))
    # only f32 tensors, only 16-bit wires
    assert _lib.lib().tips_fused_allreduce_cast(pp, pp, cp, len(sizes), _lib.FLOAT64, wcode, None) == -5
    assert _lib.lib().tips_fused_allreduce_cast(pp, pp, cp, len(sizes), _lib.FLOAT32, _lib.FLOAT32, None) == -5


@pytest.mark.parametrize("measure_pack", ["1", "0"])
@pytest.mark.parametrize("threshold", [4096, 64 << 20])
def test_fused_pack_unpack_round_trip(gpu, monkeypatch, threshold, measure_pack):
    """One rank: fused allreduce == identity. With TIPS_FUSION_MEASURE_PACK=1 the buckets are packed
    and unpacked as at N > 1, so pack -> bucket -> unpack must move every byte exactly, across many
    buckets, odd sizes, misaligned views and tensors larger than the threshold; without it, in place
    is no work and out of place one copy."""
    import torch
    monkeypatch.setenv("TIPS_FUSION_THRESHOLD", str(threshold))
    monkeypatch.setenv("TIPS_FUSION_MEASURE_PACK", measure_pack)
    rng = np.random.default_rng(20261015)
    sizes = [int(round(2 ** rng.uniform(0, 14))) for _ in range(300)] + [5000, 1]
    base = torch.randn(sum(sizes) + len(sizes) + 1, device="cuda")
    views, off = [], 1  # offset 1: misaligned views; a 1-element gap after each (no contiguous runs)
    for s in sizes:
        views.append(base[off:off + s])
        off += s + 1
    before = [v.clone() for v in views]
    gaps = base.clone()
    gpu.fused_allreduce_(views)
    gpu.fused_allreduce_(views)  # second call hits the plan cache
    torch.cuda.synchronize()
    for v, b in zip(views, before):
        assert torch.equal(v, b)
    assert torch.equal(base, gaps)
    # out of place into separate tensors: at one rank every byte must travel pack -> bucket -> unpack
    for _ in range(2):
        outs = gpu.fused_allreduce(views)
        torch.cuda.synchronize()
        for o, b in zip(outs, before):
            assert torch.equal(o, b)


def test_fused_call_captures_into_a_graph(gpu, monkeypatch):
    """tips_fused_allreduce_oop captured with torch.cuda.graph (what bench.py's graph_replayed_step
    replays): one rank in measure-pack mode, so every byte goes pack -> bucket -> unpack. Each
    replay must rewrite the outputs from the inputs' current values."""
    import torch
    monkeypatch.setenv("TIPS_FUSION_MEASURE_PACK", "1")
    monkeypatch.setenv("TIPS_FUSION_THRESHOLD", str(1 << 20))
    rng = np.random.default_rng(77)
    sizes = [int(round(2 ** rng.uniform(0, 17))) for _ in range(60)]
    ins = [torch.randn(n, device="cuda") for n in sizes]
    outs = [torch.empty_like(t) for t in ins]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        gpu.fused_allreduce(ins, out_list=outs)  # builds the plan outside the capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            gpu.fused_allreduce(ins, out_list=outs)
        for k in range(3):
            for t in ins:
                t.add_(1.0)
            for o in outs:
                o.zero_()
            g.replay()
            torch.cuda.synchronize()
            for t, o in zip(ins, outs):
                assert torch.equal(o, t)


def test_captured_fused_call_keeps_its_table():
    """a captured fused call's replays read its pointer table long after the capture.
    Capture, then 20 eager calls on other pointer sets of the same layout (more than the 16 tables
    a layout keeps, so the LRU reuses buffers) plus one from a second stream; then replay: the
    replay must still move its own tensors, bit-exact, and leave the others alone. After a
    threshold change (new fusion slots) the replay still packs into the slots it captured.
    (Its own process: the captured table stays pinned for the life of the job.)"""
    import subprocess
    import sys
    from conftest import REPO
    code = r'''
import os, numpy as np, torch
os.environ.update(TIPS_FUSION_MEASURE_PACK="1", TIPS_FUSION_THRESHOLD=str(1 << 20))
import tips_amd
from tips_amd import _lib
tips_amd.init()
rng = np.random.default_rng(78)
sizes = [int(round(2 ** rng.uniform(0, 16))) for _ in range(40)]
ins = [torch.randn(n, device="cuda") for n in sizes]
outs = [torch.empty_like(t) for t in ins]
side, other = torch.cuda.Stream(), torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    tips_amd.fused_allreduce(ins, out_list=outs)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        tips_amd.fused_allreduce(ins, out_list=outs)
torch.cuda.synchronize()
sets = []
for k in range(20):
    xi = [torch.randn(n, device="cuda") for n in sizes]
    xo = [torch.empty_like(t) for t in xi]
    with torch.cuda.stream(other if k == 19 else side):
        tips_amd.fused_allreduce(xi, out_list=xo)
    sets.append((xi, xo))
torch.cuda.synchronize()
for xi, xo in sets:
    assert all(torch.equal(a, b) for a, b in zip(xi, xo))
snap = [[o.clone() for o in xo] for _, xo in sets]
for t in ins:
    t.add_(2.0)
for o in outs:
    o.zero_()
with torch.cuda.stream(side):
    g.replay()
torch.cuda.synchronize()
assert all(torch.equal(o, t) for t, o in zip(ins, outs))
for (_, xo), sn in zip(sets, snap):
    assert all(torch.equal(a, b) for a, b in zip(xo, sn))
os.environ["TIPS_FUSION_THRESHOLD"] = str(2 << 20)  # new slots: the graph keeps packing into the old ones
xo = [torch.empty_like(t) for t in ins]
tips_amd.fused_allreduce(ins, out_list=xo)
torch.cuda.synchronize()
assert all(torch.equal(o, t) for t, o in zip(ins, xo))
for t in ins:
    t.add_(1.0)
with torch.cuda.stream(side):
    g.replay()
torch.cuda.synchronize()
assert all(torch.equal(o, t) for t, o in zip(ins, outs))
os.environ["TIPS_FUSION_THRESHOLD"] = str(1 << 20)
del g
torch.cuda.synchronize()
tips_amd.shutdown()
print("CAPTURE_TABLE_OK")
'''
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=REPO, timeout=300)
    assert "CAPTURE_TABLE_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def test_fused_views_of_one_buffer(gpu, monkeypatch):
    """Views of one flat buffer mixed with separate tensors (measure-pack mode: every byte through
    pack -> bucket -> unpack at one rank): the layout ignores where tensors lie, so the views are
    packed like any tensor; in place it must leave the bytes around them alone; out of place into
    the views of another flat buffer."""
    import torch
    monkeypatch.setenv("TIPS_FUSION_MEASURE_PACK", "1")
    monkeypatch.setenv("TIPS_FUSION_THRESHOLD", str(1 << 18))
    sizes = [1000, 3, 70000, 257, 20000]
    flat = torch.randn(sum(sizes) + 10, device="cuda")
    guard = flat[-10:].clone()
    run = list(torch.split(flat[:sum(sizes)], sizes))
    other = [torch.randn(n, device="cuda") for n in (5, 9999, 70000)]
    lst = run[:2] + other[:1] + run[2:] + other[1:]
    before = [t.clone() for t in lst]
    gpu.fused_allreduce_(lst)
    outs_flat = torch.empty(sum(t.numel() for t in lst), device="cuda")
    outs = list(torch.split(outs_flat, [t.numel() for t in lst]))
    gpu.fused_allreduce(lst, out_list=outs)
    torch.cuda.synchronize()
    for t, b, o in zip(lst, before, outs):
        assert torch.equal(t, b) and torch.equal(o, b)
    assert torch.equal(flat[-10:], guard)


@pytest.mark.parametrize("measure_pack", ["1", "0"])
@pytest.mark.parametrize("threshold", [8192, 1 << 20, 64 << 20])
def test_fused_flat_outputs(gpu, monkeypatch, threshold, measure_pack):
    """tips_fused_allreduce_flat at one rank (the identity): every tensor lands at its
    tips_fused_layout offset of one flat buffer - through the per-bucket packs (measure-pack mode,
    as at N > 1) or one copy launch - for every dtype, odd element counts (ragged 16-B ends, 2-B
    tails for 16-bit types), inputs that are only element-aligned (views at offset 1), empty tensors
    and tensors above the threshold (reduced out of place into their own region)."""
    import torch
    monkeypatch.setenv("TIPS_FUSION_THRESHOLD", str(threshold))
    monkeypatch.setenv("TIPS_FUSION_MEASURE_PACK", measure_pack)
    tdt = {F32: torch.float32, F64: torch.float64, I32: torch.int32, I64: torch.int64, F16: torch.float16,
           BF16: torch.bfloat16}
    rng = np.random.default_rng(threshold % 1000 + int(measure_pack))
    for dtype in ALL_DTYPES:
        sizes = [int(round(2 ** rng.uniform(0, 15))) for _ in range(120)] + [0, 3, 1, 40000, 7]
        base = torch.randint(-1000, 1000, (sum(sizes) + len(sizes) + 2,), device="cuda").to(tdt[dtype])
        ins, off = [], 1  # offset 1: element-aligned only
        for s in sizes:
            ins.append(base[off:off + s])
            off += s + 1
        for _ in range(2):
            outs = gpu.fused_allreduce_flat(ins)
            torch.cuda.synchronize()
            for o, t in zip(outs, ins):
                assert o.shape == t.shape and o.dtype == t.dtype and torch.equal(o, t)
            del outs
        # allreduce_grads' N > 1 body on the same list: its C++ list path (tips_amd._fast)
        import tips_amd
        for _ in range(2):
            outs = tips_amd._reduce_grads(ins)
            torch.cuda.synchronize()
            for o, t in zip(outs, ins):
                assert o.shape == t.shape and o.dtype == t.dtype and torch.equal(o, t)
            del outs


def test_fused_flat_output_reuse(gpu, monkeypatch):
    """allreduce_grads' flat outputs are reused only once the caller has released every output:
    held outputs (or a tensor derived from one) keep their buffer; a later call gets another."""
    import torch
    monkeypatch.setenv("TIPS_FUSION_MEASURE_PACK", "1")
    ins = [torch.randn(n, device="cuda") for n in (1000, 3, 70000, 257)]
    a = gpu.fused_allreduce_flat(ins)
    pa = a[0].data_ptr()
    b = gpu.fused_allreduce_flat(ins)  # a still held: a new set
    assert b[0].data_ptr() != pa
    keep = b[2][5:9]  # a derived view keeps b's storage
    del a
    c = gpu.fused_allreduce_flat(ins)  # a released: its set is handed out again
    assert c[0].data_ptr() == pa
    pb = b[0].data_ptr()
    del b, c
    d = gpu.fused_allreduce_flat(ins)
    assert d[0].data_ptr() != pb  # (b's storage is still referenced through `keep`)
    torch.cuda.synchronize()
    for o, t in zip(d, ins):
        assert torch.equal(o, t)
    assert torch.equal(keep, ins[2][5:9])


def test_fusion_caches_with_fresh_tensors(gpu, monkeypatch):
    """The fusion layout depends on the counts only: fresh tensors of the same sizes every call find
    it (tips_fusion_stats), in place, out of place and flat; the same pointers find their table too."""
    import torch
    monkeypatch.setenv("TIPS_FUSION_MEASURE_PACK", "1")
    sizes = [4099, 17, 100000, 3]
    s0 = gpu.fusion_stats()
    for step in range(4):
        ts = [torch.full((n,), float(step), device="cuda") for n in sizes]
        outs = gpu.fused_allreduce_flat(ts)
        torch.cuda.synchronize()
        assert all(torch.equal(o, t) for o, t in zip(outs, ts))
    s1 = gpu.fusion_stats()
    assert s1["layouts_built"] - s0["layouts_built"] == 1 and s1["layout_hits"] - s0["layout_hits"] >= 3
    fixed = [torch.randn(n, device="cuda") for n in sizes]
    gpu.fused_allreduce_(fixed)
    s2 = gpu.fusion_stats()
    gpu.fused_allreduce_(fixed)
    s3 = gpu.fusion_stats()
    assert s3["tables_built"] == s2["tables_built"] and s3["table_hits"] > s2["table_hits"]


def test_fused_list_reuses_arrays_and_revalidates(gpu, monkeypatch):
    """ops.FusedList (DistributedOptimizer's path without gradient bucket views): pointers read in
    C++ every call; the same tensors reuse the cached arrays, a replaced tensor is picked up, a
    count change or a second dtype is refused; one rank with the buckets kept (pack + unpack):
    the tensors come back unchanged. allreduce_grads' C++ path with fresh outputs likewise."""
    import torch
    from tips_amd.ops import FusedList
    monkeypatch.setenv("TIPS_FUSION_MEASURE_PACK", "1")
    sizes = [4099, 17, 100000, 3, 65536]
    ts = [torch.randn(n, device="cuda") for n in sizes]
    ref = [t.clone() for t in ts]
    fl = FusedList(sizes)
    for _ in range(3):
        fl.allreduce_(ts)
    ts[1] = torch.randn(17, device="cuda")
    ref[1] = ts[1].clone()
    fl.allreduce_(ts)
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(ts, ref))
    with pytest.raises(ValueError, match="element counts changed"):
        fl.allreduce_(ts[:-1] + [torch.randn(7, device="cuda")])
    with pytest.raises(TypeError):
        fl.allreduce_(ts[:-1] + [torch.randn(65536, device="cuda", dtype=torch.float64)])
    g = [torch.randn(n, device="cuda") for n in sizes]
    import tips_amd
    outs = tips_amd._reduce_grads(g)
    torch.cuda.synchronize()
    assert [o.shape for o in outs] == [t.shape for t in g] and all(torch.equal(o, t) for o, t in zip(outs, g))


@pytest.mark.parametrize("piece,first", [(256, 256), (4096, 4096), (8 << 20, 8 << 20), (65536, 1024), (16 << 20, 2 << 20)])
def test_fused_host_identity(gpu, monkeypatch, piece, first):
    """tips_fused_allreduce_host at one rank (the identity after H2D -> HBM -> D2H): many host tensors
    of every dtype, pageable numpy and CPU torch, empty ones, pieces from 256 B (tensors span many
    pieces; the copy threads split every piece) to 16 MiB, fixed or ramping up from `first` at the
    head and down to it at the tail; bit-exact, inputs unchanged."""
    import torch
    monkeypatch.setenv("TIPS_HOST_FUSED_PIECE_BYTES", str(piece))
    monkeypatch.setenv("TIPS_HOST_FUSED_FIRST_BYTES", str(first))
    rng = np.random.default_rng(piece % 977)
    for dtype in ALL_DTYPES:
        sizes = [int(round(2 ** rng.uniform(0, 14))) for _ in range(60)] + [0, 1, 3]
        ins = [rand(dtype, s, rng) for s in sizes]
        if dtype == BF16:  # (numpy has no bfloat16: CPU torch tensors)
            ins = [torch.from_numpy(x.view(np.int16)).view(torch.bfloat16) for x in ins]
        before = [x.copy() if dtype != BF16 else x.clone() for x in ins]
        outs = gpu.fused_allreduce_host(ins)
        for o, x, b in zip(outs, ins, before):
            if dtype == BF16:
                assert torch.equal(o.view(torch.int16), b.view(torch.int16)) and torch.equal(x.view(torch.int16), b.view(torch.int16))
            else:
                assert same_bits(o, b, dtype) and same_bits(x, b, dtype)
    ts = [torch.randn(n) for n in (5, 100003, 64)]
    outs = gpu.fused_allreduce_host(ts)
    assert all(torch.equal(o, t) for o, t in zip(outs, ts))
    with pytest.raises(TypeError):
        gpu.fused_allreduce_host([np.zeros(4, np.float32), np.zeros(4, np.float64)])


@pytest.mark.parametrize("threads,piece", [(1, 4096), (8, 1 << 20), (16, 8 << 20)])
def test_fused_host_flat_identity(gpu, monkeypatch, threads, piece):
    """tips_fused_allreduce_host_flat at one rank: the outputs are views of one page-locked host
    buffer (the device writes the sums straight into it), bit-exact for numpy of every dtype with
    odd sizes and empty tensors and for CPU torch bf16; a released set is reused, a held one is
    not, and a later call does not disturb the outputs a caller still holds."""
    import torch
    monkeypatch.setenv("TIPS_HOST_THREADS", str(threads))
    monkeypatch.setenv("TIPS_HOST_FUSED_PIECE_BYTES", str(piece))
    rng = np.random.default_rng(threads * 7 + piece % 1000)
    for dtype in [F32, F64, I32, I64, F16]:
        sizes = [int(round(2 ** rng.uniform(0, 16))) for _ in range(40)] + [0, 1, 3]
        ins = [rand(dtype, s, rng).reshape(-1) for s in sizes]
        outs = gpu.fused_allreduce_host_flat(ins)
        for o, x in zip(outs, ins):
            assert o.shape == x.shape and same_bits(o, x, dtype)
        base = outs[0].base.ctypes.data  # (the address: a reference to the buffer would hold it)
        held = outs
        ins2 = [x[::-1].copy() for x in ins]
        outs2 = gpu.fused_allreduce_host_flat(ins2)
        assert outs2[0].base.ctypes.data != base  # held: a new set
        for o, x, o2, x2 in zip(held, ins, outs2, ins2):
            assert same_bits(o, x, dtype) and same_bits(o2, x2, dtype)
        del held, outs, o, o2  # (the loop variables hold views too)
        outs3 = gpu.fused_allreduce_host_flat(ins)
        assert outs3[0].base.ctypes.data == base  # released: reused
        for o, x in zip(outs3, ins):
            assert same_bits(o, x, dtype)
    tb = [torch.randn(n).to(torch.bfloat16) for n in (5, 100003, 64, 0)]
    outs = gpu.fused_allreduce_host_flat(tb)
    assert all(torch.equal(o.view(torch.int16), t.view(torch.int16)) for o, t in zip(outs, tb))


def test_allreduce_grads_identity_single_rank(gpu):
    import torch
    grads = [torch.randn(10, device="cuda"), None, torch.randn(3, 3, device="cuda")]
    out = gpu.allreduce_grads(grads)
    assert out[1] is None and torch.equal(out[0], grads[0]) and torch.equal(out[2], grads[2])


# ------------------------------------------------------------------ the rest of the op surface (one rank)

@pytest.mark.parametrize("wire", ["float16", "bfloat16"])
def test_fused_cast_range_many_tiles(gpu, monkeypatch, wire):
    """A tensor above the threshold goes through the range cast (cast_range_kernel): 20,971,523
    elements = 5,120 whole 8 KiB wire tiles (more than the launch's 4,096 workgroups, so workgroups
    loop over tiles and reuse their LDS) plus 3 elements one at a time; a second, 1-element-offset
    view takes the misaligned path. Bit-exact against torch's RNE casts (as the oracle's)."""
    import torch
    monkeypatch.setenv("TIPS_FUSION_THRESHOLD", "4096")
    n = 4096 * 5120 + 3
    g = torch.Generator(device="cuda").manual_seed(11)
    base = torch.randn(n + 1, device="cuda", generator=g) * 3
    tdt = torch.float16 if wire == "float16" else torch.bfloat16
    for view in (base[:n], base[1:]):
        want = view.to(tdt).float()
        (out,) = gpu.fused_allreduce_cast([view], wire)
        torch.cuda.synchronize()
        assert torch.equal(out.view(torch.int32), want.view(torch.int32))


def test_broadcast_allgather_checked_single_rank(gpu, monkeypatch):
    import torch
    from tips_amd import _lib, ops
    t = torch.randn(3, 5, device="cuda")
    assert torch.equal(gpu.broadcast_op(t, root_rank=0), t)
    h = np.arange(12, dtype=np.int64).reshape(3, 4)
    assert np.array_equal(gpu.broadcast_op(h), h)
    g = gpu.allgather_op(t)
    assert g.shape == (3, 5) and torch.equal(g, t)
    assert np.array_equal(gpu.allgather_op(h), h)
    v = [torch.zeros(4, device="cuda") + 2, np.ones(3, np.float32)]
    gpu.broadcast_variables(v, 0)
    assert torch.equal(v[0], torch.full((4,), 2.0, device="cuda"))
    with pytest.raises(gpu.TipsError):
        gpu.broadcast_op(t, root_rank=1)  # only rank 0 exists
    ops.set_consistency_check(True)
    try:
        assert torch.equal(gpu.allreduce(t), t)
        assert np.array_equal(gpu.allgather_op(h), h)
        s = torch.tensor(3.5, device="cuda")  # scalar -> shape [1] record
        assert gpu.allreduce(s).item() == 3.5
    finally:
        ops.set_consistency_check(False)
    rec = [_lib.REQ_ALLREDUCE, 0, 2, 3, 5] + [0] * 6
    assert ops._allgather_i64(rec) == rec


def test_allgatherv_counts_validation(gpu):
    import torch
    from tips_amd import _lib
    x = torch.arange(6, dtype=torch.float32, device="cuda")
    out = torch.empty(6, device="cuda")
    cp, _k = _lib.i64_array([5])
    assert _lib.lib().tips_allgatherv(x.data_ptr(), 6, out.data_ptr(), cp, 0, None) == -1  # counts[rank] != count
    assert b"not match" in _lib.lib().tips_last_error()


@pytest.mark.parametrize("piece", [4096, 1 << 20])
def test_host_pipeline_pieces(gpu, monkeypatch, piece):
    """Host buffers larger than a piece take the pipelined H2D || allreduce || D2H path."""
    import torch
    monkeypatch.setenv("TIPS_HOST_PIECE_BYTES", str(piece))
    rng = np.random.default_rng(5)
    for n in (1000003, 262144 + 7):
        h = rng.standard_normal(n).astype(np.float32)
        assert np.array_equal(gpu.allreduce(h), h)  # one rank: SUM = identity, every piece moved exactly
        pt = torch.from_numpy(h).pin_memory()
        assert torch.equal(gpu.allreduce(pt), pt)
        # both buffers page-locked: the single-thread issue path of host_staging.cc
        po = torch.empty_like(pt).pin_memory()
        from tips_amd import _lib
        _lib.call("tips_allreduce", pt.data_ptr(), po.data_ptr(), n, _lib.FLOAT32, _lib.OP_SUM, None)
        assert torch.equal(po, pt)
        # page-locked in, pageable out: the drain-thread path
        pg = np.empty_like(h)
        _lib.call("tips_allreduce", pt.data_ptr(), pg.ctypes.data, n, _lib.FLOAT32, _lib.OP_SUM, None)
        assert np.array_equal(pg, h)
        hi = rng.integers(-2**62, 2**62, size=n // 3, dtype=np.int64)
        assert np.array_equal(gpu.allreduce(hi), hi)


def test_torch_bootstrap_creates_rccl_comm_subprocess(gpu):
    """The N>1 bootstrap flow on one GPU, in a fresh process: torch.distributed (gloo) hands rank 0's
    ncclGetUniqueId to tips_init_rank -> ncclCommInitRank; then RCCL-backed work runs on that comm."""
    import subprocess
    import sys
    from conftest import REPO
    code = r'''
import os, numpy as np, torch, torch.distributed as dist
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533", TIPS_BOOTSTRAP="torch")
dist.init_process_group("gloo", rank=0, world_size=1)
import tips_amd
from tips_amd import _lib
tips_amd.init()
assert tips_amd.size() == 1 and tips_amd.rank() == 0
tips_amd.set_algorithm("rccl")
t = torch.randn(100003, device="cuda")
assert torch.equal(tips_amd.allreduce(t), t)
tips_amd.set_algorithm("auto")
import sys; sys.path.insert(0, "tests")
from gpu_util import simulate, F32
ins = [np.random.default_rng(r).standard_normal(5000).astype(np.float32) for r in range(4)]
import oracle_bind
out = simulate("ring", ins, F32, transport=1)
assert np.array_equal(out[0], oracle_bind.ring(ins)[0])
tips_amd.shutdown()
dist.destroy_process_group()
print("BOOTSTRAP_OK")
'''
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=REPO, timeout=600)
    assert "BOOTSTRAP_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


FUZZ = [np.random.default_rng(20261015 + i) for i in range(40)]


@pytest.mark.parametrize("case", range(40))
def test_schedule_fuzz(gpu, oracle, monkeypatch, case):
    """Random (schedule, p, n, dtype, in-place, transport, pipeline depth/sub-chunk) vs the oracle, bit-exact."""
    r = FUZZ[case]
    kind = ["ring", "direct", "oneshot"][int(r.integers(3))]
    p = int(r.integers(2, 13 if kind == "ring" else 17))
    n = int(r.choice([0, 1, 2, 63, 64, 65, 255, 4096, int(r.integers(1, 300000))]))
    dtype = int(r.choice(ALL_DTYPES))
    inplace = bool(r.integers(2))
    transport = int(r.integers(2))
    monkeypatch.setenv("TIPS_PIPELINE_DEPTH", str(int(r.integers(1, 7))))
    monkeypatch.setenv("TIPS_MIN_SUBCHUNK_BYTES", str(int(r.choice([256, 4096, 65536, 8 << 20]))))
    ins = [rand(dtype, n, r) for _ in range(p)]
    if n == 0:
        return
    exp = oracle.ring(ins, code=dtype)[0] if kind == "ring" else oracle.fold(ins, code=dtype, wide_acc=True)
    for got in simulate(kind, ins, dtype, inplace=inplace, transport=transport):
        assert same_bits(got, exp, dtype), (kind, p, n, dtype, inplace, transport)


@pytest.mark.slow
@pytest.mark.parametrize("kind", ["ring", "direct"])
def test_config3_full_size_8ranks(gpu, kind):
    """BASELINE config 3 at full size on one GPU: 8 virtual ranks x 1 GiB fp32, U[0.5,1.5), seeds 3000+r.
    Expected values are recomputed on the device with torch adds in the schedule's own order
    (ring: chunk c folded in[c], in[c+1] + acc, ...; direct: rank-order fold) -> bit-exact; plus every
    rank identical and <= 1e-6 relative to the float64 sum on a strided sample."""
    import ctypes
    import torch
    from tips_amd import _lib
    p, n = 8, 268435456
    g = torch.Generator(device="cuda")
    ins = []
    for r in range(p):
        g.manual_seed(3000 + r)
        ins.append(torch.empty(n, dtype=torch.float32, device="cuda").uniform_(0.5, 1.5, generator=g))
    outs = [torch.empty_like(x) for x in ins]
    pi, _k1 = _lib.ptr_array([x.data_ptr() for x in ins])
    po, _k2 = _lib.ptr_array([o.data_ptr() for o in outs])
    fn = "tips_ring_simulate" if kind == "ring" else "tips_direct_simulate"
    _lib.dev_call(fn, po, pi, p, n, F32, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    exp = torch.empty_like(ins[0])
    if kind == "ring":
        b, e = ctypes.c_int64(), ctypes.c_int64()
        for c in range(p):
            _lib.call("tips_chunk_bounds", n, p, F32, c, ctypes.byref(b), ctypes.byref(e))
            acc = ins[c][b.value:e.value].clone()
            for k in range(1, p):
                acc = ins[(c + k) % p][b.value:e.value] + acc
            exp[b.value:e.value] = acc
    else:
        exp.copy_(ins[0])
        for r in range(1, p):
            exp += ins[r]
    for o in outs:
        assert torch.equal(o, exp)
    idx = torch.arange(0, n, 9973, device="cuda")
    ref = sum(x[idx].double() for x in ins)
    assert ((outs[0][idx].double() - ref).abs() / ref).max().item() <= 1e-6


def test_registered_host_buffer(gpu, monkeypatch):
    monkeypatch.setenv("TIPS_HOST_PIECE_BYTES", str(1 << 20))
    h = np.random.default_rng(9).standard_normal(3_000_001).astype(np.float32)
    with gpu.registered_host_buffer(h):
        assert np.array_equal(gpu.allreduce(h), h)
    assert np.array_equal(gpu.allreduce(h), h)


def test_named_async_allreduce_single_rank(gpu):
    """The negotiated path (tips_enqueue_allreduce / tips_wait) end to end on one rank."""
    import torch
    ts = [torch.randn(1000 + 37 * i, device="cuda") for i in range(10)]
    hs = [gpu.allreduce_async(t, "grad.%d" % i) for i, t in enumerate(ts)]
    for h, t in zip(hs, ts):
        assert torch.equal(gpu.synchronize(h), t)
    # A name is reserved only until negotiation resolves it; a single rank can
    # resolve it before the second call, so the duplicate may or may not be
    # refused. A single enqueue is admitted to the tables after it returns (the
    # lock-free submission, round 5), so a refusal comes through its handle.
    h = gpu.allreduce_async(ts[0], "dup")
    try:
        h2 = gpu.allreduce_async(ts[1], "dup")
    except gpu.TipsError as e:
        assert "already pending" in str(e)
        h2 = None
    assert torch.equal(gpu.synchronize(h), ts[0])
    if h2 is not None:
        try:
            assert torch.equal(gpu.synchronize(h2), ts[1])
        except gpu.TipsError as e:
            assert "already pending" in str(e)
    hp = gpu.allreduce_async(ts[2], "polled")
    while not gpu.poll(hp):
        pass
    assert torch.equal(hp.output, ts[2])
    # host tensors go through the same negotiation (the reference's op is a CPU op); the handle
    # dropped unwaited stays safe: the module keeps its buffers until the request has run
    hh = gpu.allreduce_async(torch.full((3,), 2.0), "host")
    assert torch.equal(gpu.synchronize(hh), torch.full((3,), 2.0))
    gpu.allreduce_async(torch.zeros(5), "host_dropped")
    import numpy as np
    hn = gpu.allgather_async(np.arange(6, dtype=np.int64).reshape(3, 2), "host_ag")
    assert np.array_equal(gpu.synchronize(hn), np.arange(6, dtype=np.int64).reshape(3, 2))
    # the op functions with a name go through the negotiation (the reference's ops always do)
    assert torch.equal(gpu.allreduce_op(ts[3], name="layer/1:0"), ts[3])
    assert torch.equal(gpu.broadcast_op(ts[4], 0, name="bcast w"), ts[4])
    assert torch.equal(gpu.allgather_op(ts[5].view(-1, 1), name="ag"), ts[5].view(-1, 1))


def test_named_requests_from_threads_across_a_restart():
    """Executor threads keep a per-thread view of the negotiator (negotiate.cc cached(), refreshed
    by a generation counter) and push onto per-thread submission shards. The same three pool
    threads enqueue named host requests with callbacks (tips_enqueue_allreduce_cb) and device
    requests (allreduce_async) before a shutdown and after a new init; every result is its input,
    bit for bit, in both generations. A callback request's handle is a receipt: tips_wait refuses
    it. Enqueueing between the shutdown and the new init is refused, never hangs. (Its own
    process: it restarts the library.)"""
    import subprocess
    import sys
    from conftest import REPO
    code = r'''
import ctypes, threading, numpy as np, torch
from concurrent.futures import ThreadPoolExecutor
import tips_amd
from tips_amd import _lib
L = _lib.lib()
done, lock, ev = [], threading.Lock(), threading.Event()
@_lib.DONE_FN
def on_done(ctx, status, msg):
    with lock:
        done.append((ctx, status))
        if len(done) == want[0]:
            ev.set()
want = [0]
def host_job(gen, t):
    outs = []
    for i in range(30):
        x = np.random.default_rng(gen * 1000 + t * 100 + i).random(1000 + 17 * i, dtype=np.float32)
        y = np.empty_like(x)
        shape = (ctypes.c_int64 * 1)(x.size)
        h = L.tips_enqueue_allreduce_cb(("g%d.t%d.h%d" % (gen, t, i)).encode(), x.ctypes.data, y.ctypes.data,
                                        shape, 1, _lib.FLOAT32, None, on_done, None)
        assert h > 0, _lib.last_error()
        outs.append((x, y, h))
    return outs
def dev_job(gen, t):
    xs = [torch.randn(500 + 31 * i, device="cuda") for i in range(10)]
    hs = [tips_amd.allreduce_async(x, "g%d.t%d.d%d" % (gen, t, i)) for i, x in enumerate(xs)]
    return [(x, tips_amd.synchronize(h)) for x, h in zip(xs, hs)]
pool = ThreadPoolExecutor(3)
for gen in range(2):
    tips_amd.init()
    done.clear(); ev.clear(); want[0] = 90
    hosts = [f.result() for f in [pool.submit(host_job, gen, t) for t in range(3)]]
    devs = [f.result() for f in [pool.submit(dev_job, gen, t) for t in range(3)]]
    assert ev.wait(120), len(done)
    assert all(s == 0 for _, s in done)
    assert all(np.array_equal(x, y) for outs in hosts for x, y, _ in outs)
    assert all(torch.equal(x, y) for outs in devs for x, y in outs)
    assert L.tips_wait(hosts[0][0][2]) < 0 and "unknown request handle" in _lib.last_error()
    tips_amd.shutdown()
    x = np.ones(4, dtype=np.float32); shape = (ctypes.c_int64 * 1)(4)
    h = pool.submit(lambda: L.tips_enqueue_allreduce_cb(b"after.shutdown", x.ctypes.data, x.ctypes.data, shape, 1,
                                                        _lib.FLOAT32, None, on_done, None)).result(60)
    assert h < 0, h
print("RESTART_OK")
'''
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=REPO, timeout=300)
    assert "RESTART_OK" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]


def test_named_async_many_single_rank(gpu, monkeypatch):
    """allreduce_async_many / synchronize_many (tips_enqueue_allreduce_n / tips_wait_n): 500
    named tensors in one call, fused per readiness list (1 MiB threshold: some batches, some
    singles, some empty tensors); mixed dtypes in one call are refused."""
    import torch
    monkeypatch.setenv("TIPS_FUSION_THRESHOLD", str(1 << 20))
    rng = np.random.default_rng(3)
    ts = [torch.randn(int(rng.choice([0, 1, 33, 4099, 70000, 300000])), device="cuda") for _ in range(500)]
    hs = gpu.allreduce_async_many(ts, ["many.%d" % i for i in range(len(ts))])
    outs = gpu.synchronize_many(hs)
    for o, t in zip(outs, ts):
        assert torch.equal(o, t)
    with pytest.raises(ValueError):
        gpu.allreduce_async_many([ts[0], ts[1].double()], ["a", "b"])


def test_enqueue_n_classifies_each_pointer(gpu):
    """tips_enqueue_allreduce_n remembers the device allocations it has met within one call
    (negotiate.cc PtrRanges), so a list's later tensors skip the pointer queries. In one call:
    slices of one allocation, a tensor of another, a host pair after them (still host: host memory
    is never cached) and a device-in / host-out pair, refused as a single enqueue refuses it. At one
    rank every accepted result is its input, bit for bit."""
    import ctypes
    import torch
    from tips_amd import _lib
    L = _lib.lib()
    big = torch.randn(1 << 22, device="cuda")
    dev_in = [big[0:1000], big[5000:9000], torch.randn(777, device="cuda"), big[(1 << 21):(1 << 21) + 3]]
    dev_out = [torch.empty_like(t) for t in dev_in]
    h_in = np.random.default_rng(1).random(5000).astype(np.float32)
    h_out = np.empty_like(h_in)
    items = [(t.data_ptr(), o.data_ptr(), t.numel()) for t, o in zip(dev_in, dev_out)]
    items.insert(2, (h_in.ctypes.data, h_out.ctypes.data, h_in.size))
    items.append((big[100:200].data_ptr(), h_out.ctypes.data, 100))
    n = len(items)
    names = (ctypes.c_char_p * n)(*[("ptr_ranges.%d" % i).encode() for i in range(n)])
    ins, _k1 = _lib.ptr_array([a for a, _, _ in items])
    outs, _k2 = _lib.ptr_array([b for _, b, _ in items])
    cnt, _k3 = _lib.i64_array([c for _, _, c in items])
    hs = (ctypes.c_int64 * n)()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rc = L.tips_enqueue_allreduce_n(names, ins, outs, cnt, n, _lib.FLOAT32, stream, hs)
    assert rc < 0 and "one device and one host pointer" in _lib.last_error()
    assert hs[n - 1] < 0 and all(h > 0 for h in hs[:n - 1])
    assert L.tips_wait_n(hs, n - 1) == 0, _lib.last_error()
    torch.cuda.synchronize()
    for t, o in zip(dev_in, dev_out):
        assert torch.equal(t, o)
    assert np.array_equal(h_in, h_out)


def test_single_enqueue_classified_by_the_negotiation_thread(gpu):
    """A single named request is classified (device / host) on the negotiation thread, not in the
    enqueue (Req::classify): device, host and mixed requests enqueued back to back; the mixed one is
    announced as bad and fails through tips_wait with the reason, the others complete exactly."""
    import ctypes
    import torch
    from tips_amd import _lib
    L = _lib.lib()
    d_in = torch.randn(4099, device="cuda")
    d_out = torch.empty_like(d_in)
    h_in = np.random.default_rng(2).random(3001).astype(np.float32)
    h_out = np.empty_like(h_in)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    hd = L.tips_enqueue_allreduce(b"classify.dev", ctypes.c_void_p(d_in.data_ptr()), ctypes.c_void_p(d_out.data_ptr()),
                                  d_in.numel(), _lib.FLOAT32, stream)
    hm = L.tips_enqueue_allreduce(b"classify.mixed", ctypes.c_void_p(d_in.data_ptr()), h_out.ctypes.data_as(ctypes.c_void_p),
                                  100, _lib.FLOAT32, stream)
    hh = L.tips_enqueue_allreduce(b"classify.host", h_in.ctypes.data_as(ctypes.c_void_p), h_out.ctypes.data_as(ctypes.c_void_p),
                                  h_in.size, _lib.FLOAT32, stream)
    assert hd > 0 and hm > 0 and hh > 0, _lib.last_error()
    assert L.tips_wait(hm) < 0 and "one device and one host pointer on rank 0" in _lib.last_error()
    assert L.tips_wait(hd) == 0 and L.tips_wait(hh) == 0, _lib.last_error()
    torch.cuda.synchronize()
    assert torch.equal(d_out, d_in) and np.array_equal(h_out, h_in)


def test_sparse_allreduce_single_rank(gpu):
    """The reference's IndexedSlices branch (allgather of values and indices, __init__.py:59-74) through
    tips_allgatherv on one rank: device and host, IndexedSlices and torch sparse COO."""
    import torch
    vals = torch.randn(7, 4, device="cuda")
    idx = torch.tensor([3, 0, 3, 9, 1, 1, 2], device="cuda")
    s = gpu.allreduce(gpu.IndexedSlices(vals, idx, dense_shape=(10, 4)))
    assert torch.equal(s.values, vals) and torch.equal(s.indices, idx)
    a = gpu.allreduce(gpu.IndexedSlices(vals, idx, dense_shape=(10, 4)), op=gpu.Average)
    assert torch.equal(a.values, vals)  # size() == 1
    hv = np.arange(12, dtype=np.float64).reshape(6, 2)
    hs = gpu.allreduce(gpu.IndexedSlices(hv, np.arange(6), dense_shape=(6, 2)))
    assert np.array_equal(hs.values, hv)
    for dev in ("cuda", "cpu"):
        dense = torch.zeros(50, 3, device=dev)
        dense[[3, 17, 40], 1] = torch.tensor([1.0, -2.0, 0.5], device=dev)
        out = gpu.allreduce(dense.to_sparse())
        assert out.is_sparse and torch.equal(out.to_dense(), dense)


@pytest.mark.parametrize("n", [1, 1000, 65535, 65536, 65537, 300000])
def test_host_bounce_boundary(gpu, n):
    """Host tensors on either side of the 256 KiB page-locked bounce threshold (rt.h run_staged):
    pageable in and out, in place, one side page-locked, and the broadcast host path; at one rank
    every result is the input, bit for bit."""
    import torch
    from tips_amd import _lib
    h = np.random.default_rng(n).random(n).astype(np.float32)
    out = np.full_like(h, -1.0)
    _lib.call("tips_allreduce", h.ctypes.data, out.ctypes.data, n, _lib.FLOAT32, _lib.OP_SUM, None)
    assert np.array_equal(out, h)
    g = h.copy()
    _lib.call("tips_allreduce", g.ctypes.data, g.ctypes.data, n, _lib.FLOAT32, _lib.OP_SUM, None)
    assert np.array_equal(g, h)
    pin = torch.from_numpy(h).pin_memory()
    out2 = np.full_like(h, -1.0)
    _lib.call("tips_allreduce", pin.data_ptr(), out2.ctypes.data, n, _lib.FLOAT32, _lib.OP_SUM, None)
    assert np.array_equal(out2, h)
    pout = torch.full((n,), -1.0).pin_memory()
    _lib.call("tips_allreduce", h.ctypes.data, pout.data_ptr(), n, _lib.FLOAT32, _lib.OP_SUM, None)
    assert np.array_equal(pout.numpy(), h)
    out3 = np.full_like(h, -1.0)
    _lib.call("tips_broadcast", h.ctypes.data, out3.ctypes.data, n, _lib.FLOAT32, 0, None)
    assert np.array_equal(out3, h)


@pytest.mark.parametrize("measure_pack", ["1", "0"])
@pytest.mark.parametrize("workload", ["config4", "config5"])
def test_fusion_workloads_single_rank(gpu, monkeypatch, workload, measure_pack):
    """Configs 4 and 5's tensor lists through the fusion path on one rank (pack -> bucket ->
    unpack moves every byte: the identity), in place and out of place, twice (the second call hits
    the descriptor cache); allreduce_grads and DistributedOptimizer.step() are the identity at one
    rank, as the reference's _allreduce_cond (__init__.py:94-103)."""
    import sys
    import torch
    from conftest import REPO
    sys.path.insert(0, REPO)
    import bench
    monkeypatch.setenv("TIPS_FUSION_MEASURE_PACK", measure_pack)
    sizes = bench.fused1000_sizes() if workload == "config4" else bench.resnet50_grad_sizes()
    flat = torch.randn(sum(sizes), device="cuda")
    views = list(torch.split(flat, sizes))
    ref = flat.clone()
    for _ in range(2):
        outs = gpu.fused_allreduce(views)
        torch.cuda.synchronize()
        assert torch.equal(torch.cat(outs), ref) and torch.equal(flat, ref)
        gpu.fused_allreduce_(views)
        torch.cuda.synchronize()
        assert torch.equal(flat, ref)
    assert all(a is b for a, b in zip(gpu.allreduce_grads(views), views))
    params = [torch.nn.Parameter(torch.zeros(k, device="cuda")) for k in sizes[:50]]
    for p, v in zip(params, views):
        p.grad = v.clone()
    gpu.DistributedOptimizer(torch.optim.SGD(params, lr=1.0)).step()
    assert all(torch.equal(0.0 - p.detach(), v) for p, v in zip(params, views))


def test_fusion_concurrent_streams(gpu, monkeypatch):
    """Fused calls and negotiated batches issued from two torch streams at once, with distinct data,
    share the library's fusion slots: every output must still be bit-exact (at one rank, the
    input). A 1 MiB threshold makes every call span several buckets, so a call that packed or
    unpacked another call's slot would show."""
    import torch
    monkeypatch.setenv("TIPS_FUSION_THRESHOLD", str(1 << 20))
    monkeypatch.setenv("TIPS_FUSION_MEASURE_PACK", "1")  # one rank still packs into the shared slots
    rng = np.random.default_rng(8)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    lists = []
    for k in range(6):
        sizes = [int(x) for x in rng.integers(1, 200000, size=20)]
        lists.append([torch.full((n,), float(100 * k + i), device="cuda") for i, n in enumerate(sizes)])
    expect = [[t.clone() for t in lst] for lst in lists]
    torch.cuda.synchronize()
    outs, handles = [], []
    for rep in range(3):
        for k, lst in enumerate(lists):
            with torch.cuda.stream(s1 if k % 2 == 0 else s2):
                if k % 3 == 0:
                    outs.append((expect[k], gpu.fused_allreduce(lst)))
                elif k % 3 == 1:
                    gpu.fused_allreduce_(lst)
                    outs.append((expect[k], lst))
                else:
                    names = ["c%d.%d.%d" % (rep, k, i) for i in range(len(lst))]
                    handles.append((expect[k], gpu.allreduce_async_many(lst, names)))
    for exp, hs in handles:
        outs.append((exp, gpu.synchronize_many(hs)))
    torch.cuda.synchronize()
    for exp, got in outs:
        for e, o in zip(exp, got):
            assert torch.equal(o, e)
