"""CPU: the fusion pack / unpack tables against copy_segs_kernel's rules, without a GPU.

tips_fusion_tile_table returns the records fusion.cc builds for one pointer set (the same code
that fills the device table). `run_table` below applies copy_segs_kernel's per-workgroup and
per-lane rules (tips_amd/csrc/kernels.hip) to them - the tile's byte offset from its second record,
the one-tensor fast path, the two-record select, the LDS segment list with its binary search, and
the per-vector length at a tensor's ragged end - and collects the byte ranges each launch copies.
For random lists (ragged sizes, empty tensors, tensors past the threshold, 4-B aligned tensors,
several buckets) every input byte must land at its output address exactly once and nothing else
may be written, for each tile size and for both launch orders (TIPS_COPY_ORDER: tile order, and a
group's boundary tiles first)."""
import ctypes
import os
import random

import pytest

VEC = 16
LANES = 256


def table(counts, ins, outs, dtype):
    from tips_amd import _lib
    L = _lib.dev()
    n = len(counts)
    c = (ctypes.c_int64 * n)(*counts)
    pi = (ctypes.c_int64 * n)(*ins)
    po = (ctypes.c_int64 * n)(*outs)
    nt, tb = ctypes.c_int64(), ctypes.c_int64()
    nrec = L.tips_fusion_tile_table(c, n, dtype, pi, po, None, 0, ctypes.byref(nt), ctypes.byref(tb))
    assert nrec >= 0, _lib.last_error()
    rec = (ctypes.c_int64 * (4 * nrec))()
    assert L.tips_fusion_tile_table(c, n, dtype, pi, po, rec, nrec, ctypes.byref(nt), ctypes.byref(tb)) == nrec
    r = [tuple(rec[4 * k:4 * k + 4]) for k in range(nrec)]
    return r, nt.value, tb.value


def run_table(rec, ntiles, T):
    """[(dst, src, length)] copied by one launch over all tiles, per copy_segs_kernel."""
    U = T // (LANES * VEC)
    max_seg = T // 256 + 1
    out = []
    for q in range(ntiles):
        a, b = rec[2 * q], rec[2 * q + 1]
        multi, two = a[3] < 0, b[3] > 0
        tb = (b[2] & ~(T - 1)) if two else b[2]
        if not multi and not two and a[2] <= tb and a[3] >= tb + T and ((a[0] | a[1]) & 15) == 0:
            out.append((a[1] + tb, a[0] + tb, T))
            continue
        segs = None
        if multi:
            cnt = min(a[1], max_seg)
            if cnt <= 0:
                continue
            segs = rec[2 * ntiles + a[0]:2 * ntiles + a[0] + cnt]
        for u in range(U):
            for tid in range(LANES):
                v = tb + u * LANES * VEC + tid * VEC
                if multi:
                    lo, hi = 0, len(segs) - 1
                    while lo < hi:
                        mid = (lo + hi + 1) >> 1
                        if segs[mid][2] <= v:
                            lo = mid
                        else:
                            hi = mid - 1
                    g = segs[lo]
                else:
                    g = b if (two and v >= b[2]) else a
                left = g[3] - v
                ln = min(left, VEC) if (v >= g[2] and left > 0) else 0
                if ln:
                    out.append((g[1] + v, g[0] + v, ln))
    return out


def check(counts, ins, outs, es, copies):
    """every byte of tensor i copied from ins[i] + k to outs[i] + k exactly once; nothing else"""
    want = sorted((o, i, c * es) for i, (o, c) in enumerate(zip(outs, counts)) if c > 0)
    got = sorted(copies)
    # merge the copied ranges per tensor, in destination order
    k = 0
    for dst0, i, nbytes in want:
        pos = dst0
        while pos < dst0 + nbytes:
            assert k < len(got), "tensor %d: bytes from %d not copied" % (i, pos - dst0)
            d, s, ln = got[k]
            assert d == pos, "tensor %d: expected a copy to +%d, next copy is to %d" % (i, pos - dst0, d - dst0)
            assert s - d == ins[i] - outs[i], "tensor %d: wrong source at +%d" % (i, pos - dst0)
            pos += ln
            k += 1
        assert pos == dst0 + nbytes, "tensor %d: copied past its end" % i
    assert k == len(got), "%d copies outside every tensor" % (len(got) - k)


def random_list(rng, n, es, threshold):
    counts = []
    for _ in range(n):
        r = rng.random()
        if r < 0.08:
            counts.append(0)
        elif r < 0.12:
            counts.append((threshold + rng.randrange(1, 4096)) // es)  # reduced where it lies
        elif r < 0.5:
            counts.append(rng.randrange(1, 300))
        else:
            counts.append(rng.randrange(1, 12000))
    # distinct, non-overlapping addresses: mostly 256-B aligned, some only 4-B aligned
    ins, outs = [], []
    nxt = 1 << 32
    for c in counts:
        for lst in (ins, outs):
            al = 4 if rng.random() < 0.15 else 256
            nxt = (nxt + 4095) // 4096 * 4096 + rng.randrange(0, 4096 // al) * al
            lst.append(nxt)
            nxt += c * es + 8192
    return counts, ins, outs


@pytest.mark.parametrize("tile", [4096, 8192, 16384])
@pytest.mark.parametrize("order", ["0", "1"])
def test_tables_copy_every_byte_once(monkeypatch, tile, order):
    from tips_amd import _lib
    threshold = 96 << 10  # several buckets from a short list
    monkeypatch.setenv("TIPS_FUSION_THRESHOLD", str(threshold))
    monkeypatch.setenv("TIPS_COPY_TILE_BYTES", str(tile))
    monkeypatch.setenv("TIPS_COPY_ORDER", order)
    rng = random.Random(tile * 7 + int(order))
    for dtype, es in ((_lib.FLOAT32, 4), (_lib.FLOAT16, 2), (_lib.FLOAT64, 8)):
        counts, ins, outs = random_list(rng, 40, es, threshold)
        rec, ntiles, T = table(counts, ins, outs, dtype)
        assert T == tile
        check(counts, ins, outs, es, run_table(rec, ntiles, T))


def test_boundary_tiles_come_first_in_each_group(monkeypatch):
    """TIPS_COPY_ORDER=1 (the default): within each bucket the tiles that meet a tensor boundary
    occupy the first record slots, the tiles inside one tensor the rest; the set of tiles per
    bucket is unchanged (the tile offsets in the records are a permutation of the bucket's)."""
    from tips_amd import _lib
    monkeypatch.setenv("TIPS_FUSION_THRESHOLD", str(96 << 10))
    monkeypatch.delenv("TIPS_COPY_ORDER", raising=False)
    rng = random.Random(5)
    counts, ins, outs = random_list(rng, 60, 4, 96 << 10)
    ins = [x // 256 * 256 for x in ins]
    outs = [x // 256 * 256 for x in outs]
    rec, ntiles, T = table(counts, ins, outs, _lib.FLOAT32)
    offs = []
    slow = []
    for q in range(ntiles):
        a, b = rec[2 * q], rec[2 * q + 1]
        two = b[3] > 0
        tb = (b[2] & ~(T - 1)) if two else b[2]
        offs.append(tb)
        slow.append(a[3] < 0 or two or not (a[2] <= tb and a[3] >= tb + T))
    assert sorted(offs) == [q * T for q in range(ntiles)]
    monkeypatch.setenv("TIPS_COPY_ORDER", "0")
    rec0, _, _ = table(counts, ins, outs, _lib.FLOAT32)
    base = [(rec0[2 * q + 1][2] & ~(T - 1)) if rec0[2 * q + 1][3] > 0 else rec0[2 * q + 1][2] for q in range(ntiles)]
    assert base == [q * T for q in range(ntiles)]
    # boundary-first within each run of slots holding one bucket's tiles: once a fast tile is seen,
    # no slow tile of the same bucket follows (buckets are the contiguous tile ranges of tips_fused_layout)
    assert any(slow) and not all(slow)
    assert slow[0]


def _striped_tables_child():
    """(run in a child process: TIPS_PACK_STRIPE_KIB is read once per process)"""
    from tips_amd import _lib
    threshold = 1 << 20
    os.environ["TIPS_FUSION_THRESHOLD"] = str(threshold)
    rng = random.Random(11)
    for dtype, es in ((_lib.FLOAT32, 4), (_lib.FLOAT16, 2)):
        counts, ins, outs = random_list(rng, 160, es, threshold)
        rec, ntiles, T = table(counts, ins, outs, dtype)
        check(counts, ins, outs, es, run_table(rec, ntiles, T))
    print("striped tables ok")


@pytest.mark.parametrize("stripe_kib", ["16", "64"])
def test_striped_pack_tables_copy_every_byte_once(stripe_kib):
    """TIPS_PACK_STRIPE_KIB (opt-in): the pack launch deals stripes of slots round-robin over the
    XCDs and fusion.cc's tile_order places each XCD's boundary tiles by that map. The records stay
    a permutation of the layout's tiles: every byte copied exactly once (stripes small enough that
    1 MiB buckets hold several rounds of 8)."""
    import subprocess
    import sys
    env = dict(os.environ, TIPS_PACK_STRIPE_KIB=stripe_kib)
    here = os.path.dirname(os.path.abspath(__file__))
    code = "import sys; sys.path[:0] = [%r, %r]; import test_fusion_table as t; t._striped_tables_child()" % (
        os.path.dirname(here), here)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "striped tables ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
