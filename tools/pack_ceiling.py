"""pack_ceiling.py — how close can a ~40-50 MiB copy launch get to HBM peak on this box?

The fusion pack kernel (copy_segs_kernel) moves one bucket per launch: 39.5 MiB (config 4) or
~46-52 MiB (config 5). This probe separates what the segment logic costs from what the launch
size costs, all with HIP events on one stream, 4 rotating source sets (HBM-only), launches queued
behind a spin so they run back to back, median of interleaved rounds:
  pack      tips_fused_pack_bucket over the config's own layout, one launch per bucket (what bench.py reports)
  merged    every bucket of the step in one launch (TIPS_PACK_MERGE=1, opt-in since round 6)
  contig    the same kernel on a list of ONE tensor of the bucket's byte count (every tile on the
            one-segment fast path: no segment search, no ragged ends)
  memcpy    hipMemcpyAsync D2D of the same bytes (the copy engine path torch uses for copy_)
  span_us   (launches of one bucket) one event pair around each launch instead of one pair around
            20 back-to-back launches: the launch's own span, without the boundary to the next
  sizes     `contig` at 10-640 MiB, fitted to t = t0 + bytes / BW: t0 is the per-launch ramp and
            drain, BW the streaming rate; frac(S) = 2S / t(S) / 8 TB/s
One JSON line per measurement to stdout.

usage: python3 tools/pack_ceiling.py [rounds] [--only=CASE_PREFIX ...]
       TIPS_FUSION_THRESHOLD=2147483648 python3 tools/pack_ceiling.py [rounds]   (the size series only, to 640 MiB)
"""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK = 8000.0  # GB/s
ONLY = [a[len("--only="):] for a in sys.argv[1:] if a.startswith("--only=")]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--only=")]
    rounds = int(args[0]) if args else 7
    import torch

    import bench
    import tips_amd
    from tips_amd import _lib
    L = _lib.lib()
    torch.cuda.set_device(0)
    tips_amd.init()
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    thr = 64 << 20
    dst = torch.empty(2 * thr // 4, dtype=torch.float32, device="cuda")
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]

    def timed(fn, reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(12_000_000)
        e0.record(stream)
        for k in range(reps):
            fn(k)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    def spans(fn, reps):
        """one event pair around each call, all queued behind the gate: the calls' own spans,
        without the boundary between one launch and the next"""
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
        torch.cuda._sleep(12_000_000)
        for k in range(reps):
            ev[2 * k].record(stream)
            fn(k)
            ev[2 * k + 1].record(stream)
        torch.cuda.synchronize()
        return sum(ev[2 * k].elapsed_time(ev[2 * k + 1]) for k in range(reps)) * 1e3 / reps

    only = ONLY

    def want(name):
        return not only or any(name.startswith(o) for o in only)

    cases = {}
    sizes_only = os.environ.get("TIPS_FUSION_THRESHOLD") is not None  # (the configs' layouts would change)
    workloads = () if sizes_only else (("config4", bench.fused1000_sizes()), ("config5", bench.resnet50_grad_sizes()))
    for wname, sizes in workloads:
        if only and not any(o.startswith(wname + "/") or wname.startswith(o) for o in only):
            continue
        sets = [[torch.randn(n, device="cuda") for n in sizes] for _ in range(4)]
        ptrs = [_lib.ptr_array([t.data_ptr() for t in s]) for s in sets]
        cp, _kc = _lib.i64_array(sizes)
        nb = int(_lib.check("tips_fused_pack_bucket", L.tips_fused_pack_bucket(ptrs[0][0], cp, len(sizes), _lib.FLOAT32,
                                                                              -1, None, None)))
        payload = []
        for b in range(nb):
            rc = L.tips_fused_pack_bucket(ptrs[0][0], cp, len(sizes), _lib.FLOAT32, b, dst.data_ptr(), sp)
            payload.append(int(rc))
        torch.cuda.synchronize()

        def pack(k, ptrs=ptrs, cp=cp, n=len(sizes), nb=nb):
            for b in range(nb):
                rc = L.tips_fused_pack_bucket(ptrs[k % 4][0], cp, n, _lib.FLOAT32, b, dst.data_ptr(), sp)
                if rc < 0:
                    raise _lib.TipsError("tips_fused_pack_bucket", int(rc), _lib.last_error())
        cases[wname + "/pack"] = (pack, nb, sum(payload) / nb)
        if want(wname + "/merged"):
            # the step's packs as fusion.cc issues them since round 6: every bucket in ONE launch
            # (copy_segs_groups_kernel), through tips_fused_allreduce_flat at one rank with
            # TIPS_FUSION_MEASURE_PACK=1 (pack into the flat buffer, the identity allreduce skipped)
            os.environ["TIPS_FUSION_MEASURE_PACK"] = "1"
            os.environ["TIPS_PACK_MERGE"] = "1"
            fb = int(_lib.check("tips_fused_layout", L.tips_fused_layout(cp, len(sizes), _lib.FLOAT32, None)))
            flat = torch.empty(fb // 4 + 64, dtype=torch.float32, device="cuda")

            def merged(k, ptrs=ptrs, cp=cp, n=len(sizes), flat=flat):
                rc = L.tips_fused_allreduce_flat(ptrs[k % 4][0], cp, n, _lib.FLOAT32, flat.data_ptr(), sp)
                if rc < 0:
                    raise _lib.TipsError("tips_fused_allreduce_flat", int(rc), _lib.last_error())
            merged(0)
            cases[wname + "/merged"] = (merged, 1, sum(payload))
        for b, pb in enumerate(payload):
            if not want("%s/contig_b%d" % (wname, b)) and not want("%s/memcpy_b%d" % (wname, b)):
                continue
            n1 = pb // 4
            one = [torch.randn(n1, device="cuda") for _ in range(4)]
            op = [_lib.ptr_array([t.data_ptr()]) for t in one]
            oc, _ko = _lib.i64_array([n1])
            L.tips_fused_pack_bucket(op[0][0], oc, 1, _lib.FLOAT32, 0, dst.data_ptr(), sp)

            def contig(k, op=op, oc=oc, one=one):
                L.tips_fused_pack_bucket(op[k % 4][0], oc, 1, _lib.FLOAT32, 0, dst.data_ptr(), sp)

            def memcpy(k, one=one, nbytes=n1 * 4):
                hip.hipMemcpyAsync(dst.data_ptr(), one[k % 4].data_ptr(), nbytes, 3, sp)
            cases["%s/contig_b%d" % (wname, b)] = (contig, 1, pb)
            cases["%s/memcpy_b%d" % (wname, b)] = (memcpy, 1, pb)
    for mib in (10, 20, 40, 80, 160, 320, 640):
        if not want("size/contig_%dMiB" % mib):
            continue
        n1 = (mib << 20) // 4
        one = [torch.randn(n1, device="cuda") for _ in range(4)]
        big = torch.empty(n1, device="cuda")
        op = [_lib.ptr_array([t.data_ptr()]) for t in one]
        oc, _ko = _lib.i64_array([n1])
        if n1 * 4 >= thr and not sizes_only:
            continue  # (a tensor of at least the threshold is not packed: run with TIPS_FUSION_THRESHOLD=2147483648)

        def contig(k, op=op, oc=oc, big=big):
            L.tips_fused_pack_bucket(op[k % 4][0], oc, 1, _lib.FLOAT32, 0, big.data_ptr(), sp)
        contig(0)
        cases["size/contig_%dMiB" % mib] = (contig, 1, n1 * 4)
    if only:  # (PMC passes: only the named cases' launches)
        cases = {k: v for k, v in cases.items() if any(k.startswith(o) for o in only)}
    torch.cuda.synchronize()
    res = {k: [] for k in cases}
    spn = {k: [] for k in cases}
    for r in range(rounds):
        for k, (fn, per, _b) in cases.items():
            res[k].append(timed(fn, 20) / per)
            if per == 1:
                spn[k].append(spans(fn, 20))
    fit = []
    for k, (fn, per, b) in cases.items():
        us = statistics.median(res[k])
        gbs = 2 * b / (us * 1e-6) / 1e9
        if k.startswith("size/"):
            fit.append((2 * b, us))
        print(json.dumps({"case": k, "bytes_per_launch": int(b), "us_per_launch": round(us, 2),
                          "GBps": round(gbs, 1), "frac": round(gbs / PEAK, 4),
                          "spread_us": [round(min(res[k]), 2), round(max(res[k]), 2)],
                          "span_us": round(statistics.median(spn[k]), 2) if spn[k] else None}), flush=True)
    if len(fit) >= 2:
        n = len(fit)
        mx = sum(x for x, _ in fit) / n
        my = sum(y for _, y in fit) / n
        sl = sum((x - mx) * (y - my) for x, y in fit) / sum((x - mx) ** 2 for x, _ in fit)
        t0 = my - sl * mx
        print(json.dumps({"fit": "t_us = t0 + moved_bytes / BW", "t0_us": round(t0, 2),
                          "BW_GBps": round(1e-3 / sl, 1), "points": len(fit)}), flush=True)


if __name__ == "__main__":
    main()
