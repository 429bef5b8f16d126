"""HBM-only sweep of the fold kernel's variants (tips_multi_sum_variant, f32) at the direct
schedule's shapes, rotating buffer sets, rounds interleaved. One JSON line per (p, MiB, variant)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from tips_amd import _lib  # noqa: E402

L = _lib.dev()  # (the tuning sweep entry points: include/tips_hip_dev.h)
torch.cuda.set_device(0)
s = torch.cuda.current_stream()
import os
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "0,1,2,3,4,5,6,7").split(",")]
SHAPES = [tuple(int(x) for x in sh.split("x")) for sh in os.environ.get("SHAPES", "8x32,8x8,4x64").split(",")]
for p, mib in SHAPES:
    n = mib * (1 << 18)
    sets = []
    for k in range(4):
        srcs = [torch.randn(n, device="cuda") for _ in range(p)]
        dst = torch.empty(n, device="cuda")
        ptrs, keep = _lib.ptr_array([t.data_ptr() for t in srcs])
        sets.append((srcs, dst, ptrs, keep))
    res = {v: [] for v in VARIANTS}
    ok = {}
    for rnd in range(5):
        for v in VARIANTS:
            rc = 0
            for i in range(4):
                srcs, dst, ptrs, _ = sets[i % 4]
                rc = rc or L.tips_multi_sum_variant(dst.data_ptr(), ptrs, p, n, _lib.FLOAT32, v, s.cuda_stream)
            if rc:
                res[v] = None
                continue
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for i in range(20):
                srcs, dst, ptrs, _ = sets[i % 4]
                L.tips_multi_sum_variant(dst.data_ptr(), ptrs, p, n, _lib.FLOAT32, v, s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            if res[v] is not None:
                res[v].append(e0.elapsed_time(e1) / 20 * 1e3)
            if rnd == 0:
                srcs, dst, _, _ = sets[3]
                ref = srcs[0].clone()
                for t in srcs[1:]:
                    ref += t
                ok[v] = bool(torch.equal(dst, ref))
    for v in VARIANTS:
        if res[v]:
            us = sorted(res[v])[len(res[v]) // 2]
            print(json.dumps({"p": p, "MiB": mib, "variant": v, "median_us": round(us, 2),
                              "TBps": round((p + 1) * n * 4 / us / 1e6, 3), "bit_exact": ok.get(v)}), flush=True)
    del sets
    torch.cuda.empty_cache()
