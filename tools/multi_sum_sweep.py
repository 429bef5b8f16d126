"""Round-5 sweep of the direct schedule's fold (tips_multi_sum_variant, f32) at config 3's shapes,
HBM-only, variants interleaved over rounds (median). Two source placements:
  sep   - every source its own allocation, 4 rotating sets (round 2's tools/multi_sum_rate.py);
  slots - (slots:<pad> for another pad; slotsep: each slot its own allocation) the direct plan's own layout (plan.cc direct()): the rank's input slice + p-1 staging slots
          one chunk + 4 KiB apart, the launch of sub-chunk k reading offset k of each (k = i % 4 over
          a chunk of 4 sub-chunks), so consecutive launches rotate over 4 x (p + 1) sub-chunk buffers.
One JSON line per (placement, p, MiB, variant): median us, TB/s, fraction of 8 TB/s, bit-exact."""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from tips_amd import _lib  # noqa: E402

L = _lib.dev()
torch.cuda.set_device(0)
s = torch.cuda.current_stream()
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "1,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22").split(",")]
SHAPES = [tuple(int(x) for x in sh.split("x")) for sh in os.environ.get("SHAPES", "8x32").split(",")]
PLACES = os.environ.get("PLACES", "slots,sep").split(",")
ROUNDS = int(os.environ.get("ROUNDS", "5"))
LAUNCHES = 20


def sets_sep(p, n):
    out = []
    for k in range(4):
        srcs = [torch.empty(n, device="cuda").uniform_(-1, 1) for _ in range(p)]
        dst = torch.empty(n, device="cuda")
        out.append((srcs, dst))
    return out, None


def sets_slots(p, n, pad=4096, separate=False):
    chunk = 4 * n
    stride = chunk + pad // 4
    inp = torch.empty(p * chunk, device="cuda").uniform_(-1, 1)
    if separate:  # every staging slot its own allocation
        stg = [torch.empty(stride, device="cuda").uniform_(-1, 1) for _ in range(p - 1)]
    else:
        stg = torch.empty((p - 1) * stride, device="cuda").uniform_(-1, 1)
    out = torch.empty(p * chunk, device="cuda")
    r = p // 2  # this rank's chunk
    res = []
    for k in range(4):
        srcs = []
        for j in range(p):
            if j == r:
                srcs.append(inp[r * chunk + k * n: r * chunk + (k + 1) * n])
            else:
                sl = j if j < r else j - 1
                srcs.append(stg[sl][k * n:(k + 1) * n] if separate else stg[sl * stride + k * n: sl * stride + (k + 1) * n])
        res.append((srcs, out[r * chunk + k * n: r * chunk + (k + 1) * n]))
    return res, (inp, stg, out)


for place in PLACES:
    for p, mib in SHAPES:
        n = mib * (1 << 18)
        if place.startswith("slots"):  # "slots" (the plan's 4 KiB pad), "slots:<pad bytes>", "slotsep" (separate)
            sets, keep = sets_slots(p, n, int(place.split(":")[1]) if ":" in place else 4096, place.startswith("slotsep"))
        else:
            sets, keep = sets_sep(p, n)
        ptrs = [_lib.ptr_array([t.data_ptr() for t in srcs]) for srcs, _ in sets]
        res = {v: [] for v in VARIANTS}
        ok = {}
        for rnd in range(ROUNDS):
            for v in VARIANTS:
                if res[v] is None:
                    continue
                rc = 0
                for i in range(4):
                    rc = rc or L.tips_multi_sum_variant(sets[i][1].data_ptr(), ptrs[i][0], p, n, _lib.FLOAT32, v,
                                                        s.cuda_stream)
                if rc:
                    res[v] = None
                    continue
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for i in range(LAUNCHES):
                    L.tips_multi_sum_variant(sets[i % 4][1].data_ptr(), ptrs[i % 4][0], p, n, _lib.FLOAT32, v,
                                             s.cuda_stream)
                e1.record(s)
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) / LAUNCHES * 1e3)
                if rnd == 0:
                    srcs, dst = sets[(LAUNCHES - 1) % 4]
                    ref = srcs[0].clone()
                    for t in srcs[1:]:
                        ref += t
                    ok[v] = bool(torch.equal(dst, ref))
        for v in VARIANTS:
            if res[v]:
                us = sorted(res[v])[len(res[v]) // 2]
                tb = (p + 1) * n * 4 / us / 1e6
                print(json.dumps({"place": place, "p": p, "MiB": mib, "variant": v, "median_us": round(us, 2),
                                  "min_us": round(min(res[v]), 2), "TBps": round(tb, 3), "frac": round(tb / 8.0, 4),
                                  "bit_exact": ok.get(v)}), flush=True)
            else:
                print(json.dumps({"place": place, "p": p, "MiB": mib, "variant": v, "error": "launch failed"}),
                      flush=True)
        del sets, keep, ptrs
        torch.cuda.empty_cache()
