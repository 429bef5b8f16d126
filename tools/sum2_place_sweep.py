"""Why 2 x 128 MiB sums slower than 2 x 64 or 2 x 256 MiB (tools/sum2_size_sweep.py: 0.77 against
0.84 / 0.82 of HBM, every launch shape): operand size and placement. The shipped tips_bucket_sum on
four rotating operand triples, each triple either three torch allocations ("sep") or three slices
of one allocation PAD bytes apart ("pad<k>"), at several operand sizes; best of ROUNDS interleaved
rounds. One JSON line per (size, layout)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tips_amd import _lib  # noqa: E402

L = _lib.lib()
torch.cuda.set_device(0)
s = torch.cuda.current_stream()
SIZES = [int(x) for x in os.environ.get("SIZES_MIB", "96,112,120,128,136,144,160").split(",")]
PADS = [int(x) for x in os.environ.get("PADS", "-1,0,4096,65536,2101248,16777216").split(",")]  # -1 = separate
ROUNDS = int(os.environ.get("ROUNDS", "3"))


def triple(n, pad):
    if pad < 0:
        return [torch.randn(n, device="cuda") for _ in range(3)], None
    per = n + pad // 4
    big = torch.randn(3 * per, device="cuda")
    return [big[k * per:k * per + n] for k in range(3)], big


for mib in SIZES:
    n = mib << 18
    best = {}
    for rnd in range(ROUNDS):
        for pad in (PADS if rnd % 2 == 0 else PADS[::-1]):
            sets = [triple(n, pad) for _ in range(4)]

            def launch(i):
                (a, b, c), _ = sets[i % 4]
                _lib.call("tips_bucket_sum", c.data_ptr(), a.data_ptr(), b.data_ptr(), n, _lib.FLOAT32, s.cuda_stream)
            for i in range(8):
                launch(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            K = 40
            e0.record(s)
            for i in range(K):
                launch(i)
            e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / K * 1e3
            best[pad] = min(us, best.get(pad, us))
            del sets
            torch.cuda.empty_cache()
    for pad in PADS:
        us = best[pad]
        print(json.dumps({"operand_MiB": mib, "layout": "sep" if pad < 0 else "pad%d" % pad,
                          "us_per_launch": round(us, 2), "frac_of_8TBps": round(3 * n * 4 / us / 1e6 / 8.0, 4)}),
              flush=True)
