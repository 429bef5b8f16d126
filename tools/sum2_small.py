"""HBM-only rate of the ring step's sum (dst = a + b, tips_sum_variant mode 3 = the shipped
buffer-op kernel) at ring sub-chunk sizes, 1 / 2 / 4 vectors per lane, rotating buffer sets,
rounds interleaved. One JSON line per (MiB, unroll)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from tips_amd import _lib  # noqa: E402

L = _lib.dev()  # (the tuning sweep entry points: include/tips_hip_dev.h)
torch.cuda.set_device(0)
s = torch.cuda.current_stream()
for mib in (1, 2, 4, 8, 16, 32):
    n = mib * (1 << 18)
    sets = [(torch.randn(n, device="cuda"), torch.randn(n, device="cuda"), torch.empty(n, device="cuda")) for _ in range(8)]
    res = {u: [] for u in (1, 2, 4)}
    for rnd in range(5):
        for u in (1, 2, 4):
            for i in range(8):
                a, b, c = sets[i]
                assert L.tips_sum_variant(c.data_ptr(), a.data_ptr(), b.data_ptr(), n, 0, 3, u, 1, 0, 256, s.cuda_stream) == 0
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for i in range(40):
                a, b, c = sets[i % 8]
                L.tips_sum_variant(c.data_ptr(), a.data_ptr(), b.data_ptr(), n, 0, 3, u, 1, 0, 256, s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            res[u].append(e0.elapsed_time(e1) / 40 * 1e3)
    ok = all(bool(torch.equal(c, a + b)) for a, b, c in sets)
    for u, v in res.items():
        us = sorted(v)[len(v) // 2]
        print(json.dumps({"MiB": mib, "unroll": u, "median_us": round(us, 2), "TBps": round(3 * n * 4 / us / 1e6, 3),
                          "bit_exact": ok}), flush=True)
    del sets
    torch.cuda.empty_cache()
