"""HBM-only rate of the direct schedule's fold (tips_multi_sum): p sources of one sub-chunk folded
into a destination, as the direct schedule lays them out (in[chunk r] + p-1 staging slots), over
rotating buffer sets so no launch finds its operands in the Infinity Cache. One JSON line per
(p, sub-chunk MiB)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from tips_amd import _lib  # noqa: E402

L = _lib.lib()
torch.cuda.set_device(0)
s = torch.cuda.current_stream()
for p, mib in ((8, 32), (8, 8), (4, 64), (2, 128)):
    n = mib * (1 << 18)
    sets = []
    for k in range(4):
        srcs = [torch.randn(n, device="cuda") for _ in range(p)]
        dst = torch.empty(n, device="cuda")
        ptrs, keep = _lib.ptr_array([t.data_ptr() for t in srcs])
        sets.append((srcs, dst, ptrs, keep))
    for i in range(8):
        srcs, dst, ptrs, _ = sets[i % 4]
        _lib.call("tips_multi_sum", dst.data_ptr(), ptrs, p, n, _lib.FLOAT32, s.cuda_stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    K = 40
    e0.record(s)
    for i in range(K):
        srcs, dst, ptrs, _ = sets[i % 4]
        _lib.call("tips_multi_sum", dst.data_ptr(), ptrs, p, n, _lib.FLOAT32, s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / K * 1e3
    moved = (p + 1) * n * 4
    print(json.dumps({"p": p, "sub_chunk_MiB": mib, "us_per_launch": round(us, 2), "TBps": round(moved / us / 1e6, 3),
                      "frac_of_8TBps": round(moved / us / 1e6 / 8.0, 4)}), flush=True)
    del sets
    torch.cuda.empty_cache()
