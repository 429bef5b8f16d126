"""Is the fused step capturable into a HIP graph, and what does replay save at one rank?

TIPS_FUSION_MEASURE_PACK=1 (one rank packs and unpacks its buckets as at N > 1). For config 4
and config 5 (bench.py's tensor lists, 4 rotating gradient sets): eager FusedList.allreduce_
calls vs one torch.cuda.CUDAGraph per set holding the same call, replayed. Every output is
checked bit-exact (one rank: the identity). One JSON line per workload.

The "eager" column is Python-bound: the gradient set rotates every call, so FusedList sees new
pointers each time and re-validates all tensors. bench.py's eager line passes prebuilt pointer
arrays instead (≈ 85 µs for config 4). The "graph" column is the number that matters here."""
import json
import os
import sys

os.environ["TIPS_FUSION_MEASURE_PACK"] = "1"
sys.path.insert(0, ".")
import torch  # noqa: E402

import bench  # noqa: E402
import tips_amd  # noqa: E402
from tips_amd import ops  # noqa: E402

tips_amd.init()
torch.cuda.set_device(0)
R, STEPS = 4, 40
for name, sizes in (("fused1000", bench.fused1000_sizes()), ("resnet50", bench.resnet50_grad_sizes())):
    offs, total = [], 0
    for k in sizes:
        offs.append(total)
        total += (k + 63) // 64 * 64 + 64
    sets, refs = [], []
    for r in range(R):
        x = torch.empty(total, device="cuda").uniform_(0.5, 1.5)
        sets.append([x[o:o + k] for o, k in zip(offs, sizes)])
        refs.append(x.clone())
    fl = ops.FusedList(sizes)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    res = {}
    with torch.cuda.stream(s):
        for r in range(R):  # builds every set's plan before any capture
            fl.allreduce_(sets[r])
        torch.cuda.synchronize()
        graphs = []
        for r in range(R):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                fl.allreduce_(sets[r])
            graphs.append(g)
        torch.cuda.synchronize()
        for mode in ("eager", "graph", "eager", "graph", "eager", "graph"):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for i in range(STEPS):
                if mode == "eager":
                    fl.allreduce_(sets[i % R])
                else:
                    graphs[i % R].replay()
            e1.record(s)
            torch.cuda.synchronize()
            res.setdefault(mode, []).append(e0.elapsed_time(e1) / STEPS * 1e3)
    ok = all(torch.equal(torch.cat([v.reshape(-1) for v in sets[r]]),
                         torch.cat([refs[r][o:o + k] for o, k in zip(offs, sizes)])) for r in range(R))
    nbytes = 4 * 4 * sum(sizes)  # pack + unpack: 2 reads + 2 writes of every byte
    line = {"workload": name, "tensors": len(sizes), "bit_exact": bool(ok)}
    for mode, v in res.items():
        us = sorted(v)[len(v) // 2]
        line[mode] = {"us_per_step": round(us, 2), "TBps": round(nbytes / us / 1e6, 3), "rounds_us": [round(t, 2) for t in v]}
    print(json.dumps(line), flush=True)
