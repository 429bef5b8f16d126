"""Why does config 4's pack + unpack over separately allocated gradients (bench gradient_api
packed_separate_grads) take ~2.5 x the same step over views of one buffer? One GPU,
TIPS_FUSION_MEASURE_PACK=1 (the buckets packed and unpacked as at N > 1), 4 rotating gradient sets
each way, per step: wall time (host-timed, synchronised), the host time of the calls alone (no
sync), and device time (events around the steps). Legs:
  views       - views of one flat buffer, 256 B apart (bench's fixed-view step), pointer arrays
                prebuilt, tips_fused_allreduce through ctypes;
  separate    - every gradient its own allocation (clones, as .grad tensors), same prebuilt call;
  separate_fl - the same tensors through FusedList.allreduce_ (bench's packed_separate_grads);
  sorted      - separate allocations, but the list handed over in address order.
Run under rocprofv3 --kernel-trace --stats to split the kernel time per leg (LEG=<name> runs one)."""
import json
import os
import sys
import time

os.environ.setdefault("TIPS_FUSION_MEASURE_PACK", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
import tips_amd  # noqa: E402
from tips_amd import _lib  # noqa: E402
from tips_amd.ops import FusedList  # noqa: E402

tips_amd.init()
L = _lib.lib()
sizes = bench.fused1000_sizes() if os.environ.get("WORKLOAD", "config4") == "config4" else bench.resnet50_grad_sizes()
n = len(sizes)
cp, _kc = _lib.i64_array(sizes)
s = torch.cuda.current_stream()
offs, tot = [], 0
for k in sizes:
    offs.append(tot)
    tot += (k + 63) // 64 * 64 + 64
flats = [torch.randn(tot, device="cuda") for _ in range(4)]
views = [[f[o:o + k] for o, k in zip(offs, sizes)] for f in flats]
seps = [[v.clone() for v in vs] for vs in views]
torch.cuda.synchronize()


def arrays(lst):
    return _lib.ptr_array([t.data_ptr() for t in lst])


legs = {}
va = [arrays(v) for v in views]
legs["views"] = lambda i: L.tips_fused_allreduce(va[i % 4][0], cp, n, _lib.FLOAT32, s.cuda_stream)
sa = [arrays(v) for v in seps]
legs["separate"] = lambda i: L.tips_fused_allreduce(sa[i % 4][0], cp, n, _lib.FLOAT32, s.cuda_stream)
fls = [FusedList(sizes) for _ in range(4)]
legs["separate_fl"] = lambda i: fls[i % 4].allreduce_(seps[i % 4])
order = [sorted(range(n), key=lambda j: seps[k][j].data_ptr()) for k in range(4)]
so = [arrays([seps[k][j] for j in order[k]]) for k in range(4)]
cps = [_lib.i64_array([sizes[j] for j in order[k]]) for k in range(4)]
legs["sorted"] = lambda i: L.tips_fused_allreduce(so[i % 4][0], cps[i % 4][0], n, _lib.FLOAT32, s.cuda_stream)

only = os.environ.get("LEG")
steps = int(os.environ.get("STEPS", "200"))
gaps = []
for k in range(4):  # how scattered the separate allocations are
    ps = sorted(t.data_ptr() for t in seps[k])
    gaps.append({"span_MiB": round((ps[-1] - ps[0]) / 2**20, 1),
                 "list_order_is_address_order": [t.data_ptr() for t in seps[k]] == ps})
print(json.dumps({"workload": os.environ.get("WORKLOAD", "config4"), "tensors": n, "separate_sets": gaps}), flush=True)
for rnd in range(3):
    for name, fn in legs.items():
        if only and name != only:
            continue
        for i in range(8):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(s)
        host = 0.0
        for i in range(steps):
            h0 = time.perf_counter()
            fn(i)
            host += time.perf_counter() - h0
        e1.record(s)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / steps * 1e6
        print(json.dumps({"round": rnd, "leg": name, "wall_us": round(wall, 2), "host_call_us": round(host / steps * 1e6, 2),
                          "events_us": round(e0.elapsed_time(e1) / steps * 1e3, 2)}), flush=True)
print(json.dumps({"fusion_stats": tips_amd.fusion_stats()}), flush=True)
