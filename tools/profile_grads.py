"""Host cost of allreduce_grads' N > 1 body on one GPU (tools/, not product): configs 4 and 5's
gradients as separate device tensors, _reduce_grads timed per call (plan hit: the same tensor
objects; fresh: new tensor objects each call), next to the fixed-view fused call
(FusedList.allreduce_), with a cProfile of the plan-hit path. One JSON line per workload."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("TIPS_FUSION_MEASURE_PACK", "1")

import torch  # noqa: E402

import bench  # noqa: E402
import tips_amd  # noqa: E402
from tips_amd.ops import FusedList  # noqa: E402


def timed(fn, k=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


def main():
    tips_amd.init()
    for name, sizes in (("config4", bench.fused1000_sizes()), ("config5", bench.resnet50_grad_sizes())):
        sets = [[torch.randn(n, device="cuda") for n in sizes] for _ in range(4)]
        i = [0]

        def hit():
            i[0] += 1
            tips_amd._reduce_grads(sets[i[0] % 4])

        def fresh():
            tips_amd._reduce_grads([t.view(t.shape) for t in sets[0]])  # new tensor objects, same storage

        fl = FusedList(sizes)

        def fixed():
            i[0] += 1
            fl.allreduce_(sets[i[0] % 4])

        row = {"workload": name, "tensors": len(sizes), "plan_hit_ms": timed(hit), "fresh_objects_ms": timed(fresh, 10),
               "fixed_view_ms": timed(fixed)}
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(20):
            hit()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(8)
        row["profile_plan_hit"] = s.getvalue().splitlines()[-14:]
        row["fusion_stats"] = tips_amd.fusion_stats()
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
