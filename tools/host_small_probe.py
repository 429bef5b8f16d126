"""host_small_probe.py — per-call cost of the host-memory allreduce (tips_amd.allreduce on numpy
arrays, one rank), by tensor size and over config 5's ResNet-50 gradient list. Diagnoses where
the host -> host time of bench.py's resnet50 line goes. One JSON line per row."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import tips_amd
    import bench
    tips_amd.init()
    sizes = bench.resnet50_grad_sizes()
    grads = [np.random.default_rng(i).random(k, dtype=np.float32) for i, k in enumerate(sizes)]
    for g in grads:
        tips_amd.allreduce(g)
    per = [0.0] * len(grads)
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        for i, g in enumerate(grads):
            t1 = time.perf_counter()
            tips_amd.allreduce(g)
            per[i] += time.perf_counter() - t1
    total = (time.perf_counter() - t0) / reps
    buckets = {}
    for k, t in zip(sizes, per):
        b = "<=64K" if k * 4 <= 65536 else "<=1M" if k * 4 <= 1 << 20 else "<=4M" if k * 4 <= 4 << 20 else ">4M"
        c = buckets.setdefault(b, [0, 0.0, 0])
        c[0] += 1
        c[1] += t / reps
        c[2] += k * 4
    print(json.dumps({"resnet50_ms_per_step": round(total * 1e3, 3), "sum_of_calls_ms": round(sum(per) / reps * 1e3, 3)}))
    for b, (cnt, t, byt) in sorted(buckets.items()):
        print(json.dumps({"bucket": b, "tensors": cnt, "ms": round(t * 1e3, 3), "MB": round(byt / 1e6, 2),
                          "us_per_tensor": round(t / cnt * 1e6, 1)}))


if __name__ == "__main__":
    main()
