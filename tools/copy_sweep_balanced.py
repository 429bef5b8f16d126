"""copy_sweep_balanced.py — the fusion pack kernel on the layout fusion.cc builds today (balanced
buckets, bench.fusion_layout): per-bucket launches, as fusion_allreduce issues them, for each
tips_copy_tiles_variant x tile size, 4 rotating gradient sets (HBM-only), rounds interleaved, HIP
events on the launch stream. One JSON line per (workload, tile, variant): median us per bucket
launch and GB/s = read + write bytes / time. (tools/copy_sweep.py measured round 2's first,
greedy layout: one 64 MiB and one 15 MiB launch for config 4.)

usage: python3 tools/copy_sweep_balanced.py [rounds]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    import numpy as np
    import torch

    import bench
    from tips_amd import _lib
    L = _lib.dev()  # (include/tips_hip_dev.h)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    variants, tiles = [1, 2, 5, 6], [4096, 8192, 16384]
    thr = 64 << 20
    for wname, sizes in (("config4", bench.fused1000_sizes()), ("config5", bench.resnet50_grad_sizes())):
        buckets = bench.fusion_layout(sizes)
        sets = [[torch.randn(n, device="cuda") for n in sizes] for _ in range(4)]
        slots = torch.empty(2 * thr // 4, device="cuda")
        payload = sum(sizes) * 4
        tabs = {}
        for tile in tiles:
            per_set = []
            for ts in sets:
                per_b = []
                for b, members in enumerate(buckets):
                    rec = []
                    for i, off in members:
                        nb = sizes[i] * 4
                        dst = slots.data_ptr() + (b % 2) * thr + off
                        rec += [(ts[i].data_ptr() + t, dst + t, min(tile, nb - t)) for t in range(0, nb, tile)]
                    per_b.append((torch.from_numpy(np.array(rec, dtype=np.int64)).cuda(), len(rec)))
                per_set.append(per_b)
            tabs[tile] = per_set
        times = {(t, v): [] for t in tiles for v in variants}
        for r in range(rounds):
            for tile in tiles:
                for v in variants:
                    def run(k):
                        for b in range(len(buckets)):
                            t, n = tabs[tile][k % 4][b]
                            rc = L.tips_copy_tiles_variant(t.data_ptr(), n, v, tile, sp)
                            if rc:
                                raise _lib.TipsError("tips_copy_tiles_variant", rc, _lib.last_error())
                    for k in range(4):
                        run(k)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for k in range(20):
                        run(k)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    times[(tile, v)].append(e0.elapsed_time(e1) * 1e3 / (20 * len(buckets)))
        for (tile, v), ts_ in times.items():
            us = sorted(ts_)[len(ts_) // 2]
            per_launch = 2 * payload / len(buckets)
            print(json.dumps({"workload": wname, "buckets": len(buckets), "tile": tile, "variant": v,
                              "us_median_per_bucket_launch": round(us, 2),
                              "GBps": round(per_launch / (us * 1e-6) / 1e9, 1),
                              "rounds_us": [round(x, 2) for x in ts_]}), flush=True)
        del sets, slots, tabs


if __name__ == "__main__":
    main()
