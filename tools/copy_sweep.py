"""copy_sweep.py — the fusion pack kernel's variants on the configs' real tensor lists (GPU box).

For BASELINE config 4 (1000 gradients, 2^U(8,17) elements) and config 5 (214 ResNet-50
gradients), as separate allocations: builds the pack descriptor list fusion.cc builds (tiles of
T bytes from each tensor into a 64 MiB bucket at 256-B aligned offsets), then times every
tips_copy_tiles_variant variant x tile size, rounds interleaved, each launch on one of 4
rotating tensor sets (so the bytes come from HBM, not the Infinity Cache), HIP events on the
launch stream. Prints one JSON line per (workload, tile, variant): median us per launch and
GB/s = 2 x bytes (read + write) / time; plus hipMemcpyAsync of the same bytes as one block.

usage: python3 tools/copy_sweep.py [rounds]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def tiles_for(sizes, srcs, bucket, tile, threshold=64 << 20):
    """(n, 3) int64 records {src, dst, bytes}: fusion.cc build_entry's pack tiles (one bucket slot)."""
    import numpy as np
    rec = []
    off, slot = 0, 0
    for k, s in zip(sizes, srcs):
        nb = k * 4
        off = (off + 255) // 256 * 256
        if off + nb > threshold:  # next bucket: the other slot, as fusion.cc (bucket b -> slot b % 2)
            off, slot = 0, 1 - slot
        for t in range(0, nb, tile):
            rec.append((s + t, bucket + slot * threshold + off + t, min(tile, nb - t)))
        off += nb
    return np.array(rec, dtype=np.int64)


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
    variants = [0, 1, 2, 3, 4, 5, 6, 7, 8]
    for wname, sizes in (("config4", bench.fused1000_sizes()), ("config5", bench.resnet50_grad_sizes())):
        total = sum(sizes) * 4
        sets = []
        for k in range(4):
            ts = [torch.randn(n, device="cuda") for n in sizes]
            bucket = torch.empty(2 * (64 << 20) // 4, device="cuda")
            sets.append((ts, bucket))
        for tile in (4096, 8192, 16384):
            tabs = []
            for ts, bucket in sets:
                rec = tiles_for(sizes, [t.data_ptr() for t in ts], bucket.data_ptr(), tile)
                tabs.append((torch.from_numpy(rec).cuda(), rec.shape[0]))
            times = {v: [] for v in variants}
            for r in range(rounds):
                for v in variants:
                    if v == 0 and tile > 65536:
                        continue
                    for i in range(2):  # warm
                        L.tips_copy_tiles_variant(tabs[i % 4][0].data_ptr(), tabs[i % 4][1], v, tile, sp)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    reps = 20
                    e0.record(stream)
                    for i in range(reps):
                        rc = L.tips_copy_tiles_variant(tabs[i % 4][0].data_ptr(), tabs[i % 4][1], v, tile, sp)
                        if rc:
                            raise _lib.TipsError("tips_copy_tiles_variant", rc, _lib.last_error())
                    e1.record(stream)
                    torch.cuda.synchronize()
                    times[v].append(e0.elapsed_time(e1) / reps * 1e3)
            # correctness: every variant packs exactly the bytes of every tensor
            ts, bucket = sets[0]
            ok = {}
            for v in variants:
                bucket.zero_()
                L.tips_copy_tiles_variant(tabs[0][0].data_ptr(), tabs[0][1], v, tile, sp)
                torch.cuda.synchronize()
                b8 = bucket.view(torch.uint8)
                good = True
                off, slot = 0, 0
                for t, n in zip(ts, sizes):
                    off = (off + 255) // 256 * 256
                    if off + n * 4 > (64 << 20):
                        off, slot = 0, 1 - slot
                    base = slot * (64 << 20) + off
                    good = good and torch.equal(b8[base:base + n * 4], t.view(torch.uint8))
                    off += n * 4
                ok[v] = bool(good)
            for v in variants:
                us = sorted(times[v])[len(times[v]) // 2]
                print(json.dumps({"workload": wname, "tile": tile, "variant": v, "tiles": tabs[0][1],
                                  "us_median": round(us, 2), "GBps": round(2 * total / (us * 1e-6) / 1e9, 1),
                                  "rounds_us": [round(x, 2) for x in times[v]], "bit_exact": ok[v]}), flush=True)
        # one contiguous block of the same bytes (the copy engine / blit kernel), rotating buffers
        a = [torch.empty(total // 4, device="cuda") for _ in range(4)]
        b = [torch.empty(total // 4, device="cuda") for _ in range(4)]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(20):
            b[i % 4].copy_(a[i % 4])
        e1.record(stream)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(json.dumps({"workload": wname, "variant": "torch copy_ one block", "us_median": round(us, 2),
                          "GBps": round(2 * total / (us * 1e-6) / 1e9, 1)}), flush=True)
        del sets, a, b


if __name__ == "__main__":
    main()
