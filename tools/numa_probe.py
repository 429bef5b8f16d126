"""numa_probe.py — where the GPU box's host side is: the CPUs this process may run on, their NUMA
nodes, the GPU's NUMA node (PCI sysfs), and the config-5 fused host path with its copy threads
left alone vs bound to the GPU's node (TIPS_HOST_BIND=1), interleaved. One JSON line each.
A tuning aid for host_staging.cc; not a test."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def emit(**kw):
    print(json.dumps(kw), flush=True)


def cpulist(s):
    out = []
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def main():
    allowed = sorted(os.sched_getaffinity(0))
    nodes = {}
    base = "/sys/devices/system/node"
    for d in sorted(os.listdir(base)) if os.path.isdir(base) else []:
        if d.startswith("node") and d[4:].isdigit():
            with open(os.path.join(base, d, "cpulist")) as f:
                nodes[int(d[4:])] = cpulist(f.read())
    emit(what="cpus", allowed=len(allowed), allowed_first=allowed[:8],
         allowed_per_node={n: len(set(c) & set(allowed)) for n, c in nodes.items()})
    import torch
    p = torch.cuda.get_device_properties(0)
    bus = "%04x:%02x:%02x.0" % (getattr(p, "pci_domain_id", 0), getattr(p, "pci_bus_id", 0), getattr(p, "pci_device_id", 0))
    node = None
    try:
        with open("/sys/bus/pci/devices/%s/numa_node" % bus) as f:
            node = int(f.read())
    except OSError as e:
        emit(what="gpu_numa_error", bus=bus, error=str(e))
    emit(what="gpu", bus=bus, numa_node=node)
    import numpy as np
    import bench
    import tips_amd
    tips_amd.init()
    sizes = bench.resnet50_grad_sizes()
    hg = [np.random.default_rng(i).random(k, dtype=np.float32) for i, k in enumerate(sizes)]
    total = sum(sizes) * 4
    for _ in range(3):
        tips_amd._reduce_grads(hg)
    # the same bytes as ONE host buffer through tips_amd.allreduce (the single-bucket host pipeline):
    # what a list of this total size could reach at best
    one = np.random.default_rng(7).random(sum(sizes), dtype=np.float32)
    for _ in range(2):
        tips_amd.allreduce(one)
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        r = tips_amd.allreduce(one)
        ts.append(time.perf_counter() - t0)
    del r
    ts.sort()
    emit(what="one_host_buffer_same_bytes", median_ms=round(ts[5] * 1e3, 3), best_ms=round(ts[0] * 1e3, 3),
         median_gib_s=round(total / ts[5] / 2 ** 30, 2))
    for rnd in range(3):
        for bind in ("0", "1"):
            os.environ["TIPS_HOST_BIND"] = bind
            ts = []
            for _ in range(10):
                t0 = time.perf_counter()
                outs = tips_amd._reduce_grads(hg)
                ts.append(time.perf_counter() - t0)
            del outs
            ts.sort()
            emit(what="reduce_grads_host", round=rnd, bind=bind, median_ms=round(ts[5] * 1e3, 3),
                 best_ms=round(ts[0] * 1e3, 3), median_gib_s=round(total / ts[5] / 2 ** 30, 2))
    tips_amd.shutdown()


if __name__ == "__main__":
    main()
