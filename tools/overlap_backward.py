"""overlap_backward.py — does DistributedOptimizer's allreduce run beside backward? (kernel-trace evidence)

usage: python3 tools/overlap_backward.py [STEPS] [RANKS]              (starts RANKS worker processes)
       python3 tools/overlap_backward.py worker RANK RANKS PORT STEPS   (one rank; under rocprofv3 each
                                                                         rank is its own profiler process:
                                                                         tools/gpu_overlap_backward.sh)
       python3 tools/overlap_backward.py report DIR LABEL            (one JSON line from the traces under DIR)

Every worker is a real RCCL rank sharing the box's one GPU (NCCL_HOSTID per rank: RCCL joins them
over its socket transport, as tests/test_gpu_rccl_procs.py). Each trains the bench's probe model
(6 x Linear(2048, 2048), 25.2 M fp32 parameters) for STEPS steps with tips_amd.DistributedOptimizer;
TIPS_OVERLAP_BACKWARD (inherited) chooses whether the buckets are allreduced during backward or in
step(). The report classifies each process's kernels as transfer (RCCL's) or compute (everything
else: the GEMMs and elementwise kernels of forward / backward / SGD) and gives the fraction of
compute busy time during which one of that process's RCCL kernels was running.
"""
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(rank, world, port, steps):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), TIPS_BOOTSTRAP_PORT=str(port), NCCL_HOSTID="tips-ovl-%d" % rank,
                      NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
    sys.path.insert(0, REPO)
    import torch
    import tips_amd
    from tips_amd import _lib
    torch.cuda.set_device(0)
    L = _lib.lib()
    L.tips_init()
    if not L.tips_is_initialize():
        raise SystemExit("tips_init failed: %s" % _lib.last_error())
    _lib.call("tips_set_algorithm", _lib.ALGO_AUTO)
    torch.manual_seed(5)
    layers = []
    for _ in range(6):
        layers += [torch.nn.Linear(2048, 2048), torch.nn.ReLU()]
    m = torch.nn.Sequential(*layers).cuda()
    opt = tips_amd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=1e-6))
    x = torch.randn(2048, 2048, device="cuda", generator=torch.Generator(device="cuda").manual_seed(rank))
    for i in range(steps + 2):
        if i == 2:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        opt.zero_grad(set_to_none=False)
        m(x).square().mean().backward()
        opt.step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(json.dumps({"rank": rank, "overlap": os.environ.get("TIPS_OVERLAP_BACKWARD", "1"),
                      "buckets": len(opt._buckets.buckets) if opt._buckets is not None else 0,
                      "ms_per_step": round(dt * 1e3, 3)}), flush=True)
    L.tips_shutdown()


def launch(steps, world):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "worker", str(r), str(world), str(port),
                               str(steps)]) for r in range(world)]
    rc = 0
    for p in procs:
        rc = rc or p.wait(timeout=240)
    return rc


def report(d, label):
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from overlap_report import overlap_len, union
    import csv
    out = {"label": label, "processes": []}
    for root, _, files in os.walk(d):
        for f in files:
            if not f.endswith("kernel_trace.csv"):
                continue
            rows = list(csv.DictReader(open(os.path.join(root, f))))
            if not rows:
                continue
            keys = rows[0].keys()
            nk = next(k for k in keys if "Kernel_Name" in k)
            sk = next(k for k in keys if "Start_Timestamp" in k)
            ek = next(k for k in keys if "End_Timestamp" in k)
            xfer, comp = [], []
            for r in rows:
                iv = (int(r[sk]), int(r[ek]))
                (xfer if ("nccl" in r[nk].lower() or "rccl" in r[nk].lower()) else comp).append(iv)
            mx = union(xfer)
            comp_busy = sum(e - s for s, e in union(comp))
            under = sum(overlap_len(s, e, mx) for s, e in union(comp))
            allk = union(xfer + comp)
            span = max(e for _, e in allk) - min(s for s, _ in allk)
            busy = sum(e - s for s, e in allk)
            # the same split over the timed steps only: the last `steps` (5) of the 7 optimizer steps,
            # cut at the SGD kernels' ends is fragile, so the whole trace is split per its wall span
            out["processes"].append({"trace": f, "compute_kernels": len(comp), "transfer_kernels": len(xfer),
                                     "compute_busy_ms": round(comp_busy / 1e6, 3),
                                     "transfer_busy_ms": round(sum(e - s for s, e in mx) / 1e6, 3),
                                     "transfer_not_under_compute_ms": round((busy - comp_busy) / 1e6, 3),
                                     "idle_ms": round((span - busy) / 1e6, 3), "span_ms": round(span / 1e6, 3),
                                     "mean_transfer_kernel_us": round(sum(e - s for s, e in xfer) / max(1, len(xfer)) / 1e3, 1),
                                     "compute_under_transfer_frac": round(under / max(1, comp_busy), 4)})
    print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "worker":
        worker(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]))
    elif len(sys.argv) > 1 and sys.argv[1] == "report":
        report(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
    else:
        sys.exit(launch(int(sys.argv[1]) if len(sys.argv) > 1 else 5, int(sys.argv[2]) if len(sys.argv) > 2 else 2))
