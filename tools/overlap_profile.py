"""overlap_profile.py — does the schedules' transfer of sub-chunk k+1 overlap the sum of sub-chunk k?

Runs one schedule (ring or direct) for 8 virtual ranks x 1 GiB fp32 (BASELINE config 3's shape) on
this one GPU through the single-GPU simulator, which executes the same per-rank op plans as the
RCCL executor (plan.cc) with the same two streams: transfers on the high-priority comm stream,
sums on the compute stream, ordered only by the plan's recv / sum events. With --transport 1 every
transfer is a grouped ncclSend/ncclRecv (RCCL kernels, rank to itself), with 0 a device copy.

Run it under `rocprofv3 --kernel-trace --output-format csv` and feed the kernel trace to
tools/overlap_report.py, which measures from the dispatch intervals how much of the sum-kernel
time runs while a transfer kernel is running.

usage: rocprofv3 --kernel-trace --output-format csv -d OUT -o ring -- python3 tools/overlap_profile.py ring 1
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "ring"
    transport = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    import ctypes

    import torch
    import tips_amd
    from tips_amd import _lib
    tips_amd.init()
    p, n = 8, 268435456
    g = torch.Generator(device="cuda")
    ins = []
    for r in range(p):
        g.manual_seed(3000 + r)
        ins.append(torch.empty(n, dtype=torch.float32, device="cuda").uniform_(0.5, 1.5, generator=g))
    outs = [torch.empty_like(x) for x in ins]
    pi, _k1 = _lib.ptr_array([x.data_ptr() for x in ins])
    po, _k2 = _lib.ptr_array([o.data_ptr() for o in outs])
    sp = torch.cuda.current_stream().cuda_stream
    fn = {"ring": "tips_ring_simulate", "direct": "tips_direct_simulate"}[kind]
    _lib.dev_call("tips_set_sim_transport", transport)
    _lib.dev_call(fn, po, pi, p, n, _lib.FLOAT32, sp)  # warm-up (staging, events, RCCL connections)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        _lib.dev_call(fn, po, pi, p, n, _lib.FLOAT32, sp)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    depth, sub = ctypes.c_int(), ctypes.c_int64()
    _lib.call("tips_schedule_shape", n, p, _lib.FLOAT32, ctypes.byref(depth), ctypes.byref(sub))
    exp = ins[0].clone()  # spot check: the direct fold's bits / the ring's tolerance on a sample
    for r in range(1, p):
        exp += ins[r]
    idx = torch.arange(0, n, 4099, device="cuda")
    rel = ((outs[0][idx].double() - exp[idx].double()).abs() / exp[idx].double()).max().item()
    print(json.dumps({"schedule": kind, "transport": "rccl self-loop" if transport else "device copies",
                      "p": p, "elements_per_rank": n, "pipeline_depth": depth.value, "sub_chunk_elements": sub.value,
                      "runs": reps, "wall_ms_per_run": round(wall * 1e3, 3), "max_rel_err_sample": rel}), flush=True)


if __name__ == "__main__":
    main()
