"""schedule_kernel_profile.py — the reduce kernels inside the allreduce schedules, at config 3's size.

Runs the ring and direct schedules for 8 virtual ranks x 1 GiB fp32 on this one GPU
(tips_ring_simulate / tips_direct_simulate: the real chunking, streams, events and kernels;
peer transfers as device copies). Under `rocprofv3 --kernel-trace --stats` the per-launch
durations of sum2_buf_kernel (ring: out = in + received, one 32 MiB sub-chunk) and
multi_sum_buf_kernel<f32, 8> (direct: 8-source rank-order fold of a 32 MiB sub-chunk) are the
reduce kernels as the schedules run them: one operand has just been written by the transfer.
Prints one JSON line with the schedule shape and the algorithmic bytes per launch.

usage: rocprofv3 --kernel-trace --stats -d OUT -o sched -- python3 tools/schedule_kernel_profile.py
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
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
    depth, sub = ctypes.c_int(), ctypes.c_int64()
    _lib.call("tips_schedule_shape", n, p, _lib.FLOAT32, ctypes.byref(depth), ctypes.byref(sub))
    reps = 3
    for fn in ("tips_ring_simulate", "tips_direct_simulate"):
        for _ in range(reps):
            _lib.dev_call(fn, po, pi, p, n, _lib.FLOAT32, sp)
        torch.cuda.synchronize()
    m = sub.value
    print(json.dumps({"p": p, "elements_per_rank": n, "pipeline_depth": depth.value, "sub_chunk_elements": m,
                      "ring_sum2_bytes_per_launch": 3 * m * 4, "direct_fold_bytes_per_launch": (p + 1) * m * 4,
                      "runs_per_schedule": reps}), flush=True)


if __name__ == "__main__":
    main()
