"""host_call_probe.py — where one small host-memory allreduce's time goes (one rank): the Python
surface (tips_amd.allreduce), the bare C-ABI call (tips_allreduce through ctypes), and the HIP calls
it is made of, each timed alone over many calls. One JSON line per row. A tuning aid for
run_staged (rt.h) and allreduce_op (ops.py); not a test."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def per_call(fn, reps=2000):
    for _ in range(50):
        fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return round((time.perf_counter() - t0) / reps * 1e6, 2)


def main():
    import numpy as np
    import torch
    import tips_amd
    from tips_amd import _lib
    torch.cuda.set_device(0)
    tips_amd.init()
    L = _lib.lib()
    hip = ctypes.CDLL("libamdhip64.so")
    attr = ctypes.create_string_buffer(256)
    for kib in (1, 16, 64, 256, 1024):
        x = np.random.default_rng(kib).random(kib * 256, dtype=np.float32)
        y = np.empty_like(x)
        n = x.size
        px, py = x.ctypes.data, y.ctypes.data
        row = {"KiB": kib,
               "python_allreduce_us": per_call(lambda: tips_amd.allreduce(x)),
               "c_abi_tips_allreduce_us": per_call(lambda: L.tips_allreduce(px, py, n, _lib.FLOAT32, _lib.OP_SUM, None))}
        print(json.dumps(row), flush=True)
    s = torch.cuda.Stream()
    row = {"hipPointerGetAttributes_pageable_us": per_call(lambda: hip.hipPointerGetAttributes(attr, ctypes.c_void_p(px))),
           "hipStreamSynchronize_idle_us": per_call(lambda: hip.hipStreamSynchronize(ctypes.c_void_p(s.cuda_stream))),
           "torch_empty_like_1KiB_us": per_call(lambda: np.empty_like(x[:256]))}
    d = torch.empty(256, device="cuda")
    h = torch.empty(256, pin_memory=True)
    ev = torch.cuda.Event()

    def h2d_sync():
        hip.hipMemcpyAsync(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(h.data_ptr()), ctypes.c_size_t(1024), 1,
                           ctypes.c_void_p(s.cuda_stream))
        hip.hipStreamSynchronize(ctypes.c_void_p(s.cuda_stream))

    def h2d_spin():
        hip.hipMemcpyAsync(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(h.data_ptr()), ctypes.c_size_t(1024), 1,
                           ctypes.c_void_p(s.cuda_stream))
        ev.record(s)
        while not ev.query():
            pass
    row["pinned_1KiB_h2d_then_sync_us"] = per_call(h2d_sync)
    row["pinned_1KiB_h2d_then_event_spin_us"] = per_call(h2d_spin)
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
