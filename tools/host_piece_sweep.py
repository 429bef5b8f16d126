"""host_piece_sweep.py — piece size of the pipelined host-memory allreduce (host_staging.cc).

This runs tips_allreduce(host in, host out) on one rank over 256 MiB of fp32
for each TIPS_HOST_PIECE_BYTES value. The env is read on every call, so a
single process covers them all. Three kinds of host memory are measured:
- pinned (torch pin_memory);
- pageable numpy;
- numpy registered with tips_host_register.

Each result is one JSON line with the bucket rate in GiB/s. The reference
points are the bidirectional DMA ceiling in profiles/r01_pcie_probe.jsonl
and DESIGN.md §3.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import tips_amd
    from tips_amd import _lib
    tips_amd.init()
    L = _lib.lib()
    n = 64 << 20
    bytes_ = n * 4
    pinned_in = torch.empty(n, dtype=torch.float32, pin_memory=True).uniform_()
    pinned_out = torch.empty(n, dtype=torch.float32, pin_memory=True)
    page_in = np.random.default_rng(1).random(n, dtype=np.float32)
    page_out = np.empty_like(page_in)
    reg_in = np.random.default_rng(2).random(n, dtype=np.float32)
    reg_out = np.empty_like(reg_in)
    _lib.call("tips_host_register", reg_in.ctypes.data, reg_in.nbytes)
    _lib.call("tips_host_register", reg_out.ctypes.data, reg_out.nbytes)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")  # the runtime torch already mapped
    hm = []
    for flags in (0, 2):  # hipHostMallocDefault, hipHostMallocMapped
        pair = []
        for _ in range(2):
            p = ctypes.c_void_p()
            assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(bytes_), ctypes.c_uint(flags)) == 0
            ctypes.memset(p, 0, bytes_)
            pair.append(p.value)
        hm.append(pair)
    kinds = [("pinned_torch", pinned_in.data_ptr(), pinned_out.data_ptr()),
             ("pageable_numpy", page_in.ctypes.data, page_out.ctypes.data),
             ("registered_numpy", reg_in.ctypes.data, reg_out.ctypes.data),
             ("hipHostMalloc_default", hm[0][0], hm[0][1]),
             ("hipHostMalloc_mapped", hm[1][0], hm[1][1])]
    if os.environ.get("PAGEABLE_FIRST") == "1":  # the order bench.py measures in
        kinds = [kinds[1], kinds[0]] + kinds[2:]
    extra = [torch.empty(n, dtype=torch.float32, pin_memory=True) for _ in range(int(os.environ.get("EXTRA_PINNED", "0")))]
    sizes = [int(x) for x in os.environ.get("PIECES_MIB", "4,8,16,32,64").split(",")]
    rounds = int(os.environ.get("ROUNDS", "1"))
    for mib in [m for _ in range(rounds) for m in sizes]:
        os.environ["TIPS_HOST_PIECE_BYTES"] = str(mib << 20)
        for name, pi, po in kinds:
            _lib.call("tips_allreduce", pi, po, n, _lib.FLOAT32, _lib.OP_SUM, None)
            ts = []
            for _ in range(7):
                t0 = time.perf_counter()
                _lib.call("tips_allreduce", pi, po, n, _lib.FLOAT32, _lib.OP_SUM, None)
                ts.append(time.perf_counter() - t0)
            ts.sort()
            print(json.dumps({"piece_mib": mib, "memory": name, "median_ms": round(ts[3] * 1e3, 3),
                              "gib_s": round(bytes_ / ts[3] / (1 << 30), 2)}), flush=True)
    ok = bool(np.array_equal(reg_out, reg_in)) and bool(torch.equal(pinned_out, pinned_in))
    print(json.dumps({"identity_check": ok}), flush=True)
    _lib.call("tips_host_unregister", reg_in.ctypes.data)
    _lib.call("tips_host_unregister", reg_out.ctypes.data)
    tips_amd.shutdown()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
