"""Does the fold's occupancy cap starve a transfer running beside it? One GPU, one RCCL rank: a
256 MiB ncclSend/ncclRecv to self (RCCL's p2p copy kernel, the kernel that moves xGMI transfers;
here it copies within HBM) on a high-priority stream, timed alone and with tips_multi_sum_variant
folds of 8 x 32 MiB running back to back on a second stream, per fold variant. Also the folds'
own rate beside the transfer. One JSON line per variant. (Diagnostic for DESIGN.md §3.)"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from tips_amd import _lib  # noqa: E402

L = _lib.dev()
torch.cuda.set_device(0)
rccl = ctypes.CDLL("librccl.so.1")


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


uid = UniqueId()
assert rccl.ncclGetUniqueId(ctypes.byref(uid)) == 0
comm = ctypes.c_void_p()
assert rccl.ncclCommInitRank(ctypes.byref(comm), 1, uid, 0) == 0
hi = torch.cuda.Stream(priority=-1)
lo = torch.cuda.Stream()
NB = 256 << 20
sbuf = torch.empty(NB // 4, device="cuda").uniform_()
rbuf = torch.empty_like(sbuf)


def xfer():
    assert rccl.ncclGroupStart() == 0
    assert rccl.ncclSend(ctypes.c_void_p(sbuf.data_ptr()), ctypes.c_size_t(NB), 0, 0, comm,
                         ctypes.c_void_p(hi.cuda_stream)) == 0  # ncclInt8
    assert rccl.ncclRecv(ctypes.c_void_p(rbuf.data_ptr()), ctypes.c_size_t(NB), 0, 0, comm,
                         ctypes.c_void_p(hi.cuda_stream)) == 0
    assert rccl.ncclGroupEnd() == 0


p, n = 8, 32 << 18
sets = []
for k in range(4):
    srcs = [torch.empty(n, device="cuda").uniform_() for _ in range(p)]
    sets.append((srcs, torch.empty(n, device="cuda"), _lib.ptr_array([t.data_ptr() for t in srcs])))


def folds(v, count):
    for i in range(count):
        srcs, dst, (ptrs, _) = sets[i % 4]
        L.tips_multi_sum_variant(dst.data_ptr(), ptrs, p, n, _lib.FLOAT32, v, lo.cuda_stream)


def timed_xfer(v, reps=5):
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if v is not None:
            f0.record(lo)
            folds(v, 60)  # ~3 ms of folds, longer than the transfer
            f1.record(lo)
        e0.record(hi)
        xfer()
        e1.record(hi)
        torch.cuda.synchronize()
        out.append((e0.elapsed_time(e1), f0.elapsed_time(f1) / 60 if v is not None else None))
    return out


for _ in range(3):
    xfer()
torch.cuda.synchronize()
VARIANTS = [int(x) for x in os.environ.get("VARIANTS", "1,30,27,18").split(",")]
alone = sorted(t for t, _ in timed_xfer(None, 7))
for rnd in range(2):
    print(json.dumps({"variant": None, "xfer_ms_median": round(alone[len(alone) // 2], 3)}), flush=True)
    for v in VARIANTS:
        r = timed_xfer(v)
        xs = sorted(t for t, _ in r)
        fs = sorted(f for _, f in r)
        print(json.dumps({"round": rnd, "variant": v, "xfer_ms_median": round(xs[len(xs) // 2], 3),
                          "xfer_slowdown": round(xs[len(xs) // 2] / alone[len(alone) // 2], 3),
                          "fold_us_beside_xfer": round(fs[len(fs) // 2] * 1e3, 2)}), flush=True)
rccl.ncclCommDestroy(comm)
