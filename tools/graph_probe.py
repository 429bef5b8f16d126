"""graph_probe.py — tools/graph_probe.cc's capture patterns, in a Python process with torch loaded,
i.e. on the HIP runtime and RCCL that torch bundles (the ones tips_amd runs on in Python).

Run: python tools/graph_probe.py RANK SIZE MODE ID_FILE
Modes: 1 ncclAllReduce on the origin stream; 2 grouped ncclSend/ncclRecv on the origin stream;
3 the group on a stream forked from the origin; 4 mode 3 plus a memset on a second forked stream
behind an event. Each: one eager call, capture, instantiate, 3 replays, bytes checked.
"""
import ctypes
import os
import sys
import time

import torch


def main():
    rank, size, mode, idf = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    hip = ctypes.CDLL("libamdhip64.so.7")
    nccl = ctypes.CDLL("librccl.so.1")
    ver = ctypes.c_int()
    nccl.ncclGetVersion(ctypes.byref(ver))
    print("rank %d: rccl %d, torch hip %s" % (rank, ver.value, torch.version.hip), flush=True)

    class Uid(ctypes.Structure):
        _fields_ = [("b", ctypes.c_char * 128)]
    uid = Uid()
    if rank == 0:
        assert nccl.ncclGetUniqueId(ctypes.byref(uid)) == 0
        with open(idf + ".tmp", "wb") as f:
            f.write(ctypes.string_at(ctypes.addressof(uid), 128))  # (uid.b would stop at the first NUL)
        os.rename(idf + ".tmp", idf)
    else:
        for _ in range(600):
            if os.path.exists(idf):
                break
            time.sleep(0.1)
        ctypes.memmove(ctypes.byref(uid), open(idf, "rb").read(), 128)
    comm = ctypes.c_void_p()
    assert nccl.ncclCommInitRank(ctypes.byref(comm), size, uid, rank) == 0
    n = 1 << 20
    a = torch.full((n,), float(rank + 1), device="cuda")
    b = torch.zeros(size * n, device="cuda")
    origin, s1, s2 = (torch.cuda.Stream(priority=-1 if os.environ.get("PROBE_PRIO") else 0) for _ in range(3))
    ev = [ctypes.c_void_p() for _ in range(4)]
    for e in ev:
        assert hip.hipEventCreateWithFlags(ctypes.byref(e), 2) == 0  # hipEventDisableTiming
    H = lambda s: ctypes.c_void_p(s.cuda_stream)  # noqa: E731

    def ck(rc, what):
        if rc != 0:
            raise SystemExit("rank %d: %s -> %d" % (rank, what, rc))

    def body():
        if mode == 1:
            ck(nccl.ncclAllReduce(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(a.data_ptr()), ctypes.c_size_t(n), 7, 0,
                                  comm, H(origin)), "allreduce")  # ncclFloat32 = 7, ncclSum = 0
            return
        if mode == 5:  # the executor's steps with the transfers on the origin: group, sum behind it, origin waits the sum
            for step in range(2):
                ck(nccl.ncclGroupStart(), "groupstart")
                for q in range(size):
                    ck(nccl.ncclSend(ctypes.c_void_p(a.data_ptr()), ctypes.c_size_t(4 * n), 0, q, comm, H(origin)), "send")
                    ck(nccl.ncclRecv(ctypes.c_void_p(b.data_ptr() + 4 * n * q), ctypes.c_size_t(4 * n), 0, q, comm,
                                     H(origin)), "recv")
                ck(nccl.ncclGroupEnd(), "groupend")
                ck(hip.hipEventRecord(ev[1], H(origin)), "record")
                ck(hip.hipStreamWaitEvent(H(s2), ev[1], 0), "wait")
                ck(hip.hipMemsetD32Async(ctypes.c_void_p(b.data_ptr()), 0x40A00000, ctypes.c_size_t(16), H(s2)), "memset")
                ck(hip.hipEventRecord(ev[3], H(s2)), "record")
                if step == 0:
                    ck(hip.hipStreamWaitEvent(H(origin), ev[3], 0), "wait")
            ck(hip.hipStreamWaitEvent(H(origin), ev[3], 0), "wait")
            return
        cs = origin if mode == 2 else s1
        if mode >= 3:
            ck(hip.hipEventRecord(ev[0], H(origin)), "record")
            ck(hip.hipStreamWaitEvent(H(s1), ev[0], 0), "wait")
            ck(hip.hipStreamWaitEvent(H(s2), ev[0], 0), "wait")
        ck(nccl.ncclGroupStart(), "groupstart")
        for q in range(size):
            ck(nccl.ncclSend(ctypes.c_void_p(a.data_ptr()), ctypes.c_size_t(4 * n), 0, q, comm, H(cs)), "send")
            ck(nccl.ncclRecv(ctypes.c_void_p(b.data_ptr() + 4 * n * q), ctypes.c_size_t(4 * n), 0, q, comm, H(cs)), "recv")
        ck(nccl.ncclGroupEnd(), "groupend")
        if mode == 4:
            ck(hip.hipEventRecord(ev[1], H(s1)), "record")
            ck(hip.hipStreamWaitEvent(H(s2), ev[1], 0), "wait")
            ck(hip.hipMemsetD32Async(ctypes.c_void_p(b.data_ptr()), 0x40A00000, ctypes.c_size_t(16), H(s2)), "memset")
        if mode >= 3:
            ck(hip.hipEventRecord(ev[2], H(s1)), "record")
            ck(hip.hipStreamWaitEvent(H(origin), ev[2], 0), "wait")
            ck(hip.hipEventRecord(ev[3], H(s2)), "record")
            ck(hip.hipStreamWaitEvent(H(origin), ev[3], 0), "wait")

    def check(what):
        origin.synchronize()
        ok = True
        if mode == 1:
            ok = float(a[0]) == size * (size + 1) / 2 and float(a[-1]) == size * (size + 1) / 2
        else:
            for q in range(size):
                w0 = 5.0 if mode in (4, 5) and q == 0 else float(q + 1)
                ok = ok and float(b[q * n]) == w0 and float(b[q * n + n - 1]) == float(q + 1)
        print("rank %d mode %d %s: %s" % (rank, mode, what, "ok" if ok else "WRONG"), flush=True)
        if not ok:
            raise SystemExit(1)

    def reset():
        a.fill_(float(rank + 1))
        b.zero_()
        torch.cuda.synchronize()

    reset()
    body()
    check("eager")
    torch.cuda.synchronize()
    print("rank %d mode %d: capture" % (rank, mode), flush=True)
    ck(hip.hipStreamBeginCapture(H(origin), 2), "begin capture")  # hipStreamCaptureModeRelaxed
    body()
    g = ctypes.c_void_p()
    print("rank %d mode %d: end capture" % (rank, mode), flush=True)
    ck(hip.hipStreamEndCapture(H(origin), ctypes.byref(g)), "end capture")
    print("rank %d mode %d: ended" % (rank, mode), flush=True)
    x = ctypes.c_void_p()
    ck(hip.hipGraphInstantiate(ctypes.byref(x), g, None, None, ctypes.c_size_t(0)), "instantiate")
    for _ in range(3):
        reset()
        ck(hip.hipGraphLaunch(x, H(origin)), "launch")
        check("replay")
    hip.hipGraphExecDestroy(x)
    hip.hipGraphDestroy(g)
    nccl.ncclCommDestroy(comm)
    print("rank %d mode %d: PASS" % (rank, mode), flush=True)


if __name__ == "__main__":
    main()
