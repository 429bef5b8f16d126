"""Where the fused host path's time goes (config 5 shapes, one rank): the raw rates the pipeline is
built from - host memcpy with 1..16 threads, page-locked H2D / D2H / both directions at once - next
to tips_amd._reduce_grads on 214 numpy gradients with TIPS_HOST_TRACE=1 (per-call phase split on
stderr). Prints one JSON line per measurement. Not a test; a tuning aid for host_staging.cc."""
import json
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
GIB = float(1 << 30)


def emit(**kw):
    print(json.dumps(kw), flush=True)


def memcpy_rate(nbytes, threads):
    src = np.random.default_rng(0).integers(0, 255, nbytes, dtype=np.uint8)
    dst = np.empty_like(src)
    dst[:] = src
    per = nbytes // threads

    def part(j):
        np.copyto(dst[j * per:(j + 1) * per], src[j * per:(j + 1) * per])

    best = 1e9
    for _ in range(5):
        ts = [threading.Thread(target=part, args=(j,)) for j in range(threads)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        best = min(best, time.perf_counter() - t0)
    emit(what="host_memcpy", threads=threads, bytes=nbytes, gib_s=round(nbytes / best / GIB, 2))


def link_rates(nbytes):
    h_in = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for name, fn in [("h2d", lambda: d.copy_(h_in, non_blocking=True)),
                     ("d2h", lambda: h_out.copy_(d, non_blocking=True))]:
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        emit(what=name, bytes=nbytes, gib_s=round(5 * nbytes / (time.perf_counter() - t0) / GIB, 2))
    def both(k):
        for _ in range(k):
            with torch.cuda.stream(s1):
                d.copy_(h_in, non_blocking=True)
            with torch.cuda.stream(s2):
                h_out.copy_(d2, non_blocking=True)

    both(2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    both(5)
    torch.cuda.synchronize()
    emit(what="h2d+d2h", bytes=nbytes, gib_s_each=round(5 * nbytes / (time.perf_counter() - t0) / GIB, 2))
    # D2H into host memory page-locked by hipHostRegister (the flat host outputs) vs hipHostMalloc
    import tips_amd
    from tips_amd import _lib
    tips_amd.init()
    reg = np.empty(nbytes, dtype=np.uint8)
    reg[:] = 1
    _lib.call("tips_host_register", reg.ctypes.data, nbytes)
    reg_t = torch.from_numpy(reg)
    # both directions at once, the D2H into the registered (4 KiB-page) memory, as the fused path runs
    def both_reg(k):
        for _ in range(k):
            with torch.cuda.stream(s1):
                d.copy_(h_in, non_blocking=True)
            with torch.cuda.stream(s2):
                reg_t.copy_(d2, non_blocking=True)

    both_reg(2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    both_reg(5)
    torch.cuda.synchronize()
    emit(what="h2d+d2h_registered", bytes=nbytes, gib_s_each=round(5 * nbytes / (time.perf_counter() - t0) / GIB, 2))
    for name, fn in [("d2h_registered", lambda: reg_t.copy_(d, non_blocking=True)),
                     ("h2d_registered", lambda: d.copy_(reg_t, non_blocking=True))]:
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        emit(what=name, bytes=nbytes, gib_s=round(5 * nbytes / (time.perf_counter() - t0) / GIB, 2))


def fused(sizes, label):
    import tips_amd
    hg = [np.random.default_rng(i).random(k, dtype=np.float32) for i, k in enumerate(sizes)]
    total = sum(sizes) * 4
    for _ in range(2):
        outs = tips_amd._reduce_grads(hg)
    ts = []
    for _ in range(8):
        t0 = time.perf_counter()
        outs = tips_amd._reduce_grads(hg)
        ts.append(time.perf_counter() - t0)
    ok = all(np.array_equal(o, g) for o, g in zip(outs, hg))
    emit(what="reduce_grads_host", label=label, env={k: v for k, v in os.environ.items() if k.startswith("TIPS_HOST")},
         ms=[round(t * 1e3, 3) for t in ts], gib_s_best=round(total / min(ts) / GIB, 2), ok=ok)


VARIANTS = [[("TIPS_HOST_DIRECT_OUT", "0")], [("TIPS_HOST_THREADS", "4")], [("TIPS_HOST_THREADS", "16")],
            [("TIPS_HOST_THREADS", "1")], [("TIPS_HOST_FUSED_PIECE_BYTES", str(4 << 20))],
            [("TIPS_HOST_FUSED_PIECE_BYTES", str(8 << 20))], [("TIPS_HOST_FUSED_PIECE_BYTES", str(32 << 20))]]
# --streams: the second H2D stream against one, at three piece sizes, rounds interleaved
STREAM_VARIANTS = [[]] + [[("TIPS_HOST_H2D_STREAMS", "2")] + ([("TIPS_HOST_FUSED_PIECE_BYTES", str(p))] if p else [])
                          for p in (0, 8 << 20, 32 << 20)] + [[("TIPS_HOST_FUSED_PIECE_BYTES", str(32 << 20))]]


def run_variant(sizes, kv):
    old = {k: os.environ.get(k) for k, _ in kv}
    os.environ.update(dict(kv))
    fused(sizes, ",".join("%s=%s" % x for x in kv) or "default")
    for k, v in old.items():
        if v is None:
            del os.environ[k]
        else:
            os.environ[k] = v


def main():
    import bench
    sizes = bench.resnet50_grad_sizes()
    streams = "--streams" in sys.argv
    if not streams:
        for th in (1, 4, 8, 16):
            memcpy_rate(sum(sizes) * 4, th)
        link_rates(8 << 20)
        link_rates(64 << 20)
    import tips_amd
    tips_amd.init()
    if streams:
        for _ in range(3):
            for kv in STREAM_VARIANTS:
                run_variant(sizes, kv)
    else:
        fused(sizes, "default")
        for kv in VARIANTS:
            run_variant(sizes, kv)
    tips_amd.shutdown()


if __name__ == "__main__":
    main()
