"""negotiation_latency.py — per-tensor cost of the negotiation protocol alone (last note).

This starts p processes on this host. Each one runs tips_negotiation_selftest
(negotiate.cc, dry-run executor: the real TCP lockstep cycles with rank 0, the
validation and the ordering, but no reduction) on the same n named requests.
Every rank enqueues them in its own order, so rank 0 only declares a name
ready once its last rank announces it. The clock starts after a first request
that every rank waits for, so process start-up skew is excluded. The result
is wall time from that point until every request is decided, divided by n.
Two modes are timed:
- "batch": all n requests are in flight at once. This is how gradients
  arrive in a backward pass.
- "serial": each request is waited on before the next one, which gives the
  round-trip latency of a single tensor.
This is the cost the reference pays in coordinator.cc:355-513 over ZeroMQ for
each gradient.

usage: python tools/negotiation_latency.py [--ranks 2,4,8] [--tensors 1000]
"""
import argparse
import json
import multiprocessing as mp
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, size, port, requests, q):
    import ctypes
    from tips_amd import _lib
    L = _lib.dev()  # (include/tips_hip_dev.h)
    out = ctypes.create_string_buffer(1 << 20)
    rc = L.tips_negotiation_selftest(rank, size, b"127.0.0.1", port, requests.encode(), out, len(out))
    log = out.value.decode().splitlines()
    marks = [int(l.split()[-1]) for l in log if l.startswith("# mark")]
    dt = (marks[1] - marks[0]) * 1e-6 if len(marks) == 2 else float("nan")
    q.put((rank, rc, dt, len([l for l in log if l.endswith(" OK")]) - 1))


def measure(p, n, serial):
    names = ["grad.%d" % i for i in range(n)]
    reqs = []
    for r in range(p):
        order = names if (serial or r % 2 == 0) else list(reversed(names))
        sep = "\n@wait\n" if serial else "\n"
        body = sep.join("%s 0 %d" % (nm, 1000 + int(nm.split(".")[1])) for nm in order)
        # a first request every rank waits for lines the ranks up after process start-up skew
        reqs.append("start 0 1\n@wait\n@mark\n" + body + "\n@wait\n@mark")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, p, port, reqs[r], q)) for r in range(p)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=300) for _ in procs]
    for pr in procs:
        pr.join(60)
    assert all(rc == 0 and ok == n for _, rc, _, ok in res), res
    t = max(dt for _, _, dt, _ in res)
    return {"mode": "serial" if serial else "batch", "ranks": p, "tensors": n, "seconds": round(t, 4),
            "per_tensor_us": round(t / n * 1e6, 2),
            "orders": "same order" if serial else "even ranks forward, odd ranks reversed",
            "cycle_time_us": int(os.environ.get("TIPS_CYCLE_TIME_US", "1000"))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--tensors", type=int, default=1000)
    a = ap.parse_args()
    for serial in (False, True):
        for p in [int(x) for x in a.ranks.split(",")]:
            print(json.dumps(measure(p, a.tensors if not serial else min(a.tensors, 200), serial)), flush=True)


if __name__ == "__main__":
    main()
