"""CPU: the library's multi-threaded host code under ThreadSanitizer.

tools/_bin/tsan_selftest links tools/lib/libtips_hip_tsan.so, the product sources with their host
code built -fsanitize=thread (`make tsan`, part of `make all`). Two of the library's concurrent
paths run there, each process with TSAN_OPTIONS halt_on_error=1 exitcode=66, so any data race
the sanitizer sees fails the test with its report:
  - the negotiation (negotiate.cc) across 3 rank processes: the background thread's TCP lockstep
    cycles with rank 0, the completion thread running tips_on_done callbacks, and four issuing
    threads per rank in per-rank shuffled orders (the op-body pattern, INTEGRATION.md §2;
    the reference's coordinator thread and OpRecord callbacks, coordinator.cc:355-513, ops.cc:107-110);
  - the host copy pool of the fused host path (host_staging.cc) under back-to-back runs.
The same instrumented library runs the op-body test over real RCCL ranks on the GPU box
(tools/_bin/op_body_tsan, tests/test_gpu_op_body.py::test_op_body_under_tsan)."""
import os
import random
import socket
import subprocess

import pytest

from conftest import REPO

BIN = os.path.join(REPO, "tools", "_bin", "tsan_selftest")
ENV = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66 second_deadlock_stack=1")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _op_body_scripts(ranks, names, threads, seed, batch=0, steps=1):
    """batch > 0: each thread commits its requests as lists of that many (@batch ... @endbatch,
    Negotiator::enqueue_list) instead of one at a time. steps > 1: the same names again after every
    thread has seen its callbacks (from the second step on through the response cache)."""
    out = []
    for r in range(ranks):
        rnd = random.Random(seed + r)
        body = []
        first = names[:]
        rnd.shuffle(first)
        # a name stays with one thread in every step (a thread's @wait then covers its last
        # instance: a framework never enqueues a name again while its last request is pending)
        owner = {n: k % threads for k, n in enumerate(first)}
        for step in range(steps):
            if step:
                body += ["t%d: @wait" % t for t in range(threads)]
            _op_body_step(body, rnd, first if step == 0 else rnd.sample(names, len(names)), owner, threads, batch)
        body.append("t1: @wait")
        out.append("\n".join(body) + "\n")
    return out


def _op_body_step(body, rnd, order, owner, threads, batch):
    per_thread = [0] * threads
    names = sorted(owner, key=lambda n: int(n[len("layer"):].split("/")[0]))  # (the sizes' index)
    for n in order:
        t = owner[n]
        if batch and per_thread[t] % batch == 0:
            body.append(("t%d: @endbatch\n" % t if per_thread[t] else "") + "t%d: @batch" % t)
        per_thread[t] += 1
        kind = "bc:1" if names.index(n) % 7 == 3 else "ar"
        body.append("t%d: %s %d %d - %s" % (t, n, names.index(n) % 4, 64 + names.index(n), kind))
        if rnd.random() < 0.1 and not batch:
            body.append("t%d: @sleep %d" % (t, rnd.randint(1, 3)))
    if batch:
        body += ["t%d: @endbatch" % t for t in range(threads) if per_thread[t]]


@pytest.mark.parametrize("ranks,seed,batch,steps", [(3, 100, 0, 1), (2, 7, 0, 1), (3, 11, 5, 1), (3, 21, 0, 3)])
def test_negotiation_threads_and_callbacks_race_free(tmp_path, ranks, seed, batch, steps):
    assert os.path.exists(BIN), "tools/_bin/tsan_selftest missing: run make (builds the tsan target)"
    names = ["layer%d/grad" % i for i in range(40)]
    scripts = _op_body_scripts(ranks, names, 4, seed, batch, steps)
    port = _port()
    procs = []
    for r, sc in enumerate(scripts):
        f = tmp_path / ("rank%d.txt" % r)
        f.write_text(sc)
        procs.append(subprocess.Popen([BIN, "neg", str(r), str(ranks), str(port), str(f)], env=ENV,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, o, e))
    for rc, o, e in outs:
        assert "ThreadSanitizer" not in e, e[-4000:]
        assert rc == 0, (rc, e[-2000:])
        assert o.strip().endswith("callbacks %d" % (len(names) * steps)), o[-300:]
    logs = [[l for l in o.splitlines() if l and not l.startswith("#")] for _, o, _ in outs]
    assert all(lg == logs[0] for lg in logs)  # one order on every rank


def test_host_pool_race_free():
    assert os.path.exists(BIN), "tools/_bin/tsan_selftest missing: run make (builds the tsan target)"
    for threads, runs, jobs in ((8, 3000, 16), (3, 3000, 7), (1, 500, 4)):
        p = subprocess.run([BIN, "pool", str(threads), str(runs), str(jobs)], env=ENV, capture_output=True, text=True,
                           timeout=240)
        assert "ThreadSanitizer" not in p.stderr, p.stderr[-4000:]
        assert p.returncode == 0, p.stderr[-2000:]
