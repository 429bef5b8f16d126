"""The negotiation protocol (negotiate.cc; the reference's coordinator, coordinator.cc:15-513) across
real processes on the CPU, with the dry-run executor: ranks enqueue named requests in DIFFERENT orders
and at different times; every rank must execute the same names in the same order (rank 0's
readiness order), mismatches must fail on every rank with the reference's error text, and names
missing on some rank must fail at shutdown."""
import multiprocessing as mp
import socket

import pytest


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, size, port, requests, q, env=None, delay=0.0, stats=None):
    import ctypes
    import os
    import time
    os.environ.update(env or {})  # (the join's test knobs are read once, at the first join)
    time.sleep(delay)
    from tips_amd import _lib
    L = _lib.dev()  # (tips_negotiation_selftest: the development library, tips_hip_dev.h)
    out = ctypes.create_string_buffer(1 << 16)
    rc = L.tips_negotiation_selftest(rank, size, b"127.0.0.1", port, requests.encode(), out, len(out))
    a, b = ctypes.c_int64(), ctypes.c_int64()
    L.tips_net_stats(ctypes.byref(a), ctypes.byref(b))
    res = (rank, rc, out.value.decode(), L.tips_last_error().decode())
    q.put(res + ((a.value, b.value),) if stats else res)


def run(per_rank, port=None, env=None, delay=None, stats=False):
    """Each rank's selftest in its own process; env / delay: per-rank environment and start delay."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = port or _port()
    size = len(per_rank)
    procs = [ctx.Process(target=_worker, args=(r, size, port, per_rank[r], q, (env or {}).get(r),
                                               (delay or {}).get(r, 0.0), stats)) for r in range(size)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(60)
    return res


def lines(log):
    return [l for l in log.splitlines() if l and not l.startswith("#")]


def test_same_order_everywhere_despite_different_enqueue_orders():
    names = ["grad_%d" % i for i in range(40)]
    reqs = []
    for r in range(4):
        order = names[r:] + names[:r] if r % 2 == 0 else list(reversed(names))
        body = []
        for i, n in enumerate(order):
            body.append("%s 0 %d" % (n, 100 + names.index(n)))
            if i % 7 == r:
                body.append("@sleep 3")
        reqs.append("\n".join(body))
    res = run(reqs)
    logs = [lines(log) for _, rc, log, _ in res]
    for rank, rc, log, err in res:
        assert rc == 0, err
    assert all(l == logs[0] for l in logs)
    assert sorted(logs[0]) == sorted(n + " OK" for n in names)


@pytest.mark.parametrize("expect", ["1", "0"])
def test_repeated_steps_with_growing_and_shrinking_sets(expect):
    """Training-shaped steps: the same 30 names every step (the linger ends early once the previous
    batch's names are all in again, TIPS_LINGER_EXPECT), then a step that adds 10 names after them
    on one rank and before them on the other, then a step with a subset, then the full set again.
    Every request of every step runs, in the same order on both ranks."""
    names = ["w%d" % i for i in range(30)]
    extra = ["e%d" % i for i in range(10)]
    reqs = []
    for r in range(2):
        body = []
        for step in range(3):
            order = names if (step + r) % 2 == 0 else list(reversed(names))
            body += ["%s 0 %d" % (n, 64 + names.index(n)) for n in order] + ["@wait"]
        grown = names + extra if r == 0 else extra + names
        body += ["%s 0 %d" % (n, 64 + names.index(n) if n in names else 16 + extra.index(n)) for n in grown]
        body += ["@sleep 2"] if r == 1 else []
        body += ["@wait"]
        body += ["%s 0 %d" % (n, 64 + names.index(n)) for n in names[::3]] + ["@wait"]
        body += ["%s 0 %d" % (n, 64 + names.index(n)) for n in names] + ["@wait"]
        reqs.append("\n".join(body))
    res = run(reqs, env={0: {"TIPS_LINGER_EXPECT": expect}, 1: {"TIPS_LINGER_EXPECT": expect}})
    logs = [lines(log) for _, rc, log, _ in res]
    for rank, rc, log, err in res:
        assert rc == 0, (rank, err)
    assert logs[0] == logs[1]
    want = 3 * len(names) + len(names) + len(extra) + len(names[::3]) + len(names)
    assert len(logs[0]) == want and all(l.endswith(" OK") for l in logs[0])


def cached(log):
    return int([l for l in log.splitlines() if l.startswith("# cached decisions")][0].split()[-1])


@pytest.mark.parametrize("cache", ["1", "0", "mixed"])
def test_response_cache_repeated_steps(cache):
    """The response cache: names decided OK are announced by id from then on, and when every rank
    announced an id by id rank 0 answers without the table. 3 ranks, 40 names, 4 steps, each rank in
    its own order per step: every step runs every name, the same order on every rank; with the cache
    on, steps 2-4 come back cached (one rank with it off: none are, every announce is full)."""
    names = ["w%d" % i for i in range(40)]
    reqs = []
    for r in range(3):
        body = []
        for step in range(4):
            order = names[(7 * r + step) % 40:] + names[:(7 * r + step) % 40]
            if (r + step) % 2:
                order = list(reversed(order))
            body += ["%s 0 %d" % (n, 16 + names.index(n)) for n in order] + ["@wait"]
        reqs.append("\n".join(body))
    env = {r: {"TIPS_RESPONSE_CACHE": "0" if cache == "0" or (cache == "mixed" and r == 1) else "1"}
           for r in range(3)}
    res = run(reqs, env=env)
    for rank, rc, log, err in res:
        assert rc == 0, (rank, err)
    logs = [lines(log) for _, _, log, _ in res]
    assert logs[0] == logs[1] == logs[2]
    assert sorted(logs[0]) == sorted(n + " OK" for n in names * 4)
    hits = [cached(log) for _, _, log, _ in res]
    assert len(set(hits)) == 1
    if cache == "1":
        assert hits[0] >= 2 * 40, hits  # (step 1 decides in full; a cycle may take a step's first names early)
    else:
        assert hits[0] == 0


def test_response_cache_shape_change_fails_everywhere_then_recaches():
    """A cached name whose shape changes on one rank travels in full from that rank; rank 0 puts
    the other ranks' id announces of it through the table, which fails it on every rank with the
    reference's text (coordinator.cc:134-150). The failure drops it from the cache; the next step
    with the new shape on every rank succeeds, then comes back cached."""
    steps = {0: [8, 8, 8, 9, 9, 9], 1: [8, 8, 9, 9, 9, 9]}
    reqs = []
    for r in range(2):
        body = []
        for k, n in enumerate(steps[r]):
            body += ["w 0 %d" % n, "b%d 0 4" % k, "@wait"]
        reqs.append("\n".join(body))
    res = run(reqs)
    for rank, rc, log, err in res:
        assert rc == 0, (rank, err)
    logs = [lines(log) for _, _, log, _ in res]
    assert logs[0] == logs[1]
    w = [l for l in logs[0] if l.startswith("w ")]
    assert w[:2] == ["w OK", "w OK"]
    assert w[2] == "w ERR Mismatched allreduce tensor shapes: [8] vs [9]"
    assert w[3:] == ["w OK"] * 3
    assert cached(res[0][2]) >= 2  # (steps 2 and 6 at least: w by id on both ranks)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_response_cache_random_steps(seed):
    """Random training-like steps over a pool of names, 3 ranks in their own orders: each step
    enqueues a random subset on every rank; sometimes one rank changes a name's shape, or every
    rank issues a name as a broadcast instead. A name must come out OK in every step where all
    ranks agreed and fail in the step where they did not, the same on every rank, whether its
    earlier steps were decided in full or from the response cache."""
    import random
    rng = random.Random(seed)
    pool = ["p%d" % i for i in range(24)]
    steps = []
    for s in range(6):
        names = rng.sample(pool, rng.randint(8, 24))
        odd = rng.choice(names) if rng.random() < 0.6 else None  # one rank's shape differs
        bc = rng.choice([n for n in names if n != odd]) if rng.random() < 0.4 else None  # all: broadcast
        steps.append((names, odd, bc))
    reqs = []
    for r in range(3):
        body = []
        for names, odd, bc in steps:
            order = names[:]
            random.Random(seed * 100 + r).shuffle(order)
            for n in order:
                count = 32 + pool.index(n) + (1 if (n == odd and r == 2) else 0)
                body.append("%s 0 %d - %s" % (n, count, "bc:0" if n == bc else "ar"))
            body.append("@wait")
        reqs.append("\n".join(body))
    res = run(reqs)
    for rank, rc, log, err in res:
        assert rc == 0, (rank, err)
    logs = [lines(log) for _, _, log, _ in res]
    assert logs[0] == logs[1] == logs[2]
    got = {}
    for l in logs[0]:
        n, rest = l.split(" ", 1)
        got.setdefault(n, []).append(rest)
    want = {}
    for names, odd, bc in steps:
        for n in names:
            want.setdefault(n, []).append("ERR" if n == odd else "OK")
    assert set(got) == set(want)
    for n in want:
        assert [g.split(" ")[0] for g in got[n]] == want[n], (n, got[n], want[n])
    assert cached(res[0][2]) > 0


def test_list_commits_mixed_with_single_requests():
    """Lists committed under one lock hold (Negotiator::enqueue_list, as tips_enqueue_allreduce_n):
    3 ranks, each a different mix of lists and single requests in its own order, one rank's list
    carrying a shape mismatch, and executor threads enqueueing lists beside the main thread; every
    rank runs the same names in the same order, the mismatch fails everywhere, the rest succeed."""
    names = ["g%d" % i for i in range(60)]
    reqs = []
    for r in range(3):
        order = names[r * 7:] + names[:r * 7]
        if r == 1:
            order = list(reversed(order))
        body = []
        for i, n in enumerate(order):
            if i % 10 == 0:
                body.append(("@endbatch\n" if i else "") + "@batch")
            count = 200 + names.index(n)
            if n == "g13" and r == 2:
                count += 1  # shape mismatch on one rank only
            body.append("%s 0 %d" % (n, count))
        body.append("@endbatch")
        if r == 0:  # a second thread's lists beside the main thread's
            body += ["t1: @batch"] + ["t1: x%d 0 8" % k for k in range(20)] + ["t1: @endbatch", "t1: @wait"]
        else:
            body += ["@batch"] + ["x%d 0 8" % k for k in range(19, -1, -1)] + ["@endbatch"]
        body.append("@wait")
        reqs.append("\n".join(body))
    res = run(reqs)
    logs = [[l for l in lines(log) if not l.startswith("callbacks")] for _, _, log, _ in res]
    for rank, rc, log, err in res:
        assert rc == 0, (rank, err)
    assert logs[0] == logs[1] == logs[2]
    got = dict(l.split(" ", 1) for l in logs[0])
    assert got["g13"].startswith("ERR Mismatched allreduce tensor shapes")
    assert all(got[n] == "OK" for n in names if n != "g13") and all(got["x%d" % k] == "OK" for k in range(20))


def test_mismatch_fails_everywhere_with_reference_text():
    reqs = ["a 0 8\nb 0 8\nc 0 8", "c 0 8\nb 1 8\na 0 9"]  # b: dtype mismatch; a: shape mismatch
    res = run(reqs)
    logs = [lines(log) for _, _, log, _ in res]
    assert logs[0] == logs[1]
    got = dict(l.split(" ", 1) for l in logs[0])
    assert got["c"] == "OK"
    assert got["b"] == "ERR Mismatch data types found: 0 vs 1."
    assert got["a"] == "ERR Mismatched allreduce tensor shapes: [8] vs [9]"


def test_missing_on_one_rank_fails_at_shutdown():
    res = run(["x 0 4\nonly0 0 4", "x 0 4"])
    for _, rc, log, _ in res:
        assert rc == 0
    l0 = dict(l.split(" ", 1) for l in lines(res[0][2]))
    assert l0["x"] == "OK"
    assert l0["only0"].startswith("ERR request only0 was not enqueued on every rank")
    assert lines(res[1][2]) == ["x OK"]


def test_single_rank_and_duplicate_names():
    res = run(["a 3 5\nb 3 5"])
    assert lines(res[0][2]) == ["a OK", "b OK"]


def test_readiness_order():
    """A name runs when its LAST rank announces it (ready_to_reduce, coordinator.cc:451-455): rank 1
    holds `a` back for 300 ms, so `b` (announced by both at once) is reduced first on every rank."""
    res = run(["a 0 4\nb 0 4", "b 0 4\n@sleep 300\na 0 4"])
    for _, rc, log, err in res:
        assert rc == 0, err
        assert lines(log) == ["b OK", "a OK"]


def test_shape_mismatch_with_equal_counts_fails_everywhere():
    """The negotiated path carries each tensor's shape (tips_enqueue_allreduce_shaped): [2,4] on
    rank 0 and [4,2] on rank 1 have equal element counts, and must still fail on every rank with
    ConstructResponseMessage's text (reference coordinator.cc:129-146, message at :142-143)."""
    res = run(["w 0 8 2,4\nv 0 6 3,2\nok 0 8 2,4", "ok 0 8 2,4\nv 0 6 3,2\nw 0 8 4,2"])
    logs = [dict(l.split(" ", 1) for l in lines(log)) for _, _, log, _ in res]
    for rank, rc, _, err in res:
        assert rc == 0, err
    for got in logs:
        assert got["w"] == "ERR Mismatched allreduce tensor shapes: [2,4] vs [4,2]"
        assert got["v"] == "OK" and got["ok"] == "OK"


def test_shape_rank_and_scalar():
    """Shapes of different rank fail with the reference's TensorShape text; a scalar announces [1]."""
    res = run(["a 0 4 4\nb 0 1 1\nc 1 4 4", "a 0 4 4,1\nb 0 1\nc 1 4 2,2"])
    for _, _, log, _ in res:
        got = dict(l.split(" ", 1) for l in lines(log))
        assert got["a"] == "ERR Mismatched allreduce tensor shapes: [4] vs [4,1]"
        assert got["b"] == "OK"
        assert got["c"] == "ERR Mismatched allreduce tensor shapes: [4] vs [2,2]"


def test_broadcast_and_allgather_requests():
    """Named broadcast and allgather requests (the reference's RequestType_BROADCAST / _ALLGATHER,
    coordinator.cc:129-186, 40-88) through the same negotiation, mixed with allreduces, enqueued in
    different orders: rank 0 applies each type's rule and every rank logs the same verdicts in the
    same order; an allgather's decision carries every rank's first dimension (tensor_sizes)."""
    r0 = ("g 0 12 3,4 ag\n"            # allgather: rows 3 / 5 / 1, 4 columns everywhere -> sizes 3,5,1
          "b 0 6 2,3 bc:1\n"           # broadcast from rank 1, same shape everywhere
          "s 0 8 2,4 ag\n"             # allgather: second dimension differs on rank 2
          "bs 0 8 2,4 bc:0\n"          # broadcast: shapes differ on rank 1
          "br 1 4 - bc:0\n"            # broadcast: roots differ on rank 2
          "ak 0 5 - ag\n"              # allgather of 1-d tensors of 5 / 2 / 0 rows
          "op 0 4 - ar\n"              # allreduce on ranks 0, 1 and allgather on rank 2
          "x 0 10")
    r1 = ("x 0 10\nak 0 2 - ag\nop 0 4 - ar\nbr 1 4 - bc:0\nbs 0 8 4,2 bc:0\ns 0 8 2,4 ag\nb 0 6 2,3 bc:1\n"
          "g 0 20 5,4 ag")
    r2 = ("op 0 4 - ag\nb 0 6 2,3 bc:1\ng 0 4 1,4 ag\nbr 1 4 - bc:2\nak 0 0 - ag\ns 0 6 2,3 ag\nbs 0 8 2,4 bc:0\n"
          "x 0 10")
    res = run([r0, r1, r2])
    logs = [lines(log) for _, _, log, _ in res]
    for _, rc, _, err in res:
        assert rc == 0, err
    assert logs[0] == logs[1] == logs[2]
    got = dict(l.split(" ", 1) for l in logs[0])
    assert got["g"] == "OK sizes=3,5,1"
    assert got["ak"] == "OK sizes=5,2,0"
    assert got["b"] == "OK" and got["x"] == "OK"
    assert got["s"] == "ERR Mismatched allgather tensor shapes: 1-th dimension 4 vs 3"
    assert got["bs"] == "ERR Mismatched broadcast tensor shapes: [2,4] vs [4,2]"
    assert got["br"] == "ERR Mismatched broadcast root ranks: 0 vs 2"
    assert got["op"] == "ERR Mismatched operations found: 0 vs 1."


def test_foreign_listener_on_the_negotiation_port():
    """Another program already listens on the negotiation port and accepts but never answers (as an
    RCCL socket in the same ephemeral range can): rank 0 takes the next free port, the other ranks'
    hello gets no answer there and they move on to rank 0's; every rank runs every request."""
    foreign = socket.socket()
    foreign.bind(("127.0.0.1", 0))
    foreign.listen(8)
    try:
        res = run(["a 0 10\nb 0 20", "b 0 20\na 0 10", "a 0 10\nb 0 20"], port=foreign.getsockname()[1])
    finally:
        foreign.close()
    logs = [lines(log) for _, rc, log, _ in res]
    for rank, rc, log, err in res:
        assert rc == 0, err
    assert all(l == logs[0] for l in logs) and sorted(logs[0]) == ["a OK", "b OK"]


def test_op_body_threads_with_callbacks():
    """The op-body pattern of INTEGRATION.md §2 without a GPU: on every rank four threads (a
    framework's executor threads) issue named requests, each thread in its own order and each rank
    in a different shuffle, and every request completes through a tips_on_done callback (the
    reference's OpRecord callback, ops.cc:107-110, coordinator_test.cc:10-45). Every rank executes
    the same names in the same order, and every callback fires exactly once."""
    import random
    names = ["layer%d/grad" % i for i in range(48)]
    reqs = []
    for r in range(3):
        rnd = random.Random(100 + r)
        order = names[:]
        rnd.shuffle(order)
        body = []
        for k, n in enumerate(order):
            t = k % 4
            body.append("t%d: %s 0 %d" % (t, n, 64 + names.index(n)))
            if rnd.random() < 0.1:
                body.append("t%d: @sleep %d" % (t, rnd.randint(1, 5)))
        body.append("t2: @wait")
        reqs.append("\n".join(body))
    res = run(reqs)
    logs = [lines(log) for _, _, log, _ in res]
    for rank, rc, log, err in res:
        assert rc == 0, err
        assert log.strip().endswith("callbacks %d" % len(names)), log[-200:]
    assert logs[0] == logs[1] == logs[2]
    assert sorted(l for l in logs[0] if not l.startswith("callbacks")) == sorted(n + " OK" for n in names)


def test_op_body_callbacks_carry_errors():
    """A callback reports a request's failure: a shape mismatch fails on every rank through its
    callback, the other requests of the same threads still complete."""
    r0 = "t1: a 0 8 2,4\nt2: b 0 4\nt1: c 0 4"
    r1 = "t2: c 0 4\nt1: a 0 8 4,2\nt1: b 0 4"
    res = run([r0, r1])
    for _, rc, log, err in res:
        assert rc == 0, err
        got = dict(l.split(" ", 1) for l in lines(log))
        assert got["a"] == "ERR Mismatched allreduce tensor shapes: [2,4] vs [4,2]"
        assert got["b"] == "OK" and got["c"] == "OK" and got["callbacks"] == "3"


def test_start_refused_when_sync_counts_differ():
    """Every synchronous collective issued before the negotiation starts must have its partner on
    every rank: rank 1 claims one more than rank 0, so the join's verdict fails every rank's start
    with both numbers (instead of pairing rank 1's later RCCL calls with the wrong ones)."""
    res = run(["@synccount 2\na 0 4", "@synccount 3\na 0 4"])
    for rank, rc, log, err in res:
        assert rc == -7, (rank, rc, err)
        assert "rank 1 issued 3 synchronous collectives before the negotiation started, rank 0 issued 2" in err


def test_join_survives_connecting_to_itself():
    """Rank 1 starts first and its first attempts are bound to the port they connect to
    (TIPS_TEST_SELF_CONNECT: TCP simultaneous open with itself, deterministic), before rank 0
    listens: each such socket must be dropped (tips_net_stats counts them) and the join must still
    complete. Without the check the socket would read its own hello back as rank 0's answer."""
    res = run(["a 0 4\nb 0 8", "b 0 8\na 0 4"], env={1: {"TIPS_TEST_SELF_CONNECT": "3"}}, delay={0: 1.0}, stats=True)
    for rank, rc, log, err, st in res:
        assert rc == 0, err
        assert sorted(lines(log)) == ["a OK", "b OK"]
    assert res[1][4][0] >= 1, res[1][4]  # rank 1 refused at least one connection to itself


def test_join_counts_a_rank_only_once_it_confirms():
    """Rank 1 abandons its first connection right after its hello (TIPS_TEST_DROP_FIRST_HELLO, as a
    rank whose answer did not come in time): rank 0 must not count that connection as joined (it
    waits for the rank's confirmation) and must take the rank's next connection."""
    res = run(["a 0 4", "a 0 4", "a 0 4"], env={1: {"TIPS_TEST_DROP_FIRST_HELLO": "1"}}, stats=True)
    for rank, rc, log, err, st in res:
        assert rc == 0, err
        assert lines(log) == ["a OK"]
    assert res[0][4][1] >= 1, res[0][4]  # rank 0 dropped at least one unconfirmed connection


def test_debug_state_reports_the_threads():
    """tips_debug_state (the hang report op_body's watchdog prints): while a one-rank dry-run
    negotiation runs a script with a pause in it, another thread reads a line naming the
    background thread's phase, the cycle count and the queues; outside a negotiation it says so."""
    import ctypes
    import threading
    import time
    from tips_amd import _lib
    L = _lib.dev()  # (tips_negotiation_selftest: the development library, tips_hip_dev.h)
    b = ctypes.create_string_buffer(4096)
    assert L.tips_debug_state(b, len(b)) == 0 and b.value == b"no negotiation"
    out = ctypes.create_string_buffer(1 << 16)
    rc = []
    t = threading.Thread(target=lambda: rc.append(L.tips_negotiation_selftest(
        0, 1, b"127.0.0.1", _port(), b"a 0 4\n@sleep 400\nb 0 8\n@wait", out, len(out))))
    t.start()
    seen = []
    deadline = time.time() + 20
    while t.is_alive() and time.time() < deadline:
        L.tips_debug_state(b, len(b))
        seen.append(b.value.decode())
        time.sleep(0.02)
    t.join(30)
    assert rc == [0], _lib.last_error()
    live = [s for s in seen if s.startswith("rank 0 cycles")]
    assert live, seen[:3]
    assert all("| negotiation: " in s and "| completion: " in s for s in live)
    assert any(" pending " in s for s in live)


def _stop_race_worker(gap_us, q):
    import ctypes
    import os
    os.environ["TIPS_TEST_ENQUEUE_GAP_US"] = str(gap_us)  # (read once, at the process's first enqueue)
    from tips_amd import _lib
    L = _lib.dev()
    out = []
    for stop_us in (0, 100, 1000, 3000):
        res = (ctypes.c_int64 * 4)()
        rc = L.tips_negotiation_stop_race_selftest(4, 50 if gap_us else 2000, stop_us, 3, _port(), res)
        out.append((stop_us, rc, list(res), L.tips_last_error().decode()))
    q.put(out)


@pytest.mark.parametrize("gap_us", [0, 300])
def test_enqueue_with_callbacks_races_a_stop(gap_us):
    """the lock-free enqueue checked that the negotiation accepts requests, then pushed
    its node; a stop() whose last drain fell between the two left the node unadmitted, and a
    tips_enqueue_allreduce_cb caller, already holding a handle, never saw its callback. Four threads
    enqueue callback requests while the negotiation stops; once stop() and the enqueues have
    returned, every accepted request must have been called back exactly once and no refused one.
    gap_us = 300 sleeps between the check and the push (TIPS_TEST_ENQUEUE_GAP_US) so that many
    enqueues straddle the stop: without the re-check after the push, 16-20 of ~20-60 accepted
    requests per point were never called back."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_stop_race_worker, args=(gap_us, q))
    p.start()
    out = q.get(timeout=240)
    p.join(60)
    for stop_us, rc, (accepted, called, wrong, refused), err in out:
        assert rc == 0 and wrong == 0, (stop_us, rc, accepted, called, wrong, err)
        assert called == accepted and accepted + refused == 4 * 3 * (50 if gap_us else 2000)
