"""Host-side checkers of the schedules' op plans (tips_schedule_plan, tips_amd/csrc/plan.cc).

The RCCL executor and the single-GPU simulator both run these plans, so what is
checked here is what runs on an 8-GPU node:

- pairing():  in every step, the k-th send from r to q has the k-th receive on q
  from r, with equal bytes, and no receive is left over. Every rank issues the
  same number of steps, each one ncclGroupStart/End, so with pairing inside a
  step no group can wait on a partner that never comes (deadlock freedom).
- hazards():  a happens-before model of the executor's streams and events
  (schedules.cc run_plan: prologue, per-step comm waits, recv / sum events,
  epilogue), for two back-to-back calls issued from two DIFFERENT user streams.
  Every pair of accesses to one buffer range where one is a write must be ordered
  (a data race otherwise), and every access of a call must be ordered before the
  user's next work on that call's stream.
- interpret(): executes p ranks' plans on numpy buffers, with the oracle's sum2 /
  rank-order fold as the arithmetic, so the plans' index arithmetic can be compared
  bit for bit with oracle_ring / oracle_fold on a host without a GPU.
"""
import ctypes

import numpy as np

IN, OUT, STG = 0, 1, 2
RING, DIRECT, ONESHOT = 0, 1, 3


def dump(algo, p, rank, n, dtype, depth=0):
    from tips_amd import _lib
    L = _lib.dev()
    need = L.tips_schedule_plan(algo, p, rank, n, dtype, depth, None, 0)
    assert need > 0, _lib.last_error()
    buf = (ctypes.c_int64 * need)()
    assert L.tips_schedule_plan(algo, p, rank, n, dtype, depth, buf, need) == need
    return parse(list(buf))


def parse(w):
    nsteps, staging, K = w[0], w[1], w[2]
    i = 3
    steps = []
    for _ in range(nsteps):
        wait_sum, nx, ns = w[i:i + 3]
        i += 3
        xfers = []
        for _ in range(nx):
            send, peer, buf, off, nb = w[i:i + 5]
            i += 5
            xfers.append(dict(send=bool(send), peer=peer, buf=buf, off=off, bytes=nb))
        sums = []
        for _ in range(ns):
            dbuf, doff, count, nsrc = w[i:i + 4]
            i += 4
            srcs = [(w[i + 2 * j], w[i + 2 * j + 1]) for j in range(nsrc)]
            i += 2 * nsrc
            sums.append(dict(dst=(dbuf, doff), count=count, srcs=srcs))
        steps.append(dict(wait_sum=wait_sum, xfers=xfers, sums=sums))
    assert i == len(w)
    return dict(steps=steps, staging=staging, K=K)


def pairing(plans):
    """Raise AssertionError unless every send pairs with a receive of equal bytes in the same step."""
    p = len(plans)
    nsteps = len(plans[0]["steps"])
    assert all(len(pl["steps"]) == nsteps for pl in plans), "ranks issue different numbers of groups"
    for i in range(nsteps):
        recvs = {}  # (receiver, sender) -> list of byte counts, in issue order
        sends = {}
        for r in range(p):
            for x in plans[r]["steps"][i]["xfers"]:
                assert 0 <= x["peer"] < p and x["peer"] != r, (i, r, x)
                assert x["bytes"] > 0, (i, r, x)
                if x["send"]:
                    sends.setdefault((x["peer"], r), []).append(x["bytes"])
                else:
                    recvs.setdefault((r, x["peer"]), []).append(x["bytes"])
        assert sends == recvs, "step %d: sends %s vs receives %s" % (i, sends, recvs)


def _ranges_overlap(a, b):
    return a[0] < b[1] and b[0] < a[1]


def hazards(plan, es, nbytes, inplace=False, modes=("eager", "eager"), replay_joins=True, lanes=1,
            cross_lane_waits=True):
    """Happens-before check of one rank's plan over back-to-back calls from alternating user
    streams, each call eager (schedules.cc prologue / steps / epilogue) or a replay of the captured
    plan (TIPS_GRAPHS: a graph launched on graph_stream, its nodes on streams of their own, ordered
    only by the graph's edges and by graph_stream's order).
    lanes > 1: eager step i's transfers go to lane i % lanes, each lane its own stream (and RCCL
    communicator); at entry lane 0 waits for the caller, the queued sums and every lane's queued
    transfers, and the other lanes wait for lane 0; at exit the caller waits for every lane.
    Returns a list of race descriptions (empty = race-free). nbytes = bucket bytes."""
    ops = []     # (stream, accesses) ; accesses = [(buffer_id, lo, hi, is_write)]
    preds = []   # explicit cross-stream predecessors (event waits) per op
    last = {}    # stream -> index of its last op
    pending_waits = {}  # stream -> list of op indices the next op on that stream must follow

    def add(stream, acc=()):
        idx = len(ops)
        ops.append((stream, list(acc)))
        pr = []
        if stream in last:
            pr.append(last[stream])
        pr += pending_waits.pop(stream, [])
        preds.append(pr)
        last[stream] = idx
        return idx

    def record(stream):  # an event recorded on `stream` covers its last op (a marker op keeps it explicit)
        return add(stream)

    def wait(stream, ev_op):
        pending_waits.setdefault(stream, []).append(ev_op)

    def buf_id(call, buf):
        if buf == STG:
            return "stg"
        if inplace:
            return ("io", call)
        return ("in" if buf == IN else "out", call)

    def conflict(a, b):  # (the executor compares addresses: in place, in and out are one buffer)
        return any((not x["send"] or not y["send"]) and buf_id(0, x["buf"]) == buf_id(0, y["buf"]) and
                   _ranges_overlap((x["off"], x["off"] + x["bytes"]), (y["off"], y["off"] + y["bytes"]))
                   for x in a["xfers"] for y in b["xfers"])

    def steps(call, Cs, P):
        sum_ev = {}
        group_op = {}
        nl = len(Cs)
        for i, s in enumerate(plan["steps"]):
            C = Cs[i % nl]
            if s["wait_sum"] >= 0 and s["wait_sum"] in sum_ev:
                wait(C, sum_ev[s["wait_sum"]])
            if nl > 1 and cross_lane_waits:  # schedules.cc issue_steps: the latest conflicting step on each other lane
                for lane in range(nl):
                    if lane == i % nl:
                        continue
                    for j in range(i - 1, -1, -1):
                        if j % nl == lane and conflict(plan["steps"][j], s):
                            wait(C, group_op[j])
                            break
            if s["xfers"]:
                acc = [(buf_id(call, x["buf"]), x["off"], x["off"] + x["bytes"], not x["send"]) for x in s["xfers"]]
                group_op[i] = add(C, acc)
            else:
                group_op[i] = record(C)
            if s["sums"]:
                rev = record(C)
                wait(P, rev)
                for u in s["sums"]:
                    acc = [(buf_id(call, u["dst"][0]), u["dst"][1], u["dst"][1] + u["count"] * es, True)]
                    acc += [(buf_id(call, b), o, o + u["count"] * es, False) for b, o in u["srcs"]]
                    add(P, acc)
                sum_ev[i] = record(P)

    ends = []
    graph_pending = eager_pending = False
    for call, mode in enumerate(modes):
        user = "U%d" % (call % 2)
        add(user, [(buf_id(call, IN), 0, nbytes, True)] + ([] if inplace else [(buf_id(call, OUT), 0, nbytes, True)]))
        if mode == "eager":
            if graph_pending:  # order_after_replays
                ev = record("G")
                wait("C", ev)
                wait("P", ev)
                graph_pending = False
            ev_start = record(user)
            wait("C", ev_start)
            ev_prev = record("P")
            wait("C", ev_prev)
            lane_names = ["C"] + ["C%d" % l for l in range(1, lanes)]
            for ln in lane_names[1:]:  # lane 0 after every lane's queued transfers
                wait("C", record(ln))
            if lanes > 1:
                e0 = record("C")
                for ln in lane_names[1:]:
                    wait(ln, e0)
            wait("P", ev_start)
            eager_pending = True
            steps(call, lane_names, "P")
            for ln in lane_names:
                wait(user, record(ln))
            e2 = record("P")
            wait(user, e2)
        else:  # replay
            wait("G", record(user))
            if eager_pending and replay_joins:  # (replay_joins=False: the checker's own test)
                wait("G", record("C"))
                wait("G", record("P"))
                eager_pending = False
            fork = add("G")  # the graph's root: after everything before it on graph_stream
            C, P = "GC%d" % call, "GP%d" % call  # the graph's nodes run on streams of their own
            wait(C, fork)
            wait(P, fork)
            steps(call, [C], P)
            wait("G", record(C))
            wait("G", record(P))
            add("G")  # the graph's end: before anything later on graph_stream
            wait(user, record("G"))
            graph_pending = True
        # the user's next work on this stream reads and writes this call's buffers
        ends.append(add(user, [(buf_id(call, IN), 0, nbytes, True), (buf_id(call, OUT), 0, nbytes, True)]))

    # reachability: bitset of ancestors per op (ops are created in topological order)
    anc = []
    for i in range(len(ops)):
        a = 0
        for q in preds[i]:
            a |= anc[q] | (1 << q)
        anc.append(a)

    def ordered(i, j):
        return bool(anc[j] >> i & 1) or bool(anc[i] >> j & 1)

    races = []
    flat = [(i, a) for i, (_, acc) in enumerate(ops) for a in acc]
    by_buf = {}
    for i, a in flat:
        by_buf.setdefault(a[0], []).append((i, a))
    for buf, lst in by_buf.items():
        for x in range(len(lst)):
            i, a = lst[x]
            for y in range(x + 1, len(lst)):
                j, b = lst[y]
                if i == j or not (a[3] or b[3]) or not _ranges_overlap(a[1:3], b[1:3]):
                    continue
                if not ordered(i, j):
                    races.append("%s [%d,%d)%s on %s vs [%d,%d)%s on %s" % (
                        buf, a[1], a[2], "w" if a[3] else "r", ops[i][0], b[1], b[2], "w" if b[3] else "r", ops[j][0]))
                    if len(races) > 20:
                        return races
    return races


def sums_under_transfers(plan):
    """One eager call's happens-before graph (schedules.cc issue_steps: step i's group on the comm
    stream behind its wait on an earlier step's sums, step i's sums on the compute stream behind
    step i's receive event). Returns {i: [j, ...]}: the steps j > i whose transfer group is NOT
    ordered after step i's sums, i.e. may run on the links while those sums run on the CUs."""
    steps = plan["steps"]
    group_after_sum = {}  # j -> set of sum steps the group of j is ordered after (transitively)
    sum_after = {}        # i -> set of sum steps the sums of i follow (stream order + their group)
    prev_group = set()
    prev_sums = set()
    for j, s in enumerate(steps):
        g = set(prev_group)  # the comm stream's order: everything the previous group followed
        if s["wait_sum"] >= 0:
            g |= {s["wait_sum"]} | sum_after.get(s["wait_sum"], set())
        group_after_sum[j] = g
        prev_group = g
        if s["sums"]:
            sa = prev_sums | g  # compute stream's order + this step's receive event
            sum_after[j] = sa
            prev_sums = sa | {j}
    return {i: [j for j in range(i + 1, len(steps)) if steps[j]["xfers"] and i not in group_after_sum[j]]
            for i in sum_after}


def interpret(plans, ins, dtype, inplace=False):
    """Execute p ranks' plans on host buffers: step by step, transfers first (paired as
    pairing() checks), then the step's sums with the oracle's arithmetic. Returns p outputs."""
    import oracle_bind
    p = len(plans)
    ins = [np.ascontiguousarray(x).copy() for x in ins]
    es = ins[0].itemsize
    nbytes = ins[0].nbytes
    outs = ins if inplace else [np.zeros_like(x) for x in ins]
    stg = [np.zeros(max(1, pl["staging"]), np.uint8) for pl in plans]

    def raw(r, buf):
        if buf == STG:
            return stg[r]
        return (ins if buf == IN else outs)[r].view(np.uint8)

    def view(r, buf, off, count):
        return raw(r, buf)[off:off + count * es].view(ins[0].dtype)

    for i in range(len(plans[0]["steps"])):
        moves = []
        for r in range(p):
            nth = {}
            for x in plans[r]["steps"][i]["xfers"]:
                if not x["send"]:
                    continue
                q = x["peer"]
                k = nth.get(q, 0)
                nth[q] = k + 1
                rv = [y for y in plans[q]["steps"][i]["xfers"] if not y["send"] and y["peer"] == r][k]
                moves.append((raw(r, x["buf"])[x["off"]:x["off"] + x["bytes"]].copy(), q, rv))
        for data, q, rv in moves:  # all of a step's sends read before any of its receives land
            raw(q, rv["buf"])[rv["off"]:rv["off"] + rv["bytes"]] = data
        for r in range(p):
            for u in plans[r]["steps"][i]["sums"]:
                srcs = [view(r, b, o, u["count"]).copy() for b, o in u["srcs"]]
                if len(srcs) == 2:
                    res = oracle_bind.sum2(srcs[0], srcs[1], code=dtype)
                else:
                    res = oracle_bind.fold(srcs, code=dtype, wide_acc=True)
                view(r, u["dst"][0], u["dst"][1], u["count"])[:] = res
    return outs


def proxy_order(calls, host_wait="end"):
    """RCCL's proxy thread works through the operations of one communicator in the order they are
    POSTED; the device runs the groups in stream order. A replayed plan's group posts its
    operations from a host node of the graph when the device reaches that group; an eager group
    posts them when the host issues it. `calls` = [("replay" | "eager", number of groups)] in
    issue order; the device is taken to lag the host as far as it can (it runs nothing until the
    host waits for it). host_wait is what schedules.cc order_after_replays does before an eager
    call while a replay is pending: "end" (wait until the replay has run), "start" (until its first
    group has begun) or "none". Returns (posting order, device order) of (call, group) pairs: a
    schedule is safe when they are equal (else the proxy waits on work the device has not reached
    while the device waits on the proxy - the hang of profiles/r03/k_op_body_hang.txt)."""
    from collections import deque
    device = [(c, k) for c, (_, ng) in enumerate(calls) for k in range(ng)]
    posted, deferred = [], deque()  # deferred: replay groups the device has not reached, device order
    for c, (mode, ng) in enumerate(calls):
        if mode == "replay":
            deferred.extend((c, k) for k in range(ng))
            continue
        if deferred and host_wait == "end":
            while deferred:
                posted.append(deferred.popleft())
        elif deferred and host_wait == "start":
            last = deferred[-1][0]  # the pending replay: the device has reached its first group
            while deferred and (deferred[0][0] < last or deferred[0] == (last, 0)):
                posted.append(deferred.popleft())
        posted.extend((c, k) for k in range(ng))
    posted.extend(deferred)
    return posted, device


def replay_trace(rounds, sizes, cap=2 << 20, mixed_cap=1 << 30, note_on_wait=True, fail_bytes=0):
    """schedules.cc's replay bookkeeping over `rounds` rounds of calls on the same buffers, one per
    entry of `sizes` (bytes) in order: graph_eligible (bytes <= cap, or <= mixed_cap once a host wait
    has happened; mixed_cap = 0 keeps cap), plan_graph (a key's first eligible call only records it,
    its next is captured and replayed), run_plan's staging growth (a larger plan than any before drops
    every key) and order_after_replays (an eager call after a replay waits on the host; a wait that
    widens the limit records the call's key as seen; fail_bytes > 0: the capture of a plan of at
    least that many bytes fails, and that key alone runs eagerly from then on). Returns
    [(trace token, mode)] per call, tokens as tests/peer_worker.py graphs_case prints them ("w" a host
    wait, "r" a replay, "c" a capture, "-" none) and mode "replay" | "eager" for proxy_order."""
    keys, staging, pending, mixed, out, failed = {}, 0, False, False, [], set()
    for _ in range(rounds):
        for i, b in enumerate(sizes):
            if b > staging:
                staging = b
                keys.clear()
                failed.clear()
            limit = max(cap, mixed_cap) if mixed else cap
            replay = captured = False
            if b <= limit and i not in failed:
                if i not in keys:
                    keys[i] = False
                elif not keys[i] and fail_bytes and b >= fail_bytes:
                    failed.add(i)  # the capture failed: eager now and from now on
                else:
                    captured, keys[i] = not keys[i], True
                    replay = True
            if replay:
                pending = True
                out.append(("r" + ("c" if captured else ""), "replay"))
            else:
                out.append(("w" if pending else "-", "eager"))
                mixed = mixed or pending
                pending = False
                if note_on_wait and b > limit and b <= (max(cap, mixed_cap) if mixed else cap):
                    keys.setdefault(i, False)  # the wait widened the limit: seen (run_plan's note_only)
    return out
