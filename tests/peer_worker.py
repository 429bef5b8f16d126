"""One rank of the peer schedule's multi-process test (tests/test_gpu_peer.py).

Run as: python peer_worker.py RANK SIZE UID_HEX CASES_JSON
Every rank of the job runs on GPU 0 of the test box. Two transports:
- TIPS_WORKER_ALGO=peer (default): TIPS_NO_RCCL=1, no RCCL communicator. The
  ranks share nothing but the IPC workspaces and the node-local control block,
  exactly as on an 8-GPU node, so this exercises the whole peer path: the
  shared-memory barriers, the handle exchange, the push / fold / pull kernels
  and the cross-rank count check.
- TIPS_WORKER_ALGO=ring|direct|oneshot|auto: a real RCCL communicator per
  process (tips_init: unique id over the TCP bootstrap, ncclCommInitRank). RCCL
  refuses two ranks on one GPU of one host, so each process claims its own host
  (NCCL_HOSTID=rank) and RCCL connects them with its socket transport over
  loopback: slow, but the per-rank RCCL executor (schedules.cc run_plan) runs
  exactly as on the node - same plans, groups, streams and events. Each case's inputs are seeded per
rank; every rank regenerates all ranks' inputs and checks its result bit-exact
against the oracle's rank-order fold (oracle/oracle.c: oracle_fold).
Prints one JSON line: {"rank": r, "results": [...]}.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
ALGO_NAMES = {"ring": 0, "direct": 1, "rccl": 2, "oneshot": 3, "peer": 4, "auto": -1, "tune": 5}
JOB_ALGO = ALGO_NAMES["peer"]  # the job's schedule (main sets it from TIPS_WORKER_ALGO)


def expected(ins, dtype, algo):
    """The bits the schedule must produce: the ring's chunk-rotated fold (oracle_ring) or the
    rank-order fold (oracle_fold, wide accumulation) of direct / one-shot / peer."""
    import oracle_bind
    if algo == ALGO_NAMES["ring"]:
        return oracle_bind.ring(ins, code=dtype)[0]
    return oracle_bind.fold(ins, code=dtype, wide_acc=True)


def named_case(c, rank, size, L, _lib, sp):
    """Named requests (tips_enqueue_allreduce) enqueued in a different order on every rank; the
    negotiation orders them and the executor fuses each ready run into one allreduce (readiness
    batching). Every output is checked against the oracle's fold of all ranks' inputs."""
    import numpy as np
    import oracle_bind
    from gpu_util import from_dev, rand, same_bits, to_dev
    tensors = c["named"]  # [[dtype, n], ...]
    order = list(range(len(tensors)))
    np.random.default_rng(c["seed"] * 31 + rank).shuffle(order)
    ins, outs, handles = {}, {}, {}
    for i in order:
        dtype, n = tensors[i]
        all_in = [rand(dtype, n, np.random.default_rng(c["seed"] + 1000 * i + r)) for r in range(size)]
        x = to_dev(all_in[rank])
        y = x if (i % 3 == 0) else x.new_empty(x.shape)
        ins[i], outs[i] = all_in, y
        handles[i] = L.tips_enqueue_allreduce(("t%d" % i).encode(), x.data_ptr(), y.data_ptr(), n, dtype, sp)
        ins[i] = (all_in, x)
    bad = []
    for i in range(len(tensors)):
        rc = L.tips_wait(handles[i]) if handles[i] > 0 else int(handles[i])
        dtype, n = tensors[i]
        if rc != 0:
            bad.append("t%d rc %d %s" % (i, rc, _lib.last_error()))
            continue
        exp = expected(ins[i][0], dtype, c.get("expect_algo", JOB_ALGO))
        if not same_bits(from_dev(outs[i], dtype), exp, dtype):
            bad.append("t%d (dtype %d, n %d) differs" % (i, dtype, n))
    return {"case": {"named": len(tensors), "seed": c["seed"]}, "rc": 0, "ok": not bad, "error": "; ".join(bad[:5])}


def optimizer_case(c, rank, size, L, _lib, sp):
    """tips_amd.DistributedOptimizer over torch.optim.SGD on a small model on the device: every
    rank computes its own gradients from its own seeded batch, step() sums them over the ranks
    (fusion buckets -> peer schedule) and applies SGD. Every rank recomputes all ranks' gradients
    locally and checks the updated parameters against p - lr * sum_r grad_r (summed in rank order,
    as the fold does), to within fp32 rounding of the SGD update."""
    import torch
    import tips_amd

    def model():
        torch.manual_seed(c["seed"])
        return torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 4)).cuda()

    def grads_of(r):
        m = model()
        g = torch.Generator().manual_seed(c["seed"] * 100 + r)
        x = torch.randn(8, 16, generator=g).cuda()
        m(x).pow(2).sum().backward()
        return [p.grad.detach().clone() for p in m.parameters()]

    all_g = [grads_of(r) for r in range(size)]
    m = model()
    g = torch.Generator().manual_seed(c["seed"] * 100 + rank)
    m(torch.randn(8, 16, generator=g).cuda()).pow(2).sum().backward()
    lr = 0.05
    with torch.no_grad():
        exp = []
        for i, p in enumerate(m.parameters()):
            s = all_g[0][i].clone()
            for r in range(1, size):
                s = s + all_g[r][i]
            exp.append(p - lr * s)
    opt = tips_amd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=lr))
    opt.step()
    torch.cuda.synchronize()
    ok = all(torch.allclose(p, e, rtol=0, atol=1e-6) for p, e in zip(m.parameters(), exp))
    return {"case": {"optimizer": c["seed"]}, "rc": 0, "ok": bool(ok), "error": "" if ok else "parameters differ"}


def overlap_case(c, rank, size, L, _lib, sp):
    """DistributedOptimizer with backward-overlapped gradient buckets (optim._GradBuckets): the
    hooks issue each bucket's in-place allreduce during backward, on a side stream, in bucket order.
    `passes` backwards per step (backward_passes_per_step, average_aggregated_gradients), two
    optimizer steps (the second after zero_grad(set_to_none=True): gradients copied into the views
    again). Checks: every bucket was issued before step() (by the hooks), the summed gradients
    equal the rank-order sum of all ranks' (averaged) local gradients bit for bit (AUTO at p > 2:
    one-shot / direct, the rank-order fold), and the parameters equal p - lr * sum.
    mode "auto" (c["mode"]): the measured choice (optim._OverlapChoice) over 2 warm-up + 2 x 2
    trial steps and 2 more: every step's sums still bit-exact, the hooks issue every bucket exactly
    in the steps run during backward, and every rank ends with the same choice."""
    import torch
    import tips_amd
    passes, avg = int(c.get("passes", 1)), bool(c.get("average", False))
    mode = c.get("mode", "1")
    os.environ["TIPS_GRAD_BUCKET_MIB"] = str(c.get("bucket_kib", 8) / 1024.0)
    os.environ["TIPS_OVERLAP_BACKWARD"] = mode
    os.environ["TIPS_OVERLAP_TRIAL_STEPS"] = "2"
    steps = 8 if mode == "auto" else 2

    def model():
        torch.manual_seed(c["seed"])
        # odd widths: parameters of ragged sizes, padded to 256-B aligned slices in the flat buffer
        return torch.nn.Sequential(torch.nn.Linear(64, 250), torch.nn.Tanh(), torch.nn.Linear(250, 251),
                                   torch.nn.Tanh(), torch.nn.Linear(251, 127), torch.nn.Tanh(),
                                   torch.nn.Linear(127, 10)).cuda()

    def batch(r, it, k):
        g = torch.Generator().manual_seed(c["seed"] * 1000 + r * 100 + it * 10 + k)
        return torch.randn(16, 64, generator=g).cuda()

    lr, bad = 0.01, []
    ref = model()  # replays every rank's local passes on a copy of the parameters
    m = model()
    opt = tips_amd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=lr), backward_passes_per_step=passes,
                                        average_aggregated_gradients=avg)
    if opt._buckets is None or len(opt._buckets.buckets) < 3:
        return {"case": {"overlap": c["seed"]}, "rc": 0, "ok": False, "error": "no overlapped buckets"}
    choices = []
    for it in range(steps):
        sums = None
        during = opt.overlap_choice["current"] == "during"
        choices.append(during)
        for r in range(size):
            ref.zero_grad(set_to_none=True)
            for k in range(passes):
                ref(batch(r, it, k)).pow(2).sum().backward()
            gs = [p.grad / passes if (avg and passes > 1) else p.grad.clone() for p in ref.parameters()]
            sums = gs if sums is None else [s + g for s, g in zip(sums, gs)]
        opt.zero_grad()
        for k in range(passes):
            m(batch(rank, it, k)).pow(2).sum().backward()
            if k < passes - 1:
                opt.step()  # counts the pass only
        issued = list(opt._buckets.issue_log)
        if issued != (list(range(len(opt._buckets.buckets))) if during else []):
            bad.append("it %d: hooks issued %s of %d buckets (during: %s)" % (it, issued, len(opt._buckets.buckets),
                                                                           during))
        # right after backward, work on the caller's stream already sees the reduced gradients
        # (the end-of-backward callback ordered it after the side stream), before any synchronize
        if during:
            snap = [p.grad.clone() for p in m.parameters()]
            for i, (g, s) in enumerate(zip(snap, sums)):
                if not torch.equal(g, s):
                    bad.append("it %d: grad %d read after backward differs" % (it, i))
        with torch.no_grad():
            exp = [p - lr * s for p, s in zip(ref.parameters(), sums)]
        if it == 1:
            opt.synchronize()  # as a caller that clips would: step() must not reduce again
        opt.step()
        torch.cuda.synchronize()
        for i, (p, s) in enumerate(zip(m.parameters(), sums)):
            if not torch.equal(p.grad, s):
                bad.append("it %d: grad %d differs" % (it, i))
        if not all(torch.allclose(p, e, rtol=0, atol=1e-6) for p, e in zip(m.parameters(), exp)):
            bad.append("it %d: parameters differ" % it)
        with torch.no_grad():  # keep the replica in step with the updated parameters
            for pr, p in zip(ref.parameters(), m.parameters()):
                pr.copy_(p)
    res = {"case": {"overlap": c["seed"], "passes": passes, "mode": mode}, "rc": 0, "ok": not bad,
           "error": "; ".join(bad[:4]), "choices": choices, "overlap_choice": opt.overlap_choice}
    if mode == "auto" and "chosen" not in opt.overlap_choice:
        res.update(ok=False, error="no overlap choice after %d steps" % steps)
    return res


def named_collectives_case(c, rank, size, L, _lib, sp):
    """Named broadcast / allgather / allreduce requests through the negotiation (the reference's
    three request types, coordinator.cc:243-353), enqueued in a different order on every rank:
    broadcasts from several roots, allgathers with ragged first dimensions (one rank contributing
    zero rows) and 3-d shapes, allreduces in between; then the same three types on host (numpy)
    tensors, as the reference's CPU ops. Then a broadcast whose root differs between ranks must
    fail on every rank (rank 0's root check) and a later request must still run."""
    import numpy as np
    import torch
    import tips_amd
    seed = c["seed"]

    def t(r, salt, shape, dtype=torch.float32):
        g = torch.Generator().manual_seed(seed * 1000 + 31 * salt + r)
        return (torch.randn(*shape, generator=g) * 10).to(dtype)

    jobs = []
    for k in range(6):
        jobs.append(("bc%d" % k, "bc", k % size, (7 + 3 * k, 5), torch.float32 if k % 2 else torch.int32))
        jobs.append(("ag%d" % k, "ag", None, None, torch.float32 if k % 3 else torch.bfloat16))
        jobs.append(("ar%d" % k, "ar", None, (100 + k,), torch.float32))
    order = list(range(len(jobs)))
    np.random.default_rng(seed * 7 + rank).shuffle(order)

    def ag_rows(k, r):
        return 0 if (r == 1 and k == 2) else (k + r) % 4 + 1

    handles = {}
    for i in order:
        name, kind, root, shape, dt = jobs[i]
        k = int(name[2:])
        if kind == "bc":
            handles[name] = tips_amd.broadcast_async(t(rank, i, shape, dt).cuda(), root, name)
        elif kind == "ag":
            handles[name] = tips_amd.allgather_async(t(rank, i, (ag_rows(k, rank), 3, 2), dt).cuda(), name)
        else:
            handles[name] = tips_amd.allreduce_async(t(rank, i, shape, dt).cuda(), name)
    bad = []
    for i, (name, kind, root, shape, dt) in enumerate(jobs):
        k = int(name[2:])
        got = tips_amd.synchronize(handles[name]).cpu()
        if kind == "bc":
            exp = t(root, i, shape, dt)
        elif kind == "ag":
            exp = torch.cat([t(r, i, (ag_rows(k, r), 3, 2), dt) for r in range(size)])
        else:
            exp = t(0, i, shape, dt)
            for r in range(1, size):
                exp = exp + t(r, i, shape, dt)
        same = torch.equal(got, exp) if kind != "ar" else torch.allclose(got, exp, rtol=1e-6, atol=1e-5)
        if got.shape != exp.shape or not same:
            bad.append("%s (%s) differs: %s vs %s" % (name, kind, tuple(got.shape), tuple(exp.shape)))
    # host tensors (numpy): the reference's ops are CPU ops; run on the negotiation thread, staged
    hjobs = [("h_ar%d" % k, "ar") for k in range(3)] + [("h_bc%d" % k, "bc") for k in range(3)] + \
        [("h_ag%d" % k, "ag") for k in range(3)]
    horder = list(range(len(hjobs)))
    np.random.default_rng(seed * 11 + rank).shuffle(horder)
    hh = {}
    for i in horder:
        name, kind = hjobs[i]
        k = int(name[-1])
        if kind == "ar":
            hh[name] = tips_amd.allreduce_async(t(rank, 200 + i, (4099,)).numpy(), name)
        elif kind == "bc":
            hh[name] = tips_amd.broadcast_async(t(rank, 200 + i, (33, 3), torch.int32).numpy(), k % size, name)
        else:
            hh[name] = tips_amd.allgather_async(t(rank, 200 + i, (k + rank, 5)).numpy(), name)
    for i, (name, kind) in enumerate(hjobs):
        k = int(name[-1])
        got = tips_amd.synchronize(hh[name])
        if kind == "ar":
            exp = t(0, 200 + i, (4099,))
            for r in range(1, size):
                exp = exp + t(r, 200 + i, (4099,))
            ok = isinstance(got, np.ndarray) and np.allclose(got, exp.numpy(), rtol=1e-6, atol=1e-5)
        elif kind == "bc":
            ok = isinstance(got, np.ndarray) and np.array_equal(got, t(k % size, 200 + i, (33, 3), torch.int32).numpy())
        else:
            exp = np.concatenate([t(r, 200 + i, (k + r, 5)).numpy() for r in range(size)])
            ok = isinstance(got, np.ndarray) and got.shape == exp.shape and np.array_equal(got, exp)
        if not ok:
            bad.append("host %s (%s) differs" % (name, kind))
    try:
        tips_amd.synchronize(tips_amd.broadcast_async(t(rank, 99, (16,)).cuda(), rank % 2, "bad_root"))
        bad.append("a root differing between ranks was accepted")
    except tips_amd.TipsError as e:
        if "Mismatched broadcast root ranks" not in str(e):
            bad.append("bad root: %s" % e)
    got = tips_amd.synchronize(tips_amd.broadcast_async(t(rank, 98, (16,)).cuda(), 0, "after")).cpu()
    if not torch.equal(got, t(0, 98, (16,))):
        bad.append("broadcast after the refused one differs")
    return {"case": {"named_collectives": seed}, "rc": 0, "ok": not bad, "error": "; ".join(bad[:5])}


def pattern_case(c, rank, size, L, _lib, sp):
    """A bucket past 2^31 elements (the reference's count is an int, utils.h:62) without host-side
    inputs: f16 x_r[i] = (i % 64) + r on the device, so every partial sum is a small integer (exact
    in f16 in any order) and the expected out[i] = p * (i % 64) + p (p - 1) / 2 is built on the
    device too. Past 2^31 f16 elements the byte offsets pass 2^32: any 32-bit offset arithmetic in
    the plans, the executor or the kernels would land bytes in the wrong place."""
    import torch
    n = int(c["pattern_n"])
    base = torch.arange(64, device="cuda", dtype=torch.float16)
    x = base.repeat(n // 64 + 1)[:n] + rank
    y = torch.empty_like(x)
    rc = L.tips_allreduce(x.data_ptr(), y.data_ptr(), n, 4, _lib.OP_SUM, sp)  # 4 = f16
    torch.cuda.synchronize()
    res = {"case": {"pattern_n": n}, "rc": int(rc)}
    if rc:
        res.update(ok=False, error=_lib.last_error())
        return res
    del x
    exp = (base * size + size * (size - 1) / 2).repeat(n // 64 + 1)[:n]
    res["ok"] = bool(torch.equal(y, exp))
    if not res["ok"]:
        bad = (y != exp).nonzero()
        res["error"] = "%d elements differ, first at %d" % (bad.numel(), int(bad[0]))
    return res


def tape_case(c, rank, size, L, _lib, sp):
    """tips_amd.DistributedGradientTape on the device: every rank differentiates its own seeded
    loss; gradient() returns the sum over ranks (fusion buckets -> peer schedule), which must equal
    the rank-order sum of all ranks' local gradients bit for bit (the peer fold's order)."""
    import torch
    import tips_amd
    torch.manual_seed(c["seed"])
    w = torch.randn(1000, device="cuda", requires_grad=True)
    b = torch.randn(37, device="cuda", requires_grad=True)

    def local(r):
        g = torch.Generator().manual_seed(c["seed"] * 100 + r)
        x, y = torch.randn(1000, generator=g).cuda(), torch.randn(37, generator=g).cuda()
        return (w * x).pow(2).sum() + (b * y).sum()

    all_g = [torch.autograd.grad(local(r), [w, b]) for r in range(size)]
    exp = []
    for i in range(2):
        s = all_g[0][i].clone()
        for r in range(1, size):
            s = s + all_g[r][i]
        exp.append(s)
    got = tips_amd.DistributedGradientTape().gradient(local(rank), [w, b])
    torch.cuda.synchronize()
    ok = all(torch.equal(g, e) for g, e in zip(got, exp))
    return {"case": {"tape": c["seed"]}, "rc": 0, "ok": bool(ok), "error": "" if ok else "gradients differ"}


def collectives_case(c, rank, size, L, _lib, sp):
    """broadcast_op / allgather_op / broadcast_variables and the consistency-checked allreduce
    over the peer transport (tips_broadcast, tips_allgatherv and the record exchange routed to
    peer.cc when the peer schedule is selected). Broadcast: every dtype, device and host, and one
    bucket larger than the workspace (pieces); the result must equal the root's tensor bit for
    bit. Allgather: ragged first dimensions, one rank contributing zero rows, and the reference's
    two allgather KATs (utils_test.cc:39-112). A root that differs between ranks must fail on every
    rank with TIPS_ERR_MISMATCH and leave the job usable."""
    import numpy as np
    import torch
    import tips_amd
    seed = c["seed"]
    root = seed % size
    bad = []

    def tensor(r, dtype, n, salt=0):
        g = torch.Generator().manual_seed(seed * 1000 + 17 * salt + r)
        return (torch.randn(n, generator=g) * 100).to(dtype)

    sizes = [(torch.float32, 4099), (torch.float64, 1), (torch.int32, 70001), (torch.int64, 3), (torch.float16, 513),
             (torch.bfloat16, 1000), (torch.float32, c.get("big", 0))]
    for k, (dt, n) in enumerate(sizes):
        if n == 0:
            continue
        y = tips_amd.broadcast_op(tensor(rank, dt, n, k).cuda(), root)
        torch.cuda.synchronize()
        if not torch.equal(y.cpu(), tensor(root, dt, n, k)):
            bad.append("broadcast %s x %d differs" % (dt, n))
    h = tips_amd.broadcast_op(tensor(rank, torch.float32, 777, 50).numpy(), root)
    if not np.array_equal(h, tensor(root, torch.float32, 777, 50).numpy()):
        bad.append("host broadcast differs")
    v = [tensor(rank, torch.float32, 300, 60).cuda(), tensor(rank, torch.int64, 5, 61).cuda()]
    tips_amd.broadcast_variables(v, root)
    torch.cuda.synchronize()
    if not (torch.equal(v[0].cpu(), tensor(root, torch.float32, 300, 60))
            and torch.equal(v[1].cpu(), tensor(root, torch.int64, 5, 61))):
        bad.append("broadcast_variables differs")
    rows = [(seed + 3 * r) % 5 if r != 1 else 0 for r in range(size)]
    parts = [tensor(r, torch.float32, rows[r] * 7, 70).reshape(rows[r], 7) for r in range(size)]
    g = tips_amd.allgather_op(parts[rank].cuda())
    torch.cuda.synchronize()
    if not torch.equal(g.cpu(), torch.cat(parts)):
        bad.append("allgather differs (rows %s)" % rows)
    gi = tips_amd.allgather_op(np.arange(rank + 1, dtype=np.int64) + 10 * rank)
    if not np.array_equal(gi, np.concatenate([np.arange(r + 1, dtype=np.int64) + 10 * r for r in range(size)])):
        bad.append("host allgather differs")
    # the reference's allgather KATs, their inputs and checks (tol 1e-5; exact here):
    # utils_test.cc:39-64 TestAllgatherOp - a [2, 3] float tensor of the rank's value, gathered into
    # [2 * size, 3], slice i all i;
    ka = tips_amd.allgather_op(torch.full((2, 3), float(rank), device="cuda"))
    torch.cuda.synchronize()
    if tuple(ka.shape) != (2 * size, 3) or not all(bool((ka[2 * i:2 * i + 2] == i).all()) for i in range(size)):
        bad.append("utils_test TestAllgatherOp KAT differs")
    # utils_test.cc:66-112 TestAllgathervOp - the first dimensions (int32 rank + 1) gathered first,
    # then [rank + 1, 4] float tensors of value rank + 1 gathered into [sum, 4], rows in rank order
    fr = tips_amd.allgather_op(np.array([rank + 1], dtype=np.int32))
    kv = tips_amd.allgather_op(torch.full((rank + 1, 4), float(rank + 1), device="cuda"))
    torch.cuda.synchronize()
    want = torch.cat([torch.full((r + 1, 4), float(r + 1)) for r in range(size)])
    if not np.array_equal(fr, np.arange(1, size + 1, dtype=np.int32)) or not torch.equal(kv.cpu(), want):
        bad.append("utils_test TestAllgathervOp KAT differs")
    tips_amd.set_consistency_check(True)
    try:
        x = tensor(rank, torch.float32, 1000, 80).cuda()
        y = tips_amd.allreduce(x)
        torch.cuda.synchronize()
        exp = tensor(0, torch.float32, 1000, 80)
        for r in range(1, size):
            exp = exp + tensor(r, torch.float32, 1000, 80)
        if not torch.equal(y.cpu(), exp):
            bad.append("checked allreduce differs")
    finally:
        tips_amd.set_consistency_check(False)
    try:
        tips_amd.broadcast_op(tensor(rank, torch.float32, 64, 90).cuda(), rank % 2)
        bad.append("a root differing between ranks was accepted")
    except tips_amd.TipsError as e:
        if e.code != -7:  # TIPS_ERR_MISMATCH
            bad.append("mismatched root: %s" % e)
    y = tips_amd.broadcast_op(tensor(rank, torch.float32, 64, 91).cuda(), root)
    torch.cuda.synchronize()
    if not torch.equal(y.cpu(), tensor(root, torch.float32, 64, 91)):
        bad.append("broadcast after the refused call differs")
    return {"case": {"collectives": seed}, "rc": 0, "ok": not bad, "error": "; ".join(bad[:6])}


def shapes_case(c, rank, size, L, _lib, sp):
    """Named requests with shapes (tips_amd.allreduce_async -> tips_enqueue_allreduce_shaped): a
    tensor that is [2,4] on even ranks and [4,2] on odd ones (equal counts) must fail on EVERY rank
    with the reference's text (coordinator.cc:142-143), while its neighbours still reduce."""
    import torch
    import tips_amd
    x = torch.arange(8, dtype=torch.float32, device="cuda") + rank
    good = tips_amd.allreduce_async(x.reshape(2, 4), "shapes.good")
    bad = tips_amd.allreduce_async(x.reshape(2, 4) if rank % 2 == 0 else x.reshape(4, 2), "shapes.bad")
    s = tips_amd.allreduce_async(x[3], "shapes.scalar")
    errs = []
    out = tips_amd.synchronize(good)
    exp = sum(torch.arange(8, dtype=torch.float32) + r for r in range(size)).reshape(2, 4)
    if not torch.equal(out.cpu(), exp):
        errs.append("good tensor differs")
    try:
        tips_amd.synchronize(bad)
        errs.append("mismatched shapes were accepted")
    except tips_amd.TipsError as e:
        if e.code != -7 or "Mismatched allreduce tensor shapes: [2,4] vs [4,2]" not in str(e):
            errs.append("wrong error: %s" % e)
    if float(tips_amd.synchronize(s).item()) != float(sum(3 + r for r in range(size))):
        errs.append("scalar differs")
    # A request whose pointers disagree on ONE rank (device in, host out on the last rank): that rank's
    # negotiation thread classifies it and announces it as bad; it fails on EVERY rank, naming the
    # rank, once all have announced it - no rank issues its allreduce alone - and the next one runs.
    import ctypes
    import numpy as np
    d_out = torch.empty(64, device="cuda")
    h_out = np.zeros(64, dtype=np.float32)
    xin = torch.full((64,), float(rank + 1), device="cuda")
    mixed = rank == size - 1
    out_ptr = h_out.ctypes.data if mixed else d_out.data_ptr()
    h = L.tips_enqueue_allreduce(b"ptrs.mixed", ctypes.c_void_p(xin.data_ptr()), ctypes.c_void_p(out_ptr), 64,
                                 _lib.FLOAT32, ctypes.c_void_p(sp))
    after = tips_amd.allreduce_async(xin, "ptrs.after")
    if h <= 0:
        errs.append("mixed enqueue refused at once: %s" % _lib.last_error())
    elif L.tips_wait(h) == 0:
        errs.append("a request with one device and one host pointer (rank %d) ran" % (size - 1))
    elif "one device and one host pointer on rank %d" % (size - 1) not in _lib.last_error():
        errs.append("wrong mixed-pointer error: %s" % _lib.last_error())
    if float(tips_amd.synchronize(after)[0].item()) != float(sum(r + 1 for r in range(size))):
        errs.append("the request after the mixed one differs")
    return {"case": {"shapes": True}, "rc": 0, "ok": not errs, "error": "; ".join(errs)}


def workload_sizes(name):
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    return bench.fused1000_sizes() if name == "config4" else bench.resnet50_grad_sizes()


def fused_case(c, rank, size, L, _lib, sp):
    """BASELINE config 4 (1000 fp32 grads, 2^U(8,17) elements) or config 5 (the 214 ResNet-50
    gradients) through the fusion buckets, as the named API would run them every step:
    mode "inplace" (tips_fused_allreduce), "layouts" (the same list, views of one buffer on rank 0
    and separate allocations elsewhere: the layout must not depend on addresses), "oop"
    (tips_fused_allreduce_oop), "grads"
    (tips_amd.allreduce_grads, the reference's per-gradient loop fused, __init__.py:203-222) or
    "optimizer" (DistributedOptimizer.step over SGD(lr=1): p - sum of all ranks' gradients).
    Every tensor is checked bit-exact against the oracle's rank-order fold of all ranks' inputs
    (the fold order of every schedule but the ring; run these with direct / peer / AUTO at p > 2)."""
    import numpy as np
    import torch
    import oracle_bind
    import tips_amd
    sizes = workload_sizes(c["fused"])
    mode = c.get("mode", "inplace")
    g = torch.Generator(device="cuda")

    def inputs(r):
        g.manual_seed(c["seed"] * 100 + r)
        return torch.empty(sum(sizes), dtype=torch.float32, device="cuda").uniform_(-1.0, 1.0, generator=g)

    mine = inputs(rank)
    views = list(torch.split(mine, sizes))
    before = mine.clone()
    if mode == "inplace":  # views of one flat buffer (packed like any tensors: the layout ignores addresses)
        tips_amd.fused_allreduce_(views)
        got = views
    elif mode == "inplace_separate":  # separately allocated tensors: packed into the buckets
        got = [v.clone() for v in views]
        tips_amd.fused_allreduce_(got)
    elif mode == "layouts":  # rank 0: views of one flat buffer; the others: separate tensors
        got = views if rank == 0 else [v.clone() for v in views]
        tips_amd.fused_allreduce_(got)
    elif mode == "oop":
        got = tips_amd.fused_allreduce(views)
    elif mode == "grads":
        got = tips_amd.allreduce_grads(views)
    elif mode == "grads_fresh":
        # a training loop's pattern: FRESH gradient tensors every step (new allocations, new values);
        # allreduce_grads' outputs are views of one flat buffer (tips_fused_allreduce_flat), and the
        # layout - a function of the counts alone - is built once and then found every step
        s0 = tips_amd.fusion_stats()
        steps = 4
        for step in range(steps):
            g.manual_seed(c["seed"] * 100 + rank + 7919 * (step + 1))
            fresh = [torch.empty(k, device="cuda").uniform_(-1.0, 1.0, generator=g) for k in sizes]
            out = tips_amd.allreduce_grads(fresh)
            torch.cuda.synchronize()
            allin = []
            for r in range(size):
                g.manual_seed(c["seed"] * 100 + r + 7919 * (step + 1))
                allin.append(torch.cat([torch.empty(k, device="cuda").uniform_(-1.0, 1.0, generator=g)
                                        for k in sizes]).cpu().numpy())
            exp = oracle_bind.fold(allin, code=0, wide_acc=True)
            gotf = torch.cat([t.reshape(-1) for t in out]).cpu().numpy()
            if not np.array_equal(gotf.view(np.uint32), exp.view(np.uint32)):
                return {"case": {"fused": c["fused"], "mode": mode}, "rc": 0, "ok": False,
                        "error": "step %d: %d elements differ" % (step, int((gotf != exp).sum()))}
            del out
        s1 = tips_amd.fusion_stats()
        d = {k: s1[k] - s0[k] for k in s0}
        ok = d["layouts_built"] <= 1 and d["layout_hits"] >= steps - 1
        return {"case": {"fused": c["fused"], "mode": mode}, "rc": 0, "ok": ok, "stats": d,
                "error": "" if ok else "fusion caches: %r" % d}
    elif mode == "mixed":
        # a small list (one <= 8 MiB bucket: replayed from its second call) and this workload's list
        # (buckets over 8 MiB: eager until a host wait widens the replay limit, then replayed too),
        # alternating in place round after round with new values; every round bit-exact, and the
        # replay -> eager host waits stop after the first (schedules.cc TIPS_GRAPH_MIXED_MAX_BYTES)
        import ctypes
        small = [16384] * 40  # 2.5 MiB
        rounds = c.get("rounds", 5)
        big_t = torch.empty(sum(sizes), dtype=torch.float32, device="cuda")
        small_t = torch.empty(sum(small), dtype=torch.float32, device="cuda")
        lists = [(small, small_t, [x.clone() for x in torch.split(small_t, small)]),
                 (sizes, big_t, [x.clone() for x in torch.split(big_t, sizes)])]
        waits = []
        for rnd in range(rounds):
            for li, (ks, _, ts) in enumerate(lists):
                seed = c["seed"] * 100 + 31 * rnd + 7 * li
                def vals(r, ks=ks, seed=seed):
                    g.manual_seed(seed * 10 + r)
                    return torch.empty(sum(ks), device="cuda").uniform_(-1.0, 1.0, generator=g)
                for t, v in zip(ts, torch.split(vals(rank), ks)):
                    t.copy_(v)
                tips_amd.fused_allreduce_(ts)
                torch.cuda.synchronize()
                exp = oracle_bind.fold([vals(r).cpu().numpy() for r in range(size)], code=0, wide_acc=True)
                gotf = torch.cat([t.reshape(-1) for t in ts]).cpu().numpy()
                if not np.array_equal(gotf.view(np.uint32), exp.view(np.uint32)):
                    return {"case": {"fused": c["fused"], "mode": mode}, "rc": 0, "ok": False,
                            "error": "round %d list %d: %d elements differ" % (rnd, li, int((gotf != exp).sum()))}
                w, wn = ctypes.c_int64(), ctypes.c_int64()
                _lib.call("tips_replay_order_stats", ctypes.byref(w), ctypes.byref(wn))
                waits.append(w.value)
        cap, rep, cached = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        L.tips_graph_stats(ctypes.byref(cap), ctypes.byref(rep), ctypes.byref(cached))
        return {"case": {"fused": c["fused"], "mode": mode}, "rc": 0, "ok": True, "error": "",
                "waits_after_each_call": waits, "captured": cap.value, "replayed": rep.value}
    elif mode in ("fp16", "fp16_fresh_outputs"):
        # Compression.fp16 fused into the buckets (allreduce_grads -> tips_fused_allreduce_cast): f32
        # in, f32 out, f16 on the wire; the second form releases the outputs and calls again, so the
        # flat output set is reused (and the layout and tables found)
        got = tips_amd.allreduce_grads(views, compression=tips_amd.Compression.fp16)
        if mode == "fp16_fresh_outputs":
            torch.cuda.synchronize()
            del got
            got = tips_amd.allreduce_grads(views, compression=tips_amd.Compression.fp16)
    elif mode == "bf16_wire":
        got = tips_amd.fused_allreduce_cast(views, "bfloat16")
    elif mode == "host_grads":
        # the reference's op is a CPU op (ops.cc:118): host gradients (numpy), fused into page-locked
        # pieces (tips_fused_allreduce_host) by allreduce_grads
        host = [v.cpu().numpy() for v in views]
        out = tips_amd.allreduce_grads(host)
        got = [torch.from_numpy(o).cuda() for o in out]
        if not all(np.array_equal(h, v.cpu().numpy()) for h, v in zip(host, views)):
            return {"case": {"fused": c["fused"], "mode": mode}, "rc": 0, "ok": False, "error": "inputs modified"}
    else:
        params = [torch.nn.Parameter(torch.zeros(k, device="cuda")) for k in sizes]
        for p, v in zip(params, views):
            p.grad = v.clone()
        opt = tips_amd.DistributedOptimizer(torch.optim.SGD(params, lr=1.0))
        opt.step()
        got = [0.0 - p.detach() for p in params]  # p = 0 - 1.0 * sum exactly (0 - p: no -0.0 where sum == +0)
    torch.cuda.synchronize()
    allin = np.stack([inputs(r).cpu().numpy() for r in range(size)])
    if mode in ("fp16", "fp16_fresh_outputs", "bf16_wire"):  # cast -> rank-order 16-bit fold -> cast back
        exp = oracle_bind.compressed_fold([allin[r] for r in range(size)],
                                          oracle_bind.BF16 if mode == "bf16_wire" else oracle_bind.F16)
        if not all(t.dtype == torch.float32 for t in got):
            return {"case": {"fused": c["fused"], "mode": mode}, "rc": 0, "ok": False, "error": "outputs not float32"}
    else:
        exp = oracle_bind.fold([allin[r] for r in range(size)], code=0, wide_acc=True)
    got_flat = torch.cat([t.reshape(-1) for t in got]).cpu().numpy()
    bad = []
    if not np.array_equal(got_flat.view(np.uint32), exp.view(np.uint32)):
        off, wrong = 0, []
        for i, k in enumerate(sizes):
            if not np.array_equal(got_flat[off:off + k].view(np.uint32), exp[off:off + k].view(np.uint32)):
                d = np.nonzero(got_flat[off:off + k].view(np.uint32) != exp[off:off + k].view(np.uint32))[0]
                j = off + int(d[0])
                own = "own input" if got_flat[j] == allin[rank][j] else "not own input"
                wrong.append("tensor %d (%d elems): %d differ from element %d to %d (got %r, expected %r, %s)" % (
                    i, k, d.size, int(d[0]), int(d[-1]), float(got_flat[j]), float(exp[j]), own))
            off += k
        bad.append("%d of %d tensors differ: %s" % (len(wrong), len(sizes), "; ".join(wrong[:3])))
    if mode in ("oop", "grads", "fp16", "fp16_fresh_outputs", "bf16_wire") and not torch.equal(mine, before):
        bad.append("inputs modified by an out-of-place call")
    return {"case": {"fused": c["fused"], "mode": mode}, "rc": 0, "ok": not bad, "error": "; ".join(bad)}


def graphs_case(c, rank, size, L, _lib, sp):
    """The call pattern TIPS_GRAPHS replays: the same buffers reduced round after round with new
    data in them. Buffers under the replay limit (captured on their second call, replayed from the
    third) interleave with one over it (always eager), in place and out of place, one of them called
    from a second stream; after round 3 one buffer pair is freed and the allocator emptied, so
    its successor is a new allocation (possibly at the same address: a new graph key). Every
    result is checked bit-exact against the schedule's oracle; reports capture / replay counts."""
    import ctypes
    import numpy as np
    import torch
    from gpu_util import from_dev, rand, same_bits, to_dev
    s2 = torch.cuda.Stream()
    specs = c["bufs"]  # [[dtype, n, inplace, second_stream], ...]
    bufs = []
    for dtype, n, inplace, _ in specs:
        x = to_dev(rand(dtype, n, np.random.default_rng(0)))
        bufs.append((x, x if inplace else torch.empty_like(x)))
    bad = []
    trace, trace_prev = [], [(0, 0, 0)]
    fresh = set(c.get("fresh", []))  # buffers reallocated at a new address every round (old ones kept)
    kept = []

    def renew(i, fill=True):
        dtype_, n_, inplace_, _ = specs[i]
        kept.append(bufs[i])
        x_ = to_dev(rand(dtype_, n_, np.random.default_rng(len(kept)))) if fill else torch.empty_like(bufs[i][0])
        bufs[i] = (x_, x_ if inplace_ else torch.empty_like(x_))

    for rnd in range(c.get("rounds", 6)):
        for i in sorted(fresh):
            renew(i)
        if rnd == 3 and 0 not in fresh:
            dtype, n, inplace, _ = specs[0]
            del bufs[0]
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            x = to_dev(rand(dtype, n, np.random.default_rng(1)))
            bufs.insert(0, (x, x if inplace else torch.empty_like(x)))
        for i, (dtype, n, inplace, second) in enumerate(specs):
            x, y = bufs[i]
            ins = [rand(dtype, n, np.random.default_rng(c["seed"] + 1000 * rnd + 100 * i + r)) for r in range(size)]
            x.copy_(to_dev(ins[rank]))
            if second:
                s2.wait_stream(torch.cuda.current_stream())
                stream = s2.cuda_stream
            else:
                stream = sp
            rc = L.tips_allreduce(x.data_ptr(), y.data_ptr(), n, dtype, _lib.OP_SUM, stream)
            if second:
                torch.cuda.current_stream().wait_stream(s2)
            if rc != 0:
                bad.append("round %d buf %d rc %d %s" % (rnd, i, rc, _lib.last_error()))
                continue
            if not same_bits(from_dev(y, dtype), expected(ins, dtype, JOB_ALGO), dtype):
                bad.append("round %d buf %d (dtype %d, n %d) differs" % (rnd, i, dtype, n))
            if c.get("trace"):  # per call: "w" = a host wait, "r" = a replay, "c" = a capture
                cap, rep, cached = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
                L.tips_graph_stats(ctypes.byref(cap), ctypes.byref(rep), ctypes.byref(cached))
                w, wn = ctypes.c_int64(), ctypes.c_int64()
                _lib.call("tips_replay_order_stats", ctypes.byref(w), ctypes.byref(wn))
                now = (w.value, rep.value, cap.value)
                prev = trace_prev[0]
                trace.append("w" * (now[0] - prev[0]) + "r" * (now[1] - prev[1]) + "c" * (now[2] - prev[2]) or "-")
                trace_prev[0] = now
    torch.cuda.synchronize()
    timing = {"trace": " ".join(trace)} if c.get("trace") else {}
    if c.get("time_calls"):  # host time inside tips_allreduce and wall time per call, buffer 0, back to back
        import time
        dtype, n, _, _ = specs[0]
        x, y = bufs[0]
        enq = 0.0
        t0 = time.perf_counter()
        for _ in range(c["time_calls"]):
            a = time.perf_counter()
            L.tips_allreduce(x.data_ptr(), y.data_ptr(), n, dtype, _lib.OP_SUM, sp)
            enq += time.perf_counter() - a
        torch.cuda.synchronize()
        timing = {"enqueue_us": round(enq / c["time_calls"] * 1e6, 2),
                  "call_us": round((time.perf_counter() - t0) / c["time_calls"] * 1e6, 2)}
    if c.get("time_rounds"):  # the whole mixed sequence back to back: wall per round, and the share
        import time           # of it the replay -> eager host waits took (TIPS_REPLAY_HOST_ORDER's cost)
        w0, n0 = ctypes.c_int64(), ctypes.c_int64()
        _lib.call("tips_replay_order_stats", ctypes.byref(w0), ctypes.byref(n0))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(c["time_rounds"]):
            for i in sorted(fresh):
                renew(i, fill=False)
            for i, (dtype, n, inplace, second) in enumerate(specs):
                x, y = bufs[i]
                L.tips_allreduce(x.data_ptr(), y.data_ptr(), n, dtype, _lib.OP_SUM, sp)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        w1, n1 = ctypes.c_int64(), ctypes.c_int64()
        _lib.call("tips_replay_order_stats", ctypes.byref(w1), ctypes.byref(n1))
        timing.update(round_ms=round(wall / c["time_rounds"] * 1e3, 3),
                      waits_per_round=round((w1.value - w0.value) / c["time_rounds"], 2),
                      wait_ms_per_round=round((n1.value - n0.value) / 1e6 / c["time_rounds"], 3))
    cap, rep, cached = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    off = L.tips_graph_stats(ctypes.byref(cap), ctypes.byref(rep), ctypes.byref(cached))
    waits, wait_ns = ctypes.c_int64(), ctypes.c_int64()
    _lib.call("tips_replay_order_stats", ctypes.byref(waits), ctypes.byref(wait_ns))
    return dict({"case": {"graphs": len(specs)}, "rc": 0, "ok": not bad, "error": "; ".join(bad[:5]),
                 "captured": cap.value, "replayed": rep.value, "cached": cached.value, "graphs_off": off,
                 "replay_host_waits": waits.value, "replay_host_wait_us": round(wait_ns.value / 1e3, 1)}, **timing)


def golden_case(c, rank, size, L, _lib, sp):
    """A committed golden vector (tests/golden: inputs and the reference's MPI_Allreduce output
    under MPICH) through the real multi-process product path: rank r reduces inputs[r]; the
    result must meet the reference's tolerance against MPICH and be bit-exact against the
    oracle's rank-order fold (the peer schedule's order)."""
    import numpy as np
    import oracle_bind
    from conftest import golden_cases, load_golden
    from gpu_util import F32, F64, I32, I64, from_dev, same_bits, to_dev
    name = c["golden"]
    ins, exp = load_golden(name)
    dtype = {"f32": F32, "f64": F64, "i32": I32, "i64": I64}[golden_cases()[name]["dtype"]]
    assert ins.shape[0] == size, "golden case %s is for %d ranks" % (name, ins.shape[0])
    x = to_dev(np.ascontiguousarray(ins[rank]))
    y = x.new_empty(x.shape)
    rc = L.tips_allreduce(x.data_ptr(), y.data_ptr(), x.numel(), dtype, _lib.OP_SUM, sp)
    import torch
    torch.cuda.synchronize()
    res = {"case": {"golden": name}, "rc": int(rc)}
    if rc != 0:
        res.update(ok=False, error=_lib.last_error())
        return res
    got = from_dev(y, dtype)
    fold_ok = bool(same_bits(got, expected([ins[r] for r in range(size)], dtype, c.get("expect_algo", JOB_ALGO)), dtype))
    if exp.dtype.kind == "i":
        ref_ok = bool(np.array_equal(got, exp))
    elif name.startswith("signed"):
        ref_ok = bool(np.all(np.abs(got.astype(np.float64) - exp) <= 1e-6 * np.sum(np.abs(ins.astype(np.float64)), axis=0)))
    elif name.startswith("kat"):
        ref_ok = bool(np.allclose(got, exp, rtol=0, atol=1e-6))
    else:
        ref_ok = bool((np.abs(got.astype(np.float64) - exp) / np.abs(exp)).max() <= 1e-6)
    res.update(ok=fold_ok and ref_ok, fold_bit_exact=fold_ok, within_reference_tolerance=ref_ok,
               bit_exact_vs_mpich=bool(np.array_equal(got.view(np.uint8), np.ascontiguousarray(exp).view(np.uint8))))
    return res


def main():
    rank, size, uid, cases = int(sys.argv[1]), int(sys.argv[2]), bytes.fromhex(sys.argv[3]), json.loads(sys.argv[4])
    import ctypes
    import faulthandler
    import signal
    faulthandler.register(signal.SIGUSR1, all_threads=True)  # run_job's timeout: where every thread stands

    import numpy as np
    import torch

    import oracle_bind
    from gpu_util import from_dev, rand, same_bits, to_dev
    from tips_amd import _lib

    oracle_bind.load()
    L = _lib.lib()
    torch.cuda.set_device(0)
    global JOB_ALGO
    algo = JOB_ALGO = ALGO_NAMES[os.environ.get("TIPS_WORKER_ALGO", "peer")]
    if algo == ALGO_NAMES["peer"]:
        os.environ["TIPS_NO_RCCL"] = "1"
        idbuf = ctypes.create_string_buffer(uid, len(uid))
        _lib.call("tips_init_rank", rank, size, 0, idbuf, len(uid))
    else:  # real RCCL: rank 0's ncclGetUniqueId over the TCP bootstrap (MASTER_ADDR / MASTER_PORT)
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(size), LOCAL_RANK="0", NCCL_HOSTID="tips-rank-%d" % rank)
        L.tips_init()
        if not L.tips_is_initialize():
            print(json.dumps({"rank": rank, "results": [{"case": "init", "ok": False, "error": _lib.last_error()}]}))
            return
    _lib.call("tips_set_algorithm", algo)
    sp = torch.cuda.current_stream().cuda_stream
    results = []
    base_env = dict(os.environ)
    for c in cases:
        # per-case settings the library reads per call (pipeline depth, transfer lanes, ...)
        for k in list(os.environ):
            if k.startswith("TIPS_") and k not in base_env:
                del os.environ[k]
        os.environ.update({k: base_env[k] for k in base_env if k.startswith("TIPS_")})
        os.environ.update(c.get("env", {}))
        case_algo = ALGO_NAMES[c["algo"]] if c.get("algo") else algo
        JOB_ALGO = case_algo
        if os.environ.get("TIPS_WORKER_SET_ALGO", "1") == "1":
            _lib.call("tips_set_algorithm", case_algo)
        else:  # the selection comes from TIPS_ALGO alone (equivalent to tips_set_algorithm)
            _lib.call("tips_set_algorithm", ALGO_NAMES["auto"])
        if c.get("named"):
            results.append(named_case(c, rank, size, L, _lib, sp))
            continue
        if c.get("fused"):
            results.append(fused_case(c, rank, size, L, _lib, sp))
            continue
        if c.get("shapes"):
            results.append(shapes_case(c, rank, size, L, _lib, sp))
            continue
        if c.get("golden"):
            results.append(golden_case(c, rank, size, L, _lib, sp))
            continue
        if c.get("bufs"):
            results.append(graphs_case(c, rank, size, L, _lib, sp))
            continue
        if c.get("collectives"):
            results.append(collectives_case(c, rank, size, L, _lib, sp))
            continue
        if c.get("tape"):
            results.append(tape_case(c, rank, size, L, _lib, sp))
            continue
        if c.get("optimizer"):
            results.append(optimizer_case(c, rank, size, L, _lib, sp))
            continue
        if c.get("overlap"):
            results.append(overlap_case(c, rank, size, L, _lib, sp))
            continue
        if c.get("named_collectives"):
            results.append(named_collectives_case(c, rank, size, L, _lib, sp))
            continue
        if c.get("pattern_n"):
            results.append(pattern_case(c, rank, size, L, _lib, sp))
            continue
        dtype, n, seed = c["dtype"], c["n"], c["seed"]
        if c.get("count_per_rank"):  # deliberately inconsistent counts: every rank must fail, none hang
            n = c["count_per_rank"][rank]
        ins = [rand(dtype, n, np.random.default_rng(seed + r)) for r in range(size)]
        if c.get("host"):  # host buffers: staged through the device (bounce / pipelined pieces)
            x = ins[rank].copy()
            y = x if c.get("inplace") else np.empty_like(x)
            rc = L.tips_allreduce(x.ctypes.data, y.ctypes.data, n, dtype, _lib.OP_SUM, None)
        else:
            x = to_dev(ins[rank])
            y = x if c.get("inplace") else torch.empty_like(x)
            rc = L.tips_allreduce(x.data_ptr(), y.data_ptr(), n, dtype, _lib.OP_SUM, sp)
        torch.cuda.synchronize()
        res = {"case": c, "rc": int(rc)}
        if rc == 0 and case_algo == ALGO_NAMES["tune"]:  # the bits of whichever schedule the job measured fastest
            ta, td, tl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            if L.tips_tuned_schedule(n * x.itemsize if c.get("host") else n * x.element_size(), ctypes.byref(ta),
                                     ctypes.byref(td), ctypes.byref(tl)) == 1:
                case_algo = ta.value
                res["tuned"] = [ta.value, td.value, tl.value]
            elif n * (x.itemsize if c.get("host") else x.element_size()) <= (256 << 10):
                case_algo = ALGO_NAMES["oneshot"]
        if rc == 0:
            exp = expected(ins, dtype, c.get("expect_algo", case_algo))
            got = y if c.get("host") else from_dev(y, dtype)
            res["ok"] = bool(same_bits(got, exp, dtype))
        else:
            res["error"] = _lib.last_error()
            res["ok"] = bool(c.get("expect_error")) and rc == c["expect_error"]
        results.append(res)
    L.tips_shutdown()
    print(json.dumps({"rank": rank, "results": results}), flush=True)


if __name__ == "__main__":
    main()
