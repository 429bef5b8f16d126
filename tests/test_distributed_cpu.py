"""N > 1 host-side plumbing on CPU: world_size-2 (and 4) gloo groups.

The device exchange itself needs >1 GPU (driver's 8-GPU run); what runs here is
everything around it that bench.py and tips_amd rely on at N > 1: the RCCL
unique id reaching every rank through torch.distributed, the TCP bootstrap
tips_init uses, the max-over-ranks timing and all-ranks parity vote, and the
workload shapes of configs 4 and 5.
"""
import os
import socket
import sys

import pytest

from conftest import REPO


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tips_amd.basics import share_unique_id
    import bench
    uid = share_unique_id(dist, lambda: bytes((7 * i) % 256 for i in range(128)))
    t = bench.max_over_ranks(dist, 0.5 + rank)
    ok_all = bench.all_ranks_ok(dist, True)
    ok_one_bad = bench.all_ranks_ok(dist, rank != world - 1)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, uid, t, ok_all, ok_one_bad))


def _probe_worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    out = bench.link_probe(dist, rank, world, mib=4, iters=3, backend="gloo", device="cpu")
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, out))


@pytest.mark.parametrize("world", [2, 3])
def test_link_probe_shapes(world):
    """bench.link_probe's three patterns (one way, both ways, all pairs) complete and report on
    every rank; on the GPU node the same code runs over a torch nccl (RCCL) group."""
    import torch.multiprocessing as tmp
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_probe_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, out in res:
        assert out["one_link_one_way_GBps"] > 0 and out["one_link_both_ways_GBps_per_direction"] > 0
        assert ("all_links_GBps_per_rank_per_direction" in out) == (world > 2)


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_plumbing(world):
    import torch.multiprocessing as tmp
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    expect_uid = bytes((7 * i) % 256 for i in range(128))
    for rank, uid, t, ok_all, ok_one_bad in res:
        assert uid == expect_uid
        assert t == pytest.approx(0.5 + world - 1)
        assert ok_all is True and ok_one_bad is False


def test_workload_shapes():
    sys.path.insert(0, REPO)
    import bench
    r50 = bench.resnet50_grad_sizes()
    assert len(r50) == 214 and sum(r50) == 25583592
    f = bench.fused1000_sizes()
    assert len(f) == 1000 and sum(f) == 20680288 and min(f) == 257 and max(f) == 130946  # config 4


@pytest.mark.parametrize("how", ["abort", "term", "cleared"])
def test_bench_last_words(how):
    """A fatal signal during bench.py's comparison runs still prints the line measured so far
    (tools/crash_line.c): a GPU fault is SIGABRT, torchrun stops surviving ranks with SIGTERM. The
    process still dies of that signal; once the final line is out the hook prints nothing."""
    import json
    import signal
    import subprocess
    lib = os.path.join(REPO, "tools", "lib", "libcrashline.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", REPO, "tools/lib/libcrashline.so"], check=True, capture_output=True)
    prog = ("import os, signal, sys, time\nsys.path.insert(0, %r)\nimport bench\n"
            "say = bench.crash_line()\nassert say is not None\n"
            "say('{\"metric\": \"m\", \"value\": 2.5, \"compare_error\": \"during peer\"}')\n" % REPO)
    if how == "cleared":
        prog += "say(None)\n"
    prog += "os.abort()\n" if how == "abort" else "os.kill(os.getpid(), signal.SIGTERM)\ntime.sleep(30)\n"
    r = subprocess.run([sys.executable, "-c", prog], capture_output=True, text=True, timeout=120)
    assert r.returncode == (-signal.SIGABRT if how == "abort" else -signal.SIGTERM), r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if how == "cleared":
        assert lines == []
    else:
        assert len(lines) == 1 and json.loads(lines[0])["value"] == 2.5


@pytest.mark.parametrize("state,code,expect", [
    ("done", 0, "compare_error"),     # main result finished, comparison runs hung -> the result is printed
    ("none", 3, "watchdog: no progress"),
    ("printed", 0, None),             # line already out, teardown hung -> no second line
])
def test_bench_watchdog(state, code, expect):
    import json
    import subprocess
    prog = ("import sys, time\nsys.path.insert(0, %r)\nimport bench\n" % REPO)
    if state in ("done", "printed"):
        prog += "bench._RESULT.update(line={'metric': 'm', 'value': 1.0}, done=True)\n"
    if state == "printed":
        prog += "bench._RESULT['printed'] = True\n"
    prog += "bench.start_watchdog(1, 0)\ntime.sleep(30)\n"
    r = subprocess.run([sys.executable, "-c", prog], capture_output=True, text=True, timeout=120)
    assert r.returncode == code
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if expect is None:
        assert lines == []
    else:
        assert len(lines) == 1 and expect in lines[0]
        json.loads(lines[0])


def test_gpu_topology_parse(monkeypatch):
    """bench.gpu_topology reads rocm-smi's link-type and hop matrices (the text layout of ROCm 7.2)."""
    import subprocess
    sys.path.insert(0, REPO)
    import bench
    txt = ("=== ROCm System Management Interface ===\n\n"
           "======== Hops between two GPUs ========\n"
           "       GPU0         GPU1         GPU2\n"
           "GPU0   0            1            1\n"
           "GPU1   1            0            1\n"
           "GPU2   1            1            0\n\n"
           "======== Link Type between two GPUs ========\n"
           "       GPU0         GPU1         GPU2\n"
           "GPU0   0            XGMI         XGMI\n"
           "GPU1   XGMI         0            XGMI\n"
           "GPU2   XGMI         XGMI         0\n\n"
           "======== End of ROCm SMI Log ========\n")

    class R:
        stdout = txt
    monkeypatch.setattr(subprocess, "run", lambda *a, **k: R)
    topo = bench.gpu_topology()
    assert topo["hops"] == [["0", "1", "1"], ["1", "0", "1"], ["1", "1", "0"]]
    assert topo["link_type"][1] == ["XGMI", "0", "XGMI"]


def test_cpu_ring_baseline_runs_the_reference_call():
    """bench.cpu_ring_baseline: the reference's MPI_Allreduce under MPICH at np = N (the N > 1
    lines' `cpu_ring_baseline`), here on a tiny bucket; reported in the GPU line's units."""
    sys.path.insert(0, REPO)
    import bench
    out = bench.cpu_ring_baseline(2, elems=1 << 16, iters=3)
    if "error" in out and "unavailable" in out["error"]:
        pytest.skip(out["error"])
    assert out["value"] > 0 and out["cores"] == 2 and out["kind"] == "reference", out


def test_fusion_layout_mirror():
    """bench.fusion_layout (what the one-rank pack-kernel leg times) follows fusion.cc build_entry:
    every tensor once, in order, at 256-B aligned offsets, no bucket past the threshold, and the
    balanced split - at least 2 buckets once 32 MiB are packed, no bucket far above its share."""
    sys.path.insert(0, REPO)
    import bench
    for sizes in (bench.fused1000_sizes(), bench.resnet50_grad_sizes(), [1000, 3, 70000, 257]):
        b = bench.fusion_layout(sizes)
        order = [i for m in b for i, _ in m]
        assert order == [i for i, k in enumerate(sizes) if k]
        fills = [max(off + sizes[i] * 4 for i, off in m) for m in b]
        assert all(off % 256 == 0 for m in b for _, off in m) and max(fills) <= 64 << 20
        packed = sum((k * 4 + 255) // 256 * 256 for k in sizes)
        assert len(b) == max(1, (packed + (64 << 20) - 1) // (64 << 20)) or (len(b) == 2 and packed >= 32 << 20)
        if len(b) > 1:
            share = packed / len(b)
            assert all(f <= share + max(sizes) * 4 + 256 for f in fills)


def _unused_param_worker(rank, world, port, q):
    """One rank of test_unused_parameter_differs_by_rank: gloo all_reduce stands in for the bucket
    allreduce (the same blocking pairing RCCL needs: every rank the same sequence of sizes)."""
    import datetime
    import torch
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    from tips_amd.optim import _GradBuckets
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 8))
    extra = torch.nn.Parameter(torch.ones(7))  # reversed order: in bucket 0, the first to issue
    log = []

    def issue(flat):
        log.append(flat.numel())
        dist.all_reduce(flat)

    gb = _GradBuckets(list(m.parameters()) + [extra], 1024, 1, False, issue=issue)
    g = torch.Generator().manual_seed(100 + rank)
    loss = m(torch.randn(5, 16, generator=g)).pow(2).sum()
    if rank % 2 == 1:  # only odd ranks use `extra`: whether bucket 0 fills during backward is rank-local
        loss = loss + (extra * extra).sum()
    loss.backward()
    during = list(log)
    gb.synchronize()
    grads = [p.grad.clone() if p.grad is not None else None for p in list(m.parameters()) + [extra]]
    view_extra = gb.view(extra).clone()
    gb.remove()
    dist.destroy_process_group()
    q.put((rank, during, log, [x.tolist() if x is not None else None for x in grads], view_extra.tolist()))


@pytest.mark.parametrize("world", [2, 3])
def test_unused_parameter_differs_by_rank(world):
    """a parameter that gets a gradient on some ranks only. The ranks whose hooks could
    not issue bucket 0 during backward issue every bucket from synchronize(), one by one, so every
    rank sends the same sequence of bucket allreduces (sizes in order) and the sums agree - the
    whole-group shortcut would have paired one group-sized allreduce with several bucket-sized ones."""
    import torch.multiprocessing as tmp
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_unused_param_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    seqs = [log for _, _, log, _, _ in res]
    assert all(s == seqs[0] for s in seqs) and len(seqs[0]) > 1
    assert res[0][1] == [] and res[1][1] == seqs[0]  # rank 0 issued nothing during backward; rank 1 all
    for r in range(1, world):
        assert res[r][3][:-1] == res[0][3][:-1]  # identical sums on every rank
        assert res[r][4] == res[0][4]
    n_using = world // 2
    assert res[0][4] == [2.0 * n_using] * 7  # d(extra . extra) = 2 extra, summed over the ranks that used it


def test_cpu_baseline_reports_the_host_and_openmp_legs():
    """bench.cpu_baseline's host half: the CPUs and model it ran on, and config 2's
    c = a + b as an OpenMP loop on one core and on the box's CPU share (tools/cpu_sum_bench), here on
    a tiny bucket."""
    sys.path.insert(0, REPO)
    import bench
    h = bench.host_info()
    assert h["nproc"] >= 1 and h["affinity_cpus"] >= 1 and set(h) >= {"cpu_model", "omp_num_threads"}
    one = bench.openmp_sum(1 << 16, 1, 3)
    if "error" in one:
        pytest.skip(one["error"])
    two = bench.openmp_sum(1 << 16, 2, 3)
    assert one["value"] > 0 and one["cores"] == 1 and one["check"] == "exact"
    assert two["value"] > 0 and two["cores"] == 2 and two["check"] == "exact"


def _budget_worker(rank, world, port, q):
    import time
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    job = object.__new__(bench.Job)  # (no GPU: only the budget half of a Job)
    job.dist, job.rank, job.skipped = dist, rank, []
    bench._T0 = time.time() - (50 if rank == world - 1 else 0)  # the last rank's clock started 50 s earlier
    job.budget_s = 60.0
    got = [job.afford("a", 5), job.afford("b", 20), job.afford("c", 9)]
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, got, job.skipped))


def test_bench_budget_is_decided_together():
    """bench.Job.afford: an optional leg starts only while the budget lasts on the SLOWEST rank's
    clock, so every rank takes the same branch (the legs are collectives)."""
    import torch.multiprocessing as tmp
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_budget_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    for rank, got, skipped in res:
        assert got == [True, False, True], (rank, got)
        assert skipped == ["b"]


def _child_hang_worker(rank, world, port, q):
    import time
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TIPS_BENCH_CHILD_TEST="hang")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    class Args:
        bucket_mib = None
    line = {"metric": "m", "value": 1.0, "compare_algbw_gib_s": {}, "compare_check": {}}
    t0 = time.time()
    bench._RESULT["deadline"] = t0 + 600  # (the job's watchdog, far away)
    kids = bench.child_bucket_jobs(Args(), dist, rank, world, bench.PEER_CHILDREN, timeout_s=4)
    line["peer_children"] = kids
    for name, r in kids.items():
        line["compare_algbw_gib_s"][name] = r.get("algbw_gib_s") if not r.get("error") else None
        line["compare_check"][name] = r.get("check") or ("error: %s" % r.get("error"))
    dt = time.time() - t0
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, line, dt))


def test_peer_child_that_hangs_costs_only_its_entry():
    """bench.py runs the peer schedules (push and the fused pull-fold) as child
    jobs on every N > 1 line, after the main line is measured. A child that never ends
    (TIPS_BENCH_CHILD_TEST=hang replaces it with a sleeping process) is killed with its process group
    at its budget; every rank of the parent job leaves the barrier, and the line keeps its measured
    value with the child's entry reporting the time-out."""
    import torch.multiprocessing as tmp
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_child_hang_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    line0, dt0 = res[0][1], res[0][2]
    assert line0["value"] == 1.0 and dt0 < 30
    for name in ("peer", "peer_pullfold"):
        assert "timed out" in line0["peer_children"][name]["error"], line0
        assert line0["compare_algbw_gib_s"][name] is None and line0["compare_check"][name].startswith("error: timed out")
    assert res[1][1]["peer_children"] == {}  # (the other ranks only wait)
