"""-m gpu: the TF op-body pattern through the C-ABI alone, in a plain-C host.

tools/_bin/op_body (tests/c/op_body.c) runs as one process per rank, each a real RCCL rank on the
box's one GPU (as tests/test_gpu_rccl_procs.py's workers: NCCL_HOSTID per process, socket
transport). On every rank four threads issue named requests - device f32 / i32 and host f32
allreduces and a broadcast - each thread in its own order and each rank in a different shuffle,
every request completing through a tips_on_done callback, while a fifth thread issues synchronous
tips_allreduce calls that the library routes through the same negotiation. Every output is checked
bit-exact against the oracle's rank-order fold (oracle_fold) of all ranks' regenerated inputs
(AUTO at p = 3: one-shot and direct schedules and fused batches - all rank-order folds). Two
training steps run over the same names, the second in the reversed order with fresh outputs: its
allreduces go through the negotiation's response cache (announced by id, decided without rank
0's table). The reference pins the same path with callbacks in coordinator_test.cc:10-45."""
import json
import os
import socket
import subprocess

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("p,tensors", [(3, 96), (2, 40)])
def test_op_body_over_rccl(gpu, p, tensors):
    _run_op_body(p, tensors, "op_body")


def test_op_body_under_tsan(gpu):
    """The same over 3 RCCL ranks with the library's host code built -fsanitize=thread
    (tools/_bin/op_body_tsan on tools/lib/libtips_hip_tsan.so, `make tsan`): the negotiation
    thread, the completion thread, the issuing threads and the real executor's HIP / RCCL calls,
    with any data race ThreadSanitizer sees in the library failing the test (halt_on_error). The ROCm
    runtime, HSA and RCCL are not instrumented: tools/tsan.supp suppresses reports inside them."""
    _run_op_body(3, 48, "op_body_tsan", {"TSAN_OPTIONS": "halt_on_error=1 exitcode=66 report_signal_unsafe=0 suppressions=%s" % os.path.join(REPO, "tools", "tsan.supp")})


def _run_op_body(p, tensors, binary, extra_env=None):
    exe = os.path.join(REPO, "tools", "_bin", binary)
    assert os.path.exists(exe), "build it first: make tools/_bin/%s (part of __graft_entry__.build())" % binary
    port = _port()
    procs = []
    for r in range(p):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(p), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), TIPS_BOOTSTRAP_PORT=str(port), NCCL_HOSTID="tips-op-body-%d" % r,
                   NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1", OP_BODY_TENSORS=str(tensors), **(extra_env or {}))
        procs.append(subprocess.Popen([exe], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for pr in procs:
            out, err = pr.communicate(timeout=260)
            outs.append((pr.returncode, out, err))
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
    bad = []  # every rank's story when any rank fails (a hang shows on all of them)
    for r, (rc, out, err) in enumerate(outs):
        k = err.find("WARNING: ThreadSanitizer")
        assert k < 0, "rank %d: %s" % (r, err[k:k + 12000])
        line = [l for l in out.splitlines() if l.startswith("{")]
        res = json.loads(line[-1]) if line else None
        if rc != 0 or not res or not res["ok"]:
            bad.append((r, rc, res, out[-1500:] if not res else "", err[-3000:]))
    assert not bad, "\n".join("rank %d rc %s: %s %s\nstderr: %s" % b for b in bad)
    for rc, out, err in outs:
        res = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
        assert res["callbacks"] == tensors and res["passes"] == 2


def test_op_host_config5_over_rccl(gpu):
    """Config 5 as the reference's CPU op sees it (tools/op_host.c): the 214 ResNet-50 gradients as
    named HOST allreduces (tips_enqueue_allreduce_shaped with their TF shapes + tips_on_done), issued
    by four executor threads per rank in a per-rank shuffled order, step after step, over 3 real RCCL
    ranks; every output of the last step bit-exact against the oracle's rank-order fold of all ranks'
    regenerated inputs (ops.cc:86-118, coordinator.cc:223-241). bench.py times the same binary's
    product-only build at one rank (op_host_named)."""
    exe = os.path.join(REPO, "tools", "_bin", "op_host_check")
    assert os.path.exists(exe), "build it first: make tools/_bin/op_host_check (part of __graft_entry__.build())"
    port = _port()
    procs = []
    for r in range(3):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="3", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), TIPS_BOOTSTRAP_PORT=str(port), NCCL_HOSTID="tips-op-host-%d" % r,
                   NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1", OP_HOST_STEPS="3", OP_HOST_WARMUP="1")
        procs.append(subprocess.Popen([exe], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for pr in procs:
            out, err = pr.communicate(timeout=240)
            outs.append((pr.returncode, out, err))
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
    for r, (rc, out, err) in enumerate(outs):
        line = [l for l in out.splitlines() if l.startswith("{")]
        res = json.loads(line[-1]) if line else None
        assert rc == 0 and res and res["ok"], "rank %d rc %s: %s\n%s" % (r, rc, out[-1500:], err[-3000:])
        assert res["tensors"] == 214 and res["elements"] == 25583592 and res["check"].startswith("bit-exact"), res


def _run_capture_race(churn, graphs):
    """tools/_bin/capture_race (tests/c/capture_race.c) over 2 RCCL ranks: one thread calls
    tips_allreduce directly on 40 bucket sizes (4 KiB - 4 MiB) x 3 rounds x 3 buffer sets, every
    result bit-exact against the oracle's fold, while 3 threads churn HIP calls."""
    exe = os.path.join(REPO, "tools", "_bin", "capture_race")
    assert os.path.exists(exe), "build it first: make tools/_bin/capture_race (part of __graft_entry__.build())"
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), TIPS_BOOTSTRAP_PORT=str(port), NCCL_HOSTID="tips-race-%d" % r,
                   NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1", CAPTURE_RACE_CHURN=churn,
                   TIPS_FRESH_WAIT_LIMIT="1000")
        env.pop("TIPS_GRAPHS", None)
        if graphs:
            env["TIPS_GRAPHS"] = "1"
        procs.append(subprocess.Popen([exe], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for pr in procs:
            out, err = pr.communicate(timeout=200)
            outs.append((pr.returncode, out, err))
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
    res = []
    for r, (rc, out, err) in enumerate(outs):
        line = [l for l in out.splitlines() if l.startswith("{")]
        d = json.loads(line[-1]) if line else None
        assert rc == 0 and d and d["ok"], "rank %d rc %s: %s\nstderr: %s" % (r, rc, out[-1500:], err[-3000:])
        assert d["calls"] == 3 * 3 * 40 and d["churn_ops"] > 0, d
        res.append(d)
    return res


def test_direct_calls_beside_legacy_stream_threads(gpu):
    """a C host whose other threads create and destroy blocking streams,
    hipMalloc / hipFree and copy / memset on the legacy null stream while one thread calls
    tips_allreduce directly, call after call on the same buffers. Replays are at their default,
    off: nothing is captured, every result is bit-exact and no call fails. (With TIPS_GRAPHS=1 the
    same run crashes inside RCCL: the legacy-stream calls invalidate the capture RCCL is inside,
    profiles/r06/)"""
    for d in _run_capture_race("all", graphs=False):
        assert d["captured"] == 0 and d["graph_state"] == 2, d


@pytest.mark.parametrize("churn", ["async", "streams", "free"])
def test_replays_beside_threads_that_keep_off_the_legacy_stream(gpu, churn):
    """Replays opted in (TIPS_GRAPHS=1) with the other threads' HIP calls on streams of their own:
    copies and syncs on non-blocking streams, blocking streams created and destroyed, hipMalloc /
    hipFree. Captures happen (every size's second call) and succeed, replays run, every result is
    bit-exact: what the runtime invalidates a capture for is legacy-stream work alone."""
    for d in _run_capture_race(churn, graphs=True):
        assert d["graph_state"] == 0 and d["captured"] >= 40 and d["replayed"] >= 80, d


def test_runtime_invalidates_a_capture_on_legacy_stream_work(gpu):
    """Pins the HIP runtime behaviour the replay default rests on, with no RCCL and no library
    (tools/_bin/capture_race_hip): while one thread captures on NON-BLOCKING streams, another
    thread's hipMemcpy / hipMemset on the legacy null stream fails ("operation would make the legacy
    stream depend on a capturing blocking stream") and invalidates the capture, in relaxed mode as
    in thread-local mode; copies on the other thread's own non-blocking stream disturb nothing. If a
    later runtime stops doing this, this test fails and TIPS_GRAPHS can default to on again."""
    exe = os.path.join(REPO, "tools", "_bin", "capture_race_hip")
    assert os.path.exists(exe), "build it first: make tools/_bin/capture_race_hip"
    rows = {}
    for churn, mode in (("async", "relaxed"), ("legacy", "relaxed"), ("legacy", "thread")):
        p = subprocess.run([exe, churn, "3", mode], capture_output=True, text=True, timeout=60)
        line = [l for l in p.stdout.splitlines() if l.startswith("{")]
        assert line, (p.returncode, p.stdout[-500:], p.stderr[-2000:])
        rows[churn, mode] = json.loads(line[-1])
    ok = rows["async", "relaxed"]
    assert ok["capture_failures"] == 0 and ok["churn_errors"] == 0 and ok["captures"] > 10, ok
    for key in (("legacy", "relaxed"), ("legacy", "thread")):
        r = rows[key]
        assert r["capture_failures"] > 0 and r["churn_errors"] > 0, r
        assert "legacy stream" in r["first_churn_error"], r
