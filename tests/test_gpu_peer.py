"""-m gpu: the peer schedule (TIPS_ALGO_PEER) across real processes.

p ranks run as p processes on the box's one GPU (tests/peer_worker.py,
TIPS_NO_RCCL=1): each exports its uncached workspace over IPC, opens the
others', and reduces through the push / rank-order fold / pull kernels with
the shared-memory barriers between the phases — the same code that runs one
rank per GPU over xGMI on an 8-GPU node. Results are checked bit-exact against
the oracle's rank-order fold (the direct schedule's bits). Cases cover every
dtype, ragged and empty-tail sizes, in place, workspace growth (small then
large buckets) and a cross-rank count mismatch, which must fail on every rank
with TIPS_ERR_MISMATCH and leave the job usable for the next call.
"""
import json
import os
import signal
import subprocess
import sys
import time

import pytest

from conftest import golden_cases
from gpu_util import ALL_DTYPES, F32, I64

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ERR_MISMATCH = -7


def run_job(p, cases, timeout=300, **extra_env):
    uid = os.urandom(128).hex()
    timeout = min(timeout, int(os.environ.get("TIPS_TEST_JOB_TIMEOUT", timeout)))  # a shorter cap for probes
    env = dict(os.environ, TIPS_NO_RCCL="1", TIPS_PEER_TIMEOUT_S="60", TIPS_VERBOSE="1")
    env.update(extra_env)
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "peer_worker.py"), str(r), str(p), uid,
                               json.dumps(cases)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
             for r in range(p)]
    outs = []
    try:
        for pr in procs:
            o, e = pr.communicate(timeout=timeout)
            outs.append((pr.returncode, o, e))
    except subprocess.TimeoutExpired:
        # a hang: every worker still running dumps its Python threads' stacks (faulthandler on
        # SIGUSR1), so the failure names the case and the library call each rank stands in
        for pr in procs:
            if pr.poll() is None:
                pr.send_signal(signal.SIGUSR1)
        time.sleep(2)
        tails = []
        for r, pr in enumerate(procs):
            pr.kill()
            o, e = pr.communicate()
            tails.append("rank %d (rc %s):\n%s\n--- stdout:\n%s" % (r, pr.returncode, e[-4000:], o[-2000:]))
        raise AssertionError("job timed out after %d s\n%s" % (timeout, "\n".join(tails)))
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
                pr.wait()
    results = []
    for r, (rc, o, e) in enumerate(outs):
        assert rc == 0, "rank %d exited %d:\n%s\n--- stdout:\n%s" % (r, rc, e[-3000:], o[-3000:])
        line = [ln for ln in o.splitlines() if ln.startswith("{")][-1]
        res = json.loads(line)
        res["stderr"] = e[-20000:]
        res["stdout"] = o[-20000:]
        results.append(res)
    return results


def check(results):
    bad = ["rank %d: %r" % (res["rank"], c) for res in results for c in res["results"] if not c["ok"]]
    errs = ["rank %d stderr: %s" % (res["rank"], res["stderr"]) for res in results if res["stderr"].strip()]
    assert not bad, "\n".join(bad[:12] + errs)


@pytest.mark.parametrize("ag", ["pull", "push"])
@pytest.mark.parametrize("p", [2, 3, 4])
def test_peer_schedule_all_dtypes(gpu, p, ag):
    cases = []
    for dtype in ALL_DTYPES:
        for n in (1, 7, 4099, 1000003):
            cases.append({"dtype": dtype, "n": n, "seed": 100 * dtype + n % 89})
    cases.append({"dtype": F32, "n": 262147, "seed": 5, "inplace": True})
    cases.append({"dtype": I64, "n": 4099, "seed": 6, "inplace": True})
    check(run_job(p, cases, TIPS_PEER_AG=ag))


@pytest.mark.parametrize("p", [2, 3, 4])
def test_peer_pullfold_all_dtypes(gpu, p):
    """TIPS_PEER_RS=pullfold: every rank stages its peers' chunks in its own workspace, then folds
    its chunk in one kernel reading every peer's slice through the IPC mapping (peer.cc
    peer_piece_pullfold). Same rank-order fold, so the same bits as the direct schedule."""
    cases = []
    for dtype in ALL_DTYPES:
        for n in (1, 7, 4099, 1000003):
            cases.append({"dtype": dtype, "n": n, "seed": 300 * dtype + n % 83})
    cases.append({"dtype": F32, "n": 262147, "seed": 15, "inplace": True})
    cases.append({"dtype": I64, "n": 4099, "seed": 16, "inplace": True})
    check(run_job(p, cases, TIPS_PEER_RS="pullfold"))


def test_peer_pullfold_pieces_goldens_and_mode_switch(gpu):
    """The pull-fold through a 4 MiB workspace (64 MiB buckets in many pieces, in place too), a
    count mismatch refused on every rank, every p = 4 golden vector (MPICH's outputs), and calls
    alternating with the push schedule in the same job (TIPS_PEER_RS read per call)."""
    p = 4
    names = sorted(n for n, c in golden_cases().items() if c["p"] == p)
    cases = [
        {"dtype": F32, "n": 1 << 24, "seed": 2},
        {"dtype": F32, "n": 5000, "seed": 3, "count_per_rank": [5000, 5000, 5000, 5001], "expect_error": ERR_MISMATCH},
        {"dtype": I64, "n": 3 << 20, "seed": 4},
        {"dtype": F32, "n": (1 << 24) + 3, "seed": 7, "inplace": True},
        {"dtype": F32, "n": 1 << 20, "seed": 8, "env": {"TIPS_PEER_RS": "push"}},
        {"dtype": F32, "n": 1 << 20, "seed": 9},
    ] + [{"golden": n} for n in names]
    check(run_job(p, cases, TIPS_PEER_WS_MIB="4", TIPS_PEER_RS="pullfold"))


@pytest.mark.parametrize("ag", ["pull", "push"])
def test_peer_schedule_pieces_and_mismatch(gpu, ag):
    """A 4 MiB workspace: the 64 MiB buckets go through in many pieces."""
    p = 3
    cases = [
        {"dtype": F32, "n": 1000, "seed": 1},
        {"dtype": F32, "n": 1 << 24, "seed": 2},
        {"dtype": F32, "n": 5000, "seed": 3, "count_per_rank": [5000, 5000, 5001], "expect_error": ERR_MISMATCH},
        {"dtype": I64, "n": 3 << 20, "seed": 4},             # the job still works after the refused call
        {"dtype": F32, "n": (1 << 24) + 3, "seed": 7, "inplace": True},
    ]
    results = run_job(p, cases, TIPS_PEER_WS_MIB="4", TIPS_PEER_AG=ag)
    check(results)
    for res in results:
        assert "rank 2" in res["results"][2]["error"] or "5001" in res["results"][2]["error"]


def test_named_requests_batched_across_processes(gpu):
    """The negotiated path with readiness batching, 3 processes: 300 named tensors of mixed dtypes
    and sizes (some at and above a 1 MiB fusion threshold, some empty, a third in place),
    enqueued in a different order on every rank; every result bit-exact against the fold."""
    import numpy as np
    from gpu_util import F16, F64, I32
    rng = np.random.default_rng(11)
    dts = [F32, F32, F32, F64, I32, F16]
    tensors = []
    for i in range(300):
        n = int(rng.choice([0, 1, 7, 300, 4099, 65536, 262144, 300000]))
        tensors.append([int(dts[int(rng.integers(len(dts)))]), n])
    port = str(29700 + os.getpid() % 200)
    check(run_job(3, [{"named": tensors, "seed": 5}], TIPS_FUSION_THRESHOLD=str(1 << 20), MASTER_ADDR="127.0.0.1",
                  MASTER_PORT=port, TIPS_ALGO="peer"))


@pytest.mark.parametrize("p", [2, 3, 4, 5, 8])
def test_golden_vectors_across_processes(gpu, p):
    """Every committed golden vector for p ranks (the reference's own KATs, config 1's 1 MiB
    bucket, the seeded i32/i64/f32/f64 sets: outputs of MPI_Allreduce under MPICH) through p real
    processes. p = 8 is config 3's rank count. At p = 2 the sum is order-free, so the result
    must also equal MPICH's bit for bit."""
    names = sorted(n for n, c in golden_cases().items() if c["p"] == p)
    assert names
    results = run_job(p, [{"golden": n} for n in names], TIPS_PEER_WS_MIB="16")
    check(results)
    if p == 2:
        for res in results:
            assert all(c["bit_exact_vs_mpich"] for c in res["results"])


@pytest.mark.parametrize("p", [2, 3])
def test_distributed_optimizer_across_processes(gpu, p):
    """tips_amd.DistributedOptimizer (reference __init__.py:252-456) in p real processes: each
    rank's gradients differ, step() sums them through the fusion buckets over the peer schedule,
    and every rank ends with the same parameters, p - lr * sum of all ranks' gradients."""
    check(run_job(p, [{"optimizer": True, "seed": 7}], TIPS_PEER_WS_MIB="16"))


@pytest.mark.parametrize("p", [2, 4])
def test_distributed_gradient_tape_across_processes(gpu, p):
    """tips_amd.DistributedGradientTape (reference __init__.py:460-569) in p real processes:
    gradient() returns every rank's gradients summed over the ranks, bit-exact against the
    rank-order sum (the peer schedule's fold order)."""
    check(run_job(p, [{"tape": True, "seed": 11}], TIPS_PEER_WS_MIB="16"))


@pytest.mark.parametrize("p", [2, 3, 4])
def test_broadcast_allgather_over_peer(gpu, p):
    """broadcast_op / allgather_op / broadcast_variables / the checked allreduce over the peer
    transport in p real processes (peer.cc peer_broadcast / peer_allgatherv): every dtype, host
    and device, a 6 MiB broadcast through a 4 MiB workspace (two pieces), ragged allgather with an
    empty rank, and a mismatched root refused on every rank without breaking the job."""
    check(run_job(p, [{"collectives": True, "seed": 5 + p, "big": 1536 * 1024}], TIPS_PEER_WS_MIB="4"))


@pytest.mark.parametrize("p", [2, 3])
def test_host_buffers_across_processes(gpu, p):
    """Host-memory allreduce in p real processes over the peer schedule: small pageable buffers
    through the page-locked bounce pair, large ones as pipelined pieces (1 MiB pieces here, so a
    5 MB bucket is 5 pieces, each H2D -> peer allreduce -> D2H on its own stream), in and out of
    place, every dtype; bit-exact against the oracle's fold."""
    cases = [{"dtype": d, "n": n, "seed": 40 + d, "host": True, "inplace": inplace}
             for d in ALL_DTYPES for n, inplace in ((1000, False), (1310721, False), (1310721, True))]
    check(run_job(p, cases, TIPS_PEER_WS_MIB="16", TIPS_HOST_PIECE_BYTES=str(1 << 20)))


@pytest.mark.parametrize("workload", ["config4", "config5"])
def test_fusion_workloads_8_processes(gpu, workload):
    """BASELINE configs 4 and 5 at their own workloads (the 1000-gradient 2^U(8,17) list; the 214
    ResNet-50 gradients) in 8 real processes over the peer schedule: fused in place, fused out of
    place, allreduce_grads and DistributedOptimizer.step(); every tensor bit-exact against the
    oracle's rank-order fold of the 8 ranks' gradients (reference per-gradient loop:
    tips/tensorflow/__init__.py:203-222)."""
    cases = [{"fused": workload, "seed": 3, "mode": m} for m in ("inplace", "inplace_separate", "layouts", "oop", "grads", "optimizer")]
    check(run_job(8, cases, timeout=600, TIPS_PEER_WS_MIB="64"))


def test_peer_selected_by_env_alone(gpu):
    """TIPS_ALGO=peer without tips_set_algorithm routes every collective - allreduce, broadcast,
    allgatherv and the consistency check's record exchange - over the peer workspaces: the job has
    no RCCL communicator (TIPS_NO_RCCL=1), so any RCCL fallback would fail."""
    check(run_job(3, [{"collectives": True, "seed": 9, "big": 1 << 20}, {"dtype": F32, "n": 5000, "seed": 2}],
                  TIPS_PEER_WS_MIB="4", TIPS_ALGO="peer", TIPS_WORKER_SET_ALGO="0"))


@pytest.mark.parametrize("p", [2, 3])
def test_named_shape_validation_across_processes(gpu, p):
    """allreduce_async carries the tensor's shape: [2,4] against [4,2] fails on every rank with
    TIPS_ERR_MISMATCH and the reference's message, the job keeps working (coordinator.cc:129-146)."""
    port = str(29600 + os.getpid() % 100 + p)
    check(run_job(p, [{"shapes": True}], MASTER_ADDR="127.0.0.1", MASTER_PORT=port, TIPS_PEER_WS_MIB="4"))


def test_stale_mapping_refused_on_every_rank(gpu):
    """Every rank reads each peer's workspace header back through its IPC mapping and checks the
    nonce the owner published: a header that does not match (here rank 1 writes a wrong nonce, as a
    stale import would show another buffer's) fails the call on EVERY rank with TIPS_ERR_HIP
    instead of reducing through the mapping; a clean job right after works."""
    ERR_HIP = -3
    results = run_job(3, [{"dtype": F32, "n": 1000, "seed": 1, "expect_error": ERR_HIP}], TIPS_PEER_WS_MIB="4",
                      TIPS_PEER_TEST_CORRUPT_RANK="1")
    check(results)
    for res in results:
        assert "stale or foreign IPC mapping" in res["results"][0]["error"]
    check(run_job(3, [{"dtype": F32, "n": 1000, "seed": 1}], TIPS_PEER_WS_MIB="4"))


@pytest.mark.parametrize("ag", ["pull", "push"])
def test_peer_counts_past_int32(gpu, ag):
    """A 2^31 + 13 element f16 bucket (4 GiB; byte offsets past 2^32) through the peer schedule at
    p = 3 in 256 MiB workspace pieces, both allgather modes; exact integer-valued sums checked on
    the device (peer_worker.pattern_case)."""
    check(run_job(3, [{"pattern_n": (1 << 31) + 13}], timeout=600, TIPS_PEER_WS_MIB="256", TIPS_PEER_AG=ag))


@pytest.mark.parametrize("p", [2, 4])
def test_named_broadcast_allgather_over_peer(gpu, p):
    """The negotiated broadcast / allgather / allreduce mix over the peer transport (TIPS_ALGO_PEER:
    tips_broadcast / tips_allgatherv go through the IPC workspaces); see the RCCL twin."""
    port = str(29500 + os.getpid() % 150 + 3 * p)
    check(run_job(p, [{"named_collectives": True, "seed": 13 + p}], timeout=600, TIPS_PEER_WS_MIB="4",
                  MASTER_ADDR="127.0.0.1", MASTER_PORT=port))
