"""-m gpu: replayed plans (TIPS_GRAPHS, schedules.cc) through the C-ABI on /opt/rocm's runtime.

tools/graph_repro (built by `make`, no Python in the process: the HIP runtime and RCCL of ROCm 7.2,
what a C / cgo / JNI host of libtips_hip loads) runs 2 or 3 RCCL ranks sharing the box's GPU over
the socket transport (NCCL_HOSTID per process). Three buffers are reduced round after round with
new data, from two streams, in place and out of place, one of them reallocated half way: each
plan runs eagerly on its first call, is captured into a HIP graph on its second and replayed from
then on. Every result must equal the exact sum of all ranks' inputs (integers in f32), and the
captures and replays must really happen.
"""
import json
import os
import subprocess
import tempfile

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

EXE = os.path.join(REPO, "tools", "_bin", "graph_repro")


def run_repro(p, algo, **extra):
    if not os.path.exists(EXE):
        pytest.fail("tools/_bin/graph_repro not built (make)")
    idf = tempfile.mktemp(prefix="tips_gr_")
    env = dict(os.environ, NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1", TIPS_ALGO=algo)
    env.update(extra)
    procs = [subprocess.Popen([EXE, str(r), str(p), idf], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                              env=dict(env, NCCL_HOSTID="tips-gr-%d" % r)) for r in range(p)]
    outs = []
    try:
        for pr in procs:
            o, e = pr.communicate(timeout=240)
            outs.append((pr.returncode, o, e))
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
                pr.wait()
        for f in (idf, idf + ".tmp"):
            if os.path.exists(f):
                os.unlink(f)
    res = []
    for r, (rc, o, e) in enumerate(outs):
        assert rc == 0, "rank %d exited %d:\n%s\n%s" % (r, rc, e[-3000:], o[-2000:])
        res.append(json.loads([ln for ln in o.splitlines() if ln.startswith("{")][-1]))
    return res


@pytest.mark.parametrize("algo,p", [("oneshot", 2), ("ring", 2), ("ring", 3), ("direct", 3)])
def test_replayed_plans_c_abi(gpu, algo, p):
    for r in run_repro(p, algo, TIPS_GRAPHS="1", TIPS_GRAPH_MAX_BYTES=str(2 << 20)):
        assert r["bad"] == 0 and r["graphs_off"] == 0, r
        # 3 buffers: eager on round 0, captured on round 1, replayed from then on; the reallocated
        # one is a new key at round 3 (eager), captured at 4
        assert r["captured"] >= 3 and r["replayed"] >= 11, r


def test_graphs_off_c_abi(gpu):
    for r in run_repro(2, "direct", TIPS_GRAPHS="0"):
        assert r["bad"] == 0 and r["captured"] == 0 and r["replayed"] == 0 and r["graphs_off"] == 2, r
