"""Host cost of one tips_allreduce call in a Python process (torch's bundled ROCm 7.0.2 runtime),
eager vs replayed plan (TIPS_GRAPHS): p RCCL ranks sharing the GPU over the socket transport,
400 back-to-back calls on a 16 KiB bucket after six rounds of checked calls
(tests/peer_worker.py graphs_case). One JSON line per (algo, p, graphs) with rank 0's numbers."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_gpu_peer import run_job  # noqa: E402
from test_gpu_rccl_procs import rccl_env  # noqa: E402

for algo, p in (("oneshot", 2), ("direct", 3), ("direct", 4)):
    for g in ("0", "1"):
        env = rccl_env(algo)
        env.update(TIPS_GRAPHS=g)
        case = {"bufs": [[0, 4096, False, False], [3, 70001, True, False]], "seed": 3, "rounds": 3, "time_calls": 400}
        r = run_job(p, [case], timeout=300, **env)[0]["results"][0]
        print(json.dumps({"algo": algo, "p": p, "graphs": int(g), "ok": r["ok"], "enqueue_us": r.get("enqueue_us"),
                          "call_us": r.get("call_us"), "replayed": r["replayed"], "runtime": "torch ROCm 7.0.2",
                          "transport": "RCCL socket, processes sharing one GPU"}), flush=True)
