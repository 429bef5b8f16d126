"""Run allreduce cases over real RCCL ranks sharing the GPU (socket transport) under an RCCL
setting given in the environment (e.g. NCCL_NCHANNELS_PER_PEER=8), every result checked bit-exact
against the schedule's oracle (tests/peer_worker.py). Prints one JSON line per (algo, p).
usage: python tools/rccl_env_check.py ALGO[,ALGO] P[,P] N[,N]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_gpu_peer import run_job  # noqa: E402
from test_gpu_rccl_procs import rccl_env  # noqa: E402

algos, ps, ns = (a.split(",") for a in sys.argv[1:4])
for algo in algos:
    for p in (int(x) for x in ps):
        cases = [{"dtype": 0, "n": int(n), "seed": 7 + i} for i, n in enumerate(ns)]
        env = rccl_env(algo)
        try:
            res = run_job(p, cases, timeout=int(os.environ.get("T", "200")), **env)
            out = [{"rank": r["rank"], "ok": [c["ok"] for c in r["results"]],
                    "err": [c.get("error", "")[:200] for c in r["results"] if not c["ok"]]} for r in res]
        except Exception as e:  # noqa: BLE001
            out = {"exception": str(e)[:500]}
        print(json.dumps({"algo": algo, "p": p, "ns": ns,
                          "env": {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_", "TIPS_"))},
                          "result": out}), flush=True)
