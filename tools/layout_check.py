"""Before/after check of the fusion layout across ranks whose tensors lie differently: config 5's
214 gradients on 3 real RCCL ranks, rank 0 passing views of one flat buffer and the others
separate allocations (tests/peer_worker.py fused_case mode "layouts"). Prints one JSON line.
TIPS_HIP_LIB selects the library under test (e.g. one built with an address-dependent layout)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_gpu_peer import run_job  # noqa: E402
from test_gpu_rccl_procs import rccl_env  # noqa: E402

env = rccl_env("auto")
try:
    res = run_job(3, [{"fused": "config5", "seed": 4, "mode": "layouts"}], timeout=int(os.environ.get("T", "120")), **env)
    out = {"lib": os.environ.get("TIPS_HIP_LIB", "tips_amd/lib/libtips_hip.so"),
           "ranks": [{"ok": r["results"][0]["ok"], "error": r["results"][0].get("error", "")[:300]} for r in res]}
except Exception as e:  # noqa: BLE001
    out = {"lib": os.environ.get("TIPS_HIP_LIB", "tips_amd/lib/libtips_hip.so"), "exception": str(e)[:600]}
print(json.dumps(out), flush=True)
