"""replay_wait_cost.py — what the replay -> eager host wait (TIPS_REPLAY_HOST_ORDER, schedules.cc
order_after_replays) costs where replayed and eager allreduces alternate: 2 and 3 real RCCL ranks on
the box's one GPU (tests/peer_worker.py graphs_case), a 1 MiB bucket (replayed from its third call)
between 16 and 32 MiB buckets (over TIPS_GRAPH_MAX_BYTES = 8 MiB), in place and out of place; 30
rounds of the whole sequence back to back after the checked rounds. Three settings: "keep"
(TIPS_GRAPH_MIXED_MAX_BYTES=0: the large buckets stay eager, every round waits), "mixed" (the
default: after the first wait the large buckets are replayed too) and "off" (TIPS_GRAPHS=0: no
replays, no waits). Prints one JSON line per job: wall per round, host waits per round and their
time. (The wait itself stays on: without it this pattern hung over the socket transport,
profiles/r03/k_hunt_summary.txt.)"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))

from test_gpu_peer import run_job  # noqa: E402
from test_gpu_rccl_procs import rccl_env  # noqa: E402


def fresh_main():
    """a 1 MiB bucket (replayed) alternating with a 32 MiB bucket at a new address
    every round. Modes: "yield" (default: replays yield after 4 waits at new addresses), "wait"
    (TIPS_FRESH_WAIT_LIMIT huge: round 4's behaviour, a host wait every round) and "off"."""
    f32 = 0
    bufs = [[f32, 1 << 18, True, False], [f32, 1 << 23, True, False]]
    modes = {"yield": {}, "wait": {"TIPS_FRESH_WAIT_LIMIT": "1000000000"}, "off": {"TIPS_GRAPHS": "0"}}
    for p in (2, 3):
        for mode, extra in modes.items():
            env = dict(rccl_env("direct"), TIPS_GRAPH_MAX_BYTES=str(8 << 20), **extra)
            res = run_job(p, [{"bufs": bufs, "seed": 5, "rounds": 6, "time_rounds": 30, "fresh": [1]}], timeout=240,
                          **env)
            r = [x["results"][0] for x in res]
            print(json.dumps({"case": "fresh_32MiB", "ranks": p, "mode": mode, "ok": all(x["ok"] for x in r),
                              "round_ms": max(x["round_ms"] for x in r),
                              "waits_per_round": max(x["waits_per_round"] for x in r),
                              "wait_ms_per_round": max(x["wait_ms_per_round"] for x in r),
                              "graphs_state": [x["graphs_off"] for x in r]}), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "fresh":
        return fresh_main()
    f32 = 0
    bufs = [[f32, 1 << 18, True, False], [f32, 1 << 22, True, False], [f32, 1 << 18, False, False],
            [f32, 1 << 23, False, False]]
    modes = {"keep": {"TIPS_GRAPH_MIXED_MAX_BYTES": "0"}, "mixed": {}, "off": {"TIPS_GRAPHS": "0"}}
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else list(modes)
    for p in (2, 3):
        for algo in ("oneshot", "direct"):
            for mode in only:
                env = dict(rccl_env(algo), **modes[mode])
                res = run_job(p, [{"bufs": bufs, "seed": 5, "rounds": 4, "time_rounds": 30}], timeout=240, **env)
                r = [x["results"][0] for x in res]
                print(json.dumps({"ranks": p, "algo": algo, "mode": mode, "ok": all(x["ok"] for x in r),
                                  "round_ms": max(x["round_ms"] for x in r),
                                  "waits_per_round": max(x["waits_per_round"] for x in r),
                                  "wait_ms_per_round": max(x["wait_ms_per_round"] for x in r),
                                  "replayed": [x["replayed"] for x in r]}), flush=True)


if __name__ == "__main__":
    main()
