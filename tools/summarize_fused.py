"""Print the fused-workload numbers of bench.py log files (tools/, not product): the pack kernel's
per-launch time and roofline fraction, the step, the graph-replayed step, the gradient API legs
and the host legs. Usage: python tools/summarize_fused.py LOG..."""
import json
import sys


def main():
    for f in sys.argv[1:]:
        try:
            line = [x for x in open(f) if x.startswith("{")][-1]
        except (OSError, IndexError):
            print(f, "no JSON line")
            continue
        d = json.loads(line)
        r = d["roofline"]
        out = {"pack_us": r.get("us_per_launch"), "frac": r.get("frac"), "step_ms": d["ms_per_step"],
               "graph_us": d.get("graph_replayed_step", {}).get("us_per_step")}
        ga = d.get("gradient_api", {})
        out.update({k: v.get("ms_per_step") for k, v in ga.items() if isinstance(v, dict)})
        for k in ("host_to_host_python", "host_to_host_fused"):
            if k in d:
                out[k + "_gib_s"] = d[k]["algbw_gib_s"]
        print(f, json.dumps(out))


if __name__ == "__main__":
    main()
