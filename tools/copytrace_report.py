"""copytrace_report.py — the fused host path's copies, one call at a time, from a rocprofv3
--memory-copy-trace --kernel-trace run of tools/host_fused_once.py (tools/gpu_host_copy_trace.sh):
per call, each H2D copy (DMA engine) and each D2H copy (DMA copy or the runtime's blit kernel,
__amd_rocclr_copyBuffer) as [start, end] in microseconds from the call's first H2D, the idle gaps of
the H2D stream, and the span of each direction.

usage: python tools/copytrace_report.py TRACE_DIR [--calls N]   (prints JSON, the last N calls)"""
import csv
import glob
import json
import os
import sys


def rows(d, pat):
    out = []
    for p in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def main():
    d = sys.argv[1]
    ncalls = int(sys.argv[sys.argv.index("--calls") + 1]) if "--calls" in sys.argv else 2
    ev = []
    for r in rows(d, "*memory_copy_trace.csv"):
        kind = "h2d" if "HOST_TO_DEVICE" in r["Direction"] else "d2h" if "DEVICE_TO_HOST" in r["Direction"] else None
        if kind:
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))
    for r in rows(d, "*kernel_trace.csv"):
        if "copyBuffer" in r["Kernel_Name"]:
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "blit"))
    ev.sort()
    # calls: split where the H2D stream is idle for > 2 ms
    calls, cur, last_end = [], [], None
    for e in ev:
        if last_end is not None and e[0] - last_end > 2_000_000:
            calls.append(cur)
            cur = []
        cur.append(e)
        last_end = max(last_end or 0, e[1])
    if cur:
        calls.append(cur)
    res = []
    for c in calls[-ncalls:]:
        t0 = min(e[0] for e in c if e[2] == "h2d")
        h2d = [e for e in c if e[2] == "h2d"]
        back = [e for e in c if e[2] != "h2d"]
        gaps = [round((b[0] - a[1]) / 1e3, 1) for a, b in zip(h2d, h2d[1:])]
        res.append({
            "h2d_us": [[round((s - t0) / 1e3, 1), round((e - t0) / 1e3, 1)] for s, e, _ in h2d],
            "d2h_us": [[round((s - t0) / 1e3, 1), round((e - t0) / 1e3, 1), k] for s, e, k in back],
            "h2d_gaps_us": gaps, "h2d_idle_us": round(sum(g for g in gaps if g > 0), 1),
            "h2d_span_us": round((max(e[1] for e in h2d) - t0) / 1e3, 1),
            "d2h_end_us": round((max(e[1] for e in back) - t0) / 1e3, 1) if back else None})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
