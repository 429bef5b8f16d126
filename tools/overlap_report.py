"""overlap_report.py — transfer/sum overlap from a rocprofv3 kernel trace (tools/overlap_profile.py).

usage: python3 tools/overlap_report.py KERNEL_TRACE_CSV [LABEL]

Classifies every dispatch as a sum kernel (sum2_buf_kernel: the ring's out = in + received;
multi_sum_buf_kernel: direct's rank-order fold), a transfer kernel (RCCL's kernels for the
ncclSend/ncclRecv groups, or the runtime's copy kernels for device copies) or other, and reports:
  - sum_overlapped_frac: fraction of the sum kernels' busy time during which a transfer kernel was
    running too (1.0 = every sum hidden under a transfer),
  - transfer_overlapped_frac: the same from the transfers' side,
  - per-launch sum durations and their HBM rates, overlapped vs not,
  - span vs (busy transfer + busy sum): the time the two streams saved by running together.
Prints one JSON line.
"""
import csv
import json
import sys

SUM_KEYS = ("sum2_buf_kernel", "multi_sum_buf_kernel")
XFER_KEYS = ("nccl", "rccl", "copyBuffer", "SendRecv")


def intervals(path):
    rows = list(csv.DictReader(open(path)))
    if not rows:
        return []
    keys = rows[0].keys()
    name_k = next(k for k in keys if "Kernel_Name" in k)
    s_k = next(k for k in keys if "Start_Timestamp" in k)
    e_k = next(k for k in keys if "End_Timestamp" in k)
    out = []
    for r in rows:
        nm = r[name_k]
        kind = "sum" if any(k in nm for k in SUM_KEYS) else "xfer" if any(k in nm for k in XFER_KEYS) else "other"
        out.append((int(r[s_k]), int(r[e_k]), kind, nm))
    return sorted(out)


def union(ivs):
    out = []
    for s, e in sorted(ivs):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def overlap_len(s, e, merged):
    tot = 0
    for a, b in merged:
        if b <= s:
            continue
        if a >= e:
            break
        tot += min(b, e) - max(a, s)
    return tot


def main():
    path = sys.argv[1]
    label = sys.argv[2] if len(sys.argv) > 2 else path
    iv = intervals(path)
    sums = [(s, e, nm) for s, e, k, nm in iv if k == "sum"]
    xfers = [(s, e) for s, e, k, _ in iv if k == "xfer"]
    xm = union(xfers)
    sm = union([(s, e) for s, e, _ in sums])
    sum_busy = sum(e - s for s, e in sm)
    xfer_busy = sum(e - s for s, e in xm)
    sum_ov = sum(overlap_len(s, e, xm) for s, e in sm)
    per = [(e - s, overlap_len(s, e, xm) / max(1, e - s), nm) for s, e, nm in sums]
    ov_d = [d for d, f, _ in per if f >= 0.5]
    alone_d = [d for d, f, _ in per if f < 0.5]
    span = (max(e for s, e, _, _ in iv) - min(s for s, e, _, _ in iv)) if iv else 0
    names = sorted({nm.split("(")[0] for _, _, nm in sums})

    def med(v):
        v = sorted(v)
        return v[len(v) // 2] if v else None

    print(json.dumps({
        "label": label, "sum_launches": len(sums), "transfer_dispatches": len(xfers), "sum_kernels": names,
        "sum_busy_ms": round(sum_busy / 1e6, 3), "transfer_busy_ms": round(xfer_busy / 1e6, 3),
        "span_ms": round(span / 1e6, 3),
        "sum_overlapped_frac": round(sum_ov / max(1, sum_busy), 4),
        "transfer_overlapped_frac": round(sum_ov / max(1, xfer_busy), 4),
        "sum_launch_us_median_overlapped": round(med(ov_d) / 1e3, 2) if ov_d else None,
        "sum_launch_us_median_alone": round(med(alone_d) / 1e3, 2) if alone_d else None,
        "sum_launches_mostly_overlapped": len(ov_d),
        "saved_ms_vs_serial": round(sum_ov / 1e6, 3),
    }), flush=True)


if __name__ == "__main__":
    main()
