"""cpu_ref_sweep.py — the reference's CPU data path timed on this host.

This is the baseline instrument behind DESIGN.md §7's CPU table. It does two
things:
- It runs the reference's exact hot-path call,
  `MPI_Allreduce(in, out, N, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD)`
  (tips/core/collective/utils.h:60-65). The call is made through
  oracle/build/mpi_allreduce_ref under the image's MPICH, with
  `mpirun -np p` for p in {1, 2, 4, 8}, one rank per core, on 1 MiB, 64 MiB
  and 1 GiB fp32 buckets.
- It runs config 2's `c = a + b` as an OpenMP loop (tools/cpu_sum_bench), on 1
  thread and on the box's CPU share.

It uses no GPU. Each result is one JSON line: algbw = S/t and
busbw = algbw * 2(p-1)/p, both in GiB/s, with the CPU model and core count.

usage: python tools/cpu_ref_sweep.py [--sizes-mib 1,64,1024] [--nps 1,2,4,8] [--threads 16]
"""
import argparse
import json
import os
import platform
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GIB = float(1 << 30)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def iters_for(bytes_):
    if bytes_ <= (4 << 20):
        return 50
    if bytes_ <= (256 << 20):
        return 5
    return 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mib", default="1,64,1024")
    ap.add_argument("--nps", default="1,2,4,8")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--timeout", type=int, default=300)
    args = ap.parse_args()
    host = {"cpu": cpu_model(), "os_cpu_count": os.cpu_count()}
    print(json.dumps({"host": host}), flush=True)

    harness = os.path.join(REPO, "oracle", "build", "mpi_allreduce_ref")
    mpirun = "/opt/conda/bin/mpirun"
    if not (os.path.exists(harness) and os.path.exists(mpirun)):
        print(json.dumps({"error": "reference MPI baseline unavailable on this host"}), flush=True)
    else:
        for mib in [int(x) for x in args.sizes_mib.split(",")]:
            n = (mib << 20) // 4
            for p in [int(x) for x in args.nps.split(",")]:
                iters = iters_for(mib << 20)
                cmd = [mpirun, "-np", str(p), "-bind-to", "core", harness, "bench", "0", str(n), str(iters)]
                rec = {"kind": "reference", "call": "MPI_Allreduce(MPI_FLOAT, MPI_SUM)", "mpi": "MPICH 3.3.2",
                       "np": p, "cores": p, "bucket_mib": mib, "count": n, "iters": iters}
                try:
                    r = subprocess.run(cmd, capture_output=True, text=True, timeout=args.timeout)
                    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
                    if r.returncode != 0 or not lines:
                        rec["error"] = "rc=%d %s" % (r.returncode, r.stderr.strip()[-300:])
                    else:
                        t = json.loads(lines[-1])["sec_per_call"]
                        alg = (mib << 20) / t / GIB
                        rec.update(ms_per_call=round(t * 1e3, 4), algbw_gib_s=round(alg, 4),
                                   busbw_gib_s=round(alg * 2 * (p - 1) / p, 4))
                except subprocess.TimeoutExpired:
                    rec["error"] = "timed out after %d s" % args.timeout
                print(json.dumps(rec), flush=True)

    bench = os.path.join(REPO, "tools", "cpu_sum_bench")
    if os.path.exists(bench):
        for th in sorted({1, args.threads}):
            r = subprocess.run([bench, str(64 << 20), "10", str(th)], capture_output=True, text=True,
                               timeout=args.timeout)
            lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
            rec = {"kind": "openmp c=a+b (config 2 on host cores)", "threads": th}
            if lines:
                res = json.loads(lines[-1])
                rec.update(ms_per_call=round(res["sec_per_call"] * 1e3, 3),
                           moved_gib_s=round(3 * (256 << 20) / res["sec_per_call"] / GIB, 3))
            else:
                rec["error"] = "rc=%d" % r.returncode
            print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
