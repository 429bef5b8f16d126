#!/usr/bin/env python3
"""bench.py — the TiPS gradient-bucket reduction path on MI355X.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...     (N > 1, one rank per GPU)

One JSON line (rank 0). Its headline `value` is BASELINE.json's metric:

N == 1 (configs[1], the config the metric's first half is quoted on): one step = the
device-resident sum of two 256 MiB fp32 gradient buffers, c = a + b (tips_bucket_sum: the
per-chunk MPI_SUM of tips/core/collective/utils.h:60-65 as a gfx950 kernel). value = algorithmic
bytes moved (2 reads + 1 write = 805,306,368 B per step) / time, GiB/s. Step i sums the (i % 4)-th
of four such buffer triples, so every launch reads its operands from HBM, not from the 256 MiB
Infinity Cache.

N > 1 (configs[2]): one step = allreduce of one 1 GiB fp32 bucket per GPU (tips_allreduce: RCCL
send/recv over xGMI + the sum kernels). value = N x 1 GiB / time (bucket bytes reduced by the
whole job per second, GiB/s); busbw and the xGMI fraction beside it. Each rank checks its result
against the fold of all ranks' seeded inputs after timing.

Beside the headline, the same line carries the other configs as sub-records (`configs`), each
with its own steps, rate, roofline and parity check, at every N:
  config3_bucket  (N == 1 only) config 3's 1 GiB bucket through tips_allreduce at one rank, value
                  = N x bucket bytes / time: the same definition as the N > 1 headline, so a
                  scaling curve starts from the workload it ends on;
  config4_fused1000, config5_resnet50: the fusion path (tips_fused_allreduce) over the configs'
                  gradient sets, busbw and xGMI fraction at N > 1, the pack kernel's HBM roofline
                  at N == 1; config 5 also host -> host (the 214 gradients in host memory, fused),
                  and at N == 1 as the reference's CPU op sees it: 214 named host requests from four
                  executor threads (tools/op_host.c).
Comparison schedules and probes follow, within a time budget all ranks agree on
(TIPS_BENCH_BUDGET_S, 240 s from start); what the budget leaves out is named in the line.

Inputs are synthetic seeded uniforms generated on the device and resident in HBM before the timed
region. Rank 0 also times the reference's CPU path (MPI_Allreduce, MPI_SUM under MPICH on host
cores) and an OpenMP c = a + b on a bounded sample — a reported baseline, not the target.
"""
import argparse
import json
import os
import signal
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
METRIC = "device-resident fp32 bucket-sum GiB/s (% HBM peak); allreduce GiB/s 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
XGMI_LINK_GBPS = 153.0   # per link per direction (task / SURVEY §8d)
GIB = float(1 << 30)
# the exact instantiation tips_bucket_sum launches for f32 (kernels.hip kDef*): PMC traffic is only
# reported from a profile of this kernel
DEFAULT_SUM_KERNEL = "sum2_buf_kernel<0, 2, 2, 1, 128>"
# N == 1 cycles over this many (a, b, c) triples of config 2's size (3 GiB at 4): see sum_record
ROTATING_SETS = 4
SUB_WORKLOADS = ("fused1000", "resnet50")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--sub-steps", type=int, default=20, help="timed steps of each sub-record (configs 3-5)")
    ap.add_argument("--algo", default=os.environ.get("TIPS_ALGO", "tune"),
                    choices=["auto", "ring", "direct", "rccl", "oneshot", "peer", "tune"],
                    help="N>1 schedule; tune (default): the library times ring / direct at several pipeline "
                         "depths on the first call of a size class and keeps the fastest (TIPS_ALGO_TUNE)")
    ap.add_argument("--bucket-mib", type=int, default=None, help="override the bucket size (MiB)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-compare", action="store_true", help="skip the comparison schedules and probes")
    ap.add_argument("--no-sub", action="store_true", help="the headline only: no config sub-records")
    ap.add_argument("--no-env-variants", action="store_true",
                    help="N>1: skip the child jobs that rerun direct under other RCCL settings")
    ap.add_argument("--no-extras", action="store_true",
                    help="N=1: time the headline kernel only (no same-buffer, PCIe or host-memory legs, no "
                         "sub-records), as under rocprofv3")
    ap.add_argument("--workload", default="auto", choices=["auto", "sum", "bucket", "fused1000", "resnet50", "negotiated1000"],
                    help="auto: config 2 (sum) at N=1, config 3 (bucket allreduce) at N>1, with the other configs "
                         "as sub-records; any other: that workload alone as the headline")
    return ap.parse_args()


# ----------------------------------------------------------------------------- CPU baselines (rank 0)

def host_info():
    """The host the CPU baselines ran on: CPUs the OS shows, CPUs this process may run on, the
    box's CPU share (OMP_NUM_THREADS, set to 16 per GPU on the GPU box), the CPU model."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    omp = os.environ.get("OMP_NUM_THREADS")
    return {"nproc": os.cpu_count(), "affinity_cpus": affinity, "omp_num_threads": int(omp) if omp and omp.isdigit() else None,
            "cpu_model": model}


def openmp_sum(elems, threads, iters):
    """tools/cpu_sum_bench: c = a + b over two `elems` fp32 buffers on `threads` OpenMP threads
    (config 2's step on host cores, the loop libmpi's MPI_SUM runs per chunk). GiB/s of the same 3 x
    bucket bytes as the GPU headline."""
    exe = os.path.join(REPO, "tools", "cpu_sum_bench")
    if not os.path.exists(exe):
        return {"error": "tools/cpu_sum_bench not built"}
    try:
        r = subprocess.run([exe, str(elems), str(iters), str(threads)], capture_output=True, text=True, timeout=120,
                           env=dict(os.environ, OMP_PROC_BIND="spread", OMP_PLACES="cores"))
        d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    except Exception as e:  # noqa: BLE001 - a baseline leg never fails the bench
        return {"error": repr(e)}
    t = d["sec_per_call"]
    return {"value": round(3 * elems * 4 / t / GIB, 3), "unit": "GiB/s", "cores": threads, "ms_per_call": round(t * 1e3, 3),
            "check": "exact" if d.get("check") == 0 else "FAIL",
            "sample": "tools/cpu_sum_bench: c = a + b, %d fp32 per buffer (%d MiB), %d timed calls after 1 warm-up, "
                      "OpenMP static schedule, %d thread(s)" % (elems, elems * 4 >> 20, iters, threads)}


def cpu_baseline(bucket_elems):
    """N == 1: the reference's data-path call on host cores - MPI_Allreduce(MPI_FLOAT, MPI_SUM) with
    np = 2, one 256 MiB fp32 bucket per rank, i.e. the reference computing config 2's c = a + b
    (`value`) - beside an OpenMP c = a + b on one core and on the box's CPU share, the
    host's CPUs and model. Runs BEFORE anything touches the GPU (it starts child processes)."""
    harness = os.path.join(REPO, "oracle", "build", "mpi_allreduce_ref")
    mpirun = "/opt/conda/bin/mpirun"
    host = host_info()
    out = {"value": None, "unit": "GiB/s", "cores": None, "kind": "reference", "sample": None, "host": host}
    if os.path.exists(harness) and os.path.exists(mpirun):
        iters = 50  # about 8-10 s of host work on the GPU box (a bounded sample, contract ④)
        try:
            r = subprocess.run([mpirun, "-np", "2", harness, "bench", "0", str(bucket_elems), str(iters)],
                               capture_output=True, text=True, timeout=240)
            line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
            res = json.loads(line)
            t = res["sec_per_call"]
            out.update(value=3 * bucket_elems * 4 / t / GIB, cores=2,
                       sample="MPI_Allreduce(in,out,%d,MPI_FLOAT,MPI_SUM,MPI_COMM_WORLD) as in "
                              "tips/core/collective/utils.h:60-65, MPICH 3.3.2, mpirun -np 2 (1 core each), "
                              "one %d MiB fp32 bucket per rank (= config 2's a + b), %d timed calls after 1 warm-up, "
                              "%.1f ms/call; value counts the same 3 x bucket bytes as the GPU metric"
                              % (bucket_elems, bucket_elems * 4 >> 20, iters, t * 1e3))
            out["ms_per_call"] = t * 1e3
        except Exception as e:  # noqa: BLE001 - report, never fail the bench on the baseline leg
            out["error"] = "reference MPI baseline failed: %r" % (e,)
    else:
        out["error"] = "reference MPI baseline unavailable on box (no MPICH harness)"
    share = host["omp_num_threads"] or host["affinity_cpus"] or 1
    out["openmp_1_core"] = openmp_sum(bucket_elems, 1, 10)
    out["openmp_all_cores"] = openmp_sum(bucket_elems, share, 30)
    out["openmp_all_cores"]["cores_note"] = ("the box's CPU share (OMP_NUM_THREADS=%s of %s CPUs the OS shows)"
                                             % (host["omp_num_threads"], host["nproc"]))
    # the oracle port (single thread, plain C loop) on the same buffers
    try:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import numpy as np
        import oracle_bind
        n = bucket_elems
        a = np.random.default_rng(1).random(n, dtype=np.float32)
        b = np.random.default_rng(2).random(n, dtype=np.float32)
        oracle_bind.sum2(a, b)
        t0 = time.perf_counter()
        reps = 10
        for _ in range(reps):
            oracle_bind.sum2(a, b)
        t = (time.perf_counter() - t0) / reps
        out["port_single_thread"] = {"value": 3 * n * 4 / t / GIB, "unit": "GiB/s", "cores": 1, "kind": "port",
                                     "sample": "oracle_sum2 (oracle/oracle.c) c=a+b, %d fp32, %d reps" % (n, reps)}
        if out["value"] is None:
            out.update({k: out["port_single_thread"][k] for k in ("value", "cores", "kind", "sample")})
    except Exception as e:  # noqa: BLE001
        out["port_error"] = repr(e)
    return out


def cpu_ring_baseline(world, elems=16 << 20, iters=20):
    """N > 1: the reference's allreduce at the same rank count on host cores - MPI_Allreduce
    (MPI_FLOAT, MPI_SUM) under MPICH, mpirun -np N, one bounded 64 MiB bucket per rank (config 3's
    1 GiB would take ~1 s per call at np = 8). Reported as `cpu_baseline` in the
    same units as `value` (N x bucket bytes per second). Rank 0 runs it before anything touches
    the GPU; the other ranks wait for it in the bootstrap."""
    harness = os.path.join(REPO, "oracle", "build", "mpi_allreduce_ref")
    mpirun = "/opt/conda/bin/mpirun"
    host = host_info()
    if not (os.path.exists(harness) and os.path.exists(mpirun)):
        return {"error": "reference MPI baseline unavailable on box (no MPICH harness)", "host": host}
    try:
        r = subprocess.run([mpirun, "-np", str(world), harness, "bench", "0", str(elems), str(iters)],
                           capture_output=True, text=True, timeout=150)
        t = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])["sec_per_call"]
    except Exception as e:  # noqa: BLE001 - never fail the bench on the baseline leg
        return {"error": "reference MPI baseline failed: %r" % (e,), "host": host}
    return {"value": round(world * elems * 4 / t / GIB, 3), "unit": "GiB/s", "cores": world, "kind": "reference",
            "ms_per_call": round(t * 1e3, 3), "host": host,
            "sample": "MPI_Allreduce(in,out,%d,MPI_FLOAT,MPI_SUM,MPI_COMM_WORLD) as in tips/core/collective/"
                      "utils.h:60-65, MPICH 3.3.2, mpirun -np %d (1 core each), one %d MiB fp32 bucket per rank, "
                      "%d timed calls after 1 warm-up; value = %d x bucket bytes / time, as the GPU line's"
                      % (elems, world, elems * 4 >> 20, iters, world)}


def thread_placement(names=("tips-neg", "tips-done")):
    """Where this process's main thread and the library's named threads last ran (/proc/self/task/*/stat
    field 39), each with its L3 domain (a CCD on EPYC: the first CPU sharing its L3) and socket (VERDICT
    r05 item 3: which placement makes the negotiated path slow)."""
    def cpu_info(cpu):
        base = "/sys/devices/system/cpu/cpu%d" % cpu
        try:
            with open(base + "/cache/index3/shared_cpu_list") as f:
                l3 = int(f.read().split(",")[0].split("-")[0])
        except (OSError, ValueError):
            l3 = None
        try:
            with open(base + "/topology/physical_package_id") as f:
                sock = int(f.read())
        except (OSError, ValueError):
            sock = None
        return {"cpu": cpu, "l3_first_cpu": l3, "socket": sock}

    out = {}
    try:
        for tid in os.listdir("/proc/self/task"):
            with open("/proc/self/task/%s/comm" % tid) as f:
                comm = f.read().strip()
            if int(tid) != os.getpid() and comm not in names:
                continue
            with open("/proc/self/task/%s/stat" % tid) as f:
                fields = f.read().rsplit(")", 1)[1].split()
            out["caller" if int(tid) == os.getpid() else comm] = cpu_info(int(fields[36]))  # (field 39 overall)
    except (OSError, ValueError, IndexError):
        return None
    if len(out) > 1:
        l3s = {v["l3_first_cpu"] for v in out.values()}
        socks = {v["socket"] for v in out.values()}
        out["same_l3"] = len(l3s) == 1
        out["same_socket"] = len(socks) == 1
    out["bind"] = os.environ.get("TIPS_NEG_BIND") or "l3 (the default)"
    return out


def pmc_traffic(kernel_substr, file_pattern="*pmc*.json"):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/<file_pattern>), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", file_pattern)), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
            k = d.get("kernels", {})
            for name, v in k.items():
                if kernel_substr in name and v.get("hbm_bytes_per_launch"):
                    return {"bytes": v["hbm_bytes_per_launch"], "source": os.path.relpath(path, REPO)}
        except Exception:  # noqa: BLE001
            continue
    return None



# ----------------------------------------------------------------------------- workloads, probes

def fused1000_sizes():
    """Config 4: 1000 fp32 gradients, sizes round(2**U(8,17)) from default_rng(20261015)."""
    import numpy as np
    rng = np.random.default_rng(20261015)
    return [int(round(2 ** u)) for u in rng.uniform(8, 17, size=1000)]


def resnet50_grad_sizes():
    """Config 5: Keras ResNet-50 trainable-gradient shapes, in layer-creation order:
    stem conv 7x7x3x64 + bias, BN gamma/beta; bottleneck stages [3,4,6,3] x widths 64/128/256/512
    (x4 expansion, conv biases, projection shortcut in each stage's first block); dense 2048x1000 + bias.
    214 tensors, 25,583,592 parameters."""
    shapes = [(7, 7, 3, 64), (64,), (64,), (64,)]
    cin = 64
    for f, blocks in ((64, 3), (128, 4), (256, 6), (512, 3)):
        for b in range(blocks):
            if b == 0:
                shapes += [(1, 1, cin, 4 * f), (4 * f,), (4 * f,), (4 * f,)]
            shapes += [(1, 1, cin, f), (f,), (f,), (f,), (3, 3, f, f), (f,), (f,), (f,),
                       (1, 1, f, 4 * f), (4 * f,), (4 * f,), (4 * f,)]
            cin = 4 * f
    shapes += [(2048, 1000), (1000,)]
    sizes = []
    for sh in shapes:
        k = 1
        for d in sh:
            k *= d
        sizes.append(k)
    return sizes


def gpu_topology():
    """rocm-smi's GPU-to-GPU link type and hop matrices (rank 0 at N > 1, before the GPU is used):
    what the xGMI numbers of the line ran over. None if rocm-smi is missing or fails."""
    try:
        r = subprocess.run(["rocm-smi", "--showtopotype", "--showtopohops"], capture_output=True, text=True,
                           timeout=30)
    except Exception:  # noqa: BLE001
        return None
    out, section = {}, None
    for ln in r.stdout.splitlines():
        if "Link Type between two GPUs" in ln:
            section = out.setdefault("link_type", [])
        elif "Hops between two GPUs" in ln:
            section = out.setdefault("hops", [])
        elif ln.startswith("GPU") and section is not None and len(ln.split()) > 1:
            section.append(ln.split()[1:])
        elif ln.startswith("=") or not ln.strip():
            if section is not None and section:
                section = None
    return out or None


def max_over_ranks(dist, seconds):
    """The contract's job time: the slowest rank's timed region (gloo all-reduce MAX on the host)."""
    import torch
    t = torch.tensor([float(seconds)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def all_ranks_ok(dist, ok):
    import torch
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def link_probe(dist, rank, world, mib=256, iters=5, backend="nccl", device="cuda"):
    """What one xGMI link and all of them carry, measured with RCCL point-to-point through a torch
    "nccl" group (independent of libtips_hip): rank 0 -> 1 one way, 0 <-> 1 both ways, and every
    rank exchanging mib / (world - 1) with every peer at once. Host-timed (barrier, synchronize on
    both sides), median of `iters` after one warm-up, max over ranks. GB/s = bytes each rank sends
    (and receives) per second. Grounds the xGMI roofline the allreduce lines are priced against."""
    import torch
    pg = dist.new_group(backend=backend)
    dist.all_reduce(torch.zeros(1, device=device), group=pg)  # every rank creates the communicator
    n = mib << 20
    a = torch.empty(n, dtype=torch.uint8, device=device)
    b = torch.empty(n, dtype=torch.uint8, device=device)
    sync = torch.cuda.synchronize if device == "cuda" else (lambda: None)

    def run(ops_fn):
        ts = []
        for _ in range(iters + 1):
            dist.barrier()
            sync()
            t0 = time.perf_counter()
            ops = ops_fn()
            if ops:
                for req in dist.batch_isend_irecv(ops):
                    req.wait()
            sync()
            ts.append(max_over_ranks(dist, time.perf_counter() - t0))
        return sorted(ts[1:])[iters // 2]

    def uni():
        if rank == 0:
            return [dist.P2POp(dist.isend, a, 1, group=pg)]
        return [dist.P2POp(dist.irecv, b, 0, group=pg)] if rank == 1 else []

    def bi():
        if rank in (0, 1):
            return [dist.P2POp(dist.isend, a, 1 - rank, group=pg), dist.P2POp(dist.irecv, b, 1 - rank, group=pg)]
        return []

    part = n // (world - 1) // 4096 * 4096

    def all_pairs():
        ops = []
        for d in range(1, world):
            to, frm = (rank + d) % world, (rank - d) % world
            k = d - 1
            ops.append(dist.P2POp(dist.isend, a[k * part:(k + 1) * part], to, group=pg))
            ops.append(dist.P2POp(dist.irecv, b[k * part:(k + 1) * part], frm, group=pg))
        return ops

    out = {"bytes": n, "method": "%s p2p via a torch %s group, host-timed, median of %d" % (
        "RCCL" if backend == "nccl" else backend, backend, iters)}
    out["one_link_one_way_GBps"] = round(n / run(uni) / 1e9, 1)
    out["one_link_both_ways_GBps_per_direction"] = round(n / run(bi) / 1e9, 1)
    if world > 2:
        out["all_links_GBps_per_rank_per_direction"] = round(part * (world - 1) / run(all_pairs) / 1e9, 1)
    del a, b
    dist.destroy_process_group(pg)
    return out


def fusion_layout(sizes, es=4, threshold=64 << 20, align=256):
    """The buckets fusion.cc build_entry forms from these element counts (balanced buckets, 256-B
    aligned offsets; every tensor here is under the threshold): [[(tensor index, offset), ...], ...]."""
    def up(v):
        return (v + align - 1) // align * align
    packed = sum(up(k * es) for k in sizes if k * es < threshold)
    nb = (packed + threshold - 1) // threshold
    if nb < 2 and packed >= (32 << 20):
        nb = 2
    target = min(threshold, up((packed + nb - 1) // nb)) if nb > 1 else threshold
    buckets, fill = [], 0
    for i, k in enumerate(sizes):
        nbytes = k * es
        if nbytes == 0:
            continue
        off = up(fill) if buckets else 0
        if not buckets or off + nbytes > threshold or off >= target:
            buckets.append([])
            off = 0
        buckets[-1].append((i, off))
        fill = off + nbytes
    return buckets


def fusion_one_rank_kernels(torch, L, _lib, sizes, offs, rot_sets, cp, stream, moved, tile=8192,
                            threshold=64 << 20):
    """One rank, configs 4/5: (1) the fusion's pack kernel - the launch fusion.cc issues per bucket
    (copy_segs_kernel over the bucket's tiles of the layout), through tips_fused_pack_bucket - over
    rotating gradient sets, HIP events on the launch stream: the dominant kernel's roofline (unpack
    is the same kernel with source and destination swapped); beside it the opt-in merged form, every
    bucket of the step in one launch (TIPS_PACK_MERGE=1, copy_segs_groups_kernel); (2) the whole
    fused step captured
    into one HIP graph per gradient set (torch.cuda.graph around tips_fused_allreduce) and
    replayed: the step without its host cost."""
    nb = int(_lib.check("tips_fused_pack_bucket", L.tips_fused_pack_bucket(rot_sets[0][1], cp, len(sizes),
                                                                          _lib.FLOAT32, -1, None, None)))
    dst = torch.empty(threshold // 4, dtype=torch.float32, device="cuda")
    sp = stream.cuda_stream
    payload = [0] * nb

    def launch(r, b):
        rc = L.tips_fused_pack_bucket(rot_sets[r][1], cp, len(sizes), _lib.FLOAT32, b, dst.data_ptr(), sp)
        if rc < 0:
            raise _lib.TipsError("tips_fused_pack_bucket", int(rc), _lib.last_error())
        payload[b] = int(rc)

    for r in range(len(rot_sets)):  # (builds and uploads every set's tables once)
        for b in range(nb):
            launch(r, b)
    torch.cuda.synchronize()
    # the packed bucket 0 of set 0 holds exactly its tensors' bytes, at the layout's offsets
    launch(0, 0)
    torch.cuda.synchronize()
    import ctypes
    lo = (ctypes.c_int64 * len(sizes))()
    L.tips_fused_layout(cp, len(sizes), _lib.FLOAT32, lo)
    b0 = fusion_layout(sizes, threshold=threshold)[0]
    d8, x0 = dst.view(torch.uint8), rot_sets[0][0]
    ok = all(torch.equal(d8[int(lo[i]):int(lo[i]) + sizes[i] * 4], x0[offs[i]:offs[i] + sizes[i]].view(torch.uint8))
             for i, _ in b0)
    reps = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # a gate: the stream first spins ~5 ms, so every launch below is queued before the first runs
    # and the events time the kernels back to back, not the host issuing them (each
    # tips_fused_pack_bucket call resolves its layout and pointer table on the host)
    with torch.cuda.stream(stream):
        torch.cuda._sleep(12_000_000)
    e0.record(stream)
    for k in range(reps):
        for b in range(nb):
            launch(k % len(rot_sets), b)
    e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (reps * nb)
    per_launch = 2 * sum(payload) / nb  # read + write of one bucket's tensors
    per_bucket = {"us_per_launch": round(us, 2), "algorithmic_bytes_per_launch": int(per_launch),
                  "frac": round(per_launch / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
                  "kernel": "copy_segs_kernel", "check": "bit-exact bucket bytes" if ok else "FAIL: packed bytes differ",
                  "note": "one launch per bucket (tips_fused_pack_bucket), as fusion.cc packed a step before round 6"}
    del dst
    # the step's packs as fusion.cc issues them (round 6): every bucket of the step in ONE launch
    # (copy_segs_groups_kernel, bucket 0's tiles first), timed through tips_fused_allreduce_flat at one
    # rank with TIPS_FUSION_MEASURE_PACK=1 (pack into the flat output; the identity allreduce skipped)
    flat_bytes = int(_lib.check("tips_fused_layout", L.tips_fused_layout(cp, len(sizes), _lib.FLOAT32, None)))
    flat = torch.empty(flat_bytes // 4 + 64, dtype=torch.float32, device="cuda")

    def merged(r):
        rc = L.tips_fused_allreduce_flat(rot_sets[r][1], cp, len(sizes), _lib.FLOAT32, flat.data_ptr(), sp)
        if rc < 0:
            raise _lib.TipsError("tips_fused_allreduce_flat", int(rc), _lib.last_error())

    saved = (os.environ.get("TIPS_FUSION_MEASURE_PACK"), os.environ.get("TIPS_PACK_MERGE"))
    os.environ["TIPS_FUSION_MEASURE_PACK"] = "1"
    os.environ["TIPS_PACK_MERGE"] = "1"
    try:
        for r in range(len(rot_sets)):  # (tables built and uploaded once per set)
            merged(r)
        torch.cuda.synchronize()
        fv = flat.view(torch.uint8)
        ok_m = all(torch.equal(fv[int(lo[i]):int(lo[i]) + sizes[i] * 4],
                               rot_sets[len(rot_sets) - 1][0][offs[i]:offs[i] + sizes[i]].view(torch.uint8))
                   for i in range(len(sizes)))
        with torch.cuda.stream(stream):
            torch.cuda._sleep(12_000_000)
        e0.record(stream)
        for k in range(reps):
            merged(k % len(rot_sets))
        e1.record(stream)
        torch.cuda.synchronize()
    finally:
        for k, v in zip(("TIPS_FUSION_MEASURE_PACK", "TIPS_PACK_MERGE"), saved):
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    mus = e0.elapsed_time(e1) * 1e3 / reps
    per_merged = 2 * sum(payload)  # read + write of every packed tensor of the step
    roof = {"bound": "hbm", "achieved": round(per_launch / (us * 1e-6) / 1e9, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": per_bucket["frac"], "traffic": None,
            "kernel": "copy_segs_kernel (fusion pack; unpack is the same kernel, source and destination swapped)",
            "us_per_launch": round(us, 2), "algorithmic_bytes_per_launch": int(per_launch),
            "launches_per_step": 2 * nb, "buckets": nb, "tile_bytes": tile, "check": per_bucket["check"],
            "merged_launch": {"us_per_launch": round(mus, 2), "algorithmic_bytes_per_launch": int(per_merged),
                              "frac": round(per_merged / (mus * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
                              "kernel": "copy_segs_groups_kernel",
                              "check": "bit-exact packed bytes (every tensor)" if ok_m else "FAIL: packed bytes differ",
                              "note": "TIPS_PACK_MERGE=1 (opt-in): the step's %d buckets in ONE pack launch, through "
                                      "tips_fused_allreduce_flat with TIPS_FUSION_MEASURE_PACK=1" % nb},
            "note": "per-bucket pack launches of fusion.cc's layout (tips_fused_pack_bucket), gradient set i %% %d "
                    "(HBM-only), HIP events on the launch stream; algorithmic bytes = read + write of the bucket's "
                    "tensors" % len(rot_sets)}
    del flat
    # the whole step, captured once per gradient set and replayed
    side = torch.cuda.Stream()
    side.wait_stream(stream)
    graphs = []
    with torch.cuda.stream(side):
        for xs, pp, _k in rot_sets:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                rc = L.tips_fused_allreduce(pp, cp, len(sizes), _lib.FLOAT32, side.cuda_stream)
            if rc:
                raise _lib.TipsError("tips_fused_allreduce (capture)", rc, _lib.last_error())
            graphs.append(g)
        for i in range(2 * len(graphs)):
            graphs[i % len(graphs)].replay()
        torch.cuda.synchronize()
        e0.record(side)
        for i in range(40):
            graphs[i % len(graphs)].replay()
        e1.record(side)
        torch.cuda.synchronize()
    gus = e0.elapsed_time(e1) * 1e3 / 40
    del graphs
    graph = {"us_per_step": round(gus, 2), "achieved": round(moved / (gus * 1e-6) / 1e9, 1),
             "frac": round(moved / (gus * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
             "note": "the fused step (pack, identity, unpack per bucket, stream joins) captured with "
                     "torch.cuda.graph around tips_fused_allreduce, one graph per gradient set, 40 replays"}
    return roof, graph


def gradient_api_legs(torch, dist, tips_amd, world, sizes, offs, rot_sets, steps, fixed_ms):
    """The same gradients through the training API instead of fixed views: every gradient its own
    allocation (a parameter's .grad), as a model hands them over.
      optimizer:       DistributedOptimizer.synchronize() - the allreduce half of step(): every
                       .grad a view of one flat buffer (gradient bucket views), the flat buffer
                       allreduced in place (no pack, no unpack; the first step copies .grad in)
      allreduce_grads: allreduce_grads(grads) - new output tensors, views of one flat buffer
                       (tips_fused_allreduce_flat: each bucket packed into it and allreduced in
                       place, 2 x the gradient bytes in HBM; the flat buffer and its views are
                       reused once the previous call's outputs are released)
    On one rank both are the identity, as the reference's _allreduce_cond (__init__.py:94-103);
    there the call each makes at N > 1 is timed instead.
    Host-timed like the main line, over the same rotating sets; max over ranks."""
    rot = len(rot_sets)
    params = []
    for k in range(rot):
        ps = [torch.nn.Parameter(torch.zeros(n_, device="cuda")) for n_ in sizes]
        for p_, o in zip(ps, offs):
            p_.grad = rot_sets[k][0][o:o + p_.numel()].clone()
        params.append(ps)
    grads = [[p_.grad for p_ in ps] for ps in params]
    opts = [tips_amd.DistributedOptimizer(torch.optim.SGD(ps, lr=0.0)) for ps in params]
    fp16 = tips_amd.Compression.fp16
    if world > 1:
        calls = {"optimizer": lambda i: opts[i].synchronize(whole_groups=True), "allreduce_grads": lambda i: tips_amd.allreduce_grads(grads[i]),
                 "fp16_compressed": lambda i: tips_amd.allreduce_grads(grads[i], compression=fp16)}
        what = "DistributedOptimizer.synchronize() / tips_amd.allreduce_grads (and with Compression.fp16)"
    else:
        from tips_amd.ops import FusedList
        fls = [FusedList([p_.numel() for p_ in ps]) for ps in params]
        flats = [torch.cat([g.reshape(-1) for g in gs]) for gs in grads]  # the optimizer's bucket views
        from tips_amd.optim import _allreduce_flat_
        calls = {"optimizer": lambda i: _allreduce_flat_(flats[i]),
                 "packed_separate_grads": lambda i: fls[i].allreduce_(grads[i]),
                 "allreduce_grads": lambda i: tips_amd._reduce_grads(grads[i]),
                 "fp16_compressed": lambda i: tips_amd._reduce_grads(grads[i], compression=fp16)}
        what = ("one rank: both API calls are the identity (reference _allreduce_cond); timed is what each runs at "
                "N > 1: the optimizer's in-place allreduce of the flat buffer its gradient bucket views live in "
                "(no device work at all on one rank), FusedList.allreduce_ over separately allocated gradients "
                "(pack + unpack), allreduce_grads' N > 1 body (_reduce_grads: pack into one flat output, "
                "per bucket), and the same with Compression.fp16 (one tips_fused_allreduce_cast: cast while packed, "
                "cast back while unpacked; at one rank the reference's round trip f32 -> f16 -> f32)")
    import warnings  # (the optimizer leg calls synchronize() repeatedly with no backward: it warns)
    warnings.filterwarnings("ignore", message="DistributedOptimizer.synchronize")
    out = {"calls": what, "bytes_per_rank": sum(sizes) * 4, "fixed_view_ms": round(fixed_ms, 4)}
    ref = [torch.cat([g.reshape(-1) for g in gs]) for gs in grads] if world == 1 else None
    for name, fn in calls.items():
        # warm every rotating set: a set's first call validates the list and builds its pointer table
        # (~1 ms for 1000 tensors); r04 warmed 3 of the 4 and the 10-step loop paid the fourth's
        # (packed_separate_grads "2.5 x the fixed view": tools/separate_grads_probe.py, 57 vs 58 us)
        for i in range(max(3, 2 * rot)):
            fn(i % rot)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for i in range(steps):
            fn(i % rot)
        torch.cuda.synchronize()
        t = max_over_ranks(dist, time.perf_counter() - t0) / steps
        leg = {"ms_per_step": round(t * 1e3, 4), "vs_fixed_view": round(t * 1e3 / fixed_ms, 3)}
        if world == 1:
            # bucket views: nothing to pack; flat outputs: pack only; separate outputs: pack + unpack
            # (fp16: pack reads 4 B and writes 2 B per element, unpack reads 2 B and writes 4 B)
            moved = {"optimizer": 0, "allreduce_grads": 2 * sum(sizes) * 4,
                     "fp16_compressed": 12 * sum(sizes)}.get(name, 4 * sum(sizes) * 4)
            leg["algorithmic_hbm_bytes"] = moved
            if moved:
                leg["hbm_achieved_GBps"] = round(moved / t / 1e9, 1)
                leg["frac_of_hbm"] = round(moved / t / 1e9 / HBM_PEAK_GBPS, 4)
            got = fn(0)
            torch.cuda.synchronize()
            got = {"optimizer": [flats[0]], "packed_separate_grads": grads[0]}.get(name, got)
            want = ref[0].half().float() if name == "fp16_compressed" else ref[0]  # (torch's cast: RNE, as the oracle's)
            leg["check"] = ("%s, bit-exact" % ("round trip through f16" if name == "fp16_compressed" else "identity")
                            if torch.equal(torch.cat([g.reshape(-1) for g in got]), want) else "FAIL")
            if name == "fp16_compressed" and moved:
                # the device's span: HIP events on the caller's stream around 20 back-to-back calls,
                # the best of 3 (the host-timed figure above includes the Python call per step)
                del got
                s = torch.cuda.current_stream()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                dus = None
                for _ in range(3):
                    e0.record(s)
                    for i in range(20):
                        fn(i % rot)
                    e1.record(s)
                    torch.cuda.synchronize()
                    t_ = e0.elapsed_time(e1) * 1e3 / 20
                    dus = t_ if dus is None else min(dus, t_)
                # PMC: the pack and unpack launches' HBM bytes (mean per launch, one of each per bucket)
                tp, tu = pmc_traffic("cast_segs_kernel<2, 0", "*pmc_cast_pack*.json"), \
                    pmc_traffic("cast_segs_kernel<2, 1", "*pmc_cast_unpack*.json")
                traffic = None
                if tp and tu and sizes == resnet50_grad_sizes():  # (measured on config 5's layout)
                    traffic = round(2 * (tp["bytes"] + tu["bytes"]))
                leg["roofline"] = {"bound": "hbm", "achieved": round(moved / dus / 1e3, 1), "peak": HBM_PEAK_GBPS,
                                   "unit": "GB/s", "frac": round(moved / dus / 1e3 / HBM_PEAK_GBPS, 4), "traffic": traffic,
                                   "us_per_step": round(dus, 2), "kernel": "cast_segs_kernel (pack f32 -> f16, unpack "
                                   "f16 -> f32; one of each per bucket), HIP events around 20 back-to-back calls, best of 3"}
                if traffic:
                    leg["roofline"]["traffic_source"] = "%s + %s" % (tp["source"], tu["source"])
        out[name] = leg
    if "fp16_compressed" in out and "allreduce_grads" in out:
        out["fp16_compressed"]["vs_fp32_allreduce_grads"] = round(
            out["fp16_compressed"]["ms_per_step"] / out["allreduce_grads"]["ms_per_step"], 3)
    del params, grads, opts
    return out


# RCCL reads these once, at its first communicator: a setting can only be compared in a job of its
# own. NCCL_NCHANNELS_PER_PEER is how many channels RCCL gives each peer of a point-to-point group
# (the direct schedule's whole exchange); RCCL's own all-pairs allreduce for 8 GPUs
# (share/rccl/msccl-algorithms/allreduce-allpairs-8n-*.xml) runs 8 thread blocks per peer.
# (8 per peer is left out: over RCCL's socket transport a plain grouped ncclSend/ncclRecv then
# delivers wrong bytes, no TIPS code involved - profiles/r02/rccl_nchannels_probe.txt.)
ENV_VARIANTS = [("nchannels_per_peer_4", {"NCCL_NCHANNELS_PER_PEER": "4"})]


SMALL_BUCKET_KIB = (16, 256, 512, 1024, 2048, 4096, 8192)


def small_bucket_latency(job, torch, dist, _lib, L, rank, sp, calls=40, kibs=SMALL_BUCKET_KIB):
    """Per-call time of small allreduces, 16 KiB - 8 MiB (config 1 is a 1 MiB bucket at p = 2), for
    the path the library ships (AUTO with its default one-shot threshold; replays only if the job
    opted in with TIPS_GRAPHS=1)
    and for each candidate beside it: direct eager, direct replayed as a HIP graph at any size,
    one-shot eager and one-shot replayed. The wall time of `calls` back-to-back calls on the same
    buffers (a quarter of them above 1 MiB), slowest rank; `best` names the fastest candidate and
    `shipped_vs_best` the ratio. Sizes left when the probe has run TIPS_BENCH_PROBE_BUDGET_S (90 s),
    or the job's budget is spent, are skipped, on every rank together."""
    out = {"calls": calls, "calls_above_1MiB": max(5, calls // 4), "unit": "us per call, slowest rank"}
    keys = ("TIPS_GRAPHS", "TIPS_GRAPH_MAX_BYTES")
    saved = {k: os.environ.get(k) for k in keys}
    modes = [("shipped", _lib.ALGO_AUTO, {}),
             ("ring_eager", _lib.ALGO_RING, {"TIPS_GRAPHS": "0"}),
             ("direct_eager", _lib.ALGO_DIRECT, {"TIPS_GRAPHS": "0"}),
             ("direct_graphs", _lib.ALGO_DIRECT, {"TIPS_GRAPHS": "1", "TIPS_GRAPH_MAX_BYTES": str(1 << 40)}),
             ("oneshot_eager", _lib.ALGO_ONESHOT, {"TIPS_GRAPHS": "0"}),
             ("oneshot_graphs", _lib.ALGO_ONESHOT, {"TIPS_GRAPHS": "1", "TIPS_GRAPH_MAX_BYTES": str(1 << 40)})]
    world = dist.get_world_size()

    def use(algo, env):
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(env)
        _lib.call("tips_set_algorithm", algo)

    budget = float(os.environ.get("TIPS_BENCH_PROBE_BUDGET_S", "90"))
    t_start = time.perf_counter()
    try:
        for kib in kibs:
            # a time budget, decided together (the probe's calls are collectives): over sockets at
            # N = 8 the 2-8 MiB sizes take minutes (profiles/r03/m_rehearsal_n8.jsonl), over xGMI seconds
            if max_over_ranks(dist, time.perf_counter() - t_start) > budget or job.left() < 10:
                out["%d_KiB" % kib] = "skipped: the probe's %.0f s budget was spent (TIPS_BENCH_PROBE_BUDGET_S)" % budget
                continue
            reps = calls if kib <= 1024 else max(5, calls // 4)
            n = kib * 256
            x = torch.full((n,), float(rank + 1), device="cuda")
            y = torch.empty_like(x)
            row = {}
            ok = True
            use(_lib.ALGO_AUTO, {})
            shipped = L.tips_resolve_algorithm(world, n * 4)
            # (schedules.cc: replays are opt-in since round 6, TIPS_GRAPH_MAX_BYTES's default 8 MiB)
            graphs = saved.get("TIPS_GRAPHS") not in (None, "", "0") and n * 4 <= (8 << 20)
            for rnd in range(2):  # two interleaved rounds, best of both: no mode always runs first
                for mode, algo, env in (modes if rnd == 0 else modes[::-1]):
                    use(algo, env)
                    y.zero_()
                    for _ in range(3):  # (a plan is captured on its second call)
                        L.tips_allreduce(x.data_ptr(), y.data_ptr(), n, _lib.FLOAT32, _lib.OP_SUM, sp)
                    torch.cuda.synchronize()
                    ok = ok and bool(torch.all(y == world * (world + 1) / 2).item())
                    dist.barrier()
                    t0 = time.perf_counter()
                    for _ in range(reps):
                        L.tips_allreduce(x.data_ptr(), y.data_ptr(), n, _lib.FLOAT32, _lib.OP_SUM, sp)
                    torch.cuda.synchronize()
                    us = round(max_over_ranks(dist, time.perf_counter() - t0) / reps * 1e6, 1)
                    row[mode] = min(us, row.get(mode, us))
            cands = {k: v for k, v in row.items() if k != "shipped"}
            best = min(cands, key=cands.get)
            names = {_lib.ALGO_ONESHOT: "oneshot", _lib.ALGO_RING: "ring", _lib.ALGO_DIRECT: "direct"}
            row["shipped_path"] = "%s %s" % (names.get(shipped, str(shipped)), "graphs" if graphs else "eager")
            row["best"] = best
            row["shipped_vs_best"] = round(row["shipped"] / cands[best], 3)
            row["check"] = "exact (every mode)" if all_ranks_ok(dist, ok) else "FAIL on some rank"
            out["%d_KiB" % kib] = row
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return out


def overlap_probe(torch, dist, tips_amd, _lib, algo_code, job, steps=10):
    """A training step with DistributedOptimizer, its allreduces issued after backward vs during it
    (TIPS_OVERLAP_BACKWARD=1: post-accumulate hooks issue each <= 25 MiB gradient bucket as it
    completes, on a side stream), and the optimizer's default, the measured choice between the two
    (=auto: its trial steps run first, untimed; measured_choice_detail has what it measured and kept). The model is 6 fp32 Linear(2048, 2048) layers, 25.2 M parameters
    (ResNet-50 has 25.6 M), on a 2048-row synthetic batch; wall time per step, slowest rank.
    `backward_only` is the same step without the optimizer (no allreduce): the floor overlap can
    approach. The reference's per-gradient async ops overlap backward the same way
    (__init__.py:212-222). `replay_host_waits` per variant: how often an eager RCCL call found a
    replayed plan pending and blocked the host until it had run (tips_replay_order_stats), and the
    host time it cost per step."""
    saved = os.environ.get("TIPS_OVERLAP_BACKWARD")
    _lib.call("tips_set_algorithm", algo_code)
    out = {"model": "6 x Linear(2048, 2048) + ReLU, fp32, 25.2 M parameters, batch 2048", "steps": steps,
           "unit": "ms per step (forward + backward [+ allreduce + SGD]), slowest rank"}
    g = torch.Generator(device="cuda").manual_seed(77)
    x = torch.randn(2048, 2048, device="cuda", generator=g)
    try:
        for name, overlap, sync in (("backward_only", "0", False), ("allreduce_after_backward", "0", True),
                                    ("allreduce_during_backward", "1", True), ("measured_choice", "auto", True)):
            os.environ["TIPS_OVERLAP_BACKWARD"] = overlap
            torch.manual_seed(5)
            layers = []
            for _ in range(6):
                layers += [torch.nn.Linear(2048, 2048), torch.nn.ReLU()]
            m = torch.nn.Sequential(*layers).cuda()
            opt = tips_amd.DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=1e-6))

            def run(k):
                for _ in range(k):
                    opt.zero_grad(set_to_none=False)
                    m(x).square().mean().backward()
                    if sync:
                        opt.step()

            run(3 if overlap != "auto" else 10)  # (auto: 2 warm-up + 2 x 3 trial steps decide first)
            torch.cuda.synchronize()
            dist.barrier()
            w0 = job.replay_waits()
            t0 = time.perf_counter()
            run(steps)
            torch.cuda.synchronize()
            out[name] = round(max_over_ranks(dist, time.perf_counter() - t0) / steps * 1e3, 3)
            w1 = job.replay_waits()
            out.setdefault("replay_host_waits", {})[name] = {
                "per_step": round((w1[0] - w0[0]) / steps, 2), "ms_per_step": round((w1[1] - w0[1]) / steps / 1e6, 4)}
            if overlap == "1":
                out["buckets"] = len(opt._buckets.buckets) if opt._buckets is not None else 0
            if overlap == "auto":
                out["measured_choice_detail"] = opt.overlap_choice
            del m, opt, layers
    finally:
        if saved is None:
            os.environ.pop("TIPS_OVERLAP_BACKWARD", None)
        else:
            os.environ["TIPS_OVERLAP_BACKWARD"] = saved
    return out


def run_child(cmd, env, budget):
    """One child job (its own process group), killed with its group if it outlasts `budget` s: the
    parsed last JSON line's fields and an "error" when it failed. Never raises: a child never costs
    the main line (a hang costs its own entry, tests/test_distributed_cpu.py pins that)."""
    res = {}
    try:
        if os.environ.get("TIPS_BENCH_CHILD_TEST") == "hang":  # (tests: a child that never ends)
            cmd = [sys.executable, "-c", "import time; time.sleep(100000)"]
        p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                             start_new_session=True)
        _RESULT["child_pgid"] = p.pid
        try:
            o, e = p.communicate(timeout=budget)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            o, e = p.communicate()
            res["error"] = "timed out after %d s (killed with its process group)" % budget
        _RESULT["child_pgid"] = None
        lines = [ln for ln in (o or "").splitlines() if ln.startswith("{")]
        if lines:
            res["line"] = json.loads(lines[-1])
        elif "error" not in res:
            res["error"] = "no result line (exit %s): %s" % (p.returncode, (e or "")[-400:])
    except Exception as ex:  # noqa: BLE001
        res["error"] = "%s: %s" % (type(ex).__name__, ex)
    return res


def child_bucket_jobs(args, dist, rank, world, specs, timeout_s=240):
    """Rank 0 reruns the bucket allreduce as a child job of `world` ranks (torch.distributed.run, the
    same GPUs) per (name, algo, env) in `specs`, while every rank of this job waits at a gloo barrier,
    idle on the GPU. A child that fails or outlasts its budget is killed (its own process group) and
    reported; the main line is never at stake. Returns name -> the child's result."""
    import socket
    out = {}
    for name, algo, env in specs:
        dist.barrier()
        if rank == 0:
            s_ = socket.socket()
            s_.bind(("127.0.0.1", 0))
            port = s_.getsockname()[1]
            s_.close()
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
                   "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__),
                   "--gpus", str(world), "--steps", "10", "--warmup", "2", "--algo", algo, "--no-compare",
                   "--no-sub", "--no-cpu-baseline", "--no-env-variants"] + \
                (["--bucket-mib", str(args.bucket_mib)] if args.bucket_mib else [])
            cenv = {k: v for k, v in os.environ.items()
                    if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                                 "MASTER_PORT", "TORCHELASTIC_RUN_ID", "TIPS_BOOTSTRAP_PORT")}
            cenv.update(env)
            res = {"env": env, "algorithm": algo}
            # within this job's watchdog, with a margin for the line and teardown
            budget = min(timeout_s, int(_RESULT.get("deadline", time.time() + timeout_s) - time.time()) - 40)
            if budget < min(30, timeout_s):
                out[name] = dict(res, error="skipped: %d s left before the watchdog" % (budget + 40))
                dist.barrier()
                continue
            cenv["TIPS_BENCH_WATCHDOG"] = str(max(15, budget - 15))
            r = run_child(cmd, cenv, budget)
            d = r.pop("line", None)
            res.update(r)
            if d:
                res.update({k: d.get(k) for k in ("value", "ms_per_step", "check", "error") if d.get(k) is not None})
                res["algbw_gib_s"] = d.get("algbw_gib_s")
                ring = (d.get("configs") or {}).get("config3_ring") or {}
                if ring:  # the north star's ring under this setting (more channels per xGMI link)
                    res["config3_ring"] = {k: ring.get(k) for k in ("ms_per_step", "busbw_GBps", "pipeline_depth",
                                                                    "check")}
                    res["config3_ring"]["frac_of_one_link"] = (ring.get("roofline") or {}).get("frac_of_one_link")
            out[name] = res
        dist.barrier()
    return out


def env_variant_jobs(args, dist, rank, world, timeout_s=240):
    """The direct schedule under each RCCL setting of ENV_VARIANTS, as child jobs."""
    return child_bucket_jobs(args, dist, rank, world, [(n, "direct", env) for n, env in ENV_VARIANTS], timeout_s)


# The MI355X-native peer schedules (peer.cc: our own kernels over IPC-mapped peer memory, xGMI), as
# child jobs on every N > 1 line: the push form and the fused pull-fold, whose
# reduce-scatter is one kernel per rank reading every peer's slice over its xGMI link.
PEER_CHILDREN = [("peer", "peer", {"TIPS_BENCH_CHILD_NO_RING": "1"}),
                 ("peer_pullfold", "peer", {"TIPS_PEER_RS": "pullfold", "TIPS_BENCH_CHILD_NO_RING": "1"})]


_RESULT = {}  # rank 0's finished result line, if the main measurement completed


def crash_line():
    """rank 0's last-words hook (tools/crash_line.c): once installed, a fatal signal (a GPU fault's
    SIGABRT, torchrun's SIGTERM after another rank died) still prints the line measured so far.
    Returns set(text or None), or None when the helper is not built."""
    import ctypes
    path = os.path.join(REPO, "tools", "lib", "libcrashline.so")
    if not os.path.exists(path):
        return None
    try:
        h = ctypes.CDLL(path)
    except OSError:
        return None
    h.crash_line_set.argtypes = [ctypes.c_char_p]
    if h.crash_line_install() != 0:
        return None
    return lambda text: h.crash_line_set(text.encode() if text else None)


_T0 = time.time()


def progress(rank, what):
    """Rank 0's phase log on stderr (the JSON line alone goes to stdout): a long N > 1 run, the
    socket rehearsals above all, shows where it is."""
    if rank == 0:
        print("[bench %7.1f s] %s" % (time.time() - _T0, what), file=sys.stderr, flush=True)


def start_watchdog(seconds, rank):
    """A hung collective must end the run with a message, never hang the box. If the main
    measurement already finished (only the optional comparison runs hung), its line is printed."""
    import threading

    def fire():
        sys.stderr.write("bench.py rank %d: watchdog fired after %d s (hung collective?)\n" % (rank, seconds))
        if _RESULT.get("child_pgid"):  # an RCCL-setting child job still running: it goes too
            try:
                os.killpg(_RESULT["child_pgid"], signal.SIGKILL)
            except OSError:
                pass
        line = _RESULT.get("line")
        if _RESULT.get("printed"):  # the one JSON line is out; only teardown hung
            os._exit(0)
        if rank == 0:
            if line is not None:
                line = dict(line, compare_error="comparison runs did not finish within %d s" % seconds)
            else:
                line = {"metric": METRIC, "value": None, "error": "watchdog: no progress in %d s" % seconds}
            print(json.dumps(line), flush=True)
        os._exit(0 if _RESULT.get("done") else 3)

    _RESULT["deadline"] = time.time() + seconds
    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t



# ----------------------------------------------------------------------------- the job

class Job(object):
    """What every measurement of one run shares: torch, the gloo group the ranks time and agree
    through, the library, this rank's stream, and the time budget of the optional legs."""

    def __init__(self, args, torch, dist, tips_amd, _lib):
        self.args, self.torch, self.dist, self.tips_amd, self._lib = args, torch, dist, tips_amd, _lib
        self.L = _lib.lib()
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.stream = torch.cuda.current_stream()
        self.sp = self.stream.cuda_stream
        self.algo_names = {"auto": _lib.ALGO_AUTO, "ring": _lib.ALGO_RING, "direct": _lib.ALGO_DIRECT,
                           "rccl": _lib.ALGO_RCCL, "oneshot": _lib.ALGO_ONESHOT, "peer": _lib.ALGO_PEER,
                           "tune": _lib.ALGO_TUNE}
        self.inv = {v: k for k, v in self.algo_names.items()}
        self.budget_s = float(os.environ.get("TIPS_BENCH_BUDGET_S", "240"))
        self.skipped = []

    def left(self):
        """Seconds of the budget left, the same number on every rank (slowest rank's clock): a
        collective, so every rank asks at the same points."""
        return self.budget_s - max_over_ranks(self.dist, time.time() - _T0)

    def afford(self, what, need_s):
        """True when `need_s` seconds of the budget are left (decided together); else notes `what`."""
        if self.left() >= need_s:
            return True
        self.skipped.append(what)
        progress(self.rank, "budget: skipping %s" % what)
        return False

    def replay_waits(self):
        import ctypes
        w, ns = ctypes.c_int64(), ctypes.c_int64()
        self._lib.call("tips_replay_order_stats", ctypes.byref(w), ctypes.byref(ns))
        return w.value, ns.value


# ----------------------------------------------------------------------------- N == 1: config 2's bucket sum

def sum_record(args, cpu):
    """Config 2, the N == 1 headline: tips_bucket_sum over 4 rotating 256 MiB triples."""
    steps = args.steps if args.steps is not None else 200
    warmup = args.warmup if args.warmup is not None else 20
    n = (args.bucket_mib or 256) * (1 << 20) // 4

    import torch
    import tips_amd
    from tips_amd import _lib
    L = _lib.lib()
    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    # ROTATING_SETS (a, b, c) triples, 768 MiB each: step i sums triple i % ROTATING_SETS, so 2.25 GiB
    # of other traffic separates two uses of a buffer and no launch finds its operands in the
    # 256 MiB Infinity Cache: the timed rate is HBM's. Triple 0 is config 2's seeded pair (seeds 1, 2).
    sets = []
    for k in range(ROTATING_SETS):
        x_, y_, z_ = (torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(3))
        g.manual_seed(1 if k == 0 else 10 + 2 * k)
        x_.uniform_(-1.0, 1.0, generator=g)
        g.manual_seed(2 if k == 0 else 11 + 2 * k)
        y_.uniform_(-1.0, 1.0, generator=g)
        sets.append((x_, y_, z_))
    a, b, c = sets[0]

    def step(i=0):
        x_, y_, z_ = sets[i % len(sets)]
        rc = L.tips_bucket_sum(z_.data_ptr(), x_.data_ptr(), y_.data_ptr(), n, _lib.FLOAT32, sp)
        if rc:
            raise _lib.TipsError("tips_bucket_sum", rc, _lib.last_error())

    def timed(k, same_buffers):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for i in range(k):
            step(0 if same_buffers else i)
        ev1.record(stream)
        torch.cuda.synchronize()
        return ev0.elapsed_time(ev1) / k, time.perf_counter() - t0  # HIP events on the kernel's stream

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    ms, wall = timed(steps, same_buffers=False)
    ok = all(bool(torch.equal(z_, x_ + y_)) for x_, y_, z_ in sets)  # one IEEE add per element: bit-exact

    same = None
    if not args.no_extras:
        # the same kernel re-reading ONE triple (the literal config-2 loop): part of each launch's
        # operands is still in the Infinity Cache from the launch before, so this is not an HBM rate
        step(0)
        ms_same, _ = timed(steps, same_buffers=True)
        same = {"us_per_launch": round(ms_same * 1e3, 2), "achieved_GBps": round(3 * n * 4 / (ms_same / 1e3) / 1e9, 1),
                "note": "tips_bucket_sum on the same (a, b, c) every launch: the 256 MiB Infinity Cache serves part "
                        "of the 768 MiB working set from the previous launch, so this exceeds the HBM-only rate above"}
    del sets[1:]  # (the PCIe leg below uses triple 0)

    t_host, host_rates, host_ok = None, {}, True
    if not args.no_extras:  # (skipped under rocprofv3: its kernel stats then hold only the timed launches)
        # PCIe-inclusive rate (the path starts and ends in host memory): pinned H2D a,b + sum + D2H c
        ha, hb, hc = (torch.empty(n, dtype=torch.float32, pin_memory=True) for _ in range(3))
        ha.copy_(a)
        hb.copy_(b)
        torch.cuda.synchronize()
        reps = 3
        t1 = time.perf_counter()
        for _ in range(reps):
            a.copy_(ha, non_blocking=True)
            b.copy_(hb, non_blocking=True)
            step()
            hc.copy_(c, non_blocking=True)
        torch.cuda.synchronize()
        t_host = (time.perf_counter() - t1) / reps
        del ha, hb, hc

        # host-memory leg of the drop-in path: tips_allreduce on host buffers (1 rank: H2D, device copy, D2H)
        import numpy as np
        pinned_in = torch.empty(n, dtype=torch.float32, pin_memory=True)
        pinned_out = torch.empty(n, dtype=torch.float32, pin_memory=True)
        pageable_in = np.random.default_rng(1).random(n, dtype=np.float32)
        pageable_out = np.empty_like(pageable_in)
        tips_amd.init()
        reg_in = np.random.default_rng(2).random(n, dtype=np.float32)
        reg_out = np.empty_like(reg_in)
        _lib.call("tips_host_register", reg_in.ctypes.data, reg_in.nbytes)
        _lib.call("tips_host_register", reg_out.ctypes.data, reg_out.nbytes)
        for label, src, dst in (("pageable_numpy", pageable_in.ctypes.data, pageable_out.ctypes.data),
                                ("pinned", pinned_in.data_ptr(), pinned_out.data_ptr()),
                                ("registered_numpy", reg_in.ctypes.data, reg_out.ctypes.data)):
            _lib.call("tips_allreduce", src, dst, n, _lib.FLOAT32, _lib.OP_SUM, None)  # warm (allocates staging)
            ts = []
            for _ in range(5):
                t2 = time.perf_counter()
                _lib.call("tips_allreduce", src, dst, n, _lib.FLOAT32, _lib.OP_SUM, None)
                ts.append(time.perf_counter() - t2)
            host_rates[label] = round(n * 4 / sorted(ts)[2] / GIB, 3)  # median of 5 calls
            host_rates[label + "_calls_ms"] = [round(t * 1e3, 3) for t in ts]
        host_ok = bool(np.array_equal(pageable_out, pageable_in)) and bool(np.array_equal(reg_out, reg_in))
        _lib.call("tips_host_unregister", reg_in.ctypes.data)
        _lib.call("tips_host_unregister", reg_out.ctypes.data)
        del pinned_in, pinned_out, pageable_in, pageable_out, reg_in, reg_out
    del sets, a, b, c
    torch.cuda.empty_cache()

    moved = 3 * n * 4
    t_s = ms / 1e3
    achieved = moved / t_s / 1e9
    tr = pmc_traffic(DEFAULT_SUM_KERNEL)
    line = {
        "metric": METRIC, "value": round(moved / t_s / GIB, 2), "unit": "GiB/s", "n_gpus": 1, "steps": steps,
        "warmup": warmup, "ms_per_step": round(ms, 6), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": "synthetic: fp32 U[-1,1), torch cuda generator seeds 1 and 2 (+ %d more seeded pairs), resident in HBM"
                % (ROTATING_SETS - 1),
        "config": {"workload": "config 2: c = a + b, two 256 MiB fp32 gradient buffers on one MI355X",
                   "bucket_bytes": n * 4, "elements": n, "rotating_sets": ROTATING_SETS,
                   "timing": "HIP events over the timed launches; launch i sums triple i %% %d (HBM-only: no launch "
                             "finds its operands in the 256 MiB Infinity Cache)" % ROTATING_SETS, "kernel": "tips_bucket_sum (sum2_buf_kernel<f32, nt loads, nt stores>: one 2 KiB tile per operand per 128-lane workgroup, tiles dealt to the 8 XCDs in stripes of TIPS_STRIPE_KIB, buffer_load/store_dwordx4)",
                   "parallelism": "single GPU"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": (tr["bytes"] if tr else None)},
        "cpu_baseline": cpu,
        "same_buffers_repeated": same,
        "input_bucket_gib_s": round(n * 4 / t_s / GIB, 2),
        "algorithmic_bytes_per_step": moved,
        "pcie_inclusive_gib_s": round(n * 4 / t_host / GIB, 3) if t_host else None,
        "pcie_inclusive_note": "pinned H2D of a and b + kernel + D2H of c, bucket bytes / wall time",
        "host_allreduce_gib_s": host_rates,
        "host_allreduce_note": "tips_allreduce(host in, host out) on one rank, 256 MiB: staged H2D + device + D2H, "
                               "bucket bytes / median wall time of 5 calls (all 5 listed)" + ("" if host_ok else " (RESULT MISMATCH)"),
        "check": "bit-exact vs torch a+b" if ok else "FAIL",
        "wall_s_timed_region": round(wall, 4),
    }
    if tr:
        line["roofline"]["traffic_source"] = tr["source"]
    return line, ok


# ----------------------------------------------------------------------------- one allreduce workload

class Workload(object):
    """One workload through the library at this job's N: config 3's bucket (tips_allreduce), configs
    4 / 5 fused (tips_fused_allreduce over the gradient set's views), or config 4 as 1000 named
    requests (negotiated1000). setup -> warm (schedules tuned) -> timed -> parity -> record; the
    headline's comparison schedules reuse its buffers (compare)."""

    def __init__(self, job, workload, steps, warmup):
        self.job, self.workload, self.steps, self.warmup = job, workload, steps, warmup
        torch, L, _lib, world, rank = job.torch, job.L, job._lib, job.world, job.rank
        self.measure_pack = world == 1 and workload in SUB_WORKLOADS
        # one rank: the library does no bucket work at all (the allreduce is the identity); pack and
        # unpack the buckets anyway, as at N > 1, so this record measures the fusion's per-step HBM cost
        self._saved_pack = os.environ.get("TIPS_FUSION_MEASURE_PACK")
        if self.measure_pack:
            os.environ["TIPS_FUSION_MEASURE_PACK"] = "1"
        self.g = torch.Generator(device="cuda")
        if workload == "bucket":
            sizes = [(job.args.bucket_mib or 1024) * (1 << 20) // 4]
            seed0, desc = 3000, "config 3: allreduce of one 1 GiB fp32 bucket per GPU over xGMI"
        elif workload == "fused1000":
            sizes, seed0 = fused1000_sizes(), 4000
            desc = "config 4: 1000 fp32 grads (2^U(8,17) elems) fused into 64 MiB buckets, allreduced in place"
        elif workload == "negotiated1000":
            sizes, seed0 = fused1000_sizes(), 4000
            desc = ("config 4 without fusion: 1000 fp32 grads, one named allreduce each through the negotiated "
                    "path (tips_enqueue_allreduce/tips_wait), the reference's per-tensor structure")
        else:
            sizes, seed0 = resnet50_grad_sizes(), 5000
            desc = "config 5: ResNet-50 gradient set (214 tensors, 25.6 M fp32) fused into 64 MiB buckets, in place"
        self.sizes, self.seed0, self.desc = sizes, seed0, desc
        # the schedule the (largest) reduced buffer gets: the bucket itself, or a <= 64 MiB fusion bucket
        self.qbytes = sizes[0] * 4 if workload == "bucket" else max(sizes) * 4 if workload == "negotiated1000" else 64 << 20
        self.algo = L.tips_resolve_algorithm(world, self.qbytes)
        # every tensor at a 256-B aligned offset of one flat buffer, 256 B apart at least, as separate
        # allocations of a caching allocator lie: the fusion path packs them (its layout depends only on
        # the counts). (A flat gradient buffer allreduced as one tensor is the gradient_api "optimizer" leg.)
        offs, total = [], 0
        gap = 64 if workload in SUB_WORKLOADS else 0
        for k in sizes:
            offs.append(total)
            total += (k + 63) // 64 * 64 + gap
        if workload == "bucket":
            total = sizes[0]  # the parity check compares the whole output buffer
        self.offs, self.total, self.total_elems = offs, total, sum(sizes)
        self.x = torch.empty(total, dtype=torch.float32, device="cuda")
        self.fill(self.x, rank)
        self.y = torch.empty_like(self.x) if workload == "bucket" else self.x
        views = [self.x[o:o + k] for o, k in zip(offs, sizes)]
        pp, keep1 = _lib.ptr_array([v.data_ptr() for v in views])
        self.cp, self._keep2 = _lib.i64_array(sizes)
        # The fused workloads cycle over ROTATING_SETS gradient sets (step i reduces set i % R): the
        # 83-102 MB of one set would otherwise stay in the 256 MiB Infinity Cache from one step to the
        # next, and a one-rank record (pack + unpack only) would not be an HBM rate.
        self.rot = ROTATING_SETS if workload in SUB_WORKLOADS else 1
        self.rot_sets = [(self.x, pp, keep1)]
        for k in range(1, self.rot):
            xk = torch.empty(total, dtype=torch.float32, device="cuda")
            self.fill(xk, rank + 100 * k)
            self.rot_sets.append((xk,) + _lib.ptr_array([xk[o:o + n_].data_ptr() for o, n_ in zip(offs, sizes)]))
        self.ctr = 0
        import ctypes
        self.names = [("grad.%d" % i).encode() for i in range(len(sizes))]
        self.view_ptrs = [v.data_ptr() for v in views]
        self.host_t = {"enqueue": 0.0, "wait": 0.0}
        self.per_call = False
        self.name_arr = (ctypes.c_char_p * len(self.names))(*self.names)
        self.h_arr = (ctypes.c_int64 * len(sizes))()
        self.fallbacks = []
        self.tuned = None

    def fill(self, t, r):
        self.g.manual_seed(self.seed0 + r)
        t.uniform_(0.5, 1.5, generator=self.g)

    def step(self):
        job, L, _lib = self.job, self.job.L, self.job._lib
        w = self.workload
        if w == "bucket":
            rc = L.tips_allreduce(self.x.data_ptr(), self.y.data_ptr(), self.sizes[0], _lib.FLOAT32, _lib.OP_SUM, job.sp)
        elif w == "negotiated1000" and self.per_call:  # one ctypes call per tensor (Python-bound)
            t0 = time.perf_counter()
            hs = [L.tips_enqueue_allreduce(nm, p_, p_, k, _lib.FLOAT32, job.sp)
                  for nm, p_, k in zip(self.names, self.view_ptrs, self.sizes)]
            t1 = time.perf_counter()
            rc = next((int(h) for h in hs if h < 0), 0)
            for h in hs:
                if h > 0:
                    wr = L.tips_wait(h)
                    rc = rc or (wr if wr < 0 else 0)
            self.host_t["enqueue"] += t1 - t0
            self.host_t["wait"] += time.perf_counter() - t1
        elif w == "negotiated1000":  # the same 1000 named requests, one library call each way
            t0 = time.perf_counter()
            rc = L.tips_enqueue_allreduce_n(self.name_arr, self.rot_sets[0][1], self.rot_sets[0][1], self.cp,
                                            len(self.sizes), _lib.FLOAT32, job.sp, self.h_arr)
            t1 = time.perf_counter()
            if rc == 0:
                rc = L.tips_wait_n(self.h_arr, len(self.sizes))
            self.host_t["enqueue"] += t1 - t0
            self.host_t["wait"] += time.perf_counter() - t1
        else:
            rc = L.tips_fused_allreduce(self.rot_sets[self.ctr % self.rot][1], self.cp, len(self.sizes),
                                        _lib.FLOAT32, job.sp)
            self.ctr += 1
        if rc:
            raise _lib.TipsError("allreduce", rc, _lib.last_error())

    def timed(self, k):
        job = self.job
        job.dist.barrier()
        job.torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            self.step()
        job.torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        job.dist.barrier()
        return max_over_ranks(job.dist, dt)

    def warm(self):
        """The warm-up steps (the tuner measures the schedules on its first call of a size class). A
        schedule that fails outright on this node (an error on every rank, not a hang) must not cost
        the record: the next one is measured instead and the failure is reported."""
        job, _lib = self.job, self.job._lib
        while True:
            try:
                for _ in range(self.warmup):
                    self.step()
                job.torch.cuda.synchronize()
                break
            except _lib.TipsError as e:
                nxt = {_lib.ALGO_DIRECT: _lib.ALGO_RING, _lib.ALGO_PEER: _lib.ALGO_DIRECT, _lib.ALGO_TUNE: _lib.ALGO_DIRECT,
                       _lib.ALGO_ONESHOT: _lib.ALGO_RING, _lib.ALGO_RING: _lib.ALGO_RCCL}.get(self.algo)
                if self.workload == "negotiated1000" or nxt is None:
                    raise
                self.fallbacks.append({"algorithm": job.inv.get(self.algo, str(self.algo)), "error": str(e)})
                self.algo = nxt
                _lib.call("tips_set_algorithm", self.algo)
        if self.algo == _lib.ALGO_TUNE:  # the warm-up measured the schedules; report (and check) the one kept
            import ctypes
            ta, td, tl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            if job.L.tips_tuned_schedule(self.qbytes, ctypes.byref(ta), ctypes.byref(td), ctypes.byref(tl)) == 1:
                self.tuned = {"algorithm": job.inv.get(ta.value, str(ta.value)), "pipeline_depth": td.value,
                              "lanes": tl.value}
                self.algo = ta.value

    def parity(self, algo_now):
        """One fresh call, then fold all ranks' seeded inputs on this device (rank order) and compare."""
        torch, _lib, world = self.job.torch, self.job._lib, self.job.world
        self.fill(self.x, self.job.rank)
        self.ctr = 0  # (the fused workloads: reduce set 0, i.e. x)
        self.step()
        torch.cuda.synchronize()
        tmp = torch.empty_like(self.x)
        ref = None
        for r in range(world):
            self.fill(tmp, r)
            ref = tmp.clone() if ref is None else ref + tmp
        w = self.workload
        got = torch.cat([self.y[o:o + k] for o, k in zip(self.offs, self.sizes)]) if w != "bucket" else self.y
        exp = torch.cat([ref[o:o + k] for o, k in zip(self.offs, self.sizes)]) if w != "bucket" else ref
        if algo_now in (_lib.ALGO_DIRECT, _lib.ALGO_PEER, _lib.ALGO_ONESHOT) or world == 1:
            good = bool(torch.equal(got, exp))
            msg = "bit-exact vs rank-order fold of all ranks' inputs" if good else "FAIL (not bit-exact)"
        else:
            rel = ((got.double() - exp.double()).abs() / exp.double()).max().item()
            good = rel <= 1e-6
            msg = ("max rel err %.2e vs rank-order fold (bound 1e-6)" % rel) if good else ("FAIL rel %.2e" % rel)
        del ref, tmp, got, exp
        return good, msg

    def run(self):
        """Warm, time `steps` steps (max over ranks), check parity on every rank: the record."""
        job = self.job
        self.warm()
        progress(job.rank, "%s: warm-up done" % self.workload)
        self.host_t.update(enqueue=0.0, wait=0.0)
        w0 = job.replay_waits()
        t = self.timed(self.steps)
        w1 = job.replay_waits()
        self.host_split = dict(self.host_t)
        self.ms = t / self.steps * 1e3
        progress(job.rank, "%s: %.3f ms per step" % (self.workload, self.ms))
        ok, check = self.parity(self.algo)
        self.ok = all_ranks_ok(job.dist, ok)
        progress(job.rank, "%s parity: %s" % (self.workload, check))
        return self.record(check, (w1[0] - w0[0], w1[1] - w0[1]))

    def record(self, check, waits):
        job, world, _lib = self.job, self.job.world, self.job._lib
        ms = self.ms
        algbw = self.total_elems * 4 / (ms / 1e3)  # bytes/s per rank
        busbw = algbw * 2 * (world - 1) / world
        links = 1 if self.algo == _lib.ALGO_RING else max(1, world - 1)
        rec = {
            "value": round(world * self.total_elems * 4 / (ms / 1e3) / GIB, 2), "unit": "GiB/s",
            "value_definition": "N x bytes per rank / time (bytes reduced by the whole job per second)",
            "n_gpus": world, "steps": self.steps, "warmup": self.warmup, "ms_per_step": round(ms, 4),
            "workload": self.desc, "tensors": len(self.sizes), "bytes_per_rank": self.total_elems * 4,
            "algorithm": job.inv.get(self.algo, str(self.algo)) if world > 1 else "none (1 rank)",
            "selection": ("TIPS_ALGO_TUNE: measured on the first call, kept: %s" % self.tuned) if self.tuned else job.args.algo,
            "rotating_sets": self.rot,
            "data": "synthetic: fp32 U[0.5,1.5), torch cuda generator seed %d+rank, resident in HBM" % self.seed0,
            "algbw_gib_s": round(algbw / GIB, 2), "busbw_GBps": round(busbw / 1e9, 2),
            "roofline": {"bound": "xgmi", "achieved": round(busbw / 1e9, 1), "peak": XGMI_LINK_GBPS * links,
                         "unit": "GB/s", "frac": round(busbw / 1e9 / (XGMI_LINK_GBPS * links), 4), "traffic": None,
                         "links_used": links, "frac_of_one_link": round(busbw / 1e9 / XGMI_LINK_GBPS, 4),
                         "note": "multi-GPU: the ring/all-pairs transfer, not the sum kernel, bounds the step"},
            "replay_host_waits": {"count": waits[0], "ms_total": round(waits[1] / 1e6, 3)},
            "check": check if self.ok else "FAIL on some rank",
        }
        if self.fallbacks:
            rec["failed_schedules"] = self.fallbacks
        if world == 1:  # one rank: no link carries anything; the step is HBM work on this GPU
            # bucket: the allreduce is a copy (read + write); fused: pack + unpack (2 reads + 2 writes)
            moved = (2 if self.workload == "bucket" else 4) * self.total_elems * 4
            rec["roofline"] = {"bound": "hbm", "achieved": round(moved / (ms / 1e3) / 1e9, 1), "peak": HBM_PEAK_GBPS,
                               "unit": "GB/s", "frac": round(moved / (ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                               "traffic": None,
                               "note": "one rank: the allreduce of a bucket is the identity; %s" % (
                                   "in -> out copy (copy_buf_kernel: 4 KiB tiles, nt loads, sc1 stores)" if self.workload == "bucket" else
                                   "algorithmic bytes = pack + unpack of every tensor (2 reads + 2 writes); step i "
                                   "reduces gradient set i %% %d, so no step finds its gradients in the 256 MiB "
                                   "Infinity Cache" % self.rot)}
            del rec["busbw_GBps"]
            if self.workload == "bucket":  # the copy kernel's own PMC passes (tools/gpu_pmc_round.sh)
                tr = pmc_traffic("copy_buf_kernel", "*pmc_bucket.json")
                if tr:
                    rec["roofline"]["traffic"] = round(tr["bytes"])
                    rec["roofline"]["traffic_source"] = tr["source"]
            if self.measure_pack:  # the dominant kernel (fusion pack / unpack) timed per launch; the step beside it
                rec["fusion_one_rank"] = ("TIPS_FUSION_MEASURE_PACK=1: buckets packed and unpacked as at N > 1 (the "
                                          "default one-rank path does no bucket work)")
                rec["step_roofline"] = rec["roofline"]
                rec["step_roofline"]["note"] = "whole eager step (launches, stream joins, table lookup)" + \
                    rec["step_roofline"]["note"][len("one rank"):]
                rec["roofline"], rec["graph_replayed_step"] = fusion_one_rank_kernels(
                    job.torch, job.L, _lib, self.sizes, self.offs, self.rot_sets, self.cp, job.stream, moved)
                rec["eager_vs_graph_replayed"] = round(ms * 1e3 / rec["graph_replayed_step"]["us_per_step"], 3)
                tr = pmc_traffic("copy_segs_kernel", "*pmc_%s.json" % self.workload)  # this workload's PMC passes
                if tr:
                    rec["roofline"]["traffic"] = round(tr["bytes"])
                    rec["roofline"]["traffic_source"] = tr["source"]
        if self.workload == "negotiated1000":
            rec["placement"] = thread_placement()  # (right after the timed steps: where they ran)
            rec["per_tensor_us"] = round(ms * 1e3 / len(self.sizes), 2)
            rec["host_us_per_tensor"] = {k: round(v / self.steps / len(self.sizes) * 1e6, 2) for k, v in self.host_split.items()}
            rec["api"] = "tips_enqueue_allreduce_n + tips_wait_n (1000 named requests, one call each way)"
            rec["response_cache"] = "on" if os.environ.get("TIPS_RESPONSE_CACHE", "1") != "0" else "off"
            if world > 1 and self.job.args.workload == "auto":  # (a sub-record at N > 1: the list API only)
                return rec
            self.per_call = True  # the same requests through one ctypes call per tensor, for comparison
            for _ in range(2):
                self.step()
            self.host_t.update(enqueue=0.0, wait=0.0)
            tpc = self.timed(self.steps)
            rec["per_call_api_per_tensor_us"] = round(tpc / self.steps / len(self.sizes) * 1e6, 2)
            rec["per_call_api_host_us_per_tensor"] = {k: round(v / self.steps / len(self.sizes) * 1e6, 2)
                                                      for k, v in self.host_t.items()}
            self.per_call = False
        return rec

    def reduce_kernel_roofline(self):
        """The reduce kernel of this schedule, timed alone at its per-launch shape (HBM roofline)."""
        job, torch, _lib, world = self.job, self.job.torch, self.job._lib, self.job.world
        if not (world > 1 and self.workload == "bucket" and self.algo in (_lib.ALGO_RING, _lib.ALGO_DIRECT)):
            return None
        import ctypes
        depth, sub = ctypes.c_int(), ctypes.c_int64()
        _lib.call("tips_schedule_shape", self.sizes[0], world, _lib.FLOAT32, ctypes.byref(depth), ctypes.byref(sub))
        m = sub.value
        nsrc = world if self.algo == _lib.ALGO_DIRECT else 2
        bufs = torch.empty((nsrc + 1) * m, dtype=torch.float32, device="cuda").uniform_(0.5, 1.5)
        srcs = [bufs[j * m:(j + 1) * m] for j in range(nsrc)]
        dst = bufs[nsrc * m:]
        sp_arr, _keep3 = _lib.ptr_array([t.data_ptr() for t in srcs])

        def kern():
            if nsrc == 2:
                _lib.call("tips_bucket_sum", dst.data_ptr(), srcs[0].data_ptr(), srcs[1].data_ptr(), m, _lib.FLOAT32, job.sp)
            else:
                _lib.call("tips_multi_sum", dst.data_ptr(), sp_arr, nsrc, m, _lib.FLOAT32, job.sp)

        for _ in range(3):
            kern()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(job.stream)
        for _ in range(50):
            kern()
        e1.record(job.stream)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 50 * 1e3
        kbytes = (nsrc + 1) * m * 4
        roof = {"kernel": "multi_sum_buf_kernel" if nsrc > 2 else "sum2_buf_kernel", "sources": nsrc,
                "elements_per_launch": m, "launches_per_step": depth.value * (world - 1 if nsrc == 2 else 1),
                "bound": "hbm", "achieved": round(kbytes / (us * 1e-6) / 1e9, 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(kbytes / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
                "us_per_launch": round(us, 2), "algorithmic_bytes_per_launch": kbytes,
                "note": "one launch of the schedule's sub-chunk shape, timed alone on re-read buffers "
                        "(Infinity Cache assisted: in the schedule a freshly received slot may be on-die too)"}
        if nsrc > 2:  # HBM bytes from the committed PMC passes over the fold (8 x 32 MiB, rotating sets)
            try:
                with open(os.path.join(REPO, "profiles", "r05", "pmc_multi_sum.json")) as f:
                    k = next(iter(json.load(f)["kernels"].values()))
                roof["traffic_over_algorithmic_pmc"] = round(k["traffic_over_algorithmic"], 5)
                roof["traffic_source"] = "profiles/r05/pmc_multi_sum.json (8 x 32 MiB sources, the round-5 fold)"
            except Exception:  # noqa: BLE001
                pass
        del bufs, srcs, dst
        return roof

    def close(self):
        if self.measure_pack:
            if self._saved_pack is None:
                os.environ.pop("TIPS_FUSION_MEASURE_PACK", None)
            else:
                os.environ["TIPS_FUSION_MEASURE_PACK"] = self._saved_pack
        del self.rot_sets, self.x, self.y
        self.job.torch.cuda.synchronize()
        self.job.torch.cuda.empty_cache()


def host_legs(job, w, line):
    """Config 5 host -> host (the gradients in host memory, as the reference's CPU op has them): the
    gradients through allreduce_grads' N > 1 body (one fused host call), and at one rank also one
    tips_amd.allreduce per numpy gradient (the reference's per-op structure; at N > 1 that leg would
    cost the rehearsal's budget minutes, and the fused one is what allreduce_grads runs)."""
    import numpy as np
    tips_amd, world, sizes = job.tips_amd, job.world, w.sizes
    hg = [np.random.default_rng(w.seed0 + job.rank * 1000 + i).random(k, dtype=np.float32) for i, k in enumerate(sizes)]
    hsteps = max(3, w.steps // 4)
    th = None
    if world == 1:
        for gr in hg:
            tips_amd.allreduce(gr)
        job.dist.barrier()
        t0 = time.perf_counter()
        for _ in range(hsteps):
            for gr in hg:  # each result consumed at once, as the optimizer would (no 100 MB of live outputs)
                tips_amd.allreduce(gr)
        th = max_over_ranks(job.dist, time.perf_counter() - t0) / hsteps
        outs = [tips_amd.allreduce(gr) for gr in hg]
        h_ok = all(np.array_equal(o, gr) for o, gr in zip(outs, hg))
        line["host_to_host_python"] = {
            "ms_per_step": round(th * 1e3, 3), "algbw_gib_s": round(w.total_elems * 4 / th / GIB, 2),
            "us_per_tensor": round(th * 1e6 / len(sizes), 2), "steps": hsteps,
            "check": "identity at one rank" if h_ok else "FAIL",
            "note": "214 numpy gradients, one tips_amd.allreduce each (host staged), the reference's per-op structure"}
    # The same 214 numpy gradients through allreduce_grads' N > 1 body: one fused host call
    # (tips_fused_allreduce_host_flat: host threads pack page-locked pieces, H2D -> allreduce -> D2H
    # pipelined per piece, straight into a page-locked flat output).
    for _ in range(2):
        outs = tips_amd._reduce_grads(hg)
    # each call timed on its own (max over ranks per call): the host side of the box is shared
    # with other jobs, and one call in ten can take 2-3 x the others (profiles/r03/b_host_probe.txt);
    # the median is the rate, the mean and the best are reported beside it
    fsteps = max(hsteps, 15) if world == 1 else 5
    per = []
    for _ in range(fsteps):
        job.dist.barrier()
        t0 = time.perf_counter()
        outs = tips_amd._reduce_grads(hg)
        per.append(max_over_ranks(job.dist, time.perf_counter() - t0))
    tf = sorted(per)[len(per) // 2]
    f_ok = all(np.array_equal(o, gr) for o, gr in zip(outs, hg)) if world == 1 else None
    if world > 1:  # the fused host result against the fold of every rank's regenerated inputs
        exp = None
        for r in range(world):
            xs = [np.random.default_rng(w.seed0 + r * 1000 + i).random(k, dtype=np.float32) for i, k in enumerate(sizes)]
            exp = xs if exp is None else [e + x for e, x in zip(exp, xs)]
        f_ok = all_ranks_ok(job.dist, all(np.array_equal(o, e) for o, e in zip(outs, exp)))
    line["host_to_host_fused"] = {
        "ms_per_step": round(tf * 1e3, 3), "algbw_gib_s": round(w.total_elems * 4 / tf / GIB, 2),
        "statistic": "median of %d calls, each timed alone" % fsteps,
        "ms_mean": round(sum(per) / len(per) * 1e3, 3), "ms_best": round(min(per) * 1e3, 3),
        "best_gib_s": round(w.total_elems * 4 / min(per) / GIB, 2),
        "steps": fsteps, "threads": int(os.environ.get("TIPS_HOST_THREADS", "8")),
        "piece_bytes": int(os.environ.get("TIPS_HOST_FUSED_PIECE_BYTES", str(32 << 20))),  # (host_staging.cc's default)
        "vs_per_tensor": round(th / tf, 2) if th else None,
        "check": ("identity at one rank, bit-exact" if world == 1 else "bit-exact vs rank-order fold of all ranks' inputs")
        if f_ok else "FAIL",
        "note": "the same 214 numpy gradients through allreduce_grads' N > 1 body (tips_fused_allreduce_host_flat): "
                "one call, outputs views of a page-locked flat buffer, pageable inputs; at one rank the round trip "
                "through HBM is kept"}
    del hg, outs


def op_host_leg(steps=20, warmup=3):
    """Config 5 as the reference's TF op sees it, at one rank: tools/_bin/op_host (a plain-C host on
    the product library alone) issues the 214 gradients as named HOST requests,
    tips_enqueue_allreduce_cb (request + callback), from four executor threads per step, as TF's
    executor runs MPIAllreduce's ComputeAsync (ops.cc:86-118, coordinator.cc:223-241). A child
    process (its own tips_init at one rank); median step of `steps`."""
    import socket
    exe = os.path.join(REPO, "tools", "_bin", "op_host")
    if not os.path.exists(exe):
        return {"error": "tools/_bin/op_host not built"}
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE",
                                                              "MASTER_PORT", "TIPS_BOOTSTRAP_PORT",
                                                              "TIPS_FUSION_MEASURE_PACK")}
    def child(n, w):
        s_ = socket.socket()
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
        s_.close()
        env.update(OP_HOST_STEPS=str(n), OP_HOST_WARMUP=str(w), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        r = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=120)
        return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    # The first op_host process on a box ran every step's host-to-device copy at 23 GiB/s against 36
    # in every later one (profiles/r05/z_op_host_first_process.txt), while the fused call it is
    # compared with runs in this process, long warm: one short untimed child first, its step kept.
    first = None
    try:
        first = child(3, 1).get("ms_per_step")
    except Exception:  # noqa: BLE001 - the measured run below decides
        pass
    try:
        d = child(steps, warmup)
    except Exception as e:  # noqa: BLE001 - a leg never costs the line
        return {"error": repr(e)}
    d.pop("rank", None)
    d["first_process_ms_per_step"] = first
    d["statistic"] = "median step of %d (each step: 214 enqueues from %d threads, then every callback)" % (
        steps, d.get("threads", 4))
    d["note"] = ("tools/op_host.c: 214 named host requests per step (pageable TF-style host tensors, outputs "
                 "reused), each one tips_enqueue_allreduce_cb (the request with its completion callback, as the "
                 "reference's OpRecord) from executor threads; the negotiation fuses each cycle's host requests "
                 "into one tips_fused_allreduce_host call")
    return d

# ----------------------------------------------------------------------------- the north star's ring (N > 1, mandatory)

def ring_depth_choice(job, w):
    """The ring's pipeline depth for config 3's bucket: the faster ring depth the tuner timed
    (tips_tuned_timings: the slowest rank's ms per call, the same on every rank), else the default."""
    import ctypes
    _lib, L = job._lib, job.L
    cap = 16
    al, de, la, ms = (ctypes.c_int * cap)(), (ctypes.c_int * cap)(), (ctypes.c_int * cap)(), (ctypes.c_double * cap)()
    n = L.tips_tuned_timings(w.qbytes, al, de, la, ms, cap)
    rings = sorted((ms[i], de[i]) for i in range(max(0, min(n, cap))) if al[i] == _lib.ALGO_RING and la[i] == 1)
    timed = [{"algorithm": job.inv.get(al[i], str(al[i])), "pipeline_depth": de[i], "lanes": la[i],
              "ms_per_call": round(ms[i], 3)} for i in range(max(0, min(n, cap)))]
    if rings:
        return rings[0][1], "the faster ring depth the tuner measured on this job", timed
    depth, sub = ctypes.c_int(), ctypes.c_int64()
    _lib.call("tips_schedule_shape", w.sizes[0], job.world, _lib.FLOAT32, ctypes.byref(depth), ctypes.byref(sub))
    return depth.value, "the default depth (TIPS_PIPELINE_DEPTH / TIPS_MIN_SUBCHUNK_BYTES; no tuner timings)", timed


def schedule_record(job, w, algo, env, steps):
    """Config 3's bucket (the headline's buffers) through one explicitly selected schedule: warm-up,
    `steps` timed calls (max over ranks), the parity check; the record's rate as the headline's."""
    _lib = job._lib
    saved = {k: os.environ.get(k) for k in env}
    try:
        os.environ.update(env)
        _lib.call("tips_set_algorithm", algo)
        for _ in range(2):
            w.step()
        job.torch.cuda.synchronize()
        t = w.timed(steps)
        good, msg = w.parity(algo)
        ok = all_ranks_ok(job.dist, good)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        _lib.call("tips_set_algorithm", w.algo if w.fallbacks else job.algo_names[job.args.algo])
    ms = t / steps * 1e3
    world = job.world
    algbw = w.total_elems * 4 / (ms / 1e3)
    busbw = algbw * 2 * (world - 1) / world
    return {"value": round(world * w.total_elems * 4 / (ms / 1e3) / GIB, 2), "unit": "GiB/s", "steps": steps,
            "ms_per_step": round(ms, 4), "algbw_gib_s": round(algbw / GIB, 2), "busbw_GBps": round(busbw / 1e9, 2),
            "check": msg if ok else "FAIL on some rank (%s here)" % msg}, ok


def north_star_ring(job, w, line):
    """The north star's multi-GPU target, measured right after the headline whatever schedule the
    tuner kept: config 3's 1 GiB bucket through the ring at its best measured depth (busbw against
    one xGMI link, target 0.70; the reference's data call is utils.h:60-65), and RCCL's own
    ncclAllReduce on the same bucket as a reference point. Not budgeted: every N > 1 line has both."""
    _lib = job._lib
    # 10 timed calls (the headline's steps if fewer), down to 3 when a call takes seconds (the
    # socket rehearsal): on xGMI a config-3 call is milliseconds and this costs well under a second
    kc = max(3, min(w.steps, 10, int(10.0 / max(w.ms / 1e3, 1e-3))))
    subs = line.setdefault("configs", {})
    progress(job.rank, "config3_ring")
    try:
        depth, why, timed = ring_depth_choice(job, w)
        env = {"TIPS_PIPELINE_DEPTH": str(depth), "TIPS_MIN_SUBCHUNK_BYTES": str(256)}
        rec, ok = schedule_record(job, w, _lib.ALGO_RING, env, kc)
        rb = rec["busbw_GBps"]
        rec.update({"algorithm": "ring", "pipeline_depth": depth, "depth_selection": why,
                    "workload": "config 3: allreduce of one 1 GiB fp32 bucket per GPU, ring schedule (one xGMI link "
                                "per direction per rank)",
                    "roofline": {"bound": "xgmi", "achieved": rb, "peak": XGMI_LINK_GBPS, "unit": "GB/s",
                                 "frac": round(rb / XGMI_LINK_GBPS, 4), "frac_of_one_link": round(rb / XGMI_LINK_GBPS, 4),
                                 "target_frac": 0.70, "links_used": 1}})
        if timed:
            rec["tuner_timings"] = timed
        subs["config3_ring"] = rec
        line["ring_xgmi"] = {"busbw_GBps": rb, "link_peak_GBps": XGMI_LINK_GBPS,
                             "frac_of_one_link": round(rb / XGMI_LINK_GBPS, 4), "target_frac": 0.70,
                             "pipeline_depth": depth, "check": rec["check"], "source": "configs.config3_ring"}
        line["sub_records_ok"] = line.get("sub_records_ok", True) and ok
    except Exception as e:  # noqa: BLE001 - reported, never costs the headline
        subs["config3_ring"] = {"error": "%s: %s" % (type(e).__name__, e)}
        line["sub_records_ok"] = False
    if os.environ.get("TIPS_NO_RCCL"):
        return
    progress(job.rank, "config3_rccl")
    try:
        rec, ok = schedule_record(job, w, _lib.ALGO_RCCL, {}, kc)
        rec.update({"algorithm": "ncclAllReduce (RCCL's own collective)",
                    "workload": "config 3's bucket through ncclAllReduce: the reference point for the schedules"})
        subs["config3_rccl"] = rec
        line["sub_records_ok"] = line.get("sub_records_ok", True) and ok
    except Exception as e:  # noqa: BLE001
        subs["config3_rccl"] = {"error": "%s: %s" % (type(e).__name__, e)}
        line["sub_records_ok"] = False


# ----------------------------------------------------------------------------- comparisons (after the sub-records)

def comparisons(job, w, line, last_words):
    """The headline bucket on the other schedules, RCCL's own allreduce and the probes, each only
    while the budget lasts (a skipped one is named in line["budget_skipped"]). A hang here is caught
    by the watchdog, which then still prints the line; a crash by last_words."""
    _lib, algo_names = job._lib, job.algo_names
    compare, compare_check = {}, {}

    def note_progress(what):
        """What rank 0 prints if a fatal signal ends the process during `what`."""
        progress(job.rank, what)
        if last_words:
            last_words(json.dumps(dict(line, compare_algbw_gib_s=compare, compare_check=compare_check,
                                       compare_error="process ended by a signal during %s" % what)))

    def _one_call_s():
        job.torch.cuda.synchronize()
        t0 = time.perf_counter()
        w.step()
        job.torch.cuda.synchronize()
        return time.perf_counter() - t0

    def run_variants(variants):
        kc = max(3, w.steps // 4)
        for label, name, env in variants:
            if (label == name and algo_names[name] == w.algo) or (name == "peer" and w.workload != "bucket") or \
                    (env and w.workload != "bucket"):
                continue
            # a variant costs about kc + 4 headline steps (slower schedules more): ask for 3x that
            if not job.afford("comparison %s" % label, 15 + 3 * (kc + 4) * w.ms / 1e3):
                continue
            note_progress("comparison %r" % label)
            saved = {k: os.environ.get(k) for k in env}
            try:
                os.environ.update(env)
                _lib.call("tips_set_algorithm", algo_names[name])
                for _ in range(2):
                    w.step()
                job.torch.cuda.synchronize()
                # a variant far slower than the main line (the socket rehearsal saw 100x for the
                # transfer lanes) is priced from one call, so it cannot eat the budget; every rank
                # takes the same branch (the slowest rank's time decides)
                t1 = max_over_ranks(job.dist, _one_call_s())
                if t1 > 20 * max(w.ms, 1e-3) / 1e3:
                    compare[label] = round(w.total_elems * 4 / t1 / GIB, 2)
                    compare_check[label] = "priced from one call (%.1f ms, > 20 x the main line); no parity run" % (t1 * 1e3)
                    continue
                tc = w.timed(kc)
                compare[label] = round(w.total_elems * 4 / (tc / kc) / GIB, 2)
                good, msg = w.parity(algo_names[name])
                compare_check[label] = msg if all_ranks_ok(job.dist, good) else "FAIL on some rank (%s here)" % msg
            except Exception as e:  # noqa: BLE001 - a comparison point never costs the main line
                compare[label] = None
                compare_check[label] = "error: %s" % (e,)
            finally:
                for k, v in saved.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
        _lib.call("tips_set_algorithm", w.algo if w.fallbacks else algo_names[job.args.algo])

    # (oneshot targets small buckets only.) The _k entries re-run a schedule at another sub-chunk
    # pipeline depth (read per call). Order: RCCL's allreduce and the other schedules, the link probe,
    # the probes; then the opt-in legs (IPC peer schedules, transfer lanes).
    # First, the peer schedules as child jobs (the MI355X-native exchange: our kernels over IPC-mapped
    # peer memory; TIPS_BENCH_PEER_CHILD=0 turns them off; TIPS_BENCH_PEER=1 runs them in this
    # process instead, below): a child that hangs or faults costs only its own entry.
    if job.world > 1 and w.workload == "bucket" and os.environ.get("TIPS_BENCH_PEER") != "1" and \
            os.environ.get("TIPS_BENCH_PEER_CHILD", "1") != "0" and not job.args.no_env_variants and \
            job.afford("the peer-schedule child jobs", 120):
        note_progress("the peer-schedule child jobs")
        kids = child_bucket_jobs(job.args, job.dist, job.rank, job.world, PEER_CHILDREN,
                                 timeout_s=int(os.environ.get("TIPS_BENCH_PEER_CHILD_TIMEOUT_S", "150")))
        line["peer_children"] = kids
        for name, r in kids.items():
            compare[name] = r.get("algbw_gib_s") if not r.get("error") else None
            compare_check[name] = r.get("check") or ("error: %s" % r.get("error"))
    # (ring at its best depth and ncclAllReduce are the mandatory configs.config3_ring / _rccl records)
    run_variants([("direct", "direct", {}),
                  ("direct_k1", "direct", {"TIPS_PIPELINE_DEPTH": "1"}),
                  ("direct_k8", "direct", {"TIPS_PIPELINE_DEPTH": "8", "TIPS_MIN_SUBCHUNK_BYTES": str(2 << 20)}),
                  ("ring_k8", "ring", {"TIPS_PIPELINE_DEPTH": "8", "TIPS_MIN_SUBCHUNK_BYTES": str(2 << 20)}),
                  # the same plan captured once and replayed as a HIP graph (TIPS_GRAPHS)
                  ("direct_graphs", "direct", {"TIPS_GRAPHS": "1", "TIPS_GRAPH_MAX_BYTES": str(1 << 40)})])
    if job.world > 1 and not os.environ.get("TIPS_NO_RCCL") and job.afford("the xGMI link probe", 30):
        note_progress("the xGMI link probe")
        try:
            line["xgmi_probe"] = link_probe(job.dist, job.rank, job.world)
        except Exception as e:  # noqa: BLE001
            line["xgmi_probe"] = {"error": str(e)}
    if job.world > 1 and job.afford("the backward-overlap probe", 45):
        note_progress("the backward-overlap probe")
        try:
            line["backward_overlap"] = overlap_probe(job.torch, job.dist, job.tips_amd, _lib, algo_names[job.args.algo], job)
        except Exception as e:  # noqa: BLE001
            line["backward_overlap"] = {"error": str(e)}
    if job.world > 1 and job.afford("the small-bucket latency probe", 40):
        note_progress("the small-bucket latency probe")
        try:
            line["small_bucket_latency"] = small_bucket_latency(job, job.torch, job.dist, _lib, job.L, job.rank, job.sp)
        except Exception as e:  # noqa: BLE001
            line["small_bucket_latency"] = {"error": str(e)}
    # Opt-in (TIPS_BENCH_PEER=1): the IPC peer schedules have not crossed real GPUs yet, so the
    # driver's scaling runs do not start them (a fault there would cost the whole record).
    if os.environ.get("TIPS_BENCH_PEER") == "1":
        run_variants([("peer", "peer", {}), ("peer_push", "peer", {"TIPS_PEER_AG": "push"}),
                      # the fused pull-fold reduce-scatter: one kernel per rank reads its chunk's slices
                      # from every peer's workspace over xGMI and folds them (peer.cc peer_piece_pullfold)
                      ("peer_pullfold", "peer", {"TIPS_PEER_RS": "pullfold"})])
    elif job.world > 1 and "peer" not in compare_check:
        compare_check["peer"] = "not run (peer_children: TIPS_BENCH_PEER_CHILD=0, --no-env-variants or the budget)"
    # Opt-in (TIPS_BENCH_LANES=1): transfer lanes split communicators that live to the end of
    # the job; on the socket rehearsal they ran 10x slower and slowed every later call.
    if os.environ.get("TIPS_BENCH_LANES") == "1":
        run_variants([("direct_l2", "direct", {"TIPS_LANES": "2"}),
                      ("ring_l2", "ring", {"TIPS_LANES": "2"}),
                      ("direct_k8_l4", "direct", {"TIPS_LANES": "4", "TIPS_PIPELINE_DEPTH": "8",
                                                  "TIPS_MIN_SUBCHUNK_BYTES": str(2 << 20)})])
    elif job.world > 1:
        compare_check["lanes"] = "opt-in: TIPS_BENCH_LANES=1"
    line["compare_check"] = compare_check
    line["compare_algbw_gib_s"] = compare
    # Child jobs with other RCCL settings: 4 point-to-point channels per peer (8 delivered wrong bytes
    # over the socket transport, profiles/r02/rccl_nchannels_probe.txt). Each child also measures the
    # north star's ring (config3_ring) under its setting: with RCCL's default channels per peer one
    # ring link may stay under 70 % of its bandwidth. On by default where a config-3 ring call is
    # fast (the xGMI node; the socket rehearsal's take seconds), within the budget;
    # TIPS_BENCH_ENV_VARIANTS=1 forces it, 0 turns it off.
    ev = os.environ.get("TIPS_BENCH_ENV_VARIANTS", "")
    ring_ms = ((line.get("configs") or {}).get("config3_ring") or {}).get("ms_per_step")
    if job.world > 1 and not job.args.no_env_variants and not os.environ.get("TIPS_NO_RCCL") and ev != "0" and \
            (ev == "1" or (ring_ms is not None and ring_ms < 500)) and job.afford("the RCCL-setting child jobs", 150):
        note_progress("the RCCL-setting child jobs")
        line["env_variants"] = env_variant_jobs(job.args, job.dist, job.rank, job.world)


# ----------------------------------------------------------------------------- the run

def sub_records(job, line, steps):
    """The other configs at this N, each a record of its own in line["configs"]."""
    subs = line.setdefault("configs", {})
    # config 4 as 1000 NAMED requests last (the negotiated path: readiness batches fused, the
    # response cache after the first step), only while the budget lasts
    order = ([("config3_bucket", "bucket")] if job.world == 1 else []) + \
        [("config4_fused1000", "fused1000"), ("config5_resnet50", "resnet50"), ("config4_negotiated", "negotiated1000")]
    for key, wl in order:
        # a record costs its tuning + warm-up + steps: at N = 8 over the socket rehearsal ~20 s each
        if not job.afford(key, 30):
            subs[key] = {"skipped": "time budget (TIPS_BENCH_BUDGET_S)"}
            continue
        progress(job.rank, "sub-record %s" % key)
        w = Workload(job, wl, min(steps, 10) if wl == "negotiated1000" else steps, 5 if wl != "bucket" else 3)
        try:
            rec = w.run()
            if wl in SUB_WORKLOADS and job.afford("%s gradient_api legs" % key, 25):
                rec["gradient_api"] = gradient_api_legs(job.torch, job.dist, job.tips_amd, job.world, w.sizes, w.offs,
                                                        w.rot_sets, min(steps, 10), w.ms)
                if "fp16_compressed" in rec["gradient_api"]:  # (beside the fp32 step)
                    rec["fp16_compressed"] = dict(rec["gradient_api"]["fp16_compressed"],
                                                  fp32_allreduce_grads_ms=rec["gradient_api"]["allreduce_grads"]["ms_per_step"])
            if wl == "resnet50" and job.afford("config5 host legs", 40):
                host_legs(job, w, rec)
                if job.world == 1:
                    rec["op_host_named"] = op_host_leg()
                    fused = rec.get("host_to_host_fused", {}).get("algbw_gib_s")
                    if fused and rec["op_host_named"].get("algbw_gib_s"):
                        rec["op_host_named"]["vs_host_to_host_fused"] = round(
                            rec["op_host_named"]["algbw_gib_s"] / fused, 3)
            subs[key] = rec
            line["sub_records_ok"] = line.get("sub_records_ok", True) and w.ok
        except Exception as e:  # noqa: BLE001 - a sub-record never costs the headline
            subs[key] = {"error": "%s: %s" % (type(e).__name__, e)}
            line["sub_records_ok"] = False
        finally:
            w.close()
    return subs


def bench_job(args):
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if os.environ.get("TIPS_BENCH_FAKE_HOSTS") == "1":
        # rehearsal of the N > 1 code path on a one-GPU box: every rank names its own RCCL host, so
        # RCCL accepts several ranks on one device and joins them over its socket transport
        # (tests/test_gpu_rccl_procs.py). The rates are then loopback-socket rates, not xGMI.
        os.environ["NCCL_HOSTID"] = "tips-bench-rank-%d" % rank
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    wd = start_watchdog(int(os.environ.get("TIPS_BENCH_WATCHDOG", "420")), rank)
    workload = args.workload if args.workload != "auto" else ("sum" if world == 1 else "bucket")
    headline_sum = workload == "sum"
    # CPU baselines first, on rank 0, before this process touches the GPU (they start child processes)
    topo = gpu_topology() if rank == 0 and world > 1 else None
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        if headline_sum:
            cpu = cpu_baseline((args.bucket_mib or 256) * (1 << 20) // 4)
        elif workload == "bucket":
            cpu = cpu_ring_baseline(world) if world > 1 else None
    sum_ok = True
    if headline_sum:
        line, sum_ok = sum_record(args, cpu)
        progress(rank, "config 2: %.2f GiB/s (%.4f of HBM)" % (line["value"], line["roofline"]["frac"]))
        if args.no_extras or args.no_sub:
            print(json.dumps(line), flush=True)
            wd.cancel()
            return 0 if sum_ok else 1
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))  # (several ranks per GPU only under TIPS_NO_RCCL)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import tips_amd
    from tips_amd import _lib
    tips_amd.init()  # unique id through the gloo group, one RCCL communicator per GPU
    progress(rank, "initialised: %d ranks" % world)
    job = Job(args, torch, dist, tips_amd, _lib)
    _lib.call("tips_set_algorithm", job.algo_names[args.algo])
    w = None
    all_ok = sum_ok
    if not headline_sum:
        steps = args.steps if args.steps is not None else 20
        warmup = args.warmup if args.warmup is not None else 5
        w = Workload(job, workload, steps, warmup)
        rec = w.run()
        all_ok = w.ok
        line = {"metric": METRIC, "value": rec.pop("value"), "unit": rec.pop("unit"), "n_gpus": world, "steps": steps,
                "warmup": warmup, "ms_per_step": rec.pop("ms_per_step"), "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None, "dtype": "f32", "data": rec.pop("data"),
                "config": {"workload": rec.pop("workload"), "tensors": rec.pop("tensors"),
                           "bytes_per_rank": rec.pop("bytes_per_rank"), "algorithm": rec.pop("algorithm"),
                           "selection": rec.pop("selection"), "rotating_sets": rec.pop("rotating_sets"),
                           "parallelism": "dp%d (one process per GPU, %s)" % (
                               world, "our kernels through IPC-mapped peer memory over xGMI" if w.algo == _lib.ALGO_PEER
                               else "ncclAllReduce" if w.algo == _lib.ALGO_RCCL else "RCCL p2p over xGMI")
                           if world > 1 else "single GPU: no link carries anything (the allreduce of one rank is the identity)"},
                "cpu_baseline": cpu}
        line.update(rec)
        kr = w.reduce_kernel_roofline()
        if kr:
            line["reduce_kernel_roofline"] = kr
        if workload in SUB_WORKLOADS:
            line["gradient_api"] = gradient_api_legs(torch, dist, tips_amd, world, w.sizes, w.offs, w.rot_sets, steps, w.ms)
            if workload == "resnet50":
                host_legs(job, w, line)
                if world == 1:
                    line["op_host_named"] = op_host_leg()
        if topo:
            line["gpu_topology"] = topo
    _RESULT["line"] = line if rank == 0 else None
    _RESULT["done"] = True
    # (mandatory on every N > 1 line; a peer-schedule child job skips it: its parent line has it)
    if w is not None and workload == "bucket" and world > 1 and os.environ.get("TIPS_BENCH_CHILD_NO_RING") != "1":
        north_star_ring(job, w, line)  # mandatory, before every sub-record and budgeted leg
        _RESULT["line"] = line if rank == 0 else None
    if args.workload == "auto" and not args.no_sub:
        sub_records(job, line, args.sub_steps)
        anchor = (line.get("configs") or {}).get("config3_bucket") or {}
        if world == 1 and anchor.get("value") is not None:
            # the metric names two workloads (config 2's sum at N = 1, config 3's allreduce at N > 1):
            # the same-workload point for a scaling curve is config 3 at one rank
            line["scaling_anchor"] = {"workload": "config 3 at one rank (configs.config3_bucket)",
                                      "value": anchor["value"], "unit": anchor.get("unit"),
                                      "ms_per_step": anchor.get("ms_per_step"),
                                      "note": "value(N) / (N x this) compares like with like; the N = 1 "
                                              "headline is config 2's sum kernel, a different workload"}
        _RESULT["line"] = line if rank == 0 else None
    last_words = crash_line() if rank == 0 and not args.no_compare else None
    if w is not None and workload == "bucket" and world > 1 and not args.no_compare:
        comparisons(job, w, line, last_words)
    if job.skipped:
        line["budget_skipped"] = {"legs": job.skipped, "budget_s": job.budget_s,
                                  "note": "TIPS_BENCH_BUDGET_S: optional legs start only while the budget lasts"}
    line["wall_s"] = round(time.time() - _T0, 1)
    if rank == 0:
        if last_words:
            last_words(None)
        print(json.dumps(line), flush=True)
    _RESULT["printed"] = True  # the watchdog must not print a second line
    if w is not None:
        w.close()
    dist.barrier()
    wd.cancel()
    tips_amd.shutdown()
    dist.destroy_process_group()
    return 0 if all_ok else 1


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world == 1:
        # launched without torchrun: start it as a child (never exec from a process that touched the GPU)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
               "--master-addr", "127.0.0.1", "--master-port", os.environ.get("MASTER_PORT", "29511"),
               os.path.abspath(__file__)] + sys.argv[1:]
        return subprocess.call(cmd)
    if world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29512")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    try:
        return bench_job(args)
    except Exception as e:  # one diagnosable line instead of a bare traceback
        if int(os.environ.get("RANK", "0")) == 0 and not _RESULT.get("printed"):
            line = _RESULT.get("line") or {"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": world}
            print(json.dumps(dict(line, error="%s: %s" % (type(e).__name__, e))), flush=True)
        raise


if __name__ == "__main__":
    sys.exit(main())
