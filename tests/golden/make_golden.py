#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ (run in the build container).

Inputs are seeded numpy draws; expected outputs come from the reference's
exact data-path call, MPI_Allreduce(in, out, N, T, MPI_SUM, MPI_COMM_WORLD)
(tips/core/collective/utils.h:60-65), executed by oracle/build/mpi_allreduce_ref
under the image's MPICH 3.3.2 with one process per rank (`mpirun -np p`).
The reference's own TF op cannot be built here (no TensorFlow / abseil /
flatbuffers: SURVEY §8c), so this call is the pinned behaviour.

Cases:
  kat_utils_test        p=5, 2x2 f32, x_r[i] = i*0.1*r      (utils_test.cc:12-37)
  kat_coordinator_test  p=3, 2x4 f32, x[i]   = i*0.1        (coordinator_test.cc:10-45)
  kat_mpi_allreduce     p=3, n=10 f32, x[i]  = i*0.1        (mpi_allreduce_test.cc:8-33)
  rand_{dt}_p{p}        p in {2,4,8}, dt in {f32,f64,i32,i64}, n=4099 (odd tail);
                        floats U[0.5,1.5) (positive: order-independent rel bound),
                        ints full-range (exercise wrap-around)
  signed_f32_p4         p=4, n=4099, U[-1,1) (norm-wise bound)
  cfg1_f32_p2_1MiB      p=2, 262144 f32 U[0.5,1.5), seed 1000+r (BASELINE config 1);
                        inputs regenerated from the seeds, only the output is stored

Usage: python tests/golden/make_golden.py   (needs `make -C oracle` and /opt/conda MPICH)
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(REPO, "oracle", "build", "mpi_allreduce_ref")
MPIRUN = os.environ.get("MPIRUN", "/opt/conda/bin/mpirun")

DT = {"f32": (0, np.float32), "f64": (1, np.float64), "i32": (2, np.int32), "i64": (3, np.int64)}


def kat_inputs(kind):
    if kind == "kat_utils_test":
        p, n = 5, 4
        # static_cast<float*>(...)[i] = i * 0.1 * mpi_rank();  (double product, stored as float)
        return p, np.stack([np.array([i * 0.1 * r for i in range(n)], dtype=np.float64).astype(np.float32)
                            for r in range(p)])
    if kind == "kat_coordinator_test":
        p, n = 3, 8
        return p, np.stack([np.array([i * 0.1 for i in range(n)], dtype=np.float64).astype(np.float32)] * p)
    if kind == "kat_mpi_allreduce":
        p, n = 3, 10
        # rands.push_back(i * 0.1) into a std::vector<float>
        return p, np.stack([np.array([i * 0.1 for i in range(n)], dtype=np.float64).astype(np.float32)] * p)
    raise KeyError(kind)


def rand_inputs(dt, p, n, seed, signed=False):
    _, npdt = DT[dt]
    rows = []
    for r in range(p):
        g = np.random.default_rng(seed + r)
        if npdt in (np.float32, np.float64):
            x = g.random(n) * 2.0 - 1.0 if signed else 0.5 + g.random(n)
            rows.append(x.astype(npdt))
        else:
            info = np.iinfo(npdt)
            rows.append(g.integers(info.min, info.max, size=n, dtype=npdt, endpoint=True))
    return np.stack(rows)


def cfg1_inputs():
    return np.stack([(0.5 + np.random.default_rng(1000 + r).random(262144)).astype(np.float32) for r in range(2)])


def run_mpi(dtcode, ins):
    p, n = ins.shape
    with tempfile.TemporaryDirectory() as d:
        for r in range(p):
            ins[r].tofile(os.path.join(d, "in_%d.bin" % r))
        cmd = [MPIRUN, "-np", str(p), HARNESS, "golden", str(dtcode), str(n), d]
        subprocess.run(cmd, check=True, timeout=300)
        outs = np.stack([np.fromfile(os.path.join(d, "out_%d.bin" % r), dtype=ins.dtype) for r in range(p)])
    return outs


def sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        h.update(f.read())
    return h.hexdigest()


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the harness first: make -C oracle")
    mpich = subprocess.run(["/opt/conda/bin/mpichversion"], capture_output=True, text=True).stdout.split("\n")[0]
    manifest = {"generator": "tests/golden/make_golden.py", "mpi": mpich.strip(), "cases": {}}
    cases = []
    for k in ("kat_utils_test", "kat_coordinator_test", "kat_mpi_allreduce"):
        p, ins = kat_inputs(k)
        cases.append((k, "f32", ins, {"source": "reference KAT"}))
    for dt in ("f32", "f64", "i32", "i64"):
        for p in (2, 4, 8):
            seed = 7000 + 100 * p + DT[dt][0] * 10
            cases.append(("rand_%s_p%d" % (dt, p), dt, rand_inputs(dt, p, 4099, seed), {"seed": seed, "n": 4099}))
    cases.append(("signed_f32_p4", "f32", rand_inputs("f32", 4, 4099, 9000, signed=True), {"seed": 9000, "n": 4099}))
    for name, dt, ins, meta in cases:
        outs = run_mpi(DT[dt][0], ins)
        all_equal = bool(all(np.array_equal(outs[0].view(np.uint8), o.view(np.uint8)) for o in outs))
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, inputs=ins, expected=outs[0])
        manifest["cases"][name] = dict(meta, dtype=dt, p=int(ins.shape[0]), n=int(ins.shape[1]),
                                       ranks_bitwise_equal=all_equal, sha256=sha(path))
        print(name, ins.shape, "ok", "ranks_equal=%s" % all_equal)
    ins = cfg1_inputs()
    outs = run_mpi(0, ins)
    path = os.path.join(HERE, "cfg1_f32_p2_1MiB.npz")
    np.savez_compressed(path, expected=outs[0])
    manifest["cases"]["cfg1_f32_p2_1MiB"] = {
        "dtype": "f32", "p": 2, "n": 262144, "seeds": [1000, 1001],
        "inputs": "np.random.default_rng(1000 + r).random(262144) + 0.5 -> float32 (regenerated by the test)",
        "inputs_sha256": hashlib.sha256(ins.tobytes()).hexdigest(),
        "ranks_bitwise_equal": bool(np.array_equal(outs[0], outs[1])), "sha256": sha(path)}
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", len(manifest["cases"]), "cases")


if __name__ == "__main__":
    main()
