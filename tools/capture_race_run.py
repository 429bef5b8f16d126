"""Run a C-host rank binary (tools/_bin/capture_race, op_body, ...) as p RCCL ranks on one GPU
and report every rank's JSON line and the tail of its stderr. Exit 0 only if every rank exited 0.

  python tools/capture_race_run.py BINARY P [VAR=VALUE ...]

The ranks are set up as tests/test_gpu_op_body.py sets them up (NCCL_HOSTID per process, socket
transport over lo). Used by tools/capture_race_exp.sh to run the capture experiments of DESIGN §4
one at a time."""
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    binary, p = sys.argv[1], int(sys.argv[2])
    extra = dict(a.split("=", 1) for a in sys.argv[3:])
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    exe = os.path.join(REPO, "tools", "_bin", binary)
    procs = []
    for r in range(p):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(p), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), TIPS_BOOTSTRAP_PORT=str(port), NCCL_HOSTID="tips-race-%d" % r,
                   NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1", **extra)
        procs.append(subprocess.Popen([exe], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    ok = True
    t0 = time.time()
    for r, pr in enumerate(procs):
        while True:  # (a line on stderr every 20 s: a hung rank is killed at 150 s, before gpurun's silence limit)
            try:
                out, err = pr.communicate(timeout=20)
                break
            except subprocess.TimeoutExpired:
                print("[capture_race_run] %s: waiting for rank %d, %.0f s" % (binary, r, time.time() - t0),
                      file=sys.stderr, flush=True)
                if time.time() - t0 > 150:
                    for q in procs:
                        if q.poll() is None:
                            q.kill()
        line = [l for l in out.splitlines() if l.startswith("{")]
        res = json.loads(line[-1]) if line else None
        good = pr.returncode == 0 and res is not None and res.get("ok")
        ok = ok and bool(good)
        print(json.dumps({"binary": binary, "p": p, "env": extra, "rank": r, "rc": pr.returncode, "result": res,
                          "stderr_tail": "" if good else err[-4000:]}), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
