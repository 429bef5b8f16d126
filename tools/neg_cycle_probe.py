"""The negotiation's per-cycle cost at N ranks on the CPU (no GPU): N processes run
tips_negotiation_selftest (dry-run executor) over 127.0.0.1, each enqueueing config 5's 214 names
per step (PROBE_NAMES to change it) from T executor threads (callbacks), STEPS steps; TIPS_NEG_TRACE=1 prints each cycle's
linger / exchange / execute. Prints the per-rank median of every part over the steady cycles.

  python3 tools/neg_cycle_probe.py [N=8] [STEPS=12] [THREADS=4]
"""
import multiprocessing as mp
import os
import re
import socket
import statistics
import sys
import tempfile

NAMES = int(os.environ.get("PROBE_NAMES", "214"))


def _rank(rank, size, port, script, errpath, env):
    import ctypes
    os.environ.update(env)
    fd = os.open(errpath, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    os.dup2(fd, 2)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from tips_amd import _lib
    L = _lib.dev()
    out = ctypes.create_string_buffer(1 << 20)
    rc = L.tips_negotiation_selftest(rank, size, b"127.0.0.1", port, script.encode(), out, len(out))
    if rc:
        print("rank %d: rc %d %s" % (rank, rc, L.tips_last_error().decode()), file=sys.stderr, flush=True)


def script(steps, threads):
    lines = []
    for s in range(steps):
        for t in range(threads):
            for i in range(t, NAMES, threads):
                lines.append("t%d: grad_%03d 0 %d" % (t + 1, i, 1000 + i))
            lines.append("t%d: @wait" % (t + 1))
    return "\n".join(lines)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    threads = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    d = tempfile.mkdtemp()
    env = {"TIPS_NEG_TRACE": "1"}
    env.update({k: v for k, v in os.environ.items() if k.startswith("TIPS_")})
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_rank, args=(r, n, port, script(steps, threads), os.path.join(d, "r%d.err" % r), env))
          for r in range(n)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    pat = re.compile(r"announced (\d+), decided (\d+); linger (\d+) us .*?ended (\d+) us after .*?exchange (\d+) us .*?"
                     r"execute (\d+) us")
    for r in range(n):
        rows = [tuple(map(int, m.groups())) for m in pat.finditer(open(os.path.join(d, "r%d.err" % r)).read())]
        steady = [x for x in rows[2:] if x[0] >= NAMES // 2] or rows
        med = lambda k: statistics.median(x[k] for x in steady) if steady else None  # noqa: E731
        print("rank %d: %d cycles (%d steady); median announced %s decided %s linger %s us tail %s us exchange %s us"
              % (r, len(rows), len(steady), med(0), med(1), med(2), med(3), med(4)))
        txt = open(os.path.join(d, "r%d.err" % r)).read()
        adm = [int(x) for x in re.findall(r"admissions (\d+) us", txt)][2:]
        dec = [int(x) for x in re.findall(r"rank 0's decision (\d+) us", txt)][2:]
        if adm:
            print("rank %d: admissions per cycle, median %s us" % (r, statistics.median(adm)))
        if r == 0 and dec:
            print("rank 0: decision per cycle, median %s us, total %s us over %d cycles"
                  % (statistics.median(dec), sum(dec), len(dec)))


if __name__ == "__main__":
    main()
