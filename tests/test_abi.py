"""The C-ABI boundary without a GPU: the library loads, exports every symbol
include/tips_hip.h declares and nothing else, the Python binding declares each of them, the
development library (include/tips_hip_dev.h) exports the product symbols plus its own, and the
argument / lifecycle error paths behave (no compute calls here)."""
import ctypes
import multiprocessing as mp
import os
import re
import socket

import numpy as np
import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "tips_hip.h")
DEV_HEADER = os.path.join(REPO, "include", "tips_hip_dev.h")


def header_functions(path=HEADER):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tips_\w+)\s*\(", src)))


def test_header_parses():
    names = header_functions()
    # the reference's lifecycle names (tips/core/operations.h:7-21) are all kept
    for ref in ("tips_init", "tips_shutdown", "tips_is_initialize", "tips_size", "tips_rank"):
        assert ref in names
    assert "tips_allreduce" in names and "tips_bucket_sum" in names


def test_library_exports_every_header_symbol():
    from tips_amd import _lib
    L = _lib.lib()
    missing = [n for n in header_functions() if not hasattr(L, n)]
    assert not missing, missing


def test_python_binding_declares_every_symbol():
    from tips_amd import _lib
    declared = {n for n, _, _ in _lib._SIGNATURES}
    assert set(header_functions()) == declared
    assert set(header_functions(DEV_HEADER)) == {n for n, _, _ in _lib._DEV_SIGNATURES}


def _exported(path):
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


def test_product_and_development_exports():
    """The product library exports exactly include/tips_hip.h (the drop-in boundary: the reference's
    five lifecycle symbols of operations.h:7-21 plus the data path); the simulators, self-tests and
    tuning sweeps live in tools/lib/libtips_hip_dev.so only, which exports the product symbols too
    (one complete runtime) and loads beside the product library without touching it."""
    import shutil
    if not shutil.which("nm"):
        pytest.skip("no nm")
    prod = _exported(os.path.join(REPO, "tips_amd", "lib", "libtips_hip.so"))
    dev = _exported(os.path.join(REPO, "tools", "lib", "libtips_hip_dev.so"))
    dev_only = set(header_functions(DEV_HEADER))
    assert prod == set(header_functions())
    assert not prod & dev_only
    assert dev == prod | dev_only
    assert len(dev_only) == 14  # simulators (4), self-tests (3), sweeps (4), tips_schedule_plan, tile table,
    #                             tips_tune_candidates
    from tips_amd import _lib
    D, L = _lib.dev(), _lib.lib()
    assert D is not L and not hasattr_c(L, "tips_ring_simulate") and hasattr_c(D, "tips_ring_simulate")
    # separate runtimes: the development library's state is its own
    assert D.tips_size() == -1 and L.tips_set_algorithm(_lib.ALGO_RING) == 0 and D.tips_get_algorithm() != _lib.ALGO_RING
    L.tips_set_algorithm(_lib.ALGO_AUTO)


def hasattr_c(handle, name):
    try:
        getattr(handle, name)
        return True
    except AttributeError:
        return False


def test_lifecycle_before_init():
    from tips_amd import _lib
    L = _lib.lib()
    assert not L.tips_is_initialize()
    assert L.tips_size() == -1 and L.tips_rank() == -1
    assert L.tips_version().startswith(b"tips_hip")
    assert L.tips_unique_id_bytes() == 128
    L.tips_shutdown()  # no-op when not initialised


def test_error_codes():
    from tips_amd import _lib
    L = _lib.lib()
    assert L.tips_allreduce(None, None, 10, _lib.FLOAT32, _lib.OP_SUM, None) == -2  # not initialised
    assert b"tips_init" in L.tips_last_error()
    assert L.tips_allreduce(None, None, 10, 99, _lib.OP_SUM, None) == -1  # bad dtype
    assert L.tips_allreduce(None, None, 10, _lib.FLOAT32, _lib.OP_MAX, None) == -5  # only SUM
    assert L.tips_bucket_sum(None, None, None, -1, _lib.FLOAT32, None) == -1
    assert L.tips_bucket_sum(None, None, None, 0, _lib.FLOAT32, None) == 0  # empty is a no-op
    assert L.tips_multi_sum(None, None, 17, 10, _lib.FLOAT32, None) == -1
    assert L.tips_set_algorithm(7) == -1
    assert L.tips_fused_allreduce(None, None, 0, _lib.FLOAT32, None) == -2
    with pytest.raises(_lib.TipsError) as ei:
        _lib.call("tips_allreduce", None, None, 10, 99, 0, None)
    assert ei.value.code == -1


def test_algorithm_resolution():
    from tips_amd import _lib
    L = _lib.lib()
    prev = L.tips_get_algorithm()
    assert L.tips_set_algorithm(_lib.ALGO_AUTO) == 0 and L.tips_get_algorithm() == _lib.ALGO_AUTO
    big, small = 1 << 30, 64 << 10
    assert L.tips_resolve_algorithm(2, big) == _lib.ALGO_RING
    assert L.tips_resolve_algorithm(8, big) == _lib.ALGO_DIRECT
    assert L.tips_resolve_algorithm(8, small) == _lib.ALGO_ONESHOT
    assert L.tips_resolve_algorithm(2, small) == _lib.ALGO_ONESHOT
    assert L.tips_resolve_algorithm(32, small) == _lib.ALGO_RING  # more ranks than the fold takes sources
    # p = 2: a one-shot moves the ring's bytes in one step, so it takes buckets up to 8 MiB;
    # p > 2: it moves (p - 1) x the all-pairs bytes per link, so only up to 256 KiB
    assert L.tips_resolve_algorithm(2, 8 << 20) == _lib.ALGO_ONESHOT
    assert L.tips_resolve_algorithm(2, (8 << 20) + 4) == _lib.ALGO_RING
    assert L.tips_resolve_algorithm(4, 1 << 20) == _lib.ALGO_DIRECT
    assert L.tips_resolve_algorithm(4, 256 << 10) == _lib.ALGO_ONESHOT
    L.tips_set_algorithm(_lib.ALGO_RING)
    assert L.tips_resolve_algorithm(8, small) == _lib.ALGO_RING
    L.tips_set_algorithm(_lib.ALGO_TUNE)  # measured per size class; small buckets stay one-shots
    assert L.tips_resolve_algorithm(8, big) == _lib.ALGO_TUNE
    assert L.tips_resolve_algorithm(8, small) == _lib.ALGO_ONESHOT
    assert L.tips_set_algorithm(6) == -1
    L.tips_set_algorithm(prev)


@pytest.mark.parametrize("dtype,es", [(0, 4), (1, 8), (2, 4), (3, 8), (4, 2), (5, 2)])
def test_chunk_bounds_match_oracle(oracle, dtype, es):
    from tips_amd import _lib
    L = _lib.lib()
    b, e = ctypes.c_int64(), ctypes.c_int64()
    for n in (0, 1, 7, 4099, 262144, 67108864 + 5):
        for p in (1, 2, 3, 4, 8):
            for c in range(p):
                assert L.tips_chunk_bounds(n, p, dtype, c, ctypes.byref(b), ctypes.byref(e)) == 0
                assert (b.value, e.value) == oracle.chunk_bounds(n, p, 256 // es, c)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _bootstrap_worker(rank, size, port, q):
    from tips_amd import _lib
    L = _lib.lib()
    buf = ctypes.create_string_buffer(128)
    if rank == 0:
        ctypes.memmove(buf, bytes(range(128)), 128)
    rc = L.tips_bootstrap_broadcast(rank, size, b"127.0.0.1", port, buf, 128, 60)
    q.put((rank, rc, buf.raw))


@pytest.mark.parametrize("size", [2, 4])
def test_bootstrap_broadcast_multiprocess(size):
    """The TCP id exchange tips_init uses, across real processes on CPU."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bootstrap_worker, args=(r, size, port, q)) for r in range(size)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
    for rank, rc, raw in res:
        assert rc == 0, rank
        assert raw == bytes(range(128))


def test_bootstrap_survives_a_silent_listener():
    """Rank 1 first reaches another program's socket on the port, which accepts and never answers;
    its wait for the id is bounded (5 s), so it retries and gets the id from rank 0 once rank 0
    listens there, well inside its 60 s timeout."""
    import socket
    import threading
    import time
    port = _free_port()
    foreign = socket.socket()
    foreign.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    foreign.bind(("127.0.0.1", port))
    foreign.listen(4)
    held = []
    t = threading.Thread(target=lambda: held.append(foreign.accept()[0]))
    t.start()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    r1 = ctx.Process(target=_bootstrap_worker, args=(1, 2, port, q))
    r1.start()
    t.join(60)
    foreign.close()  # the accepted connection stays open and silent
    time.sleep(0.5)
    t0 = time.time()
    r0 = ctx.Process(target=_bootstrap_worker, args=(0, 2, port, q))
    r0.start()
    res = sorted(q.get(timeout=60) for _ in range(2))
    for p_ in (r0, r1):
        p_.join(30)
    for c in held:
        c.close()
    assert [rc for _, rc, _ in res] == [0, 0]
    assert all(raw == bytes(range(128)) for _, _, raw in res)
    assert time.time() - t0 < 30


def _bootstrap_worker_env(rank, size, port, q, env, delay):
    import os
    import time
    os.environ.update(env)
    time.sleep(delay)
    from tips_amd import _lib
    L = _lib.lib()
    buf = ctypes.create_string_buffer(128)
    if rank == 0:
        ctypes.memmove(buf, bytes(range(128)), 128)
    rc = L.tips_bootstrap_broadcast(rank, size, b"127.0.0.1", port, buf, 128, 60)
    a, b = ctypes.c_int64(), ctypes.c_int64()
    L.tips_net_stats(ctypes.byref(a), ctypes.byref(b))
    q.put((rank, rc, buf.raw, a.value, b.value))


@pytest.mark.parametrize("knob,who", [("TIPS_TEST_SELF_CONNECT", 3), ("TIPS_TEST_DROP_FIRST_HELLO", 4)])
def test_bootstrap_join_edge_cases(knob, who):
    """The unique-id bootstrap's two join hazards, made deterministic:
    - TIPS_TEST_SELF_CONNECT: rank 1 starts 1 s before rank 0 and its first attempts are bound to
      the port they connect to, so they complete as a TCP simultaneous open with itself; each must
      be dropped (tips_net_stats counts them) - read as an answer it would have been 'the id';
    - TIPS_TEST_DROP_FIRST_HELLO: rank 1 gives up on its first connection right after asking (as
      a rank whose answer timed out): rank 0 counts a rank only when it confirms receipt, so it
      keeps listening and serves the retry instead of closing the listener on a rank that left."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    env = {knob: "3" if knob == "TIPS_TEST_SELF_CONNECT" else "1"}
    procs = [ctx.Process(target=_bootstrap_worker_env, args=(r, 3, port, q, env if r == 1 else {},
                                                           1.0 if (r == 0 and knob == "TIPS_TEST_SELF_CONNECT") else 0.0))
             for r in range(3)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=90) for _ in procs)
    for p in procs:
        p.join(30)
    for rank, rc, raw, selfc, unconf in res:
        assert rc == 0, rank
        assert raw == bytes(range(128))
    if knob == "TIPS_TEST_SELF_CONNECT":
        assert res[1][3] >= 1, res
    else:
        assert res[0][4] >= 1, res


def test_bootstrap_timeout():
    from tips_amd import _lib
    L = _lib.lib()
    buf = ctypes.create_string_buffer(16)
    assert L.tips_bootstrap_broadcast(1, 2, b"127.0.0.1", _free_port(), buf, 16, 1) == -6
    assert b"could not reach" in L.tips_last_error()


def test_product_has_no_oracle_dependency():
    """The shipped path never imports, links or loads oracle/ (DESIGN.md §Oracle)."""
    for root, _, files in os.walk(os.path.join(REPO, "tips_amd")):
        for f in files:
            if f.endswith((".py", ".cc", ".hip", ".h")):
                text = open(os.path.join(root, f)).read()
                assert "oracle_bind" not in text and "liboracle" not in text and "import oracle" not in text, f


def test_single_hip_runtime():
    """Exactly one libamdhip64 / libhsa-runtime64 / librccl mapped after loading the library
    (torch bundles copies with the same sonames; tips_amd._lib loads torch first)."""
    import subprocess
    import sys
    code = ("import re\nfrom tips_amd import _lib\n_lib.lib()\nimport torch\n"
            "m=open('/proc/self/maps').read()\n"
            "for k in ('libamdhip64','libhsa-runtime64','librccl'):\n"
            "    print(k, len(set(re.findall(r'(/\\S*'+k+r'\\S*)', m))))\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=REPO, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    for line in r.stdout.strip().splitlines():
        name, count = line.split()
        assert count == "1", line


# ---------------------------------------------------------------- control plane (pure host)

def _table(*recs):
    from tips_amd import _lib
    flat = []
    for typ, dt, shape in recs:
        flat += [typ, dt, len(shape)] + list(shape) + [0] * (_lib.MAX_DIMS - len(shape))
    return _lib.i64_array(flat)


@pytest.mark.parametrize("recs,msg", [
    ([(0, 0, (2, 4)), (0, 0, (2, 4)), (0, 0, (2, 4))], None),
    ([(0, 0, (2, 4)), (0, 1, (2, 4))], b"Mismatch data types found: 0 vs 1."),
    ([(0, 0, (2, 4)), (2, 0, (2, 4))], b"Mismatched operations found: 0 vs 2."),
    ([(0, 0, (2, 4)), (0, 0, (2, 3))], b"Mismatched allreduce tensor shapes: [2,4] vs [2,3]"),
    ([(2, 3, (5,)), (2, 3, (5, 1))], b"Mismatched broadcast tensor shapes: [5] vs [5,1]"),
    ([(1, 0, (3, 4)), (1, 0, (7, 4))], None),  # allgather: first dimension may differ
    ([(1, 0, (3, 4)), (1, 0, (3, 4, 1))], b"Mismatched allgather tensor shapes: rank 2 vs 3"),
    ([(1, 0, (3, 4)), (1, 0, (3, 5))], b"Mismatched allgather tensor shapes: 1-th dimension 4 vs 5"),
    ([(1, 0, ()), (1, 0, ())], b"An empty tensor found"),
])
def test_check_requests_reference_messages(recs, msg):
    """The reference's ConstructResponseMessage / GatherFirstRankSizes verdicts and error text
    (coordinator.cc:40-186), as a pure host function of the exchanged request records."""
    from tips_amd import _lib
    L = _lib.lib()
    ptr, _keep = _table(*recs)
    rc = L.tips_check_requests(ptr, len(recs))
    if msg is None:
        assert rc == 0
    else:
        assert rc == -7 and L.tips_last_error() == msg


def test_header_is_c99(tmp_path):
    """include/tips_hip.h compiles as strict C99 and links against the library (what an FFI binds)."""
    import shutil
    import subprocess
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    exe = str(tmp_path / "abi_check")
    lib_dir = os.path.join(REPO, "tips_amd", "lib")
    r = subprocess.run(["gcc", "-std=c99", "-pedantic", "-Wall", "-Werror", "-I" + os.path.join(REPO, "include"),
                        os.path.join(REPO, "tests", "c", "abi_check.c"), "-L" + lib_dir, "-ltips_hip",
                        "-Wl,-rpath," + lib_dir, "-o", exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "Mismatch data types found: 0 vs 1." in r.stdout


@pytest.mark.parametrize("count,p", [(268435456, 8), (268435456, 2), (262144, 2), (1000, 4), (0, 3)])
def test_schedule_shape(count, p, monkeypatch):
    """K = min(depth, ceil(chunk_bytes / min_sub)), sub = round_up(ceil(chunk/K), 256 B) (runtime.cc)."""
    import ctypes
    from tips_amd import _lib
    L = _lib.lib()
    d, sub = ctypes.c_int(), ctypes.c_int64()
    assert L.tips_schedule_shape(count, p, 0, ctypes.byref(d), ctypes.byref(sub)) == 0
    align = 64
    chunk = min(count, -(-(-(-count // p)) // align) * align)
    k = max(1, min(4, -(-chunk * 4 // (8 << 20))))
    assert d.value == k
    assert sub.value == min(chunk, -(-(-(-chunk // k)) // align) * align)


def test_only_the_c_abi_is_exported():
    """libtips_hip.so is built with -fvisibility=hidden: its dynamic symbol table holds exactly the
    functions include/tips_hip.h declares (internal runtime symbols stay private)."""
    import shutil
    import subprocess
    if not shutil.which("nm"):
        pytest.skip("no nm")
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(REPO, "tips_amd", "lib", "libtips_hip.so")],
                         capture_output=True, text=True, check=True).stdout
    text_syms = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert text_syms == set(header_functions())


@pytest.mark.parametrize("threads,jobs", [(2, 2), (8, 8), (16, 5), (4, 64)])
def test_host_pool_runs_every_job_once(threads, jobs):
    """The host-copy pool behind tips_fused_allreduce_host (no GPU): 20000 back-to-back fork-join
    runs, of two sizes in turn, each job exactly once. An earlier pool reset its job counter and
    its pending count as two separate stores, so a thread still leaving one run could claim a job
    of the next against the old count, and the caller waited forever (a GPU test with 256-B pieces,
    ~800 runs per call, hung in it)."""
    from tips_amd import _lib
    assert _lib.dev_call("tips_host_pool_selftest", threads, 20000, jobs) == 0
