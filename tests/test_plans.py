"""The schedules' op plans on the CPU (no GPU): tips_schedule_plan dumps exactly what the RCCL
executor issues on an 8-GPU node and what the single-GPU simulator runs (plan.cc), so these
checks cover the multi-GPU default path itself, not a twin of it:

- every send pairs with a receive of equal bytes in the same group (no deadlock), for
  p = 2..16, ragged sizes and pipeline depths K = 1..6;
- the executor's streams and events order every conflicting access, across two calls from
  different user streams (no data race, staging reuse included);
- the plans, interpreted on host buffers with the oracle's arithmetic, give oracle_ring's /
  oracle_fold's bits (the reference's AllreduceCpu<T> SUM, utils.h:52-67).
"""
import numpy as np
import pytest

import plan_util as pu
from gpu_util import BF16, F16, F32, F64, I32, I64, rand

ES = {F32: 4, F64: 8, I32: 4, I64: 8, F16: 2, BF16: 2}
SIZES = [1, 7, 64, 65, 1000, 4099, 65536 + 3, 262147]


@pytest.mark.parametrize("algo", [pu.RING, pu.DIRECT, pu.ONESHOT])
@pytest.mark.parametrize("p", range(2, 17))
def test_send_recv_pairing(algo, p):
    for n in SIZES:
        for K in (range(1, 7) if algo != pu.ONESHOT else (1,)):
            for dtype in (F32, F16):
                plans = [pu.dump(algo, p, r, n, dtype, K) for r in range(p)]
                try:
                    pu.pairing(plans)
                except AssertionError as e:
                    raise AssertionError("algo %d p %d n %d K %d dtype %d: %s" % (algo, p, n, K, dtype, e))


@pytest.mark.parametrize("algo", [pu.RING, pu.DIRECT, pu.ONESHOT])
def test_staging_size_is_rank_independent(algo):
    """Every rank's plan asks for the same staging bytes, so staging grows at the same call on
    every rank and the ranks can agree on the allocation (schedules.cc grow_staging)."""
    for p in (2, 3, 5, 8, 16):
        for n in (1, 7, 4099, 262147, (1 << 20) + 3):
            for K in ((1, 2, 4) if algo != pu.ONESHOT else (1,)):
                assert len({pu.dump(algo, p, r, n, F32, K)["staging"] for r in range(p)}) == 1, (p, n, K)


def test_bucket_bytes_conserved():
    """Config 3's shape (p = 8, 1 GiB f32): each rank sends 2(p-1)/p of the bucket in the ring and
    in direct (the bandwidth-optimal volume), (p-1) buckets in one-shot; every chunk byte is summed once."""
    n, p = 268435456, 8
    for algo in (pu.RING, pu.DIRECT):
        for r in (0, 3, 7):
            pl = pu.dump(algo, p, r, n, F32)
            sent = sum(x["bytes"] for s in pl["steps"] for x in s["xfers"] if x["send"])
            got = sum(x["bytes"] for s in pl["steps"] for x in s["xfers"] if not x["send"])
            assert sent == got == 2 * (p - 1) * n * 4 // p
            summed = sum(u["count"] for s in pl["steps"] for u in s["sums"])
            assert summed == (n // p) * ((p - 1) if algo == pu.RING else 1)
    pl = pu.dump(pu.ONESHOT, 4, 1, 1000, F32)
    assert sum(x["bytes"] for s in pl["steps"] for x in s["xfers"] if x["send"]) == 3 * 4000


@pytest.mark.parametrize("algo", [pu.RING, pu.DIRECT, pu.ONESHOT])
@pytest.mark.parametrize("p,n,K", [(2, 4099, 1), (2, 262147, 4), (3, 1000, 3), (4, 65539, 6), (5, 7, 2),
                                   (8, 262147, 4), (8, 1 << 20, 2), (16, 100003, 3)])
@pytest.mark.parametrize("inplace", [False, True])
def test_stream_event_hazards(algo, p, n, K, inplace):
    """No two conflicting accesses are unordered by the executor's streams and events, over two
    back-to-back calls issued from different user streams (the one-shot fold used to run on the
    caller's stream, unordered against the next call's receives into the same staging slots)."""
    for r in sorted({0, 1, p - 1}):
        pl = pu.dump(algo, p, r, n, F32, K)
        races = pu.hazards(pl, 4, n * 4, inplace=inplace)
        assert not races, "rank %d: %s" % (r, races[:5])


@pytest.mark.parametrize("algo", [pu.RING, pu.DIRECT, pu.ONESHOT])
@pytest.mark.parametrize("p,n,K", [(2, 262147, 4), (3, 1000, 3), (8, 262147, 4)])
@pytest.mark.parametrize("modes", [("eager", "replay", "replay", "eager", "replay"), ("replay", "eager", "eager"),
                                   ("replay", "replay", "replay")])
def test_stream_event_hazards_with_replays(algo, p, n, K, modes):
    """TIPS_GRAPHS: replays of the captured plan (a graph on graph_stream, its nodes on streams of
    their own) mixed with eager calls, from alternating user streams: still no unordered conflict
    (staging shared by all calls; the joins of replay() and order_after_replays())."""
    for r in sorted({0, p - 1}):
        pl = pu.dump(algo, p, r, n, F32, K)
        for inplace in (False, True):
            races = pu.hazards(pl, 4, n * 4, inplace=inplace, modes=modes)
            assert not races, "rank %d %s: %s" % (r, modes, races[:5])


@pytest.mark.parametrize("algo", [pu.RING, pu.DIRECT, pu.ONESHOT])
@pytest.mark.parametrize("p,n,K", [(2, 262147, 4), (3, 1000, 3), (4, 65539, 6), (8, 262147, 4), (8, 1 << 20, 2),
                                   (16, 100003, 3)])
@pytest.mark.parametrize("lanes", [2, 3])
def test_stream_event_hazards_with_lanes(algo, p, n, K, lanes):
    """Transfer lanes: step i's group on lane i % L (its own stream and split communicator), with
    the executor's cross-lane waits (the latest conflicting step on each other lane); calls from
    alternating user streams, mixed with one-lane calls and replays. No unordered conflict."""
    for r in sorted({0, 1, p - 1}):
        pl = pu.dump(algo, p, r, n, F32, K)
        for inplace in (False, True):
            races = pu.hazards(pl, 4, n * 4, inplace=inplace, lanes=lanes, modes=("eager", "eager", "replay", "eager"))
            assert not races, "rank %d: %s" % (r, races[:5])


def test_lane_checker_needs_the_cross_lane_waits():
    """Without the cross-lane waits, the ring's allgather forwards bytes on one lane that the
    previous step is still receiving on the other: the checker must see the race."""
    pl = pu.dump(pu.RING, 3, 0, 1000, F32, 3)
    assert not pu.hazards(pl, 4, 4000, lanes=2)
    assert pu.hazards(pl, 4, 4000, lanes=2, cross_lane_waits=False)


def test_hazard_checker_catches_a_missing_replay_join():
    """Drop replay()'s wait for the eager work still queued on the comm / compute streams and the
    replay's receives into staging race with the eager call's sums reading it."""
    pl = pu.dump(pu.DIRECT, 4, 1, 100000, F32, 2)
    assert pu.hazards(pl, 4, 400000, modes=("eager", "replay"), replay_joins=False)
    assert not pu.hazards(pl, 4, 400000, modes=("eager", "replay"))


def test_hazard_checker_catches_a_missing_wait():
    """The checker itself: drop the ring's comm-stream wait on the previous step's sum and it must
    report the send reading `out` before the sum wrote it."""
    pl = pu.dump(pu.RING, 4, 0, 100000, F32, 2)
    for s in pl["steps"]:
        s["wait_sum"] = -1
    assert pu.hazards(pl, 4, 400000)


def _tune_candidates(p, n, dtype=F32):
    import ctypes
    from tips_amd import _lib
    L = _lib.dev()
    cap = 16
    a, d, la = (ctypes.c_int * cap)(), (ctypes.c_int * cap)(), (ctypes.c_int * cap)()
    k = L.tips_tune_candidates(p, n, dtype, a, d, la, cap)
    assert k > 0, _lib.last_error()
    return [(a[i], d[i], la[i]) for i in range(k)]


@pytest.mark.parametrize("p", [2, 4, 8])
def test_config3_direct_fold_runs_under_the_next_transfer(p):
    """Config 3 (1 GiB f32, the chunk >= 16 MiB): every direct / ring depth the tuner may keep is
    pipelined (K >= 2), and in the executor's stream model the fold of sub-chunk k is unordered
    against the transfer group of sub-chunk k + 1, so it runs on the CUs while k + 1 is on the links
    (the N = 8 rehearsal's tuner had kept depth 1 for config 3)."""
    n = (1 << 30) // 4
    cands = _tune_candidates(p, n)
    assert {a for a, _, _ in cands} >= {pu.DIRECT, pu.RING}
    for algo, K, _ in cands:
        assert K >= 2, (algo, K, cands)
        pl = pu.dump(algo, p, p - 1, n, F32, K)
        under = pu.sums_under_transfers(pl)
        if algo == pu.DIRECT:
            for k in range(K - 1):  # reduce-scatter steps 0..K-1: fold k, then transfer k + 1
                assert k + 1 in under[k], (algo, K, k, under[k])
        else:  # ring: every step's sum overlaps the next sub-chunk's transfer of the same step
            for i, js in under.items():
                if (i + 1) % K:
                    assert i + 1 in js, (algo, K, i, js)


def test_depth_one_stays_a_candidate_below_16_mib_chunks():
    """Below the 16 MiB chunk the tuner still times depth 1 against the default (one launch per
    chunk can win there), and above it never."""
    small = _tune_candidates(8, 8 * (12 << 20) // 4)  # 12 MiB chunks: K = 2 by default
    assert (pu.DIRECT, 1, 1) in small
    for mib in (16, 32, 128):
        big = _tune_candidates(8, 8 * (mib << 20) // 4)
        assert all(K >= 2 for _, K, _ in big), (mib, big)


def test_overlap_model_sees_a_serialising_wait():
    """The model itself: make every direct transfer group wait for the previous step's fold and
    nothing runs under a transfer any more."""
    pl = pu.dump(pu.DIRECT, 8, 0, (1 << 30) // 4, F32, 4)
    assert pu.sums_under_transfers(pl)[0]
    for i, s in enumerate(pl["steps"]):
        if i > 0:
            s["wait_sum"] = i - 1
    assert not any(pu.sums_under_transfers(pl)[k] for k in range(3))


@pytest.mark.parametrize("algo", [pu.RING, pu.DIRECT, pu.ONESHOT])
@pytest.mark.parametrize("dtype", [F32, I32, F64, BF16])
@pytest.mark.parametrize("p,n,K", [(2, 4099, 1), (3, 1000, 3), (4, 65539, 4), (5, 7, 2), (8, 100003, 3),
                                   (16, 20011, 2)])
def test_interpreted_plans_match_oracle(oracle, algo, dtype, p, n, K):
    rng = np.random.default_rng(p * 1000 + n + dtype)
    ins = [rand(dtype, n, rng) for _ in range(p)]
    plans = [pu.dump(algo, p, r, n, dtype, K) for r in range(p)]
    outs = pu.interpret(plans, ins, dtype, inplace=(n % 2 == 1))
    exp = oracle.ring(ins, code=dtype)[0] if algo == pu.RING else oracle.fold(ins, code=dtype, wide_acc=True)
    for o in outs:
        assert np.array_equal(o.view(np.uint8), exp.view(np.uint8))


def test_plan_argument_errors():
    from tips_amd import _lib
    L = _lib.dev()
    assert L.tips_schedule_plan(pu.DIRECT, 17, 0, 100, F32, 1, None, 0) == -1  # fold takes <= 16 sources
    assert L.tips_schedule_plan(pu.RING, 1, 0, 100, F32, 1, None, 0) == -1
    assert L.tips_schedule_plan(pu.RING, 4, 4, 100, F32, 1, None, 0) == -1
    assert L.tips_schedule_plan(2, 4, 0, 100, F32, 1, None, 0) == -1  # ncclAllReduce has no plan
    assert L.tips_schedule_plan(pu.RING, 4, 0, 100, 42, 1, None, 0) == -1
    assert L.tips_schedule_plan(pu.RING, 32, 5, 100, F32, 2, None, 0) > 0  # the ring takes any p


# ------------------------------------------------------------------ randomized (hypothesis)

from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as hs  # noqa: E402


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.too_slow], derandomize=True)
@given(algo=hs.sampled_from([pu.RING, pu.DIRECT, pu.ONESHOT]), p=hs.integers(2, 12), n=hs.integers(0, 40000),
       K=hs.integers(1, 8), dtype=hs.sampled_from([F32, F64, I32, I64, F16, BF16]), inplace=hs.booleans(),
       lanes=hs.integers(1, 3))
def test_plans_randomized(oracle, algo, p, n, K, dtype, inplace, lanes):
    """Random schedule shapes: every property the parametrized tests check, at once - send /
    receive pairing, rank-independent staging, bit-exact interpretation against the oracle's order,
    and no unordered conflict in the executor's streams (with transfer lanes) for rank 0."""
    if n == 0:
        return  # (allreduce_device returns before any plan for an empty bucket)
    plans = [pu.dump(algo, p, r, n, dtype, K) for r in range(p)]
    pu.pairing(plans)
    assert len({pl["staging"] for pl in plans}) == 1
    rng = np.random.default_rng(n * 31 + p)
    ins = [rand(dtype, n, rng) for _ in range(p)]
    outs = pu.interpret(plans, ins, dtype, inplace=inplace)
    exp = oracle.ring(ins, code=dtype)[0] if algo == pu.RING else oracle.fold(ins, code=dtype, wide_acc=True)
    for o in outs:
        assert np.array_equal(o.view(np.uint8), exp.view(np.uint8))
    assert not pu.hazards(plans[0], ES[dtype], n * ES[dtype], inplace=inplace, lanes=lanes,
                          modes=("eager", "eager", "replay", "eager") if lanes == 1 else ("eager", "eager"))


@pytest.mark.parametrize("algo", [pu.RING, pu.DIRECT, pu.ONESHOT])
@pytest.mark.parametrize("p,n,dtype", [(2, (1 << 31) + 13, F16), (3, (1 << 31) + 13, F32), (8, (1 << 31) + 13, F32),
                                       (8, (3 << 31) + 7, F64)])
def test_counts_past_int32(algo, p, n, dtype):
    """Buckets of more than 2^31 elements (the reference's count is an int, utils.h:62; the C-ABI
    takes int64): every rank's plan pairs, stays inside in / out / staging, and its sums and
    receives together write every byte of out."""
    es = ES[dtype]
    plans = [pu.dump(algo, p, r, n, dtype) for r in range(p)]
    pu.pairing(plans)
    for r, pl in enumerate(plans):
        lim = {pu.IN: n * es, pu.OUT: n * es, pu.STG: pl["staging"]}
        writes = []
        for st in pl["steps"]:
            for x in st["xfers"]:
                assert 0 <= x["off"] and x["off"] + x["bytes"] <= lim[x["buf"]], (r, x)
                if not x["send"] and x["buf"] == pu.OUT:
                    writes.append((x["off"], x["off"] + x["bytes"]))
            for u in st["sums"]:
                nb = u["count"] * es
                for b, off in u["srcs"] + [u["dst"]]:
                    assert 0 <= off and off + nb <= lim[b], (r, u)
                if u["dst"][0] == pu.OUT:
                    writes.append((u["dst"][1], u["dst"][1] + nb))
        covered, end = 0, 0
        for s, e in sorted(writes):
            if e > end:
                covered += e - max(s, end)
                end = e
        assert covered == n * es and end == n * es, (r, covered, n * es)


def _groups(algo, p, n, K):
    """Transfer groups (one ncclGroupStart/End each) of rank 0's plan."""
    return sum(1 for s in pu.dump(algo, p, 0, n, F32, K)["steps"] if s["xfers"])


@pytest.mark.parametrize("seq", [("replay", "eager"), ("eager", "replay", "eager", "replay", "replay", "eager"),
                                 ("replay", "replay", "eager", "eager"), ("replay", "eager", "replay", "eager")])
@pytest.mark.parametrize("algo,p,n,K", [(pu.ONESHOT, 2, 65536, 1), (pu.DIRECT, 8, 262147, 2), (pu.RING, 4, 100003, 3)])
def test_eager_after_replay_takes_the_host_wait(seq, algo, p, n, K):
    """RCCL's proxy order (plan_util.proxy_order): with order_after_replays' host wait until the
    pending replay has RUN, every group's operations reach the proxy in the device's order, for any
    mix of replayed and eager calls of real plans (a replayed small bucket, an eager large one);
    without the wait an eager call after a replay is posted ahead of the replay's groups; waiting
    only for the replay's START leaves a multi-group plan's later groups behind the eager call
    (why schedules.cc waits for the end and counts the waits: tips_replay_order_stats)."""
    ng = _groups(algo, p, n, K)
    calls = [(m, ng) for m in seq]
    posted, device = pu.proxy_order(calls, "end")
    assert posted == device
    posted, device = pu.proxy_order(calls, "none")
    assert posted != device  # every sequence here has an eager call after a pending replay
    posted, device = pu.proxy_order(calls, "start")
    assert (posted == device) == (ng == 1)


# tests/test_gpu_rccl_procs.py::test_mixed_buckets_become_replays: the per-call traces a rank printed
# on the MI355X box, 6 rounds of 1.2 MB, 0.56 MB and 8 KB buckets (limit 2 MiB) and one of 12 MiB:
# before and after the widening wait recorded the waiting call's key (profiles/r04/zzb_, zzg_
# mixed_replay_trace.txt; the latter ran 7 rounds, its first 6 are these)
GPU_MIXED_TRACE_FIRST = "- - - - - - - - rc rc rc w r r r w r r r rc r r r r"
GPU_MIXED_TRACE = "- - - - - - - - rc rc rc w r r r rc r r r r r r r r"


@pytest.mark.parametrize("mixed_cap,note", [(1 << 30, True), (1 << 30, False), (0, True)])
def test_mixed_replays_model(mixed_cap, note):
    """plan_util.replay_trace restates schedules.cc's replay bookkeeping. With the default
    TIPS_GRAPH_MIXED_MAX_BYTES it reproduces the traces the GPU test printed call for call: one
    host wait, then replays only (two waits before the waiting call's key was recorded); with 0 the
    12 MiB bucket waits in every round from the third. Either way proxy_order with the host wait at
    the replay's end posts every group in device order, and once the sequence is all replays no
    wait is needed to keep it so."""
    sizes = [300007 * 4, 70001 * 8, 4099 * 2, ((3 << 20) + 17) * 4]
    tr = pu.replay_trace(6, sizes, mixed_cap=mixed_cap, note_on_wait=note)
    tokens = " ".join(t for t, _ in tr)
    if mixed_cap:
        assert tokens == (GPU_MIXED_TRACE if note else GPU_MIXED_TRACE_FIRST)
    else:
        assert tokens.split().count("w") == 4 and tokens.endswith("r r r w")
    calls = [(m, 3) for _, m in tr]
    posted, device = pu.proxy_order(calls, "end")
    assert posted == device
    tail = calls[-8:]
    if mixed_cap:
        assert all(m == "replay" for m, _ in tail)
        posted, device = pu.proxy_order(tail, "none")
        assert posted == device


def test_capture_failure_model():
    """A capture that fails (TIPS_GRAPH_TEST_FAIL_BYTES on the GPU, test_gpu_rccl_procs.py::
    test_capture_failure_after_mixing_drops_only_that_plan) leaves that key eager - a host wait
    after the replays before it, every round - and every other key replaying; RCCL's proxy still
    sees device order."""
    sizes = [300007 * 4, 70001 * 8, 4099 * 2, ((3 << 20) + 17) * 4]
    tr = pu.replay_trace(7, sizes, fail_bytes=4 << 20)
    tokens = [t for t, _ in tr]
    rounds = [tokens[i:i + 4] for i in range(0, len(tokens), 4)]
    assert all(r[3] == "w" for r in rounds[2:]) and tokens.count("w") == 5
    assert all(t == "r" for r in rounds[3:] for t in r[:3])
    posted, device = pu.proxy_order([(m, 3) for _, m in tr], "end")
    assert posted == device


@settings(max_examples=200, deadline=None)
@given(sizes=hs.lists(hs.integers(1 << 10, 64 << 20), min_size=1, max_size=6),
       groups=hs.lists(hs.integers(1, 4), min_size=6, max_size=6), rounds=hs.integers(5, 8),
       mixed=hs.booleans())
def test_replay_bookkeeping_properties(sizes, groups, rounds, mixed):
    """Any fixed list of bucket sizes called round after round (plan_util.replay_trace): with the
    host wait at the replay's end, RCCL's proxy receives every group in device order (proxy_order);
    with the mixed limit on (covering every size here), the sequence settles: from round 4 on no
    call waits, and every call of the last round is a replay once any call has replayed."""
    tr = pu.replay_trace(rounds, sizes, mixed_cap=(1 << 30) if mixed else 0)
    calls = [(m, groups[i % len(sizes)]) for i, (_, m) in enumerate(tr)]
    posted, device = pu.proxy_order(calls, "end")
    assert posted == device
    if mixed:
        late = tr[4 * len(sizes):]
        assert all(t != "w" for t, _ in late)
        if any(m == "replay" for _, m in tr):
            assert all(m == "replay" for _, m in tr[-len(sizes):])
