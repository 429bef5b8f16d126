"""-m gpu: the RCCL executor (schedules.cc run_plan) across real processes, one RCCL rank each.

The one GPU of the test box hosts every rank. RCCL refuses two ranks of one host on one device,
so each process names its own host (NCCL_HOSTID) and RCCL joins them through its socket
transport over loopback (tests/peer_worker.py). The bytes take a slow road, but the product code
is the multi-GPU code: tips_init's TCP bootstrap and ncclCommInitRank, the per-rank op plans
(plan.cc), one ncclGroupStart/End per step on the comm stream, the compute stream's sums behind
recv events, the comm stream's waits on them. Results are bit-exact against the oracle's
restatement of each schedule's order (oracle_ring for the ring, oracle_fold for direct and
one-shot) and within the reference's tolerance of MPICH on the golden vectors.
"""
import os
import socket

import pytest

from conftest import golden_cases
from gpu_util import ALL_DTYPES, BF16, F16, F32, F64, I32, I64
from test_gpu_peer import check, run_job

pytestmark = pytest.mark.gpu


def rccl_env(algo):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return dict(TIPS_WORKER_ALGO=algo, TIPS_NO_RCCL="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                TIPS_BOOTSTRAP_PORT=str(port), NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")


@pytest.mark.parametrize("algo", ["ring", "direct", "oneshot"])
@pytest.mark.parametrize("p", [2, 3, 4])
def test_rccl_schedules_across_processes(gpu, algo, p):
    cases = []
    for dtype in ALL_DTYPES:
        for n in (1, 4099, 300007):
            cases.append({"dtype": dtype, "n": n, "seed": 10 * dtype + n % 13})
    cases.append({"dtype": F32, "n": 262147, "seed": 5, "inplace": True})
    cases.append({"dtype": I64, "n": 70001, "seed": 6, "inplace": True})
    check(run_job(p, cases, **rccl_env(algo)))


@pytest.mark.parametrize("p", [2, 3, 4, 5, 8])
def test_golden_vectors_over_rccl(gpu, p):
    """Every committed golden vector for p ranks (the reference's KATs and the seeded MPICH outputs)
    through the default multi-GPU schedule AUTO picks for it, over real RCCL ranks. At p = 8 this is
    config 3's rank count."""
    names = sorted(n for n, c in golden_cases().items() if c["p"] == p)
    cases = []
    for name in names:
        for algo in (["ring", "direct", "oneshot"] if p <= 4 else ["direct", "ring"]):
            cases.append({"golden": name, "algo": algo})
    results = run_job(p, cases, timeout=600, **rccl_env("auto"))
    check(results)
    if p == 2:
        for res in results:
            assert all(c["bit_exact_vs_mpich"] for c in res["results"])


def test_rccl_transport_is_real(gpu):
    """The ranks above really are RCCL ranks joined over RCCL's network transport (NCCL_DEBUG=INFO
    shows the socket connection), not a silent fallback: and the one-shot small case agrees."""
    env = rccl_env("oneshot")
    env.update(NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,NET")
    results = run_job(2, [{"dtype": F32, "n": 1000, "seed": 1}], **env)
    assert all(c["ok"] for res in results for c in res["results"])
    log = "".join(res["stderr"] + res["stdout"] for res in results)  # (NCCL_DEBUG prints to stdout)
    assert "NET/Socket" in log, log[-3000:]
    assert "Duplicate GPU" not in log


@pytest.mark.parametrize("workload,p", [("config4", 8), ("config5", 8), ("config5", 3)])
def test_fusion_workloads_over_rccl(gpu, workload, p):
    """Configs 4 and 5 through the fusion buckets over real RCCL ranks with the default (AUTO)
    schedule: direct for every bucket at p > 2, one-shot for buckets of 256 KiB or less; in place,
    out of place, allreduce_grads and DistributedOptimizer.step(), and with rank 0's tensors views of
    one buffer while the others' are separate allocations; bit-exact against the fold."""
    cases = [{"fused": workload, "seed": 4, "mode": m}
             for m in ("inplace", "inplace_separate", "layouts", "oop", "grads", "optimizer")]
    check(run_job(p, cases, timeout=600, **rccl_env("auto")))


@pytest.mark.parametrize("workload,p", [("config4", 3), ("config5", 3), ("config4", 8), ("config5", 8)])
def test_fp16_compression_fused_over_rccl(gpu, workload, p):
    """Compression.fp16 fused into the bucket path. allreduce_grads(...,
    compression=Compression.fp16) issues ONE tips_fused_allreduce_cast per list: every f32 gradient
    cast to f16 (RNE) as it is packed, each bucket allreduced in f16 (half the bytes on the links),
    cast back as it is unpacked - no per-tensor cast launches. Bit-exact against the oracle's
    cast -> rank-order f16 fold (fp32 accumulate, one rounding) -> cast back, over 3 and 8 RCCL
    ranks, configs 4 and 5; also with the outputs released and the call repeated (flat outputs
    reused), and with a bf16 wire (tips_amd.fused_allreduce_cast(..., "bfloat16")). The reference
    casts per tensor (tips/tensorflow/compression.py:49-66); its op has no 16-bit allreduce
    (ops.cc:121), so the 16-bit fold itself is parity-unpinned."""
    cases = [{"fused": workload, "seed": 12, "mode": m} for m in ("fp16", "fp16_fresh_outputs", "bf16_wire")]
    check(run_job(p, cases, timeout=600, **rccl_env("auto")))


@pytest.mark.parametrize("variant", ["merged_signals", "merged_no_signals"])
def test_fusion_pack_launch_variants_over_rccl(gpu, variant):
    """VERDICT r05 item 4, opt-in (TIPS_PACK_MERGE=1): a step's first two pack launches (the slot
    path) and all of the flat path's are one launch (copy_segs_groups_kernel). With signals (the
    default when merged) the bucket stream waits on the device for each bucket (hipStreamWaitValue64
    on a signal word the bucket's last workgroup raises); without (TIPS_PACK_SIGNALS=0) for the
    launch as a whole. Both bit-exact over 3 RCCL ranks, configs 4 and 5, in place, out of place and
    through allreduce_grads (the flat path). Per-bucket launches (the default) are covered above."""
    env = rccl_env("auto")
    env.update(TIPS_PACK_MERGE="1")
    if variant == "merged_no_signals":
        env.update(TIPS_PACK_SIGNALS="0")
    cases = [{"fused": w, "seed": 6, "mode": m} for w in ("config4", "config5") for m in ("inplace", "oop", "grads")]
    check(run_job(3, cases, timeout=600, **env))


@pytest.mark.parametrize("p", [2, 3])
def test_fusion_buckets_mixed_with_a_replayed_list(gpu, p):
    """Config 4's fusion buckets (two of ~41 MB: eager) alternating with a 2.5 MiB list (one bucket,
    replayed from its second call), in place, new values every round, over real RCCL ranks: every
    round bit-exact against the fold, and the replay -> eager host waits stop once the first one has
    widened the replay limit (TIPS_GRAPH_MIXED_MAX_BYTES): the fusion buckets become replays too."""
    env = rccl_env("auto")
    env.update(TIPS_GRAPHS="1")  # (replays are opt-in since round 6)
    results = run_job(p, [{"fused": "config4", "seed": 3, "mode": "mixed", "rounds": 5}], timeout=600, **env)
    check(results)
    for res in results:
        c = res["results"][0]
        w = c["waits_after_each_call"]
        assert w[-1] <= 2 and w[-1] == w[-5], c  # no waits in the last two rounds
        # round 0 grows the staging (every key dropped); the small bucket replays from round 2, the
        # fusion buckets from round 3, after round 2's one wait: 1 + 3 + 3 replays, 3 captures
        assert c["replayed"] >= 7 and c["captured"] >= 3, c


@pytest.mark.parametrize("workload", ["config4", "config5"])
def test_allreduce_grads_fresh_tensors_over_rccl(gpu, workload):
    """allreduce_grads over 3 real RCCL ranks with FRESH gradient tensors every step (a training
    loop with zero_grad(set_to_none=True)): the outputs are views of one flat buffer per dtype
    (tips_fused_allreduce_flat), each step bit-exact against the oracle's fold, and the fusion layout
    (a function of the counts alone) is built once and found on every later step
    (tips_fusion_stats). Then the same gradients as host (numpy) tensors through the fused host
    path (tips_fused_allreduce_host), bit-exact."""
    cases = [{"fused": workload, "seed": 9, "mode": m} for m in ("grads_fresh", "host_grads")]
    results = run_job(3, cases, timeout=600, **rccl_env("auto"))
    check(results)
    for res in results:
        st = res["results"][0]["stats"]
        assert st["layouts_built"] <= 1 and st["layout_hits"] >= 3, st


@pytest.mark.parametrize("algo,p,lanes", [("ring", 2, 2), ("ring", 3, 3), ("direct", 3, 2), ("direct", 4, 2)])
def test_transfer_lanes_across_processes(gpu, algo, p, lanes):
    """TIPS_LANES: step i's group on lane i % L, each lane a communicator split from the job's
    (ncclCommSplit) with its own stream, plus the cross-lane waits the single comm stream gave for
    free (the ring's allgather forwarding). Deep pipelines (sub-chunks of 4 KiB) so many groups
    are in flight; ragged sizes, in place, every dtype; bit-exact against the schedule's oracle.
    The one-lane calls at the end run after the lane calls on the same staging."""
    env = rccl_env(algo)
    env.update(TIPS_LANES=str(lanes), TIPS_PIPELINE_DEPTH="4", TIPS_MIN_SUBCHUNK_BYTES="4096")
    cases = []
    for dtype in ALL_DTYPES:
        for n in (4099, 300007):
            cases.append({"dtype": dtype, "n": n, "seed": 20 * dtype + n % 11})
    cases.append({"dtype": F32, "n": 262147, "seed": 5, "inplace": True})
    cases.append({"dtype": I64, "n": 70001, "seed": 6, "inplace": True})
    check(run_job(p, cases, **env))


@pytest.mark.parametrize("algo,p", [("direct", 2), ("ring", 3), ("oneshot", 3)])
def test_replayed_plans_in_python_processes(gpu, algo, p):
    """TIPS_GRAPHS=1 in Python processes, i.e. on the HIP runtime and RCCL that torch bundles
    (ROCm 7.0.2, RCCL 2.26): the groups are captured on the graph's origin stream (a group captured
    on a forked stream crashes that runtime, tools/graph_probe.py mode 3). Buffers reduced round
    after round from two streams, one reallocated half way, interleaved with an eager bucket
    over the replay limit: replays happen and every result is bit-exact. Every eager bucket that
    follows a replay takes order_after_replays' host wait (tips_replay_order_stats counts them;
    tests/test_plans.py::test_eager_after_replay_takes_the_host_wait shows why it must). The
    eager bucket stays eager here (TIPS_GRAPH_MIXED_MAX_BYTES=0), so every round takes the wait."""
    env = rccl_env(algo)
    env.update(TIPS_GRAPHS="1", TIPS_GRAPH_MAX_BYTES=str(2 << 20), TIPS_GRAPH_MIXED_MAX_BYTES="0")
    bufs = [[F32, 300007, False, False], [I64, 70001, True, False], [BF16, 4099, False, True],
            [F32, (3 << 20) + 17, True, False]]
    results = run_job(p, [{"bufs": bufs, "seed": 8, "rounds": 6}], timeout=600, **env)
    check(results)
    for res in results:
        c = res["results"][0]
        assert c["graphs_off"] == 0 and c["captured"] >= 3 and c["replayed"] >= 9, c
        # rounds 2-5: replays of buffers 0-2, then the eager 12 MiB bucket (round 0 grows the staging)
        assert c["replay_host_waits"] >= 4, c


@pytest.mark.parametrize("algo,p", [("direct", 2), ("oneshot", 3)])
def test_mixed_buckets_become_replays(gpu, algo, p):
    """The same rounds with the default TIPS_GRAPH_MIXED_MAX_BYTES. Per-call trace (w = a host wait,
    r = a replay, c = a capture): round 0 grows the staging (which drops every graph key), round 1
    sees each small key once, round 2 captures and replays them and then the 12 MiB bucket waits:
    that wait makes plans up to 1 GiB replayable and records the bucket's key as seen, so round 3
    captures it, and from then on every call is a replay: 1 wait instead of 4, results bit-exact.
    (The reallocated buffer 0 of round 3 may land at its old address in the same allocator segment,
    the same key: it replays; tests/test_plans.py::test_mixed_replays_model has the trace.)"""
    env = rccl_env(algo)
    env.update(TIPS_GRAPHS="1", TIPS_GRAPH_MAX_BYTES=str(2 << 20))
    bufs = [[F32, 300007, False, False], [I64, 70001, True, False], [BF16, 4099, False, True],
            [F32, (3 << 20) + 17, True, False]]
    results = run_job(p, [{"bufs": bufs, "seed": 9, "rounds": 7, "trace": True}], timeout=600, **env)
    check(results)
    for res in results:
        c = res["results"][0]
        print(c["trace"])
        calls = c["trace"].split()
        rounds = [calls[i:i + len(bufs)] for i in range(0, len(calls), len(bufs))]
        assert len(rounds) == 7 and c["graphs_off"] == 0, c["trace"]
        assert c["replay_host_waits"] == 1 and "".join(calls).count("w") == 1, c["trace"]
        assert rounds[2][3] == "w" and rounds[3][3] == "rc", c["trace"]  # wait, then captured
        assert all(t in ("r", "rc") for t in rounds[4]), c["trace"]  # (a new buffer 0: captured)
        assert all(t == "r" for r in rounds[5:] for t in r), c["trace"]  # then replays only


@pytest.mark.parametrize("p", [2, 3])
def test_capture_failure_after_mixing_drops_only_that_plan(gpu, p):
    """once replayed and eager buckets mixed, the 12 MiB bucket's capture fails
    (TIPS_GRAPH_TEST_FAIL_BYTES). Only that plan stays eager - it keeps paying its host wait after
    the replays before it - while the small buckets keep replaying; graphs stay on and every
    result is bit-exact."""
    env = rccl_env("direct")
    env.update(TIPS_GRAPHS="1", TIPS_GRAPH_MAX_BYTES=str(2 << 20), TIPS_GRAPH_TEST_FAIL_BYTES=str(4 << 20))
    bufs = [[F32, 300007, False, False], [I64, 70001, True, False], [BF16, 4099, False, True],
            [F32, (3 << 20) + 17, True, False]]
    results = run_job(p, [{"bufs": bufs, "seed": 19, "rounds": 7, "trace": True}], timeout=600, **env)
    check(results)
    for res in results:
        c = res["results"][0]
        calls = c["trace"].split()
        rounds = [calls[i:i + len(bufs)] for i in range(0, len(calls), len(bufs))]
        assert len(rounds) == 7 and c["graphs_off"] == 0, c["trace"]
        assert all(r[3] == "w" for r in rounds[2:]), c["trace"]  # the failed plan: eager after a replay
        assert all(t == "r" for r in rounds[5:] for t in r[:3]), c["trace"]  # the others replay
        assert c["replay_host_waits"] == 5, c["trace"]


@pytest.mark.parametrize("p", [2, 3])
def test_fresh_address_bucket_makes_replays_yield(gpu, p):
    """a replayed small bucket alternating with a large bucket at a NEW address
    every round (the old ones kept alive, so no address repeats) can never become a replay: each of
    its calls waits on the host for the replay before it. After TIPS_FRESH_WAIT_LIMIT (4) such waits
    replays yield (tips_graph_stats 3): no further wait, every result bit-exact."""
    env = rccl_env("direct")
    env.update(TIPS_GRAPHS="1", TIPS_GRAPH_MAX_BYTES=str(2 << 20))
    bufs = [[F32, 262147, False, False], [F32, (3 << 20) + 17, True, False]]
    results = run_job(p, [{"bufs": bufs, "seed": 23, "rounds": 10, "trace": True, "fresh": [1]}], timeout=600, **env)
    check(results)
    for res in results:
        c = res["results"][0]
        calls = c["trace"].split()
        rounds = [calls[i:i + len(bufs)] for i in range(0, len(calls), len(bufs))]
        assert c["graphs_off"] == 3, c["trace"]
        assert c["replay_host_waits"] == 4, c["trace"]
        assert all(r == ["-", "-"] for r in rounds[-3:]), c["trace"]  # eager, no wait


@pytest.mark.parametrize("p", [2, 3])
def test_tuned_schedule_across_processes(gpu, p):
    """TIPS_ALGO=tune over real RCCL ranks: the first call of each size class times ring and
    direct at several pipeline depths on scratch copies, the ranks agree on one choice, and every
    call (in place too: the tuning never touches the caller's buffers) gives the bits of the chosen
    schedule; small buckets take the one-shot."""
    cases = [{"dtype": F32, "n": 3 << 20, "seed": 1}, {"dtype": F32, "n": (3 << 20) + 5, "seed": 2, "inplace": True},
             {"dtype": BF16, "n": 1 << 20, "seed": 3}, {"dtype": I64, "n": 1000, "seed": 4},
             {"dtype": F32, "n": 3 << 20, "seed": 5}]
    results = run_job(p, cases, **rccl_env("tune"))
    check(results)
    picks = [tuple(c.get("tuned", ())) for c in results[0]["results"]]
    for res in results[1:]:
        assert [tuple(c.get("tuned", ())) for c in res["results"]] == picks, "ranks disagree on the tuned schedule"


def test_tuner_scratch_failure_on_one_rank_fails_everywhere(gpu):
    """One rank cannot set up the tuner's scratch copies (TIPS_TUNE_TEST_FAIL_RANK): every rank
    learns it from one small allreduce before any candidate's transfers, and every rank's call
    fails with TIPS_ERR_HIP instead of the others waiting forever in a group for it."""
    env = rccl_env("tune")
    env["TIPS_TUNE_TEST_FAIL_RANK"] = "1"
    results = run_job(3, [{"dtype": F32, "n": 3 << 20, "seed": 1, "expect_error": -3}], **env)
    check(results)
    for res in results:
        assert "some rank" in res["results"][0].get("error", ""), res


def test_staging_failure_on_one_rank_fails_everywhere(gpu):
    """Staging grows at the same call on every rank (its size depends only on the plan's
    arguments: tests/test_plans.py::test_staging_size_is_rank_independent), so the ranks agree on
    the outcome: one rank that cannot allocate it (TIPS_STAGING_TEST_FAIL_RANK) fails that call on
    every rank rather than leaving the others in a group waiting for it; a later call that needs no
    growth runs normally, bit-exact."""
    env = rccl_env("direct")
    env["TIPS_STAGING_TEST_FAIL_RANK"] = "2"
    results = run_job(3, [{"dtype": F32, "n": 3 << 20, "seed": 1, "expect_error": -3},
                          {"dtype": F32, "n": 1 << 20, "seed": 2}], **env)
    check(results)
    for res in results:
        assert "some rank" in res["results"][0].get("error", ""), res



@pytest.mark.parametrize("p", [2, 3])
def test_control_plane_and_api_over_rccl(gpu, p):
    """The rest of the surface over real RCCL ranks (so far only run over the peer transport):
    named requests through the negotiation thread (300 tensors, 6 dtypes, a different enqueue
    order on every rank), broadcast / allgatherv / the checked allreduce on RCCL collectives,
    DistributedOptimizer, DistributedGradientTape, host buffers (bounce pair and pipelined
    pieces) and the shape validation of named requests; bit-exact against the oracle's fold."""
    import numpy as np
    from gpu_util import F16, F64, I32
    rng = np.random.default_rng(13)
    dts = [F32, F32, F32, F64, I32, F16]
    tensors = [[int(dts[int(rng.integers(len(dts)))]), int(rng.choice([0, 1, 7, 300, 4099, 65536, 300000]))]
               for _ in range(300)]
    cases = [{"named": tensors, "seed": 5}, {"collectives": True, "seed": 5 + p, "big": 1536 * 1024},
             {"optimizer": True, "seed": 7}, {"tape": True, "seed": 11}, {"shapes": True}]
    cases += [{"dtype": d, "n": n, "seed": 40 + d, "host": True, "inplace": inplace}
              for d in (F32, I32, F16) for n, inplace in ((1000, False), (1310721, True))]
    env = rccl_env("auto")
    env.update(TIPS_FUSION_THRESHOLD=str(1 << 20), TIPS_HOST_PIECE_BYTES=str(1 << 20))
    check(run_job(p, cases, timeout=600, **env))


@pytest.mark.parametrize("p", [2, 3])
def test_named_broadcast_allgather_over_rccl(gpu, p):
    """tips_enqueue_broadcast / tips_enqueue_allgather (Python broadcast_async / allgather_async)
    with named allreduces, a different enqueue order on every rank, over real RCCL ranks: rank 0's
    order and checks, the allgather's output allocated once the sizes are known; bit-exact
    broadcast and allgather, a root mismatch refused on every rank (peer_worker.named_collectives_case)."""
    check(run_job(p, [{"named_collectives": True, "seed": 3 + p}], timeout=600, **rccl_env("auto")))


@pytest.mark.parametrize("algo,p", [("ring", 2), ("direct", 3)])
def test_counts_past_int32_over_rccl(gpu, algo, p):
    """A 2^31 + 13 element f16 bucket (4 GiB: byte offsets past 2^32) over real RCCL ranks, ring and
    direct; exact integer-valued sums checked on the device (peer_worker.pattern_case)."""
    check(run_job(p, [{"pattern_n": (1 << 31) + 13}], timeout=600, **rccl_env(algo)))


@pytest.mark.parametrize("p", [2, 3])
def test_overlapped_optimizer_over_rccl(gpu, p):
    """DistributedOptimizer's backward-overlapped buckets (TIPS_OVERLAP_BACKWARD=1, and the measured
    choice, =auto) over real RCCL ranks: the post-accumulate
    hooks issue every bucket's in-place allreduce during backward (8 KiB and 64 KiB buckets, so a
    small MLP makes many), in bucket order on every rank; one and two backward passes per step,
    averaged; summed gradients bit-exact against the rank-order sum (p = 2 takes the one-shot for
    these sizes, p = 3 the one-shot / direct fold), parameters p - lr * sum."""
    cases = [{"overlap": True, "seed": 21, "bucket_kib": 8},
             {"overlap": True, "seed": 22, "bucket_kib": 64, "passes": 2, "average": True},
             {"overlap": True, "seed": 23, "bucket_kib": 8, "mode": "auto"}]
    results = run_job(p, cases, timeout=600, **rccl_env("auto"))
    check(results)
    # the measured choice (optim._OverlapChoice): warm-up steps during backward, then the trial
    # alternating during / after, then one choice - the same on every rank
    first = results[0]["results"][2]
    assert first["choices"][:6] == [True, True, True, False, True, False], first
    for res in results:
        c = res["results"][2]
        assert c["choices"] == first["choices"] and c["overlap_choice"]["chosen"] == first["overlap_choice"]["chosen"]


@pytest.mark.parametrize("p", [3, 4])
def test_randomized_schedules_over_rccl(gpu, p):
    """Seeded random cases over real RCCL ranks, each its own schedule, pipeline depth, transfer
    lanes, dtype, size and in-place flag (settings the library reads per call); every result
    bit-exact against that schedule's oracle."""
    import numpy as np
    rng = np.random.default_rng(2026 + p)
    cases = []
    for i in range(24):
        algo = ["ring", "direct", "oneshot"][int(rng.integers(3))]
        cases.append({"algo": algo, "dtype": int(rng.choice(ALL_DTYPES)), "n": int(rng.integers(1, 400000)),
                      "seed": 100 + i, "inplace": bool(rng.integers(2)),
                      "env": {"TIPS_PIPELINE_DEPTH": str(int(rng.integers(1, 7))), "TIPS_MIN_SUBCHUNK_BYTES": "4096",
                              "TIPS_LANES": str(int(rng.integers(1, 3)))}})
    check(run_job(p, cases, timeout=600, **rccl_env("direct")))

