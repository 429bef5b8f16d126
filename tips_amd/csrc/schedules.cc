// schedules.cc — the allreduce schedules' executors: over RCCL point-to-point
// (xGMI, one rank per GPU) and, for tests, for p virtual ranks on one GPU.
//
// Replaces what MPI_Allreduce does inside libmpi for AllreduceCpu<T>
// (reference tips/core/collective/utils.h:60-65): the reduce-scatter +
// allgather exchange and, at each step, the local MPI_SUM — here the gfx950
// kernels of kernels.hip. Both executors run the same per-rank op plans
// (plan.cc): the simulator is not a second implementation of the schedules.
// One comm stream carries every RCCL call of a rank (one ordered channel, as
// the reference's single MPI_COMM_WORLD); sums run on a separate compute
// stream, so sub-chunk k+1's transfer overlaps sub-chunk k's sum.
#include <string.h>

#include <algorithm>
#include <chrono>
#include <tuple>

#include "plan.h"
#include "rt.h"

namespace tips {
namespace rt {
namespace {

int launch_psum(const PSum& s, char* const* base, int dtype, hipStream_t stream) {
  void* dst = base[s.dst.buf] + s.dst.off;
  if (s.nsrc == 2) {
    HIP_TRY(tips::launch_sum2(dst, base[s.src[0].buf] + s.src[0].off, base[s.src[1].buf] + s.src[1].off, s.count,
                              dtype, stream));
    return 0;
  }
  const void* srcs[tips::kMaxSrcs];
  for (int j = 0; j < s.nsrc; j++) srcs[j] = base[s.src[j].buf] + s.src[j].off;
  HIP_TRY(tips::launch_multi_sum(dst, srcs, s.nsrc, s.count, dtype, stream));
  return 0;
}

// Eager plan work (and RCCL calls on the comm stream) after every replayed plan still in flight:
// a replay reads and writes the same staging and issues RCCL work on the same communicator.
// An eager RCCL call after a replay: on the device it waits for the replay (the comm stream joins
// the graph stream); on the HOST it also waits until the replay has run (TIPS_REPLAY_HOST_ORDER,
// default on). RCCL posts a replayed group's proxy operations from a host node of the graph, when
// the device reaches that group; an eager group posts its own when it is issued. Issued while a
// replay still waited in the queue (or between two of its groups), the eager call's operations
// reached the proxy first, the proxy worked on them, the device ran the replay first and waited for
// the replay's - on every rank. Seen as a hang of the op-body test over 3 socket-transport RCCL
// ranks: without this wait 3 of 10 runs hung, every rank in an eager call's hipStreamSynchronize;
// with it 12 of 12 ran clean, as with replays off (profiles/r03/k_op_body_hang.txt,
// k_hunt_summary.txt). Waiting for the replay's start would not do: a multi-step plan posts each
// group's operations when the device reaches that group, so only the end of the replay covers its
// last group. tests/plan_util.py proxy_order() models the hazard; tips_replay_order_stats counts
// the waits and their host time.
int order_after_replays(State& st) {
  if (!st.graph_pending) return 0;
  TRY(join(st.comm_stream, st.graph_stream, st.ev_graph[4]));
  HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.ev_graph[4], 0));
  st.graph_pending = false;
  if (env_i64("TIPS_REPLAY_HOST_ORDER", 1) != 0) {
    const auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(hipEventSynchronize(st.ev_graph[4]));
    st.replay_host_waits++;
    st.replays_mixed = true;
    st.replay_host_wait_ns +=
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  }
  return 0;
}

// Transfer lane l: the comm stream and communicator for l = 0, a split communicator after that.
hipStream_t lane_stream(State& st, int l) { return l == 0 ? st.comm_stream : st.lane_stream[l - 1]; }
ncclComm_t lane_comm(State& st, int l) { return l == 0 ? st.comm : st.lane_comm[l - 1]; }

// Lanes 1..L-1 exist. ncclCommSplit is collective: every rank reaches it at the same call, since
// every rank runs the same schedule choice (TIPS_LANES is the same everywhere; the tuner agrees).
int lanes_ensure(State& st, int L) {
  while ((int)st.lane_comm.size() < L - 1) {
    int least = 0, greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest));
    ncclComm_t c = nullptr;
    const ncclResult_t r = ncclCommSplit(st.comm, 0, st.rank, &c, nullptr);
    if (r != ncclSuccess) {
      (void)hipStreamDestroy(s);
      return fail(TIPS_ERR_RCCL, "ncclCommSplit for transfer lane %zu failed: %s", st.lane_comm.size() + 1,
                  ncclGetErrorString(r));
    }
    st.lane_comm.push_back(c);
    st.lane_stream.push_back(s);
  }
  TRY(st.lane_ev.ensure(st.lane_stream.size() + 1));
  return 0;
}

// Stream prologue shared by both executors: the comm stream waits for the caller's stream (the
// inputs are ready) and for every sum already queued on the compute stream (the previous call's
// sums have read the staging slots this call's receives overwrite, whatever stream that call
// came on); the compute stream waits for the caller's stream.
// With transfer lanes the comm stream also waits for every lane's queued transfers (an earlier
// call's receives into staging, on whatever lane), and lanes 1..L-1 start after the comm stream.
int prologue(State& st, hipStream_t user, int L = 1) {
  TRY(order_after_replays(st));
  TRY(join(st.comm_stream, user, st.ev_start));
  TRY(join(st.comm_stream, st.comp_stream, st.ev_comp_prev));
  for (size_t l = 0; l < st.lane_stream.size(); l++) TRY(join(st.comm_stream, st.lane_stream[l], st.lane_ev.ev[l + 1]));
  if (L > 1) {
    HIP_TRY(hipEventRecord(st.lane_ev.ev[0], st.comm_stream));
    for (int l = 1; l < L; l++) HIP_TRY(hipStreamWaitEvent(st.lane_stream[l - 1], st.lane_ev.ev[0], 0));
  }
  HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.ev_start, 0));
  st.eager_pending = true;
  return 0;
}

int epilogue(State& st, hipStream_t user, int L = 1) {
  TRY(join(user, st.comm_stream, st.ev_done));
  for (int l = 1; l < L; l++) TRY(join(user, st.lane_stream[l - 1], st.lane_ev.ev[l]));
  TRY(join(user, st.comp_stream, st.ev_comp_done));
  return 0;
}

// Two steps' transfer groups touch a common byte range and at least one of them writes it
// (addresses, not plan buffers: in place, in and out are one buffer).
bool xfers_conflict(const PStep& a, const PStep& b, char* const* base) {
  for (const PXfer& x : a.xfers)
    for (const PXfer& y : b.xfers) {
      if (x.send && y.send) continue;
      const char* xp = base[x.at.buf] + x.at.off;
      const char* yp = base[y.at.buf] + y.at.off;
      if (xp < yp + y.bytes && yp < xp + x.bytes) return true;
    }
  return false;
}

// One rank's plan over RCCL: each step's transfers are one ncclGroupStart/End on the comm
// stream, followed by an event the compute stream waits on before the step's sums; a step's
// wait_sum makes the comm stream wait for an earlier step's sums (what it sends, they wrote).
// With L > 1 lanes, step i's group runs on lane i % L. One comm stream ordered every group after
// the previous one; across lanes that order is restated where it matters: a step waits for the
// latest earlier step on each other lane whose transfers touch its bytes (the ring's allgather
// forwards what the previous step received). Every other order comes from wait_sum and the
// compute stream, as with one lane (tests/plan_util.py hazards(lanes=...) checks both).
int issue_steps(State& st, const Plan& pl, char* const* base, int L = 1, hipStream_t lane0 = nullptr) {
  const size_t nsteps = pl.steps.size();
  std::vector<std::vector<int>> deps(L > 1 ? nsteps : 0);
  std::vector<char> needed(L > 1 ? nsteps : 0, 0);
  if (L > 1) {
    TRY(st.xfer_ev.ensure(nsteps));
    for (size_t i = 0; i < nsteps; i++)
      for (int l = 0; l < L; l++) {
        if (l == (int)(i % L)) continue;
        for (int j = (int)i - 1; j >= 0; j--)
          if (j % L == l && xfers_conflict(pl.steps[j], pl.steps[i], base)) {
            deps[i].push_back(j);
            needed[j] = 1;
            break;
          }
      }
  }
  for (size_t i = 0; i < nsteps; i++) {
    const PStep& s = pl.steps[i];
    const int l = (int)(i % L);
    hipStream_t cs = (l == 0 && lane0) ? lane0 : lane_stream(st, l);
    ncclComm_t cc = lane_comm(st, l);
    if (s.wait_sum >= 0 && !pl.steps[s.wait_sum].sums.empty())
      HIP_TRY(hipStreamWaitEvent(cs, st.sum_ev.ev[s.wait_sum], 0));
    if (L > 1)
      for (int j : deps[i]) HIP_TRY(hipStreamWaitEvent(cs, st.xfer_ev.ev[j], 0));
    if (!s.xfers.empty()) {
      NCCL_TRY(ncclGroupStart());
      for (const PXfer& x : s.xfers) {
        char* ptr = base[x.at.buf] + x.at.off;
        if (x.send) {
          NCCL_TRY(ncclSend(ptr, (size_t)x.bytes, ncclInt8, x.peer, cc, cs));
        } else {
          NCCL_TRY(ncclRecv(ptr, (size_t)x.bytes, ncclInt8, x.peer, cc, cs));
        }
      }
      NCCL_TRY(ncclGroupEnd());
    }
    if (L > 1 && needed[i]) HIP_TRY(hipEventRecord(st.xfer_ev.ev[i], cs));
    if (!s.sums.empty()) {
      HIP_TRY(hipEventRecord(st.recv_ev.ev[i], cs));
      HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.recv_ev.ev[i], 0));
      for (const PSum& ps : s.sums) TRY(launch_psum(ps, base, pl.dtype, st.comp_stream));
      HIP_TRY(hipEventRecord(st.sum_ev.ev[i], st.comp_stream));
    }
  }
  return 0;
}

// ---------------------------------------------------------------------------
// TIPS_GRAPHS: replayed plans. A plan's host cost is one ncclGroupStart/End of up to 2(p-1)
// p2p calls per step plus its event records, waits and sum launches: ~100-250 us of HIP/RCCL API
// time at p = 8, about what moving a 10-30 MiB bucket over xGMI takes. A plan called again on
// the same buffers (the fusion slots, a training loop's gradient buckets) is captured once into a
// HIP graph - the same steps, streams and events, as graph edges - and from then on replayed with
// one hipGraphLaunch on graph_stream. Capture waits for a plan's second call, so RCCL has set up
// its connections eagerly (outside any capture) on the first. Keys carry the buffers' allocation
// ids, not only their addresses: a buffer freed and reallocated at the same address is a new key.

}  // namespace

struct PlanGraphs {
  // (algo, K, dtype, count, in, out, staging, in allocation id, out allocation id)
  using Key = std::tuple<int, int, int, int64_t, const void*, const void*, const void*, unsigned long long,
                         unsigned long long>;
  struct Ent {
    hipGraphExec_t exec = nullptr;  // null: seen once, runs eagerly
    uint64_t stamp = 0;
    bool failed = false;  // its capture failed: this key runs eagerly from now on
  };
  std::map<Key, Ent> m;
  uint64_t clock = 0;
  int failures = 0;  // captures that failed, on distinct keys
  bool off = false;  // kMaxCaptureFailures captures failed: eager for the rest of the job
};

namespace {

unsigned long long allocation_id(const void* p) {
  unsigned long long id = 0;
  if (hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return id;
}

void destroy_exec(State& st, hipGraphExec_t e) {
  if (!e) return;
  (void)hipStreamSynchronize(st.graph_stream);  // (not while a replay of it may run)
  (void)hipGraphExecDestroy(e);
}

// Replays are opt-in (TIPS_GRAPHS=1; round 6): while a plan is being captured, any
// other thread's work on the legacy null stream (hipMemcpy, hipMemset, a launch on stream 0 - torch's
// default stream) makes the HIP runtime invalidate the capture, although every stream in it is
// non-blocking ("operation would make the legacy stream depend on a capturing blocking stream", in
// relaxed, thread-local and global mode alike: tools/capture_race_hip.cc, profiles/r06/), and RCCL's
// group launch does not survive a capture invalidated under it (SIGSEGV in hipGraphRetainUserObject
// / hipLaunchHostFunc, heap corruption: the round-5 op-body crash). The library cannot see what a
// host's other threads do, so it captures only when the host says none of them uses the legacy
// stream. Where opted in, replays run where the capture pattern (capture_plan) was seen
// to replay correctly: RCCL >= 2.26 on a HIP runtime >= 7.0, i.e. torch's bundled ROCm 7.0.2 (a
// Python process) and /opt/rocm's 7.2 (a C / cgo / JNI host) - tests/test_gpu_graphs.py and
// test_gpu_rccl_procs.py::test_replayed_plans_in_python_processes - and for buckets up to
// TIPS_GRAPH_MAX_BYTES (8 MiB), where a call's host cost, not its bytes, bounds it: the host time
// of a call drops 126 -> 22 us (one-shot p = 2, Python) (profiles/r02/graph_host_cost*.jsonl), and
// on the p = 2 rehearsal a replayed one-shot was the fastest path at every size from 16 KiB to
// 8 MiB, 4-30 % under the eager one (profiles/r03/small_bucket_rehearsal_n2_before.json; round 2 stopped
// at 1 MiB). TIPS_GRAPHS=0 (the default) keeps them off; 2 forces them on any runtime (probing only).
// Once an eager plan has had to wait on the host for a replay (order_after_replays: replayed and
// eager buckets alternate, e.g. a step's buckets straddle the 8 MiB limit), plans up to
// TIPS_GRAPH_MIXED_MAX_BYTES (1 GiB; 0 keeps the limit) are replayed as well: from their third call
// on, the alternation is replay -> replay, which needs no host wait.
bool graphs_supported() {
  static std::atomic<int> ok{-1};  // (set once, by whichever thread asks first)
  int v = ok.load(std::memory_order_relaxed);
  if (v < 0) {
    int rv = 0, hv = 0;
    v = ncclGetVersion(&rv) == ncclSuccess && hipRuntimeGetVersion(&hv) == hipSuccess && rv >= 22600 && hv >= 70000000;
    (void)hipGetLastError();
    ok.store(v, std::memory_order_relaxed);
  }
  return v == 1;
}

bool graph_eligible(State& st, const Plan& pl, hipStream_t user) {
  if ((st.graphs && st.graphs->off) || st.replays_yield) return false;
  // Not on the negotiation thread: it executes named requests (and, once a negotiation runs, every
  // routed collective) while the caller's threads go on calling HIP - creating streams, copying,
  // waiting on events. A plan captured there in a C host (/opt/rocm's 7.2 runtime, RCCL 2.27) with
  // such calls in flight crashed inside RCCL at the capture (tests/c/op_body.c's second step over
  // the same names, 3 ranks); with graphs off the same run is bit-exact. Those plans run eagerly.
  if (on_negotiation_thread() && env_i64("TIPS_GRAPHS_NEGOTIATION", 0) == 0) return false;
  const int64_t want = env_i64("TIPS_GRAPHS", 0);
  if (want <= 0 || (want == 1 && !graphs_supported())) return false;
  int64_t cap = env_i64("TIPS_GRAPH_MAX_BYTES", 8 << 20);
  if (st.replays_mixed) cap = std::max(cap, env_i64("TIPS_GRAPH_MIXED_MAX_BYTES", int64_t(1) << 30));
  if (pl.n * tips::dtype_size(pl.dtype) > cap) return false;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(user, &cs) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return cs == hipStreamCaptureStatusNone;  // the caller's own capture takes the eager steps
}

// Captures the plan on graph_stream, which issues the groups itself (the comm stream's part), with
// the compute stream forked from it and joined back: the graph holds the eager executor's steps
// and edges. The groups stay on the capture's origin stream because the ROCm 7.0.2 runtime and
// RCCL 2.26 that torch bundles crash in hipStreamEndCapture when a grouped ncclSend/ncclRecv is
// captured on a forked stream (tools/graph_probe.py mode 3, no library involved), while groups on
// the origin with a forked stream beside them replay correctly there and on /opt/rocm's 7.2
// (mode 5; tests/test_gpu_graphs.py). On failure the forked stream is still joined back, so the
// capture ends and every stream leaves capture mode.
int capture_plan(State& st, const Plan& pl, char* const* base, hipGraphExec_t* exec) {
  HIP_TRY(hipStreamBeginCapture(st.graph_stream, hipStreamCaptureModeRelaxed));
  int rc = hipEventRecord(st.ev_start, st.graph_stream) == hipSuccess &&
                   hipStreamWaitEvent(st.comp_stream, st.ev_start, 0) == hipSuccess
               ? 0
               : fail(TIPS_ERR_HIP, "capture: compute stream fork failed");
  if (rc == 0) rc = issue_steps(st, pl, base, 1, st.graph_stream);
  const int jc = join(st.graph_stream, st.comp_stream, st.ev_comp_done);
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(st.graph_stream, &g);
  if (rc == 0) rc = jc;
  if (rc == 0 && (e != hipSuccess || !g)) rc = fail(TIPS_ERR_HIP, "hipStreamEndCapture failed: %s", hipGetErrorString(e));
  if (rc == 0) {
    const hipError_t ei = hipGraphInstantiate(exec, g, nullptr, nullptr, 0);
    if (ei != hipSuccess) {
      *exec = nullptr;
      rc = fail(TIPS_ERR_HIP, "hipGraphInstantiate failed: %s", hipGetErrorString(ei));
    }
  }
  if (g) (void)hipGraphDestroy(g);
  (void)hipGetLastError();
  return rc;
}

constexpr int kMaxCaptureFailures = 3;
// host waits of one plan shape at new addresses before replays yield (TIPS_FRESH_WAIT_LIMIT, 4)
int fresh_wait_limit() { return (int)std::max<int64_t>(1, env_i64("TIPS_FRESH_WAIT_LIMIT", 4)); }

// The graph to replay for this call, or null: run eagerly (first call of a key, its capture
// failed, or graphs off).
// note_only: record a new key as seen, never capture.
hipGraphExec_t plan_graph(State& st, const Plan& pl, char* const* base, bool note_only = false,
                          bool* key_new = nullptr) {
  if (!st.graphs) st.graphs = new PlanGraphs();
  PlanGraphs& G = *st.graphs;
  const unsigned long long in_id = allocation_id(base[kBufIn]), out_id = allocation_id(base[kBufOut]);
  if (!in_id || !out_id) return nullptr;
  const PlanGraphs::Key k{pl.algo, pl.K, pl.dtype, pl.n, base[kBufIn], base[kBufOut], base[kBufStaging], in_id, out_id};
  auto it = G.m.find(k);
  if (key_new) *key_new = it == G.m.end();
  if (it == G.m.end()) {
    const size_t cap = (size_t)std::max<int64_t>(1, env_i64("TIPS_GRAPH_CACHE", 64));
    while (G.m.size() >= cap) {  // least recently used out
      auto lru = G.m.begin();
      for (auto j = G.m.begin(); j != G.m.end(); ++j)
        if (j->second.stamp < lru->second.stamp) lru = j;
      destroy_exec(st, lru->second.exec);
      G.m.erase(lru);
    }
    G.m[k].stamp = ++G.clock;
    return nullptr;
  }
  it->second.stamp = ++G.clock;
  if (note_only || it->second.failed) return nullptr;
  if (!it->second.exec) {
    // (test hook: TIPS_GRAPH_TEST_FAIL_BYTES = a capture of a plan of at least that many bytes fails)
    const int64_t fail_bytes = env_i64("TIPS_GRAPH_TEST_FAIL_BYTES", 0);
    const int rc = fail_bytes > 0 && pl.n * tips::dtype_size(pl.dtype) >= fail_bytes
                       ? fail(TIPS_ERR_HIP, "capture refused by TIPS_GRAPH_TEST_FAIL_BYTES")
                       : capture_plan(st, pl, base, &it->second.exec);
    if (rc != 0) {
      // only this key runs eagerly from now on (one large plan's failure used to turn
      // replays off for every plan of the job); repeated failures mean the runtime cannot capture
      it->second.failed = true;
      it->second.exec = nullptr;
      if (++G.failures >= kMaxCaptureFailures) G.off = true;
      if (getenv("TIPS_VERBOSE"))
        fprintf(stderr, "[tips] plan capture failed (%d so far%s): %s\n", G.failures, G.off ? ", replays off" : "",
                last_error().c_str());
      return nullptr;
    }
    st.graphs_captured++;
  }
  return it->second.exec;
}

int replay(State& st, hipGraphExec_t exec, hipStream_t user) {
  TRY(join(st.graph_stream, user, st.ev_graph[0]));
  if (st.eager_pending) {  // earlier eager plans still own staging / the communicator's order
    TRY(join(st.graph_stream, st.comm_stream, st.ev_graph[1]));
    TRY(join(st.graph_stream, st.comp_stream, st.ev_graph[2]));
    for (size_t l = 0; l < st.lane_stream.size(); l++) TRY(join(st.graph_stream, st.lane_stream[l], st.lane_ev.ev[l + 1]));
    st.eager_pending = false;
  }
  HIP_TRY(hipGraphLaunch(exec, st.graph_stream));
  TRY(join(user, st.graph_stream, st.ev_graph[3]));
  st.graph_pending = true;
  st.graphs_replayed++;
  return 0;
}

// Staging grows at the same call on every rank (its size is a function of the plan, which every
// rank builds from the same arguments), so the ranks can agree on the outcome: one rank unable to
// allocate fails the call on every rank instead of leaving the others waiting in a group for it.
int grow_staging(State& st, int64_t bytes) {
  int32_t ok = st.staging.ensure((size_t)std::max<int64_t>(bytes, 1)) == 0;
  if (env_i64("TIPS_STAGING_TEST_FAIL_RANK", -1) == st.rank) ok = 0;  // (tests: one rank short of memory)
  const std::string why = ok ? std::string() : last_error();
  TRY(order_after_replays(st));
  int32_t* d = nullptr;
  int rc = 0;
  if (hipMalloc(&d, sizeof(int32_t)) != hipSuccess ||
      hipMemcpyAsync(d, &ok, sizeof ok, hipMemcpyHostToDevice, st.comm_stream) != hipSuccess ||
      ncclAllReduce(d, d, 1, ncclInt32, ncclMin, st.comm, st.comm_stream) != ncclSuccess ||
      hipMemcpyAsync(&ok, d, sizeof ok, hipMemcpyDeviceToHost, st.comm_stream) != hipSuccess ||
      hipStreamSynchronize(st.comm_stream) != hipSuccess)
    rc = fail(TIPS_ERR_RCCL, "agreeing on the staging allocation failed");
  if (d) (void)hipFree(d);
  if (rc) return rc;
  if (!ok)
    return fail(TIPS_ERR_HIP, "staging of %lld bytes could not be allocated on some rank%s%s", (long long)bytes,
                why.empty() ? "" : ": ", why.c_str());
  return 0;
}

int run_plan(State& st, const Plan& pl, const char* in, char* out, hipStream_t user, int L = 1) {
  L = std::max(1, std::min(L, (int)pl.steps.size()));
  const size_t nsteps = pl.steps.size();
  void* const stg_before = st.staging.p;
  if ((size_t)std::max<int64_t>(pl.staging_bytes, 1) > st.staging.bytes) TRY(grow_staging(st, pl.staging_bytes));
  if (st.staging.p != stg_before && st.graphs) {  // graphs of the old staging can never replay again
    for (auto& kv : st.graphs->m) destroy_exec(st, kv.second.exec);
    st.graphs->m.clear();
  }
  TRY(st.recv_ev.ensure(nsteps));
  TRY(st.sum_ev.ensure(nsteps));
  char* base[3] = {(char*)in, out, (char*)st.staging.p};
  const bool eligible = L == 1 && graph_eligible(st, pl, user);
  bool key_new = false;
  if (eligible) {
    hipGraphExec_t exec = plan_graph(st, pl, base, false, &key_new);
    if (exec) return replay(st, exec, user);
  }
  if (L > 1) TRY(lanes_ensure(st, L));
  const int64_t waits_before = st.replay_host_waits;
  TRY(prologue(st, user, L));
  // this call's host wait may just have widened the replay limit (replays_mixed): its key counts as
  // seen, so its next call is captured instead of waiting once more
  if (L == 1 && !eligible && graph_eligible(st, pl, user)) (void)plan_graph(st, pl, base, true, &key_new);
  // A bucket that waits for a replay at an address never seen before cannot become a replay by
  // its next call. One shape doing that again and again (a buffer reallocated at a new address every
  // step) would wait on every call, and each wait stalls the host until the device has run the
  // replay: the host can no longer queue ahead. Then replays yield - every plan eager, no waits
  // (tips_graph_stats returns 3).
  if (st.replay_host_waits > waits_before && key_new &&
      ++st.fresh_waits[std::make_tuple(pl.algo, pl.K, pl.dtype, pl.n)] >= fresh_wait_limit()) {
    if (!st.replays_yield && getenv("TIPS_VERBOSE"))
      fprintf(stderr, "[tips] replays yield: a %lld-element bucket waited %d times at new addresses\n",
              (long long)pl.n, fresh_wait_limit());
    st.replays_yield = true;
  }
  TRY(issue_steps(st, pl, base, L));
  return epilogue(st, user, L);
}

int plan_allreduce(State& st, const Choice& c, const char* in, char* out, int64_t n, int dtype, hipStream_t user) {
  Plan pl;
  TRY(build_schedule_plan(c.algo, st.size, st.rank, n, dtype, c.depth > 0 ? c.depth : plan_depth(st.size, n, dtype), &pl));
  return run_plan(st, pl, in, out, user, c.lanes);
}

// ---------------------------------------------------------------------------
// TIPS_ALGO_TUNE: the schedule chosen by measurement, per (ranks, dtype, size class).

int size_class(int64_t bytes) {
  int c = 0;
  while (c < 62 && (int64_t(1) << c) < bytes) c++;
  return c;  // ceil(log2(bytes))
}

int run_choice(State& st, const Choice& c, const char* in, char* out, int64_t n, int dtype, hipStream_t s) {
  if (c.algo == TIPS_ALGO_PEER) return peer_allreduce(st, in, out, n, dtype, s);
  return plan_allreduce(st, c, in, out, n, dtype, s);
}

}  // namespace

// The candidates TIPS_ALGO_TUNE times for a bucket of n elements on p ranks, in the order it runs
// them (every rank the same): direct at the default depth K, at 1 and at 2K, ring at K and 2K.
// A chunk of 16 MiB or more is always pipelined (K >= 2): the fold of sub-chunk k then runs under
// the transfer of k + 1 (tests/test_plans.py), so depth 1 is a candidate only below that, where one
// launch per chunk can beat the per-launch cost of two.
std::vector<Choice> tune_candidates(int p, int64_t n, int dtype) {
  const int64_t es = tips::dtype_size(dtype);
  const int K = plan_depth(p, n, dtype);
  const int K2 = std::min(16, 2 * K);
  const int64_t chunk_bytes = chunk_of(n, p, kAlignBytes / es, 0).len() * es;
  const bool depth1 = K > 1 && chunk_bytes < kPipelineMinChunk;
  // TIPS_TUNE_LANES=1 adds two-lane candidates (consecutive steps' groups in flight together, for
  // when one communicator's point-to-point work does not fill the links). Off by default: on the
  // socket rehearsal the split communicator slowed every later call, chosen or not
  // (profiles/r02/lanes_rehearsal.jsonl); the 8-GPU bench's direct_l2 / ring_l2 lines measure xGMI.
  const bool lanes = env_i64("TIPS_TUNE_LANES", 0) != 0;
  std::vector<Choice> cand;
  if (p <= tips::kMaxSrcs) {
    cand.push_back({TIPS_ALGO_DIRECT, K, 1});
    if (depth1) cand.push_back({TIPS_ALGO_DIRECT, 1, 1});
    if (K < 16) cand.push_back({TIPS_ALGO_DIRECT, K2, 1});
    if (lanes && K > 1) cand.push_back({TIPS_ALGO_DIRECT, K, 2});
  }
  cand.push_back({TIPS_ALGO_RING, K, 1});
  if (K < 16) cand.push_back({TIPS_ALGO_RING, K2, 1});
  if (lanes) cand.push_back({TIPS_ALGO_RING, K, 2});
  if (p <= tips::kMaxSrcs && env_i64("TIPS_TUNE_PEER", 0)) cand.push_back({TIPS_ALGO_PEER, 0, 1});
  return cand;
}

namespace {

// Every rank runs the same candidates in the same order (collectives), on scratch copies of the
// call's input (the caller's buffers are not touched: in-place calls stay correct), times each with
// events on `user` (best of 2 runs of 2 back-to-back calls, after a warm-up), and the ranks agree
// on the slowest rank's time per candidate with one small ncclAllReduce(MAX): every rank then keeps
// the same fastest candidate.
int tune(State& st, const char* in, int64_t n, int dtype, hipStream_t user, Choice* best,
         std::vector<std::pair<Choice, double>>* timed) {
  const int p = st.size;
  const int64_t bytes = n * tips::dtype_size(dtype);
  std::vector<Choice> cand = tune_candidates(p, n, dtype);
  HIP_TRY(hipStreamSynchronize(user));
  void *sin = nullptr, *sout = nullptr;
  int rc = 0;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  std::vector<double> ms(cand.size(), 1e30);
  do {
    // scratch copies of the input: every rank learns whether every rank has them before any
    // candidate's transfers start (one rank out of memory must fail the call everywhere, not
    // leave the others waiting in a group for it)
    int32_t ok = hipMalloc(&sin, (size_t)bytes) == hipSuccess && hipMalloc(&sout, (size_t)bytes) == hipSuccess &&
                 hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess &&
                 hipMemcpyAsync(sin, in, (size_t)bytes, hipMemcpyDeviceToDevice, user) == hipSuccess;
    (void)hipGetLastError();
    if (env_i64("TIPS_TUNE_TEST_FAIL_RANK", -1) == st.rank) ok = 0;  // (tests: one rank short of memory)
    int32_t* dok = nullptr;
    if ((rc = order_after_replays(st)) != 0) break;
    if (hipMalloc(&dok, sizeof(int32_t)) != hipSuccess ||
        hipMemcpyAsync(dok, &ok, sizeof ok, hipMemcpyHostToDevice, st.comm_stream) != hipSuccess ||
        ncclAllReduce(dok, dok, 1, ncclInt32, ncclMin, st.comm, st.comm_stream) != ncclSuccess ||
        hipMemcpyAsync(&ok, dok, sizeof ok, hipMemcpyDeviceToHost, st.comm_stream) != hipSuccess ||
        hipStreamSynchronize(st.comm_stream) != hipSuccess)
      rc = fail(TIPS_ERR_RCCL, "tune: agreeing on the scratch buffers failed");
    if (dok) (void)hipFree(dok);
    if (rc) break;
    if (!ok) {
      rc = fail(TIPS_ERR_HIP, "tune: scratch buffers (2 x %lld bytes) could not be set up on some rank", (long long)bytes);
      break;
    }
    for (size_t c = 0; c < cand.size() && rc == 0; c++) {
      // a warm-up call, then twice kBackToBack calls queued back to back (as a training step issues
      // them: the next call's transfers behind the last one's, no host sync between), per call
      constexpr int kBackToBack = 2;
      if (rc == 0) rc = run_choice(st, cand[c], (const char*)sin, (char*)sout, n, dtype, user);
      for (int it = 0; it < 2 && rc == 0; it++) {
        if (hipEventRecord(e0, user) != hipSuccess) rc = fail(TIPS_ERR_HIP, "tune: event");
        for (int q = 0; q < kBackToBack && rc == 0; q++)
          rc = run_choice(st, cand[c], (const char*)sin, (char*)sout, n, dtype, user);
        if (rc == 0) {
          float t = 0;
          if (hipEventRecord(e1, user) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
              hipEventElapsedTime(&t, e0, e1) != hipSuccess)
            rc = fail(TIPS_ERR_HIP, "tune: timing");
          ms[c] = std::min(ms[c], (double)t / kBackToBack);
        }
      }
    }
    if (rc) break;
    // the slowest rank's time per candidate, on every rank
    double* d = nullptr;
    if (hipMalloc(&d, sizeof(double) * cand.size()) != hipSuccess) {
      rc = fail(TIPS_ERR_HIP, "tune: hipMalloc");
      break;
    }
    const size_t nb = sizeof(double) * cand.size();
    if ((rc = order_after_replays(st)) != 0) {
      (void)hipFree(d);
      break;
    }
    if (hipMemcpyAsync(d, ms.data(), nb, hipMemcpyHostToDevice, st.comm_stream) != hipSuccess ||
        ncclAllReduce(d, d, cand.size(), ncclFloat64, ncclMax, st.comm, st.comm_stream) != ncclSuccess ||
        hipMemcpyAsync(ms.data(), d, nb, hipMemcpyDeviceToHost, st.comm_stream) != hipSuccess ||
        hipStreamSynchronize(st.comm_stream) != hipSuccess)
      rc = fail(TIPS_ERR_RCCL, "tune: agreeing on the timings failed");
    (void)hipFree(d);
  } while (0);
  HIP_TRY(hipStreamSynchronize(user));
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (sin) (void)hipFree(sin);
  if (sout) (void)hipFree(sout);
  if (rc) return rc;
  size_t b = 0;
  for (size_t c = 1; c < cand.size(); c++)
    if (ms[c] < ms[b]) b = c;
  *best = cand[b];
  timed->clear();
  for (size_t c = 0; c < cand.size(); c++) timed->emplace_back(cand[c], ms[c]);
  if (getenv("TIPS_VERBOSE") && st.rank == 0) {
    fprintf(stderr, "[tips] tune p=%d bytes=%lld:", p, (long long)bytes);
    for (size_t c = 0; c < cand.size(); c++)
      fprintf(stderr, " algo%d/K%d/L%d=%.3fms", cand[c].algo, cand[c].depth, cand[c].lanes, ms[c]);
    fprintf(stderr, " -> algo%d/K%d/L%d\n", best->algo, best->depth, best->lanes);
  }
  return 0;
}

}  // namespace

// device-resident allreduce, caller holds st.mu
int allreduce_device(State& st, const void* in, void* out, int64_t n, int dtype, hipStream_t stream) {
  if (n == 0) return 0;
  const int64_t es = tips::dtype_size(dtype);
  const int algo = resolve_algo(st.algo, st.size, n * es);
  if (algo == TIPS_ALGO_RCCL) {
    TRY(ensure_comm(st));
    TRY(rccl_enter(st, stream));
    NCCL_TRY(ncclAllReduce(in, out, (size_t)n, nccl_type(dtype), ncclSum, st.comm, stream));
    return rccl_leave(st, stream);
  }
  if (st.size == 1) {  // MPI_Allreduce on one rank returns the input
    if (in != out) HIP_TRY(tips::launch_copy_buf(out, in, n * es, stream));
    return 0;
  }
  if (algo == TIPS_ALGO_PEER && st.size <= tips::kMaxSrcs)
    return peer_allreduce(st, (const char*)in, (char*)out, n, dtype, stream);
  TRY(ensure_comm(st));  // every other schedule moves its bytes over RCCL (no half-built group on failure)
  if (algo == TIPS_ALGO_TUNE) {
    const auto key = std::make_tuple(st.size, dtype, size_class(n * es));
    auto it = st.tuned.find(key);
    if (it == st.tuned.end()) {
      Choice best;
      std::vector<std::pair<Choice, double>> timed;
      TRY(tune(st, (const char*)in, n, dtype, stream, &best, &timed));
      it = st.tuned.emplace(key, best).first;
      st.tuned_ms[key] = std::move(timed);
    }
    return run_choice(st, it->second, (const char*)in, (char*)out, n, dtype, stream);
  }
  int a = algo;
  if (st.size > tips::kMaxSrcs && (a == TIPS_ALGO_DIRECT || a == TIPS_ALGO_ONESHOT || a == TIPS_ALGO_PEER))
    a = TIPS_ALGO_RING;
  if (a != TIPS_ALGO_DIRECT && a != TIPS_ALGO_ONESHOT) a = TIPS_ALGO_RING;
  // TIPS_LANES (same on every rank): transfer lanes for the explicitly chosen schedules
  const int lanes = (int)std::max<int64_t>(1, std::min<int64_t>(8, env_i64("TIPS_LANES", 1)));
  return plan_allreduce(st, Choice{a, 0, lanes}, (const char*)in, (char*)out, n, dtype, stream);
}

void lanes_release(State& st) {
  for (hipStream_t s : st.lane_stream) (void)hipStreamSynchronize(s);
  for (ncclComm_t c : st.lane_comm) (void)ncclCommDestroy(c);
  for (hipStream_t s : st.lane_stream) (void)hipStreamDestroy(s);
  st.lane_comm.clear();
  st.lane_stream.clear();
  st.lane_ev.release();
  st.xfer_ev.release();
}

int rccl_enter(State& st, hipStream_t s) {
  TRY(order_after_replays(st));
  for (size_t l = 0; l < st.lane_stream.size(); l++) TRY(join(st.comm_stream, st.lane_stream[l], st.lane_ev.ev[l + 1]));
  if (s != st.comm_stream) TRY(join(s, st.comm_stream, st.ev_rccl[0]));
  return 0;
}

int rccl_leave(State& st, hipStream_t s) {
  if (s != st.comm_stream) TRY(join(st.comm_stream, s, st.ev_rccl[1]));
  st.eager_pending = true;  // a replay waits for the comm stream, which now waits for this
  return 0;
}

void graphs_release(State& st) {
  if (st.graph_stream) (void)hipStreamSynchronize(st.graph_stream);
  if (st.graphs) {
    for (auto& kv : st.graphs->m)
      if (kv.second.exec) (void)hipGraphExecDestroy(kv.second.exec);
    delete st.graphs;
    st.graphs = nullptr;
  }
  st.graph_pending = st.eager_pending = false;
  st.graphs_captured = st.graphs_replayed = 0;
  st.replay_host_waits = st.replay_host_wait_ns = 0;
  st.replays_mixed = false;
  st.fresh_waits.clear();
  st.replays_yield = false;
}

#ifdef TIPS_DEV  // (development surface: libtips_hip_dev.so only, include/tips_hip_dev.h)
namespace {

// Peer transfers of the single-GPU simulator, batched per plan step: device-to-device
// copies, or (sim_transport 1) the same bytes as grouped ncclSend/ncclRecv pairs to this rank
// itself, so the RCCL p2p calls the real schedules make (byte counts, grouping, stream order)
// run on a 1-GPU box.
struct SimXfer {
  State& st;
  std::vector<std::tuple<void*, const void*, size_t>> ops;
  explicit SimXfer(State& s) : st(s) {}
  void add(void* dst, const void* src, int64_t bytes) {
    if (bytes > 0) ops.emplace_back(dst, src, (size_t)bytes);
  }
  int flush() {
    if (ops.empty()) return 0;
    if (st.sim_transport == 1) {
      NCCL_TRY(ncclGroupStart());
      for (auto& o : ops) {
        NCCL_TRY(ncclSend(std::get<1>(o), std::get<2>(o), ncclInt8, 0, st.comm, st.comm_stream));
        NCCL_TRY(ncclRecv(std::get<0>(o), std::get<2>(o), ncclInt8, 0, st.comm, st.comm_stream));
      }
      NCCL_TRY(ncclGroupEnd());
    } else {
      for (auto& o : ops)
        HIP_TRY(hipMemcpyAsync(std::get<0>(o), std::get<1>(o), std::get<2>(o), hipMemcpyDeviceToDevice, st.comm_stream));
    }
    ops.clear();
    return 0;
  }
};

int sim_prepare(State& st) {
  TRY(ensure_streams(st));
  if (st.sim_transport == 1) {
    if (!st.comm && st.size > 1) return fail(TIPS_ERR_UNSUPPORTED, "RCCL self-loop simulation needs a 1-rank setup");
    if (!st.comm) {
      if (st.size < 1) st.size = 1, st.rank = 0;
      TRY(ensure_comm(st));
    }
  }
  return 0;
}

// Runs the p ranks' plans on this GPU, step by step in lockstep. Step i's transfers pair the
// k-th send from r to q with the k-th receive on q from r in q's step i (what RCCL's grouped
// p2p does); a send or receive without its partner is reported as the deadlock it would be.
// All virtual ranks share the comm and compute streams, so every event wait of the real
// executor holds here too (with more ordering, never less).
int simulate_plans(State& st, std::vector<Plan>& plans, void* const* outs, const void* const* ins, int dtype,
                   hipStream_t user) {
  const int p = (int)plans.size();
  const size_t nsteps = plans[0].steps.size();
  for (auto& pl : plans)
    if (pl.steps.size() != nsteps) return fail(TIPS_ERR_INVALID_ARG, "plans of one schedule differ in step count");
  const int64_t stg = round_up(std::max<int64_t>(plans[0].staging_bytes, 1), 4096);
  TRY(st.staging.ensure((size_t)(stg * p)));
  TRY(st.recv_ev.ensure(nsteps));
  TRY(st.sum_ev.ensure(nsteps));
  auto base = [&](int r, int buf) -> char* {
    return buf == kBufIn ? (char*)ins[r] : buf == kBufOut ? (char*)outs[r] : (char*)st.staging.p + r * stg;
  };
  SimXfer xf(st);
  TRY(prologue(st, user));
  std::vector<char> has_sums(nsteps, 0);
  for (size_t i = 0; i < nsteps; i++) {
    bool sums = false;
    std::vector<int> waited;  // one shared event per earlier step covers every rank's sums of it
    for (int r = 0; r < p; r++) {
      const PStep& s = plans[r].steps[i];
      sums = sums || !s.sums.empty();
      if (s.wait_sum >= 0 && has_sums[s.wait_sum] &&
          std::find(waited.begin(), waited.end(), s.wait_sum) == waited.end()) {
        HIP_TRY(hipStreamWaitEvent(st.comm_stream, st.sum_ev.ev[s.wait_sum], 0));
        waited.push_back(s.wait_sum);
      }
    }
    for (int r = 0; r < p; r++) {
      std::vector<int> nth(p, 0);  // sends from r to q seen so far in this step
      for (const PXfer& x : plans[r].steps[i].xfers) {
        if (!x.send) continue;
        if (x.peer < 0 || x.peer >= p || x.peer == r) return fail(TIPS_ERR_INVALID_ARG, "plan: bad peer %d", x.peer);
        int seen = 0;
        const PXfer* match = nullptr;
        for (const PXfer& y : plans[x.peer].steps[i].xfers)
          if (!y.send && y.peer == r && seen++ == nth[x.peer]) {
            match = &y;
            break;
          }
        nth[x.peer]++;
        if (!match || match->bytes != x.bytes)
          return fail(TIPS_ERR_INVALID_ARG, "plan deadlock: step %zu, rank %d sends %lld B to %d without a matching receive",
                      i, r, (long long)x.bytes, x.peer);
        xf.add(base(x.peer, match->at.buf) + match->at.off, base(r, x.at.buf) + x.at.off, x.bytes);
      }
    }
    size_t nrecv = 0, nsend = 0;
    for (int r = 0; r < p; r++)
      for (const PXfer& x : plans[r].steps[i].xfers) (x.send ? nsend : nrecv)++;
    if (nrecv != nsend) return fail(TIPS_ERR_INVALID_ARG, "plan deadlock: step %zu has %zu receives for %zu sends", i, nrecv, nsend);
    TRY(xf.flush());
    if (sums) {
      HIP_TRY(hipEventRecord(st.recv_ev.ev[i], st.comm_stream));
      HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.recv_ev.ev[i], 0));
      for (int r = 0; r < p; r++) {
        char* b[3] = {base(r, kBufIn), base(r, kBufOut), base(r, kBufStaging)};
        for (const PSum& ps : plans[r].steps[i].sums) TRY(launch_psum(ps, b, dtype, st.comp_stream));
      }
      HIP_TRY(hipEventRecord(st.sum_ev.ev[i], st.comp_stream));
      has_sums[i] = 1;
    }
  }
  return epilogue(st, user);
}

int simulate(int algo, void* const* outs, const void* const* ins, int p, int64_t n, int dtype, void* stream) {
  TRY(check_dtype(dtype));
  const int pmax = algo == TIPS_ALGO_RING ? 64 : tips::kMaxSrcs;
  if (p < 1 || p > pmax || n < 0 || !outs || !ins) return fail(TIPS_ERR_INVALID_ARG, "bad simulate args");
  if (n == 0) return 0;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  TRY(sim_prepare(st));
  hipStream_t user = (hipStream_t)stream;
  if (p == 1) {
    if (outs[0] != ins[0])
      HIP_TRY(hipMemcpyAsync(outs[0], ins[0], (size_t)(n * tips::dtype_size(dtype)), hipMemcpyDeviceToDevice, user));
    return 0;
  }
  std::vector<Plan> plans(p);
  const int K = plan_depth(p, n, dtype);
  for (int r = 0; r < p; r++) TRY(build_schedule_plan(algo, p, r, n, dtype, K, &plans[r]));
  return simulate_plans(st, plans, outs, ins, dtype, user);
}

}  // namespace
#endif  // TIPS_DEV

}  // namespace rt
}  // namespace tips

using namespace tips::rt;

extern "C" {

int tips_chunk_bounds(int64_t count, int p, int dtype, int c, int64_t* begin, int64_t* end) {
  TRY(check_dtype(dtype));
  if (p < 1 || c < 0 || c >= p || count < 0 || !begin || !end) return fail(TIPS_ERR_INVALID_ARG, "bad chunk query");
  Range r = chunk_of(count, p, kAlignBytes / tips::dtype_size(dtype), c);
  *begin = r.b;
  *end = r.e;
  return 0;
}

int tips_schedule_shape(int64_t count, int p, int dtype, int* depth, int64_t* sub_elems) {
  TRY(check_dtype(dtype));
  if (p < 1 || count < 0 || !depth || !sub_elems) return fail(TIPS_ERR_INVALID_ARG, "bad schedule query");
  const int64_t es = tips::dtype_size(dtype), align = kAlignBytes / es;
  const Range c0 = chunk_of(count, p, align, 0);
  *depth = pipeline_depth(c0.len() * es);
  *sub_elems = sub_of(c0, *depth, align, 0).len();
  return 0;
}

int tips_tuned_choice(int64_t bytes, int* algo, int* depth) {
  if (bytes < 0 || !algo || !depth) return fail(TIPS_ERR_INVALID_ARG, "bad tuned-choice query");
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  for (const auto& kv : st.tuned)  // any dtype of this job's size class
    if (std::get<0>(kv.first) == st.size && std::get<2>(kv.first) == size_class(bytes)) {
      *algo = kv.second.algo;
      *depth = kv.second.depth;
      return 1;
    }
  return 0;
}

int tips_tuned_schedule(int64_t bytes, int* algo, int* depth, int* lanes) {
  if (!lanes) return fail(TIPS_ERR_INVALID_ARG, "bad tuned-schedule query");
  const int rc = tips_tuned_choice(bytes, algo, depth);
  if (rc != 1) return rc;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  *lanes = 1;
  for (const auto& kv : st.tuned)
    if (std::get<0>(kv.first) == st.size && std::get<2>(kv.first) == size_class(bytes)) {
      *lanes = kv.second.lanes;
      break;
    }
  return 1;
}

int tips_tuned_timings(int64_t bytes, int* algos, int* depths, int* lanes, double* ms, int cap) {
  if (bytes < 0 || cap < 0 || (cap > 0 && (!algos || !depths || !lanes || !ms)))
    return fail(TIPS_ERR_INVALID_ARG, "bad tuned-timings query");
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  for (const auto& kv : st.tuned_ms)  // any dtype of this job's size class, as tips_tuned_choice
    if (std::get<0>(kv.first) == st.size && std::get<2>(kv.first) == size_class(bytes)) {
      const int n = (int)kv.second.size();
      for (int i = 0; i < n && i < cap; i++) {
        algos[i] = kv.second[i].first.algo;
        depths[i] = kv.second[i].first.depth;
        lanes[i] = kv.second[i].first.lanes;
        ms[i] = kv.second[i].second;
      }
      return n;
    }
  return 0;
}

int tips_graph_stats(int64_t* captured, int64_t* replayed, int64_t* cached) {
  if (!captured || !replayed || !cached) return fail(TIPS_ERR_INVALID_ARG, "bad graph-stats query");
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  *captured = st.graphs_captured;
  *replayed = st.graphs_replayed;
  *cached = 0;
  if (st.graphs)
    for (const auto& kv : st.graphs->m) *cached += kv.second.exec != nullptr;
  if (st.graphs && st.graphs->off) return 1;
  const int64_t want = env_i64("TIPS_GRAPHS", 0);
  if (want <= 0 || (want == 1 && !graphs_supported())) return 2;
  return st.replays_yield ? 3 : 0;
}

int tips_replay_order_stats(int64_t* host_waits, int64_t* host_wait_ns) {
  if (!host_waits || !host_wait_ns) return fail(TIPS_ERR_INVALID_ARG, "bad replay-order query");
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  *host_waits = st.replay_host_waits;
  *host_wait_ns = st.replay_host_wait_ns;
  return 0;
}

#ifdef TIPS_DEV  // (development surface: libtips_hip_dev.so only, include/tips_hip_dev.h)
int tips_tune_candidates(int p, int64_t count, int dtype, int* algos, int* depths, int* lanes, int cap) {
  TRY(check_dtype(dtype));
  if (p < 2 || count < 0 || cap < 0 || (cap > 0 && (!algos || !depths || !lanes)))
    return fail(TIPS_ERR_INVALID_ARG, "bad tune-candidates query");
  const std::vector<Choice> c = tune_candidates(p, count, dtype);
  for (int i = 0; i < (int)c.size() && i < cap; i++) {
    algos[i] = c[i].algo;
    depths[i] = c[i].depth;
    lanes[i] = c[i].lanes;
  }
  return (int)c.size();
}

int64_t tips_schedule_plan(int algo, int p, int rank, int64_t count, int dtype, int depth, int64_t* out, int64_t cap) {
  TRY(check_dtype(dtype));
  if (cap < 0 || (cap > 0 && !out)) return fail(TIPS_ERR_INVALID_ARG, "bad plan buffer");
  Plan pl;
  TRY(build_schedule_plan(algo, p, rank, count, dtype, depth > 0 ? depth : plan_depth(p, count, dtype), &pl));
  std::vector<int64_t> w = {(int64_t)pl.steps.size(), pl.staging_bytes, pl.K};
  for (const PStep& s : pl.steps) {
    w.insert(w.end(), {(int64_t)s.wait_sum, (int64_t)s.xfers.size(), (int64_t)s.sums.size()});
    for (const PXfer& x : s.xfers) w.insert(w.end(), {(int64_t)x.send, (int64_t)x.peer, (int64_t)x.at.buf, x.at.off, x.bytes});
    for (const PSum& u : s.sums) {
      w.insert(w.end(), {(int64_t)u.dst.buf, u.dst.off, u.count, (int64_t)u.nsrc});
      for (int j = 0; j < u.nsrc; j++) w.insert(w.end(), {(int64_t)u.src[j].buf, u.src[j].off});
    }
  }
  if ((int64_t)w.size() <= cap) std::copy(w.begin(), w.end(), out);
  return (int64_t)w.size();
}
#endif  // TIPS_DEV

#ifdef TIPS_DEV  // (development surface: libtips_hip_dev.so only, include/tips_hip_dev.h)
// ---------------------------------------------------------------------------
// single-GPU schedule simulators (test harnesses): the plans of all p ranks, on one device

int tips_ring_simulate(void* const* outs, const void* const* ins, int p, int64_t n, int dtype, void* stream) {
  return simulate(TIPS_ALGO_RING, outs, ins, p, n, dtype, stream);
}

int tips_direct_simulate(void* const* outs, const void* const* ins, int p, int64_t n, int dtype, void* stream) {
  return simulate(TIPS_ALGO_DIRECT, outs, ins, p, n, dtype, stream);
}

int tips_oneshot_simulate(void* const* outs, const void* const* ins, int p, int64_t n, int dtype, void* stream) {
  return simulate(TIPS_ALGO_ONESHOT, outs, ins, p, n, dtype, stream);
}
#endif  // TIPS_DEV

}  // extern "C"
