// rt.h — internal state and helpers shared by the runtime's translation units
// (runtime.cc: lifecycle + data-path C-ABI; schedules.cc: ring / direct /
// simulators; fusion.cc; host_staging.cc; control.cc). Not part of the C-ABI.
#pragma once

#include <sched.h>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <thread>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#ifdef TIPS_DEV
#include "../../include/tips_hip_dev.h"
#else
#include "../../include/tips_hip.h"
#endif
#include "kernels.h"

namespace tips {
namespace rt {

using tips::CopyTile;

constexpr int64_t kAlignBytes = 256;  // chunk / bucket-slot alignment (dwordx4 + 128-B lines)
// chunks of at least this many bytes always run pipelined under TIPS_ALGO_TUNE (K >= 2 sub-chunks)
constexpr int64_t kPipelineMinChunk = (int64_t)16 << 20;
// host-staging piece: 16 MiB sits at the top of the measured pipeline curve (profiles/r01_pcie_probe.jsonl)
constexpr int64_t kHostPieceBytes = 16 << 20;

// Records the calling thread's last error (tips_last_error) and returns `code`.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
const std::string& last_error();

#define HIP_TRY(expr)                                                                                  \
  do {                                                                                                 \
    hipError_t e_ = (expr);                                                                            \
    if (e_ != hipSuccess) return fail(TIPS_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));    \
  } while (0)

#define NCCL_TRY(expr)                                                                                 \
  do {                                                                                                 \
    ncclResult_t r_ = (expr);                                                                          \
    if (r_ != ncclSuccess) return fail(TIPS_ERR_RCCL, "%s failed: %s", #expr, ncclGetErrorString(r_)); \
  } while (0)

#define TRY(expr)            \
  do {                       \
    int rc_ = (expr);        \
    if (rc_ != 0) return rc_; \
  } while (0)

int64_t env_i64(const char* name, int64_t dflt);
int env_first_int(const char* const* names, int dflt);
inline int64_t round_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }
inline int mod(int a, int p) { return ((a % p) + p) % p; }

// ---------------------------------------------------------------------------
// chunk / sub-chunk partition (shared by ring, direct and the simulators;
// restated by oracle_chunk_bounds in oracle/oracle.c)

struct Range {
  int64_t b, e;
  int64_t len() const { return e - b; }
};

inline Range chunk_of(int64_t n, int p, int64_t align, int c) {
  int64_t per = round_up((n + p - 1) / p, align);
  int64_t b = std::min((int64_t)c * per, n), e = std::min(b + per, n);
  return {b, e};
}

inline Range sub_of(Range ch, int K, int64_t align, int k) {
  int64_t per = round_up((ch.len() + K - 1) / K, align);
  int64_t b = std::min(ch.b + (int64_t)k * per, ch.e), e = std::min(b + per, ch.e);
  return {b, e};
}

// ---------------------------------------------------------------------------
// device buffers that only grow, and event pools

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t want, bool zero = false) {
    if (want <= bytes) return 0;
    if (p) {
      hipError_t e = hipFree(p);
      (void)e;
      p = nullptr;
      bytes = 0;
    }
    want = (size_t)round_up((int64_t)want, 1 << 20);
    HIP_TRY(hipMalloc(&p, want));
    if (zero) HIP_TRY(hipMemset(p, 0, want));
    bytes = want;
    return 0;
  }
  void release() {
    if (p) {
      hipError_t e = hipFree(p);
      (void)e;
    }
    p = nullptr;
    bytes = 0;
  }
};

struct EventPool {
  std::vector<hipEvent_t> ev;
  int ensure(size_t n) {
    while (ev.size() < n) {
      hipEvent_t e;
      HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      ev.push_back(e);
    }
    return 0;
  }
  void release() {
    for (auto e : ev) {
      hipError_t r = hipEventDestroy(e);
      (void)r;
    }
    ev.clear();
  }
};

// A schedule as the executor runs it: algorithm, pipeline depth (sub-chunks per chunk) and
// transfer lanes (RCCL communicators whose groups may be in flight together).
struct Choice {
  int algo = TIPS_ALGO_RING, depth = 0, lanes = 1;
};

struct PeerState;   // peer.cc
struct FusionCache;  // fusion.cc: layouts and resolved segment tables of recent tensor lists
struct PlanGraphs;   // schedules.cc: instantiated HIP graphs of recently replayed plans

// host_staging.cc: fork-join pool for the host copies: run(n, fn) calls fn(0..n-1) on the pool's threads and the
// caller's, and returns when all n are done. Jobs are claimed from one 64-bit ticket holding
// (generation << 32 | jobs << 16 | next index), so a thread still leaving run k can never claim a job
// of run k+1, nor one past run k's end: its compare-and-swap fails on the generation.
struct Piece {
  int64_t off, len;  // bytes of a fused host stream
};
std::vector<Piece> host_pieces(int64_t total, int64_t piece, int64_t first);

class HostPool {
 public:
  explicit HostPool(int nthreads);
  ~HostPool();
  void run(int njobs, const std::function<void(int)>& fn);
  int size() const { return (int)th_.size() + 1; }
  // the CPUs the worker threads run on from their next job on: `cpus` (a cpu_set_t), or nullptr
  // for the mask they started with (TIPS_HOST_BIND: the GPU's NUMA node)
  void set_affinity(const void* cpus);

 private:
  void worker(int k);  // k: the worker's index (its L3 share of the mask, TIPS_HOST_SPREAD)
  void grab(uint64_t gen);
  std::vector<unsigned char> mask_;  // guarded by m_: the wanted cpu_set_t bytes (empty: the start mask)
  std::atomic<uint64_t> mask_gen_{0};
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  std::atomic<uint64_t> ticket_{0};
  std::atomic<int> pending_{0};
  uint64_t gen_ = 0;  // guarded by m_ (workers wait on it)
  bool stop_ = false;
  // the same two, readable without m_: workers (and run's wait for its jobs) spin on them for up to
  // spin_ns_ before blocking (TIPS_HOST_SPIN_US)
  std::atomic<uint64_t> gen_pub_{0};
  std::atomic<bool> stop_pub_{false};
  int64_t spin_ns_ = 0;
};

struct State {
  std::mutex mu;
  bool initialized = false;
  int rank = -1, size = -1, device = -1;
  ncclComm_t comm = nullptr;
  hipStream_t comm_stream = nullptr, comp_stream = nullptr, io_stream = nullptr;
  hipStream_t h2d_stream = nullptr, d2h_stream = nullptr;  // host-memory pipeline (both PCIe directions)
  hipStream_t h2d_stream2 = nullptr;  // fused host lists: odd pieces' H2D (TIPS_HOST_H2D_STREAMS=2)
  EventPool pipe_ev;
  hipStream_t fuse_stream = nullptr, bucket_stream = nullptr;  // fusion: pack/unpack || bucket allreduce
  EventPool fuse_ev;
  // fusion.cc: the stream of the fused call in progress (its pack / unpack / table work) and the chain
  // that orders every fused call after the previous one: an event at the end of each call, on the
  // stream it ran on, which a call from another stream waits for first
  hipStream_t fuse_ws = nullptr, fuse_chain_stream = nullptr;
  hipEvent_t ev_fuse_chain = nullptr;
  hipEvent_t ev_fuse_table = nullptr;  // a table uploaded on fuse_stream: the work stream waits for it
  bool fuse_chain_valid = false;
  bool fuse_chain_lazy = false;  // the last call (tips_fused_pack_bucket) left its event unrecorded
  bool fuse_capturing = false;   // the call in progress is being captured into a graph (no chain)
  bool fuse_in_call = false;     // fuse_ws is set (it may be the legacy null stream, i.e. nullptr)
  int64_t fusion_threshold = 0;  // the fusion slots' size (2 slots of it in `fusion`)
  std::vector<void*> fusion_retired;  // earlier slots a captured graph may still pack into (freed at shutdown)
  // fusion.cc, one pack launch for a step's buckets: per bucket of the launch a workgroup counter
  // (device memory, reset by the kernel) and a signal word (hipMallocSignalMemory) its last workgroup
  // raises to the next value, which the bucket stream waits for (hipStreamWaitValue64)
  unsigned* pack_counters = nullptr;
  void* pack_done[8] = {};
  uint64_t pack_done_value[8] = {};
  int pack_signals = -1;  // -1 not tried yet, 0 unavailable (events per bucket), 1 ready
  hipEvent_t ev_start = nullptr, ev_done = nullptr, ev_comp_done = nullptr, ev_comp_prev = nullptr;
  EventPool recv_ev, sum_ev;
  DevBuf staging, host_in, host_out, fusion, small;
  DevBuf cast_scratch;  // fusion.cc, fused casts: a list's tensors of at least the threshold, in the wire type
  void* bounce_in = nullptr;  // page-locked kBounceBytes each (hipHostMalloc), for small pageable host tensors
  void* bounce_out = nullptr;
  HostPool* host_pool = nullptr;  // fused host tensors: pack / unpack threads
  void* hpin[2] = {};             // fused host tensors: page-locked piece slots, in and out
  size_t hpin_bytes = 0;
  int algo = TIPS_ALGO_AUTO;
  int sim_transport = 0;  // simulators: 0 = device copies, 1 = RCCL send/recv to self
  uint64_t peer_key = 0;      // names the node-local control block of the peer schedule (hash of the unique id)
  PeerState* peer = nullptr;  // peer schedule: IPC workspaces + shared-memory barrier, created on first use
  FusionCache* fusion_cache = nullptr;  // created on first use
  // TIPS_ALGO_TUNE: (ranks, dtype, size class) -> schedule, the same on every rank
  std::map<std::tuple<int, int, int>, Choice> tuned;
  // ... and every candidate the tuner timed for it, with the slowest rank's ms per call
  std::map<std::tuple<int, int, int>, std::vector<std::pair<Choice, double>>> tuned_ms;
  // transfer lanes beyond the comm stream (TIPS_LANES, or tuned): RCCL communicators split from
  // `comm`, each with its own stream at the comm stream's priority; a plan's step i moves its
  // bytes on lane i % L, so the groups of consecutive steps can be in flight together
  std::vector<ncclComm_t> lane_comm;
  std::vector<hipStream_t> lane_stream;
  EventPool lane_ev, xfer_ev;
  // schedules.cc, TIPS_GRAPHS: a plan called again on the same buffers is captured once into a HIP
  // graph and then replayed with one launch on graph_stream, which joins the caller both ways
  hipStream_t graph_stream = nullptr;
  hipEvent_t ev_graph[5] = {};  // replay joins: caller in, comm in, comp in, caller out, eager after replays
  hipEvent_t ev_rccl[2] = {};   // rccl_enter / rccl_leave
  PlanGraphs* graphs = nullptr;
  bool graph_pending = false;  // a replay may still run on graph_stream: eager plan work waits for it
  bool eager_pending = false;  // eager plan work was queued on comm / comp since the last replay
  int64_t graphs_captured = 0, graphs_replayed = 0;
  // order_after_replays' host waits (eager RCCL work issued while a replay was pending) and their time
  int64_t replay_host_waits = 0, replay_host_wait_ns = 0;
  // an eager plan followed a replay: larger plans become replayable too (graph_eligible)
  bool replays_mixed = false;
  // host waits of eager plans whose graph key was new (a bucket at an address never seen before),
  // per plan shape (algo, K, dtype, count); at kFreshWaitLimit for one shape, replays yield: every
  // plan runs eagerly, so no eager call waits on the host again (schedules.cc run_plan)
  std::map<std::tuple<int, int, int, int64_t>, int> fresh_waits;
  bool replays_yield = false;
};

State& S();

int ensure_streams(State& st);
ncclDataType_t nccl_type(int dtype);
int pipeline_depth(int64_t chunk_bytes);
int join(hipStream_t waiter, hipStream_t src, hipEvent_t ev);  // waiter waits for all work queued on src
bool is_device_ptr(const void* p);
bool is_pinned_host(const void* p, int64_t bytes);
int check_dtype(int dtype);
int set_device(State& st);
int resolve_algo(int algo, int p, int64_t bytes);
// The peer transport is selected (tips_set_algorithm or TIPS_ALGO=peer) and can serve this job:
// the broadcast / allgatherv / record exchange then go over the IPC workspaces, not RCCL.
inline bool peer_selected(const State& st) {
  return st.size > 1 && st.size <= tips::kMaxSrcs && resolve_algo(st.algo, st.size, 0) == TIPS_ALGO_PEER;
}
int ensure_comm(State& st);
void rccl_env_defaults();  // before any ncclCommInitRank of ours

// schedules.cc: device-resident allreduce, caller holds st.mu
int allreduce_device(State& st, const void* in, void* out, int64_t n, int dtype, hipStream_t stream);
// the candidates TIPS_ALGO_TUNE times for a bucket of n elements on p ranks, in its order (schedules.cc)
std::vector<Choice> tune_candidates(int p, int64_t n, int dtype);
void graphs_release(State& st);  // schedules.cc (shutdown, before the communicator goes)
// schedules.cc: an RCCL operation on `comm` issued outside a plan (a control-plane collective, the
// TIPS_ALGO_RCCL comparison) goes on stream `s` between these two calls: after everything queued
// for the communicator (the comm stream, whose prologues also wait for the transfer lanes and the
// replayed plans), and before everything queued for it later. Two RCCL kernels of one
// communicator then never run at the same time, whatever streams the callers use.
int rccl_enter(State& st, hipStream_t s);
int rccl_leave(State& st, hipStream_t s);
void lanes_release(State& st);   // schedules.cc (shutdown: the split communicators and their streams)
// peer.cc: allreduce over IPC-mapped peer memory (1 < p <= kMaxSrcs, one node), caller holds st.mu
int peer_allreduce(State& st, const char* in, char* out, int64_t n, int dtype, hipStream_t stream);
void peer_release(State& st);  // collective (shutdown)
// peer.cc: broadcast / allgatherv over the same workspaces (byte counts; displ = byte offsets in out)
int peer_broadcast(State& st, const char* in, char* out, int64_t bytes, int root, hipStream_t stream);
int peer_allgatherv(State& st, const char* in, char* out, const int64_t* bytes, const int64_t* displ, hipStream_t stream);
// host_staging.cc: host-resident allreduce over pipelined pieces, caller holds st.mu
int allreduce_host_pipelined(State& st, const char* in, char* out, int64_t n, int dtype);
// host_staging.cc: many host tensors in one flat stream of page-locked pieces (pack by host threads,
// H2D -> allreduce -> D2H per piece, unpack into every out - or, with `flat`, the sums into one host
// buffer of fused_layout's layout); returns when they are written. Caller holds st.mu.
int fused_allreduce_host(State& st, const struct BatchItem* items, int n, int dtype, char* flat);
void host_release(State& st);  // (shutdown: the pool and the page-locked pieces)
// fusion.cc: allreduce n same-dtype device tensors, in[i] -> out[i] (in == out allowed), packed
// into buckets of at most the fusion threshold: pack -> one allreduce per bucket -> unpack.
// Stream-ordered after `stream` and before its later work; all device work runs on the fusion
// streams, so calls from different streams never share a bucket unordered. Caller holds st.mu.
struct BatchItem {
  const void* in;
  void* out;
  int64_t count;
};
int fused_allreduce(State& st, const BatchItem* items, int n, int dtype, hipStream_t stream);
// The same into one flat output laid out as the buckets (fused_layout's offsets): pack(b) straight
// into the flat buffer, allreduce there in place; no slot, no unpack. Caller holds st.mu.
int fused_allreduce_flat(State& st, const BatchItem* items, int n, int dtype, void* flat, hipStream_t stream);
int64_t fused_layout(const int64_t* counts, int n, int dtype, int64_t* offsets);  // flat bytes; pure host
int fusion_stats(State& st, int64_t* v);  // layouts built, layout hits, tables built, table hits
int64_t fusion_threshold_bytes();
// fusion.cc: Compression.fp16 fused into the buckets - n f32 device tensors in[i] -> out[i]
// (in == out allowed) reduced in `wire` (TIPS_FLOAT16 / TIPS_BFLOAT16): cast while packed (RNE),
// each bucket allreduced in the wire type, cast back while unpacked. One rank: the round trip.
int fused_allreduce_cast(State& st, const BatchItem* items, int n, int wire, hipStream_t stream);
void fusion_release(State& st);  // (shutdown)
// The CPUs this process may run on, as the thread that loaded the library saw them: the base of
// every binding the library makes. (A thread's own mask is not: the negotiation thread is pinned to
// one L3, and a pool it starts, or a mask computed on it, would inherit that.)
const cpu_set_t& process_cpus();
void pack_signals_release(State& st);  // fusion.cc: the merged pack's counters and signal words
// control.cc: ConstructResponseMessage's rules over p request records (TIPS_REQUEST_WORDS each)
int check_records(const int64_t* t, int p);
// negotiate.cc: stop the negotiation thread (collective; call without holding st.mu)
int negotiation_stop();
// negotiate.cc: a synchronous collective entry point calls this first (without holding st.mu).
// While this rank's negotiation runs, the call is routed through it - announced as a request of
// `type` with the given dtype / shape / root, its `body` (the entry point itself) run on the
// negotiation thread in rank 0's order - and true is returned with *rc = the body's status. False:
// run directly (no negotiation, or already on the negotiation thread).
bool route_collective(int type, int dtype, const int64_t* shape, int ndim, int root, const std::function<int()>& body,
                      int* rc);
// Whether the calling thread is a negotiation thread (named requests and routed calls execute there)
bool on_negotiation_thread();

// ---------------------------------------------------------------------------
// host staging: the reference's ops work on host (TF CPU) tensors (ops.cc:88-90)

// Small pageable host tensors go through a page-locked bounce pair: a copy
// from pageable memory is a synchronous, high-latency staged transfer inside
// the HIP runtime, while a page-locked one is a plain DMA.
constexpr size_t kBounceBytes = 256 << 10;
int ensure_bounce(State& st);  // host_staging.cc

// Runs enqueue(dev_in, dev_out, stream). Device pointers: on the caller's
// stream, asynchronous. Host pointers: staged through HBM on the io stream and
// synchronous on return. Caller holds st.mu.
template <class F>
int run_staged(State& st, const void* in, size_t in_bytes, void* out, size_t out_bytes, hipStream_t user, F&& enqueue) {
  const bool dout = is_device_ptr(out);
  const bool din = in_bytes == 0 ? dout : is_device_ptr(in);
  if (din != dout) return fail(TIPS_ERR_INVALID_ARG, "in and out must both be device or both be host memory");
  if (dout) return enqueue(in, out, user);
  TRY(st.host_in.ensure(std::max<size_t>(in_bytes, 1)));
  TRY(st.host_out.ensure(std::max<size_t>(out_bytes, 1)));
  const bool bounce_in = in_bytes > 0 && in_bytes <= kBounceBytes && !is_pinned_host(in, (int64_t)in_bytes);
  const bool bounce_out = out_bytes > 0 && out_bytes <= kBounceBytes && !is_pinned_host(out, (int64_t)out_bytes);
  if (bounce_in || bounce_out) TRY(ensure_bounce(st));
  if (bounce_in) memcpy(st.bounce_in, in, in_bytes);
  if (in_bytes)
    HIP_TRY(hipMemcpyAsync(st.host_in.p, bounce_in ? st.bounce_in : in, in_bytes, hipMemcpyHostToDevice, st.io_stream));
  TRY(enqueue(st.host_in.p, st.host_out.p, st.io_stream));
  if (out_bytes)
    HIP_TRY(hipMemcpyAsync(bounce_out ? st.bounce_out : out, st.host_out.p, out_bytes, hipMemcpyDeviceToHost,
                           st.io_stream));
  HIP_TRY(hipStreamSynchronize(st.io_stream));
  if (bounce_out) memcpy(out, st.bounce_out, out_bytes);
  return 0;
}

}  // namespace rt
}  // namespace tips
