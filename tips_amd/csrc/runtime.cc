// runtime.cc — host runtime and C-ABI of libtips_hip.so.
//
// Replaces, for the allreduce-SUM path of Superjomn/TiPS:
//   tips/core/operations.{h,cc}           lifecycle C-ABI (tips_init/shutdown/size/rank)
//   tips/core/collective/utils.h:52-67    AllreduceCpu<T> -> tips_allreduce
//   tips/core/collective/coordinator.cc   negotiation: with one process per GPU and
//                                         stream-ordered calls there is nothing to
//                                         negotiate per tensor (DESIGN.md §Control plane)
//   tips/core/mpi/tips_mpi.h:13-55        dtype traits -> RCCL byte transfers + dtype enum
// The data moves over RCCL point-to-point (xGMI) and is summed by the HIP
// kernels of kernels.hip. One comm stream carries every RCCL call of a rank
// (one ordered channel, as the reference's single MPI_COMM_WORLD); sums run on
// a separate compute stream so sub-chunk k+1's transfer overlaps sub-chunk k's sum.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <thread>
#include <condition_variable>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "../../include/tips_hip.h"
#include "kernels.h"

namespace tips {
int bootstrap_exchange(int rank, int size, const char* host, int port, void* id, int id_bytes, int timeout_s,
                       std::string* err);
}

namespace {

using tips::CopyTile;

constexpr int64_t kAlignBytes = 256;  // chunk / bucket-slot alignment (dwordx4 + 128-B lines)

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  if (getenv("TIPS_VERBOSE")) fprintf(stderr, "[tips] error %d: %s\n", code, buf);
  return code;
}

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

int64_t env_i64(const char* name, int64_t dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  return strtoll(v, nullptr, 10);
}

int env_first_int(const char* const* names, int dflt) {
  for (int i = 0; names[i]; i++) {
    const char* v = getenv(names[i]);
    if (v && *v) return atoi(v);
  }
  return dflt;
}

int64_t round_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }
int mod(int a, int p) { return ((a % p) + p) % p; }

// ---------------------------------------------------------------------------
// chunk / sub-chunk partition (shared by ring, direct and the simulators;
// restated by oracle_chunk_bounds in oracle/oracle.c)

struct Range {
  int64_t b, e;
  int64_t len() const { return e - b; }
};

Range chunk_of(int64_t n, int p, int64_t align, int c) {
  int64_t per = round_up((n + p - 1) / p, align);
  int64_t b = std::min((int64_t)c * per, n), e = std::min(b + per, n);
  return {b, e};
}

Range sub_of(Range ch, int K, int64_t align, int k) {
  int64_t per = round_up((ch.len() + K - 1) / K, align);
  int64_t b = std::min(ch.b + (int64_t)k * per, ch.e), e = std::min(b + per, ch.e);
  return {b, e};
}

// ---------------------------------------------------------------------------
// device buffers that only grow

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

// fusion plan: cached per (dtype, tensor list)
struct FusionBucket {
  char* buf = nullptr;        // the fusion slot this bucket packs into (slot b % 2)
  int64_t bytes = 0;          // padded bucket size
  int ntiles = 0;
  CopyTile* pack = nullptr;   // device descriptor arrays
  CopyTile* unpack = nullptr;
  std::vector<int> direct;    // tensors too large to fuse: allreduced in place
};
struct FusionPlan {
  int dtype;
  std::vector<void*> ptrs;
  std::vector<int64_t> counts;
  std::vector<FusionBucket> buckets;
  std::vector<int> unfused;  // indices allreduced in place
};

struct State {
  std::mutex mu;
  bool initialized = false;
  int rank = -1, size = -1, device = -1;
  ncclComm_t comm = nullptr;
  hipStream_t comm_stream = nullptr, comp_stream = nullptr, io_stream = nullptr;
  hipStream_t h2d_stream = nullptr, d2h_stream = nullptr;  // host-memory pipeline (both PCIe directions)
  EventPool pipe_ev;
  hipStream_t fuse_stream = nullptr, bucket_stream = nullptr;  // fusion: pack/unpack || bucket allreduce
  EventPool fuse_ev;
  int64_t fusion_threshold = 0;  // the fusion slots' size; plans hold addresses into them
  hipEvent_t ev_start = nullptr, ev_done = nullptr, ev_comp_done = nullptr;
  EventPool recv_ev, sum_ev;
  DevBuf staging, host_in, host_out, fusion, small;
  int algo = TIPS_ALGO_AUTO;
  int sim_transport = 0;  // simulators: 0 = device copies, 1 = RCCL send/recv to self
  std::unordered_map<uint64_t, FusionPlan> plans;
};

State& S() {
  static State* s = new State();  // never destroyed: safe at exit
  return *s;
}

int ensure_streams(State& st) {
  if (!st.comm_stream) HIP_TRY(hipStreamCreateWithFlags(&st.comm_stream, hipStreamNonBlocking));
  if (!st.comp_stream) HIP_TRY(hipStreamCreateWithFlags(&st.comp_stream, hipStreamNonBlocking));
  if (!st.io_stream) HIP_TRY(hipStreamCreateWithFlags(&st.io_stream, hipStreamNonBlocking));
  if (!st.h2d_stream) HIP_TRY(hipStreamCreateWithFlags(&st.h2d_stream, hipStreamNonBlocking));
  if (!st.d2h_stream) HIP_TRY(hipStreamCreateWithFlags(&st.d2h_stream, hipStreamNonBlocking));
  if (!st.fuse_stream) HIP_TRY(hipStreamCreateWithFlags(&st.fuse_stream, hipStreamNonBlocking));
  if (!st.bucket_stream) HIP_TRY(hipStreamCreateWithFlags(&st.bucket_stream, hipStreamNonBlocking));
  if (!st.ev_start) HIP_TRY(hipEventCreateWithFlags(&st.ev_start, hipEventDisableTiming));
  if (!st.ev_done) HIP_TRY(hipEventCreateWithFlags(&st.ev_done, hipEventDisableTiming));
  if (!st.ev_comp_done) HIP_TRY(hipEventCreateWithFlags(&st.ev_comp_done, hipEventDisableTiming));
  return 0;
}

ncclDataType_t nccl_type(int dtype) {
  switch (dtype) {
    case TIPS_FLOAT32: return ncclFloat32;
    case TIPS_FLOAT64: return ncclFloat64;
    case TIPS_INT32: return ncclInt32;
    case TIPS_INT64: return ncclInt64;
    case TIPS_FLOAT16: return ncclFloat16;
    case TIPS_BFLOAT16: return ncclBfloat16;
    default: return ncclInt8;
  }
}

int pipeline_depth(int64_t chunk_bytes) {
  int64_t kmax = std::max<int64_t>(1, env_i64("TIPS_PIPELINE_DEPTH", 4));
  int64_t min_sub = std::max<int64_t>(kAlignBytes, env_i64("TIPS_MIN_SUBCHUNK_BYTES", 8 << 20));
  int64_t k = (chunk_bytes + min_sub - 1) / min_sub;
  return (int)std::max<int64_t>(1, std::min(k, kmax));
}

// The sum kernel launch used by every schedule (ring step: out = local + received).
int sum2(void* dst, const void* a, const void* b, int64_t n, int dtype, hipStream_t s) {
  HIP_TRY(tips::launch_sum2(dst, a, b, n, dtype, s));
  return 0;
}

// Join: `waiter` waits for all work queued so far on `src`.
int join(hipStream_t waiter, hipStream_t src, hipEvent_t ev) {
  HIP_TRY(hipEventRecord(ev, src));
  HIP_TRY(hipStreamWaitEvent(waiter, ev, 0));
  return 0;
}

// ---------------------------------------------------------------------------
// Ring allreduce over RCCL send/recv. Own rank only.

int ring_allreduce(State& st, const char* in, char* out, int64_t n, int dtype, hipStream_t user) {
  const int p = st.size, r = st.rank, next = mod(r + 1, p), prev = mod(r - 1, p);
  const int64_t es = tips::dtype_size(dtype), align = kAlignBytes / es;
  const int64_t max_chunk = chunk_of(n, p, align, 0).len();
  const int K = pipeline_depth(max_chunk * es);
  TRY(st.staging.ensure((size_t)(2 * max_chunk * es)));
  TRY(st.recv_ev.ensure(2 * K));
  TRY(st.sum_ev.ensure(2 * K));
  char* stg[2] = {(char*)st.staging.p, (char*)st.staging.p + max_chunk * es};
  TRY(join(st.comm_stream, user, st.ev_start));
  HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.ev_start, 0));

  // reduce-scatter: at step s send chunk (r-s), receive chunk (r-s-1) and add it in
  for (int s = 0; s < p - 1; s++) {
    const Range sc = chunk_of(n, p, align, mod(r - s, p)), rc = chunk_of(n, p, align, mod(r - s - 1, p));
    const char* src = (s == 0) ? in : out;
    for (int k = 0; k < K; k++) {
      const Range ss = sub_of(sc, K, align, k), rs = sub_of(rc, K, align, k);
      if (s > 0) HIP_TRY(hipStreamWaitEvent(st.comm_stream, st.sum_ev.ev[((s - 1) & 1) * K + k], 0));
      char* land = stg[s & 1] + (rs.b - rc.b) * es;
      if (ss.len() > 0 || rs.len() > 0) {
        NCCL_TRY(ncclGroupStart());
        if (ss.len() > 0) NCCL_TRY(ncclSend(src + ss.b * es, ss.len() * es, ncclInt8, next, st.comm, st.comm_stream));
        if (rs.len() > 0) NCCL_TRY(ncclRecv(land, rs.len() * es, ncclInt8, prev, st.comm, st.comm_stream));
        NCCL_TRY(ncclGroupEnd());
      }
      hipEvent_t rev = st.recv_ev.ev[(s & 1) * K + k];
      HIP_TRY(hipEventRecord(rev, st.comm_stream));
      HIP_TRY(hipStreamWaitEvent(st.comp_stream, rev, 0));
      TRY(sum2(out + rs.b * es, in + rs.b * es, land, rs.len(), dtype, st.comp_stream));
      HIP_TRY(hipEventRecord(st.sum_ev.ev[(s & 1) * K + k], st.comp_stream));
    }
  }
  // allgather: rank r owns chunk (r+1); at step s forward chunk (r+1-s), receive chunk (r-s)
  for (int s = 0; s < p - 1; s++) {
    const Range sc = chunk_of(n, p, align, mod(r + 1 - s, p)), rc = chunk_of(n, p, align, mod(r - s, p));
    for (int k = 0; k < K; k++) {
      const Range ss = sub_of(sc, K, align, k), rs = sub_of(rc, K, align, k);
      if (s == 0) HIP_TRY(hipStreamWaitEvent(st.comm_stream, st.sum_ev.ev[((p - 2) & 1) * K + k], 0));
      if (ss.len() > 0 || rs.len() > 0) {
        NCCL_TRY(ncclGroupStart());
        if (ss.len() > 0) NCCL_TRY(ncclSend(out + ss.b * es, ss.len() * es, ncclInt8, next, st.comm, st.comm_stream));
        if (rs.len() > 0) NCCL_TRY(ncclRecv(out + rs.b * es, rs.len() * es, ncclInt8, prev, st.comm, st.comm_stream));
        NCCL_TRY(ncclGroupEnd());
      }
    }
  }
  TRY(join(user, st.comm_stream, st.ev_done));
  TRY(join(user, st.comp_stream, st.ev_comp_done));
  return 0;
}

// ---------------------------------------------------------------------------
// Direct (all-pairs) allreduce: rank r owns chunk r. Every
// peer's slice of chunk r arrives over its own xGMI link at once; one p-input
// kernel folds them in rank order; then chunk r goes to every peer at once.

int direct_allreduce(State& st, const char* in, char* out, int64_t n, int dtype, hipStream_t user) {
  const int p = st.size, r = st.rank;
  const int64_t es = tips::dtype_size(dtype), align = kAlignBytes / es;
  const int64_t max_chunk = chunk_of(n, p, align, 0).len();
  const int K = pipeline_depth(max_chunk * es);
  TRY(st.staging.ensure((size_t)((p - 1) * max_chunk * es)));
  TRY(st.recv_ev.ensure(K));
  TRY(st.sum_ev.ensure(K));
  auto slot = [&](int j) { return (char*)st.staging.p + (int64_t)(j < r ? j : j - 1) * max_chunk * es; };
  const Range mine = chunk_of(n, p, align, r);
  TRY(join(st.comm_stream, user, st.ev_start));
  HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.ev_start, 0));
  for (int k = 0; k < K; k++) {
    const Range ms = sub_of(mine, K, align, k);
    NCCL_TRY(ncclGroupStart());
    for (int d = 1; d < p; d++) {
      const int to = mod(r + d, p), from = mod(r - d, p);
      const Range ts = sub_of(chunk_of(n, p, align, to), K, align, k);
      if (ts.len() > 0) NCCL_TRY(ncclSend(in + ts.b * es, ts.len() * es, ncclInt8, to, st.comm, st.comm_stream));
      if (ms.len() > 0)
        NCCL_TRY(ncclRecv(slot(from) + (ms.b - mine.b) * es, ms.len() * es, ncclInt8, from, st.comm, st.comm_stream));
    }
    NCCL_TRY(ncclGroupEnd());
    HIP_TRY(hipEventRecord(st.recv_ev.ev[k], st.comm_stream));
    HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.recv_ev.ev[k], 0));
    const void* srcs[tips::kMaxSrcs];
    for (int j = 0; j < p; j++) srcs[j] = (j == r) ? (const void*)(in + ms.b * es) : slot(j) + (ms.b - mine.b) * es;
    HIP_TRY(tips::launch_multi_sum(out + ms.b * es, srcs, p, ms.len(), dtype, st.comp_stream));
    HIP_TRY(hipEventRecord(st.sum_ev.ev[k], st.comp_stream));
  }
  for (int k = 0; k < K; k++) {
    const Range ms = sub_of(mine, K, align, k);
    HIP_TRY(hipStreamWaitEvent(st.comm_stream, st.sum_ev.ev[k], 0));
    NCCL_TRY(ncclGroupStart());
    for (int d = 1; d < p; d++) {
      const int to = mod(r + d, p), from = mod(r - d, p);
      const Range fs = sub_of(chunk_of(n, p, align, from), K, align, k);
      if (ms.len() > 0) NCCL_TRY(ncclSend(out + ms.b * es, ms.len() * es, ncclInt8, to, st.comm, st.comm_stream));
      if (fs.len() > 0) NCCL_TRY(ncclRecv(out + fs.b * es, fs.len() * es, ncclInt8, from, st.comm, st.comm_stream));
    }
    NCCL_TRY(ncclGroupEnd());
  }
  TRY(join(user, st.comm_stream, st.ev_done));
  TRY(join(user, st.comp_stream, st.ev_comp_done));
  return 0;
}

int resolve_algo(int algo, int p) {
  if (algo != TIPS_ALGO_AUTO) return algo;
  const char* e = getenv("TIPS_ALGO");
  if (e && *e) {
    if (!strcmp(e, "ring")) return TIPS_ALGO_RING;
    if (!strcmp(e, "direct")) return TIPS_ALGO_DIRECT;
    if (!strcmp(e, "rccl")) return TIPS_ALGO_RCCL;
  }
  return p <= 2 ? TIPS_ALGO_RING : TIPS_ALGO_DIRECT;
}

int ensure_comm(State& st) {
  if (st.comm) return 0;
  if (st.size != 1) return fail(TIPS_ERR_NOT_INITIALIZED, "no RCCL communicator");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  NCCL_TRY(ncclCommInitRank(&st.comm, 1, id, 0));
  return 0;
}

// device-resident allreduce, caller holds st.mu
int allreduce_device(State& st, const void* in, void* out, int64_t n, int dtype, hipStream_t stream) {
  if (n == 0) return 0;
  const int64_t es = tips::dtype_size(dtype);
  const int algo = resolve_algo(st.algo, st.size);
  if (algo == TIPS_ALGO_RCCL) {
    TRY(ensure_comm(st));
    NCCL_TRY(ncclAllReduce(in, out, (size_t)n, nccl_type(dtype), ncclSum, st.comm, stream));
    return 0;
  }
  if (st.size == 1) {  // MPI_Allreduce on one rank returns the input
    if (in != out) HIP_TRY(hipMemcpyAsync(out, in, (size_t)(n * es), hipMemcpyDeviceToDevice, stream));
    return 0;
  }
  if (st.size > tips::kMaxSrcs && algo == TIPS_ALGO_DIRECT)
    return ring_allreduce(st, (const char*)in, (char*)out, n, dtype, stream);
  if (algo == TIPS_ALGO_DIRECT) return direct_allreduce(st, (const char*)in, (char*)out, n, dtype, stream);
  return ring_allreduce(st, (const char*)in, (char*)out, n, dtype, stream);
}

bool is_device_ptr(const void* p) {
  hipPointerAttribute_t a;
  hipError_t e = hipPointerGetAttributes(&a, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged || a.isManaged;
}

int check_dtype(int dtype) {
  if (tips::dtype_size(dtype) == 0) return fail(TIPS_ERR_INVALID_ARG, "unsupported dtype %d", dtype);
  return 0;
}

int set_device(State& st) {
  if (st.device >= 0) HIP_TRY(hipSetDevice(st.device));
  return 0;
}

// ---------------------------------------------------------------------------
// host staging: the reference's ops work on host (TF CPU) tensors (ops.cc:88-90)

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
  if (in_bytes) HIP_TRY(hipMemcpyAsync(st.host_in.p, in, in_bytes, hipMemcpyHostToDevice, st.io_stream));
  TRY(enqueue(st.host_in.p, st.host_out.p, st.io_stream));
  if (out_bytes) HIP_TRY(hipMemcpyAsync(out, st.host_out.p, out_bytes, hipMemcpyDeviceToHost, st.io_stream));
  HIP_TRY(hipStreamSynchronize(st.io_stream));
  return 0;
}

// Host-resident allreduce, pipelined over pieces so both PCIe directions and
// the device work overlap: H2D of piece i+1 (h2d stream) || allreduce of piece
// i (io stream) || D2H of piece i-1 (d2h stream). Each piece is a complete
// allreduce (same piece boundaries on every rank). A second host thread
// issues the D2H copies, because a copy from/to pageable memory blocks the
// thread that issues it. Caller holds st.mu; returns when `out` is written.
int allreduce_host_pipelined(State& st, const char* in, char* out, int64_t n, int dtype) {
  const int64_t es = tips::dtype_size(dtype);
  const int64_t piece =
      round_up(std::max<int64_t>(kAlignBytes, env_i64("TIPS_HOST_PIECE_BYTES", 32 << 20)), kAlignBytes) / es;
  const int np = (int)((n + piece - 1) / piece);
  TRY(st.host_in.ensure((size_t)(n * es)));
  TRY(st.host_out.ensure((size_t)(n * es)));
  TRY(st.pipe_ev.ensure(2 * (size_t)np));
  char* din = (char*)st.host_in.p;
  char* dout = (char*)st.host_out.p;
  std::mutex m;
  std::condition_variable cv;
  int issued = 0;
  bool abort = false;
  std::string drain_err;
  const int device = st.device;
  std::thread drain([&] {
    if (device >= 0) (void)hipSetDevice(device);
    for (int i = 0; i < np; i++) {
      {
        std::unique_lock<std::mutex> l(m);
        cv.wait(l, [&] { return issued > i || abort; });
        if (issued <= i) return;  // aborted before piece i was issued
      }
      const int64_t off = (int64_t)i * piece * es, len = std::min(piece, n - (int64_t)i * piece) * es;
      hipError_t e = hipStreamWaitEvent(st.d2h_stream, st.pipe_ev.ev[2 * i + 1], 0);
      if (e == hipSuccess) e = hipMemcpyAsync(out + off, dout + off, (size_t)len, hipMemcpyDeviceToHost, st.d2h_stream);
      if (e != hipSuccess) {
        std::lock_guard<std::mutex> l(m);
        drain_err = std::string("D2H: ") + hipGetErrorString(e);
        return;
      }
    }
  });
  int rc = 0;
  for (int i = 0; i < np && rc == 0; i++) {
    const int64_t off = (int64_t)i * piece * es, cnt = std::min(piece, n - (int64_t)i * piece);
    hipError_t e = hipMemcpyAsync(din + off, in + off, (size_t)(cnt * es), hipMemcpyHostToDevice, st.h2d_stream);
    if (e == hipSuccess) e = hipEventRecord(st.pipe_ev.ev[2 * i], st.h2d_stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(st.io_stream, st.pipe_ev.ev[2 * i], 0);
    if (e != hipSuccess) {
      rc = fail(TIPS_ERR_HIP, "H2D piece %d: %s", i, hipGetErrorString(e));
      break;
    }
    rc = allreduce_device(st, din + off, dout + off, cnt, dtype, st.io_stream);
    if (rc == 0 && (e = hipEventRecord(st.pipe_ev.ev[2 * i + 1], st.io_stream)) != hipSuccess)
      rc = fail(TIPS_ERR_HIP, "event: %s", hipGetErrorString(e));
    if (rc == 0) {
      std::lock_guard<std::mutex> l(m);
      issued = i + 1;
    }
    cv.notify_one();
  }
  {
    std::lock_guard<std::mutex> l(m);
    abort = true;
  }
  cv.notify_one();
  drain.join();
  hipError_t e = hipStreamSynchronize(st.d2h_stream);
  if (rc) return rc;
  if (!drain_err.empty()) return fail(TIPS_ERR_HIP, "%s", drain_err.c_str());
  if (e != hipSuccess) return fail(TIPS_ERR_HIP, "d2h sync: %s", hipGetErrorString(e));
  return 0;
}

// Every rank's `words` int64 values, in rank order (one small RCCL allgather + host sync).
int exchange_i64(State& st, const int64_t* mine, int words, std::vector<int64_t>* all) {
  all->assign((size_t)words * st.size, 0);
  if (st.size == 1) {
    std::copy(mine, mine + words, all->begin());
    return 0;
  }
  TRY(st.small.ensure(sizeof(int64_t) * words * (st.size + 1)));
  int64_t* d = (int64_t*)st.small.p;
  HIP_TRY(hipMemcpyAsync(d + (size_t)words * st.size, mine, sizeof(int64_t) * words, hipMemcpyHostToDevice,
                         st.io_stream));
  NCCL_TRY(ncclAllGather(d + (size_t)words * st.size, d, (size_t)words, ncclInt64, st.comm, st.io_stream));
  HIP_TRY(hipMemcpyAsync(all->data(), d, sizeof(int64_t) * words * st.size, hipMemcpyDeviceToHost, st.io_stream));
  HIP_TRY(hipStreamSynchronize(st.io_stream));
  return 0;
}

std::string shape_str(const int64_t* rec) {  // tensorflow::TensorShape::DebugString() form: [2,4]
  std::string s = "[";
  for (int64_t d = 0; d < rec[2]; d++) s += (d ? "," : "") + std::to_string(rec[3 + d]);
  return s + "]";
}

// ConstructResponseMessage (coordinator.cc:90-186) + GatherFirstRankSizes (:40-88): every
// record is compared with rank 0's; the first mismatch is reported with the reference's text.
int check_records(const int64_t* t, int p) {
  const int W = TIPS_REQUEST_WORDS;
  const int64_t* r0 = t;
  for (int i = 1; i < p; i++)
    if (t[i * W + 1] != r0[1])
      return fail(TIPS_ERR_MISMATCH, "Mismatch data types found: %lld vs %lld.", (long long)r0[1], (long long)t[i * W + 1]);
  for (int i = 1; i < p; i++)  // (the reference compares requests[0] with itself here, coordinator.cc:123-129)
    if (t[i * W + 0] != r0[0])
      return fail(TIPS_ERR_MISMATCH, "Mismatched operations found: %lld vs %lld.", (long long)r0[0], (long long)t[i * W]);
  for (int i = 0; i < p; i++)
    if (t[i * W + 2] < 0 || t[i * W + 2] > TIPS_MAX_DIMS) return fail(TIPS_ERR_INVALID_ARG, "bad ndim in request %d", i);
  if (r0[0] == TIPS_REQ_ALLREDUCE || r0[0] == TIPS_REQ_BROADCAST) {
    for (int i = 1; i < p; i++) {
      const int64_t* ri = t + i * W;
      bool same = ri[2] == r0[2];
      for (int64_t d = 0; same && d < r0[2]; d++) same = ri[3 + d] == r0[3 + d];
      if (!same)
        return fail(TIPS_ERR_MISMATCH, "Mismatched %s tensor shapes: %s vs %s",
                    r0[0] == TIPS_REQ_BROADCAST ? "broadcast" : "allreduce", shape_str(r0).c_str(), shape_str(ri).c_str());
    }
  } else if (r0[0] == TIPS_REQ_ALLGATHER) {
    if (r0[2] == 0) return fail(TIPS_ERR_MISMATCH, "An empty tensor found");
    for (int i = 1; i < p; i++) {
      const int64_t* ri = t + i * W;
      if (ri[2] != r0[2])
        return fail(TIPS_ERR_MISMATCH, "Mismatched allgather tensor shapes: rank %lld vs %lld", (long long)r0[2],
                    (long long)ri[2]);
      for (int64_t d = 1; d < r0[2]; d++)
        if (ri[3 + d] != r0[3 + d])
          return fail(TIPS_ERR_MISMATCH, "Mismatched allgather tensor shapes: %lld-th dimension %lld vs %lld",
                      (long long)d, (long long)r0[3 + d], (long long)ri[3 + d]);
    }
  } else {
    return fail(TIPS_ERR_INVALID_ARG, "Not supported request type: %lld", (long long)r0[0]);
  }
  return 0;
}

// ---------------------------------------------------------------------------
// fusion plans

uint64_t plan_key(void* const* ptrs, const int64_t* counts, int n, int dtype) {
  uint64_t h = 1469598103934665603ull ^ (uint64_t)dtype;
  auto mix = [&](uint64_t v) {
    h ^= v;
    h *= 1099511628211ull;
  };
  mix((uint64_t)n);
  for (int i = 0; i < n; i++) {
    mix((uint64_t)(uintptr_t)ptrs[i]);
    mix((uint64_t)counts[i]);
  }
  return h;
}

void free_plan(FusionPlan& pl) {
  for (auto& b : pl.buckets) {
    if (b.pack) (void)hipFree(b.pack);
    if (b.unpack) (void)hipFree(b.unpack);
  }
  pl.buckets.clear();
}

int build_plan(State& st, FusionPlan& pl, int64_t threshold) {
  const int64_t es = tips::dtype_size(pl.dtype);
  const int n = (int)pl.ptrs.size();
  std::vector<std::vector<CopyTile>> packs(1), unpacks(1);
  std::vector<int64_t> sizes(1, 0);
  for (int i = 0; i < n; i++) {
    const int64_t bytes = pl.counts[i] * es;
    if (bytes == 0) continue;
    if (bytes >= threshold) {  // already bucket-sized: reduce in place
      pl.unfused.push_back(i);
      continue;
    }
    int64_t off = round_up(sizes.back(), kAlignBytes);
    if (off + bytes > threshold) {
      packs.emplace_back();
      unpacks.emplace_back();
      sizes.push_back(0);
      off = 0;
    }
    char* base = (char*)pl.ptrs[i];
    for (int64_t t = 0; t < bytes; t += tips::kCopyTileBytes) {
      const int64_t tb = std::min(tips::kCopyTileBytes, bytes - t);
      // bucket addresses are filled in as offsets; rebased onto the fusion buffer below
      packs.back().push_back(CopyTile{base + t, (char*)(uintptr_t)(off + t), tb});
      unpacks.back().push_back(CopyTile{(const char*)(uintptr_t)(off + t), base + t, tb});
    }
    sizes.back() = off + bytes;
  }
  // two slots: bucket b packs into slot b % 2, so pack(b+1) can run while bucket b is reduced
  for (size_t b = 0; b < sizes.size(); b++) {
    if (sizes[b] == 0) continue;
    FusionBucket fbk;
    char* fb = (char*)st.fusion.p + (int64_t)(pl.buckets.size() % 2) * threshold;
    fbk.buf = fb;
    fbk.bytes = round_up(sizes[b], kAlignBytes);
    fbk.ntiles = (int)packs[b].size();
    for (auto& t : packs[b]) t.dst = fb + (uintptr_t)t.dst;
    for (auto& t : unpacks[b]) t.src = fb + (uintptr_t)t.src;
    const size_t tb = sizeof(CopyTile) * packs[b].size();
    HIP_TRY(hipMalloc(&fbk.pack, tb));
    HIP_TRY(hipMalloc(&fbk.unpack, tb));
    HIP_TRY(hipMemcpy(fbk.pack, packs[b].data(), tb, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(fbk.unpack, unpacks[b].data(), tb, hipMemcpyHostToDevice));
    pl.buckets.push_back(fbk);
  }
  return 0;
}

// Peer transfers of the single-GPU simulators, batched per pipeline step:
// device-to-device copies, or (sim_transport 1) the same bytes as grouped
// ncclSend/ncclRecv pairs to this rank itself, so the RCCL p2p calls the real
// schedules make (byte counts, grouping, stream order) run on a 1-GPU box.
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

}  // namespace

// ===========================================================================
// C-ABI

extern "C" {

const char* tips_last_error(void) { return g_last_error.c_str(); }
const char* tips_version(void) { return "tips_hip 0.1.0 (gfx950)"; }
int tips_unique_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

int tips_get_unique_id(void* out, int64_t cap) {
  if (!out || cap < (int64_t)sizeof(ncclUniqueId)) return fail(TIPS_ERR_INVALID_ARG, "unique id buffer too small");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  memcpy(out, &id, sizeof id);
  return (int)sizeof id;
}

int tips_init_rank(int rank, int size, int device, const void* unique_id, int64_t id_bytes) {
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (st.initialized) return 0;
  if (size < 1 || rank < 0 || rank >= size) return fail(TIPS_ERR_INVALID_ARG, "bad rank %d / size %d", rank, size);
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (ndev < 1) return fail(TIPS_ERR_HIP, "no HIP device visible");
  static const char* const local_vars[] = {"LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", nullptr};
  if (device < 0) device = env_first_int(local_vars, rank) % ndev;
  HIP_TRY(hipSetDevice(device));
  st.device = device;
  TRY(ensure_streams(st));
  if (size > 1 && !unique_id) return fail(TIPS_ERR_INVALID_ARG, "size > 1 needs a unique id");
  if (unique_id) {  // (a 1-rank id is accepted too: the same bootstrap, exercised on one GPU)
    if (id_bytes != (int64_t)sizeof(ncclUniqueId))
      return fail(TIPS_ERR_INVALID_ARG, "unique id must be %zu bytes", sizeof(ncclUniqueId));
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof id);
    NCCL_TRY(ncclCommInitRank(&st.comm, size, id, rank));
  }
  st.rank = rank;
  st.size = size;
  st.initialized = true;
  return 0;
}

void tips_init(void) {
  const char* const rank_vars[] = {"RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", nullptr};
  const char* const size_vars[] = {"WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", nullptr};
  const int rank = env_first_int(rank_vars, 0), size = env_first_int(size_vars, 1);
  if (S().initialized) return;
  ncclUniqueId id;
  memset(&id, 0, sizeof id);
  if (size > 1) {
    const char* host = getenv("MASTER_ADDR");
    if (!host || !*host) host = "127.0.0.1";
    const int port = (int)env_i64("TIPS_BOOTSTRAP_PORT", env_i64("MASTER_PORT", 29500) + 17);
    if (rank == 0 && ncclGetUniqueId(&id) != ncclSuccess) {
      fail(TIPS_ERR_RCCL, "ncclGetUniqueId failed");
      return;
    }
    std::string err;
    if (tips::bootstrap_exchange(rank, size, host, port, &id, (int)sizeof id, (int)env_i64("TIPS_BOOTSTRAP_TIMEOUT", 300),
                                 &err) != 0) {
      fail(TIPS_ERR_BOOTSTRAP, "%s", err.c_str());
      return;
    }
  }
  tips_init_rank(rank, size, -1, size > 1 ? &id : nullptr, size > 1 ? (int64_t)sizeof id : 0);
}

void tips_shutdown(void) {
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return;
  if (st.device >= 0) (void)hipSetDevice(st.device);
  if (st.comm_stream) (void)hipStreamSynchronize(st.comm_stream);
  if (st.comp_stream) (void)hipStreamSynchronize(st.comp_stream);
  if (st.comm) {
    (void)ncclCommDestroy(st.comm);
    st.comm = nullptr;
  }
  for (auto& kv : st.plans) free_plan(kv.second);
  st.plans.clear();
  st.staging.release();
  st.host_in.release();
  st.host_out.release();
  st.fusion.release();
  st.small.release();
  st.recv_ev.release();
  st.sum_ev.release();
  for (hipEvent_t* e : {&st.ev_start, &st.ev_done, &st.ev_comp_done})
    if (*e) {
      (void)hipEventDestroy(*e);
      *e = nullptr;
    }
  st.pipe_ev.release();
  st.fuse_ev.release();
  st.fusion_threshold = 0;
  for (hipStream_t* s : {&st.comm_stream, &st.comp_stream, &st.io_stream, &st.h2d_stream, &st.d2h_stream,
                         &st.fuse_stream, &st.bucket_stream})
    if (*s) {
      (void)hipStreamDestroy(*s);
      *s = nullptr;
    }
  st.initialized = false;
  st.rank = st.size = -1;
}

int tips_bootstrap_broadcast(int rank, int size, const char* host, int port, void* buf, int64_t bytes, int timeout_s) {
  if (size < 1 || rank < 0 || rank >= size || port <= 0 || port > 65535 || bytes < 0 || bytes > (1 << 20) ||
      (bytes > 0 && !buf))
    return fail(TIPS_ERR_INVALID_ARG, "bad bootstrap args");
  std::string err;
  if (tips::bootstrap_exchange(rank, size, (host && *host) ? host : "127.0.0.1", port, buf, (int)bytes,
                               timeout_s > 0 ? timeout_s : 300, &err) != 0)
    return fail(TIPS_ERR_BOOTSTRAP, "%s", err.c_str());
  return 0;
}

bool tips_is_initialize(void) { return S().initialized; }
int tips_size(void) { return S().initialized ? S().size : -1; }
int tips_rank(void) { return S().initialized ? S().rank : -1; }

int tips_set_algorithm(int algo) {
  if (algo < TIPS_ALGO_AUTO || algo > TIPS_ALGO_RCCL) return fail(TIPS_ERR_INVALID_ARG, "bad algorithm %d", algo);
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  st.algo = algo;
  return 0;
}

int tips_get_algorithm(void) { return S().algo; }

int tips_set_sim_transport(int transport) {
  if (transport != 0 && transport != 1) return fail(TIPS_ERR_INVALID_ARG, "bad sim transport %d", transport);
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  st.sim_transport = transport;
  return 0;
}

int tips_resolve_algorithm(int nranks) { return resolve_algo(S().algo, nranks); }

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

int tips_bucket_sum(void* dst, const void* a, const void* b, int64_t count, int dtype, void* stream) {
  TRY(check_dtype(dtype));
  if (count < 0) return fail(TIPS_ERR_INVALID_ARG, "negative count");
  if (count == 0) return 0;
  if (!dst || !a || !b) return fail(TIPS_ERR_INVALID_ARG, "null pointer");
  HIP_TRY(tips::launch_sum2(dst, a, b, count, dtype, (hipStream_t)stream));
  return 0;
}

int tips_sum_variant(void* dst, const void* a, const void* b, int64_t count, int dtype, int mode, int unroll, int nt,
                     int blocks, int threads, void* stream) {
  TRY(check_dtype(dtype));
  if (count <= 0) return 0;
  HIP_TRY(tips::launch_sum2_variant(dst, a, b, count, dtype, mode, unroll, nt, blocks, threads, (hipStream_t)stream));
  return 0;
}

int tips_multi_sum(void* dst, const void* const* srcs, int nsrc, int64_t count, int dtype, void* stream) {
  TRY(check_dtype(dtype));
  if (nsrc < 1 || nsrc > tips::kMaxSrcs) return fail(TIPS_ERR_INVALID_ARG, "nsrc must be 1..%d", tips::kMaxSrcs);
  if (count < 0) return fail(TIPS_ERR_INVALID_ARG, "negative count");
  if (count == 0) return 0;
  HIP_TRY(tips::launch_multi_sum(dst, srcs, nsrc, count, dtype, (hipStream_t)stream));
  return 0;
}

int tips_allreduce(const void* in, void* out, int64_t count, int dtype, int op, void* stream) {
  TRY(check_dtype(dtype));
  if (op != TIPS_OP_SUM) return fail(TIPS_ERR_UNSUPPORTED, "only SUM is implemented (op %d)", op);
  if (count < 0) return fail(TIPS_ERR_INVALID_ARG, "negative count");
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  if (count == 0) return 0;
  if (!in || !out) return fail(TIPS_ERR_INVALID_ARG, "null pointer");
  TRY(set_device(st));
  const size_t bytes = (size_t)count * tips::dtype_size(dtype);
  const bool dout = is_device_ptr(out);
  if (!dout && !is_device_ptr(in) && (int64_t)bytes > env_i64("TIPS_HOST_PIECE_BYTES", 32 << 20))
    return allreduce_host_pipelined(st, (const char*)in, (char*)out, count, dtype);
  return run_staged(st, in, bytes, out, bytes, (hipStream_t)stream, [&](const void* i, void* o, hipStream_t s) {
    return allreduce_device(st, i, o, count, dtype, s);
  });
}

int tips_check_requests(const int64_t* table, int p) {
  if (!table || p < 1) return fail(TIPS_ERR_INVALID_ARG, "bad request table");
  return check_records(table, p);
}

int tips_allreduce_checked(const void* in, void* out, const int64_t* shape, int ndim, int dtype, int op, void* stream) {
  TRY(check_dtype(dtype));
  if (ndim < 0 || ndim > TIPS_MAX_DIMS || (ndim > 0 && !shape)) return fail(TIPS_ERR_INVALID_ARG, "bad shape");
  int64_t count = 1;
  int64_t rec[TIPS_REQUEST_WORDS] = {TIPS_REQ_ALLREDUCE, dtype, ndim};
  for (int d = 0; d < ndim; d++) {
    if (shape[d] < 0) return fail(TIPS_ERR_INVALID_ARG, "negative dimension");
    rec[3 + d] = shape[d];
    count *= shape[d];
  }
  {
    State& st = S();
    std::lock_guard<std::mutex> lk(st.mu);
    if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
    TRY(set_device(st));
    std::vector<int64_t> all;
    TRY(exchange_i64(st, rec, TIPS_REQUEST_WORDS, &all));
    TRY(check_records(all.data(), st.size));
  }
  return tips_allreduce(in, out, count, dtype, op, stream);
}

int tips_allgather_i64(const int64_t* values, int words, int64_t* out) {
  if (!out || !values || words < 1 || words > 4096) return fail(TIPS_ERR_INVALID_ARG, "bad allgather_i64 args");
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  TRY(set_device(st));
  std::vector<int64_t> all;
  TRY(exchange_i64(st, values, words, &all));
  std::copy(all.begin(), all.end(), out);
  return 0;
}

int tips_broadcast(const void* in, void* out, int64_t count, int dtype, int root, void* stream) {
  TRY(check_dtype(dtype));
  if (count < 0) return fail(TIPS_ERR_INVALID_ARG, "negative count");
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  if (root < 0 || root >= st.size) return fail(TIPS_ERR_INVALID_ARG, "root rank %d out of range", root);
  if (count == 0) return 0;
  if (!in || !out) return fail(TIPS_ERR_INVALID_ARG, "null pointer");
  TRY(set_device(st));
  const size_t bytes = (size_t)count * tips::dtype_size(dtype);
  return run_staged(st, in, bytes, out, bytes, (hipStream_t)stream, [&](const void* i, void* o, hipStream_t s) {
    if (st.size == 1) {
      if (i != o) HIP_TRY(hipMemcpyAsync(o, i, bytes, hipMemcpyDeviceToDevice, s));
      return 0;
    }
    NCCL_TRY(ncclBroadcast(i, o, bytes, ncclInt8, root, st.comm, s));
    return 0;
  });
}

int tips_allgatherv(const void* in, int64_t count, void* out, const int64_t* counts, int dtype, void* stream) {
  TRY(check_dtype(dtype));
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  if (!counts || count < 0) return fail(TIPS_ERR_INVALID_ARG, "bad counts");
  if (counts[st.rank] != count)
    return fail(TIPS_ERR_INVALID_ARG, "input and first_ranks not match %lld vs %lld", (long long)count,
                (long long)counts[st.rank]);  // AllgathervCpu's check, utils.h:103-106
  const int64_t es = tips::dtype_size(dtype);
  std::vector<int64_t> disp(st.size + 1, 0);
  for (int r = 0; r < st.size; r++) {
    if (counts[r] < 0) return fail(TIPS_ERR_INVALID_ARG, "negative count for rank %d", r);
    disp[r + 1] = disp[r] + counts[r];
  }
  if (disp[st.size] == 0) return 0;
  if (!out || (count > 0 && !in)) return fail(TIPS_ERR_INVALID_ARG, "null pointer");
  TRY(set_device(st));
  return run_staged(st, in, (size_t)(count * es), out, (size_t)(disp[st.size] * es), (hipStream_t)stream,
                    [&](const void* i, void* o, hipStream_t s) {
                      char* ob = (char*)o;
                      if (count > 0 && (const char*)i != ob + disp[st.rank] * es)
                        HIP_TRY(hipMemcpyAsync(ob + disp[st.rank] * es, i, (size_t)(count * es),
                                               hipMemcpyDeviceToDevice, s));
                      if (st.size == 1) return 0;
                      NCCL_TRY(ncclGroupStart());
                      for (int r = 0; r < st.size; r++) {
                        if (r == st.rank) continue;
                        if (count > 0) NCCL_TRY(ncclSend(i, (size_t)(count * es), ncclInt8, r, st.comm, s));
                        if (counts[r] > 0)
                          NCCL_TRY(ncclRecv(ob + disp[r] * es, (size_t)(counts[r] * es), ncclInt8, r, st.comm, s));
                      }
                      NCCL_TRY(ncclGroupEnd());
                      return 0;
                    });
}

int tips_fused_allreduce(void* const* ptrs, const int64_t* counts, int n, int dtype, void* stream) {
  TRY(check_dtype(dtype));
  if (n < 0 || (n > 0 && (!ptrs || !counts))) return fail(TIPS_ERR_INVALID_ARG, "bad tensor list");
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  if (n == 0) return 0;
  TRY(set_device(st));
  for (int i = 0; i < n; i++)
    if (counts[i] < 0 || (counts[i] > 0 && !ptrs[i])) return fail(TIPS_ERR_INVALID_ARG, "bad tensor %d", i);
  hipStream_t s = (hipStream_t)stream;
  const int64_t es = tips::dtype_size(dtype);
  const int64_t threshold = round_up(std::max<int64_t>(kAlignBytes, env_i64("TIPS_FUSION_THRESHOLD", 64 << 20)), kAlignBytes);
  if (threshold != st.fusion_threshold) {  // slots (re)sized: every cached plan points into the old ones
    HIP_TRY(hipDeviceSynchronize());
    for (auto& kv : st.plans) free_plan(kv.second);
    st.plans.clear();
    st.fusion.release();
    TRY(st.fusion.ensure((size_t)(2 * threshold), /*zero=*/true));
    st.fusion_threshold = threshold;
  }
  const uint64_t key = plan_key(ptrs, counts, n, dtype);
  auto it = st.plans.find(key);
  bool hit = it != st.plans.end() && it->second.dtype == dtype && (int)it->second.ptrs.size() == n &&
             std::equal(ptrs, ptrs + n, it->second.ptrs.begin()) && std::equal(counts, counts + n, it->second.counts.begin());
  if (!hit) {
    if (it != st.plans.end() || st.plans.size() >= 64) {  // descriptors may still be read by queued kernels
      HIP_TRY(hipDeviceSynchronize());
      if (it != st.plans.end()) {
        free_plan(it->second);
        st.plans.erase(it);
      }
      if (st.plans.size() >= 64) {
        for (auto& kv : st.plans) free_plan(kv.second);
        st.plans.clear();
      }
    }
    FusionPlan pl;
    pl.dtype = dtype;
    pl.ptrs.assign(ptrs, ptrs + n);
    pl.counts.assign(counts, counts + n);
    int rc = build_plan(st, pl, threshold);
    if (rc) {
      free_plan(pl);
      return rc;
    }
    it = st.plans.emplace(key, std::move(pl)).first;
  }
  const FusionPlan& pl = it->second;
  const int B = (int)pl.buckets.size();
  if (B > 0 && st.size == 1) {  // nothing to overlap with: pack, (no-op) reduce, unpack on the caller's stream
    for (const auto& b : pl.buckets) {
      HIP_TRY(tips::launch_copy_tiles(b.pack, b.ntiles, s));
      TRY(allreduce_device(st, b.buf, b.buf, b.bytes / es, dtype, s));
      HIP_TRY(tips::launch_copy_tiles(b.unpack, b.ntiles, s));
    }
  } else if (B > 0) {
    // fuse stream: pack(0) pack(1) unpack(0) pack(2) unpack(1) ... unpack(B-1)
    // bucket stream: allreduce(b) after pack(b); unpack(b) after allreduce(b); pack(b+2) after unpack(b)
    TRY(st.fuse_ev.ensure(2 * (size_t)B));
    hipEvent_t* packed = st.fuse_ev.ev.data();
    hipEvent_t* reduced = st.fuse_ev.ev.data() + B;
    TRY(join(st.fuse_stream, s, st.ev_start));
    auto pack = [&](int b) -> int {
      HIP_TRY(tips::launch_copy_tiles(pl.buckets[b].pack, pl.buckets[b].ntiles, st.fuse_stream));
      HIP_TRY(hipEventRecord(packed[b], st.fuse_stream));
      return 0;
    };
    TRY(pack(0));
    for (int b = 0; b < B; b++) {
      if (b + 1 < B && b + 1 < 2) TRY(pack(b + 1));  // slot 1 is free from the start
      HIP_TRY(hipStreamWaitEvent(st.bucket_stream, packed[b], 0));
      TRY(allreduce_device(st, pl.buckets[b].buf, pl.buckets[b].buf, pl.buckets[b].bytes / es, dtype, st.bucket_stream));
      HIP_TRY(hipEventRecord(reduced[b], st.bucket_stream));
      HIP_TRY(hipStreamWaitEvent(st.fuse_stream, reduced[b], 0));
      HIP_TRY(tips::launch_copy_tiles(pl.buckets[b].unpack, pl.buckets[b].ntiles, st.fuse_stream));
      if (b + 2 < B) TRY(pack(b + 2));  // reuses slot b % 2, after unpack(b) in stream order
    }
    TRY(join(s, st.fuse_stream, st.ev_done));
  }
  for (int i : pl.unfused) TRY(allreduce_device(st, ptrs[i], ptrs[i], counts[i], dtype, s));
  return 0;
}

// ---------------------------------------------------------------------------
// single-GPU schedule simulators (test harnesses)

int tips_ring_simulate(void* const* outs, const void* const* ins, int p, int64_t n, int dtype, void* stream) {
  TRY(check_dtype(dtype));
  if (p < 1 || p > 64 || n < 0 || !outs || !ins) return fail(TIPS_ERR_INVALID_ARG, "bad simulate args");
  if (n == 0) return 0;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  TRY(sim_prepare(st));
  SimXfer xf(st);
  hipStream_t user = (hipStream_t)stream;
  const int64_t es = tips::dtype_size(dtype), align = kAlignBytes / es;
  if (p == 1) {
    if (outs[0] != ins[0]) HIP_TRY(hipMemcpyAsync(outs[0], ins[0], (size_t)(n * es), hipMemcpyDeviceToDevice, user));
    return 0;
  }
  const int64_t max_chunk = chunk_of(n, p, align, 0).len();
  const int K = pipeline_depth(max_chunk * es);
  TRY(st.staging.ensure((size_t)(2 * p * max_chunk * es)));
  TRY(st.recv_ev.ensure(2 * K));
  TRY(st.sum_ev.ensure(2 * K));
  auto stg = [&](int r, int par) { return (char*)st.staging.p + ((int64_t)r * 2 + par) * max_chunk * es; };
  TRY(join(st.comm_stream, user, st.ev_start));
  HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.ev_start, 0));
  for (int s = 0; s < p - 1; s++) {
    for (int k = 0; k < K; k++) {
      if (s > 0) HIP_TRY(hipStreamWaitEvent(st.comm_stream, st.sum_ev.ev[((s - 1) & 1) * K + k], 0));
      for (int r = 0; r < p; r++) {  // virtual rank r receives from r-1
        const int prev = mod(r - 1, p);
        const Range rc = chunk_of(n, p, align, mod(r - s - 1, p));
        const Range rs = sub_of(rc, K, align, k);
        if (rs.len() == 0) continue;
        const char* src = (s == 0) ? (const char*)ins[prev] : (const char*)outs[prev];
        xf.add(stg(r, s & 1) + (rs.b - rc.b) * es, src + rs.b * es, rs.len() * es);
      }
      TRY(xf.flush());
      hipEvent_t rev = st.recv_ev.ev[(s & 1) * K + k];
      HIP_TRY(hipEventRecord(rev, st.comm_stream));
      HIP_TRY(hipStreamWaitEvent(st.comp_stream, rev, 0));
      for (int r = 0; r < p; r++) {
        const Range rc = chunk_of(n, p, align, mod(r - s - 1, p));
        const Range rs = sub_of(rc, K, align, k);
        TRY(sum2((char*)outs[r] + rs.b * es, (const char*)ins[r] + rs.b * es, stg(r, s & 1) + (rs.b - rc.b) * es,
                 rs.len(), dtype, st.comp_stream));
      }
      HIP_TRY(hipEventRecord(st.sum_ev.ev[(s & 1) * K + k], st.comp_stream));
    }
  }
  for (int s = 0; s < p - 1; s++) {
    for (int k = 0; k < K; k++) {
      if (s == 0) HIP_TRY(hipStreamWaitEvent(st.comm_stream, st.sum_ev.ev[((p - 2) & 1) * K + k], 0));
      for (int r = 0; r < p; r++) {
        const int prev = mod(r - 1, p);
        const Range rs = sub_of(chunk_of(n, p, align, mod(r - s, p)), K, align, k);
        if (rs.len() == 0) continue;
        xf.add((char*)outs[r] + rs.b * es, (const char*)outs[prev] + rs.b * es, rs.len() * es);
      }
      TRY(xf.flush());
    }
  }
  TRY(join(user, st.comm_stream, st.ev_done));
  TRY(join(user, st.comp_stream, st.ev_comp_done));
  return 0;
}

int tips_direct_simulate(void* const* outs, const void* const* ins, int p, int64_t n, int dtype, void* stream) {
  TRY(check_dtype(dtype));
  if (p < 1 || p > tips::kMaxSrcs || n < 0 || !outs || !ins) return fail(TIPS_ERR_INVALID_ARG, "bad simulate args");
  if (n == 0) return 0;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  TRY(sim_prepare(st));
  SimXfer xf(st);
  hipStream_t user = (hipStream_t)stream;
  const int64_t es = tips::dtype_size(dtype), align = kAlignBytes / es;
  if (p == 1) {
    if (outs[0] != ins[0]) HIP_TRY(hipMemcpyAsync(outs[0], ins[0], (size_t)(n * es), hipMemcpyDeviceToDevice, user));
    return 0;
  }
  const int64_t max_chunk = chunk_of(n, p, align, 0).len();
  const int K = pipeline_depth(max_chunk * es);
  // staging[r][j]: slice of chunk r sent by virtual rank j
  TRY(st.staging.ensure((size_t)((int64_t)p * p * max_chunk * es)));
  TRY(st.recv_ev.ensure(K));
  TRY(st.sum_ev.ensure(K));
  auto slot = [&](int r, int j) { return (char*)st.staging.p + ((int64_t)r * p + j) * max_chunk * es; };
  TRY(join(st.comm_stream, user, st.ev_start));
  HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.ev_start, 0));
  for (int k = 0; k < K; k++) {
    for (int r = 0; r < p; r++) {
      const Range mine = chunk_of(n, p, align, r), ms = sub_of(mine, K, align, k);
      if (ms.len() == 0) continue;
      for (int j = 0; j < p; j++)
        if (j != r) xf.add(slot(r, j) + (ms.b - mine.b) * es, (const char*)ins[j] + ms.b * es, ms.len() * es);
    }
    TRY(xf.flush());
    HIP_TRY(hipEventRecord(st.recv_ev.ev[k], st.comm_stream));
    HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.recv_ev.ev[k], 0));
    for (int r = 0; r < p; r++) {
      const Range mine = chunk_of(n, p, align, r), ms = sub_of(mine, K, align, k);
      const void* srcs[tips::kMaxSrcs];
      for (int j = 0; j < p; j++)
        srcs[j] = (j == r) ? (const void*)((const char*)ins[r] + ms.b * es) : slot(r, j) + (ms.b - mine.b) * es;
      HIP_TRY(tips::launch_multi_sum((char*)outs[r] + ms.b * es, srcs, p, ms.len(), dtype, st.comp_stream));
    }
    HIP_TRY(hipEventRecord(st.sum_ev.ev[k], st.comp_stream));
  }
  for (int k = 0; k < K; k++) {
    HIP_TRY(hipStreamWaitEvent(st.comm_stream, st.sum_ev.ev[k], 0));
    for (int r = 0; r < p; r++) {
      const Range ms = sub_of(chunk_of(n, p, align, r), K, align, k);
      if (ms.len() == 0) continue;
      for (int j = 0; j < p; j++)
        if (j != r) xf.add((char*)outs[j] + ms.b * es, (const char*)outs[r] + ms.b * es, ms.len() * es);
    }
    TRY(xf.flush());
  }
  TRY(join(user, st.comm_stream, st.ev_done));
  TRY(join(user, st.comp_stream, st.ev_comp_done));
  return 0;
}

}  // extern "C"
