// rt_common.cc — error reporting, process state, streams and small helpers of the runtime.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "rt.h"

namespace tips {
namespace rt {

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

const std::string& last_error() { return g_last_error; }

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

State& S() {
  static State* s = new State();  // never destroyed: safe at exit
  return *s;
}

int ensure_streams(State& st) {
  if (!st.comm_stream) {
    // The transfers get the device's highest stream priority: a sum kernel of ~10^5 workgroups
    // on the compute stream must not keep the next sub-chunk's RCCL kernel waiting for CUs, or
    // the transfer/sum overlap of the pipelined schedules is lost.
    int least = 0, greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_TRY(hipStreamCreateWithPriority(&st.comm_stream, hipStreamNonBlocking, greatest));
  }
  if (!st.graph_stream) {  // replayed plans carry the same RCCL kernels: the same priority
    int least = 0, greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_TRY(hipStreamCreateWithPriority(&st.graph_stream, hipStreamNonBlocking, greatest));
  }
  for (hipEvent_t& e : st.ev_graph)
    if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (hipEvent_t& e : st.ev_rccl)
    if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (!st.comp_stream) HIP_TRY(hipStreamCreateWithFlags(&st.comp_stream, hipStreamNonBlocking));
  if (!st.io_stream) HIP_TRY(hipStreamCreateWithFlags(&st.io_stream, hipStreamNonBlocking));
  if (!st.h2d_stream) HIP_TRY(hipStreamCreateWithFlags(&st.h2d_stream, hipStreamNonBlocking));
  if (!st.d2h_stream) HIP_TRY(hipStreamCreateWithFlags(&st.d2h_stream, hipStreamNonBlocking));
  if (!st.h2d_stream2) HIP_TRY(hipStreamCreateWithFlags(&st.h2d_stream2, hipStreamNonBlocking));
  if (!st.fuse_stream) HIP_TRY(hipStreamCreateWithFlags(&st.fuse_stream, hipStreamNonBlocking));
  if (!st.bucket_stream) HIP_TRY(hipStreamCreateWithFlags(&st.bucket_stream, hipStreamNonBlocking));
  if (!st.ev_start) HIP_TRY(hipEventCreateWithFlags(&st.ev_start, hipEventDisableTiming));
  if (!st.ev_done) HIP_TRY(hipEventCreateWithFlags(&st.ev_done, hipEventDisableTiming));
  if (!st.ev_comp_done) HIP_TRY(hipEventCreateWithFlags(&st.ev_comp_done, hipEventDisableTiming));
  if (!st.ev_comp_prev) HIP_TRY(hipEventCreateWithFlags(&st.ev_comp_prev, hipEventDisableTiming));
  if (!st.ev_fuse_table) HIP_TRY(hipEventCreateWithFlags(&st.ev_fuse_table, hipEventDisableTiming));
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

// Join: `waiter` waits for all work queued so far on `src`.
int join(hipStream_t waiter, hipStream_t src, hipEvent_t ev) {
  HIP_TRY(hipEventRecord(ev, src));
  HIP_TRY(hipStreamWaitEvent(waiter, ev, 0));
  return 0;
}

// Buckets up to this go one-shot (one exchange + one fold kernel) under AUTO and TUNE. At p = 2
// a one-shot moves the same bytes over the link as the ring (S each way) in one step instead of
// two, so it wins at every size the fold's staging stays small for: 8 MiB (the p = 2 rehearsal,
// profiles/r03/small_bucket_rehearsal_n2_before.json, measured it fastest at 16 KiB - 8 MiB). For p > 2 it
// moves (p - 1) x the bytes of the all-pairs schedule per link, so it stays a latency tool: 256 KiB.
// TIPS_ONESHOT_BYTES overrides both.
int64_t oneshot_bytes(int p) {
  return env_i64("TIPS_ONESHOT_BYTES", p == 2 ? (int64_t)8 << 20 : (int64_t)256 << 10);
}

int resolve_algo(int algo, int p, int64_t bytes) {
  if (algo == TIPS_ALGO_AUTO) {
    const char* e = getenv("TIPS_ALGO");
    if (e && *e) {
      if (!strcmp(e, "ring")) algo = TIPS_ALGO_RING;
      if (!strcmp(e, "direct")) algo = TIPS_ALGO_DIRECT;
      if (!strcmp(e, "rccl")) algo = TIPS_ALGO_RCCL;
      if (!strcmp(e, "oneshot")) algo = TIPS_ALGO_ONESHOT;
      if (!strcmp(e, "peer")) algo = TIPS_ALGO_PEER;
      if (!strcmp(e, "tune")) algo = TIPS_ALGO_TUNE;
    }
  }
  if (algo == TIPS_ALGO_TUNE) {  // measured per size class; small buckets stay latency-bound one-shots
    if (p > 1 && p <= tips::kMaxSrcs && bytes <= oneshot_bytes(p)) return TIPS_ALGO_ONESHOT;
    return TIPS_ALGO_TUNE;
  }
  if (algo != TIPS_ALGO_AUTO) return algo;
  // small buckets: one exchange + one kernel beats 2(p-1) pipelined steps (latency-bound);
  // large: ring on one link pair (p <= 2), all-pairs over every xGMI link otherwise
  if (p > 1 && p <= tips::kMaxSrcs && bytes <= oneshot_bytes(p)) return TIPS_ALGO_ONESHOT;
  return (p <= 2 || p > tips::kMaxSrcs) ? TIPS_ALGO_RING : TIPS_ALGO_DIRECT;
}

const cpu_set_t& process_cpus() {
  static const cpu_set_t set = [] {
    cpu_set_t s;
    if (sched_getaffinity(0, sizeof s, &s) != 0) {
      CPU_ZERO(&s);
      for (int i = 0; i < CPU_SETSIZE; i++) CPU_SET(i, &s);
    }
    return s;
  }();
  return set;
}

namespace {
// captured when the library is loaded, on the loading thread (before any thread of ours is pinned)
__attribute__((constructor)) void capture_process_cpus() { (void)process_cpus(); }
}  // namespace

void rccl_env_defaults() {
  // Captured plans (TIPS_GRAPHS) key their graphs by buffer address and allocation id; RCCL's
  // graph-time buffer registration would pin peers' mappings of a buffer past its free, so with
  // replays on it is off unless the user sets it (read by RCCL at its first communicator).
  if (env_i64("TIPS_GRAPHS", 0) > 0) setenv("NCCL_GRAPH_REGISTER", "0", 0);
}

int ensure_comm(State& st) {
  if (st.comm) return 0;
  if (st.size != 1) return fail(TIPS_ERR_NOT_INITIALIZED, "no RCCL communicator");
  rccl_env_defaults();
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  NCCL_TRY(ncclCommInitRank(&st.comm, 1, id, 0));
  return 0;
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

// Page-locked host memory (hipHostMalloc / hipHostRegister / torch pin_memory) over the whole range:
// copies from and to it are asynchronous DMA and never block the issuing thread.
bool is_pinned_host(const void* p, int64_t bytes) {
  for (const char* q : {(const char*)p, (const char*)p + (bytes > 0 ? bytes - 1 : 0)}) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, q) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    if (a.type != hipMemoryTypeHost) return false;
  }
  return true;
}

int check_dtype(int dtype) {
  if (tips::dtype_size(dtype) == 0) return fail(TIPS_ERR_INVALID_ARG, "unsupported dtype %d", dtype);
  return 0;
}

int set_device(State& st) {
  if (st.device >= 0) HIP_TRY(hipSetDevice(st.device));
  return 0;
}

}  // namespace rt
}  // namespace tips
