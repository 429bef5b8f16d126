// graph_probe.cc — which HIP-graph capture patterns this ROCm / RCCL accepts (TIPS_GRAPHS).
// Build: make repro (tools/_bin/graph_probe)
// Run:   graph_probe RANK SIZE MODE ID_FILE   (SIZE > 1: one process per rank; with NCCL_HOSTID
//        set per process they may share one GPU over RCCL's socket transport)
// Modes (each: eager warm-up call, capture, instantiate, 3 replays, check the bytes):
//   0 kernels and events only: fork two streams from the origin, join back
//   1 ncclAllReduce on the origin stream
//   2 grouped ncclSend/ncclRecv on the origin stream
//   3 grouped ncclSend/ncclRecv on a stream forked from the origin (the executor's pattern)
//   4 mode 3 plus a kernel on a second forked stream behind an event (the full pattern)
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <vector>

#define CK(x)                                                                                     \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      fprintf(stderr, "rank %d: %s -> %s\n", rank, #x, hipGetErrorString(e_));                   \
      return 1;                                                                                   \
    }                                                                                             \
  } while (0)
#define NK(x)                                                                                     \
  do {                                                                                            \
    ncclResult_t r_ = (x);                                                                        \
    if (r_ != ncclSuccess) {                                                                      \
      fprintf(stderr, "rank %d: %s -> %s\n", rank, #x, ncclGetErrorString(r_));                  \
      return 1;                                                                                   \
    }                                                                                             \
  } while (0)

__global__ void add_one(float* p, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1.0f;
}

static int rank = 0;

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: graph_probe RANK SIZE MODE ID_FILE\n");
    return 2;
  }
  rank = atoi(argv[1]);
  const int size = atoi(argv[2]), mode = atoi(argv[3]);
  const char* idf = argv[4];
  CK(hipSetDevice(0));
  ncclUniqueId id;
  if (rank == 0) {
    NK(ncclGetUniqueId(&id));
    char tmp[512];
    snprintf(tmp, sizeof tmp, "%s.tmp", idf);
    FILE* f = fopen(tmp, "wb");
    fwrite(&id, sizeof id, 1, f);
    fclose(f);
    rename(tmp, idf);
  } else {
    FILE* f = nullptr;
    for (int i = 0; i < 600 && !(f = fopen(idf, "rb")); i++) usleep(100000);
    if (!f || fread(&id, sizeof id, 1, f) != 1) {
      fprintf(stderr, "rank %d: no id\n", rank);
      return 1;
    }
    fclose(f);
  }
  ncclComm_t comm;
  NK(ncclCommInitRank(&comm, size, id, rank));
  const size_t n = getenv("PROBE_N") ? (size_t)atoll(getenv("PROBE_N")) : (size_t)1 << 20;  // floats per buffer
  float *a, *b;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4 * (size_t)size));
  hipStream_t origin, s1, s2;
  // PROBE_PRIO=1: origin and s1 at the device's highest priority (the executor's comm and graph streams)
  int least = 0, greatest = 0;
  CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  const bool prio = getenv("PROBE_PRIO") != nullptr, nosync = getenv("PROBE_NOSYNC") != nullptr,
             dangling = getenv("PROBE_DANGLING") != nullptr;
  CK(hipStreamCreateWithPriority(&origin, hipStreamNonBlocking, prio ? greatest : least));
  CK(hipStreamCreateWithPriority(&s1, hipStreamNonBlocking, prio ? greatest : least));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ev[5];
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  std::vector<float> h(n, (float)(rank + 1));

  auto body = [&](void) -> int {
    if (mode == 0) {
      CK(hipEventRecord(ev[0], origin));
      CK(hipStreamWaitEvent(s1, ev[0], 0));
      CK(hipStreamWaitEvent(s2, ev[0], 0));
      add_one<<<(unsigned)(n / 256), 256, 0, s1>>>(a, n);
      CK(hipEventRecord(ev[1], s1));
      CK(hipStreamWaitEvent(s2, ev[1], 0));
      add_one<<<(unsigned)(n / 256), 256, 0, s2>>>(a, n);
      CK(hipEventRecord(ev[2], s1));
      CK(hipStreamWaitEvent(origin, ev[2], 0));
      CK(hipEventRecord(ev[3], s2));
      CK(hipStreamWaitEvent(origin, ev[3], 0));
    } else if (mode == 1) {
      NK(ncclAllReduce(a, a, n, ncclFloat32, ncclSum, comm, origin));
    } else {
      hipStream_t cs = mode == 2 ? origin : s1;
      if (mode >= 3) {
        CK(hipEventRecord(ev[0], origin));
        CK(hipStreamWaitEvent(s1, ev[0], 0));
        CK(hipStreamWaitEvent(s2, ev[0], 0));
      }
      NK(ncclGroupStart());
      for (int q = 0; q < size; q++) {
        NK(ncclSend(a, n * 4, ncclInt8, q, comm, cs));
        NK(ncclRecv(b + (size_t)q * n, n * 4, ncclInt8, q, comm, cs));
      }
      NK(ncclGroupEnd());
      if (mode == 4) {
        CK(hipEventRecord(ev[1], s1));
        CK(hipStreamWaitEvent(s2, ev[1], 0));
        add_one<<<(unsigned)(n / 256), 256, 0, s2>>>(b, n);
        if (dangling) CK(hipEventRecord(ev[4], s2));  // recorded, never waited on inside the capture
      }
      if (mode >= 3) {
        CK(hipEventRecord(ev[2], s1));
        CK(hipStreamWaitEvent(origin, ev[2], 0));
        CK(hipEventRecord(ev[3], s2));
        CK(hipStreamWaitEvent(origin, ev[3], 0));
      }
    }
    return 0;
  };
  auto reset = [&]() -> int {
    CK(hipMemcpy(a, h.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(b, 0, n * 4 * (size_t)size));
    return 0;
  };
  auto check = [&](const char* what) -> int {
    CK(hipStreamSynchronize(origin));
    std::vector<float> ha(n), hb(n * (size_t)size);
    CK(hipMemcpy(ha.data(), a, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), b, n * 4 * (size_t)size, hipMemcpyDeviceToHost));
    float want_a = mode == 0 ? rank + 3.0f : mode == 1 ? size * (size + 1) / 2.0f : (float)(rank + 1);
    bool ok = ha[0] == want_a && ha[n - 1] == want_a;
    if (mode >= 2)
      for (int q = 0; q < size; q++) {
        float w = (float)(q + 1) + (mode == 4 && q == 0 ? 1.0f : 0.0f);
        ok = ok && hb[(size_t)q * n] == w && hb[(size_t)q * n + n - 1] == w;
      }
    printf("rank %d mode %d %s: %s (a=%g b0=%g)\n", rank, mode, what, ok ? "ok" : "WRONG", ha[0], hb[0]);
    fflush(stdout);
    return ok ? 0 : 1;
  };
  if (reset() || body() || check("eager")) return 1;
  if (getenv("PROBE_EAGER_ONLY")) {
    for (int it = 0; it < 3; it++)
      if (reset() || body() || check("eager again")) return 1;
    NK(ncclCommDestroy(comm));
    printf("rank %d mode %d: PASS (eager only)\n", rank, mode);
    return 0;
  }
  if (nosync) {  // more eager calls still in flight when the capture starts (PROBE_NOSYNC=1)
    if (reset()) return 1;
    for (int it = 0; it < 2; it++)
      if (body()) return 1;
  } else {
    CK(hipDeviceSynchronize());
  }
  printf("rank %d mode %d: capture\n", rank, mode);
  fflush(stdout);
  CK(hipStreamBeginCapture(origin, hipStreamCaptureModeRelaxed));
  if (body()) return 1;
  hipGraph_t g = nullptr;
  printf("rank %d mode %d: end capture\n", rank, mode);
  fflush(stdout);
  CK(hipStreamEndCapture(origin, &g));
  size_t nn = 0;
  CK(hipGraphGetNodes(g, nullptr, &nn));
  printf("rank %d mode %d: graph of %zu nodes\n", rank, mode, nn);
  fflush(stdout);
  hipGraphExec_t x;
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  for (int it = 0; it < 3; it++) {
    if (reset()) return 1;
    CK(hipGraphLaunch(x, origin));
    if (check("replay")) return 1;
  }
  CK(hipGraphExecDestroy(x));
  CK(hipGraphDestroy(g));
  NK(ncclCommDestroy(comm));
  printf("rank %d mode %d: PASS\n", rank, mode);
  return 0;
}
