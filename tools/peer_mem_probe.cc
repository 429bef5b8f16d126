// peer_mem_probe.cc — local-HBM cost of the peer schedule's memory kinds (one GPU).
//
// The peer schedule keeps its IPC workspace in uncached device memory so that
// no GPU's L2 holds a stale line of it (peer.cc). This measures what that costs
// on the local side, for the peer schedule's two kernels at config-3 shapes
// (p = 8, 1 GiB bucket: 128 MiB chunks):
//   xfer:  7 segments of 128 MiB, coarse -> {coarse, fine, uncached} (push's
//          local analogue) and {coarse, fine, uncached} -> coarse (pull's);
//   fold:  multi_sum of 8 sources of 128 MiB (1 coarse + 7 of the kind) into
//          one of the kind.
// Variants interleaved over rounds in one process; median ms and GB/s of
// algorithmic bytes. One JSON line per variant.
//   hipcc --offload-arch=gfx950 -O2 -o tools/peer_mem_probe tools/peer_mem_probe.cc -Iinclude -Ltools/lib -ltips_hip_dev
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../include/tips_hip_dev.h"

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e = (x);                                                                  \
    if (e != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));   \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

static void* alloc(size_t bytes, int kind) {
  void* p = nullptr;
  if (kind == 0) CHECK(hipMalloc(&p, bytes));
  else CHECK(hipExtMallocWithFlags(&p, bytes, kind == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached));
  CHECK(hipMemset(p, 1, bytes));
  return p;
}

int main(int argc, char** argv) {
  const int64_t seg = (argc > 1 ? atoll(argv[1]) : 128) << 20;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5, iters = argc > 3 ? atoi(argv[3]) : 10;
  const int nseg = 7;
  const char* kn[] = {"coarse", "fine", "uncached"};
  void* coarse_src = alloc(nseg * seg, 0);
  void* coarse_dst = alloc(nseg * seg, 0);
  void* kind_buf[3];
  for (int k = 0; k < 3; k++) kind_buf[k] = alloc((nseg + 1) * seg, k);
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  struct V { std::string name; int op, kind; double bytes; std::vector<double> ms; };
  std::vector<V> vs;
  for (int k = 0; k < 3; k++) {
    vs.push_back({std::string("xfer_to_") + kn[k], 0, k, 2.0 * nseg * seg, {}});
    vs.push_back({std::string("xfer_from_") + kn[k], 1, k, 2.0 * nseg * seg, {}});
    vs.push_back({std::string("fold8_") + kn[k], 2, k, 9.0 * seg, {}});
  }
  auto run = [&](const V& v) {
    if (v.op < 2) {
      void* d[nseg];
      const void* sr[nseg];
      int64_t b[nseg];
      for (int i = 0; i < nseg; i++) {
        char* kb = (char*)kind_buf[v.kind] + i * seg;
        d[i] = v.op == 0 ? (void*)kb : (char*)coarse_dst + i * seg;
        sr[i] = v.op == 0 ? (const void*)((char*)coarse_src + i * seg) : kb;
        b[i] = seg;
      }
      if (tips_xfer(d, sr, b, nseg, s)) { fprintf(stderr, "%s\n", tips_last_error()); exit(1); }
    } else {
      const void* sr[8];
      sr[0] = coarse_src;
      for (int i = 1; i < 8; i++) sr[i] = (char*)kind_buf[v.kind] + (i - 1) * seg;
      if (tips_multi_sum((char*)kind_buf[v.kind] + 7 * seg, sr, 8, seg / 4, 0, s)) exit(1);
    }
  };
  for (auto& v : vs) run(v);
  CHECK(hipStreamSynchronize(s));
  for (int r = 0; r < rounds; r++)
    for (auto& v : vs) {
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < iters; i++) run(v);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / iters);
    }
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    double med = v.ms[v.ms.size() / 2];
    printf("{\"variant\": \"%s\", \"segment_mib\": %lld, \"ms_median\": %.4f, \"ms_min\": %.4f, \"GBps\": %.1f}\n",
           v.name.c_str(), (long long)(seg >> 20), med, v.ms[0], v.bytes / (med * 1e-3) / 1e9);
  }
  return 0;
}
