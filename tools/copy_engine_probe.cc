// copy_engine_probe.cc — which engine moves the host path's copies, and what each direction gets
// when both run at once (DESIGN.md §6 "Host path"). Page-locked host buffers (hipHostMalloc) and
// device buffers of PIECES x PIECE_MIB; per mode, H2D pieces on one stream and D2H pieces on
// another, issued together; each direction's span from HIP events. Modes:
//   default   hipMemcpyAsync H2D + hipMemcpyAsync D2H (what host_staging.cc issues)
//   nocu_d2h  D2H as hipMemcpyDeviceToDeviceNoCU (the host pointer is device-accessible)
//   nocu_both both directions as hipMemcpyDeviceToDeviceNoCU
//   h2d_only / d2h_only / d2h_only_nocu  one direction alone
//   d2h_streamsK / both_streamsK  the D2H pieces round-robin over K streams (K DMA queues)
//   d2h_kernel / both_kernel  the D2H as a copy kernel writing the page-locked buffer through its
//     device mapping (WGS workgroups of 256 lanes, 16 B per lane per iteration)
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/_bin/copy_engine_probe tools/copy_engine_probe.cc
// Run under rocprofv3 --kernel-trace to see which copies became blit kernels.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ void d2h_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(src[i], dst + i);
}

int main() {
  const int pieces = getenv("PIECES") ? atoi(getenv("PIECES")) : 8;
  const size_t piece = (size_t)(getenv("PIECE_MIB") ? atoi(getenv("PIECE_MIB")) : 16) << 20;
  const int reps = 5;
  char *hin, *hout, *din, *dout;
  CK(hipHostMalloc((void**)&hin, piece * pieces, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&hout, piece * pieces, hipHostMallocDefault));
  CK(hipMalloc((void**)&din, piece * pieces));
  CK(hipMalloc((void**)&dout, piece * pieces));
  memset(hin, 1, piece * pieces);
  CK(hipMemset(dout, 2, piece * pieces));
  hipStream_t sh, sd;
  CK(hipStreamCreateWithFlags(&sh, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sd, hipStreamNonBlocking));
  hipEvent_t a0, a1, b0, b1;
  CK(hipEventCreate(&a0));
  CK(hipEventCreate(&a1));
  CK(hipEventCreate(&b0));
  CK(hipEventCreate(&b1));
  const int wgs = getenv("WGS") ? atoi(getenv("WGS")) : 64;
  std::vector<hipStream_t> extra(4);
  for (auto& x : extra) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  const char* modes[] = {"default", "nocu_d2h", "nocu_both", "h2d_only", "d2h_only", "d2h_only_nocu",
                         "d2h_streams2", "d2h_streams4", "both_streams2", "both_streams4", "d2h_kernel", "both_kernel"};
  for (const char* m : modes) {
    const bool h2d = strncmp(m, "d2h_", 4) != 0;
    const bool d2h = strcmp(m, "h2d_only") != 0;
    const int ks = strstr(m, "streams4") ? 4 : strstr(m, "streams2") ? 2 : 1;
    const bool kern = strstr(m, "kernel") != nullptr;
    const bool nocu_d = strstr(m, "nocu") != nullptr;
    const bool nocu_h = strcmp(m, "nocu_both") == 0;
    std::vector<float> th, td;
    for (int r = 0; r < reps + 1; r++) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a0, sh));
      CK(hipEventRecord(b0, sd));
      for (int k = 0; k < ks && ks > 1; k++) CK(hipStreamWaitEvent(extra[k], b0, 0));
      for (int i = 0; i < pieces; i++) {
        if (h2d)
          CK(hipMemcpyAsync(din + i * piece, hin + i * piece, piece,
                            nocu_h ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyHostToDevice, sh));
        if (d2h && kern) {
          hipLaunchKernelGGL(d2h_copy, dim3(wgs), dim3(256), 0, sd, (const u32x4*)(dout + i * piece),
                             (u32x4*)(hout + i * piece), piece / 16);
          CK(hipGetLastError());
        } else if (d2h) {
          hipStream_t q = ks == 1 ? sd : extra[i % ks];
          CK(hipMemcpyAsync(hout + i * piece, dout + i * piece, piece,
                            nocu_d ? hipMemcpyDeviceToDeviceNoCU : hipMemcpyDeviceToHost, q));
        }
      }
      if (ks > 1) {  // (the extra streams join sd before its end event)
        for (int k = 0; k < ks; k++) {
          hipEvent_t e;
          CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
          CK(hipEventRecord(e, extra[k]));
          CK(hipStreamWaitEvent(sd, e, 0));
          CK(hipEventDestroy(e));
        }
      }
      CK(hipEventRecord(a1, sh));
      CK(hipEventRecord(b1, sd));
      CK(hipDeviceSynchronize());
      float x = 0, y = 0;
      CK(hipEventElapsedTime(&x, a0, a1));
      CK(hipEventElapsedTime(&y, b0, b1));
      if (r) th.push_back(x), td.push_back(y);
    }
    auto med = [](std::vector<float> v) {
      std::sort(v.begin(), v.end());
      return v[v.size() / 2];
    };
    const double gib = (double)piece * pieces / (1 << 30);
    printf("{\"mode\": \"%s\", \"bytes_each_way\": %zu, \"h2d_ms\": %.3f, \"h2d_gib_s\": %.1f, \"d2h_ms\": %.3f, "
           "\"d2h_gib_s\": %.1f}\n", m, piece * pieces, h2d ? med(th) : 0.0, h2d ? gib / (med(th) / 1e3) : 0.0,
           d2h ? med(td) : 0.0, d2h ? gib / (med(td) / 1e3) : 0.0);
    fflush(stdout);
  }
  // the bytes landed (the NoCU modes must copy too)
  CK(hipMemcpy(hout, dout, piece, hipMemcpyDeviceToHost));
  printf("{\"check\": %s}\n", hout[piece - 1] == 2 ? "\"ok\"" : "\"BAD\"");
  return 0;
}
