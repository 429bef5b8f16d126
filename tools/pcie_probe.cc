// pcie_probe.cc — host-link measurements behind the host-staging design (DESIGN.md §host staging).
//
// On one MI355X, with 256 MiB pinned host buffers, it compares the DMA
// engines (hipMemcpyAsync) with copy kernels that read or write host memory
// directly through its device mapping (zero-copy). It measures each direction
// alone and both directions at once. Prints one JSON line per case, in GB/s
// (1e9 B/s).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// grid-stride 16-B copy; U vectors in flight per lane
template <int U>
__global__ __launch_bounds__(256) void copy16(u32x4* __restrict__ dst, const u32x4* __restrict__ src, int64_t nvec) {
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  for (int64_t i = (int64_t)blockIdx.x * 256 * U + threadIdx.x; i < nvec; i += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (i + u * 256 < nvec) v[u] = __builtin_nontemporal_load(src + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++)
      if (i + u * 256 < nvec) __builtin_nontemporal_store(v[u], dst + i + u * 256);
  }
}

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? atoll(argv[1]) : 256) << 20;
  const int iters = argc > 2 ? atoi(argv[2]) : 10;
  const int64_t nvec = (int64_t)(bytes / 16);
  void *h_in, *h_out, *d_in, *d_out;
  CHECK(hipHostMalloc(&h_in, bytes, hipHostMallocMapped));
  CHECK(hipHostMalloc(&h_out, bytes, hipHostMallocMapped));
  memset(h_in, 1, bytes);
  memset(h_out, 0, bytes);
  CHECK(hipMalloc(&d_in, bytes));
  CHECK(hipMalloc(&d_out, bytes));
  void *m_in, *m_out;  // device views of the pinned host buffers
  CHECK(hipHostGetDevicePointer(&m_in, h_in, 0));
  CHECK(hipHostGetDevicePointer(&m_out, h_out, 0));
  hipStream_t s1, s2;
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));

  auto timeit = [&](const std::string& name, double moved_bytes, auto&& body) {
    body();  // warm
    CHECK(hipDeviceSynchronize());
    std::vector<double> ms;
    for (int r = 0; r < iters; r++) {
      CHECK(hipEventRecord(e0, 0));
      CHECK(hipStreamWaitEvent(s1, e0, 0));
      CHECK(hipStreamWaitEvent(s2, e0, 0));
      body();
      hipEvent_t a, b;
      CHECK(hipEventCreate(&a));
      CHECK(hipEventCreate(&b));
      CHECK(hipEventRecord(a, s1));
      CHECK(hipEventRecord(b, s2));
      CHECK(hipStreamWaitEvent(0, a, 0));
      CHECK(hipStreamWaitEvent(0, b, 0));
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float t = 0;
      CHECK(hipEventElapsedTime(&t, e0, e1));
      ms.push_back(t);
      CHECK(hipEventDestroy(a));
      CHECK(hipEventDestroy(b));
    }
    std::sort(ms.begin(), ms.end());
    const double med = ms[ms.size() / 2];
    printf("{\"case\": \"%s\", \"bytes\": %.0f, \"median_ms\": %.3f, \"GBps\": %.2f, \"GBps_best\": %.2f}\n",
           name.c_str(), moved_bytes, med, moved_bytes / (med * 1e-3) / 1e9, moved_bytes / (ms[0] * 1e-3) / 1e9);
    fflush(stdout);
  };
  const double B = (double)bytes;
  timeit("dma_h2d", B, [&] { CHECK(hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, s1)); });
  timeit("dma_d2h", B, [&] { CHECK(hipMemcpyAsync(h_out, d_out, bytes, hipMemcpyDeviceToHost, s1)); });
  timeit("dma_h2d+d2h", 2 * B, [&] {
    CHECK(hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, s1));
    CHECK(hipMemcpyAsync(h_out, d_out, bytes, hipMemcpyDeviceToHost, s2));
  });
  const size_t piece = 32 << 20;
  timeit("dma_h2d_32MiB_pieces", B, [&] {
    for (size_t o = 0; o < bytes; o += piece)
      CHECK(hipMemcpyAsync((char*)d_in + o, (char*)h_in + o, std::min(piece, bytes - o), hipMemcpyHostToDevice, s1));
  });
  for (int blocks : {256, 1024, 4096}) {
    const std::string g = "_g" + std::to_string(blocks);
    timeit("kern_h2d" + g, B, [&] {
      hipLaunchKernelGGL(copy16<4>, dim3(blocks), dim3(256), 0, s1, (u32x4*)d_in, (const u32x4*)m_in, nvec);
    });
    timeit("kern_d2h" + g, B, [&] {
      hipLaunchKernelGGL(copy16<4>, dim3(blocks), dim3(256), 0, s1, (u32x4*)m_out, (const u32x4*)d_out, nvec);
    });
    timeit("kern_h2d+d2h" + g, 2 * B, [&] {
      hipLaunchKernelGGL(copy16<4>, dim3(blocks), dim3(256), 0, s1, (u32x4*)d_in, (const u32x4*)m_in, nvec);
      hipLaunchKernelGGL(copy16<4>, dim3(blocks), dim3(256), 0, s2, (u32x4*)m_out, (const u32x4*)d_out, nvec);
    });
  }
  timeit("dma_h2d+kern_d2h_g1024", 2 * B, [&] {
    CHECK(hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, s1));
    hipLaunchKernelGGL(copy16<4>, dim3(1024), dim3(256), 0, s2, (u32x4*)m_out, (const u32x4*)d_out, nvec);
  });
  timeit("kern_h2d_g1024+dma_d2h", 2 * B, [&] {
    hipLaunchKernelGGL(copy16<4>, dim3(1024), dim3(256), 0, s1, (u32x4*)d_in, (const u32x4*)m_in, nvec);
    CHECK(hipMemcpyAsync(h_out, d_out, bytes, hipMemcpyDeviceToHost, s2));
  });
  // host -> host through the device mapping in one kernel (a 1-rank host allreduce with no staging)
  timeit("kern_h2h_g1024", 2 * B, [&] {
    hipLaunchKernelGGL(copy16<4>, dim3(1024), dim3(256), 0, s1, (u32x4*)m_out, (const u32x4*)m_in, nvec);
  });
  // the host-staging pipeline shape (host_staging.cc) issued from ONE thread: H2D piece i (s1) ->
  // device stage (s3: D2D copy, the 1-rank allreduce) -> D2H piece i (s2), events between the stages
  hipStream_t s3;
  CHECK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(2 * (bytes / (1 << 20)) + 2);
  for (auto& x : ev) CHECK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  for (int stage : {1, 0})
    for (size_t pmib : {4, 8, 16, 32, 64}) {
      const size_t pc = pmib << 20;
      const std::string nm = std::string(stage ? "pipe_h2d_d2d_d2h_" : "pipe_h2d_d2h_") + std::to_string(pmib) + "MiB";
      timeit(nm, B, [&] {
        int k = 0;
        for (size_t o = 0; o < bytes; o += pc, k++) {
          const size_t len = std::min(pc, bytes - o);
          CHECK(hipMemcpyAsync((char*)d_in + o, (char*)h_in + o, len, hipMemcpyHostToDevice, s1));
          CHECK(hipEventRecord(ev[2 * k], s1));
          const void* src = (char*)d_in + o;
          if (stage) {
            CHECK(hipStreamWaitEvent(s3, ev[2 * k], 0));
            CHECK(hipMemcpyAsync((char*)d_out + o, src, len, hipMemcpyDeviceToDevice, s3));
            CHECK(hipEventRecord(ev[2 * k + 1], s3));
            src = (char*)d_out + o;
          }
          CHECK(hipStreamWaitEvent(s2, ev[2 * k + stage], 0));
          CHECK(hipMemcpyAsync((char*)h_out + o, src, len, hipMemcpyDeviceToHost, s2));
        }
        // s3 joins the timing through s2's last wait
      });
    }
  // HW-queue sharing: GPU_MAX_HW_QUEUES (4 here) queues are dealt to streams in creation order.
  // Bidirectional DMA on a stream pair k apart, k = 1..8: a pair that lands on one queue serializes.
  {
    std::vector<hipStream_t> extra(9);
    for (auto& x : extra) CHECK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    for (int k = 1; k <= 8; k++) {
      timeit("dma_h2d+d2h_streams_" + std::to_string(k) + "_apart", 2 * B, [&] {
        CHECK(hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, extra[0]));
        CHECK(hipMemcpyAsync(h_out, d_out, bytes, hipMemcpyDeviceToHost, extra[k]));
        hipEvent_t a, b;
        CHECK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
        CHECK(hipEventCreateWithFlags(&b, hipEventDisableTiming));
        CHECK(hipEventRecord(a, extra[0]));
        CHECK(hipEventRecord(b, extra[k]));
        CHECK(hipStreamWaitEvent(s1, a, 0));
        CHECK(hipStreamWaitEvent(s2, b, 0));
        CHECK(hipEventDestroy(a));
        CHECK(hipEventDestroy(b));
      });
    }
    int lo = 0, hi = 0;
    CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    hipStream_t p1, p2;
    CHECK(hipStreamCreateWithPriority(&p1, hipStreamNonBlocking, hi));
    CHECK(hipStreamCreateWithPriority(&p2, hipStreamNonBlocking, hi));
    timeit("dma_h2d+d2h_high_priority_pair", 2 * B, [&] {
      CHECK(hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, p1));
      CHECK(hipMemcpyAsync(h_out, d_out, bytes, hipMemcpyDeviceToHost, p2));
      hipEvent_t a, b;
      CHECK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
      CHECK(hipEventCreateWithFlags(&b, hipEventDisableTiming));
      CHECK(hipEventRecord(a, p1));
      CHECK(hipEventRecord(b, p2));
      CHECK(hipStreamWaitEvent(s1, a, 0));
      CHECK(hipStreamWaitEvent(s2, b, 0));
      CHECK(hipEventDestroy(a));
      CHECK(hipEventDestroy(b));
    });
  }
  CHECK(hipDeviceSynchronize());
  // sanity: the last kernel copied h_in into h_out
  if (memcmp(h_in, h_out, bytes) != 0) {
    fprintf(stderr, "zero-copy result mismatch\n");
    return 1;
  }
  return 0;
}
