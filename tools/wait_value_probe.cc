// wait_value_probe.cc - can one stream wait, on the device, for a bucket that a kernel running on
// another stream has finished (hipStreamWaitValue64 on signal memory), before that kernel ends?
// The fused pack's one-launch form (fusion.cc) rests on it.
//
// Stream A: one long kernel of G workgroups over two halves ("buckets") of a buffer; the last
// workgroup of each half (a device counter per half, reset by that workgroup) stores the half's
// target into that half's signal word (system-scope release). Stream B: wait for half 0's signal,
// then a kernel that checks half 0's bytes and records the device clock. Prints whether B's kernel
// saw every byte, and when it started relative to A's end (negative: it overlapped A).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      printf("{\"ok\": false, \"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));     \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

__global__ void fill_halves(unsigned* buf, long n, unsigned val, unsigned* counters, unsigned long long** sig,
                            unsigned long long target, long long* t_end, int spin) {
  const long half = n / 2;
  const int h = blockIdx.x < gridDim.x / 2 ? 0 : 1;
  const long per = half / (gridDim.x / 2);
  const long b0 = h * half + (long)(blockIdx.x - h * (gridDim.x / 2)) * per;
  for (long i = b0 + threadIdx.x; i < b0 + per; i += blockDim.x) buf[i] = val + (unsigned)i;
  if (h == 1)  // the second half is slow: half 0's waiter should start well before the launch ends
    for (int k = 0; k < spin; k++) __builtin_amdgcn_s_sleep(127);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned last = gridDim.x / 2 - 1;
    if (__hip_atomic_fetch_add(&counters[h], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == last) {
      __hip_atomic_store(&counters[h], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sig[h], target, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (h == 1) *t_end = (long long)wall_clock64();
    }
  }
}

__global__ void check_half(const unsigned* buf, long n, unsigned val, int* bad, long long* t_start) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *t_start = (long long)wall_clock64();
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n / 2; i += (long)gridDim.x * blockDim.x)
    if (buf[i] != val + (unsigned)i) atomicAdd(bad, 1);
}

int main(int argc, char** argv) {
  const int spin = argc > 1 ? atoi(argv[1]) : 200;
  int can = 0;
  CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0));
  const long n = 64L << 20;  // 256 MiB of u32
  unsigned* buf;
  unsigned* counters;
  long long* times;
  int* bad;
  void* sigp[2] = {};
  CK(hipMalloc(&buf, n * 4));
  CK(hipMalloc(&counters, 64));
  CK(hipMemset(counters, 0, 64));
  CK(hipMalloc(&times, 64));
  CK(hipMalloc(&bad, 4));
  // (one 8-byte signal word per allocation; the kernel gets both through a device array)
  CK(hipExtMallocWithFlags(&sigp[0], 8, hipMallocSignalMemory));
  CK(hipExtMallocWithFlags(&sigp[1], 8, hipMallocSignalMemory));
  CK(hipMemset(sigp[0], 0, 8));
  CK(hipMemset(sigp[1], 0, 8));
  unsigned long long** sig = nullptr;
  CK(hipMalloc(&sig, 16));
  CK(hipMemcpy(sig, sigp, 16, hipMemcpyHostToDevice));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  CK(hipDeviceSynchronize());
  int fails = 0;
  double overlap_us_sum = 0;
  const int reps = 20;
  long long clk_hz = 100000000;  // wall_clock64: 100 MHz on gfx9
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0) == hipSuccess && khz > 0) clk_hz = (long long)khz * 1000;
  for (int r = 1; r <= reps; r++) {
    CK(hipMemsetAsync(bad, 0, 4, b));
    fill_halves<<<2048, 256, 0, a>>>(buf, n, 1000u * r, counters, sig, (unsigned long long)r, times, spin);
    CK(hipGetLastError());
    CK(hipStreamWaitValue64(b, sigp[0], (uint64_t)r, hipStreamWaitValueGte));
    check_half<<<1024, 256, 0, b>>>(buf, n, 1000u * r, bad, times + 1);
    CK(hipDeviceSynchronize());
    long long t[2];
    int nb = 0;
    CK(hipMemcpy(t, times, 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
    fails += nb != 0;
    overlap_us_sum += (double)(t[1] - t[0]) * 1e6 / (double)clk_hz;
  }
  printf("{\"ok\": %s, \"can_use_stream_wait_value\": %d, \"reps\": %d, \"reps_with_stale_bytes\": %d, "
         "\"mean_waiter_start_minus_fill_end_us\": %.2f, \"spin\": %d}\n",
         fails == 0 ? "true" : "false", can, reps, fails, overlap_us_sum / reps, spin);
  return fails == 0 ? 0 : 3;
}
