// host_staging.cc — the host-memory leg of the path. The reference's op works
// on TF CPU tensors (tips/tensorflow/ops.cc:88-90), so gradients arrive in
// host memory and must return there: this file moves them through HBM with
// both PCIe directions and the device allreduce overlapped.
#include <algorithm>
#include <condition_variable>
#include <thread>

#include "rt.h"

namespace tips {
namespace rt {

int ensure_bounce(State& st) {
  if (!st.bounce_in) HIP_TRY(hipHostMalloc(&st.bounce_in, kBounceBytes, hipHostMallocDefault));
  if (!st.bounce_out) HIP_TRY(hipHostMalloc(&st.bounce_out, kBounceBytes, hipHostMallocDefault));
  return 0;
}

// Host-resident allreduce, pipelined over pieces so both PCIe directions and
// the device work overlap: H2D of piece i+1 (h2d stream) || allreduce of piece
// i (io stream) || D2H of piece i-1 (d2h stream). Each piece is a complete
// allreduce (same piece boundaries on every rank). When both buffers are
// page-locked every copy is asynchronous and one thread issues all three
// stages; otherwise a second host thread issues the D2H copies, because a
// copy from/to pageable memory blocks the thread that issues it. Caller holds
// st.mu; returns when `out` is written.
int allreduce_host_pipelined(State& st, const char* in, char* out, int64_t n, int dtype) {
  const int64_t es = tips::dtype_size(dtype);
  const int64_t piece =
      round_up(std::max<int64_t>(kAlignBytes, env_i64("TIPS_HOST_PIECE_BYTES", kHostPieceBytes)), kAlignBytes) / es;
  const int np = (int)((n + piece - 1) / piece);
  TRY(st.host_in.ensure((size_t)(n * es)));
  TRY(st.host_out.ensure((size_t)(n * es)));
  TRY(st.pipe_ev.ensure(2 * (size_t)np));
  char* din = (char*)st.host_in.p;
  char* dout = (char*)st.host_out.p;
  if (is_pinned_host(in, n * es) && is_pinned_host(out, n * es)) {
    for (int i = 0; i < np; i++) {
      const int64_t off = (int64_t)i * piece * es, cnt = std::min(piece, n - (int64_t)i * piece);
      HIP_TRY(hipMemcpyAsync(din + off, in + off, (size_t)(cnt * es), hipMemcpyHostToDevice, st.h2d_stream));
      HIP_TRY(hipEventRecord(st.pipe_ev.ev[2 * i], st.h2d_stream));
      HIP_TRY(hipStreamWaitEvent(st.io_stream, st.pipe_ev.ev[2 * i], 0));
      TRY(allreduce_device(st, din + off, dout + off, cnt, dtype, st.io_stream));
      HIP_TRY(hipEventRecord(st.pipe_ev.ev[2 * i + 1], st.io_stream));
      HIP_TRY(hipStreamWaitEvent(st.d2h_stream, st.pipe_ev.ev[2 * i + 1], 0));
      HIP_TRY(hipMemcpyAsync(out + off, dout + off, (size_t)(cnt * es), hipMemcpyDeviceToHost, st.d2h_stream));
    }
    HIP_TRY(hipStreamSynchronize(st.d2h_stream));
    return 0;
  }
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

}  // namespace rt
}  // namespace tips

using namespace tips::rt;

extern "C" {

int tips_host_register(void* ptr, int64_t bytes) {
  if (!ptr || bytes <= 0) return fail(TIPS_ERR_INVALID_ARG, "bad host range");
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  TRY(set_device(st));
  HIP_TRY(hipHostRegister(ptr, (size_t)bytes, hipHostRegisterDefault));
  return 0;
}

int tips_host_unregister(void* ptr) {
  if (!ptr) return fail(TIPS_ERR_INVALID_ARG, "null pointer");
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  TRY(set_device(st));
  HIP_TRY(hipHostUnregister(ptr));
  return 0;
}

}  // extern "C"
