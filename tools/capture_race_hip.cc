// capture_race_hip.cc - does the HIP runtime alone (no RCCL, no libtips_hip) survive a relaxed-mode
// stream capture on one thread while other threads of the process make ordinary HIP calls?
//
// The capturing thread repeats what a captured tips plan does once RCCL is inside it
// (schedules.cc capture_plan + RCCL's ncclGroupEnd under capture): begin a relaxed capture on a
// non-blocking stream, fork a second non-blocking stream into it by an event, launch kernels on
// both, add a host function on the forked stream (RCCL's proxy hand-over) and retain a user object
// on the capture's graph (RCCL's persistent-plan destructor), join, end, instantiate, replay, check.
//
// Churn threads (argv[1]):
//   none      no other thread
//   async     non-blocking streams, hipMemcpyAsync + hipStreamSynchronize on them (buffers fixed)
//   streams   hipStreamCreate (blocking) / hipStreamDestroy only
//   free      non-blocking streams; hipMalloc / hipFree every iteration
//   legacy    hipMemcpy / hipMemset on the legacy null stream (buffers fixed)
//   all       blocking streams, hipMalloc, hipMemcpy, hipMemset, hipFree (tests/c/op_body.c's mix)
// argv[2]: seconds to run (default 15). argv[3]: the capture mode, relaxed (default) | thread | global.
// A failed call does not end the run: churn errors and captures that failed (the capture then ends
// and its graph, if any, is dropped) are counted. Prints one JSON line; exit 0 = no failure. A
// watchdog prints progress every second and, when the capturing thread makes no progress for 10 s,
// every thread's stack (module+offset frames) and exits 5: a stall, not a time limit.
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <dirent.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <chrono>

#include <atomic>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

__global__ void add_one(int* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1;
}

std::atomic<bool> g_stop{false};
std::atomic<long> g_iters{0};
std::atomic<int> g_phase{0};  // where the capturing thread is (the stall report)

void on_usr1(int) {
  void* fr[48];
  const int n = backtrace(fr, 48);
  char hdr[64];
  const int l = snprintf(hdr, sizeof hdr, "--- thread %ld\n", (long)syscall(SYS_gettid));
  if (write(2, hdr, (size_t)l) < 0) return;
  backtrace_symbols_fd(fr, n, 2);
}

void dump_stacks() {
  signal(SIGUSR1, on_usr1);
  const long self = (long)syscall(SYS_gettid);
  DIR* d = opendir("/proc/self/task");
  if (!d) return;
  while (dirent* e = readdir(d)) {
    const long tid = atol(e->d_name);
    if (tid <= 0 || tid == self) continue;
    syscall(SYS_tgkill, (long)getpid(), tid, SIGUSR1);
    usleep(50000);
  }
  closedir(d);
}
std::atomic<long> g_churn_ops{0};
std::atomic<long> g_churn_errors{0};
std::atomic<long> g_capture_failures{0};
std::string g_first_capture_error, g_first_churn_error;
std::mutex g_err_mu;
std::atomic<int> g_host_fn{0};
std::atomic<int> g_destroyed{0};

void host_fn(void*) { g_host_fn.fetch_add(1, std::memory_order_relaxed); }
void destroy_fn(void*) { g_destroyed.fetch_add(1, std::memory_order_relaxed); }

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return false;                                                                  \
    }                                                                                \
  } while (0)

bool churn(const std::string& mode, int id) {
  const size_t n = 1 << 16;
  std::vector<int> h(n, id);
  int* fixed = nullptr;
  CK(hipMalloc(&fixed, n * sizeof(int)));
  hipStream_t own = nullptr;
  if (mode == "async" || mode == "legacy") CK(hipStreamCreateWithFlags(&own, hipStreamNonBlocking));
  while (!g_stop.load(std::memory_order_relaxed)) {
    if (mode == "async") {
      CK(hipMemcpyAsync(fixed, h.data(), n * sizeof(int), hipMemcpyHostToDevice, own));
      CK(hipStreamSynchronize(own));
      CK(hipMemcpyAsync(h.data(), fixed, n * sizeof(int), hipMemcpyDeviceToHost, own));
      CK(hipStreamSynchronize(own));
    } else if (mode == "streams") {
      hipStream_t s;
      CK(hipStreamCreate(&s));
      CK(hipStreamDestroy(s));
    } else if (mode == "free") {
      hipStream_t s;
      int* d = nullptr;
      CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      CK(hipMalloc(&d, n * sizeof(int)));
      CK(hipMemcpyAsync(d, h.data(), n * sizeof(int), hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      CK(hipFree(d));
      CK(hipStreamDestroy(s));
    } else if (mode == "legacy") {
      for (hipError_t e : {hipMemcpy(fixed, h.data(), n * sizeof(int), hipMemcpyHostToDevice),
                           hipMemset(fixed, 0, n * sizeof(int)),
                           hipMemcpy(h.data(), fixed, n * sizeof(int), hipMemcpyDeviceToHost)})
        if (e != hipSuccess) {
          if (g_churn_errors.fetch_add(1) == 0) {
            std::lock_guard<std::mutex> l(g_err_mu);
            g_first_churn_error = hipGetErrorString(e);
          }
          (void)hipGetLastError();
        }
    } else if (mode == "all") {
      hipStream_t s;
      int* d = nullptr;
      CK(hipStreamCreate(&s));
      CK(hipMalloc(&d, n * sizeof(int)));
      CK(hipMemcpy(d, h.data(), n * sizeof(int), hipMemcpyHostToDevice));
      CK(hipMemset(d, 0, n * sizeof(int)));
      CK(hipMemcpy(h.data(), d, n * sizeof(int), hipMemcpyDeviceToHost));
      CK(hipFree(d));
      CK(hipStreamDestroy(s));
    } else {
      return true;
    }
    g_churn_ops.fetch_add(1, std::memory_order_relaxed);
  }
  (void)hipFree(fixed);
  if (own) (void)hipStreamDestroy(own);
  return true;
}

hipStreamCaptureMode g_mode = hipStreamCaptureModeRelaxed;

struct Cap {
  hipStream_t gs, fs;
  hipEvent_t fork, join;
  int *a, *b;
  int n;
};

void capture_failed(const char* what, hipError_t e) {
  if (g_capture_failures.fetch_add(1) == 0) {
    std::lock_guard<std::mutex> l(g_err_mu);
    g_first_capture_error = std::string(what) + ": " + hipGetErrorString(e);
  }
  (void)hipGetLastError();
}

// One capture + replay; false (counted) when a call failed. The capture is always ended.
bool capture_once(Cap& c) {
#define CC(x)                        \
  do {                               \
    hipError_t e_ = (x);             \
    if (e_ != hipSuccess) {          \
      capture_failed(#x, e_);        \
      ok = false;                    \
    }                                \
  } while (0)
  bool ok = true;
  g_phase = 1;
  CC(hipStreamBeginCapture(c.gs, g_mode));
  if (!ok) return false;
  CC(hipEventRecord(c.fork, c.gs));
  if (ok) CC(hipStreamWaitEvent(c.fs, c.fork, 0));
  if (ok) {
    add_one<<<c.n / 256, 256, 0, c.gs>>>(c.a, c.n);
    add_one<<<c.n / 256, 256, 0, c.fs>>>(c.b, c.n);
    CC(hipGetLastError());
  }
  if (ok) CC(hipLaunchHostFunc(c.fs, host_fn, nullptr));
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t cg = nullptr;
  if (ok) CC(hipStreamGetCaptureInfo_v2(c.gs, &cs, &id, &cg, nullptr, nullptr));
  if (ok && cs != hipStreamCaptureStatusActive) {
    capture_failed("capture status not active", hipErrorStreamCaptureInvalidated);
    ok = false;
  }
  if (ok) {
    hipUserObject_t uo = nullptr;
    CC(hipUserObjectCreate(&uo, nullptr, destroy_fn, 1, hipUserObjectNoDestructorSync));
    if (ok) CC(hipGraphRetainUserObject(cg, uo, 1, hipGraphUserObjectMove));
  }
  // join the forked stream back (also on failure, so that it leaves the capture)
  (void)hipEventRecord(c.join, c.fs);
  (void)hipStreamWaitEvent(c.gs, c.join, 0);
  hipGraph_t g = nullptr;
  g_phase = 2;
  const hipError_t ee = hipStreamEndCapture(c.gs, &g);
  if (ok && ee != hipSuccess) CC(ee);
  (void)hipGetLastError();
  if (ok && g) {
    hipGraphExec_t ex = nullptr;
    g_phase = 3;
    CC(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    if (ok) {
      g_phase = 4;
      CC(hipGraphLaunch(ex, c.gs));
      g_phase = 5;
      CC(hipStreamSynchronize(c.gs));
      g_phase = 6;
      (void)hipGraphExecDestroy(ex);
    }
  }
  if (g) (void)hipGraphDestroy(g);
#undef CC
  return ok;
}

bool capture_loop(double seconds, int* bad) {
  Cap c{};
  c.n = 4096;
  CK(hipMalloc(&c.a, c.n * sizeof(int)));
  CK(hipMalloc(&c.b, c.n * sizeof(int)));
  CK(hipMemset(c.a, 0, c.n * sizeof(int)));
  CK(hipMemset(c.b, 0, c.n * sizeof(int)));
  CK(hipDeviceSynchronize());
  CK(hipStreamCreateWithFlags(&c.gs, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c.fs, hipStreamNonBlocking));
  CK(hipEventCreateWithFlags(&c.fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&c.join, hipEventDisableTiming));
  std::vector<int> h(c.n);
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(seconds);
  long replays = 0;
  for (int it = 0; std::chrono::steady_clock::now() < t_end; it++) {
    if (capture_once(c)) replays++;
    g_iters.fetch_add(1);
    if (it % 100 == 99) {  // (a failed capture replays nothing: a counts the good ones)
      CK(hipMemcpyAsync(h.data(), c.a, c.n * sizeof(int), hipMemcpyDeviceToHost, c.gs));
      CK(hipStreamSynchronize(c.gs));
      for (int j = 0; j < c.n; j++)
        if (h[j] != (int)replays) {
          (*bad)++;
          break;
        }
    }
  }
  (void)hipStreamDestroy(c.gs);
  (void)hipStreamDestroy(c.fs);
  (void)hipFree(c.a);
  (void)hipFree(c.b);
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "all";
  const double seconds = argc > 2 ? atof(argv[2]) : 15.0;
  const std::string cmode = argc > 3 ? argv[3] : "relaxed";
  g_mode = cmode == "thread" ? hipStreamCaptureModeThreadLocal
           : cmode == "global" ? hipStreamCaptureModeGlobal
                               : hipStreamCaptureModeRelaxed;
  if (hipSetDevice(0) != hipSuccess) return 2;
  std::thread([&] {  // watchdog (detached: the process ends with main)
    long last = -1;
    int still = 0;
    for (int t = 1;; t++) {
      sleep(1);
      const long it = g_iters.load();
      fprintf(stderr, "[capture_race_hip %s] t=%ds captures %ld churn %ld phase %d\n", mode.c_str(), t, it,
              g_churn_ops.load(), g_phase.load());
      still = it == last ? still + 1 : 0;
      last = it;
      if (still >= 10) {
        fprintf(stderr, "[capture_race_hip %s] STALLED at phase %d\n", mode.c_str(), g_phase.load());
        dump_stacks();
        printf("{\"mode\": \"%s\", \"stalled\": true, \"phase\": %d, \"captures\": %ld, \"churn_ops\": %ld}\n",
               mode.c_str(), g_phase.load(), it, g_churn_ops.load());
        fflush(stdout);
        _exit(5);
      }
    }
  }).detach();
  std::vector<std::thread> th;
  std::atomic<int> churn_fail{0};
  if (mode != "none")
    for (int k = 0; k < 3; k++) th.emplace_back([&, k] { if (!churn(mode, k)) churn_fail++; });
  int bad = 0;
  const bool ok = capture_loop(seconds, &bad);
  g_stop = true;
  for (auto& t : th) t.join();
  (void)hipDeviceSynchronize();
  printf("{\"mode\": \"%s\", \"capture_mode\": \"%s\", \"captures\": %ld, \"capture_failures\": %ld, "
         "\"first_capture_error\": \"%s\", \"bad_replays\": %d, \"churn_ops\": %ld, \"churn_errors\": %ld, "
         "\"first_churn_error\": \"%s\", \"churn_failed\": %d, \"host_fns\": %d, \"user_objects_destroyed\": %d}\n",
         mode.c_str(), cmode.c_str(), g_iters.load(), g_capture_failures.load(), g_first_capture_error.c_str(), bad,
         g_churn_ops.load(), g_churn_errors.load(), g_first_churn_error.c_str(), churn_fail.load(), g_host_fn.load(),
         g_destroyed.load());
  return ok && bad == 0 && churn_fail == 0 && g_capture_failures == 0 && g_churn_errors == 0 ? 0 : 1;
}
