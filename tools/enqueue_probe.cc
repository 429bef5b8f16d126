// enqueue_probe.cc — what the HIP calls a named-request enqueue makes cost on this box (diagnostic).
//
// A TF-style host enqueues one request per gradient from executor threads; tips_enqueue_* asks
// hipPointerGetAttributes whether each pointer is device memory. This times that call on pageable
// host memory (config 5's 214 gradient sizes), on page-locked memory and on device memory, from one
// thread and from four at once, next to hipSetDevice and an uncontended / contended std::mutex.
// Build: make tools/_bin/enqueue_probe. Prints one JSON line (ns per call).
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

static double ns_per(int n, const std::chrono::steady_clock::time_point& t0) {
  return std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count() / n;
}

int main() {
  if (hipSetDevice(0) != hipSuccess) {
    fprintf(stderr, "no device\n");
    return 1;
  }
  const int kBufs = 214, kIters = 20000;
  std::vector<void*> host(kBufs);
  for (int i = 0; i < kBufs; i++) {
    const size_t bytes = (size_t)4 << (8 + i % 14);  // 1 KiB .. 8 MiB, as config 5's spread
    host[i] = malloc(bytes);
    if (!host[i]) return 1;
    ((char*)host[i])[0] = 1;
  }
  void *pinned = nullptr, *dev = nullptr;
  if (hipHostMalloc(&pinned, 1 << 20, hipHostMallocDefault) != hipSuccess || hipMalloc(&dev, 1 << 20) != hipSuccess) return 1;
  auto attr = [](const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    return (int)a.type;
  };
  volatile int sink = 0;
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < kIters; i++) sink += attr(host[i % kBufs]);
  const double pageable = ns_per(kIters, t0);
  t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < kIters; i++) sink += attr(pinned);
  const double locked = ns_per(kIters, t0);
  t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < kIters; i++) sink += attr(dev);
  const double device = ns_per(kIters, t0);
  t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < kIters; i++) (void)hipSetDevice(0);
  const double setdev = ns_per(kIters, t0);
  std::mutex mu;
  t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < kIters; i++) {
    std::lock_guard<std::mutex> l(mu);
    sink += i;
  }
  const double lock1 = ns_per(kIters, t0);
  // four threads at once: the pageable lookup, and a short critical section on one mutex
  auto four = [&](auto body) {
    std::atomic<int> go{0};
    std::vector<std::thread> th;
    for (int t = 0; t < 4; t++)
      th.emplace_back([&, t] {
        while (!go.load()) {
        }
        for (int i = 0; i < kIters; i++) body(t, i);
      });
    const auto s = std::chrono::steady_clock::now();
    go = 1;
    for (auto& x : th) x.join();
    return ns_per(kIters, s);  // wall ns per iteration of each thread
  };
  const double pageable4 = four([&](int t, int i) { sink += attr(host[(i + 50 * t) % kBufs]); });
  const double lock4 = four([&](int, int i) {
    std::lock_guard<std::mutex> l(mu);
    sink += i;
  });
  printf("{\"pageable_attr_ns\": %.1f, \"pinned_attr_ns\": %.1f, \"device_attr_ns\": %.1f, \"set_device_ns\": %.1f, "
         "\"mutex_ns\": %.1f, \"pageable_attr_4threads_wall_ns\": %.1f, \"mutex_4threads_wall_ns\": %.1f}\n",
         pageable, locked, device, setdev, lock1, pageable4, lock4);
  for (void* p : host) free(p);
  (void)hipHostFree(pinned);
  (void)hipFree(dev);
  return sink == 42 ? 2 : 0;
}
