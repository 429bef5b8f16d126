// host_staging.cc — the host-memory leg of the path. The reference's op works
// on TF CPU tensors (tips/tensorflow/ops.cc:88-90), so gradients arrive in
// host memory and must return there: this file moves them through HBM with
// both PCIe directions and the device allreduce overlapped.
#include <immintrin.h>
#include <sched.h>

#include <algorithm>
#include <array>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <thread>

#include <pthread.h>

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

// ---------------------------------------------------------------------------
// Many host tensors, fused (round 3). The reference's op is a CPU op (ops.cc:118): a model's
// gradients arrive as many host tensors. One staged allreduce per tensor pays the host link's
// latency per tensor (config 5: 214 tensors, 8.6 GiB/s); here the list is packed by host threads
// into page-locked pieces of a flat byte stream (the layout a function of the counts alone, 64-B
// aligned offsets), and each piece runs H2D -> allreduce in place in HBM -> D2H on three streams
// while the threads pack the next piece and unpack the previous one.

// A fused host call runs its pool once per piece and direction, 20 fork-joins for config 5, each
// a few hundred microseconds apart: a worker that blocked on the condition variable between them
// pays a futex wake-up and a reschedule every time. Workers (and the caller waiting for its jobs)
// therefore spin for TIPS_HOST_SPIN_US (300 us) before they block, which keeps them hot through one
// call and idle between calls.
namespace {
inline int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

HostPool::HostPool(int nthreads) : spin_ns_(std::max<int64_t>(0, env_i64("TIPS_HOST_SPIN_US", 300)) * 1000) {
  for (int i = 1; i < nthreads; i++)
    th_.emplace_back([this, i] {
      (void)pthread_setname_np(pthread_self(), "tips-host");  // (/proc/<pid>/task/*/comm: placement records)
      worker(i - 1);
    });
}

namespace {
bool read_cpulist(const std::string& path, cpu_set_t* set);  // (below)

// Worker k's share of a pool mask (TIPS_HOST_SPREAD, default 1): the CPUs of the mask that share an
// L3 (one CCD on EPYC) with the mask's (k mod domains)-th L3 domain. Left to the scheduler, the
// workers woken by one thread gather on its CCD, and one CCD's link to the I/O die caps what its
// cores copy: config 5 as named host requests took 3.2-4.7 ms per step with the pool gathered on the
// pinned negotiation thread's CCD (profiles/r06/op_host_bind_ab_r6q/r6r/r6s.txt) and 2.89-3.22 with
// the workers spread, against 3.00-3.12 unpinned (op_host_bind_ab_r6t.txt).
bool l3_share(const cpu_set_t& mask, int k, cpu_set_t* out) {
  std::vector<cpu_set_t> groups;
  std::vector<int> firsts;
  for (int c = 0; c < CPU_SETSIZE; c++) {
    if (!CPU_ISSET(c, &mask)) continue;
    bool known = false;
    for (const cpu_set_t& g : groups) known = known || CPU_ISSET(c, &g);
    if (known) continue;
    cpu_set_t g;
    if (!read_cpulist("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/cache/index3/shared_cpu_list", &g))
      return false;
    CPU_AND(&g, &g, &mask);
    if (CPU_COUNT(&g) == 0) return false;
    groups.push_back(g);
  }
  if (groups.size() < 2) return false;
  *out = groups[(size_t)k % groups.size()];
  return true;
}
}  // namespace

HostPool::~HostPool() {
  {
    std::lock_guard<std::mutex> l(m_);
    stop_ = true;
    stop_pub_.store(true, std::memory_order_release);
  }
  cv_.notify_all();
  for (auto& t : th_) t.join();
}

void HostPool::grab(uint64_t gen) {  // claim jobs of run `gen` until none is left
  uint64_t cur = ticket_.load();
  // the ticket is (generation << 32 | jobs << 16 | next index): one atomic snapshot says whether
  // this run still has a job, whatever a later run has written to fn_ / njobs_ meanwhile
  while ((cur >> 32) == gen && (cur & 0xffff) < ((cur >> 16) & 0xffff)) {
    if (!ticket_.compare_exchange_weak(cur, cur + 1)) continue;  // (cur reloaded)
    (*fn_)((int)(cur & 0xffff));
    if (pending_.fetch_sub(1) == 1) {
      std::lock_guard<std::mutex> l(m_);
      done_cv_.notify_all();
    }
    cur = ticket_.load();
  }
}

void HostPool::worker(int k) {
  uint64_t seen = 0, mask_seen = 0;
  // unbound, a worker may run anywhere the process may - not only where the thread that started the
  // pool may (the negotiation thread that runs named host requests is pinned to one L3)
  cpu_set_t start = process_cpus();
  const bool have_start = true;
  (void)sched_setaffinity(0, sizeof start, &start);
  while (true) {
    uint64_t gen;
    std::vector<unsigned char> want;
    bool remask = false;
    if (spin_ns_ > 0) {  // the next run of this call is usually a few hundred microseconds away
      const int64_t t0 = now_ns();
      while (gen_pub_.load(std::memory_order_acquire) == seen && !stop_pub_.load(std::memory_order_acquire) &&
             now_ns() - t0 < spin_ns_)
        _mm_pause();
    }
    {
      std::unique_lock<std::mutex> l(m_);
      cv_.wait(l, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen = gen_;
      if (mask_gen_.load() != mask_seen) {
        mask_seen = mask_gen_.load();
        want = mask_;
        remask = true;
      }
    }
    if (remask) {  // (best effort: a refused mask leaves the thread where it was)
      if (want.size() == sizeof(cpu_set_t)) {
        const cpu_set_t* m = (const cpu_set_t*)want.data();
        cpu_set_t share;
        if (env_i64("TIPS_HOST_SPREAD", 1) != 0 && l3_share(*m, k, &share)) m = &share;
        (void)sched_setaffinity(0, sizeof(cpu_set_t), m);
      } else if (have_start) {
        (void)sched_setaffinity(0, sizeof start, &start);
      }
    }
    grab(gen);
  }
}

void HostPool::set_affinity(const void* cpus) {
  std::lock_guard<std::mutex> l(m_);
  std::vector<unsigned char> m;
  if (cpus) m.assign((const unsigned char*)cpus, (const unsigned char*)cpus + sizeof(cpu_set_t));
  if (m == mask_) return;
  mask_ = std::move(m);
  mask_gen_.fetch_add(1);
}

void HostPool::run(int njobs, const std::function<void(int)>& fn) {
  if (njobs <= 0) return;
  if (njobs > 0xffff) {  // (the ticket holds 16 bits of job index; callers use one job per thread)
    for (int j = 0; j < njobs; j += 0xffff)
      run(std::min(0xffff, njobs - j), [&](int k) { fn(j + k); });
    return;
  }
  uint64_t gen;
  {
    std::lock_guard<std::mutex> l(m_);
    fn_ = &fn;
    pending_.store(njobs);
    gen = ++gen_ & 0xffffffffull;
    ticket_.store(gen << 32 | (uint64_t)njobs << 16);  // (published last: a claim of this run sees fn_, pending_)
    gen_pub_.store(gen_, std::memory_order_release);
  }
  if (njobs > 1) cv_.notify_all();
  grab(gen);
  if (spin_ns_ > 0) {  // the other workers' last jobs are usually microseconds from done
    const int64_t t0 = now_ns();
    while (pending_.load(std::memory_order_acquire) != 0 && now_ns() - t0 < spin_ns_) _mm_pause();
  }
  std::unique_lock<std::mutex> l(m_);
  done_cv_.wait(l, [&] { return pending_.load() == 0; });
}

// The pieces of a fused host stream of `total` bytes: at most `piece` bytes each, but ramping up
// from `first` (doubling) at the start and back down to it at the end, so the first H2D starts
// after a small pack and the last D2H is a short tail - with 16 MiB pieces throughout, the head
// (one pack) and the tail (one D2H) cost 0.6 ms of a 3.3 ms config-5 call. A function of the sizes
// alone: every rank cuts the same pieces (each piece is one allreduce). Offsets 256-B aligned.
std::vector<Piece> host_pieces(int64_t total, int64_t piece, int64_t first) {
  piece = std::max<int64_t>(kAlignBytes, round_up(piece, kAlignBytes));
  first = std::min(piece, std::max<int64_t>(kAlignBytes, round_up(first, kAlignBytes)));
  std::vector<int64_t> head, tail;
  int64_t rest = total;
  for (int64_t s = first; s < piece && rest > 0; s *= 2) {  // ramp up at the head, down at the tail
    for (std::vector<int64_t>* v : {&head, &tail}) {
      const int64_t take = std::min(s, rest);
      if (take > 0) v->push_back(take);
      rest -= take;
    }
  }
  std::vector<Piece> out;
  int64_t off = 0;
  for (int64_t len : head) out.push_back(Piece{off, len}), off += len;
  if (rest > 0) {
    const int64_t n = (rest + piece - 1) / piece, per = round_up((rest + n - 1) / n, kAlignBytes);
    for (int64_t k = 0; k < n && rest > 0; k++) {
      const int64_t len = std::min(per, rest);
      out.push_back(Piece{off, len});
      off += len;
      rest -= len;
    }
  }
  for (auto it = tail.rbegin(); it != tail.rend(); ++it) out.push_back(Piece{off, *it}), off += *it;
  return out;
}

namespace {

bool read_cpulist(const std::string& path, cpu_set_t* set) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return false;
  char buf[4096] = {0};
  const bool ok = fgets(buf, sizeof buf, f) != nullptr;
  fclose(f);
  if (!ok) return false;
  CPU_ZERO(set);
  for (char* p = buf; *p && *p != '\n';) {
    char* e = nullptr;
    long a = strtol(p, &e, 10);
    if (e == p) return false;
    long b = a;
    if (*e == '-') {
      p = e + 1;
      b = strtol(p, &e, 10);
      if (e == p) return false;
    }
    for (long c = a; c <= b && c < CPU_SETSIZE; c++) CPU_SET((int)c, set);
    p = *e == ',' ? e + 1 : e;
  }
  return true;
}

// The CPUs of the device's NUMA node that this process may run on (PCI sysfs): where the fused host
// path's copy threads sit (TIPS_HOST_BIND, default on), next to the root complex the DMA engines use.
// False when the node is unknown or none of its CPUs is allowed.
bool gpu_local_cpus(int device, cpu_set_t* out) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, device) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  for (char* c = bus; *c; c++) *c = (char)tolower((unsigned char)*c);
  FILE* f = fopen((std::string("/sys/bus/pci/devices/") + bus + "/numa_node").c_str(), "r");
  if (!f) return false;
  int node = -1;
  const int got = fscanf(f, "%d", &node);
  fclose(f);
  if (got != 1 || node < 0) return false;
  cpu_set_t local, allowed = process_cpus();  // (not this thread's mask: it may be the pinned negotiation thread)
  if (!read_cpulist("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist", &local)) return false;
  CPU_AND(out, &local, &allowed);
  return CPU_COUNT(out) > 0;
}

// Host copies of the fused path: bytes that the DMA engine (pack) or the caller (unpack) reads next,
// not this thread. Streaming stores skip the read-for-ownership of every destination line and keep
// the slots out of the caches; glibc's memcpy only streams above ~3/4 of the shared cache, far above
// the per-thread share of a piece (16 MiB / 8 threads = 2 MiB). 32-B streaming stores after an
// unaligned head; loads unaligned (numpy's buffers are 16-B aligned at best).
__attribute__((target("avx2"))) void copy_stream_avx2(char* d, const char* s, size_t n) {
  const size_t head = std::min(n, (size_t)((32 - ((uintptr_t)d & 31)) & 31));
  memcpy(d, s, head);
  d += head, s += head, n -= head;
  size_t i = 0;
  for (; i + 128 <= n; i += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 64));
    const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i), a);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 96), e);
  }
  for (; i + 32 <= n; i += 32)
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i), _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i)));
  memcpy(d + i, s + i, n - i);
  _mm_sfence();  // (streaming stores are weakly ordered: visible before the job reports done)
}

// (the pool's threads reach this concurrently on their first job: the setting is an atomic, set by
// whichever thread comes first - the same value every time - not a function-local static, whose
// first use ThreadSanitizer reported as a race on the GPU box, profiles/r03/l_tsan_report.txt)
std::atomic<int> g_stream_stores{-1};

void copy_stream(char* d, const char* s, size_t n) {
  int ok = g_stream_stores.load(std::memory_order_relaxed);
  if (ok < 0) {
    ok = __builtin_cpu_supports("avx2") && env_i64("TIPS_HOST_STREAM_STORES", 1) != 0;
    g_stream_stores.store(ok, std::memory_order_relaxed);
  }
  if (ok && n >= 4096) copy_stream_avx2(d, s, n);
  else memcpy(d, s, n);
}

struct HostSeg {
  int64_t off, bytes;  // in the flat byte stream
  const char* in;
  char* out;
};

// Copy flat bytes [a, b) between the stream's segments and `buf` (which holds stream bytes from
// base on): pack = tensors -> buf, else buf -> tensors. The padding between segments is skipped.
void copy_range(const std::vector<HostSeg>& segs, int64_t a, int64_t b, char* buf, int64_t base, bool pack) {
  auto it = std::upper_bound(segs.begin(), segs.end(), a,
                             [](int64_t v, const HostSeg& s) { return v < s.off + s.bytes; });  // first with end > a
  for (; it != segs.end() && it->off < b; ++it) {
    const int64_t s = std::max(a, it->off), e = std::min(b, it->off + it->bytes);
    if (e <= s) continue;
    if (pack) copy_stream(buf + (s - base), it->in + (s - it->off), (size_t)(e - s));
    else copy_stream(it->out + (s - it->off), buf + (s - base), (size_t)(e - s));
  }
}

}  // namespace

// The byte stream is the fusion layout of the list (fused_layout: 256-B aligned offsets, a function
// of the counts alone, the same as tips_fused_allreduce_flat's), so every rank cuts the same pieces
// and a flat host output has the device flat output's layout. With `flat` (host memory laid out so),
// the sums land there: straight from the device when it is page-locked (no unpack at all), else
// through a page-locked slot and one contiguous copy per piece. Without it, they are unpacked into
// every items[i].out.
int fused_allreduce_host(State& st, const BatchItem* items, int n, int dtype, char* flat) {
  const int64_t es = tips::dtype_size(dtype);
  std::vector<int64_t> counts((size_t)n), offs((size_t)n);
  for (int i = 0; i < n; i++) counts[i] = items[i].count;
  int64_t total = fused_layout(counts.data(), n, dtype, offs.data());
  std::vector<HostSeg> segs;
  segs.reserve((size_t)n);
  for (int i = 0; i < n; i++)
    if (counts[i] > 0) segs.push_back(HostSeg{offs[i], counts[i] * es, (const char*)items[i].in, (char*)items[i].out});
  if (segs.empty()) return 0;
  std::sort(segs.begin(), segs.end(), [](const HostSeg& x, const HostSeg& y) { return x.off < y.off; });
  total = round_up(total, kAlignBytes);
  // 32 MiB middle pieces (between the 2 MiB ramps): config 5 host -> host 31-32 GiB/s best, 3.06-3.31 ms
  // median, against 26-31 GiB/s / 3.38-4.25 ms at 16 MiB and 24-28 at 8 MiB (3 interleaved rounds on one
  // box, profiles/r03/e_host_probe_streams.jsonl); a second H2D stream did not help reliably
  const int64_t piece = std::min<int64_t>(
      total, round_up(std::max<int64_t>(kAlignBytes, env_i64("TIPS_HOST_FUSED_PIECE_BYTES", 32 << 20)), kAlignBytes));
  const std::vector<Piece> pieces = host_pieces(total, piece, env_i64("TIPS_HOST_FUSED_FIRST_BYTES", 2 << 20));
  const int np = (int)pieces.size();
  // page-locked slots per direction (piece i uses slot i % R), and how many pieces behind the one
  // being packed the unpack runs: with lag 2 the thread unpacks a piece whose D2H finished while
  // the previous piece was packed, instead of waiting for the one just sent (TIPS_HOST_SLOTS,
  // TIPS_HOST_UNPACK_LAG; lag <= R - 1, since D2H(i + 1) reuses the slot unpack(i + 1 - R) freed)
  const int R = (int)std::max<int64_t>(2, std::min<int64_t>(8, env_i64("TIPS_HOST_SLOTS", 4)));
  const int nthreads = (int)std::max<int64_t>(1, std::min<int64_t>(64, env_i64("TIPS_HOST_THREADS", 8)));
  if (!st.host_pool || st.host_pool->size() != nthreads) {
    delete st.host_pool;
    st.host_pool = new HostPool(nthreads);
  }
  // TIPS_HOST_BIND (default 1): the pool's threads on the GPU's NUMA node, as RCCL places its own
  // threads (the caller's thread stays put). Config 5 host -> host: 0.5-1.5 % faster in each of 3
  // interleaved rounds on a box whose process may run on both nodes (profiles/r03/p_numa_probe.jsonl)
  static int local_ok = -1;
  static cpu_set_t local;
  const bool host_bind = env_i64("TIPS_HOST_BIND", 1) != 0;
  if (host_bind) {
    if (local_ok < 0) local_ok = gpu_local_cpus(st.device, &local) ? 1 : 0;
    st.host_pool->set_affinity(local_ok == 1 ? &local : nullptr);
  } else {
    st.host_pool->set_affinity(nullptr);
  }
  // The negotiation thread runs named host requests' fused calls, and it is pinned to its caller's
  // L3 (TIPS_NEG_BIND): for the call it moves to the GPU's node, where the pool and the DMA engines
  // are (it packs and unpacks a share and issues every copy), and back after it. A user's thread is
  // never moved. Config 5 as named host requests: 3.37-3.47 ms per step with the thread left on the
  // caller's L3 on the other socket, 3.08-3.22 unbound (profiles/r06/op_host_bind_ab_r6r.txt).
  struct Near {
    bool moved = false;
    cpu_set_t saved;
    Near(bool want, const cpu_set_t* to) {
      if (want && to && pthread_getaffinity_np(pthread_self(), sizeof saved, &saved) == 0 &&
          pthread_setaffinity_np(pthread_self(), sizeof(cpu_set_t), to) == 0)
        moved = true;
    }
    ~Near() {
      if (moved) (void)pthread_setaffinity_np(pthread_self(), sizeof saved, &saved);
    }
  } near(host_bind && local_ok == 1 && on_negotiation_thread(), &local);
  if (st.hpin_bytes < (size_t)(R * piece)) {
    for (void*& p : st.hpin)
      if (p) (void)hipHostFree(p), p = nullptr;
    st.hpin_bytes = 0;
    for (void*& p : st.hpin) HIP_TRY(hipHostMalloc(&p, (size_t)(R * piece), hipHostMallocDefault));
    st.hpin_bytes = (size_t)(R * piece);
  }
  TRY(st.host_in.ensure((size_t)total));
  TRY(st.pipe_ev.ensure(3 * (size_t)np));
  char* dev = (char*)st.host_in.p;
  char* pin_in = (char*)st.hpin[0];
  char* pin_out = (char*)st.hpin[1];
  // TIPS_HOST_H2D_KERNEL=1 (an A/B knob, off): the H2D of each piece by copy_buf_kernel reading the
  // page-locked slot through its device mapping (zero-copy) instead of a hipMemcpyAsync on the DMA
  // engine. The runtime does the D2H with a blit kernel, and a DMA H2D issued while such a blit runs
  // starts only when the blit ends (profiles/r04/ze_host_copytrace.json); but a kernel H2D holds the
  // CUs while it waits on PCIe reads and starves the D2H blits: config 5 host -> host 4.1-4.4 ms
  // against 2.6-3.2 ms (profiles/r04/zk_host_h2d_ab.txt).
  char* pin_in_dev = nullptr;
  if (env_i64("TIPS_HOST_H2D_KERNEL", 0) != 0 && hipHostGetDevicePointer((void**)&pin_in_dev, pin_in, 0) != hipSuccess) {
    (void)hipGetLastError();
    pin_in_dev = nullptr;
  }
  // D2H straight into the output (TIPS_HOST_DIRECT_OUT=0: through the page-locked slots, probing only)
  const bool direct_out = flat && env_i64("TIPS_HOST_DIRECT_OUT", 1) != 0 && is_pinned_host(flat, total);

  hipEvent_t* ev = st.pipe_ev.ev.data();  // [3i] H2D done, [3i+1] reduced, [3i+2] D2H done
  const int parts = nthreads;
  auto host_copy = [&](int i, bool pack) {
    const int64_t p0 = pieces[(size_t)i].off, p1 = p0 + pieces[(size_t)i].len;
    char* buf = (pack ? pin_in : pin_out) + (int64_t)(i % R) * piece;
    const int64_t per = round_up((p1 - p0 + parts - 1) / parts, 64);
    st.host_pool->run(parts, [&](int j) {
      const int64_t a = p0 + j * per, b = std::min(p1, a + per);
      if (a >= b) return;
      if (!pack && flat) copy_stream(flat + a, buf + (a - p0), (size_t)(b - a));  // (padding included: contiguous)
      else copy_range(segs, a, b, buf, p0, pack);
    });
  };
  const int lag = direct_out ? np : (int)std::max<int64_t>(1, std::min<int64_t>(R - 1, env_i64("TIPS_HOST_UNPACK_LAG", 2)));
  // TIPS_HOST_TRACE=1: where one call's time goes (stderr), for tuning the piece and thread counts
  static const int64_t trace_level = env_i64("TIPS_HOST_TRACE", 0);
  const bool trace = trace_level != 0;
  // TIPS_HOST_TRACE=2: also each piece's host timeline (us from the call's start): slot free, packed,
  // issued, unpacked - to line up with a rocprofv3 memory-copy trace (tools/copytrace_report.py)
  std::vector<std::array<double, 4>> tl(trace_level >= 2 ? (size_t)np : 0, std::array<double, 4>{0, 0, 0, 0});
  double t_pack = 0, t_wait = 0, t_unpack = 0, t_issue = 0;
  const auto t_start = std::chrono::steady_clock::now();
  auto since = [](std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count();
  };
  static hipEvent_t tev[3];  // (trace only) first H2D issued, last H2D done, last D2H done
  if (trace && !tev[0])
    for (auto& e : tev) HIP_TRY(hipEventCreate(&e));
  auto report = [&] {
    if (!trace) return;
    float h2d = 0, d2h = 0;
    (void)hipEventSynchronize(tev[2]);
    (void)hipEventElapsedTime(&h2d, tev[0], tev[1]);
    (void)hipEventElapsedTime(&d2h, tev[0], tev[2]);
    fprintf(stderr, "[tips host] bytes %lld pieces %d threads %d direct_out %d: pack %.0f us, wait %.0f us, "
            "unpack %.0f us, issue %.0f us, total %.0f us; device: first H2D -> last H2D %.0f us "
            "(%.1f GiB/s), -> last D2H %.0f us\n", (long long)total, np, nthreads, (int)direct_out, t_pack, t_wait,
            t_unpack, t_issue, since(t_start), h2d * 1e3, total / (h2d * 1e-3) / 1073741824.0, d2h * 1e3);
    for (size_t i = 0; i < tl.size(); i++)
      fprintf(stderr, "[tips host]   piece %zu %lld B: slot %.0f packed %.0f issued %.0f unpacked %.0f us\n", i,
              (long long)pieces[i].len, tl[i][0], tl[i][1], tl[i][2], tl[i][3]);
  };
  // TIPS_HOST_H2D_STREAMS=2: odd pieces' H2D on a second stream (a second DMA queue), so the link
  // does not idle between one piece's copy and the next while the runtime starts it
  const bool two_h2d = env_i64("TIPS_HOST_H2D_STREAMS", 1) >= 2;
  for (int i = 0; i < np; i++) {
    const int64_t off = pieces[(size_t)i].off, len = pieces[(size_t)i].len;
    hipStream_t hs = two_h2d && (i & 1) ? st.h2d_stream2 : st.h2d_stream;
    auto t0 = std::chrono::steady_clock::now();
    if (i >= R) HIP_TRY(hipEventSynchronize(ev[3 * (i - R)]));  // slot i % R: its last H2D has read it
    t_wait += since(t0);
    if (!tl.empty()) tl[(size_t)i][0] = since(t_start);
    t0 = std::chrono::steady_clock::now();
    host_copy(i, true);
    t_pack += since(t0);
    if (!tl.empty()) tl[(size_t)i][1] = since(t_start);
    t0 = std::chrono::steady_clock::now();
    if (trace && i == 0) HIP_TRY(hipEventRecord(tev[0], hs));
    if (pin_in_dev) HIP_TRY(tips::launch_copy_buf(dev + off, pin_in_dev + (int64_t)(i % R) * piece, len, hs));
    else HIP_TRY(hipMemcpyAsync(dev + off, pin_in + (int64_t)(i % R) * piece, (size_t)len, hipMemcpyHostToDevice, hs));
    HIP_TRY(hipEventRecord(ev[3 * i], hs));
    HIP_TRY(hipStreamWaitEvent(st.io_stream, ev[3 * i], 0));
    TRY(allreduce_device(st, dev + off, dev + off, len / es, dtype, st.io_stream));
    HIP_TRY(hipEventRecord(ev[3 * i + 1], st.io_stream));
    HIP_TRY(hipStreamWaitEvent(st.d2h_stream, ev[3 * i + 1], 0));
    // (slot i % R of pin_out was unpacked at iteration i - R + lag < i)
    char* d2h = direct_out ? flat + off : pin_out + (int64_t)(i % R) * piece;
    HIP_TRY(hipMemcpyAsync(d2h, dev + off, (size_t)len, hipMemcpyDeviceToHost, st.d2h_stream));
    HIP_TRY(hipEventRecord(ev[3 * i + 2], st.d2h_stream));
    if (trace && i == np - 1) {
      HIP_TRY(hipEventRecord(tev[1], hs));
      HIP_TRY(hipEventRecord(tev[2], st.d2h_stream));
    }
    t_issue += since(t0);
    if (!tl.empty()) tl[(size_t)i][2] = since(t_start);
    if (i >= lag) {
      t0 = std::chrono::steady_clock::now();
      HIP_TRY(hipEventSynchronize(ev[3 * (i - lag) + 2]));
      t_wait += since(t0);
      t0 = std::chrono::steady_clock::now();
      host_copy(i - lag, false);
      t_unpack += since(t0);
      if (!tl.empty()) tl[(size_t)(i - lag)][3] = since(t_start);
    }
  }
  if (direct_out) {
    auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(hipStreamSynchronize(st.d2h_stream));
    t_wait += since(t0);
    report();
    return 0;
  }
  for (int j = std::max(0, np - lag); j < np; j++) {
    auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(hipEventSynchronize(ev[3 * j + 2]));
    t_wait += since(t0);
    t0 = std::chrono::steady_clock::now();
    host_copy(j, false);
    t_unpack += since(t0);
    if (!tl.empty()) tl[(size_t)j][3] = since(t_start);
  }
  report();
  return 0;
}

void host_release(State& st) {
  delete st.host_pool;
  st.host_pool = nullptr;
  for (void*& p : st.hpin)
    if (p) (void)hipHostFree(p), p = nullptr;
  st.hpin_bytes = 0;
}

}  // namespace rt
}  // namespace tips

using namespace tips::rt;

extern "C" {

#ifdef TIPS_DEV  // (development surface: libtips_hip_dev.so only, include/tips_hip_dev.h)
int tips_host_pool_selftest(int nthreads, int runs, int njobs) {
  if (nthreads < 1 || nthreads > 64 || runs < 0 || njobs < 0) return fail(TIPS_ERR_INVALID_ARG, "bad arguments");
  HostPool pool(nthreads);
  std::vector<std::atomic<int>> hits((size_t)njobs);
  for (int r = 0; r < runs; r++) {
    for (auto& h : hits) h.store(0);
    const int n = r % 3 == 2 ? njobs / 2 : njobs;  // (runs of different sizes back to back)
    std::function<void(int)> fn = [&](int j) { hits[(size_t)j].fetch_add(1); };
    pool.run(n, fn);
    for (int j = 0; j < njobs; j++)
      if (hits[(size_t)j].load() != (j < n ? 1 : 0))
        return fail(TIPS_ERR_MISMATCH, "run %d: job %d ran %d times", r, j, hits[(size_t)j].load());
  }
  return 0;
}
#endif  // TIPS_DEV

int tips_fused_allreduce_host(const void* const* ins, void* const* outs, const int64_t* counts, int n, int dtype) {
  TRY(check_dtype(dtype));
  if (n < 0 || (n > 0 && (!ins || !outs || !counts))) return fail(TIPS_ERR_INVALID_ARG, "bad tensor list");
  std::vector<BatchItem> items((size_t)n);
  for (int i = 0; i < n; i++) {
    if (counts[i] < 0 || (counts[i] > 0 && (!ins[i] || !outs[i]))) return fail(TIPS_ERR_INVALID_ARG, "bad tensor %d", i);
    items[i] = BatchItem{ins[i], outs[i], counts[i]};
  }
  int routed_rc;
  int64_t shape[2] = {n, 0};
  for (int i = 0; i < n; i++) shape[1] += counts[i];
  if (route_collective(TIPS_REQ_ALLREDUCE, dtype, shape, 2, 0,
                       [&] { return tips_fused_allreduce_host(ins, outs, counts, n, dtype); }, &routed_rc))
    return routed_rc;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  if (n == 0) return 0;
  TRY(set_device(st));
  for (int i = 0; i < n; i++)
    if (items[i].count > 0 && (is_device_ptr(items[i].in) || is_device_ptr(items[i].out)))
      return fail(TIPS_ERR_INVALID_ARG, "tips_fused_allreduce_host: tensor %d is in device memory", i);
  return fused_allreduce_host(st, items.data(), n, dtype, nullptr);
}

int tips_fused_allreduce_host_flat(const void* const* ins, const int64_t* counts, int n, int dtype, void* flat) {
  TRY(check_dtype(dtype));
  if (n < 0 || (n > 0 && (!ins || !counts || !flat))) return fail(TIPS_ERR_INVALID_ARG, "bad tensor list");
  std::vector<BatchItem> items((size_t)n);
  for (int i = 0; i < n; i++) {
    if (counts[i] < 0 || (counts[i] > 0 && !ins[i])) return fail(TIPS_ERR_INVALID_ARG, "bad tensor %d", i);
    items[i] = BatchItem{ins[i], flat, counts[i]};
  }
  int routed_rc;
  int64_t shape[2] = {n, 0};
  for (int i = 0; i < n; i++) shape[1] += counts[i];
  if (route_collective(TIPS_REQ_ALLREDUCE, dtype, shape, 2, 0,
                       [&] { return tips_fused_allreduce_host_flat(ins, counts, n, dtype, flat); }, &routed_rc))
    return routed_rc;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  if (n == 0) return 0;
  TRY(set_device(st));
  if (is_device_ptr(flat)) return fail(TIPS_ERR_INVALID_ARG, "tips_fused_allreduce_host_flat: flat is device memory");
  for (int i = 0; i < n; i++)
    if (items[i].count > 0 && is_device_ptr(items[i].in))
      return fail(TIPS_ERR_INVALID_ARG, "tips_fused_allreduce_host_flat: tensor %d is in device memory", i);
  return fused_allreduce_host(st, items.data(), n, dtype, (char*)flat);
}

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
