// negotiate.cc — asynchronous, named allreduce requests with cross-rank negotiation.
//
// Replaces the reference's coordinator (tips/core/collective/coordinator.cc):
//   EnqueueTensorCollective (:223-241)  -> tips_enqueue_allreduce
//   BackgroundThreadLoop (:355-513)     -> Negotiator::loop
//   IncreTensorCount (:15-38)           -> Table::announce (per-name ready count)
//   ConstructResponseMessage (:90-186)  -> check_records (control.cc), same error text
//   PerformCollectiveOp (:243-353)      -> execute(): allreduce_device on the request's stream
// TF runs ops in different orders on different ranks, so every rank must agree
// on WHICH named tensors are ready everywhere and in WHAT order to reduce them.
// Here one background thread per rank runs cycles in lockstep with rank 0 over
// one persistent TCP connection (the reference: a ZeroMQ PUSH/PULL RPC with
// flatbuffers, naive_rpc.cc): each cycle every rank sends the requests it has
// newly enqueued; rank 0 queues each name when its last rank announces it, validates
// every name all ranks have announced, and answers with the list to run; every
// rank then reduces that list in that order on the owning request's stream.
// Only control records travel here; tensor bytes go over RCCL / xGMI.
//
// Dry-run mode (tips_negotiation_selftest) runs the same protocol with an
// executor that only logs the order, so it is testable across processes on a
// host without a GPU.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <pthread.h>
#include <sched.h>
#include <sys/prctl.h>
#include <deque>
#include <memory>
#include <thread>

#include "net.h"
#include "rt.h"

namespace tips {
namespace rt {
namespace {

using namespace tips::net;

// One completion event shared by the requests of a fused batch. `done` is set once a wait on it
// has returned: the batch's other requests then skip the HIP call (a batch of 1000 named
// gradients otherwise synchronizes the same finished event 1000 times).
struct GroupEv {
  hipEvent_t ev = nullptr;
  std::atomic<bool> done{false};
  ~GroupEv() {
    if (ev) (void)hipEventDestroy(ev);
  }
};

// The request tables' lock (and the negotiator's): glibc's adaptive mutex, which spins briefly
// before it sleeps. Executor threads enqueueing at once hold it for well under a microsecond; with
// std::mutex each hand-over between them went through a futex wake, and four threads enqueueing
// config 5's 214 requests took longer than one thread (tools/op_host.c, OP_HOST_TRACE).
inline int64_t steady_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

class AdaptiveMutex {
 public:
  AdaptiveMutex() {
    pthread_mutexattr_t a;
    pthread_mutexattr_init(&a);
    // (TIPS_ADAPTIVE_LOCKS=0: a plain mutex, as std::mutex, for A/B runs of tools/op_host_sweep.sh)
    pthread_mutexattr_settype(&a, env_i64("TIPS_ADAPTIVE_LOCKS", 1) ? PTHREAD_MUTEX_ADAPTIVE_NP : PTHREAD_MUTEX_NORMAL);
    pthread_mutex_init(&m_, &a);
    pthread_mutexattr_destroy(&a);
  }
  ~AdaptiveMutex() { pthread_mutex_destroy(&m_); }
  AdaptiveMutex(const AdaptiveMutex&) = delete;
  AdaptiveMutex& operator=(const AdaptiveMutex&) = delete;
  void lock() { pthread_mutex_lock(&m_); }
  bool try_lock() { return pthread_mutex_trylock(&m_) == 0; }
  void unlock() { pthread_mutex_unlock(&m_); }

 private:
  pthread_mutex_t m_;
};

struct Req {
  int64_t handle = 0;
  std::string name;
  uint64_t name_hash = 0;  // (of name, made by the enqueuing thread: the linger's expected set)
  const void* in = nullptr;
  void* out = nullptr;
  int64_t count = 0;
  std::vector<int64_t> shape;  // dims (the reference's TensorShape; [count] for unshaped requests)
  int dtype = 0;
  int type = TIPS_REQ_ALLREDUCE;  // message::RequestType: allreduce, allgather, broadcast
  int root = 0;                   // broadcast
  tips_alloc_fn alloc = nullptr;  // allgather: output allocator, called once the sizes are known
  void* actx = nullptr;
  int64_t* out_rows = nullptr;
  bool host = false;  // host memory (the reference's CPU op): run synchronously, staged through HBM
  hipStream_t stream = nullptr;
  hipEvent_t ev = nullptr;
  std::shared_ptr<GroupEv> gev;  // set when the request ran inside a fused batch (then ev is unused)
  int state = 0;  // 0 queued, 1 announced, 2 launched (ev recorded), 3 done (host / dry run / routed), -1 error
  int code = TIPS_ERR_MISMATCH;  // the failure's status (a routed collective's own; a negotiation error's)
  std::string err;
  // A synchronous collective routed through the negotiation (route_collective): its body runs on
  // the negotiation thread when rank 0's order reaches it, like any named request.
  std::function<int()> body;
  // tips_on_done: called once from the completion thread when the request has finished
  tips_done_fn cb = nullptr;
  void* cb_ctx = nullptr;
  bool cb_queued = false;
  bool cb_only = false;  // enqueued with its callback (tips_enqueue_allreduce_cb): not in the handle table
  // A single enqueue does not ask HIP where its pointers live: hipPointerGetAttributes takes a
  // runtime-wide lock, and TF-style executor threads enqueueing at once queued on it (4 threads:
  // 1.38 us per lookup, 0.10 alone; tools/enqueue_probe.cc). The negotiation thread classifies
  // the cycle's requests before announcing them, one thread, no contention; a request whose two
  // pointers disagree is announced as bad and fails on every rank once all have announced it.
  bool classify = false;
  std::string bad;
};

// Request handles, process-wide (per-thread blocks of 256: Negotiator::prepare); the submission
// stack shard of each enqueuing thread (Negotiator::enqueue)
std::atomic<uint64_t> g_next_shard{0};
// Request handles, process-wide (per-thread blocks of 256: Negotiator::prepare)
std::atomic<int64_t> g_next_handle{0};

// The negotiation thread itself: a collective entry point called there runs directly (it is the
// body of a routed request, or the executor's own call), never routed again.
thread_local bool tl_negotiation_thread = false;
// Synchronous collectives this process issued directly (no negotiation running) while size > 1:
// every rank must have issued the same number when the negotiation starts (checked at the join).
std::atomic<int64_t> g_sync_direct{0};

// The device allocations one list call (tips_enqueue_allreduce_n / _shaped_n) has met so far: a
// gradient list lies in a few of the caching allocator's segments, so after a segment's first
// pointer (hipPointerGetAttributes, then hipMemGetAddressRange) the rest of its tensors are known
// to be device memory without a HIP call - two calls per request otherwise, most of enqueue's cost.
// Lives for one list call, during which the caller keeps every pointer of the list alive. Host
// pointers are never cached: each takes its own hipPointerGetAttributes, as a single enqueue does.
struct PtrRanges {
  struct Range {
    uintptr_t lo, len;
  };
  std::vector<Range> r;
  size_t last = 0;
  bool is_device(const void* p) {
    const uintptr_t a = (uintptr_t)p;
    if (last < r.size() && a - r[last].lo < r[last].len) return true;
    for (size_t k = 0; k < r.size(); k++)
      if (a - r[k].lo < r[k].len) {
        last = k;
        return true;
      }
    if (!is_device_ptr(p)) return false;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) == hipSuccess && size > 0) {
      r.push_back(Range{(uintptr_t)base, (uintptr_t)size});
      last = r.size() - 1;
    } else {
      (void)hipGetLastError();
    }
    return true;
  }
};

// ---- wire format: flat little-endian records ----------------------------------
struct Writer {
  std::string b;
  template <class T>
  void put(T v) {
    b.append(reinterpret_cast<const char*>(&v), sizeof v);
  }
  void str(const std::string& s) {
    put<uint32_t>((uint32_t)s.size());
    b += s;
  }
};

struct Reader {
  const std::string& b;
  size_t off = 0;
  bool ok = true;
  explicit Reader(const std::string& s) : b(s) {}
  template <class T>
  T get() {
    T v{};
    if (off + sizeof v > b.size()) {
      ok = false;
      return v;
    }
    memcpy(&v, b.data() + off, sizeof v);
    off += sizeof v;
    return v;
  }
  std::string str() {
    std::string s;
    str_into(s);
    return s;
  }
  void str_into(std::string& s) {  // (into a reused string: no allocation once its capacity fits)
    const uint32_t n = get<uint32_t>();
    if (!ok || off + n > b.size()) {
      ok = false;
      s.clear();
      return;
    }
    s.assign(b.data() + off, n);
    off += n;
  }
};

// announce (rank -> rank 0): u8 shutdown, u32 n,
//   n x {i32 type, i32 root, i32 dtype, i64 count, u32 ndim, ndim x i64 dim, str name}
//   (the fields of the reference's RequestMessage, collective_messages.fbs: request type, dtype,
//   name, shape; plus the broadcast root, which the reference never sends)
// response (rank 0 -> all):  u8 shutdown, u32 n, n x {u8 ok, str name, str error, u32 m, m x i64 size}
//   (sizes: an allgather's first dimension per rank, the ResponseMessage's tensor_sizes)
struct Announce {
  int type = TIPS_REQ_ALLREDUCE, root = 0;
  bool bad = false;  // the announcing rank found the request unusable (its pointers disagree)
  int dtype;
  int64_t count;
  std::vector<int64_t> shape;
  std::string name;
};

struct Decision {
  bool ok;
  std::string name, err;
  std::vector<int64_t> sizes;
};

// ---- rank 0's table (IncreTensorCount + ConstructResponseMessage) ---------------
// A name joins the ready queue the moment its last rank announces it (or a
// rank announces it twice), as IncreTensorCount feeds ready_to_reduce
// (coordinator.cc:15-38, 451-455): rank 0's readiness order, O(1) per announce.
struct Table {
  struct Row {
    std::vector<int64_t> rec;  // p records of TIPS_REQUEST_WORDS
    std::vector<int> roots;    // broadcast root each rank named
    std::vector<char> seen;
    int nseen = 0;
    bool queued = false;
    std::string dup;  // set when a rank announced this name twice while unresolved
    std::string bad;  // set when a rank announced this name as unusable (failed once all announced)
  };
  int p = 1;
  std::unordered_map<std::string, Row> rows;
  std::vector<std::string> ready_q;  // [0, nready): names that became ready (slots reused across cycles)
  size_t nready = 0;
  // Rows resolved in earlier cycles, kept with their map node, key and vectors: a new name reuses
  // one instead of allocating all four (a 1000-gradient step resolves 1000 names a cycle).
  std::vector<std::unordered_map<std::string, Row>::node_type> spare;

  void announce(int rank, const Announce& a) {
    auto it = rows.find(a.name);
    if (it == rows.end()) {
      if (!spare.empty()) {
        auto nh = std::move(spare.back());
        spare.pop_back();
        nh.key() = a.name;
        Row& r = nh.mapped();
        r.rec.assign((size_t)p * TIPS_REQUEST_WORDS, 0);
        r.seen.assign(p, 0);
        r.roots.assign(p, 0);
        r.nseen = 0;
        r.queued = false;
        r.dup.clear();
        r.bad.clear();
        it = rows.insert(std::move(nh)).position;
      } else {
        Row r;
        r.rec.assign((size_t)p * TIPS_REQUEST_WORDS, 0);
        r.seen.assign(p, 0);
        r.roots.assign(p, 0);
        it = rows.emplace(a.name, std::move(r)).first;
      }
    }
    Row& r = it->second;
    if (r.seen[rank]) {
      if (r.dup.empty()) r.dup = "rank " + std::to_string(rank) + " enqueued " + a.name + " twice";
    } else {
      r.seen[rank] = 1;
      r.nseen++;
      if (a.bad && r.bad.empty())
        r.bad = "named request " + a.name + ": one device and one host pointer on rank " + std::to_string(rank);
      int64_t* rec = &r.rec[(size_t)rank * TIPS_REQUEST_WORDS];
      rec[0] = a.type;
      rec[1] = a.dtype;
      r.roots[rank] = a.root;
      rec[2] = (int64_t)a.shape.size();  // (<= TIPS_MAX_DIMS: checked at enqueue and on decode)
      for (size_t d = 0; d < a.shape.size(); d++) rec[3 + d] = a.shape[d];
    }
    if (!r.queued && (!r.dup.empty() || r.nseen == p)) {
      r.queued = true;
      if (nready < ready_q.size()) ready_q[nready] = a.name;  // (assign into a kept string: no allocation)
      else ready_q.push_back(a.name);
      nready++;
    }
  }

  // The names that became ready since the last call, in readiness order, each with its verdict,
  // written straight into rank 0's response (ok, name, error, allgather sizes): no per-name
  // Decision objects on the way. Returns how many.
  uint32_t write_ready(Writer& w) {
    const int W = TIPS_REQUEST_WORDS;
    for (size_t q = 0; q < nready; q++) {
      const std::string& name = ready_q[q];
      auto it = rows.find(name);
      Row& r = it->second;
      const std::string* err = &r.dup;
      std::string why;
      bool ok = false;
      if (r.dup.empty() && !r.bad.empty()) {
        err = &r.bad;
      } else if (r.dup.empty()) {
        ok = check_records(r.rec.data(), p) == 0;
        if (!ok) why = last_error();
        if (ok && r.rec[0] == TIPS_REQ_BROADCAST)
          for (int i = 1; i < p && ok; i++)
            if (r.roots[i] != r.roots[0]) {
              ok = false;
              why = "Mismatched broadcast root ranks: " + std::to_string(r.roots[0]) + " vs " + std::to_string(r.roots[i]);
            }
        err = &why;
      }
      w.put<uint8_t>(ok ? 1 : 0);
      w.str(name);
      w.str(ok ? std::string() : *err);
      if (ok && r.rec[0] == TIPS_REQ_ALLGATHER) {  // GatherFirstRankSizes (coordinator.cc:40-88)
        w.put<uint32_t>((uint32_t)p);
        for (int i = 0; i < p; i++) w.put<int64_t>(r.rec[(size_t)i * W + 3]);
      } else {
        w.put<uint32_t>(0);
      }
      if (spare.size() < 4096) spare.push_back(rows.extract(it));
      else rows.erase(it);
    }
    const uint32_t n = (uint32_t)nready;
    nready = 0;
    return n;
  }
};

// The name table's key carries the name's hash, made by the enqueuing thread (Req::name_hash): the
// negotiation thread admits a request without reading the name's bytes, which another core wrote
// (an insertion compares the cached hash first, the strings only when the hashes are equal).
struct NameKey {
  uint64_t h;
  std::string s;
  bool operator==(const NameKey& o) const { return h == o.h && s == o.s; }
};
struct NameKeyHash {
  size_t operator()(const NameKey& k) const { return (size_t)k.h; }
};
using NameMap = std::unordered_map<NameKey, std::shared_ptr<Req>, NameKeyHash>;
using HandleMap = std::unordered_map<int64_t, std::shared_ptr<Req>>;


// Where the negotiation's threads run (1000 named requests at one rank took
// 0.40 or 0.87-1.85 us per tensor, bimodal across processes on one box). The caller, the negotiation
// thread and the completion thread hand every request over through shared cache lines; on the GPU
// box's 2-socket EPYC 9575F (16 CCDs of one L3 each) the scheduler put the negotiation thread on
// another CCD than the caller in every slow process and on the same one in every fast process:
// unbound 1.01-1.60 us per tensor with the threads on different L3s (4 of 4 runs), bound to the
// caller's L3 or core 0.39-0.41 (8 of 8; profiles/r06/neg_placement/). So TIPS_NEG_BIND=l3, the
// default, pins both threads to the CPUs that share an L3 with the thread that started the
// negotiation; =core to that thread's SMT siblings; =0 leaves them free. The threads are named
// (tips-neg, tips-done: /proc/<pid>/task/*/comm), so bench.py records where each last ran.
bool cpu_list(const std::string& path, cpu_set_t* set) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return false;
  char buf[4096] = {};
  const bool ok = fgets(buf, sizeof buf, f) != nullptr;
  fclose(f);
  if (!ok) return false;
  CPU_ZERO(set);
  int n = 0;
  for (char* q = buf; *q && *q != '\n';) {
    char* e = nullptr;
    const long a = strtol(q, &e, 10);
    if (e == q) break;
    long b = a;
    if (*e == '-') b = strtol(e + 1, &e, 10);
    for (long c = a; c <= b && c < CPU_SETSIZE; c++) CPU_SET((int)c, set), n++;
    q = *e == ',' ? e + 1 : e;
  }
  return n > 0;
}

// The CPU set TIPS_NEG_BIND asks for around `cpu` (the starting thread's), within the process's
// affinity; false: leave the thread unbound.
bool neg_bind_set(int cpu, cpu_set_t* out) {
  const char* v = getenv("TIPS_NEG_BIND");
  if (!v || !*v) v = "l3";
  if (!strcmp(v, "0") || !strcmp(v, "off") || cpu < 0) return false;
  const std::string base = "/sys/devices/system/cpu/cpu" + std::to_string(cpu);
  cpu_set_t want;
  if (!strcmp(v, "l3")) {
    if (!cpu_list(base + "/cache/index3/shared_cpu_list", &want)) return false;
  } else if (!strcmp(v, "core")) {
    if (!cpu_list(base + "/topology/thread_siblings_list", &want)) return false;
  } else {
    return false;
  }
  cpu_set_t allowed = process_cpus();
  CPU_AND(out, &want, &allowed);
  return CPU_COUNT(out) > 0;
}

// At the top of a negotiation thread: its name, and its CPUs when TIPS_NEG_BIND asks.
void neg_thread_setup(const char* name, int start_cpu) {
  (void)pthread_setname_np(pthread_self(), name);
  cpu_set_t set;
  if (neg_bind_set(start_cpu, &set)) (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
}

class Negotiator {
 public:
  // Rank 0 listens on the first free port of [port, port + kPortTries); every other rank connects
  // and says hello {magic, job key, rank, size}; rank 0 answers {magic, job key}. A rank counts as
  // joined only after that answer: a connect that reached another program's listener on one of
  // these ports (RCCL's own sockets live in the same ephemeral range), or this socket itself
  // (TCP simultaneous open), is closed and the next candidate tried, instead of leaving rank 0
  // waiting for a rank that believes it has joined.
  static constexpr int kPortTries = 16;
  static constexpr uint64_t kMagic = 0x30474e4553504954ull;  // "TIPSNEG0"
  static constexpr uint64_t kConfirm = 0x31474e4553504954ull;  // "TIPSNEG1"
  struct Hello {
    uint64_t magic, key;
    int32_t rank, size;
    int64_t sync_direct;  // synchronous collectives this rank issued before the negotiation started
  };
  struct Ack {
    uint64_t magic, key;
  };

  // The join, a collective with one verdict for every rank:
  //   joiner -> rank 0: Hello; rank 0 -> joiner: Ack; joiner -> rank 0: Confirm (it has the Ack and is
  //   committed). Rank 0 counts a rank as joined only at its Confirm: a joiner that gave up before
  //   the Ack arrived (it closed the socket) is not counted and its retry is accepted later.
  //   Once every rank is in, rank 0 sends each the verdict: every rank must have issued the same
  //   number of synchronous collectives before this point (their RCCL calls pair up only then).
  int start(int rank, int size, const char* host, int port, bool dry_run, int timeout_s, uint64_t key = 0,
            int64_t sync_direct = 0) {
    rank_ = rank;
    size_ = size;
    dry_ = dry_run;
    timeout_ms_ = timeout_s * 1000;
    table_.p = size;
    by_name_.reserve(4096);  // (no rehash under the lock for a few thousand requests in flight)
    by_handle_.reserve(4096);
    std::string err;
    if (size > 1) {
      const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms_);
      auto ms_left = [&] {
        const auto l = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now()).count();
        return l > 0 ? (int)l : 0;
      };
      if (rank == 0) {
        for (int k = 0; k < kPortTries && lfd_ < 0; k++) lfd_ = listen_on(port + k, size, &err);
        if (lfd_ < 0) return fail(TIPS_ERR_BOOTSTRAP, "negotiation: ports %d-%d: %s", port, port + kPortTries - 1, err.c_str());
        peers_.assign(size, -1);
        std::vector<int64_t> counts(size, sync_direct);
        for (int joined = 0; joined < size - 1;) {
          pollfd pfd{lfd_, POLLIN, 0};
          if (ms_left() <= 0 || ::poll(&pfd, 1, ms_left()) <= 0)
            return fail(TIPS_ERR_BOOTSTRAP, "negotiation: %d rank(s) did not connect", size - 1 - joined);
          int c = ::accept(lfd_, nullptr, nullptr);
          if (c < 0) continue;
          Hello h{};
          const Ack a{kMagic, key};
          uint64_t confirm = 0;
          if (!recv_all(c, &h, sizeof h, 2000) || h.magic != kMagic || h.key != key || h.size != size || h.rank <= 0 ||
              h.rank >= size || !send_all(c, &a, sizeof a)) {
            ::close(c);
            continue;
          }
          if (!recv_all(c, &confirm, sizeof confirm, 2000) || confirm != kConfirm) {
            unconfirmed_joins()++;  // the joiner gave up on this connection; it will try again
            ::close(c);
            continue;
          }
          set_nodelay(c);
          if (peers_[h.rank] >= 0) {  // (a rank whose earlier connection was confirmed and then lost: its latest wins)
            ::close(peers_[h.rank]);
            joined--;
          }
          peers_[h.rank] = c;
          counts[h.rank] = h.sync_direct;
          joined++;
        }
        std::string verdict;
        for (int r = 1; r < size && verdict.empty(); r++)
          if (counts[r] != counts[0])
            verdict = "rank " + std::to_string(r) + " issued " + std::to_string(counts[r]) +
                      " synchronous collectives before the negotiation started, rank 0 issued " +
                      std::to_string(counts[0]) + ": the first named request must come at the same point of "
                      "the collective order on every rank";
        Writer w;
        w.put<uint8_t>(verdict.empty() ? 1 : 0);
        w.str(verdict);
        for (int r = 1; r < size; r++) (void)send_msg(peers_[r], w.b);
        if (!verdict.empty()) {
          close_all();
          return fail(TIPS_ERR_MISMATCH, "negotiation: %s", verdict.c_str());
        }
      } else {
        const Hello h{kMagic, key, rank, size, sync_direct};
        static std::atomic<int> drop_first{-1};  // TIPS_TEST_DROP_FIRST_HELLO=1 (tests only): abandon the
        if (drop_first.load() < 0) {             // first connection right after its hello, as a joiner
          const char* v = getenv("TIPS_TEST_DROP_FIRST_HELLO");  // whose answer timed out would
          int expect = -1;
          drop_first.compare_exchange_strong(expect, v ? atoi(v) : 0);
        }
        while (up_ < 0) {
          for (int k = 0; k < kPortTries && up_ < 0; k++) {
            sockaddr_in sa;
            if (!resolve(host, port + k, &sa)) return fail(TIPS_ERR_BOOTSTRAP, "negotiation: cannot resolve %s", host);
            const int fd = connect_peer(sa);
            if (fd < 0) continue;
            Ack a{};
            const uint64_t confirm = kConfirm;
            if (send_all(fd, &h, sizeof h) && drop_first.load() > 0) {
              drop_first--;
              ::close(fd);
              continue;
            }
            if (recv_all(fd, &a, sizeof a, 5000) && a.magic == kMagic && a.key == key &&
                send_all(fd, &confirm, sizeof confirm)) {
              set_nodelay(fd);
              up_ = fd;
            } else {
              ::close(fd);
            }
          }
          if (up_ >= 0) break;
          if (ms_left() <= 0)
            return fail(TIPS_ERR_BOOTSTRAP, "negotiation: rank %d could not reach rank 0 at %s:%d-%d", rank, host, port,
                        port + kPortTries - 1);
          std::this_thread::sleep_for(std::chrono::milliseconds(20));
        }
        std::string v;
        if (!recv_msg(up_, &v, std::max(ms_left(), 1000))) {
          close_all();
          return fail(TIPS_ERR_BOOTSTRAP, "negotiation: rank %d got no verdict from rank 0", rank);
        }
        Reader rd(v);
        const bool ok = rd.get<uint8_t>() != 0;
        const std::string msg = rd.str();
        if (!ok || !rd.ok) {
          close_all();
          return fail(TIPS_ERR_MISMATCH, "negotiation: %s", rd.ok ? msg.c_str() : "malformed verdict");
        }
      }
    }
    lockfree_ = env_i64("TIPS_ENQUEUE_LOCKFREE", 1) != 0;
    running_ = true;
    accepting_.store(true, std::memory_order_release);
    start_cpu_ = sched_getcpu();  // (the starting thread's CPU: TIPS_NEG_BIND's anchor)
    thread_ = std::thread([this] {
      tl_negotiation_thread = true;
      neg_thread_setup("tips-neg", start_cpu_);
      loop();
    });
    return 0;
  }

  void close_all() {
    for (int& fd : peers_)
      if (fd >= 0) ::close(fd), fd = -1;
    if (up_ >= 0) ::close(up_);
    if (lfd_ >= 0) ::close(lfd_);
    up_ = lfd_ = -1;
  }

  // A request made ready for the tables outside their lock (enqueue, enqueue_list)
  struct Prepared {
    std::shared_ptr<Req> r;
    NameMap::node_type name_node;
    HandleMap::node_type handle_node;
  };

  // Everything of an enqueue that needs no lock: the request, where its memory lives, its two
  // table entries (allocated here: executor threads enqueue at once, and the lock's hold time, not
  // the work, bounded them - 4 threads enqueueing config 5 were no faster than one).
  int prepare(Prepared& p, const std::string& name, const void* in, void* out, const int64_t* shape, int ndim,
              int dtype, hipStream_t s, int type, int root, tips_alloc_fn alloc, void* actx, int64_t* out_rows,
              std::function<int()> body, PtrRanges* pr, bool handle_entry = true) {
    if (ndim < 0 || ndim > TIPS_MAX_DIMS) return fail(TIPS_ERR_INVALID_ARG, "bad ndim %d", ndim);
    if (type == TIPS_REQ_ALLGATHER && ndim < 1) return fail(TIPS_ERR_INVALID_ARG, "An empty tensor found");
    auto r = std::make_shared<Req>();
    r->body = std::move(body);
    r->name = name;
    r->name_hash = std::hash<std::string>()(name);
    r->type = type;
    r->root = root;
    r->alloc = alloc;
    r->actx = actx;
    r->out_rows = out_rows;
    r->in = in;
    r->out = out;
    r->count = 1;
    r->shape.reserve((size_t)std::max(ndim, 1));
    for (int d = 0; d < ndim; d++) {
      if (shape[d] < 0) return fail(TIPS_ERR_INVALID_ARG, "negative dimension");
      r->shape.push_back(shape[d]);
      r->count *= shape[d];
    }
    if (ndim == 0) r->shape.push_back(1);  // a scalar travels as shape [1] (CreateNoEmptyTfShape, coordinator.cc:212-221)
    r->dtype = dtype;
    r->stream = s;
    if (!dry_ && !r->body && r->count > 0) {  // the real executor (the dry run touches no memory; a routed body checks its own)
      // device tensors run stream-ordered on `s`; host tensors (the reference's MPIAllreduce is a
      // CPU op, ops.cc:118) run synchronously on the executor thread, staged through HBM as
      // tips_allreduce stages them. Both pointers of a request live on the same side. A list
      // enqueue knows its allocations (pr: one HIP lookup per segment) and checks here; a single
      // request is classified by the negotiation thread (Req::classify).
      static const bool at_enqueue = env_i64("TIPS_CLASSIFY_AT_ENQUEUE", 0) != 0;  // (A/B: round 3's place)
      PtrRanges one;
      if (!pr && at_enqueue) pr = &one;
      if (pr) {
        const bool din = pr->is_device(in), dout = type == TIPS_REQ_ALLGATHER ? din : pr->is_device(out);
        if (din != dout) return fail(TIPS_ERR_INVALID_ARG, "named request %s: one device and one host pointer", name.c_str());
        r->host = !din;
      } else {
        r->classify = true;
      }
    }
    {  // handles in per-thread blocks of a process-wide counter: unique across negotiators, and one
       // contended increment per 256 requests instead of one per request
      thread_local int64_t tl_next = 0, tl_end = 0;
      if (tl_next == tl_end) {
        tl_next = g_next_handle.fetch_add(256) + 1;
        tl_end = tl_next + 256;
      }
      r->handle = tl_next++;
    }
    thread_local NameMap name_scratch;
    thread_local HandleMap handle_scratch;
    name_scratch.emplace(NameKey{r->name_hash, name}, r);
    p.name_node = name_scratch.extract(name_scratch.begin());
    if (handle_entry) {  // (a request enqueued with its callback has none: nothing looks it up)
      handle_scratch.emplace(r->handle, r);
      p.handle_node = handle_scratch.extract(handle_scratch.begin());
    }
    p.r = std::move(r);
    return 0;
  }

  // Under m_: the request's table entries and the fresh queue. The handle, or < 0. (Its completion
  // event, if it ever needs one, is taken when it runs: take_event.)
  int64_t commit(Prepared& p) {
    Req& r = *p.r;
    if (!running_) return fail(TIPS_ERR_NOT_INITIALIZED, "negotiation thread is not running");
    if (!by_name_.insert(std::move(p.name_node)).inserted)
      return fail(TIPS_ERR_INVALID_ARG, "a request named %s is already pending", r.name.c_str());
    if (p.handle_node) by_handle_.insert(std::move(p.handle_node));
    admit(std::move(p.r));
    return r.handle;
  }

  int64_t enqueue(const std::string& name, const void* in, void* out, const int64_t* shape, int ndim, int dtype,
                  hipStream_t s, int type = TIPS_REQ_ALLREDUCE, int root = 0, tips_alloc_fn alloc = nullptr,
                  void* actx = nullptr, int64_t* out_rows = nullptr, std::function<int()> body = nullptr,
                  PtrRanges* pr = nullptr, tips_done_fn cb = nullptr, void* cb_ctx = nullptr) {
    Prepared p;
    TRY(prepare(p, name, in, out, shape, ndim, dtype, s, type, root, alloc, actx, out_rows, std::move(body), pr,
                cb == nullptr));
    if (cb) {  // tips_enqueue_allreduce_cb: the callback travels with the request (one lock, as OpRecord)
      p.r->cb = cb;
      p.r->cb_ctx = cb_ctx;
      p.r->cb_only = true;
    }
    // (no st.mu: the executor holds it while it reduces, and nothing here needs it)
    if (cb && !waiter_started_.load(std::memory_order_acquire)) {
      std::lock_guard<AdaptiveMutex> l(m_);
      // (only while running: a waiter started after stop() joined the last one is never joined,
      // and the negotiator's destructor would end the process on it - ADVICE r05)
      if (!running_ || waiter_stop_) return fail(TIPS_ERR_NOT_INITIALIZED, "negotiation thread is not running");
      start_waiter_locked();
    }
    if (!lockfree_) {  // (TIPS_ENQUEUE_LOCKFREE=0: round 4's locked commit, for A/B runs only)
      std::unique_lock<AdaptiveMutex> l(m_);
      drain_locked();
      const int64_t h = commit(p);
      if (h > 0) {
        last_arrival_ns_.store(steady_ns(), std::memory_order_release);
        if (fresh_.size() == 1) cv_.notify_all();
      }
      return h;
    }
    if (!accepting_.load(std::memory_order_acquire))
      return fail(TIPS_ERR_NOT_INITIALIZED, "negotiation thread is not running");
    const int64_t h = p.r->handle;
    static std::atomic<int64_t> gap_us{-1};  // (tests: TIPS_TEST_ENQUEUE_GAP_US widens the check-to-push window)
    int64_t gap = gap_us.load(std::memory_order_relaxed);
    if (gap < 0) gap_us.store(gap = std::max<int64_t>(0, env_i64("TIPS_TEST_ENQUEUE_GAP_US", 0)), std::memory_order_relaxed);
    if (gap > 0) std::this_thread::sleep_for(std::chrono::microseconds(gap));
    Pending* node = new Pending{std::move(p), nullptr};
    // (each thread pushes onto its own shard of the stack: drain_locked walks the shards' chains
    // side by side, so their cache misses overlap)
    thread_local const int tl_shard = (int)(g_next_shard.fetch_add(1, std::memory_order_relaxed) % kShards);
    std::atomic<Pending*>& head = shards_[tl_shard].head;
    Pending* old = head.load(std::memory_order_relaxed);
    do {
      node->next = old;
    } while (!head.compare_exchange_weak(old, node, std::memory_order_seq_cst, std::memory_order_relaxed));
    // the linger's quiet time, to a few microseconds (a store per request would bounce the line)
    const int64_t now = steady_ns();
    if (now - last_arrival_ns_.load(std::memory_order_relaxed) > 2000)
      last_arrival_ns_.store(now, std::memory_order_release);
    // Wake the background thread only while it waits idle for a cycle's first request (idle_):
    // lingering, it sees later arrivals anyway, and a wake there would cut its linger window short
    // and make this thread wait for m_. The push and the flag are sequentially consistent and the
    // thread sets the flag before it checks the stack, so a wake cannot be lost; under m_, so it
    // cannot fall between that check and the wait.
    if (!old && idle_.load(std::memory_order_seq_cst)) {
      std::lock_guard<AdaptiveMutex> l(m_);
      cv_.notify_all();
    }
    // A stop may have closed the door between the check above and the push, and run its last
    // drain before the push: nobody would ever admit this node, and a callback request's done()
    // would never fire. The push and this load are sequentially consistent, as are
    // stop's store and its drain's exchange: either that drain saw the node, or this load sees the
    // door closed and the node is failed here.
    if (!accepting_.load(std::memory_order_seq_cst)) reclaim_after_stop();
    return h;
  }

  // (the lock-free enqueue, after a stop) Fail whatever is left on the submission stacks. While the
  // completion thread still runs it calls the callbacks (drain_locked queues them); once it has
  // ended they are called here, outside the lock, as the completion thread would.
  void reclaim_after_stop() {
    std::vector<std::shared_ptr<Req>> orphans;
    {
      std::lock_guard<AdaptiveMutex> l(m_);
      drain_locked(waiter_stop_ ? &orphans : nullptr);
    }
    for (auto& r : orphans) r->cb(r->cb_ctx, r->code, r->err.c_str());
  }

  // (m_ held) the completion thread, if it is not running yet
  void start_waiter_locked() {
    if (!waiter_.joinable())
      waiter_ = std::thread([this] {
        neg_thread_setup("tips-done", start_cpu_);
        waiter_loop();
      });
    waiter_started_.store(true, std::memory_order_release);
  }

  // (m_ held) Admit the lock-free stack's requests to the tables, each thread's in its order, as
  // commit() does for a list; a request that cannot be admitted (a duplicate name, the thread stopped) fails
  // through its handle or callback instead of at its enqueue.
  // orphans: the completion thread has ended; failed callback requests go there instead of to it.
  int drain_locked(std::vector<std::shared_ptr<Req>>* orphans = nullptr) {
    Pending* heads[kShards];
    int m = 0;
    for (Shard& sh : shards_)  // (seq_cst: pairs with the enqueue's push and its re-check after a stop)
      if (Pending* h = sh.head.exchange(nullptr, std::memory_order_seq_cst)) heads[m++] = h;
    if (!m) return 0;
    int count = 0;
    int64_t t = adm_prof_ ? steady_ns() : 0;
    auto lap = [&](int k) {  // (TIPS_NEG_TRACE: where an admission's time goes)
      if (!adm_prof_) return;
      const int64_t u = steady_ns();
      adm_ns_[k] += u - t;
      t = u;
    };
    // Each chain reversed to its thread's order, one node of every chain per step: the nodes and
    // requests were written by other cores, and the walks' misses overlap instead of following one
    // another (the requests are fetched while the walk goes on, for the admissions below).
    Pending* rev[kShards] = {};
    for (bool more = true; more;) {
      more = false;
      for (int k = 0; k < m; k++)
        if (Pending* h = heads[k]) {
          heads[k] = h->next;
          __builtin_prefetch(h->p.r.get(), 1);
          h->next = rev[k];
          rev[k] = h;
          more = true;
        }
    }
    lap(0);
    for (int k = 0; k < m; k++) {
      for (Pending* q = rev[k]; q;) {
        Pending* n = q->next;
        Prepared& p = q->p;
        Req& r = *p.r;
        std::string why;
        int code = TIPS_ERR_INVALID_ARG;
        if (!running_) {
          why = "negotiation thread is not running";
          code = TIPS_ERR_NOT_INITIALIZED;
        }
        if (why.empty() && !by_name_.insert(std::move(p.name_node)).inserted)
          why = "a request named " + r.name + " is already pending";
        lap(1);
        if (p.handle_node) by_handle_.insert(std::move(p.handle_node));
        lap(2);
        if (why.empty()) {
          admit(std::move(p.r));
        } else {
          r.state = -1;
          r.code = code;
          r.err = why;
          if (r.cb) {
            if (orphans) orphans->push_back(p.r);
            else queue_done(p.r);
          }
          cv_.notify_all();
        }
        lap(3);
        delete q;
        lap(4);
        q = n;
        count++;
      }
    }
    return count;
  }

  // (m_ held) A request joins the next announce; counted when the previous batch named it
  void admit(std::shared_ptr<Req>&& r) {
    if (!expect_.empty() && std::binary_search(expect_.begin(), expect_.end(), r->name_hash)) expect_hits_++;
    fresh_.push_back(std::move(r));
  }

  // A list (tips_enqueue_*_n): every request prepared before the lock, all of them committed under
  // one hold, one wake-up. The negotiation then sees the list arrive at once instead of lingering
  // through it (1000 requests one lock each took ~0.9 ms on the GPU box). handles[i] < 0 entries
  // (refused before, or here) are skipped / set; returns the first refusal or 0.
  int enqueue_list(std::vector<Prepared>& ps, int64_t* handles, std::string* first_err) {
    int rc = 0;
    std::unique_lock<AdaptiveMutex> l(m_);
    drain_locked();  // (earlier single enqueues first)
    bool any = false;
    for (size_t i = 0; i < ps.size(); i++) {
      if (!ps[i].r) continue;
      handles[i] = commit(ps[i]);
      if (handles[i] < 0 && rc == 0) {
        rc = (int)handles[i];
        *first_err = last_error();
      }
      any |= handles[i] > 0;
    }
    if (any) {
      last_arrival_ns_.store(steady_ns(), std::memory_order_release);
      cv_.notify_all();
    }
    return rc;
  }

  // 1 = done, 0 = pending, < 0 = error; a finished handle is released by the call that reports it.
  // routed = the caller of a routed collective: waits until its body has run (state 3), never for
  // device completion (the body queued that on the caller's stream, as a direct call would).
  int poll(int64_t h, bool block, bool routed = false) {
    std::shared_ptr<Req> r;
    {
      std::unique_lock<AdaptiveMutex> l(m_);
      drain_locked();
      auto it = by_handle_.find(h);
      if (it == by_handle_.end()) return fail(TIPS_ERR_INVALID_ARG, "unknown request handle %lld", (long long)h);
      r = it->second;
      if (r->cb) return fail(TIPS_ERR_INVALID_ARG, "request %s completes through its callback (tips_on_done)", r->name.c_str());
      if (block) cv_.wait(l, [&] { return r->state >= 2 || r->state < 0; });
      if (r->state == 0 || r->state == 1) return 0;
    }
    int rc = 1;
    if (r->state < 0) {
      rc = fail(r->code, "%s", r->err.c_str());
    } else if (r->state == 2 && !routed && !(r->gev && r->gev->done.load(std::memory_order_acquire))) {
      hipEvent_t ev = r->gev ? r->gev->ev : r->ev;
      hipError_t e = block ? hipEventSynchronize(ev) : hipEventQuery(ev);
      if (e == hipErrorNotReady) return 0;
      if (e != hipSuccess) rc = fail(TIPS_ERR_HIP, "request %s: %s", r->name.c_str(), hipGetErrorString(e));
      else if (r->gev) r->gev->done.store(true, std::memory_order_release);
    }
    release(h, r);
    return rc;
  }

  void release(int64_t h, const std::shared_ptr<Req>& r) {
    std::lock_guard<AdaptiveMutex> l(m_);
    if (r->ev) ev_pool_.push_back(r->ev);  // reused by the next request
    r->ev = nullptr;
    r->gev.reset();
    by_handle_.erase(h);
  }

  // tips_on_done: fn(ctx, status, message) is called once, from the completion thread, when the
  // request has finished (a device request: when its work on the device is done); the handle is
  // released then. A request that has already finished is queued at once.
  int on_done(int64_t h, tips_done_fn fn, void* ctx) {
    std::lock_guard<AdaptiveMutex> l(m_);
    drain_locked();
    auto it = by_handle_.find(h);
    if (it == by_handle_.end()) return fail(TIPS_ERR_INVALID_ARG, "unknown request handle %lld", (long long)h);
    auto& r = it->second;
    if (r->cb) return fail(TIPS_ERR_INVALID_ARG, "request %s already has a completion callback", r->name.c_str());
    if (waiter_stop_) {  // (after stop: no completion thread will come; the request has finished)
      fn(ctx, r->state < 0 ? r->code : 0, r->state < 0 ? r->err.c_str() : "");
      return 0;
    }
    r->cb = fn;
    r->cb_ctx = ctx;
    start_waiter_locked();
    if (r->state >= 2 || r->state < 0) queue_done(r);
    return 0;
  }

  // collective: every rank's loop learns from rank 0 that all ranks asked to stop
  int stop() {
    {
      std::lock_guard<AdaptiveMutex> l(m_);
      if (!running_ && !thread_.joinable() && !waiter_.joinable()) return 0;
      want_stop_ = true;
      cv_.notify_all();
    }
    if (thread_.joinable()) thread_.join();
    {  // the completion thread drains what is queued (the loop failed every unmatched request), then ends
      std::lock_guard<AdaptiveMutex> l(m_);
      accepting_.store(false, std::memory_order_seq_cst);
      drain_locked();  // enqueued during the stop: failed (not running)
      waiter_stop_ = true;
      done_cv_.notify_all();
    }
    if (waiter_.joinable()) waiter_.join();
    close_all();
    peers_.clear();
    release_device_resources();
    return loop_err_.empty() ? 0 : fail(TIPS_ERR_BOOTSTRAP, "%s", loop_err_.c_str());
  }

  // number of completion callbacks called so far (the selftest's log)
  // decisions that came back as "cached OK" (the response cache; read after stop())
  int64_t cached_decisions() const { return cached_decisions_.load(std::memory_order_relaxed); }

  int64_t callbacks_called() {
    std::lock_guard<AdaptiveMutex> l(m_);
    return cb_called_;
  }

  // The negotiation's own HIP objects, released by stop() (a stopped negotiator can
  // outlive it in a thread's cached() copy, and its destructor may then run at any time, even
  // after tips_shutdown or during the runtime's teardown at exit). Only host memory is left to the
  // destructor, plus the events of requests nobody polled after the stop.
  void release_device_resources() {
    std::vector<hipEvent_t> evs;
    {
      std::lock_guard<AdaptiveMutex> l(m_);
      evs.swap(ev_pool_);
    }
    for (hipEvent_t e : evs) (void)hipEventDestroy(e);
    join_ev_.release();
    if (neg_stream_) (void)hipStreamDestroy(neg_stream_);
    neg_stream_ = nullptr;
  }

  ~Negotiator() {
    {  // a completion thread still running (the negotiator was never stopped): let it drain, join it
      std::lock_guard<AdaptiveMutex> l(m_);
      waiter_stop_ = true;
      done_cv_.notify_all();
    }
    if (waiter_.joinable()) waiter_.join();
    std::vector<std::shared_ptr<Req>> orphans;  // never admitted: failed, their callbacks called
    {
      std::lock_guard<AdaptiveMutex> l(m_);
      running_ = false;
      drain_locked(&orphans);
    }
    for (auto& r : orphans) r->cb(r->cb_ctx, r->code, r->err.c_str());
    for (auto& kv : by_handle_)  // never polled to completion
      if (kv.second->ev) ev_pool_.push_back(kv.second->ev);
    for (hipEvent_t e : ev_pool_) (void)hipEventDestroy(e);
    join_ev_.release();
    if (neg_stream_) (void)hipStreamDestroy(neg_stream_);
  }

  bool running() {
    std::lock_guard<AdaptiveMutex> l(m_);
    return running_;
  }
  std::vector<std::string> log() {
    std::lock_guard<AdaptiveMutex> l(m_);
    return log_;
  }
  void note(const std::string& s) {
    std::lock_guard<AdaptiveMutex> l(m_);
    log_.push_back(s);
  }

 private:
  void loop() {
    // The linger's timed waits end within a microsecond or two of their deadline, not Linux's
    // default 50 us timer slack later: the slack alone had each 30 us linger window last ~80 us,
    // three windows past a burst of 214 requests (TIPS_NEG_TIMER_SLACK_NS).
    (void)prctl(PR_SET_TIMERSLACK, (unsigned long)std::max<int64_t>(1, env_i64("TIPS_NEG_TIMER_SLACK_NS", 1000)), 0, 0, 0);
    const auto cycle = std::chrono::microseconds(std::max<int64_t>(50, env_i64("TIPS_CYCLE_TIME_US", 1000)));
    const auto linger = std::chrono::microseconds(std::max<int64_t>(0, env_i64("TIPS_BATCH_LINGER_US", 30)));
    // TIPS_LINGER_SPIN=1: spin through the linger instead of timed waits. With the 1 us timer slack
    // below it ended cycles no sooner (38-112 us after the latest arrival against 55-80 us waiting,
    // profiles/r05/aa_op_host_ab.txt) and keeps a core busy, so it is off.
    const bool spin_linger = env_i64("TIPS_LINGER_SPIN", 0) != 0;
    // Once every name of the last two cycles is in again (a training step's gradients: the same
    // names every step), the linger ends after TIPS_LINGER_EXPECT_US of quiet instead of
    // TIPS_BATCH_LINGER_US: the 30 us quiet time exists to catch the rest of a burst, and the burst
    // is known to be complete. A step that adds requests after them goes on in the next cycle. (Two
    // cycles, not one: a step that was split over two cycles once, its executor threads issuing in
    // another order the next step, would otherwise keep splitting.) TIPS_LINGER_EXPECT=0: off.
    // (Delimiting steps by the thread's idle waits does not work: the next step's first requests
    // arrive while this cycle still executes.)
    const bool expect_on = env_i64("TIPS_LINGER_EXPECT", 1) != 0;
    const int64_t expect_quiet_ns = 1000 * std::max<int64_t>(0, env_i64("TIPS_LINGER_EXPECT_US", 4));
    // (the waits while the set is not complete are stepped, so its completion is seen within this)
    const int64_t expect_step_ns = 8000;
    std::vector<std::shared_ptr<Req>> prev;  // the previous cycle's named requests
    auto complete = [&] { return expect_on && !expect_.empty() && expect_hits_ == expect_.size(); };
    // TIPS_NEG_TRACE=1: per cycle with requests, on stderr: the batch, and how long the linger, the
    // exchange with rank 0 and the execution took (microseconds)
    const bool trace = env_i64("TIPS_NEG_TRACE", 0) != 0;
    {
      std::lock_guard<AdaptiveMutex> l(m_);
      adm_prof_ = trace;
    }
    auto us_since = [](std::chrono::steady_clock::time_point t) {
      return (long long)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t).count();
    };
    // (kept across cycles: the announce, the response and the decided list reuse their buffers)
    Writer w;
    std::string resp;
    std::vector<Decision> ds;
    std::vector<uint32_t> cids;
    std::vector<Req*> full;
    // TIPS_RESPONSE_CACHE=0: announce every request in full (A/B; every rank keeps the cache's
    // bookkeeping either way, so ranks may differ in this setting). Rank 0 counts ids in a 64-bit
    // rank mask: above 64 ranks everything travels in full.
    const bool send_ids = env_i64("TIPS_RESPONSE_CACHE", 1) != 0 && size_ <= 64;
    while (true) {
      std::vector<std::shared_ptr<Req>> batch;
      bool stopping;
      set_phase("waiting for requests");
      long long t_linger = 0, t_tail = 0;
      int windows = 0, last_drained = 0;
      int64_t drain_ns = 0, last_drain_ns = 0, wait_ns = 0;
      auto timed_drain = [&] {  // (the trace's account of the admissions)
        const int64_t a = steady_ns();
        last_drained = drain_locked();
        last_drain_ns = steady_ns() - a;
        drain_ns += last_drain_ns;
      };
      {
        std::unique_lock<AdaptiveMutex> l(m_);
        idle_.store(true, std::memory_order_seq_cst);
        cv_.wait_for(l, cycle, [&] {
          return !fresh_.empty() || any_pending() || want_stop_;
        });
        idle_.store(false, std::memory_order_relaxed);
        drain_locked();
        // Linger while requests keep arriving (a gradient list is enqueued in a burst), so one
        // cycle announces - and one fused batch reduces - the whole burst instead of its first
        // few tensors. Bounded by the cycle time; TIPS_BATCH_LINGER_US = 0 turns it off.
        const auto t0 = std::chrono::steady_clock::now();
        windows = 0;
        if (!fresh_.empty() && !want_stop_ && linger.count() > 0) {
          // Until TIPS_BATCH_LINGER_US have passed since the latest arrival (bounded by the cycle):
          // each wait lasts just what is left of that quiet time. (Round 3 waited in whole 30 us
          // windows until one saw no arrival; a timed wait oversleeps by ~50 us on the GPU box, so
          // a cycle lingered one to two 83 us windows past the burst. Spinning instead was no
          // faster within noise and kept a core busy: profiles/r04/zs_op_linger_ab.txt.)
          const int64_t start = steady_ns(), linger_ns = (int64_t)linger.count() * 1000,
                        cycle_ns = (int64_t)cycle.count() * 1000;
          while (!want_stop_) {
            timed_drain();  // admit what arrived so far while the burst goes on, not all of it after
            const int64_t now = steady_ns(), quiet = now - last_arrival_ns_.load(std::memory_order_acquire);
            const bool done = complete();
            const int64_t need = done ? std::min(expect_quiet_ns, linger_ns) : linger_ns;
            if (quiet >= need || now - start >= cycle_ns) break;
            windows++;
            if (spin_linger) {
              // Spin (without m_) until the quiet time is reached, bounded by one linger window; the
              // loop re-checks.
              l.unlock();
              const int64_t stop_at = std::min(now + linger_ns, start + cycle_ns);
              for (int64_t t = steady_ns(); t < stop_at; t = steady_ns()) {
                if (t - last_arrival_ns_.load(std::memory_order_acquire) >= linger_ns) break;
                __builtin_ia32_pause();
              }
              l.lock();
            } else {
              int64_t wait = std::min(need - quiet, cycle_ns - (now - start));
              if (expect_on && !expect_.empty() && !done) wait = std::min(wait, expect_step_ns);
              const int64_t a = steady_ns();
              cv_.wait_for(l, std::chrono::nanoseconds(wait));
              wait_ns += steady_ns() - a;
            }
          }
        }
        timed_drain();
        batch.assign(fresh_.begin(), fresh_.end());
        fresh_.clear();
        if (expect_on) {  // the next cycle expects this one's names and the previous one's
          std::vector<std::shared_ptr<Req>> cur;  // (routed ~sync requests are named per call: never expected)
          for (auto& r : batch)
            if (r->name.compare(0, 6, "~sync.") != 0) cur.push_back(r);
          // (kept as it is when this cycle named exactly the expected set: the previous one's
          // names are in it already)
          if (!cur.empty() && !(expect_hits_ == expect_.size() && cur.size() == expect_.size())) {
            expect_.clear();
            for (auto& r : cur) expect_.push_back(r->name_hash);
            for (auto& r : prev) expect_.push_back(r->name_hash);
            std::sort(expect_.begin(), expect_.end());
            expect_.erase(std::unique(expect_.begin(), expect_.end()), expect_.end());
          }
          if (!cur.empty()) prev.swap(cur);
          expect_hits_ = 0;
        }
        for (auto& r : batch) r->state = 1;
        stopping = want_stop_;
        t_linger = us_since(t0);
        t_tail = (steady_ns() - last_arrival_ns_.load(std::memory_order_acquire)) / 1000;
      }
      for (auto& r : batch)
        if (r->classify) {  // (see Req::classify; nothing else reads host / bad before execute)
          const bool din = is_device_ptr(r->in), dout = r->type == TIPS_REQ_ALLGATHER ? din : is_device_ptr(r->out);
          if (din != dout) r->bad = "one device and one host pointer";
          r->host = !din;
          r->classify = false;
        }
      const auto t_x = std::chrono::steady_clock::now();
      w.b.clear();
      w.put<uint8_t>(stopping ? 1 : 0);
      // a request the response cache holds with the same dtype and shape travels as its cache id
      // (4 bytes; rank 0 counts it without a name); the rest as full records
      cids.clear();
      full.clear();
      for (auto& r : batch) {
        const int32_t id = send_ids ? cached_id(*r) : -1;
        if (id >= 0) cids.push_back((uint32_t)id);
        else full.push_back(r.get());
      }
      w.put<uint32_t>((uint32_t)full.size());
      for (Req* r : full) {
        w.put<int32_t>(r->type);
        w.put<int32_t>(r->root);
        w.put<uint8_t>(r->bad.empty() ? 0 : 1);
        w.put<int32_t>(r->dtype);
        w.put<int64_t>(r->count);
        w.put<uint32_t>((uint32_t)r->shape.size());
        for (int64_t d : r->shape) w.put<int64_t>(d);
        w.str(r->name);
      }
      w.put<uint32_t>((uint32_t)cids.size());
      for (uint32_t id : cids) w.put<uint32_t>(id);
      set_phase("exchange (cycle " + std::to_string((long long)cycles_) + ", announcing " + std::to_string(batch.size()) + ")");
      if (!exchange(w.b, &resp)) break;
      {
        std::lock_guard<std::mutex> l(phase_mu_);
        cycles_++;
      }
      Reader rd(resp);
      const bool shutdown = rd.get<uint8_t>() != 0;
      const uint32_t n = rd.get<uint32_t>();
      size_t nd = 0;
      for (uint32_t i = 0; i < n && rd.ok; i++) {
        if (nd == ds.size()) ds.emplace_back();
        Decision& d = ds[nd++];  // (a kept slot: its strings keep their capacity)
        const uint8_t tag = rd.get<uint8_t>();
        d.sizes.clear();
        d.err.clear();
        if (tag == kCachedOk) {  // a cached allreduce every rank announced by id
          const uint32_t id = rd.get<uint32_t>();
          if (id >= cache_.size() || !cache_[id].live) {
            rd.ok = false;
            break;
          }
          d.ok = true;
          d.name.assign(cache_[id].name);
          cached_decisions_.fetch_add(1, std::memory_order_relaxed);
          continue;
        }
        d.ok = tag != 0;
        rd.str_into(d.name);
        rd.str_into(d.err);
        const uint32_t m = rd.get<uint32_t>();
        for (uint32_t k = 0; k < m && rd.ok && k < (1u << 20); k++) d.sizes.push_back(rd.get<int64_t>());
      }
      if (!rd.ok) {
        set_loop_error("negotiation: malformed response");
        break;
      }
      const long long t_exchange = us_since(t_x);
      const auto t_e = std::chrono::steady_clock::now();
      execute(ds, nd);
      if (trace && (!batch.empty() || nd))
        fprintf(stderr, "[tips neg] rank %d cycle %lld: announced %zu, decided %zu; linger %lld us (%d windows, "
                "ended %lld us after the latest arrival; waits %lld us, admissions %lld us, the last %d in %lld us), exchange %lld us "
                "(rank 0's decision %lld us), execute %lld us\n", rank_, (long long)cycles_, batch.size(), nd, t_linger, windows,
                t_tail, (long long)(wait_ns / 1000), (long long)(drain_ns / 1000), last_drained, (long long)(last_drain_ns / 1000),
                t_exchange, (long long)(rank_ == 0 ? decide_ns_ / 1000 : -1), us_since(t_e));
      if (trace && (!batch.empty() || nd)) {
        std::lock_guard<AdaptiveMutex> l(m_);
        fprintf(stderr, "[tips neg]   admission phases (us): walk %lld, name table %lld, handle table %lld, queue %lld, "
                "free %lld\n", (long long)(adm_ns_[0] / 1000), (long long)(adm_ns_[1] / 1000), (long long)(adm_ns_[2] / 1000),
                (long long)(adm_ns_[3] / 1000), (long long)(adm_ns_[4] / 1000));
        for (int64_t& x : adm_ns_) x = 0;
      }
      if (shutdown) break;
    }
    std::lock_guard<AdaptiveMutex> l(m_);
    accepting_.store(false, std::memory_order_seq_cst);
    drain_locked();  // (admitted while still running: they join the unmatched below)
    running_ = false;
    std::vector<std::string> unmatched;
    for (auto& kv : by_name_) unmatched.push_back(kv.first.s);
    std::sort(unmatched.begin(), unmatched.end());
    for (auto& name : unmatched) {  // never matched on every rank before the stop
      auto& r = by_name_.find(NameKey{std::hash<std::string>()(name), name})->second;
      r->state = -1;
      r->code = TIPS_ERR_MISMATCH;
      r->err = "request " + name + " was not enqueued on every rank before shutdown";
      if (dry_) log_.push_back(name + " ERR " + r->err);
      if (r->cb) queue_done(r);
    }
    by_name_.clear();
    cv_.notify_all();
  }

  // (m_ held) hand a finished request with a callback to the completion thread
  void queue_done(const std::shared_ptr<Req>& r) {
    if (r->cb_queued) return;
    r->cb_queued = true;
    done_q_.push_back(r);
    done_cv_.notify_all();
  }

  // The completion thread: in the order requests finished, wait for a device request's work, call
  // its callback (without the lock: a callback may enqueue more requests) and release its handle.
  // The completion thread: takes every queued request at once (a fused batch of host requests is
  // queued together: config 5's 214 in one go), runs each callback - for device work after its
  // event - and releases the batch's handles with one lock. Its phase for tips_debug_state is the
  // request it is at, formatted only when asked (a string per request cost ~1 ms per config-5 step).
  void waiter_loop() {
    std::deque<std::shared_ptr<Req>> batch;
    while (true) {
      {
        std::unique_lock<AdaptiveMutex> l(m_);
        done_cv_.wait(l, [&] { return !done_q_.empty() || waiter_stop_; });
        if (done_q_.empty()) return;
        batch.swap(done_q_);
      }
      for (auto& r : batch) {
        int status = 0;
        std::string msg;
        if (r->state < 0) {
          status = r->code;
          msg = r->err;
        } else if (r->state == 2 && !(r->gev && r->gev->done.load(std::memory_order_acquire))) {
          set_waiter_req(r, true);
          hipEvent_t ev = r->gev ? r->gev->ev : r->ev;
          const hipError_t e = hipEventSynchronize(ev);
          if (e != hipSuccess) {
            status = TIPS_ERR_HIP;
            msg = std::string("request ") + r->name + ": " + hipGetErrorString(e);
          } else if (r->gev) {
            r->gev->done.store(true, std::memory_order_release);
          }
        }
        set_waiter_req(r, false);
        r->cb(r->cb_ctx, status, msg.c_str());
      }
      set_waiter_req(nullptr, false);
      std::vector<HandleMap::node_type> gone;  // (freed after the lock: enqueueing threads wait on it)
      gone.reserve(batch.size());
      {
        std::lock_guard<AdaptiveMutex> l(m_);
        for (auto& r : batch) {  // (release() for the whole batch)
          if (r->ev) ev_pool_.push_back(r->ev);
          r->ev = nullptr;
          r->gev.reset();
          if (!r->cb_only) gone.push_back(by_handle_.extract(r->handle));
        }
        cb_called_ += (int64_t)batch.size();
      }
      gone.clear();
      batch.clear();
    }
  }

  // One lockstep cycle: my announce goes up, rank 0's decision comes back.
  bool exchange(const std::string& mine, std::string* resp) {
    if (size_ == 1) {
      const int64_t a = steady_ns();
      const bool ok = decide({mine}, resp);
      decide_ns_ = steady_ns() - a;
      return ok;
    }
    if (rank_ != 0) {
      if (!send_msg(up_, mine) || !recv_msg(up_, resp, timeout_ms_)) {
        set_loop_error("negotiation: lost rank 0");
        return false;
      }
      return true;
    }
    std::vector<std::string> all(size_);
    all[0] = mine;
    for (int r = 1; r < size_; r++)
      if (!recv_msg(peers_[r], &all[r], timeout_ms_)) {
        set_loop_error("negotiation: lost rank " + std::to_string(r));
        return false;
      }
    const int64_t a = steady_ns();
    if (!decide(all, resp)) return false;
    decide_ns_ = steady_ns() - a;
    for (int r = 1; r < size_; r++)
      if (!send_msg(peers_[r], *resp)) {
        set_loop_error("negotiation: lost rank " + std::to_string(r));
        return false;
      }
    return true;
  }

  // rank 0: fold every rank's announce into the table, answer with the ready list
  bool decide(const std::vector<std::string>& all, std::string* resp) {
    bool everyone_stops = true;
    for (int r = 0; r < (int)all.size(); r++) {
      Reader rd(all[r]);
      everyone_stops &= rd.get<uint8_t>() != 0;
      const uint32_t n = rd.get<uint32_t>();
      Announce a;  // (one, reused: its shape and name keep their allocations)
      for (uint32_t i = 0; i < n && rd.ok; i++) {
        a.shape.clear();
        a.type = rd.get<int32_t>();
        a.root = rd.get<int32_t>();
        a.bad = rd.get<uint8_t>() != 0;
        a.dtype = rd.get<int32_t>();
        a.count = rd.get<int64_t>();
        const uint32_t ndim = rd.get<uint32_t>();
        if (ndim > TIPS_MAX_DIMS) rd.ok = false;
        for (uint32_t d = 0; d < ndim && rd.ok; d++) a.shape.push_back(rd.get<int64_t>());
        rd.str_into(a.name);
        if (!rd.ok) break;
        // a full record of a name others announced by id this round: theirs join the table too
        if (!cache_ids_.empty()) {
          const int32_t id = cache_lookup(a.name, std::hash<std::string>()(a.name));
          if (id >= 0) to_table(id);
        }
        table_.announce(r, a);
      }
      const uint32_t k = rd.get<uint32_t>();
      for (uint32_t i = 0; i < k && rd.ok; i++) {
        const uint32_t id = rd.get<uint32_t>();
        if (id >= cache_.size() || !cache_[id].live) {
          rd.ok = false;
          break;
        }
        if (idst_.size() < cache_.size()) idst_.resize(cache_.size());
        IdState& st = idst_[id];
        const uint64_t bit = 1ull << r;
        if (st.table || (st.mask & bit)) {  // (a rank's second announce: the table names the duplicate)
          to_table(id);
          table_.announce(r, expand(id));
          continue;
        }
        st.mask |= bit;
        if (++st.n == (int)all.size()) {  // every rank, every one by id: ready, valid as cached
          st.mask = 0;
          st.n = 0;
          id_ready_.push_back(id);
        }
      }
      if (!rd.ok) {
        set_loop_error("negotiation: malformed announce from rank " + std::to_string(r));
        return false;
      }
    }
    for (size_t q = 0; q < table_.nready; q++) {  // (decided now: later ids of these names count anew)
      const int32_t id = idst_.empty() ? -1 : cache_lookup(table_.ready_q[q], std::hash<std::string>()(table_.ready_q[q]));
      if (id >= 0 && (size_t)id < idst_.size()) idst_[id].table = false;
    }
    Writer w;
    w.b.swap(*resp);  // (the previous response's buffer, reused)
    w.b.clear();
    w.put<uint8_t>(everyone_stops ? 1 : 0);
    const size_t count_at = w.b.size();
    w.put<uint32_t>(0);
    uint32_t n = table_.write_ready(w);
    for (uint32_t id : id_ready_) {  // after the table's: readiness order among themselves
      w.put<uint8_t>(kCachedOk);
      w.put<uint32_t>(id);
    }
    n += (uint32_t)id_ready_.size();
    id_ready_.clear();
    memcpy(&w.b[count_at], &n, sizeof n);
    resp->swap(w.b);
    return true;
  }

  // ---- response cache (rank-0 side and the shared bookkeeping) ----------------------------
  // An allreduce decided OK is cached on every rank under an id: the position of its first OK
  // decision in the response stream, which every rank reads in the same order (execute()), so the
  // ids agree without being sent. A later request with that name, dtype and shape is announced
  // by id; when every rank announced an id by id, rank 0 answers "cached OK" without the table:
  // the checks ConstructResponseMessage makes (coordinator.cc:90-186) passed for exactly these
  // parameters. Any full record of the name (changed shape, an unusable pointer, a rank with the
  // cache off) sends the round's ids of that name through the table, which then checks and
  // words every failure as before. A failure drops the name from the cache on every rank.
  int32_t cache_lookup(const std::string& name, uint64_t h) {
    cache_look_.h = h;
    cache_look_.s.assign(name);
    auto it = cache_ids_.find(cache_look_);
    return it == cache_ids_.end() ? -1 : (int32_t)it->second;
  }
  int32_t cached_id(const Req& r) {
    if (r.type != TIPS_REQ_ALLREDUCE || !r.bad.empty() || cache_ids_.empty()) return -1;
    const int32_t id = cache_lookup(r.name, r.name_hash);
    if (id < 0) return -1;
    const CacheEntry& e = cache_[(size_t)id];
    return e.dtype == r.dtype && e.shape == r.shape ? id : -1;
  }
  Announce expand(uint32_t id) {
    const CacheEntry& e = cache_[id];
    Announce a;
    a.type = TIPS_REQ_ALLREDUCE;
    a.dtype = e.dtype;
    a.count = e.count;
    a.shape = e.shape;
    a.name = e.name;
    return a;
  }
  // (rank 0) this round's announces of id go to the table from now on, the ones counted so far too
  void to_table(int32_t id) {
    if ((size_t)id >= idst_.size()) idst_.resize(cache_.size());
    IdState& st = idst_[(size_t)id];
    if (st.table) return;
    st.table = true;
    for (int q = 0; q < 64 && st.mask; q++)
      if (st.mask & (1ull << q)) {
        st.mask &= ~(1ull << q);
        table_.announce(q, expand((uint32_t)id));
      }
    st.n = 0;
  }
  // (every rank, execute(), in response order) an OK allreduce joins the cache or refreshes its
  // parameters; a failure leaves it
  void cache_note(const Decision& d, const Req* r) {
    if (d.name.compare(0, 6, "~sync.") == 0) return;  // (routed calls: a name per call)
    const int32_t id = cache_lookup(d.name, std::hash<std::string>()(d.name));
    if (!d.ok || !r || r->type != TIPS_REQ_ALLREDUCE) {
      if (id >= 0) {
        cache_[(size_t)id].live = false;
        cache_ids_.erase(cache_look_);
      }
      return;
    }
    if (id >= 0) {
      CacheEntry& e = cache_[(size_t)id];
      e.dtype = r->dtype;
      e.count = r->count;
      e.shape = r->shape;
      return;
    }
    if (cache_.size() >= kCacheCap) return;  // (full: later names travel in full, on every rank alike)
    cache_ids_.emplace(NameKey{std::hash<std::string>()(d.name), d.name}, (uint32_t)cache_.size());
    cache_.push_back(CacheEntry{d.name, r->dtype, r->count, r->shape, true});
  }

  // PerformCollectiveOp for one cycle's ready list, in rank 0's order. Readiness
  // batching: a run of consecutive ready requests of one dtype, each under the fusion
  // threshold and together within it, is reduced as ONE fused allreduce (pack, one
  // bucket exchange, unpack; fusion.cc) instead of one exchange per tensor. Every rank
  // received the same list, so every rank forms the same batches.
  void execute(const std::vector<Decision>& ds, size_t n) {  // ds[0, n): this cycle's decisions
    std::vector<std::shared_ptr<Req>> reqs(n);
    std::vector<NameMap::node_type> gone;  // (freed after the lock: enqueueing threads wait on it)
    gone.reserve(n);
    {
      std::lock_guard<AdaptiveMutex> l(m_);
      for (size_t i = 0; i < n; i++) {
        look_.h = std::hash<std::string>()(ds[i].name);
        look_.s.assign(ds[i].name);  // (a kept key: no allocation per lookup)
        auto it = by_name_.find(look_);
        if (it == by_name_.end()) continue;  // (cannot happen: every rank announced it)
        reqs[i] = it->second;
        gone.push_back(by_name_.extract(it));
        if (dry_) {
          std::string sz;
          for (size_t k = 0; k < ds[i].sizes.size(); k++) sz += (k ? "," : " sizes=") + std::to_string(ds[i].sizes[k]);
          log_.push_back(ds[i].name + (ds[i].ok ? " OK" + sz : " ERR " + ds[i].err));
        }
      }
    }
    gone.clear();
    for (size_t i = 0; i < n; i++) cache_note(ds[i], reqs[i].get());  // (every rank, this order)
    std::vector<int> state(n, 0), code(n, TIPS_ERR_MISMATCH);
    std::vector<std::string> msg(n);
    for (size_t i = 0; i < n; i++) {
      state[i] = ds[i].ok ? (dry_ ? 3 : 2) : -1;
      msg[i] = ds[i].err;
    }
    auto failed = [&](size_t k, int rc) {
      state[k] = -1;
      code[k] = rc;
      msg[k] = last_error();
    };
    if (!dry_) {
      State& st = S();
      const bool fuse = env_i64("TIPS_NEGOTIATED_FUSION", 1) != 0;
      const int64_t threshold = fusion_threshold_bytes();
      for (size_t i = 0; i < n;) {
        if (!reqs[i] || state[i] != 2) {
          i++;
          continue;
        }
        {  // (the request itself is kept; debug_state formats the line only when asked)
          std::lock_guard<std::mutex> l(phase_mu_);
          executed_++;
          exec_i_ = i;
          exec_n_ = n;
          exec_req_ = reqs[i];
        }
        if (reqs[i]->body) {  // a routed synchronous collective: its own call, here, in rank 0's order
          const int rc = reqs[i]->body();
          if (rc != 0) failed(i, rc);
          else state[i] = 3;
          i++;
          continue;
        }
        const int dtype = reqs[i]->dtype;
        if (reqs[i]->type == TIPS_REQ_ALLREDUCE && reqs[i]->host && fuse) {
          // a run of host allreduces of one dtype: one fused host call (page-locked pieces, H2D ->
          // allreduce -> D2H pipelined, unpacked into each output), not one staged call per tensor
          size_t j = i;
          while (j < n && reqs[j] && state[j] == 2 && !reqs[j]->body && reqs[j]->type == TIPS_REQ_ALLREDUCE &&
                 reqs[j]->host && reqs[j]->dtype == dtype)
            j++;
          if (j - i >= 2) {
            std::vector<BatchItem> items;
            for (size_t k = i; k < j; k++) items.push_back(BatchItem{reqs[k]->in, reqs[k]->out, reqs[k]->count});
            int rc;
            {
              std::lock_guard<std::mutex> lk(st.mu);
              rc = set_device(st);
              if (rc == 0) rc = fused_allreduce_host(st, items.data(), (int)items.size(), dtype, nullptr);
            }
            for (size_t k = i; k < j; k++) {
              if (rc != 0) failed(k, rc);
              else state[k] = 3;
            }
            i = j;
            continue;
          }
        }
        if (reqs[i]->type != TIPS_REQ_ALLREDUCE || reqs[i]->host) {  // broadcast / allgather / host: one at a time
          const int rc = run_other(*reqs[i], ds[i].sizes);
          if (rc != 0) failed(i, rc);
          else if (reqs[i]->host) state[i] = 3;  // finished: the host call returned with out written
          i++;
          continue;
        }
        std::lock_guard<std::mutex> lk(st.mu);
        const int rc0 = set_device(st);
        const int64_t es = tips::dtype_size(dtype);
        size_t j = i;
        int64_t bytes = 0;
        while (fuse && j < n && reqs[j] && state[j] == 2 && !reqs[j]->body && reqs[j]->type == TIPS_REQ_ALLREDUCE &&
               !reqs[j]->host && reqs[j]->dtype == dtype && reqs[j]->count * es < threshold &&
               round_up(bytes, kAlignBytes) + reqs[j]->count * es <= threshold) {
          bytes = round_up(bytes, kAlignBytes) + reqs[j]->count * es;
          j++;
        }
        int rc = rc0;
        if (j - i >= 2) {
          if (rc == 0) rc = run_batch(st, reqs, i, j);
        } else {
          j = i + 1;
          auto& r = reqs[i];
          if (rc == 0) rc = allreduce_device(st, r->in, r->out, r->count, r->dtype, r->stream);
          if (rc == 0) rc = take_event(*r);
          if (rc == 0 && hipEventRecord(r->ev, r->stream) != hipSuccess) rc = fail(TIPS_ERR_HIP, "hipEventRecord failed");
        }
        if (rc != 0)
          for (size_t k = i; k < j; k++) failed(k, rc);
        i = j;
      }
    }
    std::lock_guard<AdaptiveMutex> l(m_);
    for (size_t i = 0; i < n; i++)
      if (reqs[i]) {
        reqs[i]->state = state[i];
        reqs[i]->code = code[i];
        reqs[i]->err = msg[i];
        if (reqs[i]->cb) queue_done(reqs[i]);
      }
    cv_.notify_all();
  }

  // A single device request's completion event, taken when it runs (a fused batch shares one
  // GroupEv, a host request finishes before it is reported): most requests never need one, and an
  // admission that took one touched the pool and the request for nothing.
  int take_event(Req& r) {
    {
      std::lock_guard<AdaptiveMutex> l(m_);
      if (!ev_pool_.empty()) {
        r.ev = ev_pool_.back();
        ev_pool_.pop_back();
        return 0;
      }
    }
    TRY(set_device(S()));
    HIP_TRY(hipEventCreateWithFlags(&r.ev, hipEventDisableTiming));
    return 0;
  }

  // PerformCollectiveOp's broadcast and allgather branches (coordinator.cc:275-336) for one
  // decided request, through the synchronous collectives (they take st.mu themselves). The
  // allgather's output is allocated only now, when rank 0 has sent every rank's first
  // dimension, as the reference's allocate_output; its first dimension goes to *out_rows.
  int run_other(Req& r, const std::vector<int64_t>& sizes) {
    if (r.type == TIPS_REQ_ALLREDUCE) {  // a host allreduce (device ones are fused above)
      TRY(tips_allreduce(r.in, r.out, r.count, r.dtype, TIPS_OP_SUM, r.stream));
    } else if (r.type == TIPS_REQ_BROADCAST) {
      TRY(tips_broadcast(r.in, r.out, r.count, r.dtype, r.root, r.stream));
    } else {
      const int64_t es = tips::dtype_size(r.dtype);
      int64_t row = 1, rows = 0;
      for (size_t d = 1; d < r.shape.size(); d++) row *= r.shape[d];
      std::vector<int64_t> counts;
      for (int64_t v : sizes) {
        counts.push_back(v * row);
        rows += v;
      }
      if ((int)counts.size() != S().size) return fail(TIPS_ERR_MISMATCH, "allgather %s: sizes of %zu ranks", r.name.c_str(), counts.size());
      const int64_t bytes = rows * row * es;
      std::string why;
      if (bytes > 0) {
        if (!r.alloc) why = "no output allocator";
        else if (!(r.out = r.alloc(r.actx, bytes))) why = "the output allocator returned NULL for " + std::to_string(bytes) + " B";
      }
      // every rank learns whether every rank has its output before any transfer: a rank that
      // failed alone would otherwise leave the others waiting in the gather (one small exchange)
      const int64_t mine = why.empty() ? 1 : 0;
      std::vector<int64_t> all((size_t)S().size, 1);
      TRY(tips_allgather_i64(&mine, 1, all.data()));
      if (!why.empty()) return fail(TIPS_ERR_HIP, "allgather %s: %s", r.name.c_str(), why.c_str());
      for (int q = 0; q < S().size; q++)
        if (!all[q]) return fail(TIPS_ERR_HIP, "allgather %s: rank %d could not allocate its output", r.name.c_str(), q);
      if (r.out_rows) *r.out_rows = rows;
      TRY(tips_allgatherv(r.in, r.count, r.out, counts.data(), r.dtype, r.stream));
    }
    if (!r.host) {
      TRY(take_event(r));
      HIP_TRY(hipEventRecord(r.ev, r.stream));
    }
    return 0;
  }

  // reqs[i, j): one fused allreduce on their stream (or, if they came on several, on a
  // negotiation stream joined with each of them both ways); one shared completion event.
  int run_batch(State& st, std::vector<std::shared_ptr<Req>>& reqs, size_t i, size_t j) {
    std::vector<hipStream_t> streams;
    for (size_t k = i; k < j; k++)
      if (std::find(streams.begin(), streams.end(), reqs[k]->stream) == streams.end()) streams.push_back(reqs[k]->stream);
    hipStream_t s = streams[0];
    if (streams.size() > 1) {
      if (!neg_stream_) HIP_TRY(hipStreamCreateWithFlags(&neg_stream_, hipStreamNonBlocking));
      s = neg_stream_;
      TRY(join_ev_.ensure(streams.size()));
      for (size_t k = 0; k < streams.size(); k++) TRY(join(s, streams[k], join_ev_.ev[k]));
    }
    std::vector<BatchItem> items;
    items.reserve(j - i);
    for (size_t k = i; k < j; k++) items.push_back(BatchItem{reqs[k]->in, reqs[k]->out, reqs[k]->count});
    TRY(fused_allreduce(st, items.data(), (int)items.size(), reqs[i]->dtype, s));
    auto g = std::make_shared<GroupEv>();
    HIP_TRY(hipEventCreateWithFlags(&g->ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(g->ev, s));
    if (streams.size() > 1)
      for (hipStream_t u : streams) HIP_TRY(hipStreamWaitEvent(u, g->ev, 0));  // results in stream order for each owner
    for (size_t k = i; k < j; k++) reqs[k]->gev = g;
    return 0;
  }

  void set_loop_error(const std::string& e) {
    std::lock_guard<AdaptiveMutex> l(m_);
    if (loop_err_.empty()) loop_err_ = e;
  }

  int rank_ = 0, size_ = 1, timeout_ms_ = 600000;
  bool dry_ = false;
  int lfd_ = -1, up_ = -1;
  std::vector<int> peers_;
  Table table_;
  std::thread thread_;
  AdaptiveMutex m_;
  std::condition_variable_any cv_;
  bool running_ = false, want_stop_ = false;
  std::atomic<bool> accepting_{false};  // running_, readable without m_ (the lock-free enqueue's check)
  // Single enqueues (TF-style executor threads, many at once) are pushed onto this lock-free stack
  // and admitted to the tables by whoever next holds m_ (drain_locked): the negotiation thread
  // before each announce, poll / wait / on_done before a lookup. An enqueue then touches one
  // contended cache line (this head) instead of two locks and a reference count (round 5: 4
  // threads enqueueing 214 requests took 250 us against 180 us from one thread; the C entry
  // points' own lock and count went too, cached()).
  struct Pending {
    Prepared p;
    Pending* next = nullptr;
  };
  static constexpr int kShards = 8;
  struct alignas(64) Shard {
    std::atomic<Pending*> head{nullptr};
  };
  Shard shards_[kShards];
  bool any_pending() {
    for (Shard& sh : shards_)
      if (sh.head.load(std::memory_order_seq_cst)) return true;
    return false;
  }
  std::atomic<bool> idle_{false};  // the background thread waits for a cycle's first request
  bool lockfree_ = true;           // (set in start(), before any enqueue)
  std::atomic<bool> waiter_started_{false};
  std::deque<std::shared_ptr<Req>> fresh_;
  // (m_) The names the last two cycles announced (routed ~sync requests aside) and how many of them
  // fresh_ holds: a training step enqueues the same gradients every step, and once all of them are
  // in the linger need not wait out its quiet time (loop()).
  // (sorted name hashes, made by the enqueuing threads: admit() compares integers, and a collision
  // only ends a linger early or late, never changes what runs)
  std::vector<uint64_t> expect_;
  bool adm_prof_ = false;     // (TIPS_NEG_TRACE) drain_locked's phases, per cycle in the trace
  int64_t adm_ns_[5] = {};
  size_t expect_hits_ = 0;
  std::atomic<int64_t> last_arrival_ns_{0};  // (steady clock) the latest enqueue: the linger's clock
  NameMap by_name_;
  NameKey look_{0, std::string()};  // (m_) execute()'s lookup key
  // the response cache (the negotiation thread's own: no lock)
  static constexpr uint8_t kCachedOk = 2;  // a response entry: a cached name decided OK (then its id)
  static constexpr size_t kCacheCap = 1 << 16;
  struct CacheEntry {
    std::string name;
    int dtype;
    int64_t count;
    std::vector<int64_t> shape;
    bool live;
  };
  struct IdState {  // (rank 0) this round's announces of a cached name
    uint64_t mask = 0;   // the ranks that announced it by id
    int n = 0;
    bool table = false;  // a full record came: the rest of the round goes through the table
  };
  std::vector<CacheEntry> cache_;
  std::unordered_map<NameKey, uint32_t, NameKeyHash> cache_ids_;
  NameKey cache_look_{0, std::string()};
  std::vector<IdState> idst_;
  std::vector<uint32_t> id_ready_;
  std::atomic<int64_t> cached_decisions_{0};
  int64_t decide_ns_ = 0;  // (rank 0, the trace) the last cycle's decide()
  HandleMap by_handle_;
  std::vector<std::string> log_;
  std::vector<hipEvent_t> ev_pool_;
  std::string loop_err_;
  hipStream_t neg_stream_ = nullptr;  // fused batches whose requests came on several streams
  std::thread waiter_;                // completion callbacks (started by the first tips_on_done)
  int start_cpu_ = -1;                // the CPU of the thread that started the negotiation (TIPS_NEG_BIND)
  std::deque<std::shared_ptr<Req>> done_q_;
  std::condition_variable_any done_cv_;
  bool waiter_stop_ = false;
  int64_t cb_called_ = 0;

  EventPool join_ev_;

  // what the two threads are doing now (tips_debug_state): guarded by phase_mu_, never held across
  // a blocking call, so a dump from a watchdog always gets through
  std::mutex phase_mu_;
  std::string phase_ = "start";
  std::shared_ptr<Req> waiter_req_;  // the request the completion thread is at (null: idle)
  bool waiter_syncing_ = false;      // ... waiting for its device work (else: in its callback)
  int64_t cycles_ = 0, executed_ = 0;
  size_t exec_i_ = 0, exec_n_ = 0;
  std::shared_ptr<Req> exec_req_;  // the request execute() is on (phase_ "execute")
  void set_phase(std::string p) {
    std::lock_guard<std::mutex> l(phase_mu_);
    phase_ = std::move(p);
    exec_req_.reset();
  }
  void set_waiter_req(const std::shared_ptr<Req>& r, bool syncing) {
    std::lock_guard<std::mutex> l(phase_mu_);
    waiter_req_ = r;
    waiter_syncing_ = syncing;
  }

 public:
  std::atomic<int64_t> sync_seq{0};  // routed synchronous collectives so far: their names

  // one line of state for a hang report: the threads' phases, the cycle count and the request
  // queues (try_lock on the request lock: a dump never waits for a thread that might be stuck)
  std::string debug_state() {
    std::string out;
    {
      std::lock_guard<std::mutex> l(phase_mu_);
      std::string ph = phase_;
      if (exec_req_) {
        const Req& r = *exec_req_;
        ph = "execute " + std::to_string(exec_i_) + "/" + std::to_string(exec_n_) + ": " + r.name +
             (r.body ? " (routed call)" : r.host ? " (host)" : r.type != TIPS_REQ_ALLREDUCE ? " (other)" : "");
      }
      out = "rank " + std::to_string(rank_) + " cycles " + std::to_string((long long)cycles_) + " executed " +
            std::to_string((long long)executed_) + " | negotiation: " + ph + " | completion: " +
            (!waiter_req_ ? std::string("idle")
                          : waiter_syncing_ ? "hipEventSynchronize of " + waiter_req_->name + (waiter_req_->gev ? " (fused batch)" : "")
                                            : "callback of " + waiter_req_->name);
    }
    std::unique_lock<AdaptiveMutex> l(m_, std::try_to_lock);
    if (!l.owns_lock()) return out + " | (request lock held)";
    out += " | fresh " + std::to_string(fresh_.size()) + " pending " + std::to_string(by_name_.size()) + " handles " +
           std::to_string(by_handle_.size()) + " done_q " + std::to_string(done_q_.size()) + " callbacks " +
           std::to_string((long long)cb_called_);
    int k = 0;
    for (auto& kv : by_name_) {
      if (k++ == 8) break;
      out += (k == 1 ? " | waiting for other ranks: " : ", ") + kv.first.s + "(state " + std::to_string(kv.second->state) + ")";
    }
    if (!done_q_.empty()) out += " | next callback: " + done_q_.front()->name + "(state " + std::to_string(done_q_.front()->state) + ")";
    return out;
  }
};

AdaptiveMutex g_neg_mu;
std::shared_ptr<Negotiator> g_neg;  // (shared: a caller waiting on a request keeps it alive through a shutdown)
std::atomic<uint64_t> g_neg_gen{0};  // bumped whenever g_neg changes (cached(): per-thread copies)
std::string g_neg_failed;           // a failed start's verdict: later named requests fail with it at once
Negotiator* g_selftest_neg = nullptr;  // a running tips_negotiation_selftest's own (tips_debug_state)

int negotiation_port() {
  return (int)env_i64("TIPS_NEGOTIATION_PORT", env_i64("MASTER_PORT", 29500) + 19);
}

const char* master_addr() {
  const char* h = getenv("MASTER_ADDR");
  return (h && *h) ? h : "127.0.0.1";
}

}  // namespace

bool on_negotiation_thread() { return tl_negotiation_thread; }

int negotiation_stop() {
  std::shared_ptr<Negotiator> n;
  {
    std::lock_guard<AdaptiveMutex> l(g_neg_mu);
    n.swap(g_neg);
    g_neg_gen.fetch_add(1, std::memory_order_release);
    g_neg_failed.clear();
  }
  g_sync_direct = 0;
  return n ? n->stop() : 0;
}

// A synchronous collective entry point (tips_allreduce, tips_broadcast, tips_allgatherv, the fused
// calls, ...) while this rank's negotiation runs - named requests may be in flight, and TF-like
// callers issue them from other threads - is routed through it: it becomes request "~sync.<k>" (k
// counts this rank's routed calls; announced with its type, dtype and shape, so rank 0 checks it
// like any request), and its body runs on the negotiation thread when rank 0's order reaches it.
// So every RCCL call of a rank is issued from one thread in one order, the same on every rank, as
// the reference's coordinator issues every collective (coordinator.cc:355-513). Returns false when
// the call is to run directly (no negotiation, one rank, or already on the negotiation thread);
// else true, with *rc = the body's status (its error message in tips_last_error). A device call
// returns once its work is queued on the caller's stream, a host call once it is done.
bool route_collective(int type, int dtype, const int64_t* shape, int ndim, int root, const std::function<int()>& body,
                      int* rc) {
  if (tl_negotiation_thread) return false;
  std::shared_ptr<Negotiator> n;
  {
    std::lock_guard<AdaptiveMutex> l(g_neg_mu);
    n = g_neg;
  }
  if (!n || !n->running()) {
    State& st = S();
    if (st.initialized && st.size > 1) g_sync_direct++;
    return false;
  }
  const std::string name = "~sync." + std::to_string((long long)n->sync_seq++);
  const int64_t h = n->enqueue(name, nullptr, nullptr, shape, ndim, dtype, nullptr, type, root, nullptr, nullptr,
                               nullptr, body);
  if (h < 0) {
    *rc = (int)h;
    return true;
  }
  const int w = n->poll(h, true, /*routed=*/true);
  *rc = w == 1 ? 0 : w;
  return true;
}

}  // namespace rt
}  // namespace tips

using namespace tips::rt;


namespace {

std::shared_ptr<Negotiator> negotiator(int* code) {  // started by the first named request (collective)
  std::lock_guard<AdaptiveMutex> l(g_neg_mu);
  if (!g_neg) {
    if (!g_neg_failed.empty()) {
      *code = fail(TIPS_ERR_MISMATCH, "%s", g_neg_failed.c_str());
      return nullptr;
    }
    State& st = S();
    int rank, size;
    uint64_t key;
    {
      std::lock_guard<std::mutex> lk(st.mu);
      if (!st.initialized) {
        *code = fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
        return nullptr;
      }
      rank = st.rank;
      size = st.size;
      key = st.peer_key;  // the job's unique-id hash: a hello from another job is refused
    }
    auto neg = std::make_shared<Negotiator>();
    const int rc = neg->start(rank, size, master_addr(), negotiation_port(), false,
                              (int)env_i64("TIPS_NEGOTIATION_TIMEOUT", 600), key, g_sync_direct.load());
    if (rc) {
      *code = rc;
      if (rc == TIPS_ERR_MISMATCH) g_neg_failed = last_error();
      return nullptr;
    }
    g_neg = std::move(neg);
    g_neg_gen.fetch_add(1, std::memory_order_release);
  }
  return g_neg;
}

std::shared_ptr<Negotiator> current() {
  std::lock_guard<AdaptiveMutex> l(g_neg_mu);
  return g_neg;
}

// The single-request entry points' view of g_neg: a per-thread copy, refreshed when g_neg_gen
// moves (a start or a stop). Executor threads enqueueing at once each took g_neg_mu and bumped the
// negotiator's shared count per request, two cache lines bounced between them on every enqueue.
// The thread's copy keeps the negotiator alive while the pointer is used; one that was stopped
// refuses (not accepting) until the thread's next call sees the new generation.
Negotiator* cached(bool create, int* code) {
  thread_local std::shared_ptr<Negotiator> tl;
  thread_local uint64_t tl_gen = ~0ull;
  const uint64_t g = g_neg_gen.load(std::memory_order_acquire);
  if (g == tl_gen && tl) return tl.get();
  tl = create ? negotiator(code) : current();
  tl_gen = g;  // (read before the lookup: a start or stop in between only makes the next call look again)
  return tl.get();
}

// The argument checks of a named request (before any negotiation state is touched)
int check_named(const char* name, const void* in, void* out, const int64_t* shape, int ndim, int dtype, int type,
                int root, tips_alloc_fn alloc) {
  TRY(check_dtype(dtype));
  if (!name || !*name || ndim < 0 || ndim > TIPS_MAX_DIMS || (ndim > 0 && !shape))
    return fail(TIPS_ERR_INVALID_ARG, "bad named request");
  int64_t count = 1;
  for (int d = 0; d < ndim; d++) count *= shape[d] < 0 ? 0 : shape[d];
  if (count > 0 && (!in || (type != TIPS_REQ_ALLGATHER && !out))) return fail(TIPS_ERR_INVALID_ARG, "bad named request");
  if (type == TIPS_REQ_ALLGATHER && !alloc) return fail(TIPS_ERR_INVALID_ARG, "named allgather needs an output allocator");
  if (type == TIPS_REQ_BROADCAST) {
    const int size = tips_size();
    if (root < 0 || (size > 0 && root >= size)) return fail(TIPS_ERR_INVALID_ARG, "root rank %d out of range", root);
  }
  return 0;
}

int64_t enqueue_named(const char* name, const void* in, void* out, const int64_t* shape, int ndim, int dtype,
                      void* stream, int type = TIPS_REQ_ALLREDUCE, int root = 0, tips_alloc_fn alloc = nullptr,
                      void* actx = nullptr, int64_t* out_rows = nullptr) {
  TRY(check_named(name, in, out, shape, ndim, dtype, type, root, alloc));
  int code = TIPS_ERR_NOT_INITIALIZED;
  Negotiator* n = cached(true, &code);
  if (!n) return code;
  return n->enqueue(name, in, out, shape, ndim, dtype, (hipStream_t)stream, type, root, alloc, actx, out_rows, nullptr);
}

// tips_enqueue_allreduce[_shaped]_n: request i has shape dims(i) = {pointer, ndim}. Every request is
// checked and prepared first, then all are committed at once (Negotiator::enqueue_list); handles[i]
// < 0 for a refused one, the first refusal returned.
template <class Dims>
int enqueue_named_list(const char* const* names, const void* const* ins, void* const* outs, int n, int dtype,
                       void* stream, int64_t* handles, Dims dims) {
  int rc = 0;
  std::string first_err;
  auto refused = [&](int i, int code) {
    handles[i] = code;
    if (rc == 0) {
      rc = code;
      first_err = last_error();
    }
  };
  int code = TIPS_ERR_NOT_INITIALIZED;
  std::shared_ptr<Negotiator> neg;
  std::vector<Negotiator::Prepared> ps((size_t)n);
  PtrRanges pr;  // (the list's device allocations, one HIP lookup per segment)
  for (int i = 0; i < n; i++) {
    const std::pair<const int64_t*, int> d = dims(i);
    // (ndim -1: a bad request; -2: one whose reason dims() has already set)
    int e = d.second == -2 ? (int)TIPS_ERR_INVALID_ARG
            : d.second < 0 ? fail(TIPS_ERR_INVALID_ARG, "bad named allreduce request")
                           : check_named(names[i], ins[i], outs[i], d.first, d.second, dtype, TIPS_REQ_ALLREDUCE, 0, nullptr);
    if (e == 0 && !neg && !(neg = negotiator(&code))) e = code;
    if (e == 0)
      e = neg->prepare(ps[(size_t)i], names[i], ins[i], outs[i], d.first, d.second, dtype, (hipStream_t)stream,
                       TIPS_REQ_ALLREDUCE, 0, nullptr, nullptr, nullptr, nullptr, &pr);
    if (e) refused(i, e);
  }
  if (neg && env_i64("TIPS_LIST_ONE_LOCK", 1) == 0) {  // (A/B: one commit per request, as round 3)
    std::vector<Negotiator::Prepared> one(1);
    for (int i = 0; i < n; i++) {
      if (!ps[(size_t)i].r) continue;
      one[0] = std::move(ps[(size_t)i]);
      std::string err;
      const int e = neg->enqueue_list(one, handles + i, &err);
      if (e && rc == 0) {
        rc = e;
        first_err = err;
      }
    }
  } else if (neg) {
    std::string err;
    const int e = neg->enqueue_list(ps, handles, &err);
    if (e && rc == 0) {
      rc = e;
      first_err = err;
    }
  }
  return rc ? fail(rc, "%s", first_err.c_str()) : 0;
}


}  // namespace

extern "C" {

int64_t tips_enqueue_allreduce(const char* name, const void* in, void* out, int64_t count, int dtype, void* stream) {
  if (count < 0) return fail(TIPS_ERR_INVALID_ARG, "bad named allreduce request");
  return enqueue_named(name, in, out, &count, 1, dtype, stream);  // shape [count]
}

int64_t tips_enqueue_allreduce_shaped(const char* name, const void* in, void* out, const int64_t* shape, int ndim,
                                      int dtype, void* stream) {
  return enqueue_named(name, in, out, shape, ndim, dtype, stream);
}

int64_t tips_enqueue_broadcast(const char* name, const void* in, void* out, const int64_t* shape, int ndim,
                               int dtype, int root, void* stream) {
  return enqueue_named(name, in, out, shape, ndim, dtype, stream, TIPS_REQ_BROADCAST, root);
}

int64_t tips_enqueue_allgather(const char* name, const void* in, const int64_t* shape, int ndim, int dtype,
                               void* stream, tips_alloc_fn alloc, void* ctx, int64_t* out_rows) {
  return enqueue_named(name, in, nullptr, shape, ndim, dtype, stream, TIPS_REQ_ALLGATHER, 0, alloc, ctx, out_rows);
}


int tips_poll(int64_t handle) {
  int code = 0;
  Negotiator* n = cached(false, &code);
  if (!n) return fail(TIPS_ERR_NOT_INITIALIZED, "no named request was ever enqueued");
  return n->poll(handle, false);
}

int tips_wait(int64_t handle) {
  int code = 0;
  Negotiator* n = cached(false, &code);
  if (!n) return fail(TIPS_ERR_NOT_INITIALIZED, "no named request was ever enqueued");
  const int rc = n->poll(handle, true);
  return rc == 1 ? 0 : rc;
}

int64_t tips_enqueue_allreduce_cb(const char* name, const void* in, void* out, const int64_t* shape, int ndim, int dtype,
                                  void* stream, tips_done_fn fn, void* ctx) {
  if (!fn) return fail(TIPS_ERR_INVALID_ARG, "null completion callback");
  TRY(check_named(name, in, out, shape, ndim, dtype, TIPS_REQ_ALLREDUCE, 0, nullptr));
  int code = TIPS_ERR_NOT_INITIALIZED;
  Negotiator* n = cached(true, &code);
  if (!n) return code;
  return n->enqueue(name, in, out, shape, ndim, dtype, (hipStream_t)stream, TIPS_REQ_ALLREDUCE, 0, nullptr, nullptr,
                    nullptr, nullptr, nullptr, fn, ctx);
}

int tips_on_done(int64_t handle, tips_done_fn fn, void* ctx) {
  if (!fn) return fail(TIPS_ERR_INVALID_ARG, "null completion callback");
  int code = 0;
  Negotiator* n = cached(false, &code);
  if (!n) return fail(TIPS_ERR_NOT_INITIALIZED, "no named request was ever enqueued");
  return n->on_done(handle, fn, ctx);
}

int tips_debug_state(char* out, int64_t cap) {
  if (!out || cap < 1) return fail(TIPS_ERR_INVALID_ARG, "tips_debug_state: no buffer");
  std::string st = "no negotiation";
  std::unique_lock<AdaptiveMutex> l(g_neg_mu, std::try_to_lock);
  if (!l.owns_lock()) st = "(negotiation being started or stopped)";
  else if (g_neg) st = g_neg->debug_state();
  else if (g_selftest_neg) st = g_selftest_neg->debug_state();
  snprintf(out, (size_t)cap, "%s", st.c_str());
  return 0;
}

int tips_net_stats(int64_t* self_connects_refused, int64_t* unconfirmed_joins_refused) {
  if (self_connects_refused) *self_connects_refused = tips::net::self_connects().load();
  if (unconfirmed_joins_refused) *unconfirmed_joins_refused = tips::net::unconfirmed_joins().load();
  return 0;
}

int tips_enqueue_allreduce_n(const char* const* names, const void* const* ins, void* const* outs, const int64_t* counts,
                             int n, int dtype, void* stream, int64_t* handles) {
  if (n < 0 || (n > 0 && (!names || !ins || !outs || !counts || !handles)))
    return fail(TIPS_ERR_INVALID_ARG, "bad named allreduce list");
  return enqueue_named_list(names, ins, outs, n, dtype, stream, handles, [&](int i) {
    return std::make_pair(&counts[i], counts[i] < 0 ? -1 : 1);  // shape [count]
  });
}

int tips_enqueue_allreduce_shaped_n(const char* const* names, const void* const* ins, void* const* outs,
                                    const int* ndims, const int64_t* dims, int n, int dtype, void* stream,
                                    int64_t* handles) {
  if (n < 0 || (n > 0 && (!names || !ins || !outs || !ndims || !handles)))
    return fail(TIPS_ERR_INVALID_ARG, "bad named allreduce list");
  std::vector<int64_t> offs((size_t)n + 1, 0);  // where request i's dims start (bad entries take none)
  for (int i = 0; i < n; i++) offs[(size_t)i + 1] = offs[(size_t)i] + (ndims[i] > 0 && ndims[i] <= TIPS_MAX_DIMS ? ndims[i] : 0);
  return enqueue_named_list(names, ins, outs, n, dtype, stream, handles, [&](int i) {
    const bool ok = ndims[i] >= 0 && ndims[i] <= TIPS_MAX_DIMS && (ndims[i] == 0 || dims);
    if (!ok) fail(TIPS_ERR_INVALID_ARG, "bad ndim %d for %s", ndims[i], names[i] ? names[i] : "?");
    return std::make_pair(dims ? dims + offs[(size_t)i] : (const int64_t*)nullptr, ok ? ndims[i] : -2);
  });
}

int tips_wait_n(const int64_t* handles, int n) {
  if (n < 0 || (n > 0 && !handles)) return fail(TIPS_ERR_INVALID_ARG, "bad handle list");
  int rc = 0;
  std::string first_err;
  for (int i = 0; i < n; i++) {
    if (handles[i] <= 0) continue;
    const int w = tips_wait(handles[i]);
    if (w < 0 && rc == 0) {
      rc = w;
      first_err = last_error();
    }
  }
  return rc ? fail(rc, "%s", first_err.c_str()) : 0;
}

#ifdef TIPS_DEV  // (development surface: libtips_hip_dev.so only, include/tips_hip_dev.h)
namespace {

struct SelftestCount {
  std::atomic<int64_t> done{0};
};

void selftest_done(void* ctx, int status, const char* message) {
  (void)status;
  (void)message;
  static_cast<SelftestCount*>(ctx)->done++;
}

}  // namespace

int tips_negotiation_selftest(int rank, int size, const char* host, int port, const char* requests, char* out,
                              int64_t cap) {
  if (size < 1 || rank < 0 || rank >= size || !requests || !out || cap < 1)
    return fail(TIPS_ERR_INVALID_ARG, "bad selftest args");
  // lines: "name dtype count [d0,d1,...|-] [ar|ag|bc:ROOT]" (shape: default [count]; request type:
  // default allreduce), "@batch" ... "@endbatch" (the requests between them committed as one list,
  // as tips_enqueue_allreduce_n does), "@sleep ms", "@wait" (all so far resolved), "@mark" (log "# mark us"),
  // "@synccount N" (this rank claims N synchronous collectives before the join). A line "tK: ..."
  // belongs to thread K: threads 1.. issue their lines concurrently with the main thread's (thread
  // 0), as a framework's executor threads issue ops, and every request then completes through a
  // tips_on_done callback (its "@wait" waits for its own callbacks); the log ends "callbacks N".
  std::vector<std::vector<std::string>> per(1);
  int64_t synccount = 0;
  for (const char* p = requests; *p;) {
    const char* e = strchr(p, '\n');
    std::string line(p, e ? (size_t)(e - p) : strlen(p));
    p = e ? e + 1 : p + line.size();
    if (line.empty()) continue;
    if (line.rfind("@synccount ", 0) == 0) {
      synccount = atoll(line.c_str() + 11);
      continue;
    }
    size_t k = 0;
    if (line[0] == 't' && line.find(':') != std::string::npos && isdigit((unsigned char)line[1])) {
      k = (size_t)atoi(line.c_str() + 1);
      line = line.substr(line.find(':') + 1);
      while (!line.empty() && line[0] == ' ') line.erase(0, 1);
      if (k > 64) return fail(TIPS_ERR_INVALID_ARG, "selftest: thread %zu", k);
    }
    if (per.size() <= k) per.resize(k + 1);
    per[k].push_back(line);
  }
  const bool cbs = per.size() > 1;
  Negotiator neg;
  TRY(neg.start(rank, size, (host && *host) ? host : "127.0.0.1", port, true, 120, 0, synccount));
  struct Registered {  // visible to tips_debug_state while it runs
    explicit Registered(Negotiator* n) {
      std::lock_guard<AdaptiveMutex> l(g_neg_mu);
      g_selftest_neg = n;
    }
    ~Registered() {
      std::lock_guard<AdaptiveMutex> l(g_neg_mu);
      g_selftest_neg = nullptr;
    }
  } registered(&neg);
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<SelftestCount> counts(per.size());
  std::vector<int> issued(per.size(), 0), rcs(per.size(), 0);
  auto run = [&](size_t k) {
    std::vector<int64_t> handles;
    bool batching = false;  // between "@batch" and "@endbatch": one list commit (Negotiator::enqueue_list)
    std::vector<Negotiator::Prepared> batch;
    auto issued_one = [&](int64_t h) -> bool {
      if (h < 0) {
        rcs[k] = (int)h;
        return false;
      }
      if (cbs) {
        issued[k]++;
        if (neg.on_done(h, selftest_done, &counts[k]) != 0) {
          rcs[k] = TIPS_ERR_INVALID_ARG;
          return false;
        }
      } else {
        handles.push_back(h);
      }
      return true;
    };
    for (const std::string& line : per[k]) {
      char nm[256], dims[256] = "", kind[64] = "ar";
      long long dt = 0, cnt = 0;
      if (line == "@batch") {
        batching = true;
        batch.clear();
      } else if (line == "@endbatch") {
        batching = false;
        std::vector<int64_t> hs(batch.size(), 0);
        std::string err;
        if (neg.enqueue_list(batch, hs.data(), &err) != 0) {
          rcs[k] = TIPS_ERR_INVALID_ARG;
          return;
        }
        for (int64_t h : hs)
          if (!issued_one(h)) return;
      } else if (line.rfind("@sleep ", 0) == 0) {
        std::this_thread::sleep_for(std::chrono::milliseconds(atoi(line.c_str() + 7)));
      } else if (line == "@wait") {
        if (cbs) {
          while (counts[k].done.load() < issued[k]) std::this_thread::sleep_for(std::chrono::milliseconds(1));
        } else {
          for (int64_t h : handles) (void)neg.poll(h, true);
          handles.clear();
        }
      } else if (line == "@mark") {
        const auto us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0);
        neg.note("# mark " + std::to_string((long long)us.count()));
      } else if (sscanf(line.c_str(), "%255s %lld %lld %255s %63s", nm, &dt, &cnt, dims, kind) >= 3) {
        std::vector<int64_t> shape;
        if (strcmp(dims, "-") == 0) dims[0] = 0;
        const int type = strncmp(kind, "ag", 2) == 0 ? TIPS_REQ_ALLGATHER : strncmp(kind, "bc", 2) == 0 ? TIPS_REQ_BROADCAST
                                                                                                    : TIPS_REQ_ALLREDUCE;
        const int root = (type == TIPS_REQ_BROADCAST && kind[2] == ':') ? atoi(kind + 3) : 0;
        for (const char* q = dims; *q;) {
          shape.push_back(strtoll(q, nullptr, 10));
          q = strchr(q, ',');
          q = q ? q + 1 : "";
        }
        if (shape.empty()) shape.push_back(cnt);
        if (batching) {
          batch.emplace_back();
          if (neg.prepare(batch.back(), nm, nullptr, nullptr, shape.data(), (int)shape.size(), (int)dt, nullptr, type,
                          root, nullptr, nullptr, nullptr, nullptr, nullptr) != 0) {
            rcs[k] = TIPS_ERR_INVALID_ARG;
            return;
          }
        } else if (!issued_one(neg.enqueue(nm, nullptr, nullptr, shape.data(), (int)shape.size(), (int)dt, nullptr,
                                           type, root))) {
          return;
        }
      }
    }
    if (!cbs)
      for (int64_t h : handles) (void)neg.poll(h, false);
  };
  std::vector<std::thread> threads;
  for (size_t k = 1; k < per.size(); k++) threads.emplace_back(run, k);
  run(0);
  for (auto& t : threads) t.join();
  const int rc = neg.stop();  // collective: requests every rank announced are decided before it returns;
                              // the completion thread has called every callback when it returns
  for (int r : rcs)
    if (r) return r;
  std::string log;
  for (auto& l : neg.log()) log += l + "\n";
  log += "# cached decisions " + std::to_string((long long)neg.cached_decisions()) + "\n";
  if (cbs) {  // (the last line)
    int64_t n = 0;
    for (auto& c : counts) n += c.done.load();
    log += "callbacks " + std::to_string((long long)n) + "\n";
  }
  snprintf(out, (size_t)cap, "%s", log.c_str());
  return rc;
}

// Enqueue-vs-stop race check, one rank, dry executor: `threads` threads enqueue
// callback requests (tips_enqueue_allreduce_cb's path) as fast as they can while the calling thread
// stops the negotiation after stop_after_us; `rounds` times. Every enqueue that returned a handle
// must see its callback exactly once (OK if it ran before the stop, an error after it), and a
// refused one never. result[0..3]: accepted, callbacks, requests whose callback count was not 1,
// refusals. TIPS_OK when result[2] == 0 in every round.
int tips_negotiation_stop_race_selftest(int threads, int per_thread, int stop_after_us, int rounds, int port,
                                        int64_t* result) {
  if (threads < 1 || per_thread < 1 || rounds < 1 || !result) return fail(TIPS_ERR_INVALID_ARG, "bad args");
  for (int k = 0; k < 4; k++) result[k] = 0;
  struct Slot {
    std::atomic<int> calls{0};
    bool accepted = false;
  };
  auto count_cb = [](void* ctx, int, const char*) { static_cast<Slot*>(ctx)->calls.fetch_add(1); };
  for (int round = 0; round < rounds; round++) {
    std::vector<Slot> slots((size_t)threads * per_thread);
    {
      Negotiator neg;
      TRY(neg.start(0, 1, "127.0.0.1", port, true, 30, 0, 0));
      std::atomic<bool> go{false};
      std::vector<std::thread> th;
      for (int t = 0; t < threads; t++)
        th.emplace_back([&, t] {
          while (!go.load()) std::this_thread::yield();
          const int64_t shape[1] = {4};
          for (int i = 0; i < per_thread; i++) {
            Slot& sl = slots[(size_t)t * per_thread + i];
            const std::string name = "r" + std::to_string(round) + "/t" + std::to_string(t) + "/" + std::to_string(i);
            const int64_t h = neg.enqueue(name, nullptr, nullptr, shape, 1, TIPS_FLOAT32, nullptr, TIPS_REQ_ALLREDUCE, 0,
                                          nullptr, nullptr, nullptr, nullptr, nullptr, count_cb, &sl);
            sl.accepted = h > 0;
          }
        });
      go.store(true);
      std::this_thread::sleep_for(std::chrono::microseconds(stop_after_us));
      (void)neg.stop();  // (its verdict is not the point: the callbacks are)
      for (auto& x : th) x.join();
      // counted before the destructor, which would fail and call back whatever is still stacked:
      // once stop() has returned and the enqueues have, every callback must have been called
      for (auto& sl : slots) {
        const int c = sl.calls.load();
        result[0] += sl.accepted;
        result[1] += c;
        result[2] += sl.accepted ? c != 1 : c != 0;
        result[3] += !sl.accepted;
      }
    }
  }
  return result[2] == 0 ? TIPS_OK : fail(TIPS_ERR_MISMATCH, "%lld requests saw a wrong number of callbacks", (long long)result[2]);
}
#endif  // TIPS_DEV

}  // extern "C"
