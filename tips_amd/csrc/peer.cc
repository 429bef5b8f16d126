// peer.cc — the xGMI peer schedule (TIPS_ALGO_PEER): the allreduce's transfers
// done by our own kernels through IPC-mapped peer memory, not by RCCL.
//
// Same arithmetic as the direct schedule (schedules.cc) and so the same bits:
// rank r owns chunk r and folds the p contributions to it in rank order with
// one multi_sum launch (the MPI_SUM of AllreduceCpu<T>, reference
// tips/core/collective/utils.h:60-65). What changes is the transport:
//   push    one xfer_kernel writes in[chunk d] straight into peer d's slot for
//           r, for all d at once (segments interleaved over the workgroups, so
//           all 7 xGMI links of an MI355X carry traffic together);
//   reduce  multi_sum over in[chunk r] and the p-1 local slots -> red;
//   pull    one xfer_kernel reads every peer's red (its reduced chunk) into out.
// TIPS_PEER_RS=pullfold (opt-in) replaces push + reduce with a local stage of the peers' chunks and
// one fold kernel per rank that reads its chunk's slices from every peer's workspace over xGMI
// (peer_piece_pullfold).
// Each rank's workspace {p-1 slots, red} is one uncached device allocation,
// exported once with hipIpcGetMemHandle and opened by every peer. Uncached
// memory keeps no line of it in any L2, so a peer's write is what the next
// kernel reads, without cache maintenance across GPUs.
//
// Phases are ordered by the host: a stream synchronize, then a barrier in a
// POSIX shared-memory block all ranks of the node map. No kernel ever waits on
// a flag written by another GPU, so no wave can spin forever. Barrier 0 of
// every call also checks that all ranks passed the same count and dtype
// before any remote write (a mismatch fails on every rank, with both values).
// Single node only (xGMI; the shared-memory block is node-local).
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <sched.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <vector>

#include "rt.h"

namespace tips {
namespace rt {

namespace {

constexpr int kPeerMaxRanks = tips::kMaxSrcs;
constexpr uint64_t kPeerMagic = 0x5449505350454552ull;  // "TIPSPEER"
constexpr int64_t kPeerSlotPad = 4096;  // slots not at power-of-two strides (as plan.cc kSlotPad)
constexpr int64_t kWsHeader = 4096;     // each workspace starts with its WsHeader; slots follow

enum Phase : int32_t {
  kCall = 1, kPushed = 2, kReduced = 3, kPublish = 4, kShutdown = 5, kGathered = 6, kUnpacked = 7,
  kBcastCall = 8, kGatherCall = 9, kStaged = 10, kPulled = 11, kVerified = 12
};

struct Post {
  int64_t count;
  int32_t dtype;
  int32_t phase;
  int64_t aux;  // broadcast: the root rank; kVerified: -1 if every header checked out, else the failing owner
  int64_t ws_bytes;
  uint64_t nonce;  // kPublish: the nonce the owner wrote at its workspace head
  hipIpcMemHandle_t handle;
};

// Written by the owner at the head of its workspace before it publishes the IPC handle, and read
// back by every peer THROUGH its mapping: a mapping that shows another buffer (a stale import
// was once seen on this ROCm's dmabuf IPC) fails the job instead of summing
// wrong data.
struct WsHeader {
  uint64_t magic;
  uint64_t key;    // the job's unique-id hash
  int64_t rank;    // owner
  int64_t bytes;   // workspace size
  uint64_t nonce;  // per allocation
  uint64_t pad[3];
};

struct alignas(64) PeerRank {
  std::atomic<uint64_t> epoch;
  Post post[2];  // by epoch parity: a rank overwrites parity e only at e + 2, after everyone posted e + 1
};

struct PeerCtl {
  std::atomic<uint64_t> magic;
  std::atomic<int32_t> attached;
  int32_t size;
  uint64_t key;
  PeerRank rk[kPeerMaxRanks];
};

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void backoff(int64_t it) {
  if (it < 4096) {
    __builtin_ia32_pause();
  } else if (it < 65536) {
    sched_yield();
  } else {
    struct timespec ts = {0, 50 * 1000};
    nanosleep(&ts, nullptr);
  }
}

}  // namespace

struct PeerState {
  PeerCtl* ctl = nullptr;
  uint64_t epoch = 0;
  void* ws = nullptr;        // this rank's workspace (uncached device memory, IPC-exported)
  int64_t ws_bytes = 0;      // data bytes after the header
  void* remote[kPeerMaxRanks] = {};  // peers' workspaces as IPC-opened (remote[rank] = ws)
  char* rdata[kPeerMaxRanks] = {};   // their data regions (after the WsHeader): what the schedule uses
  void* hdr_dev = nullptr;           // p headers read back through the mappings
  hipEvent_t pulled = nullptr;        // after the last call's pull (which reads the peers' red)
  bool pull_pending = false;
  bool broken = false;  // a failure past barrier 0 leaves the ranks out of step: refuse further calls
};

namespace {

double peer_timeout() { return (double)env_i64("TIPS_PEER_TIMEOUT_S", 120); }

// All ranks post `mine` and wait for each other; `all[j]` = rank j's post.
int barrier(State& st, PeerState& ps, const Post& mine, Post* all, double timeout_s) {
  const uint64_t e = ++ps.epoch;
  PeerRank& me = ps.ctl->rk[st.rank];
  me.post[e & 1] = mine;
  me.epoch.store(e, std::memory_order_release);
  const double deadline = now_s() + timeout_s;
  for (int j = 0; j < st.size; j++) {
    int64_t it = 0;
    while (ps.ctl->rk[j].epoch.load(std::memory_order_acquire) < e) {
      backoff(it++);
      if ((it & 1023) == 0 && now_s() > deadline)
        return fail(TIPS_ERR_HIP, "peer schedule: rank %d did not reach barrier %llu (phase %d) within %.0f s", j,
                    (unsigned long long)e, mine.phase, timeout_s);
    }
    const Post& pj = ps.ctl->rk[j].post[e & 1];
    if (pj.phase != mine.phase)
      return fail(TIPS_ERR_MISMATCH, "peer schedule out of step: at barrier %llu rank %d is in phase %d, rank %d in phase %d",
                  (unsigned long long)e, j, pj.phase, st.rank, mine.phase);
    if (all) all[j] = pj;
  }
  return 0;
}

int attach(State& st, PeerState& ps) {
  if (ps.ctl) return 0;
  if (!st.peer_key) return fail(TIPS_ERR_NOT_INITIALIZED, "peer schedule needs the bootstrap unique id (tips_init_rank)");
  if (st.size > kPeerMaxRanks) return fail(TIPS_ERR_UNSUPPORTED, "peer schedule supports at most %d ranks", kPeerMaxRanks);
  char name[64];
  snprintf(name, sizeof name, "/tips_peer_%016llx", (unsigned long long)st.peer_key);
  const size_t bytes = sizeof(PeerCtl);
  const double deadline = now_s() + peer_timeout();
  PeerCtl* ctl = nullptr;
  if (st.rank == 0) {
    shm_unlink(name);  // a stale block of the same key cannot be ours
    int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) return fail(TIPS_ERR_HIP, "peer schedule: shm_open(%s) failed: %s", name, strerror(errno));
    if (ftruncate(fd, (off_t)bytes) != 0) {
      close(fd);
      shm_unlink(name);
      return fail(TIPS_ERR_HIP, "peer schedule: ftruncate failed: %s", strerror(errno));
    }
    void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) {
      shm_unlink(name);
      return fail(TIPS_ERR_HIP, "peer schedule: mmap failed: %s", strerror(errno));
    }
    ctl = (PeerCtl*)m;  // zero-filled by ftruncate
    ctl->size = st.size;
    ctl->key = st.peer_key;
    ctl->magic.store(kPeerMagic, std::memory_order_release);
  } else {
    for (;;) {
      int fd = shm_open(name, O_RDWR, 0600);
      struct stat sb;
      if (fd >= 0 && fstat(fd, &sb) == 0 && (size_t)sb.st_size >= bytes) {
        void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (m != MAP_FAILED) {
          PeerCtl* c = (PeerCtl*)m;
          if (c->magic.load(std::memory_order_acquire) == kPeerMagic && c->key == st.peer_key) {
            ctl = c;
            break;
          }
          munmap(m, bytes);
        }
      } else if (fd >= 0) {
        close(fd);
      }
      if (now_s() > deadline) return fail(TIPS_ERR_HIP, "peer schedule: rank 0's control block %s did not appear", name);
      struct timespec ts = {0, 1000 * 1000};
      nanosleep(&ts, nullptr);
    }
  }
  if (ctl->size != st.size) {
    munmap(ctl, bytes);
    return fail(TIPS_ERR_MISMATCH, "peer schedule: control block is for %d ranks, this job has %d", ctl->size, st.size);
  }
  ctl->attached.fetch_add(1, std::memory_order_acq_rel);
  if (st.rank == 0) {  // everyone has it mapped: remove the name, so nothing is left in /dev/shm
    for (int64_t it = 0; ctl->attached.load(std::memory_order_acquire) < st.size; it++) {
      backoff(it);
      if ((it & 1023) == 0 && now_s() > deadline) {
        const int got = ctl->attached.load();
        shm_unlink(name);
        munmap(ctl, bytes);
        return fail(TIPS_ERR_HIP, "peer schedule: only %d of %d ranks attached", got, st.size);
      }
    }
    shm_unlink(name);
  }
  ps.ctl = ctl;
  ps.epoch = 0;
  return 0;
}

void close_remotes(State& st, PeerState& ps) {
  for (int j = 0; j < kPeerMaxRanks; j++) {
    if (ps.remote[j] && j != st.rank) (void)hipIpcCloseMemHandle(ps.remote[j]);
    ps.remote[j] = nullptr;
  }
}

int alloc_ws(void** p, int64_t bytes) {
  // TIPS_PEER_MEM: 0 uncached (default), 1 fine-grained, 2 coarse (plain hipMalloc; experiments only)
  const int64_t kind = env_i64("TIPS_PEER_MEM", 0);
  if (kind == 2) {
    HIP_TRY(hipMalloc(p, (size_t)bytes));
  } else {
    HIP_TRY(hipExtMallocWithFlags(p, (size_t)bytes, kind == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached));
  }
  return 0;
}

// The workspace is allocated, exported and opened once per job, at a fixed size
// (TIPS_PEER_WS_MIB); buckets larger than it go through in pieces. Growing it
// instead (free, re-export, re-open) was seen to go wrong on ROCm's dmabuf IPC
// with 4 processes: an export refused with "invalid argument", and, worse, an
// import that still showed a peer's previous buffer (wrong sums, no error).
int setup_ws(State& st, PeerState& ps) {
  if (ps.ws) return 0;
  const int64_t bytes = round_up(std::max<int64_t>(4, env_i64("TIPS_PEER_WS_MIB", 1088)) << 20, 2 << 20);
  Post mine{};
  mine.phase = kPublish;
  mine.ws_bytes = bytes;
  // an export that is refused is retried on a second allocation (at another address:
  // the refused buffers stay allocated until then)
  std::vector<void*> refused;
  int rc = 0;
  for (int attempt = 0;; attempt++) {
    rc = alloc_ws(&ps.ws, bytes + kWsHeader);
    if (rc) break;
    hipError_t he = hipIpcGetMemHandle(&mine.handle, ps.ws);
    if (he == hipSuccess) break;
    (void)hipGetLastError();
    refused.push_back(ps.ws);
    ps.ws = nullptr;
    if (attempt == 3) {
      rc = fail(TIPS_ERR_HIP, "hipIpcGetMemHandle (workspace of %lld B) failed %d times: %s", (long long)bytes,
                attempt + 1, hipGetErrorString(he));
      break;
    }
  }
  for (void* q : refused) (void)hipFree(q);
  if (rc) return rc;
  ps.ws_bytes = bytes;
  // the header: this job's key, the owner, the size and a nonce that no earlier buffer carried
  WsHeader h{};
  h.magic = kPeerMagic;
  h.key = st.peer_key;
  h.rank = st.rank;
  h.bytes = bytes;
  h.nonce = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() * 6364136223846793005ull ^
            (uint64_t)(uintptr_t)ps.ws ^ ((uint64_t)getpid() << 32) ^ (uint64_t)st.rank;
  mine.nonce = h.nonce;
  if (env_i64("TIPS_PEER_TEST_CORRUPT_RANK", -1) == st.rank) h.nonce ^= 1;  // test hook: a header peers must refuse
  HIP_TRY(hipMemcpy(ps.ws, &h, sizeof h, hipMemcpyHostToDevice));
  Post all[kPeerMaxRanks];
  TRY(barrier(st, ps, mine, all, peer_timeout()));
  for (int j = 0; j < st.size; j++) {
    if (j == st.rank) {
      ps.remote[j] = ps.ws;
    } else {
      if (all[j].ws_bytes != bytes)
        return fail(TIPS_ERR_MISMATCH, "peer schedule: rank %d workspace %lld B, rank %d %lld B (TIPS_PEER_WS_MIB must match)",
                    j, (long long)all[j].ws_bytes, st.rank, (long long)bytes);
      HIP_TRY(hipIpcOpenMemHandle(&ps.remote[j], all[j].handle, hipIpcMemLazyEnablePeerAccess));
    }
    ps.rdata[j] = (char*)ps.remote[j] + kWsHeader;
  }
  // every peer's header, read through the mapping by a kernel (uncached memory: what the owner
  // wrote, not a stale line), checked against what the owner published at the barrier
  const int p = st.size;
  if (!ps.hdr_dev) HIP_TRY(hipMalloc(&ps.hdr_dev, sizeof(WsHeader) * kPeerMaxRanks));
  tips::XferSeg segs[tips::kMaxXferSegs];
  for (int j = 0; j < p; j++) segs[j] = {(const char*)ps.remote[j], (char*)ps.hdr_dev + j * sizeof(WsHeader), (int64_t)sizeof(WsHeader)};
  HIP_TRY(tips::launch_xfer(segs, p, st.io_stream));
  WsHeader seen[kPeerMaxRanks];
  HIP_TRY(hipMemcpyAsync(seen, ps.hdr_dev, sizeof(WsHeader) * p, hipMemcpyDeviceToHost, st.io_stream));
  HIP_TRY(hipStreamSynchronize(st.io_stream));
  int bad = -1;
  for (int j = 0; j < p && bad < 0; j++)
    if (seen[j].magic != kPeerMagic || seen[j].key != st.peer_key || seen[j].rank != j || seen[j].bytes != bytes ||
        seen[j].nonce != all[j].nonce)
      bad = j;
  Post v{};
  v.phase = kVerified;
  v.aux = bad < 0 ? -1 : bad;
  TRY(barrier(st, ps, v, all, peer_timeout()));
  for (int j = 0; j < p; j++)
    if (all[j].aux >= 0)
      return fail(TIPS_ERR_HIP,
                  "peer schedule: rank %d's mapping of rank %lld's workspace does not show the header rank %lld wrote "
                  "(stale or foreign IPC mapping); refusing to reduce through it",
                  j, (long long)all[j].aux, (long long)all[j].aux);
  return 0;
}

}  // namespace

void peer_release(State& st) {
  PeerState* ps = st.peer;
  if (!ps) return;
  if (ps->ctl) {
    (void)hipDeviceSynchronize();
    Post q{};
    q.phase = kShutdown;
    (void)barrier(st, *ps, q, nullptr, 10.0);  // no rank frees its workspace while a peer still reads it
    close_remotes(st, *ps);
    munmap(ps->ctl, sizeof(PeerCtl));
  }
  if (ps->ws) (void)hipFree(ps->ws);
  if (ps->hdr_dev) (void)hipFree(ps->hdr_dev);
  if (ps->pulled) (void)hipEventDestroy(ps->pulled);
  delete ps;
  st.peer = nullptr;
}

namespace {

// One piece (<= the workspace): push, barrier, fold, barrier, pull; or, with the push
// allgather (TIPS_PEER_AG=push), push, barrier, fold, barrier, push, barrier, local copy.
int peer_piece(State& st, PeerState& ps, const char* in, char* out, int64_t n, int dtype, hipStream_t user,
               bool ag_push) {
  const int p = st.size, r = st.rank;
  const int64_t es = tips::dtype_size(dtype), align = kAlignBytes / es;
  const int64_t cap = round_up(chunk_of(n, p, align, 0).len() * es, kAlignBytes) + kPeerSlotPad;
  // workspace: slot s (s = j < owner ? j : j - 1) holds source j's slice of the owner's chunk; red after them
  auto slot_of = [&](int owner, int j) { return (int64_t)(j < owner ? j : j - 1) * cap; };
  const int64_t red_off = (int64_t)(p - 1) * cap;
  if (red_off + cap > ps.ws_bytes) return fail(TIPS_ERR_INVALID_ARG, "peer schedule: piece exceeds the workspace");

  // push: in[chunk d] -> peer d's slot for r, every peer in one launch. The peers' folds
  // of the previous piece / call read their slots before the last barrier.
  tips::XferSeg segs[tips::kMaxXferSegs];
  int m = 0;
  for (int d = 1; d < p; d++) {
    const int to = mod(r + d, p);
    const Range c = chunk_of(n, p, align, to);
    segs[m++] = {in + c.b * es, ps.rdata[to] + slot_of(to, r), c.len() * es};
  }
  HIP_TRY(tips::launch_xfer(segs, m, user));
  HIP_TRY(hipStreamSynchronize(user));  // also: our previous pull has read the peers' red
  Post q{};
  q.count = n;
  q.dtype = dtype;
  q.phase = kPushed;
  TRY(barrier(st, ps, q, nullptr, peer_timeout()));

  // fold: rank-order sum of chunk r (same bits as the direct schedule). With the push
  // allgather it lands in out directly (the pushes below read it from there).
  const Range mine = chunk_of(n, p, align, r);
  const void* srcs[tips::kMaxSrcs];
  for (int j = 0; j < p; j++) srcs[j] = (j == r) ? (const void*)(in + mine.b * es) : ps.rdata[r] + slot_of(r, j);
  char* red = ag_push ? out + mine.b * es : ps.rdata[r] + red_off;
  HIP_TRY(tips::launch_multi_sum(red, srcs, p, mine.len(), dtype, user));
  HIP_TRY(hipStreamSynchronize(user));
  q.phase = kReduced;
  TRY(barrier(st, ps, q, nullptr, peer_timeout()));

  if (!ag_push) {
    // pull: every rank's reduced chunk -> out, stream-ordered (the next push's sync and
    // barrier keep the peers from overwriting red before this has read it)
    m = 0;
    for (int d = 0; d < p; d++) {
      const int from = mod(r + d, p);
      const Range c = chunk_of(n, p, align, from);
      segs[m++] = {ps.rdata[from] + red_off, out + c.b * es, c.len() * es};
    }
    HIP_TRY(tips::launch_xfer(segs, m, user));
    return 0;
  }
  // push allgather: my reduced chunk -> every peer's slot for r (every fold has consumed
  // the slots: barrier above), then each rank copies its slots into out
  m = 0;
  for (int d = 1; d < p; d++) segs[m++] = {red, ps.rdata[mod(r + d, p)] + slot_of(mod(r + d, p), r), mine.len() * es};
  HIP_TRY(tips::launch_xfer(segs, m, user));
  HIP_TRY(hipStreamSynchronize(user));
  q.phase = kGathered;
  TRY(barrier(st, ps, q, nullptr, peer_timeout()));
  m = 0;
  for (int d = 1; d < p; d++) {
    const int from = mod(r + d, p);
    const Range c = chunk_of(n, p, align, from);
    segs[m++] = {ps.rdata[r] + slot_of(r, from), out + c.b * es, c.len() * es};
  }
  HIP_TRY(tips::launch_xfer(segs, m, user));
  return 0;
}

// One piece with the fused pull-fold reduce-scatter (TIPS_PEER_RS=pullfold, opt-in): every rank
// stages the chunks its peers own in its own workspace (a local copy), barrier; then rank r folds
// chunk r in ONE kernel that reads every peer's staged slice over its xGMI link plus its own input
// slice, in rank order (launch_multi_sum_remote: the same bits as the direct schedule), and writes
// red once; barrier; pull as above. The received slices are never written to this GPU's HBM and
// re-read by a separate fold: the reduction consumes them as they arrive, with every link busy.
// Workspace: chunk c of the staged piece at c x cap (cap = padded chunk), red after the p chunks.
int peer_piece_pullfold(State& st, PeerState& ps, const char* in, char* out, int64_t n, int dtype, hipStream_t user) {
  const int p = st.size, r = st.rank;
  const int64_t es = tips::dtype_size(dtype), align = kAlignBytes / es;
  const int64_t cap = round_up(chunk_of(n, p, align, 0).len() * es, kAlignBytes) + kPeerSlotPad;
  const int64_t red_off = (int64_t)p * cap;
  if (red_off + cap > ps.ws_bytes) return fail(TIPS_ERR_INVALID_ARG, "peer schedule: piece exceeds the workspace");
  // stage: in[chunk c] -> my workspace at c x cap for every c != r (peers read it after the barrier;
  // their reads of the previous piece ended before its kReduced barrier)
  for (int c = 0; c < p; c++) {
    if (c == r) continue;
    const Range rc = chunk_of(n, p, align, c);
    if (rc.len() > 0) HIP_TRY(tips::launch_copy_buf(ps.rdata[r] + (int64_t)c * cap, in + rc.b * es, rc.len() * es, user));
  }
  HIP_TRY(hipStreamSynchronize(user));  // also: our previous pull has read the peers' red
  Post q{};
  q.count = n;
  q.dtype = dtype;
  q.phase = kStaged;
  TRY(barrier(st, ps, q, nullptr, peer_timeout()));
  // pull-fold: chunk r from every rank, rank order, straight from the peers' workspaces
  const Range mine = chunk_of(n, p, align, r);
  const void* srcs[tips::kMaxSrcs];
  for (int j = 0; j < p; j++) srcs[j] = (j == r) ? (const void*)(in + mine.b * es) : ps.rdata[j] + (int64_t)r * cap;
  char* red = ps.rdata[r] + red_off;
  HIP_TRY(tips::launch_multi_sum_remote(red, srcs, p, mine.len(), dtype, user));
  HIP_TRY(hipStreamSynchronize(user));
  q.phase = kReduced;
  TRY(barrier(st, ps, q, nullptr, peer_timeout()));
  // pull: every rank's reduced chunk -> out (as peer_piece)
  tips::XferSeg segs[tips::kMaxXferSegs];
  int m = 0;
  for (int d = 0; d < p; d++) {
    const int from = mod(r + d, p);
    const Range c = chunk_of(n, p, align, from);
    segs[m++] = {ps.rdata[from] + red_off, out + c.b * es, c.len() * es};
  }
  HIP_TRY(tips::launch_xfer(segs, m, user));
  return 0;
}

int peer_allreduce_impl(State& st, PeerState& ps, const char* in, char* out, int64_t n, int dtype, hipStream_t user,
                        bool* clean) {
  TRY(attach(st, ps));
  const int p = st.size, r = st.rank;
  const int64_t es = tips::dtype_size(dtype);
  if (ps.pull_pending) {  // the last call's pull (or slot copy), on whatever stream it ran, is done
    HIP_TRY(hipEventSynchronize(ps.pulled));
    ps.pull_pending = false;
  }
  Post call{};
  call.count = n;
  call.dtype = dtype;
  call.phase = kCall;
  Post all[kPeerMaxRanks];
  TRY(barrier(st, ps, call, all, peer_timeout()));
  for (int j = 0; j < p; j++)
    if (all[j].count != n || all[j].dtype != dtype)
      return fail(TIPS_ERR_MISMATCH, "peer schedule: rank %d allreduces %lld elements of dtype %d, rank %d %lld of dtype %d",
                  j, (long long)all[j].count, all[j].dtype, r, (long long)n, dtype);  // every rank, same barrier
  *clean = false;  // from here on a failure leaves the ranks out of step
  TRY(setup_ws(st, ps));
  // TIPS_PEER_RS=pullfold: the fused pull-fold reduce-scatter (its pull allgather), else push + fold
  const char* rsv = getenv("TIPS_PEER_RS");
  const bool pullfold = rsv && !strcmp(rsv, "pullfold");
  // piece: the largest multiple of p 256-B-aligned chunks whose slots fit the workspace (p slots;
  // pull-fold: p staged chunks and red)
  const int64_t per_chunk = (ps.ws_bytes / (pullfold ? p + 1 : p) - kPeerSlotPad) / kAlignBytes * kAlignBytes;
  const int64_t piece = per_chunk / es * p;
  const char* agv = getenv("TIPS_PEER_AG");
  const bool ag_push = !pullfold && agv && !strcmp(agv, "push");
  for (int64_t b = 0; b < n; b += piece) {
    if (b > 0 && ag_push) {  // every rank's local copy out of its slots is done before new pushes land
      HIP_TRY(hipStreamSynchronize(user));
      Post u = call;
      u.phase = kUnpacked;
      TRY(barrier(st, ps, u, nullptr, peer_timeout()));
    }
    if (pullfold)
      TRY(peer_piece_pullfold(st, ps, in + b * es, out + b * es, std::min(piece, n - b), dtype, user));
    else
      TRY(peer_piece(st, ps, in + b * es, out + b * es, std::min(piece, n - b), dtype, user, ag_push));
  }
  if (!ps.pulled) HIP_TRY(hipEventCreateWithFlags(&ps.pulled, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(ps.pulled, user));
  ps.pull_pending = true;
  return 0;
}

// Entry of a broadcast / allgatherv call: the last call's pull is done, then the call barrier
// (every rank's post in all[]).
int peer_enter(State& st, PeerState& ps, const Post& call, Post* all) {
  TRY(attach(st, ps));
  if (ps.pull_pending) {
    HIP_TRY(hipEventSynchronize(ps.pulled));
    ps.pull_pending = false;
  }
  TRY(barrier(st, ps, call, all, peer_timeout()));
  return 0;
}

int peer_leave(PeerState& ps, hipStream_t user) {
  if (!ps.pulled) HIP_TRY(hipEventCreateWithFlags(&ps.pulled, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(ps.pulled, user));
  ps.pull_pending = true;
  return 0;
}

// Broadcast (MPI_Bcast of BroadcastCpu, reference tips/core/collective/utils.h:118-134): per
// piece of up to the workspace, the root stages its bytes in its own workspace, barrier, every
// other rank reads them from there into out in one xfer launch (all its peers' links idle but
// the root's: a broadcast is bounded by the root's outgoing links, which the p-1 readers share).
int peer_broadcast_impl(State& st, PeerState& ps, const char* in, char* out, int64_t bytes, int root, hipStream_t user,
                        bool* clean) {
  const int p = st.size, r = st.rank;
  Post call{};
  call.count = bytes;
  call.aux = root;
  call.phase = kBcastCall;
  Post all[kPeerMaxRanks];
  TRY(peer_enter(st, ps, call, all));
  for (int j = 0; j < p; j++)
    if (all[j].count != bytes || all[j].aux != root)
      return fail(TIPS_ERR_MISMATCH, "peer broadcast: rank %d broadcasts %lld B from root %lld, rank %d %lld B from root %d",
                  j, (long long)all[j].count, (long long)all[j].aux, r, (long long)bytes, root);
  *clean = false;
  TRY(setup_ws(st, ps));
  const int64_t piece = ps.ws_bytes / kAlignBytes * kAlignBytes;
  Post q = call;
  for (int64_t b = 0; b < bytes; b += piece) {
    const int64_t len = std::min(piece, bytes - b);
    if (b > 0) {  // every reader has its copy of the previous piece before the root overwrites it
      HIP_TRY(hipStreamSynchronize(user));
      q.phase = kPulled;
      TRY(barrier(st, ps, q, nullptr, peer_timeout()));
    }
    if (r == root) {
      tips::XferSeg segs[2] = {{in + b, ps.rdata[r], len}, {in + b, out + b, in == out ? 0 : len}};
      HIP_TRY(tips::launch_xfer(segs, 2, user));
      HIP_TRY(hipStreamSynchronize(user));
    }
    q.phase = kStaged;
    TRY(barrier(st, ps, q, nullptr, peer_timeout()));
    if (r != root) {
      tips::XferSeg seg = {ps.rdata[root], out + b, len};
      HIP_TRY(tips::launch_xfer(&seg, 1, user));
    }
  }
  return peer_leave(ps, user);
}

// Allgatherv (MPI_Allgatherv of AllgathervCpu, utils.h:83-116): per piece, every rank stages
// its next bytes in its own workspace and copies them to its place in out, barrier, then one
// xfer launch reads every peer's piece into out (one segment per peer: all links at once).
// Barrier 0 checks every rank's byte count against the counts the caller passed.
int peer_allgatherv_impl(State& st, PeerState& ps, const char* in, char* out, const int64_t* bytes, const int64_t* displ,
                         hipStream_t user, bool* clean) {
  const int p = st.size, r = st.rank;
  Post call{};
  call.count = bytes[r];
  call.phase = kGatherCall;
  Post all[kPeerMaxRanks];
  TRY(peer_enter(st, ps, call, all));
  int64_t longest = 0;
  for (int j = 0; j < p; j++) {
    if (all[j].count != bytes[j])
      return fail(TIPS_ERR_MISMATCH, "peer allgatherv: rank %d contributes %lld B, rank %d expects %lld B from it", j,
                  (long long)all[j].count, r, (long long)bytes[j]);
    longest = std::max(longest, bytes[j]);
  }
  *clean = false;
  TRY(setup_ws(st, ps));
  const int64_t piece = ps.ws_bytes / kAlignBytes * kAlignBytes;
  Post q = call;
  for (int64_t b = 0; b < longest; b += piece) {
    auto len_of = [&](int j) { return std::max<int64_t>(0, std::min(piece, bytes[j] - b)); };
    if (b > 0) {
      HIP_TRY(hipStreamSynchronize(user));
      q.phase = kPulled;
      TRY(barrier(st, ps, q, nullptr, peer_timeout()));
    }
    const bool self_in_place = (in + b == out + displ[r] + b);
    tips::XferSeg mine[2] = {{in + b, ps.rdata[r], len_of(r)}, {in + b, out + displ[r] + b, self_in_place ? 0 : len_of(r)}};
    HIP_TRY(tips::launch_xfer(mine, 2, user));
    HIP_TRY(hipStreamSynchronize(user));
    q.phase = kStaged;
    TRY(barrier(st, ps, q, nullptr, peer_timeout()));
    tips::XferSeg segs[tips::kMaxXferSegs];
    int m = 0;
    for (int d = 1; d < p; d++) {
      const int from = mod(r + d, p);
      segs[m++] = {ps.rdata[from], out + displ[from] + b, len_of(from)};
    }
    HIP_TRY(tips::launch_xfer(segs, m, user));
  }
  return peer_leave(ps, user);
}

PeerState& peer_state(State& st) {
  if (!st.peer) st.peer = new PeerState();
  return *st.peer;
}

int refuse_if_broken(PeerState& ps) {
  if (ps.broken)
    return fail(TIPS_ERR_HIP, "peer schedule: an earlier call failed part-way and left the ranks out of step; "
                              "shut down and re-initialise");
  return 0;
}

}  // namespace

int peer_broadcast(State& st, const char* in, char* out, int64_t bytes, int root, hipStream_t user) {
  PeerState& ps = peer_state(st);
  TRY(refuse_if_broken(ps));
  bool clean = true;
  const int rc = peer_broadcast_impl(st, ps, in, out, bytes, root, user, &clean);
  if (rc && !clean) ps.broken = true;
  return rc;
}

int peer_allgatherv(State& st, const char* in, char* out, const int64_t* bytes, const int64_t* displ, hipStream_t user) {
  PeerState& ps = peer_state(st);
  TRY(refuse_if_broken(ps));
  bool clean = true;
  const int rc = peer_allgatherv_impl(st, ps, in, out, bytes, displ, user, &clean);
  if (rc && !clean) ps.broken = true;
  return rc;
}

// device-resident allreduce over IPC-mapped peer memory, caller holds st.mu, 1 < p <= 16
int peer_allreduce(State& st, const char* in, char* out, int64_t n, int dtype, hipStream_t user) {
  if (!st.peer) st.peer = new PeerState();
  PeerState& ps = *st.peer;
  if (ps.broken)
    return fail(TIPS_ERR_HIP, "peer schedule: an earlier call failed part-way and left the ranks out of step; "
                              "shut down and re-initialise");
  bool clean = true;
  const int rc = peer_allreduce_impl(st, ps, in, out, n, dtype, user, &clean);
  if (rc && !clean) ps.broken = true;
  return rc;
}

}  // namespace rt
}  // namespace tips
