// schedules.cc — the allreduce schedules over RCCL point-to-point (xGMI) and
// their single-GPU simulators.
//
// Replaces what MPI_Allreduce does inside libmpi for AllreduceCpu<T>
// (reference tips/core/collective/utils.h:60-65): the reduce-scatter +
// allgather exchange and, at each step, the local MPI_SUM — here the gfx950
// kernels of kernels.hip. One comm stream carries every RCCL call of a rank
// (one ordered channel, as the reference's single MPI_COMM_WORLD); sums run on
// a separate compute stream so sub-chunk k+1's transfer overlaps sub-chunk k's
// sum.
#include <string.h>

#include <algorithm>
#include <tuple>

#include "rt.h"

namespace tips {
namespace rt {
namespace {

// Staging slots that feed one multi_sum launch sit one slot plus 4 KiB apart:
// sources at power-of-two strides read ~7 % slower (profiles/r01_sum_sweep_multi_pad.jsonl).
constexpr int64_t kSlotPad = 4096;

// The sum kernel launch used by every schedule (ring step: out = local + received).
int sum2(void* dst, const void* a, const void* b, int64_t n, int dtype, hipStream_t s) {
  HIP_TRY(tips::launch_sum2(dst, a, b, n, dtype, s));
  return 0;
}

// ---------------------------------------------------------------------------
// Ring allreduce over RCCL send/recv. Own rank only.

int ring_allreduce(State& st, const char* in, char* out, int64_t n, int dtype, hipStream_t user) {
  const int p = st.size, r = st.rank, next = mod(r + 1, p), prev = mod(r - 1, p);
  const int64_t es = tips::dtype_size(dtype), align = kAlignBytes / es;
  const int64_t max_chunk = chunk_of(n, p, align, 0).len();
  const int K = pipeline_depth(max_chunk * es);
  TRY(st.staging.ensure((size_t)(2 * max_chunk * es)));
  TRY(st.recv_ev.ensure(2 * K));
  TRY(st.sum_ev.ensure(2 * K));
  char* stg[2] = {(char*)st.staging.p, (char*)st.staging.p + max_chunk * es};
  TRY(join(st.comm_stream, user, st.ev_start));
  HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.ev_start, 0));

  // reduce-scatter: at step s send chunk (r-s), receive chunk (r-s-1) and add it in
  for (int s = 0; s < p - 1; s++) {
    const Range sc = chunk_of(n, p, align, mod(r - s, p)), rc = chunk_of(n, p, align, mod(r - s - 1, p));
    const char* src = (s == 0) ? in : out;
    for (int k = 0; k < K; k++) {
      const Range ss = sub_of(sc, K, align, k), rs = sub_of(rc, K, align, k);
      if (s > 0) HIP_TRY(hipStreamWaitEvent(st.comm_stream, st.sum_ev.ev[((s - 1) & 1) * K + k], 0));
      char* land = stg[s & 1] + (rs.b - rc.b) * es;
      if (ss.len() > 0 || rs.len() > 0) {
        NCCL_TRY(ncclGroupStart());
        if (ss.len() > 0) NCCL_TRY(ncclSend(src + ss.b * es, ss.len() * es, ncclInt8, next, st.comm, st.comm_stream));
        if (rs.len() > 0) NCCL_TRY(ncclRecv(land, rs.len() * es, ncclInt8, prev, st.comm, st.comm_stream));
        NCCL_TRY(ncclGroupEnd());
      }
      hipEvent_t rev = st.recv_ev.ev[(s & 1) * K + k];
      HIP_TRY(hipEventRecord(rev, st.comm_stream));
      HIP_TRY(hipStreamWaitEvent(st.comp_stream, rev, 0));
      TRY(sum2(out + rs.b * es, in + rs.b * es, land, rs.len(), dtype, st.comp_stream));
      HIP_TRY(hipEventRecord(st.sum_ev.ev[(s & 1) * K + k], st.comp_stream));
    }
  }
  // allgather: rank r owns chunk (r+1); at step s forward chunk (r+1-s), receive chunk (r-s)
  for (int s = 0; s < p - 1; s++) {
    const Range sc = chunk_of(n, p, align, mod(r + 1 - s, p)), rc = chunk_of(n, p, align, mod(r - s, p));
    for (int k = 0; k < K; k++) {
      const Range ss = sub_of(sc, K, align, k), rs = sub_of(rc, K, align, k);
      if (s == 0) HIP_TRY(hipStreamWaitEvent(st.comm_stream, st.sum_ev.ev[((p - 2) & 1) * K + k], 0));
      if (ss.len() > 0 || rs.len() > 0) {
        NCCL_TRY(ncclGroupStart());
        if (ss.len() > 0) NCCL_TRY(ncclSend(out + ss.b * es, ss.len() * es, ncclInt8, next, st.comm, st.comm_stream));
        if (rs.len() > 0) NCCL_TRY(ncclRecv(out + rs.b * es, rs.len() * es, ncclInt8, prev, st.comm, st.comm_stream));
        NCCL_TRY(ncclGroupEnd());
      }
    }
  }
  TRY(join(user, st.comm_stream, st.ev_done));
  TRY(join(user, st.comp_stream, st.ev_comp_done));
  return 0;
}

// ---------------------------------------------------------------------------
// Direct (all-pairs) allreduce: rank r owns chunk r. Every
// peer's slice of chunk r arrives over its own xGMI link at once; one p-input
// kernel folds them in rank order; then chunk r goes to every peer at once.

int direct_allreduce(State& st, const char* in, char* out, int64_t n, int dtype, hipStream_t user) {
  const int p = st.size, r = st.rank;
  const int64_t es = tips::dtype_size(dtype), align = kAlignBytes / es;
  const int64_t max_chunk = chunk_of(n, p, align, 0).len();
  const int K = pipeline_depth(max_chunk * es);
  const int64_t stride = max_chunk * es + kSlotPad;
  TRY(st.staging.ensure((size_t)((p - 1) * stride)));
  TRY(st.recv_ev.ensure(K));
  TRY(st.sum_ev.ensure(K));
  auto slot = [&](int j) { return (char*)st.staging.p + (int64_t)(j < r ? j : j - 1) * stride; };
  const Range mine = chunk_of(n, p, align, r);
  TRY(join(st.comm_stream, user, st.ev_start));
  HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.ev_start, 0));
  for (int k = 0; k < K; k++) {
    const Range ms = sub_of(mine, K, align, k);
    NCCL_TRY(ncclGroupStart());
    for (int d = 1; d < p; d++) {
      const int to = mod(r + d, p), from = mod(r - d, p);
      const Range ts = sub_of(chunk_of(n, p, align, to), K, align, k);
      if (ts.len() > 0) NCCL_TRY(ncclSend(in + ts.b * es, ts.len() * es, ncclInt8, to, st.comm, st.comm_stream));
      if (ms.len() > 0)
        NCCL_TRY(ncclRecv(slot(from) + (ms.b - mine.b) * es, ms.len() * es, ncclInt8, from, st.comm, st.comm_stream));
    }
    NCCL_TRY(ncclGroupEnd());
    HIP_TRY(hipEventRecord(st.recv_ev.ev[k], st.comm_stream));
    HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.recv_ev.ev[k], 0));
    const void* srcs[tips::kMaxSrcs];
    for (int j = 0; j < p; j++) srcs[j] = (j == r) ? (const void*)(in + ms.b * es) : slot(j) + (ms.b - mine.b) * es;
    HIP_TRY(tips::launch_multi_sum(out + ms.b * es, srcs, p, ms.len(), dtype, st.comp_stream));
    HIP_TRY(hipEventRecord(st.sum_ev.ev[k], st.comp_stream));
  }
  for (int k = 0; k < K; k++) {
    const Range ms = sub_of(mine, K, align, k);
    HIP_TRY(hipStreamWaitEvent(st.comm_stream, st.sum_ev.ev[k], 0));
    NCCL_TRY(ncclGroupStart());
    for (int d = 1; d < p; d++) {
      const int to = mod(r + d, p), from = mod(r - d, p);
      const Range fs = sub_of(chunk_of(n, p, align, from), K, align, k);
      if (ms.len() > 0) NCCL_TRY(ncclSend(out + ms.b * es, ms.len() * es, ncclInt8, to, st.comm, st.comm_stream));
      if (fs.len() > 0) NCCL_TRY(ncclRecv(out + fs.b * es, fs.len() * es, ncclInt8, from, st.comm, st.comm_stream));
    }
    NCCL_TRY(ncclGroupEnd());
  }
  TRY(join(user, st.comm_stream, st.ev_done));
  TRY(join(user, st.comp_stream, st.ev_comp_done));
  return 0;
}

// One-shot (small buckets): every rank sends its whole bucket to
// every peer in one grouped step (all xGMI links at once) and folds the p
// buckets locally in rank order with one multi_sum launch. (p-1)·S bytes per
// rank instead of 2(p-1)/p·S, but 1 exchange + 1 kernel instead of 2(p-1)
// pipelined steps: latency-optimal. Same bits as direct (rank-order fold).
int oneshot_allreduce(State& st, const char* in, char* out, int64_t n, int dtype, hipStream_t user) {
  const int p = st.size, r = st.rank;
  const int64_t bytes = n * tips::dtype_size(dtype);
  const int64_t stride = (bytes + kAlignBytes - 1) / kAlignBytes * kAlignBytes + kSlotPad;
  TRY(st.staging.ensure((size_t)((p - 1) * stride)));
  auto slot = [&](int j) { return (char*)st.staging.p + (int64_t)(j < r ? j : j - 1) * stride; };
  TRY(join(st.comm_stream, user, st.ev_start));
  NCCL_TRY(ncclGroupStart());
  for (int d = 1; d < p; d++) {
    const int to = mod(r + d, p), from = mod(r - d, p);
    NCCL_TRY(ncclSend(in, (size_t)bytes, ncclInt8, to, st.comm, st.comm_stream));
    NCCL_TRY(ncclRecv(slot(from), (size_t)bytes, ncclInt8, from, st.comm, st.comm_stream));
  }
  NCCL_TRY(ncclGroupEnd());
  TRY(join(user, st.comm_stream, st.ev_done));  // the fold runs on the caller's stream
  const void* srcs[tips::kMaxSrcs];
  for (int j = 0; j < p; j++) srcs[j] = (j == r) ? (const void*)in : slot(j);
  HIP_TRY(tips::launch_multi_sum(out, srcs, p, n, dtype, user));
  return 0;
}

}  // namespace

// device-resident allreduce, caller holds st.mu
int allreduce_device(State& st, const void* in, void* out, int64_t n, int dtype, hipStream_t stream) {
  if (n == 0) return 0;
  const int64_t es = tips::dtype_size(dtype);
  const int algo = resolve_algo(st.algo, st.size, n * es);
  if (algo == TIPS_ALGO_RCCL) {
    TRY(ensure_comm(st));
    NCCL_TRY(ncclAllReduce(in, out, (size_t)n, nccl_type(dtype), ncclSum, st.comm, stream));
    return 0;
  }
  if (st.size == 1) {  // MPI_Allreduce on one rank returns the input
    if (in != out) HIP_TRY(hipMemcpyAsync(out, in, (size_t)(n * es), hipMemcpyDeviceToDevice, stream));
    return 0;
  }
  if (algo == TIPS_ALGO_PEER && st.size <= tips::kMaxSrcs)
    return peer_allreduce(st, (const char*)in, (char*)out, n, dtype, stream);
  TRY(ensure_comm(st));  // every other schedule moves its bytes over RCCL (no half-built group on failure)
  if (st.size > tips::kMaxSrcs && (algo == TIPS_ALGO_DIRECT || algo == TIPS_ALGO_ONESHOT || algo == TIPS_ALGO_PEER))
    return ring_allreduce(st, (const char*)in, (char*)out, n, dtype, stream);
  if (algo == TIPS_ALGO_ONESHOT) return oneshot_allreduce(st, (const char*)in, (char*)out, n, dtype, stream);
  if (algo == TIPS_ALGO_DIRECT) return direct_allreduce(st, (const char*)in, (char*)out, n, dtype, stream);
  return ring_allreduce(st, (const char*)in, (char*)out, n, dtype, stream);
}

// Peer transfers of the single-GPU simulators, batched per pipeline step:
// device-to-device copies, or (sim_transport 1) the same bytes as grouped
// ncclSend/ncclRecv pairs to this rank itself, so the RCCL p2p calls the real
// schedules make (byte counts, grouping, stream order) run on a 1-GPU box.
struct SimXfer {
  State& st;
  std::vector<std::tuple<void*, const void*, size_t>> ops;
  explicit SimXfer(State& s) : st(s) {}
  void add(void* dst, const void* src, int64_t bytes) {
    if (bytes > 0) ops.emplace_back(dst, src, (size_t)bytes);
  }
  int flush() {
    if (ops.empty()) return 0;
    if (st.sim_transport == 1) {
      NCCL_TRY(ncclGroupStart());
      for (auto& o : ops) {
        NCCL_TRY(ncclSend(std::get<1>(o), std::get<2>(o), ncclInt8, 0, st.comm, st.comm_stream));
        NCCL_TRY(ncclRecv(std::get<0>(o), std::get<2>(o), ncclInt8, 0, st.comm, st.comm_stream));
      }
      NCCL_TRY(ncclGroupEnd());
    } else {
      for (auto& o : ops)
        HIP_TRY(hipMemcpyAsync(std::get<0>(o), std::get<1>(o), std::get<2>(o), hipMemcpyDeviceToDevice, st.comm_stream));
    }
    ops.clear();
    return 0;
  }
};

int sim_prepare(State& st) {
  TRY(ensure_streams(st));
  if (st.sim_transport == 1) {
    if (!st.comm && st.size > 1) return fail(TIPS_ERR_UNSUPPORTED, "RCCL self-loop simulation needs a 1-rank setup");
    if (!st.comm) {
      if (st.size < 1) st.size = 1, st.rank = 0;
      TRY(ensure_comm(st));
    }
  }
  return 0;
}

}  // namespace rt
}  // namespace tips

using namespace tips::rt;

extern "C" {

int tips_chunk_bounds(int64_t count, int p, int dtype, int c, int64_t* begin, int64_t* end) {
  TRY(check_dtype(dtype));
  if (p < 1 || c < 0 || c >= p || count < 0 || !begin || !end) return fail(TIPS_ERR_INVALID_ARG, "bad chunk query");
  Range r = chunk_of(count, p, kAlignBytes / tips::dtype_size(dtype), c);
  *begin = r.b;
  *end = r.e;
  return 0;
}

int tips_schedule_shape(int64_t count, int p, int dtype, int* depth, int64_t* sub_elems) {
  TRY(check_dtype(dtype));
  if (p < 1 || count < 0 || !depth || !sub_elems) return fail(TIPS_ERR_INVALID_ARG, "bad schedule query");
  const int64_t es = tips::dtype_size(dtype), align = kAlignBytes / es;
  const Range c0 = chunk_of(count, p, align, 0);
  *depth = pipeline_depth(c0.len() * es);
  *sub_elems = sub_of(c0, *depth, align, 0).len();
  return 0;
}

// ---------------------------------------------------------------------------
// single-GPU schedule simulators (test harnesses)

int tips_ring_simulate(void* const* outs, const void* const* ins, int p, int64_t n, int dtype, void* stream) {
  TRY(check_dtype(dtype));
  if (p < 1 || p > 64 || n < 0 || !outs || !ins) return fail(TIPS_ERR_INVALID_ARG, "bad simulate args");
  if (n == 0) return 0;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  TRY(sim_prepare(st));
  SimXfer xf(st);
  hipStream_t user = (hipStream_t)stream;
  const int64_t es = tips::dtype_size(dtype), align = kAlignBytes / es;
  if (p == 1) {
    if (outs[0] != ins[0]) HIP_TRY(hipMemcpyAsync(outs[0], ins[0], (size_t)(n * es), hipMemcpyDeviceToDevice, user));
    return 0;
  }
  const int64_t max_chunk = chunk_of(n, p, align, 0).len();
  const int K = pipeline_depth(max_chunk * es);
  TRY(st.staging.ensure((size_t)(2 * p * max_chunk * es)));
  TRY(st.recv_ev.ensure(2 * K));
  TRY(st.sum_ev.ensure(2 * K));
  auto stg = [&](int r, int par) { return (char*)st.staging.p + ((int64_t)r * 2 + par) * max_chunk * es; };
  TRY(join(st.comm_stream, user, st.ev_start));
  HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.ev_start, 0));
  for (int s = 0; s < p - 1; s++) {
    for (int k = 0; k < K; k++) {
      if (s > 0) HIP_TRY(hipStreamWaitEvent(st.comm_stream, st.sum_ev.ev[((s - 1) & 1) * K + k], 0));
      for (int r = 0; r < p; r++) {  // virtual rank r receives from r-1
        const int prev = mod(r - 1, p);
        const Range rc = chunk_of(n, p, align, mod(r - s - 1, p));
        const Range rs = sub_of(rc, K, align, k);
        if (rs.len() == 0) continue;
        const char* src = (s == 0) ? (const char*)ins[prev] : (const char*)outs[prev];
        xf.add(stg(r, s & 1) + (rs.b - rc.b) * es, src + rs.b * es, rs.len() * es);
      }
      TRY(xf.flush());
      hipEvent_t rev = st.recv_ev.ev[(s & 1) * K + k];
      HIP_TRY(hipEventRecord(rev, st.comm_stream));
      HIP_TRY(hipStreamWaitEvent(st.comp_stream, rev, 0));
      for (int r = 0; r < p; r++) {
        const Range rc = chunk_of(n, p, align, mod(r - s - 1, p));
        const Range rs = sub_of(rc, K, align, k);
        TRY(sum2((char*)outs[r] + rs.b * es, (const char*)ins[r] + rs.b * es, stg(r, s & 1) + (rs.b - rc.b) * es,
                 rs.len(), dtype, st.comp_stream));
      }
      HIP_TRY(hipEventRecord(st.sum_ev.ev[(s & 1) * K + k], st.comp_stream));
    }
  }
  for (int s = 0; s < p - 1; s++) {
    for (int k = 0; k < K; k++) {
      if (s == 0) HIP_TRY(hipStreamWaitEvent(st.comm_stream, st.sum_ev.ev[((p - 2) & 1) * K + k], 0));
      for (int r = 0; r < p; r++) {
        const int prev = mod(r - 1, p);
        const Range rs = sub_of(chunk_of(n, p, align, mod(r - s, p)), K, align, k);
        if (rs.len() == 0) continue;
        xf.add((char*)outs[r] + rs.b * es, (const char*)outs[prev] + rs.b * es, rs.len() * es);
      }
      TRY(xf.flush());
    }
  }
  TRY(join(user, st.comm_stream, st.ev_done));
  TRY(join(user, st.comp_stream, st.ev_comp_done));
  return 0;
}

int tips_direct_simulate(void* const* outs, const void* const* ins, int p, int64_t n, int dtype, void* stream) {
  TRY(check_dtype(dtype));
  if (p < 1 || p > tips::kMaxSrcs || n < 0 || !outs || !ins) return fail(TIPS_ERR_INVALID_ARG, "bad simulate args");
  if (n == 0) return 0;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  TRY(sim_prepare(st));
  SimXfer xf(st);
  hipStream_t user = (hipStream_t)stream;
  const int64_t es = tips::dtype_size(dtype), align = kAlignBytes / es;
  if (p == 1) {
    if (outs[0] != ins[0]) HIP_TRY(hipMemcpyAsync(outs[0], ins[0], (size_t)(n * es), hipMemcpyDeviceToDevice, user));
    return 0;
  }
  const int64_t max_chunk = chunk_of(n, p, align, 0).len();
  const int K = pipeline_depth(max_chunk * es);
  // staging[r][j]: slice of chunk r sent by virtual rank j
  TRY(st.staging.ensure((size_t)((int64_t)p * p * max_chunk * es)));
  TRY(st.recv_ev.ensure(K));
  TRY(st.sum_ev.ensure(K));
  auto slot = [&](int r, int j) { return (char*)st.staging.p + ((int64_t)r * p + j) * max_chunk * es; };
  TRY(join(st.comm_stream, user, st.ev_start));
  HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.ev_start, 0));
  for (int k = 0; k < K; k++) {
    for (int r = 0; r < p; r++) {
      const Range mine = chunk_of(n, p, align, r), ms = sub_of(mine, K, align, k);
      if (ms.len() == 0) continue;
      for (int j = 0; j < p; j++)
        if (j != r) xf.add(slot(r, j) + (ms.b - mine.b) * es, (const char*)ins[j] + ms.b * es, ms.len() * es);
    }
    TRY(xf.flush());
    HIP_TRY(hipEventRecord(st.recv_ev.ev[k], st.comm_stream));
    HIP_TRY(hipStreamWaitEvent(st.comp_stream, st.recv_ev.ev[k], 0));
    for (int r = 0; r < p; r++) {
      const Range mine = chunk_of(n, p, align, r), ms = sub_of(mine, K, align, k);
      const void* srcs[tips::kMaxSrcs];
      for (int j = 0; j < p; j++)
        srcs[j] = (j == r) ? (const void*)((const char*)ins[r] + ms.b * es) : slot(r, j) + (ms.b - mine.b) * es;
      HIP_TRY(tips::launch_multi_sum((char*)outs[r] + ms.b * es, srcs, p, ms.len(), dtype, st.comp_stream));
    }
    HIP_TRY(hipEventRecord(st.sum_ev.ev[k], st.comp_stream));
  }
  for (int k = 0; k < K; k++) {
    HIP_TRY(hipStreamWaitEvent(st.comm_stream, st.sum_ev.ev[k], 0));
    for (int r = 0; r < p; r++) {
      const Range ms = sub_of(chunk_of(n, p, align, r), K, align, k);
      if (ms.len() == 0) continue;
      for (int j = 0; j < p; j++)
        if (j != r) xf.add((char*)outs[j] + ms.b * es, (const char*)outs[r] + ms.b * es, ms.len() * es);
    }
    TRY(xf.flush());
  }
  TRY(join(user, st.comm_stream, st.ev_done));
  TRY(join(user, st.comp_stream, st.ev_comp_done));
  return 0;
}

int tips_oneshot_simulate(void* const* outs, const void* const* ins, int p, int64_t n, int dtype, void* stream) {
  TRY(check_dtype(dtype));
  if (p < 1 || p > tips::kMaxSrcs || n < 0 || !outs || !ins) return fail(TIPS_ERR_INVALID_ARG, "bad simulate args");
  if (n == 0) return 0;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  TRY(sim_prepare(st));
  SimXfer xf(st);
  hipStream_t user = (hipStream_t)stream;
  const int64_t bytes = n * tips::dtype_size(dtype);
  if (p == 1) {
    if (outs[0] != ins[0]) HIP_TRY(hipMemcpyAsync(outs[0], ins[0], (size_t)bytes, hipMemcpyDeviceToDevice, user));
    return 0;
  }
  // staging[r][j]: rank j's bucket as received by virtual rank r
  TRY(st.staging.ensure((size_t)((int64_t)p * p * bytes)));
  auto slot = [&](int r, int j) { return (char*)st.staging.p + ((int64_t)r * p + j) * bytes; };
  TRY(join(st.comm_stream, user, st.ev_start));
  for (int r = 0; r < p; r++)
    for (int j = 0; j < p; j++)
      if (j != r) xf.add(slot(r, j), ins[j], bytes);
  TRY(xf.flush());
  TRY(join(user, st.comm_stream, st.ev_done));
  for (int r = 0; r < p; r++) {
    const void* srcs[tips::kMaxSrcs];
    for (int j = 0; j < p; j++) srcs[j] = (j == r) ? ins[r] : (const void*)slot(r, j);
    HIP_TRY(tips::launch_multi_sum(outs[r], srcs, p, n, dtype, user));
  }
  return 0;
}

}  // extern "C"
