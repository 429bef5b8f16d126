// plan.cc — builds the per-rank op plans of the ring, direct and one-shot
// allreduce schedules (plan.h). Every index the schedules use lives here and
// only here: the RCCL executor, the single-GPU simulator and the CPU tests all
// consume these plans (schedules.cc, tips_schedule_plan).
//
// The arithmetic each plan encodes is the reference's out-of-place SUM
// (AllreduceCpu<T>, tips/core/collective/utils.h:52-67): the exchange that
// MPI_Allreduce does inside libmpi, and its per-chunk MPI_SUM as sum kernels.
#include "plan.h"

#include <algorithm>

#include "rt.h"

namespace tips {
namespace rt {

namespace {

// Staging slots that feed one multi_sum launch sit one slot plus 4 KiB apart:
// sources at power-of-two strides read ~7 % slower (profiles/r01_sum_sweep_multi_pad.jsonl).
constexpr int64_t kSlotPad = 4096;

PRef at(int buf, int64_t off) { return PRef{buf, off}; }

void xfer(PStep& st, int send, int peer, PRef where, int64_t bytes) {
  if (bytes > 0) st.xfers.push_back(PXfer{send, peer, where, bytes});  // empty transfers are skipped on both sides
}

void sum_of(PStep& st, PRef dst, const PRef* srcs, int nsrc, int64_t count) {
  if (count <= 0) return;
  PSum s{};
  s.dst = dst;
  s.nsrc = nsrc;
  for (int j = 0; j < nsrc; j++) s.src[j] = srcs[j];
  s.count = count;
  st.sums.push_back(s);
}

// Ring: reduce-scatter step s, rank r sends chunk (r-s) to r+1 and receives
// chunk (r-s-1) from r-1, which it adds to its own input: out = in + received (the fold order
// oracle_ring restates). Staging is double-buffered by step parity. Sub-chunk k of step s+1
// is sent only after the sum of sub-chunk k of step s (it sends what that sum wrote), so the
// transfer of sub-chunk k+1 overlaps the sum of sub-chunk k. Allgather: p-1 forwarding steps
// straight into out, rank r starting with the chunk (r+1) it completed last.
void ring(Plan& pl) {
  const int p = pl.p, r = pl.rank, K = pl.K, next = mod(r + 1, p), prev = mod(r - 1, p);
  const int64_t es = tips::dtype_size(pl.dtype), align = kAlignBytes / es, n = pl.n;
  const int64_t max_chunk = chunk_of(n, p, align, 0).len();
  pl.staging_bytes = 2 * max_chunk * es;
  for (int s = 0; s < p - 1; s++) {
    const Range sc = chunk_of(n, p, align, mod(r - s, p)), rc = chunk_of(n, p, align, mod(r - s - 1, p));
    const int64_t stg = (int64_t)(s & 1) * max_chunk * es;
    for (int k = 0; k < K; k++) {
      const Range ss = sub_of(sc, K, align, k), rs = sub_of(rc, K, align, k);
      PStep st;
      if (s > 0) st.wait_sum = (s - 1) * K + k;
      const PRef land = at(kBufStaging, stg + (rs.b - rc.b) * es);
      xfer(st, 1, next, at(s == 0 ? kBufIn : kBufOut, ss.b * es), ss.len() * es);
      xfer(st, 0, prev, land, rs.len() * es);
      const PRef srcs[2] = {at(kBufIn, rs.b * es), land};
      sum_of(st, at(kBufOut, rs.b * es), srcs, 2, rs.len());
      pl.steps.push_back(st);
    }
  }
  for (int s = 0; s < p - 1; s++) {
    const Range sc = chunk_of(n, p, align, mod(r + 1 - s, p)), rc = chunk_of(n, p, align, mod(r - s, p));
    for (int k = 0; k < K; k++) {
      const Range ss = sub_of(sc, K, align, k), rs = sub_of(rc, K, align, k);
      PStep st;
      if (s == 0) st.wait_sum = (p - 2) * K + k;
      xfer(st, 1, next, at(kBufOut, ss.b * es), ss.len() * es);
      xfer(st, 0, prev, at(kBufOut, rs.b * es), rs.len() * es);
      pl.steps.push_back(st);
    }
  }
}

// Direct / all-pairs: rank r owns chunk r. Per sub-chunk k, every peer's
// slice of chunk r arrives over its own xGMI link in one group, one p-input kernel folds the
// p contributions in rank order (slot j holds rank j's slice); then chunk r goes to every peer
// at once. Staging: p-1 slots, one per peer, kSlotPad apart.
void direct(Plan& pl) {
  const int p = pl.p, r = pl.rank, K = pl.K;
  const int64_t es = tips::dtype_size(pl.dtype), align = kAlignBytes / es, n = pl.n;
  const int64_t max_chunk = chunk_of(n, p, align, 0).len();
  const int64_t stride = max_chunk * es + kSlotPad;
  pl.staging_bytes = (int64_t)(p - 1) * stride;
  auto slot = [&](int j) { return (int64_t)(j < r ? j : j - 1) * stride; };
  const Range mine = chunk_of(n, p, align, r);
  for (int k = 0; k < K; k++) {
    const Range ms = sub_of(mine, K, align, k);
    PStep st;
    for (int d = 1; d < p; d++) {
      const int to = mod(r + d, p), from = mod(r - d, p);
      const Range ts = sub_of(chunk_of(n, p, align, to), K, align, k);
      xfer(st, 1, to, at(kBufIn, ts.b * es), ts.len() * es);
      xfer(st, 0, from, at(kBufStaging, slot(from) + (ms.b - mine.b) * es), ms.len() * es);
    }
    PRef srcs[tips::kMaxSrcs];
    for (int j = 0; j < p; j++)
      srcs[j] = (j == r) ? at(kBufIn, ms.b * es) : at(kBufStaging, slot(j) + (ms.b - mine.b) * es);
    sum_of(st, at(kBufOut, ms.b * es), srcs, p, ms.len());
    pl.steps.push_back(st);
  }
  for (int k = 0; k < K; k++) {
    const Range ms = sub_of(mine, K, align, k);
    PStep st;
    st.wait_sum = k;
    for (int d = 1; d < p; d++) {
      const int to = mod(r + d, p), from = mod(r - d, p);
      const Range fs = sub_of(chunk_of(n, p, align, from), K, align, k);
      xfer(st, 1, to, at(kBufOut, ms.b * es), ms.len() * es);
      xfer(st, 0, from, at(kBufOut, fs.b * es), fs.len() * es);
    }
    pl.steps.push_back(st);
  }
}

// One-shot (small buckets): every rank sends its whole bucket to every peer in
// one group (all xGMI links at once) and folds the p buckets in rank order with one multi_sum:
// (p-1)·S bytes per rank instead of 2(p-1)/p·S, but one exchange and one kernel. Same bits as
// direct.
void oneshot(Plan& pl) {
  const int p = pl.p, r = pl.rank;
  const int64_t bytes = pl.n * tips::dtype_size(pl.dtype);
  const int64_t stride = round_up(bytes, kAlignBytes) + kSlotPad;
  pl.staging_bytes = (int64_t)(p - 1) * stride;
  auto slot = [&](int j) { return (int64_t)(j < r ? j : j - 1) * stride; };
  PStep st;
  for (int d = 1; d < p; d++) {
    const int to = mod(r + d, p), from = mod(r - d, p);
    xfer(st, 1, to, at(kBufIn, 0), bytes);
    xfer(st, 0, from, at(kBufStaging, slot(from)), bytes);
  }
  PRef srcs[tips::kMaxSrcs];
  for (int j = 0; j < p; j++) srcs[j] = (j == r) ? at(kBufIn, 0) : at(kBufStaging, slot(j));
  sum_of(st, at(kBufOut, 0), srcs, p, pl.n);
  pl.steps.push_back(st);
}

}  // namespace

int plan_depth(int p, int64_t n, int dtype) {
  const int64_t es = tips::dtype_size(dtype);
  return pipeline_depth(chunk_of(n, p, kAlignBytes / es, 0).len() * es);
}

int build_schedule_plan(int algo, int p, int r, int64_t n, int dtype, int K, Plan* out) {
  if (tips::dtype_size(dtype) == 0) return fail(TIPS_ERR_INVALID_ARG, "unsupported dtype %d", dtype);
  if (p < 2 || r < 0 || r >= p || n < 0 || K < 1 || K > 1024)
    return fail(TIPS_ERR_INVALID_ARG, "bad plan request (p %d, rank %d, n %lld, K %d)", p, r, (long long)n, K);
  if ((algo == TIPS_ALGO_DIRECT || algo == TIPS_ALGO_ONESHOT) && p > tips::kMaxSrcs)
    return fail(TIPS_ERR_INVALID_ARG, "%s folds at most %d ranks", algo == TIPS_ALGO_DIRECT ? "direct" : "oneshot",
                tips::kMaxSrcs);
  Plan pl;
  pl.algo = algo;
  pl.p = p;
  pl.rank = r;
  pl.n = n;
  pl.dtype = dtype;
  pl.K = algo == TIPS_ALGO_ONESHOT ? 1 : K;
  switch (algo) {
    case TIPS_ALGO_RING: ring(pl); break;
    case TIPS_ALGO_DIRECT: direct(pl); break;
    case TIPS_ALGO_ONESHOT: oneshot(pl); break;
    default: return fail(TIPS_ERR_INVALID_ARG, "no plan for algorithm %d", algo);
  }
  *out = std::move(pl);
  return 0;
}

}  // namespace rt
}  // namespace tips
