// plan.h — the per-rank op plan of an allreduce schedule: the single source of
// truth for the ring, direct (all-pairs) and one-shot schedules.
//
// A plan is what one rank issues, as data: a list of steps, each at most
//   1. a wait of the comm stream for the sums of an earlier step,
//   2. one group of point-to-point transfers (one ncclGroupStart/End),
//   3. the sums that consume what the group received, on the compute stream.
// Buffers are named, not pointed to (the rank's in, out and staging, with byte
// offsets), so the same plan is
//   - executed by the RCCL executor on one rank per GPU (schedules.cc),
//   - executed for p virtual ranks on one GPU by the simulator (schedules.cc),
//   - dumped through tips_schedule_plan and checked on the CPU by the tests
//     (send/recv pairing, stream/event hazards, a numpy interpreter vs the oracle).
// What it replaces: the exchange + per-chunk MPI_SUM inside MPI_Allreduce,
// reached from AllreduceCpu<T> (reference tips/core/collective/utils.h:60-65).
#pragma once

#include <stdint.h>

#include <vector>

#include "kernels.h"

namespace tips {
namespace rt {

enum PlanBuf : int { kBufIn = 0, kBufOut = 1, kBufStaging = 2 };

struct PRef {
  int buf;      // PlanBuf
  int64_t off;  // bytes
};

// One point-to-point transfer of a step's group: send `bytes` from `at` to `peer`, or receive
// `bytes` from `peer` into `at`. Within one group, the k-th send from r to q pairs with the k-th
// receive on q from r.
struct PXfer {
  int send;  // 1 send, 0 receive
  int peer;
  PRef at;
  int64_t bytes;
};

// dst = ((src[0] + src[1]) + ...) over `count` elements: sum2 for nsrc == 2 (ring step), the
// rank-order fold (multi_sum) otherwise.
struct PSum {
  PRef dst;
  int nsrc;
  PRef src[tips::kMaxSrcs];
  int64_t count;
};

struct PStep {
  int wait_sum = -1;  // before the group: the comm stream waits for the sums of step `wait_sum`
  std::vector<PXfer> xfers;
  std::vector<PSum> sums;  // after the group has landed (comp stream waits on it)
};

struct Plan {
  int algo = 0, p = 1, rank = 0, dtype = 0, K = 1;
  int64_t n = 0;
  int64_t staging_bytes = 0;
  std::vector<PStep> steps;
};

// The plan rank `r` of `p` issues to allreduce `n` elements of `dtype` with schedule `algo`
// (TIPS_ALGO_RING / DIRECT / ONESHOT) and K sub-chunks per chunk (ignored by ONESHOT).
// Every rank's plan has the same number of steps. Returns 0 or a TIPS_ERR_* code.
int build_schedule_plan(int algo, int p, int r, int64_t n, int dtype, int K, Plan* out);

// Pipeline depth the runtime picks for a schedule (TIPS_PIPELINE_DEPTH / TIPS_MIN_SUBCHUNK_BYTES).
int plan_depth(int p, int64_t n, int dtype);

}  // namespace rt
}  // namespace tips
