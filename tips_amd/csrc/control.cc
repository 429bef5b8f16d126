// control.cc — the control plane and the other collectives of the op surface.
//
// Replaces the reference's rank-0 negotiation checks (ConstructResponseMessage,
// tips/core/collective/coordinator.cc:90-186; GatherFirstRankSizes :40-88)
// with one small RCCL exchange of request records, after which every rank
// applies the same rules (so every rank reaches the same verdict); and the
// broadcast / allgatherv collectives (utils.h:83-134, ops.cc:156-286).
#include <algorithm>
#include <vector>

#include "rt.h"

namespace tips {
namespace rt {
namespace {

// Every rank's `words` int64 values, in rank order (one small RCCL allgather + host sync).
int exchange_i64(State& st, const int64_t* mine, int words, std::vector<int64_t>* all) {
  all->assign((size_t)words * st.size, 0);
  if (st.size == 1) {
    std::copy(mine, mine + words, all->begin());
    return 0;
  }
  TRY(st.small.ensure(sizeof(int64_t) * words * (st.size + 1)));
  int64_t* d = (int64_t*)st.small.p;
  HIP_TRY(hipMemcpyAsync(d + (size_t)words * st.size, mine, sizeof(int64_t) * words, hipMemcpyHostToDevice,
                         st.io_stream));
  if (peer_selected(st)) {
    std::vector<int64_t> b(st.size, (int64_t)sizeof(int64_t) * words), disp(st.size);
    for (int r = 0; r < st.size; r++) disp[r] = (int64_t)sizeof(int64_t) * words * r;
    TRY(peer_allgatherv(st, (const char*)(d + (size_t)words * st.size), (char*)d, b.data(), disp.data(), st.io_stream));
  } else {
    TRY(ensure_comm(st));
    TRY(rccl_enter(st, st.io_stream));
    NCCL_TRY(ncclAllGather(d + (size_t)words * st.size, d, (size_t)words, ncclInt64, st.comm, st.io_stream));
    TRY(rccl_leave(st, st.io_stream));
  }
  HIP_TRY(hipMemcpyAsync(all->data(), d, sizeof(int64_t) * words * st.size, hipMemcpyDeviceToHost, st.io_stream));
  HIP_TRY(hipStreamSynchronize(st.io_stream));
  return 0;
}

}  // namespace

std::string shape_str(const int64_t* rec) {  // tensorflow::TensorShape::DebugString() form: [2,4]
  std::string s = "[";
  for (int64_t d = 0; d < rec[2]; d++) s += (d ? "," : "") + std::to_string(rec[3 + d]);
  return s + "]";
}

// ConstructResponseMessage (coordinator.cc:90-186) + GatherFirstRankSizes (:40-88): every
// record is compared with rank 0's; the first mismatch is reported with the reference's text.
int check_records(const int64_t* t, int p) {
  const int W = TIPS_REQUEST_WORDS;
  const int64_t* r0 = t;
  for (int i = 1; i < p; i++)
    if (t[i * W + 1] != r0[1])
      return fail(TIPS_ERR_MISMATCH, "Mismatch data types found: %lld vs %lld.", (long long)r0[1], (long long)t[i * W + 1]);
  for (int i = 1; i < p; i++)  // (the reference compares requests[0] with itself here, coordinator.cc:123-129)
    if (t[i * W + 0] != r0[0])
      return fail(TIPS_ERR_MISMATCH, "Mismatched operations found: %lld vs %lld.", (long long)r0[0], (long long)t[i * W]);
  for (int i = 0; i < p; i++)
    if (t[i * W + 2] < 0 || t[i * W + 2] > TIPS_MAX_DIMS) return fail(TIPS_ERR_INVALID_ARG, "bad ndim in request %d", i);
  if (r0[0] == TIPS_REQ_ALLREDUCE || r0[0] == TIPS_REQ_BROADCAST) {
    for (int i = 1; i < p; i++) {
      const int64_t* ri = t + i * W;
      bool same = ri[2] == r0[2];
      for (int64_t d = 0; same && d < r0[2]; d++) same = ri[3 + d] == r0[3 + d];
      if (!same)
        return fail(TIPS_ERR_MISMATCH, "Mismatched %s tensor shapes: %s vs %s",
                    r0[0] == TIPS_REQ_BROADCAST ? "broadcast" : "allreduce", shape_str(r0).c_str(), shape_str(ri).c_str());
    }
  } else if (r0[0] == TIPS_REQ_ALLGATHER) {
    if (r0[2] == 0) return fail(TIPS_ERR_MISMATCH, "An empty tensor found");
    for (int i = 1; i < p; i++) {
      const int64_t* ri = t + i * W;
      if (ri[2] != r0[2])
        return fail(TIPS_ERR_MISMATCH, "Mismatched allgather tensor shapes: rank %lld vs %lld", (long long)r0[2],
                    (long long)ri[2]);
      for (int64_t d = 1; d < r0[2]; d++)
        if (ri[3 + d] != r0[3 + d])
          return fail(TIPS_ERR_MISMATCH, "Mismatched allgather tensor shapes: %lld-th dimension %lld vs %lld",
                      (long long)d, (long long)r0[3 + d], (long long)ri[3 + d]);
    }
  } else {
    return fail(TIPS_ERR_INVALID_ARG, "Not supported request type: %lld", (long long)r0[0]);
  }
  return 0;
}

}  // namespace rt
}  // namespace tips

using namespace tips::rt;

extern "C" {

int tips_check_requests(const int64_t* table, int p) {
  if (!table || p < 1) return fail(TIPS_ERR_INVALID_ARG, "bad request table");
  return check_records(table, p);
}

int tips_allreduce_checked(const void* in, void* out, const int64_t* shape, int ndim, int dtype, int op, void* stream) {
  TRY(check_dtype(dtype));
  if (ndim < 0 || ndim > TIPS_MAX_DIMS || (ndim > 0 && !shape)) return fail(TIPS_ERR_INVALID_ARG, "bad shape");
  int64_t count = 1;
  int64_t rec[TIPS_REQUEST_WORDS] = {TIPS_REQ_ALLREDUCE, dtype, ndim};
  for (int d = 0; d < ndim; d++) {
    if (shape[d] < 0) return fail(TIPS_ERR_INVALID_ARG, "negative dimension");
    rec[3 + d] = shape[d];
    count *= shape[d];
  }
  int routed_rc;  // (through the negotiation, when it runs: rank 0 then checks the shape itself)
  if (route_collective(TIPS_REQ_ALLREDUCE, dtype, shape, ndim, 0,
                       [&] { return tips_allreduce_checked(in, out, shape, ndim, dtype, op, stream); }, &routed_rc))
    return routed_rc;
  {
    State& st = S();
    std::lock_guard<std::mutex> lk(st.mu);
    if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
    TRY(set_device(st));
    std::vector<int64_t> all;
    TRY(exchange_i64(st, rec, TIPS_REQUEST_WORDS, &all));
    TRY(check_records(all.data(), st.size));
  }
  return tips_allreduce(in, out, count, dtype, op, stream);
}

int tips_allgather_i64(const int64_t* values, int words, int64_t* out) {
  if (!out || !values || words < 1 || words > 4096) return fail(TIPS_ERR_INVALID_ARG, "bad allgather_i64 args");
  int routed_rc;
  const int64_t shape[2] = {1, words};
  if (route_collective(TIPS_REQ_ALLGATHER, TIPS_INT64, shape, 2, 0, [&] { return tips_allgather_i64(values, words, out); },
                       &routed_rc))
    return routed_rc;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  TRY(set_device(st));
  std::vector<int64_t> all;
  TRY(exchange_i64(st, values, words, &all));
  std::copy(all.begin(), all.end(), out);
  return 0;
}

int tips_broadcast(const void* in, void* out, int64_t count, int dtype, int root, void* stream) {
  TRY(check_dtype(dtype));
  if (count < 0) return fail(TIPS_ERR_INVALID_ARG, "negative count");
  int routed_rc;
  const int64_t shape[1] = {count};
  if (route_collective(TIPS_REQ_BROADCAST, dtype, shape, 1, root,
                       [&] { return tips_broadcast(in, out, count, dtype, root, stream); }, &routed_rc))
    return routed_rc;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  if (root < 0 || root >= st.size) return fail(TIPS_ERR_INVALID_ARG, "root rank %d out of range", root);
  if (count == 0) return 0;
  if (!in || !out) return fail(TIPS_ERR_INVALID_ARG, "null pointer");
  TRY(set_device(st));
  const size_t bytes = (size_t)count * tips::dtype_size(dtype);
  return run_staged(st, in, bytes, out, bytes, (hipStream_t)stream, [&](const void* i, void* o, hipStream_t s) {
    if (st.size == 1) {
      if (i != o) HIP_TRY(tips::launch_copy_buf(o, i, (int64_t)bytes, s));
      return 0;
    }
    if (peer_selected(st))
      return peer_broadcast(st, (const char*)i, (char*)o, (int64_t)bytes, root, s);
    TRY(ensure_comm(st));
    // every rank must name the same root and size, or ncclBroadcast pairs nothing (the peer
    // schedule checks the same at its call barrier): one small exchange, the same verdict everywhere
    const int64_t mine[2] = {root, (int64_t)bytes};
    std::vector<int64_t> all;
    TRY(exchange_i64(st, mine, 2, &all));
    for (int j = 0; j < st.size; j++)
      if (all[2 * j] != root || all[2 * j + 1] != (int64_t)bytes)
        return fail(TIPS_ERR_MISMATCH, "broadcast: rank %d broadcasts %lld B from root %lld, rank %d %lld B from root %d",
                    j, (long long)all[2 * j + 1], (long long)all[2 * j], st.rank, (long long)bytes, root);
    TRY(rccl_enter(st, s));
    NCCL_TRY(ncclBroadcast(i, o, bytes, ncclInt8, root, st.comm, s));
    return rccl_leave(st, s);
  });
}

int tips_allgatherv(const void* in, int64_t count, void* out, const int64_t* counts, int dtype, void* stream) {
  TRY(check_dtype(dtype));
  int routed_rc;
  const int64_t shape[1] = {count < 0 ? 0 : count};
  if (route_collective(TIPS_REQ_ALLGATHER, dtype, shape, 1, 0,
                       [&] { return tips_allgatherv(in, count, out, counts, dtype, stream); }, &routed_rc))
    return routed_rc;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  if (!counts || count < 0) return fail(TIPS_ERR_INVALID_ARG, "bad counts");
  if (counts[st.rank] != count)
    return fail(TIPS_ERR_INVALID_ARG, "input and first_ranks not match %lld vs %lld", (long long)count,
                (long long)counts[st.rank]);  // AllgathervCpu's check, utils.h:103-106
  const int64_t es = tips::dtype_size(dtype);
  std::vector<int64_t> disp(st.size + 1, 0);
  for (int r = 0; r < st.size; r++) {
    if (counts[r] < 0) return fail(TIPS_ERR_INVALID_ARG, "negative count for rank %d", r);
    disp[r + 1] = disp[r] + counts[r];
  }
  if (disp[st.size] == 0) return 0;
  if (!out || (count > 0 && !in)) return fail(TIPS_ERR_INVALID_ARG, "null pointer");
  TRY(set_device(st));
  return run_staged(st, in, (size_t)(count * es), out, (size_t)(disp[st.size] * es), (hipStream_t)stream,
                    [&](const void* i, void* o, hipStream_t s) {
                      char* ob = (char*)o;
                      if (count > 0 && (const char*)i != ob + disp[st.rank] * es)
                        HIP_TRY(hipMemcpyAsync(ob + disp[st.rank] * es, i, (size_t)(count * es),
                                               hipMemcpyDeviceToDevice, s));
                      if (st.size == 1) return 0;
                      if (peer_selected(st)) {
                        std::vector<int64_t> b(st.size), d(st.size);
                        for (int r = 0; r < st.size; r++) b[r] = counts[r] * es, d[r] = disp[r] * es;
                        return peer_allgatherv(st, (const char*)i, ob, b.data(), d.data(), s);
                      }
                      TRY(ensure_comm(st));
                      TRY(rccl_enter(st, s));
                      NCCL_TRY(ncclGroupStart());
                      for (int r = 0; r < st.size; r++) {
                        if (r == st.rank) continue;
                        if (count > 0) NCCL_TRY(ncclSend(i, (size_t)(count * es), ncclInt8, r, st.comm, s));
                        if (counts[r] > 0)
                          NCCL_TRY(ncclRecv(ob + disp[r] * es, (size_t)(counts[r] * es), ncclInt8, r, st.comm, s));
                      }
                      NCCL_TRY(ncclGroupEnd());
                      return rccl_leave(st, s);
                    });
}

}  // extern "C"
