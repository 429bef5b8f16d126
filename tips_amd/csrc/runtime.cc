// runtime.cc — lifecycle and data-path entry points of libtips_hip.so's C-ABI.
//
// Replaces, for the allreduce-SUM path of Superjomn/TiPS:
//   tips/core/operations.{h,cc}           lifecycle C-ABI (tips_init/shutdown/size/rank)
//   tips/core/collective/utils.h:52-67    AllreduceCpu<T> -> tips_allreduce
//   tips/core/collective/coordinator.cc   negotiation: with one process per GPU and
//                                         stream-ordered calls there is nothing to
//                                         negotiate per tensor (DESIGN.md §Control plane)
//   tips/core/mpi/tips_mpi.h:13-55        dtype traits -> RCCL byte transfers + dtype enum
// The data moves over RCCL point-to-point (xGMI) and is summed by the HIP
// kernels of kernels.hip. One comm stream carries every RCCL call of a rank
// (one ordered channel, as the reference's single MPI_COMM_WORLD); sums run on
// a separate compute stream so sub-chunk k+1's transfer overlaps sub-chunk k's sum.
#include <string.h>

#include <string>

#include "rt.h"

namespace tips {
int bootstrap_exchange(int rank, int size, const char* host, int port, void* id, int id_bytes, int timeout_s,
                       std::string* err);
}

using namespace tips::rt;

extern "C" {

const char* tips_last_error(void) { return last_error().c_str(); }
const char* tips_version(void) { return "tips_hip 0.1.0 (gfx950)"; }
int tips_unique_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

int tips_get_unique_id(void* out, int64_t cap) {
  if (!out || cap < (int64_t)sizeof(ncclUniqueId)) return fail(TIPS_ERR_INVALID_ARG, "unique id buffer too small");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  memcpy(out, &id, sizeof id);
  return (int)sizeof id;
}

int tips_init_rank(int rank, int size, int device, const void* unique_id, int64_t id_bytes) {
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (st.initialized) return 0;
  if (size < 1 || rank < 0 || rank >= size) return fail(TIPS_ERR_INVALID_ARG, "bad rank %d / size %d", rank, size);
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (ndev < 1) return fail(TIPS_ERR_HIP, "no HIP device visible");
  static const char* const local_vars[] = {"LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", nullptr};
  if (device < 0) device = env_first_int(local_vars, rank) % ndev;
  HIP_TRY(hipSetDevice(device));
  st.device = device;
  TRY(ensure_streams(st));
  if (size > 1 && !unique_id) return fail(TIPS_ERR_INVALID_ARG, "size > 1 needs a unique id");
  if (unique_id) {  // (a 1-rank id is accepted too: the same bootstrap, exercised on one GPU)
    if (id_bytes != (int64_t)sizeof(ncclUniqueId))
      return fail(TIPS_ERR_INVALID_ARG, "unique id must be %zu bytes", sizeof(ncclUniqueId));
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof id);
    // TIPS_NO_RCCL=1: no communicator (only the peer schedule, which needs none, can run). Lets
    // several ranks share one GPU, which RCCL refuses: the peer schedule's multi-process tests.
    rccl_env_defaults();
    if (!env_i64("TIPS_NO_RCCL", 0)) NCCL_TRY(ncclCommInitRank(&st.comm, size, id, rank));
    uint64_t h = 1469598103934665603ull;  // FNV-1a of the id: the peer schedule's node-local block name
    for (size_t i = 0; i < sizeof id; i++) h = (h ^ ((const unsigned char*)unique_id)[i]) * 1099511628211ull;
    st.peer_key = h ? h : 1;
  }
  st.rank = rank;
  st.size = size;
  st.initialized = true;
  return 0;
}

void tips_init(void) {
  const char* const rank_vars[] = {"RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", nullptr};
  const char* const size_vars[] = {"WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", nullptr};
  const int rank = env_first_int(rank_vars, 0), size = env_first_int(size_vars, 1);
  if (S().initialized) return;
  ncclUniqueId id;
  memset(&id, 0, sizeof id);
  if (size > 1) {
    const char* host = getenv("MASTER_ADDR");
    if (!host || !*host) host = "127.0.0.1";
    const int port = (int)env_i64("TIPS_BOOTSTRAP_PORT", env_i64("MASTER_PORT", 29500) + 17);
    if (rank == 0 && ncclGetUniqueId(&id) != ncclSuccess) {
      fail(TIPS_ERR_RCCL, "ncclGetUniqueId failed");
      return;
    }
    std::string err;
    if (tips::bootstrap_exchange(rank, size, host, port, &id, (int)sizeof id, (int)env_i64("TIPS_BOOTSTRAP_TIMEOUT", 300),
                                 &err) != 0) {
      fail(TIPS_ERR_BOOTSTRAP, "%s", err.c_str());
      return;
    }
  }
  tips_init_rank(rank, size, -1, size > 1 ? &id : nullptr, size > 1 ? (int64_t)sizeof id : 0);
}

void tips_shutdown(void) {
  (void)negotiation_stop();  // collective, like the reference's collective_shutdown service
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return;
  if (st.device >= 0) (void)hipSetDevice(st.device);
  if (st.comm_stream) (void)hipStreamSynchronize(st.comm_stream);
  if (st.comp_stream) (void)hipStreamSynchronize(st.comp_stream);
  graphs_release(st);  // replayed plans hold RCCL work: gone before the communicator
  lanes_release(st);   // (split from it)
  peer_release(st);  // collective: no rank frees its IPC workspace while a peer may still read it
  st.peer_key = 0;
  if (st.comm) {
    (void)ncclCommDestroy(st.comm);
    st.comm = nullptr;
  }
  fusion_release(st);
  if (st.d2h_stream) (void)hipStreamSynchronize(st.d2h_stream);
  host_release(st);
  st.staging.release();
  st.host_in.release();
  st.host_out.release();
  for (void** b : {&st.bounce_in, &st.bounce_out})
    if (*b) {
      (void)hipHostFree(*b);
      *b = nullptr;
    }
  st.fusion.release();
  st.small.release();
  st.cast_scratch.release();
  st.tuned.clear();
  st.recv_ev.release();
  st.sum_ev.release();
  for (hipEvent_t* e : {&st.ev_start, &st.ev_done, &st.ev_comp_done, &st.ev_comp_prev, &st.ev_graph[0],
                        &st.ev_graph[1], &st.ev_graph[2], &st.ev_graph[3], &st.ev_graph[4], &st.ev_rccl[0],
                        &st.ev_rccl[1]})
    if (*e) {
      (void)hipEventDestroy(*e);
      *e = nullptr;
    }
  st.pipe_ev.release();
  st.fuse_ev.release();
  st.fusion_threshold = 0;
  for (hipStream_t* s : {&st.comm_stream, &st.comp_stream, &st.io_stream, &st.h2d_stream, &st.d2h_stream,
                         &st.h2d_stream2, &st.fuse_stream, &st.bucket_stream, &st.graph_stream})
    if (*s) {
      (void)hipStreamDestroy(*s);
      *s = nullptr;
    }
  st.initialized = false;
  st.rank = st.size = -1;
}

int tips_bootstrap_broadcast(int rank, int size, const char* host, int port, void* buf, int64_t bytes, int timeout_s) {
  if (size < 1 || rank < 0 || rank >= size || port <= 0 || port > 65535 || bytes < 0 || bytes > (1 << 20) ||
      (bytes > 0 && !buf))
    return fail(TIPS_ERR_INVALID_ARG, "bad bootstrap args");
  std::string err;
  if (tips::bootstrap_exchange(rank, size, (host && *host) ? host : "127.0.0.1", port, buf, (int)bytes,
                               timeout_s > 0 ? timeout_s : 300, &err) != 0)
    return fail(TIPS_ERR_BOOTSTRAP, "%s", err.c_str());
  return 0;
}

bool tips_is_initialize(void) { return S().initialized; }
int tips_size(void) { return S().initialized ? S().size : -1; }
int tips_rank(void) { return S().initialized ? S().rank : -1; }

int tips_set_algorithm(int algo) {
  if (algo < TIPS_ALGO_AUTO || algo > TIPS_ALGO_TUNE) return fail(TIPS_ERR_INVALID_ARG, "bad algorithm %d", algo);
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  st.algo = algo;
  return 0;
}

int tips_get_algorithm(void) { return S().algo; }

#ifdef TIPS_DEV  // (development surface: libtips_hip_dev.so only, include/tips_hip_dev.h)
int tips_set_sim_transport(int transport) {
  if (transport != 0 && transport != 1) return fail(TIPS_ERR_INVALID_ARG, "bad sim transport %d", transport);
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  st.sim_transport = transport;
  return 0;
}
#endif  // TIPS_DEV

int tips_resolve_algorithm(int nranks, int64_t bytes) { return resolve_algo(S().algo, nranks, bytes); }

int tips_bucket_sum(void* dst, const void* a, const void* b, int64_t count, int dtype, void* stream) {
  TRY(check_dtype(dtype));
  if (count < 0) return fail(TIPS_ERR_INVALID_ARG, "negative count");
  if (count == 0) return 0;
  if (!dst || !a || !b) return fail(TIPS_ERR_INVALID_ARG, "null pointer");
  HIP_TRY(tips::launch_sum2(dst, a, b, count, dtype, (hipStream_t)stream));
  return 0;
}

#ifdef TIPS_DEV  // (development surface: libtips_hip_dev.so only, include/tips_hip_dev.h)
int tips_sum_variant(void* dst, const void* a, const void* b, int64_t count, int dtype, int mode, int unroll, int nt,
                     int blocks, int threads, void* stream) {
  TRY(check_dtype(dtype));
  if (count <= 0) return 0;
  HIP_TRY(tips::launch_sum2_variant(dst, a, b, count, dtype, mode, unroll, nt, blocks, threads, (hipStream_t)stream));
  return 0;
}
#endif  // TIPS_DEV

#ifdef TIPS_DEV  // (development surface: libtips_hip_dev.so only, include/tips_hip_dev.h)
int tips_multi_sum_variant(void* dst, const void* const* srcs, int nsrc, int64_t count, int dtype, int variant,
                           void* stream) {
  TRY(check_dtype(dtype));
  if (count <= 0) return 0;
  if (!srcs || nsrc < 1 || nsrc > tips::kMaxSrcs) return fail(TIPS_ERR_INVALID_ARG, "bad source list");
  HIP_TRY(tips::launch_multi_sum_variant(dst, srcs, nsrc, count, dtype, variant, (hipStream_t)stream));
  return 0;
}
#endif  // TIPS_DEV

int tips_multi_sum(void* dst, const void* const* srcs, int nsrc, int64_t count, int dtype, void* stream) {
  TRY(check_dtype(dtype));
  if (nsrc < 1 || nsrc > tips::kMaxSrcs) return fail(TIPS_ERR_INVALID_ARG, "nsrc must be 1..%d", tips::kMaxSrcs);
  if (count < 0) return fail(TIPS_ERR_INVALID_ARG, "negative count");
  if (count == 0) return 0;
  HIP_TRY(tips::launch_multi_sum(dst, srcs, nsrc, count, dtype, (hipStream_t)stream));
  return 0;
}

#ifdef TIPS_DEV  // (development surface: libtips_hip_dev.so only, include/tips_hip_dev.h)
int tips_copy_tiles_variant(const void* tiles, int ntiles, int variant, int64_t max_tile_bytes, void* stream) {
  if (ntiles < 0 || (ntiles > 0 && !tiles) || max_tile_bytes < 1 || max_tile_bytes > tips::kCopyTileBytes)
    return fail(TIPS_ERR_INVALID_ARG, "bad copy-tile arguments");
  HIP_TRY(tips::launch_copy_tiles_variant((const tips::CopyTile*)tiles, ntiles, variant, max_tile_bytes,
                                          (hipStream_t)stream));
  return 0;
}
#endif  // TIPS_DEV

#ifdef TIPS_DEV  // (development surface: libtips_hip_dev.so only, include/tips_hip_dev.h)
int tips_xfer(void* const* dsts, const void* const* srcs, const int64_t* bytes, int n, void* stream) {
  if (n < 0 || n > tips::kMaxXferSegs || (n > 0 && (!dsts || !srcs || !bytes)))
    return fail(TIPS_ERR_INVALID_ARG, "tips_xfer takes 0..%d segments", tips::kMaxXferSegs);
  tips::XferSeg segs[tips::kMaxXferSegs];
  for (int i = 0; i < n; i++) {
    if (bytes[i] < 0 || (bytes[i] > 0 && (!dsts[i] || !srcs[i]))) return fail(TIPS_ERR_INVALID_ARG, "bad segment %d", i);
    segs[i] = {(const char*)srcs[i], (char*)dsts[i], bytes[i]};
  }
  HIP_TRY(tips::launch_xfer(segs, n, (hipStream_t)stream));
  return 0;
}
#endif  // TIPS_DEV

int tips_allreduce(const void* in, void* out, int64_t count, int dtype, int op, void* stream) {
  TRY(check_dtype(dtype));
  if (op != TIPS_OP_SUM) return fail(TIPS_ERR_UNSUPPORTED, "only SUM is implemented (op %d)", op);
  if (count < 0) return fail(TIPS_ERR_INVALID_ARG, "negative count");
  int routed_rc;
  const int64_t shape[1] = {count};
  if (route_collective(TIPS_REQ_ALLREDUCE, dtype, shape, 1, 0,
                       [&] { return tips_allreduce(in, out, count, dtype, op, stream); }, &routed_rc))
    return routed_rc;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  if (count == 0) return 0;
  if (!in || !out) return fail(TIPS_ERR_INVALID_ARG, "null pointer");
  TRY(set_device(st));
  const size_t bytes = (size_t)count * tips::dtype_size(dtype);
  const bool dout = is_device_ptr(out);
  if (!dout && !is_device_ptr(in) && (int64_t)bytes > env_i64("TIPS_HOST_PIECE_BYTES", kHostPieceBytes))
    return allreduce_host_pipelined(st, (const char*)in, (char*)out, count, dtype);
  return run_staged(st, in, bytes, out, bytes, (hipStream_t)stream, [&](const void* i, void* o, hipStream_t s) {
    return allreduce_device(st, i, o, count, dtype, s);
  });
}

}  // extern "C"
