/*
 * tips_hip.h — C-ABI of libtips_hip.so, the MI355X-native gradient-bucket
 * reduction path behind TiPS's collective-allreduce API.
 *
 * Plain C: pointers, sizes, ints. No torch / TF / HIP types in any signature
 * (streams travel as `void*` = hipStream_t, NULL = the legacy default stream).
 * No exception crosses this boundary: every data-path call returns an int
 * status (TIPS_OK = 0, negative = error) and tips_last_error() returns the
 * message of the calling thread's last failure.
 *
 * Which reference interface each entry point replaces is cited per symbol.
 * Reference = Superjomn/TiPS.
 */
#ifndef TIPS_HIP_H_
#define TIPS_HIP_H_

#include <stdbool.h>
#include <stdint.h>

#if defined(__GNUC__)
#define TIPS_API __attribute__((visibility("default")))
#else
#define TIPS_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* dtype codes: values 0-3 are message::DataType (tips/core/message/
 * collective_messages.fbs:17-23: TF_FLOAT32=0, TF_FLOAT64=1, TF_INT32=2,
 * TF_INT64=3). 4 and 5 are new in this build (the reference has no 16-bit
 * allreduce). */
enum tips_dtype {
  TIPS_FLOAT32 = 0,
  TIPS_FLOAT64 = 1,
  TIPS_INT32 = 2,
  TIPS_INT64 = 3,
  TIPS_FLOAT16 = 4,
  TIPS_BFLOAT16 = 5,
};

/* reduction codes = CollectiveOpKind (tips/core/collective/utils.h:21-25).
 * The reference only ever issues SUM (coordinator.cc:256-274); so does this
 * build: MAX/MIN return TIPS_ERR_UNSUPPORTED. */
enum tips_op {
  TIPS_OP_SUM = 0,
  TIPS_OP_MAX = 1,
  TIPS_OP_MIN = 2,
};

/* status codes (the reference returns tensorflow::Status, utils.h:66) */
enum tips_status {
  TIPS_OK = 0,
  TIPS_ERR_INVALID_ARG = -1,
  TIPS_ERR_NOT_INITIALIZED = -2,
  TIPS_ERR_HIP = -3,
  TIPS_ERR_RCCL = -4,
  TIPS_ERR_UNSUPPORTED = -5,
  TIPS_ERR_BOOTSTRAP = -6,
  TIPS_ERR_MISMATCH = -7,
};

/* allreduce algorithms (tips_set_algorithm). */
enum tips_algorithm {
  TIPS_ALGO_AUTO = -1,  /* oneshot for small buckets (<= TIPS_ONESHOT_BYTES, 256 KiB), else ring for
                           p <= 2 and direct otherwise; TIPS_ALGO env overrides */
  TIPS_ALGO_RING = 0,   /* RCCL send/recv ring, RS + AG, sub-chunk pipelined */
  TIPS_ALGO_DIRECT = 1, /* all-pairs RS over every xGMI link + p-input sum kernel + AG */
  TIPS_ALGO_RCCL = 2,   /* ncclAllReduce, kept as a comparison point only */
  TIPS_ALGO_ONESHOT = 3, /* whole bucket to every peer in one step + one p-input fold (small buckets) */
  TIPS_ALGO_PEER = 4,    /* direct's exchange by our own kernels through IPC-mapped peer memory (no RCCL):
                            push + rank-order fold + pull, phases ordered by a node-local shared-memory barrier.
                            Host-synchronous: a device-pointer call under PEER returns only after its push and
                            fold have run on every rank (each phase ends in a stream synchronize + barrier); only
                            the final pull is left queued on the caller's stream. */
  TIPS_ALGO_TUNE = 5,    /* measured choice: on the first call of each bucket-size class (a power of two), every
                            rank times ring and direct at several pipeline depths on scratch copies of the call's
                            input, the ranks agree on the slowest rank's times (one small ncclAllReduce MAX) and
                            all keep the fastest for that class; small buckets take AUTO's one-shot. The peer
                            schedule joins the candidates with TIPS_TUNE_PEER=1. tips_tuned_choice reports it. */
};

/* ---- lifecycle: same names and types as tips/core/operations.h:7-21 ---- */

/* Replaces tips_init (operations.cc:12-22). Collective over all ranks.
 * Reads RANK / WORLD_SIZE / LOCAL_RANK (torchrun) or OMPI_COMM_WORLD_* /
 * PMI_* (mpirun); WORLD_SIZE unset = one rank. For size > 1 the RCCL unique
 * id is exchanged over TCP: rank 0 listens on MASTER_ADDR:TIPS_BOOTSTRAP_PORT
 * (default MASTER_PORT + 17). Errors are reported by tips_last_error() and
 * tips_is_initialize() stays false (the reference CHECK-fails instead). */
TIPS_API void tips_init(void);
/* Replaces tips_shutdown (operations.cc:24-44). Safe to call twice. */
TIPS_API void tips_shutdown(void);
/* Replaces tips_is_initialize (operations.cc:46). */
TIPS_API bool tips_is_initialize(void);
/* Replace tips_size / tips_rank (operations.cc:48,50). -1 before init. */
TIPS_API int tips_size(void);
TIPS_API int tips_rank(void);

/* ---- lifecycle extensions (no reference counterpart) ---- */

/* Bytes of an RCCL unique id (128). */
TIPS_API int tips_unique_id_bytes(void);
/* Writes a fresh unique id into out[0..cap). Call on rank 0 only; returns bytes or <0. */
TIPS_API int tips_get_unique_id(void* out, int64_t cap);
/* Initialise with an id distributed by the caller (e.g. through a
 * torch.distributed store). device < 0: LOCAL_RANK % device count. */
TIPS_API int tips_init_rank(int rank, int size, int device, const void* unique_id, int64_t id_bytes);
/* The TCP exchange tips_init uses for the unique id, exposed for callers
 * that bootstrap themselves (and for CPU tests): rank 0's buf[0..bytes) is
 * delivered into every other rank's buf. Rank 0 listens on port; others
 * connect to host:port, retrying for up to timeout_s seconds. */
TIPS_API int tips_bootstrap_broadcast(int rank, int size, const char* host, int port, void* buf, int64_t bytes, int timeout_s);
/* Join counters of this process (both TCP joins: the bootstrap and the negotiation channel):
 * connections a joining rank dropped because they reached itself (TCP simultaneous open), and
 * connections rank 0 dropped because the joiner never confirmed them (it gave up waiting). */
TIPS_API int tips_net_stats(int64_t* self_connects_refused, int64_t* unconfirmed_joins_refused);
/* Diagnostics (no reference counterpart): one line on what the negotiation's threads are doing now
 * - the background thread's phase (waiting, exchanging cycle k, executing request i of a cycle's
 * list), the completion thread's (which request's device work it waits for), the request queues and
 * the names still waiting for other ranks. Never blocks on the library's locks: for a watchdog's
 * hang report. */
TIPS_API int tips_debug_state(char* out, int64_t cap);
/* Message of the calling thread's last failed call ("" if none). */
TIPS_API const char* tips_last_error(void);
/* Library version string. */
TIPS_API const char* tips_version(void);

/* ---- data path ---- */

/* dst[i] = a[i] + b[i] on the device: the per-chunk MPI_SUM local reduce
 * that MPI_Allreduce runs at every reduce-scatter step (reached from
 * AllreduceCpu<T>, tips/core/collective/utils.h:60-65). In-place (dst == a
 * or dst == b) allowed. count in elements (int64: lifts the reference's
 * int limit, utils.h:62). Device pointers only. Stream-ordered, async. */
TIPS_API int tips_bucket_sum(void* dst, const void* a, const void* b, int64_t count, int dtype, void* stream);

/* dst[i] = ((srcs[0][i] + srcs[1][i]) + srcs[2][i]) + ... (rank-order fold),
 * 1 <= nsrc <= 16. f16/bf16 partials are kept in fp32 and rounded once. */
TIPS_API int tips_multi_sum(void* dst, const void* const* srcs, int nsrc, int64_t count, int dtype, void* stream);

/* Replaces AllreduceCpu<T> (tips/core/collective/utils.h:52-67) and the
 * MPIAllreduce op's data path (tips/tensorflow/ops.cc:86-115):
 * out = SUM over ranks of in, out-of-place (in == out allowed).
 * Device pointers: stream-ordered, returns after enqueue (TIPS_ALGO_PEER excepted: it
 * blocks the host through its push and fold phases, see enum tips_algorithm).
 * Host pointers (both): staged through HBM, returns when out is written.
 * op must be TIPS_OP_SUM. */
TIPS_API int tips_allreduce(const void* in, void* out, int64_t count, int dtype, int op, void* stream);

/* ---- control plane: cross-rank request validation ---- */

/* request types = message::RequestType (collective_messages.fbs:3-7) */
enum tips_request_type {
  TIPS_REQ_ALLREDUCE = 0,
  TIPS_REQ_ALLGATHER = 1,
  TIPS_REQ_BROADCAST = 2,
};
#define TIPS_MAX_DIMS 8
/* one request record: {request_type, dtype, ndim, dims[TIPS_MAX_DIMS]} */
#define TIPS_REQUEST_WORDS (3 + TIPS_MAX_DIMS)

/* Replaces ConstructResponseMessage (coordinator.cc:90-186) and
 * GatherFirstRankSizes (coordinator.cc:40-88): table holds p request records
 * (rank order); each is compared with rank 0's. Returns TIPS_OK, or
 * TIPS_ERR_MISMATCH with the reference's error text in tips_last_error()
 * ("Mismatch data types found: 0 vs 1.", "Mismatched allreduce tensor shapes:
 * [2,4] vs [2,3]", "Mismatched allgather tensor shapes: 1-th dimension 3 vs 4",
 * ...). Pure host function. */
TIPS_API int tips_check_requests(const int64_t* table, int p);

/* tips_allreduce preceded by that validation: the records of all ranks are
 * exchanged (one small RCCL allgather + host sync), so every rank reaches the
 * same verdict; on a mismatch no rank reduces. shape = the tensor's dims. */
TIPS_API int tips_allreduce_checked(const void* in, void* out, const int64_t* shape, int ndim, int dtype, int op, void* stream);

/* ---- the other collectives of the op surface ---- */

/* out[r*words + w] = values[w] of rank r (host memory, blocking; words <= 4096). */
TIPS_API int tips_allgather_i64(const int64_t* values, int words, int64_t* out);
/* Replaces BroadcastCpu (utils.h:130-134) / MPIBroadcast (ops.cc:214-286):
 * out = root's in on every rank (in == out allowed). Any root (the reference
 * only supports 0, ops.cc:219). Host or device pointers, as tips_allreduce. */
TIPS_API int tips_broadcast(const void* in, void* out, int64_t count, int dtype, int root, void* stream);
/* Replaces AllgathervCpu (utils.h:83-128) / MPIAllgather (ops.cc:156-212):
 * out = concatenation over ranks of in, rank r contributing counts[r]
 * elements (counts[rank] must equal count). Host or device pointers. */
TIPS_API int tips_allgatherv(const void* in, int64_t count, void* out, const int64_t* counts, int dtype, void* stream);

/* Page-lock a long-lived host buffer (hipHostRegister) so host-memory calls on
 * it take the asynchronous DMA path (pinned: 40 GiB/s vs 29 GiB/s pageable for
 * a 256 MiB bucket). The caller must unregister before freeing
 * the memory. */
TIPS_API int tips_host_register(void* ptr, int64_t bytes);
TIPS_API int tips_host_unregister(void* ptr);

/* Tensor fusion (no reference counterpart): allreduce n device
 * tensors in place, packed into buckets of at most the fusion threshold
 * (TIPS_FUSION_THRESHOLD bytes, default 64 MiB; tensors at or above it are
 * reduced on their own). One dtype for all. The bucket layout depends only on
 * counts, dtype and threshold, never on where the tensors lie, so every rank
 * pairs the same elements. Stream-ordered on `stream`: the pack / unpack launches
 * run on `stream` itself (the bucket allreduces at N > 1 on a library stream forked
 * from it and joined back). Calls from different streams are safe: the fused calls
 * form one chain (each ends with an event a call from another stream waits for),
 * since the fusion slots and pointer tables are shared.
 * Graph capture: a fused call made under stream capture must find its pointer table
 * built (the same call made once before the capture) and stays out of the chain. The
 * table it used is then kept for the life of the job - never refilled, reused or freed
 * - and so are the fusion slots it packs into, past a change of TIPS_FUSION_THRESHOLD
 * (new slots are allocated beside them; all are freed at tips_shutdown). The replays
 * share those slots with eager fused calls: order a replay with fused calls on other
 * streams yourself (launch it on the same stream, or join the streams), as for any
 * graph that uses a shared workspace. */
TIPS_API int tips_fused_allreduce(void* const* ptrs, const int64_t* counts, int n, int dtype, void* stream);
/* The same, out of place: outs[i] = SUM over ranks of ins[i] (ins[i] == outs[i]
 * allowed); the inputs are left unchanged. What the reference's per-gradient
 * allreduce loop returns (tips/tensorflow/__init__.py:203-222), fused. */
TIPS_API int tips_fused_allreduce_oop(const void* const* ins, void* const* outs, const int64_t* counts, int n,
                                      int dtype, void* stream);

/* Compression.fp16 fused into the buckets (tips/tensorflow/compression.py:49-66 cast per tensor
 * before and after the allreduce, __init__.py:81-88): n f32 device tensors in[i] -> out[i]
 * (in == out allowed) allreduced in `wire_dtype` (TIPS_FLOAT16 or TIPS_BFLOAT16). Each tensor is cast
 * to the wire type (round to nearest even) as it is packed into a fusion bucket, every bucket is
 * allreduced in the wire type (half the bytes on the links), and cast back to f32 as it is
 * unpacked: one pack and one unpack launch per bucket instead of two casts per tensor. The
 * results are those of the per-tensor compress -> allreduce -> decompress. At one rank: the round
 * trip through the wire type. dtype must be TIPS_FLOAT32 (else TIPS_ERR_UNSUPPORTED), device memory,
 * stream-ordered as tips_fused_allreduce; routed through the negotiation (announced with the wire
 * type) once one runs. */
TIPS_API int tips_fused_allreduce_cast(const void* const* ins, void* const* outs, const int64_t* counts, int n,
                                       int dtype, int wire_dtype, void* stream);
/* The byte offset of each tensor of a fused list in ONE flat buffer laid out as the fusion buckets
 * (offsets[i], 256-B aligned; may be NULL); returns the flat buffer's size in bytes (< 0 = error).
 * A pure host function of counts, dtype and TIPS_FUSION_THRESHOLD - the same on every rank. */
TIPS_API int64_t tips_fused_layout(const int64_t* counts, int n, int dtype, int64_t* offsets);
/* flat = SUM over ranks of ins, tensor i at offsets[i] of tips_fused_layout (device memory of its
 * size): each bucket is packed straight into its region of `flat` and allreduced there in place -
 * no fusion slot, no unpack (2 x the gradient bytes of HBM traffic instead of 4 x). What
 * allreduce_grads returns views of (the reference's per-gradient loop, __init__.py:203-222). Inputs
 * unchanged; padding bytes of `flat` unspecified. One rank: one copy launch. Stream-ordered. */
TIPS_API int tips_fused_allreduce_flat(const void* const* ins, const int64_t* counts, int n, int dtype, void* flat,
                                       void* stream);
/* Measurement entry (bench.py, tools/copy_sweep_balanced.py): the pack launch the fusion issues for
 * bucket `bucket` of this list's layout (copy_segs_kernel over the bucket's tiles), into `dst` (device
 * memory of the bucket's padded size), on `stream`. Returns the bytes of the tensors the bucket holds
 * (the launch reads and writes each once), or with bucket < 0 the number of buckets; < 0 = error.
 * Part of the fusion chain like the calls above, except that it leaves the chain's end event to be
 * recorded on `stream` by the next fused call from another stream (so launches queue back to back):
 * `stream` must still exist then. */
TIPS_API int64_t tips_fused_pack_bucket(const void* const* ins, const int64_t* counts, int n, int dtype, int bucket,
                                        void* dst, void* stream);
/* Fusion caches of this process: layouts built / found (a layout is a function of the counts only,
 * so fresh gradient tensors every step still hit), and per-call pointer tables built (uploaded) /
 * found. Any pointer may be NULL. */
TIPS_API int tips_fusion_stats(int64_t* layouts_built, int64_t* layout_hits, int64_t* tables_built,
                               int64_t* table_hits);
/* Host tensors (numpy / CPU framework tensors, pageable or page-locked): outs[i] = SUM over ranks of
 * ins[i]. The list is packed by the library's host threads (TIPS_HOST_THREADS, 8) into page-locked
 * pieces of one byte stream (TIPS_HOST_FUSED_PIECE_BYTES, 32 MiB, ramped from 2 MiB at both ends);
 * each piece runs H2D -> allreduce in HBM -> D2H pipelined on separate streams while the threads
 * pack the next and unpack the previous.
 * The layout depends on the counts only. Blocks until every out is written (the reference's op is a
 * CPU op, ops.cc:118; its per-gradient loop, __init__.py:212-222, fused). */
TIPS_API int tips_fused_allreduce_host(const void* const* ins, void* const* outs, const int64_t* counts, int n,
                                       int dtype);
/* The same into ONE host buffer laid out as tips_fused_layout (the device flat layout): tensor i's sum at
 * offsets[i] of `flat`. When `flat` is page-locked (tips_host_register) each piece's D2H lands in it
 * directly - no unpack at all; otherwise through a page-locked slot and one contiguous copy per piece.
 * What allreduce_grads returns views of for host gradients. Blocks until `flat` is written. */
TIPS_API int tips_fused_allreduce_host_flat(const void* const* ins, const int64_t* counts, int n, int dtype,
                                            void* flat);

/* ---- named, asynchronous allreduce with cross-rank negotiation ---- */

/* Replaces EnqueueTensorCollective + the coordinator's background loop
 * (coordinator.cc:223-241, 355-513): requests may be enqueued in any order on
 * different ranks. A background thread per rank agrees with rank 0 (TCP,
 * MASTER_ADDR:TIPS_NEGOTIATION_PORT, default MASTER_PORT + 19) which names
 * every rank has enqueued, validates them with ConstructResponseMessage's
 * rules and error text, and every rank reduces them in rank 0's
 * readiness order (as ready_to_reduce), on the stream passed here. Device pointers run
 * stream-ordered; host pointers (both in and out host, as the reference's MPIAllreduce is a CPU
 * op, ops.cc:118) run on the negotiation thread, staged through HBM like tips_allreduce's, and
 * are done when tips_wait returns. Returns a handle > 0, or a negative status. The first call starts the
 * thread (collective: every rank's first named request must come after the same synchronous
 * collectives - their number is compared at the join, and a difference fails every rank's start
 * with both numbers instead of pairing RCCL calls wrongly). tips_shutdown stops it (collective).
 * From then on every synchronous collective of this library (tips_allreduce, tips_allreduce_checked,
 * tips_broadcast, tips_allgatherv, tips_allgather_i64, the tips_fused_* calls), from any thread, is
 * routed through the same negotiation: announced as request "~sync.<k>" (k-th such call of the rank)
 * with its type, dtype and shape, checked by rank 0 like any request, and run on the negotiation
 * thread in rank 0's order - so a rank's RCCL calls are issued from one thread in one order, the same
 * on every rank, as the reference's coordinator issues every collective. A routed call returns when
 * its device work is queued on the caller's stream (host memory: when it is done), as a direct call.
 * Synchronous calls from several threads at once must still come in the same order on every rank. */
TIPS_API int64_t tips_enqueue_allreduce(const char* name, const void* in, void* out, int64_t count, int dtype,
                                        void* stream);
/* The same with the tensor's shape (ndim <= TIPS_MAX_DIMS; ndim 0 = a scalar, announced as
 * shape [1] as CreateNoEmptyTfShape does, coordinator.cc:212-221): rank 0 validates shapes
 * with ConstructResponseMessage's rule and text (coordinator.cc:129-146), so a [2,4] request
 * on one rank and [4,2] on another fails on every rank with "Mismatched allreduce tensor
 * shapes: [2,4] vs [4,2]" although the element counts agree. tips_enqueue_allreduce
 * announces shape [count]. */
TIPS_API int64_t tips_enqueue_allreduce_shaped(const char* name, const void* in, void* out, const int64_t* shape,
                                               int ndim, int dtype, void* stream);
/* 1 = done (handle released), 0 = pending, < 0 = error (message in tips_last_error). */
TIPS_API int tips_poll(int64_t handle);
/* Blocks until the request is reduced (TIPS_OK, handle released) or failed (< 0). */
TIPS_API int tips_wait(int64_t handle);
/* n named requests in one call (what a framework's gradient hook hands over at once):
 * handles[i] = tips_enqueue_allreduce(names[i], ins[i], outs[i], counts[i], dtype, stream).
 * Returns TIPS_OK, or the first failure (its handles[i] < 0; the others are enqueued). */
TIPS_API int tips_enqueue_allreduce_n(const char* const* names, const void* const* ins, void* const* outs,
                                      const int64_t* counts, int n, int dtype, void* stream, int64_t* handles);
/* Shaped form of tips_enqueue_allreduce_n: tensor i has ndims[i] dims, taken in order from the
 * concatenated dims array (sum of ndims entries). */
TIPS_API int tips_enqueue_allreduce_shaped_n(const char* const* names, const void* const* ins, void* const* outs,
                                             const int* ndims, const int64_t* dims, int n, int dtype, void* stream,
                                             int64_t* handles);
/* tips_wait on each of n handles (handles <= 0 are skipped): TIPS_OK or the first failure. */
TIPS_API int tips_wait_n(const int64_t* handles, int n);
/* Completion callback of a named request (the reference's OpRecord::callback, ops.cc:107-110,
 * which sets the op's status and calls TF's done()): status TIPS_OK or a negative status, message
 * the failure's text ("" on success; valid during the call only). */
typedef void (*tips_done_fn)(void* ctx, int status, const char* message);
/* Register fn for the request `handle` (any of the three types): the library calls fn(ctx, status,
 * message) exactly once, from its completion thread, when the request has finished - for device
 * memory when its work on the device has completed - and releases the handle (tips_wait / tips_poll
 * on it then fail). A request that has already finished is called back at once (from that thread).
 * What an AsyncOpKernel body needs: enqueue, register, return; done() from the callback
 * (INTEGRATION.md §2). */
TIPS_API int tips_on_done(int64_t handle, tips_done_fn fn, void* ctx);
/* tips_enqueue_allreduce_shaped and tips_on_done in one call, as the reference enqueues one
 * OpRecord that carries its callback (EnqueueTensorCollective, coordinator.cc:223-241; CHECK(record.
 * callback)): one lock instead of two per request for an op body on many executor threads. Returns
 * the handle (> 0; it completes only through fn, and tips_wait / tips_poll / tips_on_done do not
 * know it) or < 0, in which case fn is never called. */
TIPS_API int64_t tips_enqueue_allreduce_cb(const char* name, const void* in, void* out, const int64_t* shape, int ndim,
                                           int dtype, void* stream, tips_done_fn fn, void* ctx);
/* Named broadcast through the same negotiation (the reference's MPIBroadcast op,
 * ops.cc:214-286 -> EnqueueTensorCollective(RequestType_BROADCAST); PerformCollectiveOp's
 * broadcast branch, coordinator.cc:275-295): rank 0 checks dtype and shape with
 * ConstructResponseMessage's rules and text ("Mismatched broadcast tensor shapes: ..."), and
 * that every rank names the same root. out = root's `in`, on `stream`, in rank 0's readiness
 * order with the other requests. (The reference's branch always broadcasts from rank 0 -
 * "root_rank should be passed in", coordinator.cc:280; here `root` is honoured.) */
TIPS_API int64_t tips_enqueue_broadcast(const char* name, const void* in, void* out, const int64_t* shape, int ndim,
                                        int dtype, int root, void* stream);
/* Output allocator of a named allgather: returns device memory of `bytes` (or NULL). Called
 * once, from the negotiation thread, when the output's size is known - as the reference's
 * PerformCollectiveOp allocates the op's output only then (context->allocate_output,
 * coordinator.cc:305-313). The caller owns what it returns. */
typedef void* (*tips_alloc_fn)(void* ctx, int64_t bytes);
/* Named allgather (MPIAllgather, ops.cc:156-212 -> RequestType_ALLGATHER): every rank's tensor
 * concatenated along dimension 0, in rank order. Rank 0 checks ndim and every dimension but
 * the first (GatherFirstRankSizes's rules and text, coordinator.cc:40-88) and sends every rank
 * the first dimensions; each rank then allocates its output through alloc(ctx, bytes), stores
 * the output's first dimension in *out_rows (valid once tips_wait / tips_poll report done) and
 * gathers on `stream`. ndim >= 1. A host `in` gets a host output: alloc must then return host memory. */
TIPS_API int64_t tips_enqueue_allgather(const char* name, const void* in, const int64_t* shape, int ndim, int dtype,
                                        void* stream, tips_alloc_fn alloc, void* ctx, int64_t* out_rows);

/* Select the allreduce algorithm (enum tips_algorithm). Returns TIPS_OK or an error. */
TIPS_API int tips_set_algorithm(int algo);
/* The algorithm currently selected (may be TIPS_ALGO_AUTO). */
TIPS_API int tips_get_algorithm(void);
/* The algorithm the current selection resolves to for a bucket of `bytes` on `nranks`. */
TIPS_API int tips_resolve_algorithm(int nranks, int64_t bytes);
/* Under TIPS_ALGO_TUNE: the schedule and pipeline depth this job measured for buckets of
 * `bytes`' size class. Returns 1 (and fills algo / depth) once that class has been tuned,
 * 0 before; < 0 on error. */
TIPS_API int tips_tuned_choice(int64_t bytes, int* algo, int* depth);
/* The same, with the number of transfer lanes the choice runs on: RCCL communicators split from
 * the job's, whose groups of consecutive plan steps are in flight together (1 = the comm stream
 * alone). TIPS_LANES sets it (the same on every rank) for an explicitly selected schedule. */
TIPS_API int tips_tuned_schedule(int64_t bytes, int* algo, int* depth, int* lanes);
/* Every candidate the tuner timed for `bytes`' size class: schedule, pipeline depth, lanes and
 * the slowest rank's ms per call (the numbers the choice was made on; the same on every rank).
 * Fills up to `cap` entries and returns how many candidates there were (0 before that class was
 * tuned; cap 0 asks the count), < 0 on error. */
TIPS_API int tips_tuned_timings(int64_t bytes, int* algos, int* depths, int* lanes, double* ms, int cap);
/* Replayed plans (TIPS_GRAPHS=1, opt-in; default 0): a ring / direct / one-shot call of at most
 * TIPS_GRAPH_MAX_BYTES (8 MiB: latency-bound buckets) made again on the same buffers (same
 * addresses and allocations) is captured once into a HIP graph and replayed with one launch;
 * streams, events and results are those of the eager steps. Needs ROCm >= 7.0 / RCCL >= 2.26
 * (torch's bundled runtime and /opt/rocm's 7.2 are both tested). Opt in only when no other thread
 * of the process issues work on the legacy null stream (hipMemcpy, hipMemset, launches on stream
 * 0, torch's default stream): such work invalidates a capture in progress on any stream, and RCCL
 * crashes inside the invalidated capture. Plans executed by the negotiation thread
 * (named requests, routed collectives) are never captured.
 * Reports this process's captures, replays and cached graphs.
 * A plan whose capture fails runs eagerly from then on; the others keep replaying.
 * Returns 0 (graphs on), 1 (3 failed captures turned them off for the job), 2 (off: not asked
 * for, or an older runtime), 3 (replays yielded: one bucket shape kept arriving at new addresses
 * after replays - TIPS_FRESH_WAIT_LIMIT host waits, 4 - so every plan now runs eagerly and no call
 * waits on the host), < 0 on error. */
TIPS_API int tips_graph_stats(int64_t* captured, int64_t* replayed, int64_t* cached);
/* The cost of keeping RCCL's order after replays: how many times an eager RCCL call (a larger
 * bucket, a fused call, a synchronous collective) found a replay still pending and blocked the
 * calling host thread until it had run (TIPS_REPLAY_HOST_ORDER, default 1), and the host time those
 * waits took in total (ns). Counts since tips_init. */
TIPS_API int tips_replay_order_stats(int64_t* host_waits, int64_t* host_wait_ns);


/* Pipeline shape the ring/direct schedules use for a bucket: depth = K
 * sub-chunks per chunk, sub_elems = elements in a (first) sub-chunk, i.e. the
 * size of one reduce-kernel launch (TIPS_PIPELINE_DEPTH, TIPS_MIN_SUBCHUNK_BYTES). */
TIPS_API int tips_schedule_shape(int64_t count, int p, int dtype, int* depth, int64_t* sub_elems);

/* Chunk partition the ring uses (element offsets), for tests. */
TIPS_API int tips_chunk_bounds(int64_t count, int p, int dtype, int c, int64_t* begin, int64_t* end);


#ifdef __cplusplus
}
#endif
#endif /* TIPS_HIP_H_ */
