/*
 * tips_hip_dev.h — the development surface of this build: libtips_hip_dev.so (tools/lib/), the same
 * runtime as libtips_hip.so plus the entry points its tests, tuning sweeps and probes call. None of
 * them has a reference counterpart and none is part of the drop-in boundary (include/tips_hip.h,
 * which libtips_hip.so exports alone; tests/test_abi.py checks both export lists).
 *
 * The development library is a second, complete copy of the runtime (its own state, streams and
 * communicator): load it beside the product library only for these calls (Python: tips_amd._lib.dev(),
 * RTLD_LOCAL; it binds its own symbols, -Bsymbolic), never to run a job's collectives.
 */
#ifndef TIPS_HIP_DEV_H_
#define TIPS_HIP_DEV_H_

#include "tips_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Test / diagnostics (no reference counterpart): the segment-copy records fusion.cc builds for
 * one pointer set of a list - the layout of (counts, dtype) and the in -> out addresses given as
 * integers - exactly as the device table of an out-of-place copy call holds them: 4 x int64 per
 * record {src, dst, begin, end}, 2 per tile (in the launch's order) then one per segment. Host only,
 * nothing is uploaded: tests/test_fusion_table.py runs copy_segs_kernel's per-lane rules over them
 * on the CPU. Returns the record count (records may be NULL to ask) or < 0; *ntiles, *tile_bytes. */
TIPS_API int64_t tips_fusion_tile_table(const int64_t* counts, int n, int dtype, const int64_t* ins, const int64_t* outs,
                                       int64_t* records, int64_t cap, int64_t* ntiles, int64_t* tile_bytes);

/* Host-copy pool check (no GPU): `runs` back-to-back fork-join runs of njobs (every third run
 * njobs / 2) on a pool of nthreads; TIPS_OK when every job of every run ran exactly once. For the
 * CPU tests of the pool behind tips_fused_allreduce_host. */
TIPS_API int tips_host_pool_selftest(int nthreads, int runs, int njobs);

/* The negotiation protocol with an executor that only logs (no GPU): each
 * rank enqueues the newline-separated "name dtype count" lines of `requests`
 * ("@batch" ... "@endbatch" commits the lines between as one list, as
 * tips_enqueue_allreduce_n does; "@sleep ms" pauses, "@wait" blocks until every earlier request is
 * decided, "@mark" logs "# mark <microseconds since the call began>"), stops,
 * and writes its execution log ("name OK" / "name ERR message", one per line,
 * in execution order) into out. For tests and the latency tool. */
TIPS_API int tips_negotiation_selftest(int rank, int size, const char* host, int port, const char* requests,
                                       char* out, int64_t cap);

/* The lock-free enqueue against a stop, one rank, no GPU: `threads` threads enqueue callback
 * requests while the caller stops the negotiation after stop_after_us, `rounds` times. result[0..3]:
 * accepted enqueues, callbacks called, requests whose callback count was wrong (an accepted one must
 * be called back exactly once, a refused one never), refusals. TIPS_OK when result[2] is 0. */
TIPS_API int tips_negotiation_stop_race_selftest(int threads, int per_thread, int stop_after_us, int rounds, int port,
                                                 int64_t* result);

/* ---- single-GPU harnesses (tests and benchmarks) ---- */

/* Runs the device ring schedule for p virtual ranks on this one GPU:
 * ins[r] / outs[r] are device buffers of rank r; the peer transfers are
 * device-to-device copies in the same order the RCCL ring issues them, and
 * the sums are the same tips_bucket_sum launches. Lets the ring's chunk
 * arithmetic be checked bit-exact against oracle_ring on one device. */
TIPS_API int tips_ring_simulate(void* const* outs, const void* const* ins, int p, int64_t count, int dtype, void* stream);
/* The same for the one-shot schedule (checked against oracle_fold, wide_acc=1). */
TIPS_API int tips_oneshot_simulate(void* const* outs, const void* const* ins, int p, int64_t count, int dtype,
                                   void* stream);
/* The same for the direct algorithm (checked against oracle_fold, wide_acc=1). */
TIPS_API int tips_direct_simulate(void* const* outs, const void* const* ins, int p, int64_t count, int dtype, void* stream);

/* How the simulators move a virtual rank's bytes to its peer: 0 = device
 * copies (default), 1 = ncclSend/ncclRecv pairs from this rank to itself in
 * one group per pipeline step (exercises the RCCL p2p calls on one GPU;
 * needs a single-rank setup). */
TIPS_API int tips_set_sim_transport(int transport);

/* Explicit variant of the 2-input sum kernel, for the gfx950 tuning sweep
 * (tools/sum_sweep.cc): mode 0 = grid-stride over `blocks` workgroups,
 * mode 1 = one tile per workgroup, mode 2 = the same in XCD-contiguous order,
 * mode 3 = buffer-op forms (nt = cache-policy pair; blocks = bytes of LDS
 * reserved per workgroup, 0-65536, to cap workgroups per CU), mode 4 = LDS-staged
 * through direct-to-LDS loads (unroll 1/2/4, 256 threads), mode 5 = persistent
 * streaming, 256 x unroll workgroups each walking one contiguous range;
 * unroll = 16-B vectors per lane in flight;
 * nt: 0 plain, 1 non-temporal loads+stores, 2 nt loads only, 3 nt stores only;
 * threads = workgroup size. Non-default variants exist for f32 only
 * (others return TIPS_ERR_HIP). tips_bucket_sum uses the default chosen
 * from that sweep. */
TIPS_API int tips_sum_variant(void* dst, const void* a, const void* b, int64_t count, int dtype, int mode, int unroll, int nt,
                     int blocks, int threads, void* stream);

/* Tuning entry for the multi-input sum (tools/sum_sweep.cc): f32 only,
 * nsrc 2, 4 or 8, 16-B aligned pointers. variant 0 = global non-temporal
 * loads, 1 = buffer nt loads 1 vector per lane, 2 = the same with 2 vectors,
 * 3 = buffer plain loads, 4 = buffer nt loads 4 vectors per lane; 8-49 = round 5's sweep of
 * tile order, store policy, lanes, workgroups per CU and grid-stride forms (kernels.hip
 * run_multi_x lists them; tools/multi_sum_sweep.py); 36 = round 4's shipped fold; 50 = what
 * tips_multi_sum launches now. Others: TIPS_ERR_HIP. tips_multi_sum uses the default chosen from
 * those sweeps. */
TIPS_API int tips_multi_sum_variant(void* dst, const void* const* srcs, int nsrc, int64_t count, int dtype, int variant,
                                    void* stream);

/* Tuning entry for the fusion pack / unpack kernel (tools/copy_sweep.py): `tiles` is a device
 * array of ntiles {const char* src; char* dst; int64_t bytes} records (24 B each), every
 * bytes <= max_tile_bytes. variant 0 = the shipped kernel (one tile per workgroup); 1-8 = the
 * grouped kernel (G tiles per workgroup, cache policies: kernels.hip copy_variant_u),
 * max_tile_bytes <= 16384 for those. */
TIPS_API int tips_copy_tiles_variant(const void* tiles, int ntiles, int variant, int64_t max_tile_bytes, void* stream);

/* The peer schedule's transfer kernel on its own (tests, tools/peer_mem_probe.cc):
 * copies bytes[i] from srcs[i] to dsts[i] for n <= 16 segments in one launch,
 * any alignment; pointers may be IPC-mapped peer memory. */
TIPS_API int tips_xfer(void* const* dsts, const void* const* srcs, const int64_t* bytes, int n, void* stream);

/* The op plan rank `rank` of `p` issues for an allreduce of `count` elements with
 * schedule `algo` (TIPS_ALGO_RING / DIRECT / ONESHOT) and `depth` sub-chunks per
 * chunk (<= 0: the runtime's choice). The RCCL executor and the single-GPU
 * simulators run exactly these plans (tips_amd/csrc/plan.cc); this dump is for
 * host-side checks (pairing, stream hazards, a CPU interpreter). Pure host
 * function. Writes the plan as int64 words into out[0..cap) when it fits and
 * returns the number of words (< 0 = error). Layout:
 *   {nsteps, staging_bytes, K}, then per step {wait_sum, nxfer, nsum},
 *   nxfer x {send, peer, buf, byte_off, bytes}, nsum x {dst_buf, dst_off, count,
 *   nsrc, nsrc x {buf, byte_off}}; buf 0 = in, 1 = out, 2 = staging. */
TIPS_API int64_t tips_schedule_plan(int algo, int p, int rank, int64_t count, int dtype, int depth, int64_t* out,
                                    int64_t cap);

/* The candidates TIPS_ALGO_TUNE would time for a bucket of `count` elements on p ranks, in the order
 * it runs them (schedule, pipeline depth, lanes; TIPS_TUNE_LANES / TIPS_TUNE_PEER read as at a call).
 * Pure host function: fills up to cap entries and returns the number of candidates (< 0 = error).
 * tests/test_plans.py checks that a chunk of 16 MiB or more is never offered unpipelined. */
TIPS_API int tips_tune_candidates(int p, int64_t count, int dtype, int* algos, int* depths, int* lanes, int cap);

#ifdef __cplusplus
}
#endif
#endif /* TIPS_HIP_DEV_H_ */
