// kernels.h — launchers for the gfx950 kernels of the bucket-reduction path.
// Internal to libtips_hip.so (not part of the C-ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace tips {

int dtype_size(int dtype);  // 0 for unknown dtypes

// dst = a + b, elementwise (the per-chunk MPI_SUM step).
hipError_t launch_sum2(void* dst, const void* a, const void* b, int64_t n, int dtype, hipStream_t s);

// dst = rank-order fold of srcs[0..nsrc), nsrc <= kMaxSrcs.
constexpr int kMaxSrcs = 16;
hipError_t launch_multi_sum(void* dst, const void* const* srcs, int nsrc, int64_t n, int dtype, hipStream_t s);
// The same fold when most sources are peers' memory read over xGMI (the peer schedule's pull-fold,
// peer.cc): remote loads take microseconds, so every lane keeps 4 x 16 B per source in flight
// (256 lanes, 16 KiB per source per workgroup, no occupancy cap). Same bits as launch_multi_sum.
hipError_t launch_multi_sum_remote(void* dst, const void* const* srcs, int nsrc, int64_t n, int dtype, hipStream_t s);

// Batched byte copy for fusion pack/unpack: one workgroup per tile.
struct CopyTile {
  const char* src;
  char* dst;
  int64_t bytes;  // <= kCopyTileBytes
};
constexpr int64_t kCopyTileBytes = 64 * 1024;
hipError_t launch_copy_tiles(const CopyTile* tiles_dev, int ntiles, hipStream_t s);
// The fusion pack / unpack launcher: copy_tiles_g_kernel, one tile of <= 16 KiB per workgroup
// held in registers (nt loads, sc1 stores, 16-B vectors + bytewise tail): 0-9 % faster than
// copy_tiles_kernel on the configs' tensor lists (tools/copy_sweep.py); larger tiles fall back.
hipError_t launch_pack_tiles(const CopyTile* tiles_dev, int ntiles, int64_t max_tile_bytes, hipStream_t s);
// Tuning sweep (tools/copy_sweep.py): 0 = the shipped kernel; 1-8 = copy_tiles_g_kernel with G
// tiles per workgroup and load / store cache policies (kernels.hip); tiles of at most
// max_tile_bytes (<= 16 KiB for variants 1-8).
hipError_t launch_copy_tiles_variant(const CopyTile* tiles_dev, int ntiles, int variant, int64_t max_tile_bytes,
                                     hipStream_t s);

// Segment copy over a virtual byte space (fusion pack / unpack / identity copy, fusion.cc): tensor
// k occupies virtual bytes [begin, end) and byte v of it lives at src + v on the source side and
// dst + v on the destination side. Tiles of tile_bytes (4, 8 or 16 KiB) are cut from the virtual
// space; tiles[2t], tiles[2t + 1] (two per tile of the whole space) are the records of the one or
// two segments tile t meets (the second {0,0,0,0} when one), or {first segment, number of segments,
// -, -1} when it meets more (then read from segs[]).
// Segments begin 256-B aligned and in order. One launch copies tiles [tile0, tile0 + ntiles).
// pol = store cache policy: 0 plain, 1 nt, 2 sc1.
struct CopySeg {
  int64_t src, dst;  // addresses of virtual byte 0 (as integers: src + v = the byte's address)
  int64_t begin, end;
};
hipError_t launch_copy_segs(const CopySeg* tiles, const CopySeg* segs, int tile0, int ntiles, int64_t tile_bytes,
                            int pol, hipStream_t s);
// The pack launch's workgroup -> slot map: 1 MiB-style XCD stripes of this many 16-B vectors
// (TIPS_PACK_STRIPE_KIB; 0, the default, = one contiguous eighth of the slots per XCD), and the
// XCD / issue position of every slot under it (fusion.cc's tile_order places boundary tiles by it).
int64_t pack_stripe_vecs();
void stripe_slots(int64_t nslots, int64_t C, std::vector<int>* xcd, std::vector<int64_t>* pos);

// Several tile groups (a step's fusion buckets) in one launch: group k copies record slots
// [tile0[k], tile0[k] + ntiles[k]) with workgroups [blk0[k], blk0[k + 1]) (the launcher fills blk0).
// done[k] != null: when group k is complete its last workgroup stores sig_value[k] into *done[k]
// (signal memory: another stream waits for it with hipStreamWaitValue64); counters[k] (device
// memory, zero before the first launch) count the group's workgroups and are left at zero.
constexpr int kMaxPackGroups = 8;
struct PackGroups {
  int n;
  int tile0[kMaxPackGroups], ntiles[kMaxPackGroups];
  unsigned blk0[kMaxPackGroups + 1];
  unsigned* counters;
  unsigned long long* done[kMaxPackGroups];
  unsigned long long sig_value[kMaxPackGroups];
};
hipError_t launch_copy_segs_groups(const CopySeg* tiles, const CopySeg* segs, PackGroups g, int64_t tile_bytes, int pol,
                                   hipStream_t s);

// The segment copy with a cast (fused Compression.fp16): the byte space is the wire type's (wire =
// f16 or bf16 dtype code); the f32 side of a segment is at its record's address + 2 v. dir 0: pack
// (f32 -> wire, round to nearest even), dir 1: unpack (wire -> f32). And one contiguous range cast.
hipError_t launch_cast_segs(const CopySeg* tiles, const CopySeg* segs, int tile0, int ntiles, int64_t tile_bytes,
                            int dir, int wire, hipStream_t s);
hipError_t launch_cast_range(void* dst, const void* src, int64_t n, int dir, int wire, hipStream_t s);

// One contiguous device-to-device copy of `bytes` (tips_allreduce / tips_broadcast at one rank, out
// of place): copy_buf_kernel when both pointers are 16-B aligned, else hipMemcpyAsync.
hipError_t launch_copy_buf(void* dst, const void* src, int64_t bytes, hipStream_t s);

// Peer transfers of the xGMI peer schedule (peer.cc): up to kMaxXferSegs byte
// segments {src, dst, bytes} copied by one launch, segments interleaved over
// the workgroups so every xGMI link carries traffic at once. src/dst may be
// IPC-mapped peer memory. Passed by value (kernel argument), no descriptor upload.
struct XferSeg {
  const char* src;
  char* dst;
  int64_t bytes;
};
constexpr int kMaxXferSegs = 16;
constexpr int64_t kXferTileBytes = 16 * 1024;  // per workgroup: 256 lanes x 4 x 16 B
hipError_t launch_xfer(const XferSeg* segs, int nseg, hipStream_t s);

// Tuning/sweep entry for the multi-input sum (f32, nsrc 2/4/8); variants in kernels.hip.
hipError_t launch_multi_sum_variant(void* dst, const void* const* srcs, int nsrc, int64_t n, int dtype, int variant,
                                   hipStream_t s);

// Tuning/sweep entry: explicit variant of the 2-input sum.
//   mode 0 = grid-stride over (blocks) workgroups, mode 1 = one tile per workgroup
//   unroll = 16-B vectors per lane in flight, nt: 0 plain, 1 non-temporal loads+stores,
//   2 nt loads only, 3 nt stores only; threads = workgroup size. Non-default variants are f32 only.
//   mode 3 = buffer-op forms (nt = cache-policy pair index), mode 4 = LDS-staged through gfx950's
//   direct-to-LDS loads (unroll 1, 2 or 4; 256 threads), mode 5 = persistent streaming (unroll =
//   workgroups per CU: 1, 2, 4 or 8).
hipError_t launch_sum2_variant(void* dst, const void* a, const void* b, int64_t n, int dtype, int mode, int unroll,
                               int nt, int blocks, int threads, hipStream_t s);

}  // namespace tips
