// fusion.cc — tensor fusion: many gradients, few allreduces.
//
// The reference issues one MPIAllreduce per gradient, each negotiated through
// rank 0 (tips/tensorflow/__init__.py:212-222, coordinator.cc:355-513). Here a
// list of device tensors is packed into buckets of at most the fusion
// threshold (TIPS_FUSION_THRESHOLD, 64 MiB) by copy_tiles_kernel, each bucket
// is allreduced once, and the sums are unpacked in place. Pack/unpack
// descriptors are built once per distinct tensor list and cached in HBM.
#include <string.h>

#include <algorithm>

#include "rt.h"

namespace tips {
namespace rt {

namespace {

constexpr int64_t kDefaultCopyTile = 8 * 1024;  // tools/fusion_tile_sweep.sh: 8 KiB beat 16-64 KiB

uint64_t plan_key(void* const* ptrs, const int64_t* counts, int n, int dtype) {
  uint64_t h = 1469598103934665603ull ^ (uint64_t)dtype;
  auto mix = [&](uint64_t v) {
    h ^= v;
    h *= 1099511628211ull;
  };
  mix((uint64_t)n);
  for (int i = 0; i < n; i++) {
    mix((uint64_t)(uintptr_t)ptrs[i]);
    mix((uint64_t)counts[i]);
  }
  return h;
}

}  // namespace

void free_plan(FusionPlan& pl) {
  for (auto& b : pl.buckets) {
    if (b.pack) (void)hipFree(b.pack);
    if (b.unpack) (void)hipFree(b.unpack);
  }
  pl.buckets.clear();
}

namespace {

int build_plan(State& st, FusionPlan& pl, int64_t threshold) {
  // pack/unpack work unit (one workgroup each); TIPS_COPY_TILE_BYTES for tuning
  const int64_t tile_bytes = std::min<int64_t>(
      tips::kCopyTileBytes, round_up(std::max<int64_t>(4096, env_i64("TIPS_COPY_TILE_BYTES", kDefaultCopyTile)), 4096));
  const int64_t es = tips::dtype_size(pl.dtype);
  const int n = (int)pl.ptrs.size();
  std::vector<std::vector<CopyTile>> packs(1), unpacks(1);
  std::vector<int64_t> sizes(1, 0);
  for (int i = 0; i < n; i++) {
    const int64_t bytes = pl.counts[i] * es;
    if (bytes == 0) continue;
    if (bytes >= threshold) {  // already bucket-sized: reduce in place
      pl.unfused.push_back(i);
      continue;
    }
    int64_t off = round_up(sizes.back(), kAlignBytes);
    if (off + bytes > threshold) {
      packs.emplace_back();
      unpacks.emplace_back();
      sizes.push_back(0);
      off = 0;
    }
    char* base = (char*)pl.ptrs[i];
    for (int64_t t = 0; t < bytes; t += tile_bytes) {
      const int64_t tb = std::min(tile_bytes, bytes - t);
      // bucket addresses are filled in as offsets; rebased onto the fusion buffer below
      packs.back().push_back(CopyTile{base + t, (char*)(uintptr_t)(off + t), tb});
      unpacks.back().push_back(CopyTile{(const char*)(uintptr_t)(off + t), base + t, tb});
    }
    sizes.back() = off + bytes;
  }
  // two slots: bucket b packs into slot b % 2, so pack(b+1) can run while bucket b is reduced
  for (size_t b = 0; b < sizes.size(); b++) {
    if (sizes[b] == 0) continue;
    FusionBucket fbk;
    char* fb = (char*)st.fusion.p + (int64_t)(pl.buckets.size() % 2) * threshold;
    fbk.buf = fb;
    fbk.bytes = round_up(sizes[b], kAlignBytes);
    fbk.ntiles = (int)packs[b].size();
    for (auto& t : packs[b]) t.dst = fb + (uintptr_t)t.dst;
    for (auto& t : unpacks[b]) t.src = fb + (uintptr_t)t.src;
    const size_t tb = sizeof(CopyTile) * packs[b].size();
    HIP_TRY(hipMalloc(&fbk.pack, tb));
    HIP_TRY(hipMalloc(&fbk.unpack, tb));
    HIP_TRY(hipMemcpy(fbk.pack, packs[b].data(), tb, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(fbk.unpack, unpacks[b].data(), tb, hipMemcpyHostToDevice));
    pl.buckets.push_back(fbk);
  }
  return 0;
}

}  // namespace

int64_t fusion_threshold_bytes() {
  return round_up(std::max<int64_t>(kAlignBytes, env_i64("TIPS_FUSION_THRESHOLD", 64 << 20)), kAlignBytes);
}

// Readiness batching. The tensors differ from cycle to cycle, so no plan is cached:
// descriptors are written to a page-locked slot and copied to HBM on the stream.
// A ring of slots lets the host fill the next one while earlier batches still run.
struct BatchFusion {
  static constexpr int kSlots = 4;
  struct Slot {
    CopyTile* host = nullptr;  // hipHostMalloc
    size_t cap = 0;            // tiles
    DevBuf dev;
    hipEvent_t done = nullptr;  // after the unpack that last read dev
    bool used = false;
  } slot[kSlots];
  int next = 0;
  DevBuf bucket;
};

void batch_release(State& st) {
  BatchFusion* b = st.batch;
  if (!b) return;
  for (auto& sl : b->slot) {
    if (sl.done) (void)hipEventSynchronize(sl.done), (void)hipEventDestroy(sl.done);
    if (sl.host) (void)hipHostFree(sl.host);
    sl.dev.release();
  }
  b->bucket.release();
  delete b;
  st.batch = nullptr;
}

int batch_fused_allreduce(State& st, const BatchItem* items, int n, int dtype, hipStream_t stream) {
  if (!st.batch) st.batch = new BatchFusion();
  BatchFusion& bf = *st.batch;
  const int64_t es = tips::dtype_size(dtype);
  const int64_t tile = kDefaultCopyTile;
  std::vector<CopyTile> tiles;  // pack tiles, then unpack tiles (bucket offsets, rebased below)
  int64_t off = 0;
  for (int i = 0; i < n; i++) {
    const int64_t bytes = items[i].count * es;
    off = round_up(off, kAlignBytes);
    for (int64_t t = 0; t < bytes; t += tile)
      tiles.push_back(CopyTile{(const char*)items[i].in + t, (char*)(uintptr_t)(off + t), std::min(tile, bytes - t)});
    off += bytes;
  }
  const int64_t total = round_up(off, kAlignBytes);
  if (total == 0) return 0;
  if ((size_t)total > bf.bucket.bytes)  // the old bucket is freed: no queued batch may still use it
    for (auto& sl : bf.slot)
      if (sl.used) HIP_TRY(hipEventSynchronize(sl.done));
  TRY(bf.bucket.ensure((size_t)total));  // (padding between tensors is reduced too, never unpacked)
  const size_t npack = tiles.size();
  for (size_t k = 0; k < npack; k++) tiles[k].dst = (char*)bf.bucket.p + (uintptr_t)tiles[k].dst;
  // unpack mirrors pack: bucket -> out
  {
    int64_t o = 0;
    for (int i = 0; i < n; i++) {
      const int64_t bytes = items[i].count * es;
      o = round_up(o, kAlignBytes);
      for (int64_t t = 0; t < bytes; t += tile)
        tiles.push_back(CopyTile{(const char*)bf.bucket.p + o + t, (char*)items[i].out + t, std::min(tile, bytes - t)});
      o += bytes;
    }
  }
  BatchFusion::Slot& sl = bf.slot[bf.next];
  bf.next = (bf.next + 1) % BatchFusion::kSlots;
  if (sl.used) HIP_TRY(hipEventSynchronize(sl.done));  // the kernels that last read this slot are done
  if (tiles.size() > sl.cap) {
    if (sl.host) HIP_TRY(hipHostFree(sl.host));
    sl.host = nullptr;
    sl.cap = 0;
    const size_t cap = std::max<size_t>(tiles.size(), 4096);
    HIP_TRY(hipHostMalloc((void**)&sl.host, cap * sizeof(CopyTile), hipHostMallocDefault));
    sl.cap = cap;
  }
  if (!sl.done) HIP_TRY(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
  const size_t dbytes = tiles.size() * sizeof(CopyTile);
  TRY(sl.dev.ensure(dbytes));
  memcpy(sl.host, tiles.data(), dbytes);
  HIP_TRY(hipMemcpyAsync(sl.dev.p, sl.host, dbytes, hipMemcpyHostToDevice, stream));
  CopyTile* dev = (CopyTile*)sl.dev.p;
  HIP_TRY(tips::launch_copy_tiles(dev, (int)npack, stream));
  TRY(allreduce_device(st, bf.bucket.p, bf.bucket.p, total / es, dtype, stream));
  HIP_TRY(tips::launch_copy_tiles(dev + npack, (int)(tiles.size() - npack), stream));
  HIP_TRY(hipEventRecord(sl.done, stream));
  sl.used = true;
  return 0;
}

}  // namespace rt
}  // namespace tips

using namespace tips::rt;

extern "C" {

int tips_fused_allreduce(void* const* ptrs, const int64_t* counts, int n, int dtype, void* stream) {
  TRY(check_dtype(dtype));
  if (n < 0 || (n > 0 && (!ptrs || !counts))) return fail(TIPS_ERR_INVALID_ARG, "bad tensor list");
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  if (n == 0) return 0;
  TRY(set_device(st));
  for (int i = 0; i < n; i++)
    if (counts[i] < 0 || (counts[i] > 0 && !ptrs[i])) return fail(TIPS_ERR_INVALID_ARG, "bad tensor %d", i);
  hipStream_t s = (hipStream_t)stream;
  const int64_t es = tips::dtype_size(dtype);
  const int64_t threshold = round_up(std::max<int64_t>(kAlignBytes, env_i64("TIPS_FUSION_THRESHOLD", 64 << 20)), kAlignBytes);
  const int64_t tile_env = env_i64("TIPS_COPY_TILE_BYTES", 0);
  if (threshold != st.fusion_threshold || tile_env != st.fusion_tile_env) {  // slots (re)sized: every cached plan points into the old ones
    HIP_TRY(hipDeviceSynchronize());
    for (auto& kv : st.plans) free_plan(kv.second);
    st.plans.clear();
    st.fusion.release();
    TRY(st.fusion.ensure((size_t)(2 * threshold), /*zero=*/true));
    st.fusion_threshold = threshold;
    st.fusion_tile_env = tile_env;
  }
  const uint64_t key = plan_key(ptrs, counts, n, dtype);
  auto it = st.plans.find(key);
  bool hit = it != st.plans.end() && it->second.dtype == dtype && (int)it->second.ptrs.size() == n &&
             std::equal(ptrs, ptrs + n, it->second.ptrs.begin()) && std::equal(counts, counts + n, it->second.counts.begin());
  if (!hit) {
    if (it != st.plans.end() || st.plans.size() >= 64) {  // descriptors may still be read by queued kernels
      HIP_TRY(hipDeviceSynchronize());
      if (it != st.plans.end()) {
        free_plan(it->second);
        st.plans.erase(it);
      }
      if (st.plans.size() >= 64) {
        for (auto& kv : st.plans) free_plan(kv.second);
        st.plans.clear();
      }
    }
    FusionPlan pl;
    pl.dtype = dtype;
    pl.ptrs.assign(ptrs, ptrs + n);
    pl.counts.assign(counts, counts + n);
    int rc = build_plan(st, pl, threshold);
    if (rc) {
      free_plan(pl);
      return rc;
    }
    it = st.plans.emplace(key, std::move(pl)).first;
  }
  const FusionPlan& pl = it->second;
  const int B = (int)pl.buckets.size();
  if (B > 0 && st.size == 1) {  // nothing to overlap with: pack, (no-op) reduce, unpack on the caller's stream
    for (const auto& b : pl.buckets) {
      HIP_TRY(tips::launch_copy_tiles(b.pack, b.ntiles, s));
      TRY(allreduce_device(st, b.buf, b.buf, b.bytes / es, dtype, s));
      HIP_TRY(tips::launch_copy_tiles(b.unpack, b.ntiles, s));
    }
  } else if (B > 0) {
    // fuse stream: pack(0) pack(1) unpack(0) pack(2) unpack(1) ... unpack(B-1)
    // bucket stream: allreduce(b) after pack(b); unpack(b) after allreduce(b); pack(b+2) after unpack(b)
    TRY(st.fuse_ev.ensure(2 * (size_t)B));
    hipEvent_t* packed = st.fuse_ev.ev.data();
    hipEvent_t* reduced = st.fuse_ev.ev.data() + B;
    TRY(join(st.fuse_stream, s, st.ev_start));
    auto pack = [&](int b) -> int {
      HIP_TRY(tips::launch_copy_tiles(pl.buckets[b].pack, pl.buckets[b].ntiles, st.fuse_stream));
      HIP_TRY(hipEventRecord(packed[b], st.fuse_stream));
      return 0;
    };
    TRY(pack(0));
    for (int b = 0; b < B; b++) {
      if (b + 1 < B && b + 1 < 2) TRY(pack(b + 1));  // slot 1 is free from the start
      HIP_TRY(hipStreamWaitEvent(st.bucket_stream, packed[b], 0));
      TRY(allreduce_device(st, pl.buckets[b].buf, pl.buckets[b].buf, pl.buckets[b].bytes / es, dtype, st.bucket_stream));
      HIP_TRY(hipEventRecord(reduced[b], st.bucket_stream));
      HIP_TRY(hipStreamWaitEvent(st.fuse_stream, reduced[b], 0));
      HIP_TRY(tips::launch_copy_tiles(pl.buckets[b].unpack, pl.buckets[b].ntiles, st.fuse_stream));
      if (b + 2 < B) TRY(pack(b + 2));  // reuses slot b % 2, after unpack(b) in stream order
    }
    TRY(join(s, st.fuse_stream, st.ev_done));
  }
  for (int i : pl.unfused) TRY(allreduce_device(st, ptrs[i], ptrs[i], counts[i], dtype, s));
  return 0;
}

}  // extern "C"
