// fusion.cc — tensor fusion: many gradients, few allreduces.
//
// The reference issues one MPIAllreduce per gradient, each negotiated through
// rank 0 (tips/tensorflow/__init__.py:212-222, coordinator.cc:355-513). Here a
// list of device tensors is packed into buckets of at most the fusion
// threshold (TIPS_FUSION_THRESHOLD, 64 MiB) by copy_tiles_kernel, each bucket
// is allreduced once, and the sums are unpacked into the outputs (in place or
// not). One path serves tips_fused_allreduce (in place), tips_fused_allreduce_oop
// and the negotiated path's readiness batches (negotiate.cc).
//
// Streams: every device operation of a call runs on the two fusion streams
// (pack / unpack on fuse_stream, bucket allreduces on bucket_stream), joined with
// the caller's stream at entry and exit. Calls from different caller streams are
// therefore ordered through fuse_stream and can never write a shared bucket slot
// concurrently. Descriptor tables ({src, dst, bytes} per 8 KiB tile) are built on
// the host once per distinct tensor list and cached in HBM; a new list uploads
// its table on fuse_stream, and an evicted table is freed stream-ordered behind
// its last use. Nothing here synchronises the device.
#include <string.h>

#include <algorithm>

#include "rt.h"

namespace tips {
namespace rt {

namespace {

constexpr int64_t kDefaultCopyTile = 8 * 1024;  // tools/fusion_tile_sweep.sh: 8 KiB beat 16-64 KiB
constexpr size_t kMaxEntries = 32;             // cached tensor lists
constexpr int kUploadSlots = 4;                // page-locked staging of descriptor uploads

int64_t copy_tile_bytes() {
  return std::min<int64_t>(tips::kCopyTileBytes,
                           round_up(std::max<int64_t>(4096, env_i64("TIPS_COPY_TILE_BYTES", kDefaultCopyTile)), 4096));
}

struct Bucket {
  int64_t bytes;       // padded size reduced
  char* buf;           // its fusion slot (bucket b uses slot b % 2)
  int64_t pack0, npack;  // tiles [pack0, pack0 + npack) pack, the same count after unpack0 unpack
  int64_t unpack0;
};

struct Entry {
  uint64_t key = 0;
  bool identity = false;  // one rank: only the out-of-place copies (dev[0..ntiles)), no buckets
  int dtype = 0;
  int64_t tile = 0;
  std::vector<const void*> ins;
  std::vector<void*> outs;
  std::vector<int64_t> counts;
  std::vector<Bucket> buckets;
  std::vector<BatchItem> direct;  // tensors of at least the threshold, reduced where they lie (build_entry)
  CopyTile* dev = nullptr;   // descriptor table in HBM
  size_t ntiles = 0;
  uint64_t stamp = 0;        // last use (LRU)
};

uint64_t key_of(const BatchItem* items, int n, int dtype, int64_t tile) {
  uint64_t h = 1469598103934665603ull ^ (uint64_t)dtype;
  auto mix = [&](uint64_t v) {
    h ^= v;
    h *= 1099511628211ull;
  };
  mix((uint64_t)n);
  mix((uint64_t)tile);
  for (int i = 0; i < n; i++) {
    mix((uint64_t)(uintptr_t)items[i].in);
    mix((uint64_t)(uintptr_t)items[i].out);
    mix((uint64_t)items[i].count);
  }
  return h;
}

bool same_list(const Entry& e, const BatchItem* items, int n, int dtype, int64_t tile) {
  if (e.dtype != dtype || e.tile != tile || (int)e.counts.size() != n) return false;
  for (int i = 0; i < n; i++)
    if (e.ins[i] != items[i].in || e.outs[i] != items[i].out || e.counts[i] != items[i].count) return false;
  return true;
}

}  // namespace

struct FusionCache {
  std::vector<Entry*> entries;
  uint64_t clock = 0;
  struct Upload {
    CopyTile* host = nullptr;  // hipHostMalloc
    size_t cap = 0;            // tiles
    hipEvent_t done = nullptr;  // after the copy that last read it
    bool used = false;
  } up[kUploadSlots];
  int next_up = 0;
};

namespace {

void free_entry(State& st, Entry* e) {
  if (e->dev) (void)hipFreeAsync(e->dev, st.fuse_stream);  // behind its last use on fuse_stream
  delete e;
}

// Build a tensor list's buckets and descriptors; upload the table on fuse_stream.
//
// The layout is a function of the element counts, the dtype and the threshold alone - never of
// where the tensors lie - because every rank must issue the same allreduces over the same bucket
// offsets: a tensor of at least the threshold is reduced where it lies (its own allreduce, only
// its own bytes touched); every other tensor is packed into the current bucket at a 256-B aligned
// offset. (An earlier version reduced tensors that happened to lie back to back in memory as one
// run; an allocator that placed them so on one rank and not on another would have paired
// different elements across ranks. A flat buffer is reduced without copies by allreducing the
// buffer itself: DistributedOptimizer does that with its gradient bucket views.)
int build_entry(State& st, FusionCache& fc, Entry* e, const BatchItem* items, int n, int64_t threshold) {
  const int64_t es = tips::dtype_size(e->dtype), tile = e->tile;
  std::vector<CopyTile> pack, unpack;
  std::vector<int64_t> sizes;  // per bucket
  std::vector<int64_t> first;  // per bucket: first tile index into pack / unpack
  // Balanced buckets: B = the fewest buckets of at most `threshold` that hold the packed bytes,
  // at least 2 once there are 32 MiB (so pack(1) overlaps the exchange of bucket 0), filled up to
  // total / B each instead of greedily to the threshold. A greedy split of config 4 leaves a
  // 15 MiB tail bucket (a launch that small ramps up and drains at 4.3 TB/s) and exposes a
  // full 64 MiB pack before the first exchange.
  int64_t target = threshold;
  if (!e->identity) {
    int64_t packed = 0;  // upper bound of the packed bytes: every tensor below the threshold
    for (int i = 0; i < n; i++) {
      const int64_t b = items[i].count * es;
      if (b < threshold) packed += round_up(b, kAlignBytes);
    }
    int64_t nb = (packed + threshold - 1) / threshold;
    if (nb < 2 && packed >= (32 << 20) && env_i64("TIPS_FUSION_BALANCE", 1)) nb = 2;
    if (nb > 1 && env_i64("TIPS_FUSION_BALANCE", 1)) target = std::min(threshold, round_up((packed + nb - 1) / nb, kAlignBytes));
  }
  auto place = [&](const char* in, char* out, int64_t bytes) {
    if (e->identity) {  // one rank: in place nothing, out of place a copy
      for (int64_t t = 0; in != out && t < bytes; t += tile)
        pack.push_back(CopyTile{in + t, out + t, std::min(tile, bytes - t)});
      return;
    }
    if (bytes >= threshold) {
      e->direct.push_back(BatchItem{in, out, bytes / es});
      return;
    }
    int64_t off = sizes.empty() ? 0 : round_up(sizes.back(), kAlignBytes);
    // a new bucket when this one would pass the threshold, or has reached its balanced share
    if (sizes.empty() || off + bytes > threshold || off >= target) {
      sizes.push_back(0);
      first.push_back((int64_t)pack.size());
      off = 0;
    }
    char* slot = (char*)st.fusion.p + (int64_t)((sizes.size() - 1) % 2) * threshold;
    for (int64_t t = 0; t < bytes; t += tile) {
      const int64_t tb = std::min(tile, bytes - t);
      pack.push_back(CopyTile{in + t, slot + off + t, tb});
      unpack.push_back(CopyTile{slot + off + t, out + t, tb});
    }
    sizes.back() = off + bytes;
  };
  for (int i = 0; i < n; i++) {
    const int64_t bytes = items[i].count * es;
    if (bytes > 0) place((const char*)items[i].in, (char*)items[i].out, bytes);
  }
  const int64_t npack = (int64_t)pack.size();
  for (size_t b = 0; b < sizes.size(); b++) {
    const int64_t end = b + 1 < sizes.size() ? first[b + 1] : npack;
    e->buckets.push_back(Bucket{round_up(sizes[b], kAlignBytes), (char*)st.fusion.p + (int64_t)(b % 2) * threshold,
                                first[b], end - first[b], npack + first[b]});
  }
  e->ntiles = pack.size() + unpack.size();
  if (e->ntiles == 0) return 0;
  const size_t bytes = e->ntiles * sizeof(CopyTile);
  HIP_TRY(hipMallocAsync((void**)&e->dev, bytes, st.fuse_stream));
  FusionCache::Upload& u = fc.up[fc.next_up];
  fc.next_up = (fc.next_up + 1) % kUploadSlots;
  if (u.used) HIP_TRY(hipEventSynchronize(u.done));  // the copy that last read this slot has run
  if (u.cap < e->ntiles) {
    if (u.host) HIP_TRY(hipHostFree(u.host));
    u.host = nullptr;
    u.cap = 0;
    const size_t cap = std::max<size_t>(e->ntiles, 16384);
    HIP_TRY(hipHostMalloc((void**)&u.host, cap * sizeof(CopyTile), hipHostMallocDefault));
    u.cap = cap;
  }
  if (!u.done) HIP_TRY(hipEventCreateWithFlags(&u.done, hipEventDisableTiming));
  memcpy(u.host, pack.data(), pack.size() * sizeof(CopyTile));
  memcpy(u.host + pack.size(), unpack.data(), unpack.size() * sizeof(CopyTile));
  HIP_TRY(hipMemcpyAsync(e->dev, u.host, bytes, hipMemcpyHostToDevice, st.fuse_stream));
  HIP_TRY(hipEventRecord(u.done, st.fuse_stream));
  u.used = true;
  return 0;
}

// The fusion slots: two buckets of `threshold` bytes, zeroed once (padding between packed
// tensors is reduced too, never unpacked). A new threshold drops every cached table (they
// hold addresses in the old slots), after the fusion streams have finished with them.
int ensure_slots(State& st, FusionCache& fc, int64_t threshold) {
  if (threshold == st.fusion_threshold && st.fusion.p) return 0;
  HIP_TRY(hipStreamSynchronize(st.fuse_stream));
  HIP_TRY(hipStreamSynchronize(st.bucket_stream));
  for (Entry* e : fc.entries) free_entry(st, e);
  fc.entries.clear();
  HIP_TRY(hipStreamSynchronize(st.fuse_stream));
  st.fusion.release();
  TRY(st.fusion.ensure((size_t)(2 * threshold), /*zero=*/true));
  st.fusion_threshold = threshold;
  return 0;
}

}  // namespace

int64_t fusion_threshold_bytes() {
  return round_up(std::max<int64_t>(kAlignBytes, env_i64("TIPS_FUSION_THRESHOLD", 64 << 20)), kAlignBytes);
}

void fusion_release(State& st) {
  FusionCache* fc = st.fusion_cache;
  if (!fc) return;
  for (Entry* e : fc->entries) free_entry(st, e);
  if (st.fuse_stream) (void)hipStreamSynchronize(st.fuse_stream);
  for (auto& u : fc->up) {
    if (u.done) (void)hipEventSynchronize(u.done), (void)hipEventDestroy(u.done);
    if (u.host) (void)hipHostFree(u.host);
  }
  delete fc;
  st.fusion_cache = nullptr;
}

int fused_allreduce(State& st, const BatchItem* items, int n, int dtype, hipStream_t user) {
  if (n <= 0) return 0;
  if (!st.fusion_cache) st.fusion_cache = new FusionCache();
  FusionCache& fc = *st.fusion_cache;
  const int64_t threshold = fusion_threshold_bytes(), tile = copy_tile_bytes();
  const int64_t es = tips::dtype_size(dtype);
  TRY(ensure_slots(st, fc, threshold));
  // One rank: the allreduce of anything is the identity (as allreduce_device's), so a tensor
  // reduced in place needs no work and one out of place a copy - no bucket. TIPS_FUSION_MEASURE_PACK=1
  // keeps the buckets anyway, to measure on one GPU what packing costs a step at N > 1.
  const bool identity = st.size == 1 && !env_i64("TIPS_FUSION_MEASURE_PACK", 0);
  const uint64_t key = key_of(items, n, dtype, tile) ^ (identity ? 0x9e3779b97f4a7c15ull : 0);
  Entry* e = nullptr;
  for (Entry* c : fc.entries)
    if (c->key == key && c->identity == identity && same_list(*c, items, n, dtype, tile)) {
      e = c;
      break;
    }
  if (e && identity && e->ntiles == 0) {  // every tensor in place: nothing to do
    e->stamp = ++fc.clock;
    return 0;
  }
  TRY(join(st.fuse_stream, user, st.ev_start));  // inputs ready (the bucket stream waits for it too)
  if (st.size > 1) HIP_TRY(hipStreamWaitEvent(st.bucket_stream, st.ev_start, 0));
  if (!e) {
    if (fc.entries.size() >= kMaxEntries) {  // evict the least recently used list
      auto lru = std::min_element(fc.entries.begin(), fc.entries.end(),
                                  [](const Entry* a, const Entry* b) { return a->stamp < b->stamp; });
      free_entry(st, *lru);
      fc.entries.erase(lru);
    }
    e = new Entry();
    e->key = key;
    e->identity = identity;
    e->dtype = dtype;
    e->tile = tile;
    for (int i = 0; i < n; i++) {
      e->ins.push_back(items[i].in);
      e->outs.push_back(items[i].out);
      e->counts.push_back(items[i].count);
    }
    const int rc = build_entry(st, fc, e, items, n, threshold);
    if (rc) {
      free_entry(st, e);
      return rc;
    }
    fc.entries.push_back(e);
  }
  e->stamp = ++fc.clock;

  const int B = (int)e->buckets.size();
  auto pack = [&](int b) -> int {
    HIP_TRY(tips::launch_pack_tiles(e->dev + e->buckets[b].pack0, (int)e->buckets[b].npack, e->tile, st.fuse_stream));
    return 0;
  };
  auto unpack = [&](int b) -> int {
    HIP_TRY(tips::launch_pack_tiles(e->dev + e->buckets[b].unpack0, (int)e->buckets[b].npack, e->tile, st.fuse_stream));
    return 0;
  };
  if (identity) {  // one rank: the out-of-place tensors' copies, one launch
    if (e->ntiles) HIP_TRY(tips::launch_pack_tiles(e->dev, (int)e->ntiles, e->tile, st.fuse_stream));
    TRY(join(user, st.fuse_stream, st.ev_done));
    return 0;
  }
  if (st.size == 1) {  // TIPS_FUSION_MEASURE_PACK: pack, (identity), unpack, in stream order
    for (int b = 0; b < B; b++) {
      TRY(pack(b));
      TRY(unpack(b));
    }
    for (const BatchItem& d : e->direct) TRY(allreduce_device(st, d.in, d.out, d.count, dtype, st.fuse_stream));
    TRY(join(user, st.fuse_stream, st.ev_done));
    return 0;
  } else {
    // bucket stream: the direct tensors first (nothing to pack: their exchange starts at once and
    //                overlaps pack(0)), then allreduce(b) after pack(b)
    // fuse stream:   pack(0) pack(1) | unpack(0) pack(2) | unpack(1) pack(3) | ... unpack(B-1);
    //                unpack(b) after allreduce(b); pack(b+2) reuses slot b % 2 after unpack(b)
    for (const BatchItem& d : e->direct) TRY(allreduce_device(st, d.in, d.out, d.count, dtype, st.bucket_stream));
    TRY(st.fuse_ev.ensure(2 * (size_t)B));
    hipEvent_t* packed = st.fuse_ev.ev.data();
    hipEvent_t* reduced = st.fuse_ev.ev.data() + B;
    for (int b = 0; b < std::min(B, 2); b++) {
      TRY(pack(b));
      HIP_TRY(hipEventRecord(packed[b], st.fuse_stream));
    }
    for (int b = 0; b < B; b++) {
      HIP_TRY(hipStreamWaitEvent(st.bucket_stream, packed[b], 0));
      TRY(allreduce_device(st, e->buckets[b].buf, e->buckets[b].buf, e->buckets[b].bytes / es, dtype, st.bucket_stream));
      HIP_TRY(hipEventRecord(reduced[b], st.bucket_stream));
      HIP_TRY(hipStreamWaitEvent(st.fuse_stream, reduced[b], 0));
      TRY(unpack(b));
      if (b + 2 < B) {
        TRY(pack(b + 2));
        HIP_TRY(hipEventRecord(packed[b + 2], st.fuse_stream));
      }
    }
  }
  TRY(join(user, st.fuse_stream, st.ev_done));
  TRY(join(user, st.bucket_stream, st.ev_comp_done));
  return 0;
}

}  // namespace rt
}  // namespace tips

using namespace tips::rt;

namespace {

int fused_entry(const void* const* ins, void* const* outs, const int64_t* counts, int n, int dtype, void* stream) {
  TRY(check_dtype(dtype));
  if (n < 0 || (n > 0 && (!ins || !outs || !counts))) return fail(TIPS_ERR_INVALID_ARG, "bad tensor list");
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  if (n == 0) return 0;
  TRY(set_device(st));
  std::vector<BatchItem> items((size_t)n);
  for (int i = 0; i < n; i++) {
    if (counts[i] < 0 || (counts[i] > 0 && (!ins[i] || !outs[i]))) return fail(TIPS_ERR_INVALID_ARG, "bad tensor %d", i);
    items[i] = BatchItem{ins[i], outs[i], counts[i]};
  }
  return fused_allreduce(st, items.data(), n, dtype, (hipStream_t)stream);
}

}  // namespace

extern "C" {

int tips_fused_allreduce(void* const* ptrs, const int64_t* counts, int n, int dtype, void* stream) {
  return fused_entry((const void* const*)ptrs, ptrs, counts, n, dtype, stream);
}

int tips_fused_allreduce_oop(const void* const* ins, void* const* outs, const int64_t* counts, int n, int dtype,
                             void* stream) {
  return fused_entry(ins, outs, counts, n, dtype, stream);
}

}  // extern "C"
