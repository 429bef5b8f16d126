// fusion.cc — tensor fusion: many gradients, few allreduces.
//
// The reference issues one MPIAllreduce per gradient, each negotiated through
// rank 0 (tips/tensorflow/__init__.py:212-222, coordinator.cc:355-513). Here a
// list of tensors is laid out in buckets of at most the fusion threshold
// (TIPS_FUSION_THRESHOLD, 64 MiB), each bucket is allreduced once, and the sums
// land in the outputs. Three forms share one layout:
//   - tips_fused_allreduce (in place) / _oop: pack -> bucket slot -> allreduce -> unpack;
//   - tips_fused_allreduce_flat: pack straight into one flat output buffer laid out as the
//     buckets, allreduce each bucket there in place (no slot, no unpack: 2 x the bytes of HBM
//     traffic instead of 4 x) - what allreduce_grads returns views of;
//   - the negotiated path's readiness batches (negotiate.cc) use the first form.
//
// Layouts are a function of (dtype, counts, threshold, tile) alone, never of where the tensors
// lie: every rank must issue the same allreduces over the same bucket offsets, and a training
// loop hands over fresh gradient tensors every step. A layout is built once (bucket cut, a
// 256-B aligned byte offset per tensor in one "flat" byte space, the segments each tile of that
// space meets). Per call only the pointers change: they are resolved on the host into one
// {src, dst, begin, end} record per tensor and two per tile (the tile's one or two segments, or
// where its segments start: copy_segs_kernel reads them with one scalar load before its first
// data load) and uploaded
// through a page-locked ring - unless this layout saw the same pointer set recently
// (LRU of 16 per layout), in which case nothing is uploaded. tips_fusion_stats counts both caches.
//
// Streams: a call's pack / unpack launches and table uploads run on the CALLER's stream (the
// "work stream"; TIPS_FUSION_CALLER_STREAM=0: on the library's fuse_stream, joined with the caller
// both ways as rounds 1-3 did), its bucket allreduces at N > 1 on bucket_stream, forked from and
// joined back to the work stream. The slots and tables are shared by every call, so the calls form
// one chain: each records an event at its end on its work stream, and a call from another stream
// first waits for it (fusion_enter / fusion_leave). A step from one stream then crosses no queue
// at all at one rank (the two joins per call cost ~25 us of cross-queue latency per step: config 4
// eager 87 us vs 62 us replayed as one graph, profiles/r03/r_bench_fused1000.jsonl). Nothing here
// synchronises the device.
#include <string.h>

#include <algorithm>

#include "rt.h"

namespace tips {
namespace rt {

namespace {

constexpr int64_t kDefaultCopyTile = 8 * 1024;  // tools/copy_sweep_balanced.py: 8 KiB beat 4 / 16 KiB
constexpr size_t kMaxLayouts = 32;
constexpr size_t kMaxTables = 16;  // pointer sets per layout
constexpr int kUploadSlots = 4;    // page-locked staging of table uploads

int64_t copy_tile_bytes() {
  const int64_t t = env_i64("TIPS_COPY_TILE_BYTES", kDefaultCopyTile);
  return t <= 4096 ? 4096 : t <= 8192 ? 8192 : 16384;
}

// the fused cast's tile (wire bytes; TIPS_CAST_TILE_BYTES): 4 KiB, against the copy's 8 KiB. A
// cast launch moves 3 wire bytes per wire byte of tile, so at the copy's tile config 4's 20 MB
// buckets were 2,500 workgroups (1.2 x what the chip holds at once) and the round trip took
// 49.7 us; at 4 KiB, 46.1 us (profiles/r06/cast/sweep_cast_tile_*.jsonl)
int64_t cast_tile_bytes() {
  const int64_t t = env_i64("TIPS_CAST_TILE_BYTES", 4096);
  return t <= 4096 ? 4096 : t <= 8192 ? 8192 : 16384;
}

// store cache policy of the segment copy: 2 = sc1 (default: the line leaves the XCD's L2, as the
// sum kernels' stores), 1 = nt, 0 = plain (TIPS_COPY_STORE_POLICY, the tuning sweep's knob)
int copy_store_policy() { return (int)std::min<int64_t>(2, std::max<int64_t>(0, env_i64("TIPS_COPY_STORE_POLICY", 2))); }

enum Mode { kSlot = 0, kCopy = 1, kFlat = 2, kSlotCast = 3 };  // kSlotCast: kSlot with f32 tensors, wire-type slots
inline int tables_of(int mode) { return mode == kSlot || mode == kSlotCast ? 2 : 1; }

struct Bucket {
  int64_t off;    // byte offset in the flat space (tile-aligned, so no tile straddles two buckets)
  int64_t bytes;  // padded size reduced (a multiple of 256)
  int tile0, ntiles;
};

struct Table {  // resolved segment records of one pointer set
  uint64_t hash = 0;
  int mode = 0;
  std::vector<const void*> ins;
  std::vector<void*> outs;
  const void* base = nullptr;  // the flat output (kFlat) or the slot base (kSlot)
  CopySeg* dev = nullptr;      // kSlot: [pack | unpack], else one table; nseg records each
  uint64_t stamp = 0;
  // a call captured into a graph read this table: a replay may read it at any later time, so it is
  // never refilled, reused or freed (until tips_shutdown), its layout is never evicted, and the
  // slots it packs into outlive a threshold change (State::fusion_retired)
  bool pinned = false;
};

}  // namespace

struct Layout {
  uint64_t key = 0;
  int dtype = 0;
  int64_t tile = 0, threshold = 0;
  bool balance = true;
  std::vector<int64_t> counts;
  std::vector<int64_t> off;     // per tensor: byte offset in the flat space (-1: empty tensor)
  std::vector<int> bucket;      // per tensor: its bucket, -1 = reduced where it lies (>= threshold) or empty
  std::vector<Bucket> buckets;
  std::vector<int> direct;      // tensors of at least the threshold, list order
  std::vector<int> seg_tensor;  // segment k -> tensor (segments in flat order; empty tensors have none)
  std::vector<int> tiles;       // per tile of the flat space: {first segment meeting it, how many}
  int64_t flat_bytes = 0;
  int ntiles = 0;
  std::vector<Table*> tables;
  uint64_t stamp = 0;
  bool pinned() const {
    for (const Table* t : tables)
      if (t->pinned) return true;
    return false;
  }
};

// Bucket cut and offsets: a pure function of (dtype, counts, threshold, tile, balance).
// Balanced buckets: B = the fewest buckets of at most `threshold` that hold the packed bytes, at
// least 2 once there are 32 MiB (so pack(1) overlaps the exchange of bucket 0), filled up to
// total / B each instead of greedily to the threshold (a greedy split of config 4 leaves a 15 MiB
// tail bucket, a launch that small ramps up and drains at 4.3 TB/s). A tensor of at least the
// threshold gets a region of its own after the buckets and is reduced where it lies.
void build_layout(Layout* L, const int64_t* counts, int n) {
  const int64_t es = tips::dtype_size(L->dtype), threshold = L->threshold, tile = L->tile;
  L->counts.assign(counts, counts + n);
  L->off.assign(n, -1);
  L->bucket.assign(n, -1);
  int64_t packed = 0;
  for (int i = 0; i < n; i++) {
    const int64_t b = counts[i] * es;
    if (b > 0 && b < threshold) packed += round_up(b, kAlignBytes);
  }
  int64_t target = threshold;
  int64_t nb = (packed + threshold - 1) / threshold;
  if (nb < 2 && packed >= (32 << 20) && L->balance) nb = 2;
  if (nb > 1 && L->balance) target = std::min(threshold, round_up((packed + nb - 1) / nb, kAlignBytes));
  int64_t cur = 0;  // bytes placed in the current bucket
  for (int i = 0; i < n; i++) {
    const int64_t bytes = counts[i] * es;
    if (bytes <= 0) continue;
    if (bytes >= threshold) {
      L->direct.push_back(i);
      continue;
    }
    int64_t o = round_up(cur, kAlignBytes);
    if (L->buckets.empty() || o + bytes > threshold || o >= target) {  // a new bucket
      L->buckets.push_back(Bucket{0, 0, 0, 0});
      o = 0;
    }
    L->bucket[i] = (int)L->buckets.size() - 1;
    L->off[i] = o;  // bucket-relative for now
    cur = o + bytes;
    L->buckets.back().bytes = round_up(cur, kAlignBytes);
  }
  int64_t f = 0;
  for (Bucket& b : L->buckets) {
    b.off = f;
    b.tile0 = (int)(f / tile);
    b.ntiles = (int)((b.bytes + tile - 1) / tile);
    f = round_up(f + b.bytes, tile);
  }
  for (int i = 0; i < n; i++)
    if (L->bucket[i] >= 0) L->off[i] += L->buckets[L->bucket[i]].off;
  for (int i : L->direct) {
    L->off[i] = f;
    f = round_up(f + counts[i] * es, kAlignBytes);
  }
  L->flat_bytes = f;
  L->ntiles = (int)((f + tile - 1) / tile);
  // segments in flat order: the buckets' tensors (list order within each bucket, buckets in order
  // = list order), then the direct tensors
  for (int i = 0; i < n; i++)
    if (L->bucket[i] >= 0) L->seg_tensor.push_back(i);
  for (int i : L->direct) L->seg_tensor.push_back(i);
  // tile t meets segments [first, first + count): first = the first ending past the tile's start,
  // and every one after it that begins before the tile's end (at most tile / 256 + 1: segments
  // begin 256-B aligned)
  const int nseg = (int)L->seg_tensor.size();
  L->tiles.assign(2 * (size_t)L->ntiles, 0);
  int k = 0, e = 0;
  for (int t = 0; t < L->ntiles; t++) {
    const int64_t start = (int64_t)t * tile, stop = start + tile;
    while (k < nseg && L->off[L->seg_tensor[k]] + counts[L->seg_tensor[k]] * es <= start) k++;
    e = std::max(e, k);
    while (e < nseg && L->off[L->seg_tensor[e]] < stop) e++;
    L->tiles[2 * t] = k;
    L->tiles[2 * t + 1] = e - k;
  }
}

struct FusionCache {
  std::vector<Layout*> layouts;
  uint64_t clock = 0;
  struct Upload {
    void* host = nullptr;  // hipHostMalloc
    size_t cap = 0;        // bytes
    hipEvent_t done = nullptr;  // after the copy that last read it
    bool used = false;
  } up[kUploadSlots];
  int next_up = 0;
  int64_t layouts_built = 0, layout_hits = 0, tables_built = 0, table_hits = 0;
};

namespace {

// the chain's event, recorded now if the last call left it unrecorded (see fusion_leave)
int chain_event(State& st) {
  if (st.fuse_chain_lazy) {
    HIP_TRY(hipEventRecord(st.ev_fuse_chain, st.fuse_chain_stream));
    st.fuse_chain_lazy = false;
  }
  return 0;
}

// Table memory (hipMallocAsync, the uploads, hipFreeAsync) lives on the library's fuse_stream, behind
// every earlier fused call (the chain's event): a table freed or refilled there was last read by an
// earlier call. A call that built a table waits for the upload on its work stream (find_table).
// Only cache misses touch fuse_stream, so a call that finds its table crosses no queue.
hipStream_t table_stream(State& st) {
  if (st.fuse_chain_valid && chain_event(st) == 0) (void)hipStreamWaitEvent(st.fuse_stream, st.ev_fuse_chain, 0);
  return st.fuse_stream;
}

void free_table(State& st, Table* t) {
  if (t->dev) (void)hipFreeAsync(t->dev, table_stream(st));  // behind its last use: the chain
  delete t;
}

void free_layout(State& st, Layout* L) {
  for (Table* t : L->tables) free_table(st, t);
  delete L;
}

// Host -> device on the work stream through a page-locked slot (the pageable path would block).
// A slot is reused once the copy that last read it has run; with 4 slots that wait is rare.
int upload(State& st, FusionCache& fc, void* dev, const void* src, size_t bytes) {
  FusionCache::Upload& u = fc.up[fc.next_up];
  fc.next_up = (fc.next_up + 1) % kUploadSlots;
  if (u.used) HIP_TRY(hipEventSynchronize(u.done));
  if (u.cap < bytes) {
    if (u.host) HIP_TRY(hipHostFree(u.host));
    u.host = nullptr;
    u.cap = 0;
    const size_t cap = std::max<size_t>(bytes, 256 << 10);
    HIP_TRY(hipHostMalloc(&u.host, cap, hipHostMallocDefault));
    u.cap = cap;
  }
  if (!u.done) HIP_TRY(hipEventCreateWithFlags(&u.done, hipEventDisableTiming));
  memcpy(u.host, src, bytes);
  const hipStream_t ws = table_stream(st);
  HIP_TRY(hipMemcpyAsync(dev, u.host, bytes, hipMemcpyHostToDevice, ws));
  HIP_TRY(hipEventRecord(u.done, ws));
  u.used = true;
  return 0;
}

uint64_t fnv(uint64_t h, uint64_t v) { return (h ^ v) * 1099511628211ull; }

Layout* find_layout(State& st, FusionCache& fc, const int64_t* counts, int n, int dtype, int64_t threshold,
                    int64_t tile, bool balance) {
  uint64_t h = fnv(fnv(fnv(fnv(1469598103934665603ull, (uint64_t)dtype), (uint64_t)threshold), (uint64_t)tile),
                   (uint64_t)balance);
  h = fnv(h, (uint64_t)n);
  for (int i = 0; i < n; i++) h = fnv(h, (uint64_t)counts[i]);
  for (Layout* L : fc.layouts)
    if (L->key == h && L->dtype == dtype && L->threshold == threshold && L->tile == tile && L->balance == balance &&
        (int)L->counts.size() == n && std::equal(L->counts.begin(), L->counts.end(), counts)) {
      L->stamp = ++fc.clock;
      fc.layout_hits++;
      return L;
    }
  if (fc.layouts.size() >= kMaxLayouts) {  // evict the least recently used layout no captured graph uses
    auto lru = fc.layouts.end();
    for (auto it = fc.layouts.begin(); it != fc.layouts.end(); ++it)
      if (!(*it)->pinned() && (lru == fc.layouts.end() || (*it)->stamp < (*lru)->stamp)) lru = it;
    if (lru != fc.layouts.end()) {
      free_layout(st, *lru);
      fc.layouts.erase(lru);
    }
  }
  Layout* L = new Layout();
  L->key = h;
  L->dtype = dtype;
  L->threshold = threshold;
  L->tile = tile;
  L->balance = balance;
  build_layout(L, counts, n);
  L->stamp = ++fc.clock;
  fc.layouts.push_back(L);
  fc.layouts_built++;
  return L;
}

// The resolved segment table(s) of this call's pointers: a cached one when this layout saw the
// same pointers (and mode and base) recently, else built on the host and uploaded.
// The order a launch's workgroups take a group's tiles in (a group: one bucket, or the region of
// tensors reduced where they lie; launches cover whole groups). The tiles that meet a tensor
// boundary (two or more segments, or a segment that does not cover the tile) are the slow ones.
// TIPS_COPY_ORDER=2 (default): each XCD's range of slots gets an equal share of them, first; config
// 4's pack 14.0 against 14.5-14.7 us per bucket launch (profiles/r04/zzl_pack_order_ab.txt).
// 1: all of them first (they then land on the first XCDs); 0: tile order.
std::vector<int> tile_order(const Layout& L) {
  std::vector<int> order(L.ntiles);
  for (int j = 0; j < L.ntiles; j++) order[j] = j;
  const int64_t mode = env_i64("TIPS_COPY_ORDER", 2);
  if (mode == 0) return order;
  const int64_t es = tips::dtype_size(L.dtype);
  auto covered = [&](int j) {
    if (L.tiles[2 * j + 1] != 1) return false;
    const int i = L.seg_tensor[L.tiles[2 * j]];
    return L.off[i] <= (int64_t)j * L.tile && L.off[i] + L.counts[i] * es >= (int64_t)(j + 1) * L.tile;
  };
  std::vector<int> bounds;
  for (const Bucket& b : L.buckets) bounds.push_back(b.tile0);
  bounds.push_back(L.buckets.empty() ? 0 : L.buckets.back().tile0 + L.buckets.back().ntiles);
  bounds.push_back(L.ntiles);
  const bool spread = mode == 2;
  for (size_t g = 0; g + 1 < bounds.size(); g++) {
    const int g0 = bounds[g], g1 = std::min(bounds[g + 1], L.ntiles);
    if (g1 <= g0) continue;
    auto mid = std::stable_partition(order.begin() + g0, order.begin() + g1, [&](int j) { return !covered(j); });
    if (!spread) continue;
    // TIPS_COPY_ORDER=2: the launch deals slot s to XCD s / R (R = grid / 8, xcd_tile in
    // kernels.hip), so "boundary tiles first" puts them all on the first XCDs. Instead each XCD's
    // range gets an equal share of them, first in the range, then interior tiles.
    const int n = g1 - g0, R = (int)(std::max<int64_t>(8, ((int64_t)n + 7) / 8 * 8) / 8);
    std::vector<int> slow(order.begin() + g0, mid), fast(mid, order.begin() + g1);
    const int64_t C = tips::pack_stripe_vecs() * 16 / std::max<int64_t>(1, L.tile);
    if (C > 0 && (int64_t)n > 8 * C) {
      // Striped launch (TIPS_PACK_STRIPE_KIB): XCD x issues its slots in stripe order. Each XCD's
      // first-issued slots get an equal share of the boundary tiles; the interior tiles keep
      // address order over the slots left, so every stripe still streams one run of the bucket.
      std::vector<int> sx;
      std::vector<int64_t> sp;
      tips::stripe_slots(n, C, &sx, &sp);
      std::vector<std::vector<int>> by(8);
      for (int t = 0; t < n; t++) by[sx[t]].push_back(t);
      for (auto& v : by) std::stable_sort(v.begin(), v.end(), [&](int a, int b) { return sp[a] < sp[b]; });
      std::vector<char> taken(n, 0);
      size_t si = 0;
      for (int x = 0; x < 8 && si < slow.size(); x++) {
        const size_t share = std::min(by[x].size(), (slow.size() - si + (7 - x)) / (8 - x));
        for (size_t k = 0; k < share; k++) order[g0 + by[x][k]] = slow[si++], taken[by[x][k]] = 1;
      }
      size_t fi = 0;
      for (int t = 0; t < n; t++) {
        if (taken[t]) continue;
        order[g0 + t] = si < slow.size() ? slow[si++] : fast[fi++];
      }
      continue;
    }
    std::vector<std::vector<int>> xcd(8);
    size_t si = 0, fi = 0;
    for (int x = 0; x < 8; x++) {
      const int cap = std::max(0, std::min(R, n - x * R));
      const size_t share = std::min<size_t>((size_t)cap, (slow.size() - si + (7 - x)) / (8 - x));
      for (size_t k = 0; k < share; k++) xcd[x].push_back(slow[si++]);
    }
    for (int x = 0; x < 8; x++) {  // (slow tiles a full range could not take go to later ranges)
      const int cap = std::max(0, std::min(R, n - x * R));
      while ((int)xcd[x].size() < cap && si < slow.size()) xcd[x].push_back(slow[si++]);
      while ((int)xcd[x].size() < cap && fi < fast.size()) xcd[x].push_back(fast[fi++]);
    }
    int at = g0;
    for (int x = 0; x < 8; x++)
      for (int j : xcd[x]) order[at++] = j;
  }
  return order;
}

// One table's records for a pointer set: [2 per tile | one per segment] (twice for kSlot: pack,
// then unpack). Host only: find_table uploads them; tips_fusion_tile_table returns them to the CPU
// tests' interpreter of copy_segs_kernel.
void fill_records(const Layout& L, int mode, const BatchItem* items, const void* base, std::vector<CopySeg>* dst) {
  const int nseg = (int)L.seg_tensor.size();
  const int ntab = tables_of(mode);
  const size_t per = 2 * (size_t)L.ntiles + nseg;
  const int64_t es = tips::dtype_size(L.dtype);
  std::vector<CopySeg>& rec = *dst;
  rec.assign(ntab * per, CopySeg{0, 0, 0, 0});
  for (int k = 0; k < nseg; k++) {
    const int i = L.seg_tensor[k];
    const int64_t b = L.off[i], e = b + L.counts[i] * es;
    const int64_t in = (int64_t)(uintptr_t)items[i].in - b, out = (int64_t)(uintptr_t)items[i].out - b;
    CopySeg* r = rec.data() + 2 * L.ntiles + k;
    if (mode == kSlot || mode == kSlotCast) {
      const int bk = L.bucket[i];
      // bucket bk lives in slot bk % 2: virtual byte v of it at slot + (v - bucket offset)
      const int64_t slot = bk < 0 ? 0 : (int64_t)(uintptr_t)base + (int64_t)(bk % 2) * L.threshold - L.buckets[bk].off;
      // kSlotCast: the tensors are f32 and the space the wire type's, so the f32 side of virtual
      // byte v is at base + 2 v (cast_segs_kernel)
      const int64_t win = (int64_t)(uintptr_t)items[i].in - 2 * b, wout = (int64_t)(uintptr_t)items[i].out - 2 * b;
      r[0] = mode == kSlot ? CopySeg{in, slot, b, e} : CopySeg{win, slot, b, e};       // pack
      r[per] = mode == kSlot ? CopySeg{slot, out, b, e} : CopySeg{slot, wout, b, e};   // unpack
    } else if (mode == kCopy) {
      r[0] = CopySeg{in, out, b, e};
    } else {  // kFlat: straight into the flat output
      r[0] = CopySeg{in, (int64_t)(uintptr_t)base, b, e};
    }
  }
  // tile records (two per tile): the segment itself when the tile meets one, both when it meets
  // two (a tensor's end and the next one's start), else where its segments start. Record slot q
  // holds tile order[q]; the tile's byte offset travels in the second record (its begin when that
  // record is unused; when it is the second segment, that segment begins in the tile, so the
  // kernel rounds its begin down to the tile).
  const std::vector<int> order = tile_order(L);
  for (int tb = 0; tb < ntab; tb++) {
    CopySeg* T = rec.data() + tb * per;
    const CopySeg* S = T + 2 * L.ntiles;
    for (int q = 0; q < L.ntiles; q++) {
      const int j = order[q];
      const int first = L.tiles[2 * j], cnt = L.tiles[2 * j + 1];
      T[2 * q] = cnt <= 2 ? S[first] : CopySeg{first, cnt, 0, -1};
      T[2 * q + 1] = cnt == 2 ? S[first + 1] : CopySeg{0, 0, (int64_t)j * L.tile, 0};
    }
  }
}

Table* find_table(State& st, FusionCache& fc, Layout& L, int mode, const BatchItem* items, int n,
                  const void* base) {
  uint64_t h = fnv(fnv(1469598103934665603ull, (uint64_t)mode), (uint64_t)(uintptr_t)base);
  for (int i = 0; i < n; i++) h = fnv(fnv(h, (uint64_t)(uintptr_t)items[i].in), (uint64_t)(uintptr_t)items[i].out);
  for (Table* t : L.tables) {
    if (t->hash != h || t->mode != mode || t->base != base) continue;
    bool same = true;
    for (int i = 0; i < n && same; i++) same = t->ins[i] == items[i].in && t->outs[i] == items[i].out;
    if (same) {
      t->stamp = ++fc.clock;
      fc.table_hits++;
      if (st.fuse_capturing) t->pinned = true;  // the graph's replays read it from now on
      return t;
    }
  }
  if (st.fuse_capturing) {  // (before any table is touched: nothing may be refilled under capture)
    fail(TIPS_ERR_INVALID_ARG, "fusion: a fused call under stream capture must find its pointer table built: make "
                               "the same call once before the capture");
    return nullptr;
  }
  Table* t = nullptr;
  size_t unpinned = 0;
  for (const Table* u : L.tables) unpinned += !u->pinned;
  if (unpinned >= kMaxTables) {  // reuse the least recently used unpinned table's device buffer (stream
    auto lru = L.tables.end();    // order keeps its earlier readers first); pinned ones are never touched
    for (auto it = L.tables.begin(); it != L.tables.end(); ++it)
      if (!(*it)->pinned && (lru == L.tables.end() || (*it)->stamp < (*lru)->stamp)) lru = it;
    if ((*lru)->mode == mode) {
      t = *lru;
    } else {
      free_table(st, *lru);
      L.tables.erase(lru);
    }
  }
  const int nseg = (int)L.seg_tensor.size();
  const int ntab = tables_of(mode);
  const size_t per = 2 * (size_t)L.ntiles + nseg;  // one table: [2 records per tile | segment records]
  if (!t) {
    t = new Table();
    if (hipMallocAsync((void**)&t->dev, ntab * per * sizeof(CopySeg), table_stream(st)) != hipSuccess) {
      delete t;
      fail(TIPS_ERR_HIP, "fusion: hipMallocAsync of a segment table failed");
      return nullptr;
    }
    L.tables.push_back(t);
  }
  t->hash = h;
  t->mode = mode;
  t->base = base;
  t->ins.resize(n);
  t->outs.resize(n);
  for (int i = 0; i < n; i++) {
    t->ins[i] = items[i].in;
    t->outs[i] = items[i].out;
  }
  std::vector<CopySeg> rec;
  fill_records(L, mode, items, base, &rec);
  t->stamp = ++fc.clock;
  fc.tables_built++;
  if (upload(st, fc, t->dev, rec.data(), rec.size() * sizeof(CopySeg)) != 0 ||
      (st.fuse_in_call && join(st.fuse_ws, st.fuse_stream, st.ev_fuse_table) != 0)) {  // the launches after it
    t->hash = 0;  // (a failed upload must never be matched)
    t->ins.clear();
    return nullptr;
  }
  return t;
}

// The fusion slots: two buckets of `threshold` bytes (padding between packed tensors is reduced
// too, never unpacked). A new threshold drops every cached table (they hold slot addresses),
// after the fusion streams have finished with them.
int ensure_slots(State& st, FusionCache& fc, int64_t threshold) {
  if (threshold == st.fusion_threshold && st.fusion.p) return 0;
  bool pinned = false;  // a captured graph's replays pack into the current slots: they must stay
  for (const Layout* L : fc.layouts) pinned = pinned || L->pinned();
  if (st.fuse_chain_valid) {
    TRY(chain_event(st));
    HIP_TRY(hipEventSynchronize(st.ev_fuse_chain));
  }
  HIP_TRY(hipStreamSynchronize(st.fuse_stream));
  HIP_TRY(hipStreamSynchronize(st.bucket_stream));
  for (Layout* L : fc.layouts) {  // pinned tables keep the old slots' addresses and stay valid
    std::vector<Table*> keep;
    for (Table* t : L->tables) {
      if (t->pinned) keep.push_back(t);
      else free_table(st, t);
    }
    L->tables.swap(keep);
  }
  HIP_TRY(hipStreamSynchronize(st.fuse_stream));
  if (pinned && st.fusion.p) {  // retired, not freed: freed at tips_shutdown (fusion_release)
    st.fusion_retired.push_back(st.fusion.p);
    st.fusion.p = nullptr;
    st.fusion.bytes = 0;
  }
  st.fusion.release();
  TRY(st.fusion.ensure((size_t)(2 * threshold), /*zero=*/true));
  st.fusion_threshold = threshold;
  return 0;
}

FusionCache& cache(State& st) {
  if (!st.fusion_cache) st.fusion_cache = new FusionCache();
  return *st.fusion_cache;
}

int copy_tiles(const Layout& L, const Table& t, int table, int tile0, int ntiles, hipStream_t s) {
  const CopySeg* base = t.dev + (size_t)table * (2 * (size_t)L.ntiles + L.seg_tensor.size());
  HIP_TRY(tips::launch_copy_segs(base, base + 2 * L.ntiles, tile0, ntiles, L.tile, copy_store_policy(), s));
  return 0;
}

// One pack launch for a step's buckets: TIPS_PACK_MERGE=1, opt-in. The idea was
// that each launch pays ~1.7 us of ramp and drain, so a step of two ~41-51 MB buckets
// paid it twice. Measured (profiles/r06/pack_merged.jsonl): back-to-back launches on one stream do not
// pay it - config 4's two packs take 28.56 us merged against 2 x 14.11 us, config 5's 33.14 against
// 2 x 16.56 - so per-bucket launches stay the default; the merged form (bit-exact, with device-side
// per-bucket completion signals) is kept for the N = 8 node to A/B.
bool pack_merge(const State& st) { return !st.fuse_capturing && env_i64("TIPS_PACK_MERGE", 0) != 0; }

// Whether the bucket stream can wait on the device for one bucket of a merged pack launch
// (hipStreamWaitValue64 on signal memory, raised by the bucket's last workgroup); sets up the
// counters and the signal words once. Without it a merged launch is waited for as a whole.
bool pack_signals_ready(State& st, hipStream_t ws) {
  if (st.pack_signals >= 0) return st.pack_signals == 1;
  st.pack_signals = 0;
  if (env_i64("TIPS_PACK_SIGNALS", 1) == 0) return false;
  int can = 0;
  if (hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, st.device) != hipSuccess || !can) {
    (void)hipGetLastError();
    return false;
  }
  bool ok = hipMalloc((void**)&st.pack_counters, tips::kMaxPackGroups * sizeof(unsigned)) == hipSuccess &&
            hipMemsetAsync(st.pack_counters, 0, tips::kMaxPackGroups * sizeof(unsigned), ws) == hipSuccess;
  for (int k = 0; k < tips::kMaxPackGroups && ok; k++) {
    ok = hipExtMallocWithFlags(&st.pack_done[k], sizeof(uint64_t), hipMallocSignalMemory) == hipSuccess &&
         hipMemsetAsync(st.pack_done[k], 0, sizeof(uint64_t), ws) == hipSuccess;
    st.pack_done_value[k] = 0;
  }
  if (!ok) {
    (void)hipGetLastError();
    pack_signals_release(st);
    return false;
  }
  st.pack_signals = 1;
  return true;
}

// Buckets [b0, b0 + nb) of table `table` in one launch, nb <= kMaxPackGroups, in bucket order.
// signal: bucket b0 + k's completion raises signal word k to values[k] (wait_packed).
int pack_buckets(State& st, const Layout& L, const Table& t, int table, int b0, int nb, bool signal, uint64_t* values,
                 hipStream_t s) {
  tips::PackGroups g{};
  g.n = nb;
  g.counters = signal ? st.pack_counters : nullptr;
  for (int k = 0; k < nb; k++) {
    g.tile0[k] = L.buckets[b0 + k].tile0;
    g.ntiles[k] = L.buckets[b0 + k].ntiles;
    if (signal) {
      g.done[k] = static_cast<unsigned long long*>(st.pack_done[k]);
      g.sig_value[k] = st.pack_done_value[k] + 1;
    }
  }
  const CopySeg* base = t.dev + (size_t)table * (2 * (size_t)L.ntiles + L.seg_tensor.size());
  HIP_TRY(tips::launch_copy_segs_groups(base, base + 2 * L.ntiles, g, L.tile, copy_store_policy(), s));
  if (signal)
    for (int k = 0; k < nb; k++) values[k] = ++st.pack_done_value[k];
  return 0;
}

// The bucket stream waits until signal word k has reached value (its bucket is packed).
int wait_packed(State& st, int k, uint64_t value) {
  HIP_TRY(hipStreamWaitValue64(st.bucket_stream, st.pack_done[k], value, hipStreamWaitValueGte, ~0ull));
  return 0;
}

// A fused call's entry: the work stream (the caller's, or fuse_stream under
// TIPS_FUSION_CALLER_STREAM=0) after the chain's previous call and after the caller's own work.
// A call captured into a graph (torch.cuda.graph around it) stays out of the chain: the capture
// may not wait for an event recorded outside it, and an event recorded inside it is a graph node,
// not a point later calls could wait for; the graph's replays are ordered by the stream they are
// launched on. Such a call must find its tables built (the same call made once before the
// capture, as CUDA-graph users warm up), since uploading them would be captured too.
int fusion_enter(State& st, hipStream_t user, hipStream_t* ws) {
  if (!st.ev_fuse_chain) HIP_TRY(hipEventCreateWithFlags(&st.ev_fuse_chain, hipEventDisableTiming));
  *ws = env_i64("TIPS_FUSION_CALLER_STREAM", 1) != 0 ? user : st.fuse_stream;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(user, &cs) != hipSuccess) {
    (void)hipGetLastError();
    cs = hipStreamCaptureStatusNone;
  }
  st.fuse_capturing = cs != hipStreamCaptureStatusNone;
  if (!st.fuse_capturing && st.fuse_chain_valid && st.fuse_chain_stream != *ws) {
    TRY(chain_event(st));
    HIP_TRY(hipStreamWaitEvent(*ws, st.ev_fuse_chain, 0));
  }
  if (*ws != user) TRY(join(*ws, user, st.ev_start));
  st.fuse_ws = *ws;
  st.fuse_in_call = true;
  return 0;
}

// ... and its exit: the caller after the work stream, the chain's event at the end of the call.
// lazy (tips_fused_pack_bucket, a measurement entry whose launches are timed back to back): the
// event is recorded only when a later call needs it - a call from another stream, a table freed
// behind the chain, new slots - on the stream this call used, which must then still exist.
int fusion_leave(State& st, hipStream_t user, bool lazy = false) {
  const hipStream_t ws = st.fuse_ws;
  st.fuse_ws = nullptr;
  st.fuse_in_call = false;
  if (ws != user) TRY(join(user, ws, st.ev_done));
  if (st.fuse_capturing) {
    st.fuse_capturing = false;
    return 0;
  }
  st.fuse_chain_stream = ws;
  st.fuse_chain_valid = true;
  st.fuse_chain_lazy = lazy && ws == user;
  if (!st.fuse_chain_lazy) HIP_TRY(hipEventRecord(st.ev_fuse_chain, ws));
  return 0;
}

// fusion_enter ... fusion_leave around `body(ws)`; the exit runs on failure too (the chain's event
// then covers whatever the body queued)
template <typename F>
int in_fusion(State& st, hipStream_t user, F body, bool lazy = false) {
  hipStream_t ws = nullptr;
  TRY(fusion_enter(st, user, &ws));
  const int rc = body(ws);
  const int rc2 = fusion_leave(st, user, lazy);
  return rc ? rc : rc2;
}

}  // namespace

int64_t fusion_threshold_bytes() {
  return round_up(std::max<int64_t>(kAlignBytes, env_i64("TIPS_FUSION_THRESHOLD", 64 << 20)), kAlignBytes);
}

void pack_signals_release(State& st) {
  if (st.pack_counters) (void)hipFree(st.pack_counters);
  st.pack_counters = nullptr;
  for (void*& p : st.pack_done) {
    if (p) (void)hipFree(p);
    p = nullptr;
  }
  st.pack_signals = -1;
}

void fusion_release(State& st) {
  FusionCache* fc = st.fusion_cache;
  if (st.ev_fuse_chain) {
    // a lazy chain end (tips_fused_pack_bucket) is not recorded here: its stream may be gone by
    // shutdown; the device synchronize covers what it would have waited for
    if (st.fuse_chain_valid && st.fuse_chain_lazy) {
      (void)hipDeviceSynchronize();
      st.fuse_chain_lazy = false;
      st.fuse_chain_valid = false;
    }
    if (st.fuse_chain_valid && chain_event(st) == 0) (void)hipEventSynchronize(st.ev_fuse_chain);
    (void)hipEventDestroy(st.ev_fuse_chain);
    st.ev_fuse_chain = nullptr;
    st.fuse_chain_valid = false;
  }
  if (st.pack_counters || st.pack_signals == 1) {  // (no launch may still raise them)
    (void)hipDeviceSynchronize();
    pack_signals_release(st);
  }
  st.pack_signals = -1;
  if (!fc) return;
  for (Layout* L : fc->layouts) free_layout(st, L);
  if (st.fuse_stream) (void)hipStreamSynchronize(st.fuse_stream);
  for (void* q : st.fusion_retired) (void)hipFree(q);
  st.fusion_retired.clear();
  for (auto& u : fc->up) {
    if (u.done) (void)hipEventSynchronize(u.done), (void)hipEventDestroy(u.done);
    if (u.host) (void)hipHostFree(u.host);
  }
  delete fc;
  st.fusion_cache = nullptr;
}

int fusion_stats(State& st, int64_t* v) {
  FusionCache& fc = cache(st);
  v[0] = fc.layouts_built;
  v[1] = fc.layout_hits;
  v[2] = fc.tables_built;
  v[3] = fc.table_hits;
  return 0;
}

// The layout's byte offsets, for callers that allocate the flat output (tips_fused_layout).
int64_t fused_layout(const int64_t* counts, int n, int dtype, int64_t* offsets) {
  Layout L;
  L.dtype = dtype;
  L.threshold = fusion_threshold_bytes();
  L.tile = copy_tile_bytes();
  L.balance = env_i64("TIPS_FUSION_BALANCE", 1) != 0;
  build_layout(&L, counts, n);
  if (offsets)
    for (int i = 0; i < n; i++) offsets[i] = L.off[i] < 0 ? 0 : L.off[i];
  return L.flat_bytes;
}

int fused_allreduce(State& st, const BatchItem* items, int n, int dtype, hipStream_t user) {
  if (n <= 0) return 0;
  FusionCache& fc = cache(st);
  const int64_t threshold = fusion_threshold_bytes();
  TRY(ensure_slots(st, fc, threshold));
  // One rank: the allreduce of anything is the identity (as allreduce_device's), so a list reduced
  // in place needs no work and one out of place one copy launch - no bucket. TIPS_FUSION_MEASURE_PACK=1
  // keeps the buckets anyway, to measure on one GPU what packing costs a step at N > 1.
  const bool identity = st.size == 1 && !env_i64("TIPS_FUSION_MEASURE_PACK", 0);
  bool in_place = true;
  for (int i = 0; i < n && in_place; i++) in_place = items[i].in == items[i].out || items[i].count == 0;
  if (identity && in_place) return 0;
  std::vector<int64_t> counts((size_t)n);
  for (int i = 0; i < n; i++) counts[i] = items[i].count;
  return in_fusion(st, user, [&](hipStream_t ws) -> int {
    if (st.size > 1) {  // inputs ready for the bucket stream too (the direct tensors start at once)
      HIP_TRY(hipEventRecord(st.ev_start, ws));
      HIP_TRY(hipStreamWaitEvent(st.bucket_stream, st.ev_start, 0));
    }
    Layout* L = find_layout(st, fc, counts.data(), n, dtype, threshold, copy_tile_bytes(),
                            env_i64("TIPS_FUSION_BALANCE", 1) != 0);
    if (!L) return TIPS_ERR_HIP;
    if (L->seg_tensor.empty()) return 0;
    const int64_t es = tips::dtype_size(dtype);
    if (identity) {  // one rank, out of place: every tensor copied in -> out, one launch over the whole space
      Table* t = find_table(st, fc, *L, kCopy, items, n, nullptr);
      if (!t) return TIPS_ERR_HIP;
      return copy_tiles(*L, *t, 0, 0, L->ntiles, ws);
    }
    const int B = (int)L->buckets.size();
    Table* t = B ? find_table(st, fc, *L, kSlot, items, n, st.fusion.p) : nullptr;
    if (B && !t) return TIPS_ERR_HIP;
    auto pack = [&](int b) { return copy_tiles(*L, *t, 0, L->buckets[b].tile0, L->buckets[b].ntiles, ws); };
    auto unpack = [&](int b) { return copy_tiles(*L, *t, 1, L->buckets[b].tile0, L->buckets[b].ntiles, ws); };
    auto slot = [&](int b) { return (char*)st.fusion.p + (int64_t)(b % 2) * threshold; };
    // pack(0) and pack(1) (both slots) go first: one launch when merged, bucket 0's tiles first
    const int first = std::min(B, 2);
    const bool merge = first > 1 && pack_merge(st);
    if (st.size == 1) {  // TIPS_FUSION_MEASURE_PACK: the N > 1 step's launches, the allreduces left out
      if (merge) TRY(pack_buckets(st, *L, *t, 0, 0, first, false, nullptr, ws));
      else
        for (int b = 0; b < first; b++) TRY(pack(b));
      for (int b = 0; b < B; b++) {
        TRY(unpack(b));
        if (b + 2 < B) TRY(pack(b + 2));
      }
      for (int i : L->direct) TRY(allreduce_device(st, items[i].in, items[i].out, items[i].count, dtype, ws));
      return 0;
    }
    // bucket stream: the direct tensors first (nothing to pack: their exchange starts at once and
    //                overlaps pack(0)), then allreduce(b) after pack(b)
    // work stream:   pack(0) pack(1) | unpack(0) pack(2) | unpack(1) pack(3) | ... unpack(B-1);
    //                unpack(b) after allreduce(b); pack(b+2) reuses slot b % 2 after unpack(b)
    for (int i : L->direct) TRY(allreduce_device(st, items[i].in, items[i].out, items[i].count, dtype, st.bucket_stream));
    TRY(st.fuse_ev.ensure(2 * (size_t)B));
    hipEvent_t* packed = st.fuse_ev.ev.data();
    hipEvent_t* reduced = st.fuse_ev.ev.data() + B;
    // merged: the bucket stream waits for each bucket's signal word (or, without signals, for the
    // whole launch)
    const bool signal = merge && pack_signals_ready(st, ws);
    uint64_t sigv[2] = {};
    if (merge) {
      TRY(pack_buckets(st, *L, *t, 0, 0, first, signal, sigv, ws));
      HIP_TRY(hipEventRecord(packed[0], ws));  // (read when !signal: the launch as a whole)
    } else {
      for (int b = 0; b < first; b++) {
        TRY(pack(b));
        HIP_TRY(hipEventRecord(packed[b], ws));
      }
    }
    for (int b = 0; b < B; b++) {
      if (signal && b < first) TRY(wait_packed(st, b, sigv[b]));
      else HIP_TRY(hipStreamWaitEvent(st.bucket_stream, packed[merge && b < first ? 0 : b], 0));
      TRY(allreduce_device(st, slot(b), slot(b), L->buckets[b].bytes / es, dtype, st.bucket_stream));
      HIP_TRY(hipEventRecord(reduced[b], st.bucket_stream));
      HIP_TRY(hipStreamWaitEvent(ws, reduced[b], 0));
      TRY(unpack(b));
      if (b + 2 < B) {
        TRY(pack(b + 2));
        HIP_TRY(hipEventRecord(packed[b + 2], ws));
      }
    }
    return join(ws, st.bucket_stream, st.ev_comp_done);  // (the direct tensors' allreduces too)
  });
}

// flat = SUM over ranks of the inputs, tensor i at its layout offset: pack(b) straight into the
// flat buffer's bucket b, allreduce it there in place. Every bucket has its own region, so all
// packs go ahead on fuse_stream and allreduce(b) only waits for pack(b).
int fused_allreduce_flat(State& st, const BatchItem* items, int n, int dtype, void* flat, hipStream_t user) {
  if (n <= 0) return 0;
  FusionCache& fc = cache(st);
  const int64_t threshold = fusion_threshold_bytes();
  std::vector<int64_t> counts((size_t)n);
  for (int i = 0; i < n; i++) counts[i] = items[i].count;
  return in_fusion(st, user, [&](hipStream_t ws) -> int {
    if (st.size > 1) {
      HIP_TRY(hipEventRecord(st.ev_start, ws));
      HIP_TRY(hipStreamWaitEvent(st.bucket_stream, st.ev_start, 0));
    }
    Layout* L = find_layout(st, fc, counts.data(), n, dtype, threshold, copy_tile_bytes(),
                            env_i64("TIPS_FUSION_BALANCE", 1) != 0);
    if (!L) return TIPS_ERR_HIP;
    if (L->seg_tensor.empty()) return 0;
    Table* t = find_table(st, fc, *L, kFlat, items, n, flat);
    if (!t) return TIPS_ERR_HIP;
    const int64_t es = tips::dtype_size(dtype);
    const bool measure = st.size == 1 && env_i64("TIPS_FUSION_MEASURE_PACK", 0);
    if (st.size == 1 && !measure)  // one rank: the identity - every tensor copied into place, one launch
      return copy_tiles(*L, *t, 0, 0, L->ntiles, ws);
    const int B = (int)L->buckets.size();
    hipStream_t red = st.size > 1 ? st.bucket_stream : ws;
    for (int i : L->direct)
      TRY(allreduce_device(st, items[i].in, (char*)flat + L->off[i], items[i].count, dtype, red));
    TRY(st.fuse_ev.ensure((size_t)B));
    // merged: every bucket's pack in launches of up to kMaxPackGroups buckets, bucket order, each
    // bucket's allreduce behind its signal word (or, without signals, behind its launch)
    const bool merge = B > 1 && pack_merge(st);
    const bool signal = merge && st.size > 1 && pack_signals_ready(st, ws);
    for (int b0 = 0; b0 < B;) {
      const int nb = merge ? std::min(B - b0, tips::kMaxPackGroups) : 1;
      uint64_t sigv[tips::kMaxPackGroups] = {};
      if (merge) TRY(pack_buckets(st, *L, *t, 0, b0, nb, signal, sigv, ws));
      else TRY(copy_tiles(*L, *t, 0, L->buckets[b0].tile0, L->buckets[b0].ntiles, ws));
      if (st.size > 1) {
        if (!signal) {
          HIP_TRY(hipEventRecord(st.fuse_ev.ev[b0], ws));
          HIP_TRY(hipStreamWaitEvent(st.bucket_stream, st.fuse_ev.ev[b0], 0));
        }
        for (int k = 0; k < nb; k++) {
          if (signal) TRY(wait_packed(st, k, sigv[k]));
          char* p = (char*)flat + L->buckets[b0 + k].off;
          TRY(allreduce_device(st, p, p, L->buckets[b0 + k].bytes / es, dtype, st.bucket_stream));
        }
      }
      b0 += nb;
    }
    if (st.size > 1) TRY(join(ws, st.bucket_stream, st.ev_comp_done));
    return 0;
  });
}

int fused_allreduce_cast(State& st, const BatchItem* items, int n, int wire, hipStream_t user) {
  if (n <= 0) return 0;
  FusionCache& fc = cache(st);
  const int64_t threshold = fusion_threshold_bytes();
  TRY(ensure_slots(st, fc, threshold));
  std::vector<int64_t> counts((size_t)n);
  for (int i = 0; i < n; i++) counts[i] = items[i].count;
  return in_fusion(st, user, [&](hipStream_t ws) -> int {
    if (st.size > 1) {  // inputs ready for the bucket stream too (the large tensors start at once)
      HIP_TRY(hipEventRecord(st.ev_start, ws));
      HIP_TRY(hipStreamWaitEvent(st.bucket_stream, st.ev_start, 0));
    }
    // the layout of the WIRE type's bytes: buckets of at most the threshold in wire bytes
    Layout* L = find_layout(st, fc, counts.data(), n, wire, threshold, cast_tile_bytes(),
                            env_i64("TIPS_FUSION_BALANCE", 1) != 0);
    if (!L) return TIPS_ERR_HIP;
    if (L->seg_tensor.empty()) return 0;
    const int64_t es = tips::dtype_size(wire);
    const int B = (int)L->buckets.size();
    Table* t = B ? find_table(st, fc, *L, kSlotCast, items, n, st.fusion.p) : nullptr;
    if (B && !t) return TIPS_ERR_HIP;
    const size_t per = 2 * (size_t)L->ntiles + L->seg_tensor.size();
    auto cast = [&](int dir, int b) -> int {
      const CopySeg* base = t->dev + (size_t)dir * per;
      HIP_TRY(tips::launch_cast_segs(base, base + 2 * L->ntiles, L->buckets[b].tile0, L->buckets[b].ntiles, L->tile, dir,
                                     wire, ws));
      return 0;
    };
    auto slot = [&](int b) { return (char*)st.fusion.p + (int64_t)(b % 2) * threshold; };
    // tensors of at least the threshold (in wire bytes): one at a time through a scratch buffer of
    // the wire type - cast in, allreduce in place, cast out - on the bucket stream (their exchange
    // starts at once) or, at one rank, on the work stream (the round trip)
    hipStream_t big = st.size > 1 ? st.bucket_stream : ws;
    for (int i : L->direct) {
      TRY(st.cast_scratch.ensure((size_t)(items[i].count * es)));
      HIP_TRY(tips::launch_cast_range(st.cast_scratch.p, items[i].in, items[i].count, 0, wire, big));
      if (st.size > 1) TRY(allreduce_device(st, st.cast_scratch.p, st.cast_scratch.p, items[i].count, wire, big));
      HIP_TRY(tips::launch_cast_range(items[i].out, st.cast_scratch.p, items[i].count, 1, wire, big));
    }
    if (st.size == 1) {  // one rank: the allreduce is the identity; the casts are the reference's
      for (int b = 0; b < B; b++) {
        TRY(cast(0, b));
        TRY(cast(1, b));
      }
      return 0;
    }
    // as fused_allreduce: pack(0) pack(1) | unpack(0) pack(2) | ..., allreduce(b) on the bucket
    // stream between pack(b) and unpack(b), in the wire type
    TRY(st.fuse_ev.ensure(2 * (size_t)B));
    hipEvent_t* packed = st.fuse_ev.ev.data();
    hipEvent_t* reduced = st.fuse_ev.ev.data() + B;
    for (int b = 0; b < std::min(B, 2); b++) {
      TRY(cast(0, b));
      HIP_TRY(hipEventRecord(packed[b], ws));
    }
    for (int b = 0; b < B; b++) {
      HIP_TRY(hipStreamWaitEvent(st.bucket_stream, packed[b], 0));
      TRY(allreduce_device(st, slot(b), slot(b), L->buckets[b].bytes / es, wire, st.bucket_stream));
      HIP_TRY(hipEventRecord(reduced[b], st.bucket_stream));
      HIP_TRY(hipStreamWaitEvent(ws, reduced[b], 0));
      TRY(cast(1, b));
      if (b + 2 < B) {
        TRY(cast(0, b + 2));
        HIP_TRY(hipEventRecord(packed[b + 2], ws));
      }
    }
    return join(ws, st.bucket_stream, st.ev_comp_done);  // (the large tensors' work too)
  });
}

}  // namespace rt
}  // namespace tips

using namespace tips::rt;

namespace {

int check_list(const void* const* ins, const int64_t* counts, int n, int dtype, std::vector<BatchItem>* items,
               void* const* outs) {
  TRY(check_dtype(dtype));
  if (n < 0 || (n > 0 && (!ins || !counts))) return fail(TIPS_ERR_INVALID_ARG, "bad tensor list");
  items->resize((size_t)n);
  for (int i = 0; i < n; i++) {
    void* o = outs ? outs[i] : const_cast<void*>(ins[i]);
    if (counts[i] < 0 || (counts[i] > 0 && (!ins[i] || !o))) return fail(TIPS_ERR_INVALID_ARG, "bad tensor %d", i);
    (*items)[i] = BatchItem{ins[i], o, counts[i]};
  }
  return 0;
}

// the shape a fused list is announced with when it is routed through the negotiation: [n, elements]
void list_shape(const int64_t* counts, int n, int64_t* shape) {
  shape[0] = n;
  shape[1] = 0;
  for (int i = 0; i < n; i++) shape[1] += counts[i];
}

int fused_entry(const void* const* ins, void* const* outs, const int64_t* counts, int n, int dtype, void* stream) {
  if (!outs && n > 0) return fail(TIPS_ERR_INVALID_ARG, "bad tensor list");
  std::vector<BatchItem> items;
  TRY(check_list(ins, counts, n, dtype, &items, outs));
  int routed_rc;
  int64_t shape[2];
  list_shape(counts, n, shape);
  if (route_collective(TIPS_REQ_ALLREDUCE, dtype, shape, 2, 0,
                       [&] { return fused_entry(ins, outs, counts, n, dtype, stream); }, &routed_rc))
    return routed_rc;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  if (n == 0) return 0;
  TRY(set_device(st));
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

int tips_fused_allreduce_cast(const void* const* ins, void* const* outs, const int64_t* counts, int n, int dtype,
                              int wire_dtype, void* stream) {
  if (dtype != TIPS_FLOAT32)
    return fail(TIPS_ERR_UNSUPPORTED, "tips_fused_allreduce_cast: the tensors must be TIPS_FLOAT32 (got dtype %d)", dtype);
  if (wire_dtype != TIPS_FLOAT16 && wire_dtype != TIPS_BFLOAT16)
    return fail(TIPS_ERR_UNSUPPORTED, "tips_fused_allreduce_cast: the wire type must be TIPS_FLOAT16 or TIPS_BFLOAT16 "
                                      "(got %d)", wire_dtype);
  if (!outs && n > 0) return fail(TIPS_ERR_INVALID_ARG, "bad tensor list");
  std::vector<BatchItem> items;
  TRY(check_list(ins, counts, n, dtype, &items, outs));
  int routed_rc;
  int64_t shape[2];
  list_shape(counts, n, shape);
  // (announced with the wire type: a rank compressing to f16 and one to bf16 fail as mismatched dtypes)
  if (route_collective(TIPS_REQ_ALLREDUCE, wire_dtype, shape, 2, 0,
                       [&] { return tips_fused_allreduce_cast(ins, outs, counts, n, dtype, wire_dtype, stream); },
                       &routed_rc))
    return routed_rc;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  if (n == 0) return 0;
  TRY(set_device(st));
  return fused_allreduce_cast(st, items.data(), n, wire_dtype, (hipStream_t)stream);
}

#ifdef TIPS_DEV  // (development surface: libtips_hip_dev.so only, include/tips_hip_dev.h)
int64_t tips_fusion_tile_table(const int64_t* counts, int n, int dtype, const int64_t* ins, const int64_t* outs,
                               int64_t* records, int64_t cap, int64_t* ntiles, int64_t* tile_bytes) {
  TRY(check_dtype(dtype));
  if (n < 0 || (n > 0 && (!counts || !ins || !outs))) return fail(TIPS_ERR_INVALID_ARG, "bad list");
  for (int i = 0; i < n; i++)
    if (counts[i] < 0) return fail(TIPS_ERR_INVALID_ARG, "negative count %d", i);
  Layout L;
  L.dtype = dtype;
  L.threshold = fusion_threshold_bytes();
  L.tile = copy_tile_bytes();
  L.balance = env_i64("TIPS_FUSION_BALANCE", 1) != 0;
  build_layout(&L, counts, n);
  std::vector<BatchItem> items((size_t)n);
  for (int i = 0; i < n; i++) items[i] = BatchItem{(const void*)(uintptr_t)ins[i], (void*)(uintptr_t)outs[i], counts[i]};
  std::vector<tips::CopySeg> rec;
  fill_records(L, kCopy, items.data(), nullptr, &rec);
  if (ntiles) *ntiles = L.ntiles;
  if (tile_bytes) *tile_bytes = L.tile;
  if (records) {
    if (cap < (int64_t)rec.size()) return fail(TIPS_ERR_INVALID_ARG, "tips_fusion_tile_table: %zu records, room for %lld", rec.size(), (long long)cap);
    memcpy(records, rec.data(), rec.size() * sizeof(tips::CopySeg));
  }
  return (int64_t)rec.size();
}
#endif  // TIPS_DEV

int64_t tips_fused_layout(const int64_t* counts, int n, int dtype, int64_t* offsets) {
  TRY(check_dtype(dtype));
  if (n < 0 || (n > 0 && !counts)) return fail(TIPS_ERR_INVALID_ARG, "bad count list");
  for (int i = 0; i < n; i++)
    if (counts[i] < 0) return fail(TIPS_ERR_INVALID_ARG, "negative count %d", i);
  return fused_layout(counts, n, dtype, offsets);
}

int tips_fused_allreduce_flat(const void* const* ins, const int64_t* counts, int n, int dtype, void* flat,
                              void* stream) {
  std::vector<BatchItem> items;
  TRY(check_list(ins, counts, n, dtype, &items, nullptr));
  int routed_rc;
  int64_t shape[2];
  list_shape(counts, n, shape);
  if (route_collective(TIPS_REQ_ALLREDUCE, dtype, shape, 2, 0,
                       [&] { return tips_fused_allreduce_flat(ins, counts, n, dtype, flat, stream); }, &routed_rc))
    return routed_rc;
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  if (n == 0) return 0;
  if (!flat) return fail(TIPS_ERR_INVALID_ARG, "null flat output");
  TRY(set_device(st));
  if (!is_device_ptr(flat)) return fail(TIPS_ERR_INVALID_ARG, "tips_fused_allreduce_flat needs device memory");
  for (auto& it : items) it.out = it.count ? flat : nullptr;
  return fused_allreduce_flat(st, items.data(), n, dtype, flat, (hipStream_t)stream);
}

int64_t tips_fused_pack_bucket(const void* const* ins, const int64_t* counts, int n, int dtype, int bucket, void* dst,
                               void* stream) {
  std::vector<BatchItem> items;
  TRY(check_list(ins, counts, n, dtype, &items, nullptr));
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  if (!st.initialized) return fail(TIPS_ERR_NOT_INITIALIZED, "tips_init has not been called");
  if (n == 0) return 0;
  TRY(set_device(st));
  FusionCache& fc = cache(st);
  Layout* L = find_layout(st, fc, counts, n, dtype, fusion_threshold_bytes(), copy_tile_bytes(),
                          env_i64("TIPS_FUSION_BALANCE", 1) != 0);
  if (!L) return TIPS_ERR_HIP;
  const int B = (int)L->buckets.size();
  if (bucket < 0) return B;
  if (bucket >= B || !dst) return fail(TIPS_ERR_INVALID_ARG, "bucket %d of %d", bucket, B);
  const Bucket& bk = L->buckets[bucket];
  for (auto& it : items) it.out = (char*)dst - bk.off;
  // in the fusion chain like any fused call (the table's upload and later reuse stay ordered), with
  // the chain's event left to the next call that needs it: no marker between back-to-back launches
  TRY(in_fusion(st, (hipStream_t)stream, [&](hipStream_t ws) -> int {
    Table* t = find_table(st, fc, *L, kFlat, items.data(), n, (char*)dst - bk.off);
    if (!t) return TIPS_ERR_HIP;
    return copy_tiles(*L, *t, 0, bk.tile0, bk.ntiles, ws);
  }, /*lazy=*/true));
  int64_t payload = 0;
  for (int i = 0; i < n; i++)
    if (L->bucket[i] == bucket) payload += counts[i] * tips::dtype_size(dtype);
  return payload;
}

int tips_fusion_stats(int64_t* layouts_built, int64_t* layout_hits, int64_t* tables_built, int64_t* table_hits) {
  State& st = S();
  std::lock_guard<std::mutex> lk(st.mu);
  int64_t v[4];
  fusion_stats(st, v);
  if (layouts_built) *layouts_built = v[0];
  if (layout_hits) *layout_hits = v[1];
  if (tables_built) *tables_built = v[2];
  if (table_hits) *table_hits = v[3];
  return 0;
}

}  // extern "C"
