// kernels.hip — gfx950 (CDNA4) kernels of the gradient-bucket reduction path.
//
// What they replace: the local MPI_SUM reduction libmpi runs on every
// received chunk inside MPI_Allreduce, reached from AllreduceCpu<T>
// (reference tips/core/collective/utils.h:60-65, op from utils.cc:6-16).
//
// Design: the add is memory-bound — 1 flop per 12 B for
// f32 — so there is no MFMA and no LDS round trip; every lane moves 16 B per
// load/store (global_load_dwordx4 / global_store_dwordx4: one wave touches
// 1 KiB contiguous), UNROLL independent 16-B vectors per operand are issued
// before the first add so each lane keeps 2*UNROLL loads in flight, and the
// grid either covers the bucket one tile per workgroup (mode 1; mode 2 = the
// same with an XCD-contiguous tile order, the default) or grid-strides over a
// CU-multiple of workgroups (mode 0). Elements that do
// not fill a 16-B vector (the "tail", < 8 elements) are done scalar by
// workgroup 0. Integer adds wrap (two's complement, as MPI_SUM on MPI_INT /
// MPI_LONG_LONG); f16 adds are v_pk_add_f16 (correctly rounded, = fp32 add
// rounded to half); bf16 adds in fp32 and rounds to nearest-even.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "kernels.h"

namespace tips {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

enum { kF32 = 0, kF64 = 1, kI32 = 2, kI64 = 3, kF16 = 4, kBF16 = 5 };
constexpr int kBlock = 256;  // 4 waves of 64

int dtype_size(int dtype) {
  switch (dtype) {
    case kF32: return 4;
    case kF64: return 8;
    case kI32: return 4;
    case kI64: return 8;
    case kF16: return 2;
    case kBF16: return 2;
    default: return 0;
  }
}

// ---------------------------------------------------------------------------
// 16-byte loads / stores

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
  if constexpr (NT) {
    return __builtin_nontemporal_load(p);
  } else {
    return *p;
  }
}

template <bool NT>
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
  if constexpr (NT) {
    __builtin_nontemporal_store(v, p);
  } else {
    *p = v;
  }
}

// ---------------------------------------------------------------------------
// bf16 helpers: exact same rounding as oracle_float_to_bf16 (oracle/oracle.c)

__device__ __forceinline__ unsigned bf16_round_bits(unsigned x) {
  return ((x & 0x7fffffffu) > 0x7f800000u) ? ((x >> 16) | 0x40u) : ((x + 0x7fffu + ((x >> 16) & 1u)) >> 16);
}

__device__ __forceinline__ u32x4 bf16_pack(f32x4 lo, f32x4 hi) {
  u32x4 l = __builtin_bit_cast(u32x4, lo), h = __builtin_bit_cast(u32x4, hi);
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; i++) r[i] = bf16_round_bits(l[i]) | (bf16_round_bits(h[i]) << 16);
  return r;
}

__device__ __forceinline__ f32x4 bf16_lo(u32x4 v) { return __builtin_bit_cast(f32x4, v << 16u); }
__device__ __forceinline__ f32x4 bf16_hi(u32x4 v) { return __builtin_bit_cast(f32x4, v & 0xffff0000u); }

// ---------------------------------------------------------------------------
// 16-byte vector add per dtype (storage-precision result: one MPI_SUM step)

template <int DT>
__device__ __forceinline__ u32x4 add16(u32x4 a, u32x4 b);

template <>
__device__ __forceinline__ u32x4 add16<kF32>(u32x4 a, u32x4 b) {
  return __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, a) + __builtin_bit_cast(f32x4, b));
}
template <>
__device__ __forceinline__ u32x4 add16<kF64>(u32x4 a, u32x4 b) {
  return __builtin_bit_cast(u32x4, __builtin_bit_cast(f64x2, a) + __builtin_bit_cast(f64x2, b));
}
template <>
__device__ __forceinline__ u32x4 add16<kI32>(u32x4 a, u32x4 b) {
  return a + b;
}
template <>
__device__ __forceinline__ u32x4 add16<kI64>(u32x4 a, u32x4 b) {
  return __builtin_bit_cast(u32x4, __builtin_bit_cast(u64x2, a) + __builtin_bit_cast(u64x2, b));
}
template <>
__device__ __forceinline__ u32x4 add16<kF16>(u32x4 a, u32x4 b) {
  return __builtin_bit_cast(u32x4, __builtin_bit_cast(f16x8, a) + __builtin_bit_cast(f16x8, b));
}
template <>
__device__ __forceinline__ u32x4 add16<kBF16>(u32x4 a, u32x4 b) {
  return bf16_pack(bf16_lo(a) + bf16_lo(b), bf16_hi(a) + bf16_hi(b));
}

// Scalar element add for the tail (same arithmetic as add16, one element).
template <int DT>
__device__ __forceinline__ void add_elem(void* dst, const void* a, const void* b, int64_t i);

template <>
__device__ __forceinline__ void add_elem<kF32>(void* d, const void* a, const void* b, int64_t i) {
  ((float*)d)[i] = ((const float*)a)[i] + ((const float*)b)[i];
}
template <>
__device__ __forceinline__ void add_elem<kF64>(void* d, const void* a, const void* b, int64_t i) {
  ((double*)d)[i] = ((const double*)a)[i] + ((const double*)b)[i];
}
template <>
__device__ __forceinline__ void add_elem<kI32>(void* d, const void* a, const void* b, int64_t i) {
  ((unsigned*)d)[i] = ((const unsigned*)a)[i] + ((const unsigned*)b)[i];
}
template <>
__device__ __forceinline__ void add_elem<kI64>(void* d, const void* a, const void* b, int64_t i) {
  ((unsigned long long*)d)[i] = ((const unsigned long long*)a)[i] + ((const unsigned long long*)b)[i];
}
template <>
__device__ __forceinline__ void add_elem<kF16>(void* d, const void* a, const void* b, int64_t i) {
  ((_Float16*)d)[i] = ((const _Float16*)a)[i] + ((const _Float16*)b)[i];
}
template <>
__device__ __forceinline__ void add_elem<kBF16>(void* d, const void* a, const void* b, int64_t i) {
  unsigned x = (unsigned)((const unsigned short*)a)[i] << 16, y = (unsigned)((const unsigned short*)b)[i] << 16;
  float s = __builtin_bit_cast(float, x) + __builtin_bit_cast(float, y);
  ((unsigned short*)d)[i] = (unsigned short)bf16_round_bits(__builtin_bit_cast(unsigned, s));
}

// XCD-contiguous tile order: workgroups are dealt round-robin over the 8 XCDs
// (b and b+8 share one), so tile = (b % 8) * (grid / 8) + b / 8 hands each XCD
// one contiguous stretch. Needs grid % 8 == 0; speed only, never correctness.
__device__ __forceinline__ int64_t xcd_tile(unsigned b, unsigned grid) {
  return (int64_t)(b & 7u) * (grid >> 3) + (b >> 3);
}

// XCD stripes (round 6): the tiles cut into stripes of C tiles (1 MiB of each operand), stripe s
// on XCD s % 8, and workgroup j of an XCD takes the j-th tile of that XCD's stripes. With one
// contiguous eighth per XCD (xcd_tile) the 8 XCDs' streams sit at the same offset of their
// eighths, all 3 operands' alike; at 128 MiB operands that cost the 2-input sum 6 % (0.774 against
// 0.820 in 1 MiB stripes, profiles/r06/stripes/sum2_map_sweep.jsonl), at 256 MiB it ties. C <= 0, or one
// stripe per XCD or fewer (the grid's eighth R <= C), is xcd_tile. The grid must then cover whole
// rounds of 8 stripes (stripe_grid): R a multiple of C, so the map is a bijection onto [0, grid).
__device__ __forceinline__ int64_t stripe_tile(unsigned b, unsigned grid, int64_t C) {
  const int64_t R = grid >> 3;
  if (C <= 0 || R <= C) return xcd_tile(b, grid);
  const int64_t j = b >> 3;
  return ((j / C) * 8 + (b & 7u)) * C + j % C;
}

// ---------------------------------------------------------------------------
// 2-input sum: dst = a + b

template <int DT, int MODE, int UNROLL, bool NTL, bool NTS, int BLOCK>
__global__ __launch_bounds__(BLOCK) void sum2_kernel(u32x4* __restrict__ dst, const u32x4* __restrict__ a,
                                                    const u32x4* __restrict__ b, int64_t nvec, int64_t tail_begin,
                                                    int64_t n) {
  constexpr int64_t kTile = (int64_t)BLOCK * UNROLL;  // vectors per workgroup-iteration
  const int tid = threadIdx.x;
  // MODE 2: XCD-contiguous placement. Workgroups are dealt round-robin over the 8 XCDs
  // (b and b+8 share one), so tile = (b % 8) * (grid / 8) + b / 8 gives each XCD one
  // contiguous stretch of the bucket (speed only: any placement is correct).
  int64_t t = (MODE == 2) ? xcd_tile(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
  const int64_t tstride = (MODE == 0) ? (int64_t)gridDim.x : 0;
  do {
    const int64_t base = t * kTile + tid;
    if (base + (UNROLL - 1) * BLOCK < nvec) {
      u32x4 x[UNROLL], y[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; u++) x[u] = ld16<NTL>(a + base + u * BLOCK);
#pragma unroll
      for (int u = 0; u < UNROLL; u++) y[u] = ld16<NTL>(b + base + u * BLOCK);
#pragma unroll
      for (int u = 0; u < UNROLL; u++) st16<NTS>(dst + base + u * BLOCK, add16<DT>(x[u], y[u]));
    } else {
#pragma unroll
      for (int u = 0; u < UNROLL; u++) {
        const int64_t i = base + u * BLOCK;
        if (i < nvec) st16<NTS>(dst + i, add16<DT>(ld16<NTL>(a + i), ld16<NTL>(b + i)));
      }
    }
    t += tstride;
  } while (MODE == 0 && t * kTile < nvec);
  if (blockIdx.x == 0 && tail_begin + tid < n) add_elem<DT>(dst, a, b, tail_begin + tid);
}

// The shipped 2-input sum (and, with other CPol bits, the cache-policy sweep
// variants): one tile of U x BLOCK vectors per operand per workgroup, placed by stripe_tile,
// through buffer_load/store_dwordx4 with explicit CPol bits (aux: 1 = sc0,
// 2 = nt, 16 = sc1). The product launch (kDef* below): BLOCK = 128, nt loads and nt stores,
// 512 KiB stripes (round 6; rounds 2-5: 256 lanes with sc1 stores, which won when one buffer
// triple was re-read, 7.46 vs 7.10 TB/s, profiles/r01_sum_sweep_f.jsonl). Each workgroup's
// descriptors cover exactly its tile, so the hardware range check drops lanes past the end.
template <int DT, int LAUX, int SAUX, int U = 1, int BLOCK = 256>
__global__ __launch_bounds__(BLOCK) void sum2_buf_kernel(u32x4* __restrict__ dst, const u32x4* __restrict__ a,
                                                        const u32x4* __restrict__ b, int64_t nvec,
                                                        int64_t tail_begin, int64_t n, int64_t stripe) {
  constexpr int64_t kTile = (int64_t)BLOCK * U;
  const int64_t t = stripe_tile(blockIdx.x, gridDim.x, stripe);
  const int64_t first = t * kTile;
  if (first < nvec) {
    const int rec = (int)(((nvec - first) < kTile ? (nvec - first) : kTile) * 16);
    __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)(a + first), (short)0, rec, 0x00020000);
    __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)(b + first), (short)0, rec, 0x00020000);
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(dst + first), (short)0, rec, 0x00020000);
    u32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, (u * BLOCK + (int)threadIdx.x) * 16, 0, LAUX);
#pragma unroll
    for (int u = 0; u < U; u++) y[u] = __builtin_amdgcn_raw_buffer_load_b128(rb, (u * BLOCK + (int)threadIdx.x) * 16, 0, LAUX);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(add16<DT>(x[u], y[u]), rd, (u * BLOCK + (int)threadIdx.x) * 16, 0, SAUX);
  }
  if (blockIdx.x == 0 && tail_begin + (int64_t)threadIdx.x < n) add_elem<DT>(dst, a, b, tail_begin + threadIdx.x);
}

// The shipped sum with other workgroup -> tile maps (tuning sweep only, f32; the 128 MiB dip,
// DESIGN.md §3): stripe = 0 address order; else the tiles cut into stripes of `stripe` tiles dealt
// round-robin over the 8 XCDs (stripe s to XCD s % 8; the shipped map is one stripe per XCD), and
// workgroup j of XCD x takes the j-th tile of that XCD's stripes. The grid covers whole rounds of
// 8 stripes (the workgroups past the last tile exit at once).
#ifdef TIPS_DEV  // (tuning sweeps: libtips_hip_dev.so only)
__global__ __launch_bounds__(256) void sum2_map_kernel(u32x4* __restrict__ dst, const u32x4* __restrict__ a,
                                                       const u32x4* __restrict__ b, int64_t nvec, int64_t tail_begin,
                                                       int64_t n, int64_t stripe) {
  constexpr int64_t kTile = 256;
  const int64_t bx = blockIdx.x, x = bx & 7, j = bx >> 3;
  const int64_t t = stripe == 0 ? bx : (x + 8 * (j / stripe)) * stripe + j % stripe;
  const int64_t first = t * kTile;
  if (first < nvec) {
    const int rec = (int)(((nvec - first) < kTile ? (nvec - first) : kTile) * 16);
    __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)(a + first), (short)0, rec, 0x00020000);
    __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)(b + first), (short)0, rec, 0x00020000);
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(dst + first), (short)0, rec, 0x00020000);
    const u32x4 xv = __builtin_amdgcn_raw_buffer_load_b128(ra, (int)threadIdx.x * 16, 0, 2);
    const u32x4 yv = __builtin_amdgcn_raw_buffer_load_b128(rb, (int)threadIdx.x * 16, 0, 2);
    __builtin_amdgcn_raw_buffer_store_b128(add16<kF32>(xv, yv), rd, (int)threadIdx.x * 16, 0, 16);
  }
  if (blockIdx.x == 0 && tail_begin + (int64_t)threadIdx.x < n) add_elem<kF32>(dst, a, b, tail_begin + threadIdx.x);
}
#endif  // TIPS_DEV

// LDS-staged 2-input sum (tuning sweep only, f32): both operand tiles go global -> LDS with
// gfx950's direct-to-LDS loads (global_load_lds_dwordx4 nt: no VGPR destination, each
// wave-instruction lands 1 KiB at a wave-uniform LDS base + lane x 16 B), then LDS -> VGPRs
// (ds_read_b128), add, sc1 buffer store as the shipped kernel. It measures what an LDS hop
// costs a stream that reads every byte once. Partial last tile: plain loads.
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

#ifdef TIPS_DEV  // (tuning sweeps: libtips_hip_dev.so only)
template <int U>
__global__ __launch_bounds__(256) void sum2_lds_kernel(u32x4* __restrict__ dst, const u32x4* __restrict__ a,
                                                       const u32x4* __restrict__ b, int64_t nvec, int64_t tail_begin,
                                                       int64_t n) {
  __shared__ u32x4 stage[2 * 256 * U];  // one array: [a tile | b tile]
  constexpr int64_t kTile = 256 * U;
  const int tid = threadIdx.x, wbase = tid & ~63;
  const int64_t first = xcd_tile(blockIdx.x, gridDim.x) * kTile;
  if (first + kTile <= nvec) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(a + first + u * 256 + tid), (lds_ptr_t)(stage + u * 256 + wbase),
                                       16, 0, 2);
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(b + first + u * 256 + tid),
                                       (lds_ptr_t)(stage + kTile + u * 256 + wbase), 16, 0, 2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(dst + first), (short)0, (int)(kTile * 16),
                                                                  0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(add16<kF32>(stage[u * 256 + tid], stage[kTile + u * 256 + tid]), rd,
                                             (u * 256 + tid) * 16, 0, 16);
  } else if (first < nvec) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int64_t i = first + u * 256 + tid;
      if (i < nvec) dst[i] = add16<kF32>(a[i], b[i]);
    }
  }
  if (blockIdx.x == 0 && tail_begin + (int64_t)threadIdx.x < n) add_elem<kF32>(dst, a, b, tail_begin + threadIdx.x);
}
#endif  // TIPS_DEV

// Persistent streaming 2-input sum (tuning sweep only, f32): gridDim = 256 CUs x WPC
// workgroups, each owning one contiguous range of the bucket (XCD-contiguous order), walked
// 4 KiB per operand at a time with the next tile's loads issued before the current tile's add
// and sc1 store (2-deep software pipeline). Tests whether long sequential runs per CU beat one
// short tile per workgroup on DRAM efficiency.
#ifdef TIPS_DEV  // (tuning sweeps: libtips_hip_dev.so only)
__global__ __launch_bounds__(256) void sum2_stream_kernel(u32x4* __restrict__ dst, const u32x4* __restrict__ a,
                                                          const u32x4* __restrict__ b, int64_t nvec,
                                                          int64_t tail_begin, int64_t n) {
  const int64_t G = gridDim.x;
  const int64_t per = ((nvec + G - 1) / G + 255) / 256 * 256;
  const int64_t beg = xcd_tile(blockIdx.x, gridDim.x) * per;
  const int64_t end = beg + per < nvec ? beg + per : nvec;
  const int tid = threadIdx.x;
  if (beg < end) {
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(dst + beg), (short)0,
                                                                  (int)((end - beg) * 16), 0x00020000);
    const int64_t iters = (end - beg + 255) / 256;
    int64_t i = beg + tid;
    u32x4 x0 = {}, y0 = {};
    if (i < end) {
      x0 = ld16<true>(a + i);
      y0 = ld16<true>(b + i);
    }
    for (int64_t k = 0; k < iters; k++) {
      const int64_t j = i + 256;
      u32x4 x1 = {}, y1 = {};
      if (j < end) {
        x1 = ld16<true>(a + j);
        y1 = ld16<true>(b + j);
      }
      if (i < end) __builtin_amdgcn_raw_buffer_store_b128(add16<kF32>(x0, y0), rd, (int)((i - beg) * 16), 0, 16);
      x0 = x1;
      y0 = y1;
      i = j;
    }
  }
  if (blockIdx.x == 0 && tail_begin + (int64_t)threadIdx.x < n) add_elem<kF32>(dst, a, b, tail_begin + threadIdx.x);
}
#endif  // TIPS_DEV

// Unaligned fallback (any pointer not 16-B aligned): one element per lane.
template <int DT>
__global__ __launch_bounds__(kBlock) void sum2_scalar_kernel(void* dst, const void* a, const void* b, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
    add_elem<DT>(dst, a, b, i);
}

// ---------------------------------------------------------------------------
// Multi-input sum: dst = ((s0 + s1) + s2) + ...  (rank-order fold)
// f16/bf16 accumulate in fp32 and round once; others accumulate in storage type.

template <int DT>
struct Wide;
template <>
struct Wide<kF32> {
  using A = f32x4;
  static __device__ A load(u32x4 v) { return __builtin_bit_cast(f32x4, v); }
  static __device__ u32x4 store(A a) { return __builtin_bit_cast(u32x4, a); }
};
template <>
struct Wide<kF64> {
  using A = f64x2;
  static __device__ A load(u32x4 v) { return __builtin_bit_cast(f64x2, v); }
  static __device__ u32x4 store(A a) { return __builtin_bit_cast(u32x4, a); }
};
template <>
struct Wide<kI32> {
  using A = u32x4;
  static __device__ A load(u32x4 v) { return v; }
  static __device__ u32x4 store(A a) { return a; }
};
template <>
struct Wide<kI64> {
  using A = u64x2;
  static __device__ A load(u32x4 v) { return __builtin_bit_cast(u64x2, v); }
  static __device__ u32x4 store(A a) { return __builtin_bit_cast(u32x4, a); }
};
template <>
struct Wide<kF16> {
  using A = f32x8;
  static __device__ A load(u32x4 v) { return __builtin_convertvector(__builtin_bit_cast(f16x8, v), f32x8); }
  static __device__ u32x4 store(A a) { return __builtin_bit_cast(u32x4, __builtin_convertvector(a, f16x8)); }
};
template <>
struct Wide<kBF16> {
  using A = f32x8;
  static __device__ A load(u32x4 v) {
    f32x4 lo = bf16_lo(v), hi = bf16_hi(v);
    return A{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
  static __device__ u32x4 store(A a) {
    return bf16_pack(f32x4{a[0], a[1], a[2], a[3]}, f32x4{a[4], a[5], a[6], a[7]});
  }
};

template <int DT>
struct ScalarOf;
template <>
struct ScalarOf<kF32> {
  using T = float;
};
template <>
struct ScalarOf<kF64> {
  using T = double;
};
template <>
struct ScalarOf<kI32> {
  using T = unsigned;
};
template <>
struct ScalarOf<kI64> {
  using T = unsigned long long;
};
template <>
struct ScalarOf<kF16> {
  using T = _Float16;
};
template <>
struct ScalarOf<kBF16> {
  using T = unsigned short;
};

template <int DT>
__device__ __forceinline__ void fold_elem(void* dst, const void* const* srcs, int nsrc, int64_t i) {
  if constexpr (DT == kF16) {
    float acc = (float)((const _Float16*)srcs[0])[i];
    for (int j = 1; j < nsrc; j++) acc += (float)((const _Float16*)srcs[j])[i];
    ((_Float16*)dst)[i] = (_Float16)acc;
  } else if constexpr (DT == kBF16) {
    float acc = __builtin_bit_cast(float, (unsigned)((const unsigned short*)srcs[0])[i] << 16);
    for (int j = 1; j < nsrc; j++) acc += __builtin_bit_cast(float, (unsigned)((const unsigned short*)srcs[j])[i] << 16);
    ((unsigned short*)dst)[i] = (unsigned short)bf16_round_bits(__builtin_bit_cast(unsigned, acc));
  } else {
    // storage-type fold in a register (dst may alias one of srcs: in-place)
    using T = typename ScalarOf<DT>::T;
    T acc = ((const T*)srcs[0])[i];
    for (int j = 1; j < nsrc; j++) acc = acc + ((const T*)srcs[j])[i];
    ((T*)dst)[i] = acc;
  }
}

struct SrcList {
  const u32x4* p[kMaxSrcs];
};

template <int DT, int NSRC, int UNROLL>
__global__ __launch_bounds__(kBlock) void multi_sum_kernel(u32x4* __restrict__ dst, SrcList srcs, int64_t nvec,
                                                          int64_t tail_begin, int64_t n) {
  using W = Wide<DT>;
  constexpr int64_t kTile = (int64_t)kBlock * UNROLL;
  const int tid = threadIdx.x;
  const int64_t first = xcd_tile(blockIdx.x, gridDim.x) * kTile;
  const int64_t base = first + tid;
  // sc1 stores through a descriptor covering this tile (as sum2_buf_kernel)
  const int64_t left = nvec - first;
  __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(dst + first), (short)0, (int)((left < kTile ? (left > 0 ? left : 0) : kTile) * 16), 0x00020000);
#pragma unroll
  for (int u = 0; u < UNROLL; u++) {
    const int64_t i = base + u * kBlock;
    if (i < nvec) {
      u32x4 v[NSRC];
#pragma unroll
      for (int j = 0; j < NSRC; j++) v[j] = ld16<true>(srcs.p[j] + i);
      typename W::A acc = W::load(v[0]);
#pragma unroll
      for (int j = 1; j < NSRC; j++) acc = acc + W::load(v[j]);
      __builtin_amdgcn_raw_buffer_store_b128(W::store(acc), rd, (int)((i - first) * 16), 0, 16);
    }
  }
  if (blockIdx.x == 0 && NSRC > 1 && tail_begin + tid < n) {
    const void* s[NSRC];
#pragma unroll
    for (int j = 0; j < NSRC; j++) s[j] = srcs.p[j];
    fold_elem<DT>(dst, s, NSRC, tail_begin + tid);
  }
}

// Buffer-op form of the multi-input sum: one descriptor per source covering
// this workgroup's tile, cache-policy bits on the loads (LAUX) and sc1 stores,
// every source's vectors in flight before the fold (as sum2_buf_kernel).
template <int DT, int NSRC, int U, int LAUX, int BLOCK = kBlock, int SAUX = 16>
__global__ __launch_bounds__(BLOCK) void multi_sum_buf_kernel(u32x4* __restrict__ dst, SrcList srcs, int64_t nvec,
                                                             int64_t tail_begin, int64_t n, int64_t stripe) {
  using W = Wide<DT>;
  constexpr int64_t kTile = (int64_t)BLOCK * U;
  const int tid = threadIdx.x;
  const int64_t first = stripe_tile(blockIdx.x, gridDim.x, stripe) * kTile;
  if (first < nvec) {
    const int rec = (int)(((nvec - first) < kTile ? (nvec - first) : kTile) * 16);
    u32x4 v[U][NSRC];
#pragma unroll
    for (int j = 0; j < NSRC; j++) {
      __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(srcs.p[j] + first), (short)0, rec, 0x00020000);
#pragma unroll
      for (int u = 0; u < U; u++) v[u][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (u * BLOCK + tid) * 16, 0, LAUX);
    }
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(dst + first), (short)0, rec, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++) {
      typename W::A acc = W::load(v[u][0]);
#pragma unroll
      for (int j = 1; j < NSRC; j++) acc = acc + W::load(v[u][j]);
      __builtin_amdgcn_raw_buffer_store_b128(W::store(acc), rd, (u * BLOCK + tid) * 16, 0, SAUX);
    }
  }
  if (blockIdx.x == 0 && NSRC > 1 && tail_begin + tid < n) {
    const void* s[NSRC];
#pragma unroll
    for (int j = 0; j < NSRC; j++) s[j] = srcs.p[j];
    fold_elem<DT>(dst, s, NSRC, tail_begin + tid);
  }
}

#ifdef TIPS_DEV  // (tuning sweeps: libtips_hip_dev.so only)
// Round-5 sweep form of the fold (f32): ORDER 0 = XCD-contiguous tiles, 1 = address order (the
// 8 XCDs on neighbouring tiles, so the chip reads NSRC + 1 moving windows instead of 8 x that),
// 2 = XCD-contiguous with each XCD's stretch cut into 8 interleaved runs; ITER consecutive tiles
// per workgroup, one after the other (longer-lived workgroups, fewer ramps); ROT: the sources'
// load order rotated by workgroup (the fold order is unchanged); SAUX store policy; BLOCK lanes.
template <int NSRC, int U, int SAUX, int ORDER, int ITER, int ROT, int BLOCK>
__global__ __launch_bounds__(BLOCK) void multi_sum_x_kernel(u32x4* __restrict__ dst, SrcList srcs, int64_t nvec,
                                                            int64_t tail_begin, int64_t n) {
  constexpr int64_t kTile = (int64_t)BLOCK * U;
  const int tid = threadIdx.x;
  int64_t g;
  if constexpr (ORDER == 0) {
    g = xcd_tile(blockIdx.x, gridDim.x);
  } else if constexpr (ORDER == 1) {
    g = blockIdx.x;
  } else {  // XCD x owns stretch x; inside it, its workgroups walk 8 sub-runs round-robin
    const int64_t per = gridDim.x >> 3, k = blockIdx.x >> 3, runs = per >= 64 ? 8 : 1;
    g = (int64_t)(blockIdx.x & 7u) * per + (k % runs) * (per / runs) + k / runs;
  }
  for (int it = 0; it < ITER; it++) {
    const int64_t first = (g * ITER + it) * kTile;
    if (first >= nvec) break;
    const int rec = (int)(((nvec - first) < kTile ? (nvec - first) : kTile) * 16);
    u32x4 v[U][NSRC];
#pragma unroll
    for (int jj = 0; jj < NSRC; jj++) {
      const int j = ROT ? (int)((jj + blockIdx.x) % NSRC) : jj;
      __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(srcs.p[j] + first), (short)0, rec, 0x00020000);
#pragma unroll
      for (int u = 0; u < U; u++) {
        u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, (u * BLOCK + tid) * 16, 0, 2);
        if constexpr (ROT) {
#pragma unroll
          for (int q = 0; q < NSRC; q++)
            if (q == j) v[u][q] = x;
        } else {
          v[u][jj] = x;
        }
      }
    }
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(dst + first), (short)0, rec, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++) {
      f32x4 acc = __builtin_bit_cast(f32x4, v[u][0]);
#pragma unroll
      for (int j = 1; j < NSRC; j++) acc = acc + __builtin_bit_cast(f32x4, v[u][j]);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc), rd, (u * BLOCK + tid) * 16, 0, SAUX);
    }
  }
  if (blockIdx.x == 0 && NSRC > 1 && tail_begin + tid < n) {
    const void* s[NSRC];
#pragma unroll
    for (int j = 0; j < NSRC; j++) s[j] = srcs.p[j];
    fold_elem<kF32>(dst, s, NSRC, tail_begin + tid);
  }
}

// Grid-stride form (round-5 sweep, f32): gridDim = 256 CUs x W workgroups, XCD x walking its
// stretch with its grid / 8 workgroups side by side (tile = stretch start + k x grid / 8 + slot).
// The chip's loads in flight are capped by the grid, not by reserved LDS or registers, so a
// transfer kernel beside the fold still finds room on every CU. PIPE: the next tile's loads are
// issued before this tile's add and store.
template <int NSRC, int BLOCK, int PIPE>
__global__ __launch_bounds__(BLOCK) void multi_sum_gs_kernel(u32x4* __restrict__ dst, SrcList srcs, int64_t nvec,
                                                             int64_t tail_begin, int64_t n) {
  constexpr int64_t kTile = BLOCK;
  const int tid = threadIdx.x;
  const int64_t ntiles = (nvec + kTile - 1) / kTile;
  const int64_t per_xcd = (ntiles + 7) / 8, wg_xcd = gridDim.x >> 3;
  const int64_t x = blockIdx.x & 7u, slot = blockIdx.x >> 3;
  const int64_t beg = x * per_xcd, end = beg + per_xcd < ntiles ? beg + per_xcd : ntiles;
  auto load = [&](int64_t t, u32x4 (&v)[NSRC]) {
    const int64_t first = t * kTile;
    const int rec = (int)(((nvec - first) < kTile ? (nvec - first) : kTile) * 16);
#pragma unroll
    for (int j = 0; j < NSRC; j++) {
      __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(srcs.p[j] + first), (short)0, rec, 0x00020000);
      v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, tid * 16, 0, 2);
    }
  };
  auto fold_store = [&](int64_t t, const u32x4 (&v)[NSRC]) {
    const int64_t first = t * kTile;
    const int rec = (int)(((nvec - first) < kTile ? (nvec - first) : kTile) * 16);
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(dst + first), (short)0, rec, 0x00020000);
    f32x4 acc = __builtin_bit_cast(f32x4, v[0]);
#pragma unroll
    for (int j = 1; j < NSRC; j++) acc = acc + __builtin_bit_cast(f32x4, v[j]);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc), rd, tid * 16, 0, 16);
  };
  int64_t t = beg + slot;
  if constexpr (PIPE) {
    u32x4 a[NSRC], b[NSRC];
    if (t < end) load(t, a);
    while (t < end) {
      const int64_t t2 = t + wg_xcd;
      if (t2 < end) load(t2, b);
      fold_store(t, a);
#pragma unroll
      for (int j = 0; j < NSRC; j++) a[j] = b[j];
      t = t2;
    }
  } else {
    for (; t < end; t += wg_xcd) {
      u32x4 v[NSRC];
      load(t, v);
      fold_store(t, v);
    }
  }
  if (blockIdx.x == 0 && NSRC > 1 && tail_begin + tid < n) {
    const void* s[NSRC];
#pragma unroll
    for (int j = 0; j < NSRC; j++) s[j] = srcs.p[j];
    fold_elem<kF32>(dst, s, NSRC, tail_begin + tid);
  }
}
#endif  // TIPS_DEV

template <int DT>
__global__ __launch_bounds__(kBlock) void multi_sum_scalar_kernel(void* dst, SrcList srcs, int nsrc, int64_t n) {
  const void* s[kMaxSrcs];
  for (int j = 0; j < nsrc; j++) s[j] = srcs.p[j];
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
    fold_elem<DT>(dst, s, nsrc, i);
}

// ---------------------------------------------------------------------------
// Batched copy (fusion pack / unpack)

#ifdef TIPS_DEV  // (tuning sweeps: libtips_hip_dev.so only)
__global__ __launch_bounds__(kBlock) void copy_tiles_kernel(const CopyTile* __restrict__ tiles, int ntiles) {
  const int64_t ti = xcd_tile(blockIdx.x, gridDim.x);
  if (ti >= ntiles) return;
  const CopyTile t = tiles[ti];
  const int tid = threadIdx.x;
  if (((reinterpret_cast<uintptr_t>(t.src) | reinterpret_cast<uintptr_t>(t.dst) | (uintptr_t)t.bytes) & 15) == 0) {
    const u32x4* s = reinterpret_cast<const u32x4*>(t.src);
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(t.dst, (short)0, (int)t.bytes, 0x00020000);
    const int64_t nv = t.bytes >> 4;
    constexpr int U = 4;
    for (int64_t i = tid; i < nv; i += kBlock * U) {
      u32x4 v[U] = {};
#pragma unroll
      for (int u = 0; u < U; u++)
        if (i + u * kBlock < nv) v[u] = ld16<true>(s + i + u * kBlock);
#pragma unroll
      for (int u = 0; u < U; u++)  // sc1 stores; lanes past the tile fall off the descriptor's range
        __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, (int)((i + u * kBlock) * 16), 0, 16);
    }
  } else if (((reinterpret_cast<uintptr_t>(t.src) | reinterpret_cast<uintptr_t>(t.dst) | (uintptr_t)t.bytes) & 3) == 0) {
    const unsigned* s = reinterpret_cast<const unsigned*>(t.src);
    unsigned* d = reinterpret_cast<unsigned*>(t.dst);
    for (int64_t i = tid; i < (t.bytes >> 2); i += kBlock) d[i] = s[i];
  } else {
    for (int64_t i = tid; i < t.bytes; i += kBlock) t.dst[i] = t.src[i];
  }
}
#endif  // TIPS_DEV

// Grouped variant (tuning sweep, tools/copy_sweep.py): each workgroup copies G consecutive tiles
// of at most 256 x U x 16 B. The G descriptors are read up front (independent scalar loads, one
// latency for all), then every lane issues its G x U 16-B loads before the first store, so one
// workgroup keeps G tiles in flight and the descriptor latency is paid once per G tiles. A tile
// whose ends are 16-B aligned moves its whole 16-B vectors through buffer ops (range = those
// vectors, so lanes past them fall off) and its < 16 trailing bytes bytewise; a misaligned tile
// goes bytewise whole.
#ifdef TIPS_DEV  // (tuning sweeps: libtips_hip_dev.so only)
template <int G, int U, int LAUX, int SAUX>
__global__ __launch_bounds__(kBlock) void copy_tiles_g_kernel(const CopyTile* __restrict__ tiles, int ntiles) {
  const int64_t t0 = xcd_tile(blockIdx.x, gridDim.x) * G;
  if (t0 >= ntiles) return;
  const int tid = threadIdx.x;
  CopyTile d[G];
  int vec[G];  // bytes moved as 16-B vectors
#pragma unroll
  for (int g = 0; g < G; g++) {
    d[g] = (t0 + g < ntiles) ? tiles[t0 + g] : CopyTile{nullptr, nullptr, 0};
    const bool al = ((reinterpret_cast<uintptr_t>(d[g].src) | reinterpret_cast<uintptr_t>(d[g].dst)) & 15) == 0;
    vec[g] = al ? (int)(d[g].bytes & ~(int64_t)15) : 0;
  }
  u32x4 v[G][U];
#pragma unroll
  for (int g = 0; g < G; g++) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)d[g].src, (short)0, vec[g], 0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++) v[g][u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (u * kBlock + tid) * 16, 0, LAUX);
  }
#pragma unroll
  for (int g = 0; g < G; g++) {
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(d[g].dst, (short)0, vec[g], 0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++) __builtin_amdgcn_raw_buffer_store_b128(v[g][u], rd, (u * kBlock + tid) * 16, 0, SAUX);
    for (int64_t i = vec[g] + tid; i < d[g].bytes; i += kBlock) d[g].dst[i] = d[g].src[i];
  }
}
#endif  // TIPS_DEV

// ---------------------------------------------------------------------------
// Contiguous copy: the out-of-place allreduce at one rank (MPI_Allreduce returns the input). Shaped
// as sum2_buf_kernel with one operand: one 4 KiB tile per 256-lane workgroup in XCD-contiguous
// order, buffer loads nt, buffer stores sc1 (the line leaves the XCD's L2), descriptors covering
// exactly the tile; the < 16 trailing bytes go bytewise in workgroup 0. (hipMemcpyAsync's D2D blit
// moved config 3's 1 GiB at 0.62 of HBM, profiles/r04/n_bench_n1.jsonl.)
template <int U, int SAUX = 16, int BLOCK = kBlock>
__global__ __launch_bounds__(BLOCK) void copy_buf_kernel(u32x4* __restrict__ dst, const u32x4* __restrict__ src,
                                                         int64_t nvec, int64_t tail_begin, int64_t bytes, int64_t stripe) {
  constexpr int64_t kTile = (int64_t)BLOCK * U;
  const int64_t first = stripe_tile(blockIdx.x, gridDim.x, stripe) * kTile;
  const int tid = threadIdx.x;
  if (first < nvec) {
    const int rec = (int)(((nvec - first) < kTile ? (nvec - first) : kTile) * 16);
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(src + first), (short)0, rec, 0x00020000);
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(dst + first), (short)0, rec, 0x00020000);
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (u * BLOCK + tid) * 16, 0, 2);
#pragma unroll
    for (int u = 0; u < U; u++) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, (u * BLOCK + tid) * 16, 0, SAUX);
  }
  if (blockIdx.x == 0 && tail_begin + tid < bytes)
    reinterpret_cast<char*>(dst)[tail_begin + tid] = reinterpret_cast<const char*>(src)[tail_begin + tid];
}

// Stripe size for stripe_tile, in 16-B vectors of one operand (TIPS_STRIPE_KIB, default 1 MiB;
// 0: xcd_tile's contiguous eighths), and the grid that covers `tiles` tiles of `tile` vectors:
// whole rounds of 8 stripes once there are more than 8 stripes' worth of tiles.
int64_t stripe_vecs() {
  static const int64_t v = [] {
    const char* e = getenv("TIPS_STRIPE_KIB");
    const long kib = e && *e ? atol(e) : 1024;
    return (int64_t)std::max<long>(0, kib) * 1024 / 16;
  }();
  return v;
}

// The fusion pack's stripe (TIPS_PACK_STRIPE_KIB, default 0 = xcd_tile), in 16-B vectors; the
// layout's tile order (fusion.cc tile_order) places boundary tiles by the same map.
int64_t pack_stripe_vecs() {
  static const int64_t v = [] {
    const char* e = getenv("TIPS_PACK_STRIPE_KIB");
    const long kib = e && *e ? atol(e) : 0;
    return (int64_t)std::max<long>(0, kib) * 1024 / 16;
  }();
  return v;
}

int64_t stripe_of(int64_t tile) { return stripe_vecs() / std::max<int64_t>(1, tile); }

// The 2-input sum's own stripe (TIPS_SUM_STRIPE_KIB, default 512 KiB; 0: eighths): with its
// 128-lane launch, 512 KiB stripes ran config 2 0.6-0.8 % faster than 1 MiB, while the copy
// kept 1 MiB (profiles/r06/sum2_focus/, stripe512/). Unset, TIPS_STRIPE_KIB=0 also turns it off.
int64_t sum_stripe_of(int64_t tile) {
  static const int64_t v = [] {
    const char* e = getenv("TIPS_SUM_STRIPE_KIB");
    const char* g = getenv("TIPS_STRIPE_KIB");
    const long kib = e && *e ? atol(e) : (g && *g && atol(g) == 0 ? 0 : 512);
    return (int64_t)std::max<long>(0, kib) * 1024 / 16;
  }();
  return v / std::max<int64_t>(1, tile);
}

int64_t stripe_grid(int64_t tiles, int64_t C) {
  if (C <= 0 || tiles <= 8 * C) return std::max<int64_t>(8, (tiles + 7) / 8 * 8);
  return (tiles + 8 * C - 1) / (8 * C) * (8 * C);
}

void stripe_slots(int64_t nslots, int64_t C, std::vector<int>* xcd, std::vector<int64_t>* pos) {
  xcd->assign((size_t)nslots, 0);
  pos->assign((size_t)nslots, 0);
  const int64_t grid = stripe_grid(nslots, C), R = grid >> 3;
  for (int64_t b = 0; b < grid; b++) {  // (host restatement of stripe_tile)
    const int64_t j = b >> 3;
    const int64_t t = (C <= 0 || R <= C) ? (b & 7) * R + j : ((j / C) * 8 + (b & 7)) * C + j % C;
    if (t < nslots) (*xcd)[t] = (int)(b & 7), (*pos)[t] = j;
  }
}

hipError_t launch_copy_buf(void* dst, const void* src, int64_t bytes, hipStream_t s) {
  if (bytes <= 0 || dst == src) return hipSuccess;
  if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) != 0)
    return hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, s);
  // TIPS_COPY_BUF_VARIANT (a sweep knob, read once; tools/copy_buf_sweep.sh): 0 = 4 KiB tiles, sc1
  // stores (shipped: 0.81-0.83 of HBM on config 3's 1 GiB, profiles/r04/z_copy_buf_sweep.txt);
  // 1 = 8 KiB tiles (0.71-0.75); 2 = 16 KiB tiles (0.73); 3 = 4 KiB tiles, nt stores;
  // 4 = hipMemcpyAsync (0.59-0.65); 5 / 6 = 128-lane workgroups (2 KiB tiles), sc1 / nt stores
  // (round 6: the 2-input sum's shipped shape)
  static const int variant = [] {
    const char* v = getenv("TIPS_COPY_BUF_VARIANT");
    return v && *v ? atoi(v) : 0;
  }();
  if (variant == 4) return hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, s);
  const int U = variant == 1 ? 2 : variant == 2 ? 4 : 1;
  const int64_t B = (variant == 5 || variant == 6) ? 128 : kBlock;
  const int64_t nvec = bytes / 16;
  const int64_t stripe = stripe_of(B * U);
  const int64_t grid = stripe_grid((nvec + B * U - 1) / (B * U), stripe);
  if (grid > 0x7fffffff) return hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, s);
  const dim3 g((unsigned)grid), b((unsigned)B);
  if (variant == 5)
    hipLaunchKernelGGL((copy_buf_kernel<1, 16, 128>), g, b, 0, s, (u32x4*)dst, (const u32x4*)src, nvec, nvec * 16, bytes, stripe);
  else if (variant == 6)
    hipLaunchKernelGGL((copy_buf_kernel<1, 2, 128>), g, b, 0, s, (u32x4*)dst, (const u32x4*)src, nvec, nvec * 16, bytes, stripe);
  else if (variant == 1)
    hipLaunchKernelGGL((copy_buf_kernel<2>), g, b, 0, s, (u32x4*)dst, (const u32x4*)src, nvec, nvec * 16, bytes, stripe);
  else if (variant == 2)
    hipLaunchKernelGGL((copy_buf_kernel<4>), g, b, 0, s, (u32x4*)dst, (const u32x4*)src, nvec, nvec * 16, bytes, stripe);
  else if (variant == 3)
    hipLaunchKernelGGL((copy_buf_kernel<1, 2>), g, b, 0, s, (u32x4*)dst, (const u32x4*)src, nvec, nvec * 16, bytes, stripe);
  else
    hipLaunchKernelGGL((copy_buf_kernel<1>), g, b, 0, s, (u32x4*)dst, (const u32x4*)src, nvec, nvec * 16, bytes, stripe);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Segment copy (fusion pack / unpack / identity copy since round 3; fusion.cc)
//
// Tiles are cut from a virtual byte space (a fusion bucket, or the flat layout of a whole tensor
// list), not per tensor: every workgroup moves T = 4 KiB x U bytes of the space, whatever tensors
// it meets; only the padding between tensors (< 256 B each) is skipped. The round-2 kernel cut
// tiles per tensor, so ~75 % of config 4's 1000 tensors ended in a partly empty workgroup, and
// moved a tile's last < 16 bytes one byte per lane. Tensors begin 256-B aligned in the space, so a
// tile meets at most T / 256 + 1 segments: the workgroup stages them in LDS (one load per lane,
// one barrier), each lane finds the segment of each of its 16-B vectors by binary search, issues
// all its nt loads, then its stores. A vector at a tensor's ragged end, or of a tensor that is not
// 16-B aligned, moves as dwords (shorts for 2-B element types) - one lane per tensor end.
// (The addresses are built from integers, so they are cast to the global address space: a generic
// pointer makes the compiler emit flat_load / flat_store, which also count against lgkmcnt.)
typedef __attribute__((address_space(1))) u32x4 g_u32x4;
typedef __attribute__((address_space(1))) unsigned g_u32;
typedef __attribute__((address_space(1))) unsigned short g_u16;
typedef __attribute__((address_space(1))) char g_u8;

template <int POL>
__device__ __forceinline__ void store16_pol(int64_t d, u32x4 x) {
  if constexpr (POL == 0) {
    *reinterpret_cast<g_u32x4*>(d) = x;
  } else if constexpr (POL == 1) {
    __builtin_nontemporal_store(x, reinterpret_cast<g_u32x4*>(d));
  } else {  // sc1: the line leaves the XCD's L2 (a vector store; the asm ends with the store's 2 wait states)
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(reinterpret_cast<g_u32x4*>(d)), "v"(x)
                 : "memory");
  }
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) u32x2 g_u32x2;

// the 8-B form (the wire side of the cast kernels: 4 half-width elements per lane)
__device__ __forceinline__ void store8_sc1(int64_t d, u32x2 x) {
  asm volatile("global_store_dwordx2 %0, %1, off sc1\n\ts_nop 1" ::"v"(reinterpret_cast<g_u32x2*>(d)), "v"(x)
               : "memory");
}

// The < 16 bytes of a vector at a tensor's ragged end, or a whole vector of a tensor that is not
// 16-B aligned: loaded as dwords (shorts when the tensor's offset or length is only 2-B aligned,
// 16-bit types) - phase 1 issues the loads, phase 2 the stores, so a lane waits for memory once.
struct Small {
  unsigned w[4];
  unsigned short h[8];
};

__device__ __forceinline__ void small_load(int64_t s, int64_t d, int len, Small& m) {
  if (((s | d | (int64_t)len) & 3) == 0) {
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (4 * k < len) m.w[k] = *reinterpret_cast<const g_u32*>(s + 4 * k);
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++)
      if (2 * k < len) m.h[k] = *reinterpret_cast<const g_u16*>(s + 2 * k);
  }
}

__device__ __forceinline__ void small_store(int64_t s, int64_t d, int len, const Small& m) {
  if (((s | d | (int64_t)len) & 3) == 0) {
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (4 * k < len) *reinterpret_cast<g_u32*>(d + 4 * k) = m.w[k];
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++)
      if (2 * k < len) *reinterpret_cast<g_u16*>(d + 2 * k) = m.h[k];
  }
}

// tiles[2t], tiles[2t + 1] (record slot t of the launch; fusion.cc puts a group's boundary tiles
// first): the tile's segment and {0, 0, tile byte, 0}; or its two segments (the tensor ending in
// it, the tensor starting in it); or {first segment, count, -, -1} and {0, 0, tile byte, 0} when
// it meets more than two (then staged from segs[] in LDS).
template <int U>
struct SegStage {  // a multi-segment tile's records, staged in LDS
  CopySeg L[(int)((int64_t)kBlock * 16 * U / 256) + 1];
};

// One tile of the segment copy: record slot t. Called by whole workgroups (the multi-segment
// branch has a barrier; every branch to it is workgroup-uniform).
template <int U, int POL>
__device__ __forceinline__ void copy_seg_tile(const CopySeg* __restrict__ tiles, const CopySeg* __restrict__ segs,
                                              int t, CopySeg* L) {
  constexpr int64_t kTileBytes = (int64_t)kBlock * 16 * U;
  constexpr int kMaxSeg = (int)(kTileBytes / 256) + 1;
  // One (scalar) load of both records before the first data load. (A tile -> segment index
  // followed by the segment's record puts two dependent loads there: 17.5 against 14.1 us per
  // config-4 bucket, measured.)
  // (field by field: a record selected as a whole per lane becomes a private-memory copy)
  const int64_t* tr = reinterpret_cast<const int64_t*>(tiles + 2 * (int64_t)t);
  const int64_t a_src = tr[0], a_dst = tr[1], a_beg = tr[2], a_end = tr[3];
  const int64_t b_src = tr[4], b_dst = tr[5], b_beg = tr[6], b_end = tr[7];
  const int tid = threadIdx.x;
  const bool multi = a_end < 0, two = b_end > 0;
  // the tile's first byte: the second record's begin, rounded down to the tile when that record is
  // the segment starting inside the tile
  const int64_t tb = two ? (b_beg & ~(kTileBytes - 1)) : b_beg;
  if (!multi && !two && a_beg <= tb && a_end >= tb + kTileBytes && ((a_src | a_dst) & 15) == 0) {
    // the tile lies inside one 16-B aligned tensor (most tiles): both sides are wave-uniform
    // contiguous ranges, moved as the round-2 kernel moved a whole tile - buffer loads nt, buffer
    // stores with the policy's cache bits, each store behind its own load
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(a_src + tb), (short)0, (int)kTileBytes,
                                                                  0x00020000);
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)(a_dst + tb), (short)0, (int)kTileBytes,
                                                                  0x00020000);
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (u * kBlock + tid) * 16, 0, 2);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, (u * kBlock + tid) * 16, 0, POL == 0 ? 0 : POL == 1 ? 2 : 16);
    return;
  }
  int cnt = 1;
  if (multi) {  // workgroup-uniform branch
    const int s0 = (int)a_src;
    cnt = min((int)a_dst, kMaxSeg);
    if (cnt <= 0) return;  // (uniform: no segment meets this tile)
    if (tid < cnt) L[tid] = segs[s0 + tid];
    __syncthreads();
  }
  int64_t sp[U], dp[U];
  int len[U];
  bool full[U];
  u32x4 x[U];
  Small m[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const int64_t v = tb + (int64_t)u * (kBlock * 16) + (int64_t)tid * 16;
    int64_t g_src, g_dst, g_beg, g_end;
    if (multi) {
      int lo = 0, hi = cnt - 1;  // the last segment beginning at or before v
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (L[mid].begin <= v) lo = mid;
        else hi = mid - 1;
      }
      g_src = L[lo].src;
      g_dst = L[lo].dst;
      g_beg = L[lo].begin;
      g_end = L[lo].end;
    } else {
      const bool b = two && v >= b_beg;
      g_src = b ? b_src : a_src;
      g_dst = b ? b_dst : a_dst;
      g_beg = b ? b_beg : a_beg;
      g_end = b ? b_end : a_end;
    }
    const int64_t left = g_end - v;
    len[u] = (v >= g_beg && left > 0) ? (int)(left < 16 ? left : 16) : 0;
    sp[u] = g_src + v;
    dp[u] = g_dst + v;
    full[u] = len[u] == 16 && ((sp[u] | dp[u]) & 15) == 0;
    if (full[u]) x[u] = __builtin_nontemporal_load(reinterpret_cast<const g_u32x4*>(sp[u]));
    else if (len[u] > 0) small_load(sp[u], dp[u], len[u], m[u]);
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    if (full[u]) store16_pol<POL>(dp[u], x[u]);
    else if (len[u] > 0) small_store(sp[u], dp[u], len[u], m[u]);
  }
}

template <int U, int POL>
__global__ __launch_bounds__(kBlock) void copy_segs_kernel(const CopySeg* __restrict__ tiles,
                                                          const CopySeg* __restrict__ segs, int tile0, int ntiles,
                                                          int64_t stripe) {
  __shared__ SegStage<U> st;
  const int64_t tt = stripe_tile(blockIdx.x, gridDim.x, stripe);
  if (tt >= ntiles) return;  // (whole workgroup: before any barrier)
  copy_seg_tile<U, POL>(tiles, segs, tile0 + (int)tt, st.L);  // (fusion.cc may order a group's tiles: slow ones first)
}

// ---------------------------------------------------------------------------
// Fusion pack / unpack with a cast (Compression.fp16 fused into the buckets):
// the layout's byte space is the WIRE type's (f16 or bf16, 2 B per element); the f32 side of a
// segment lives at base + 2 v for virtual byte v (fusion.cc's kSlotCast records). DIR 0 (pack):
// f32 source -> wire destination, RNE as oracle_float_to_half / oracle_float_to_bf16 (the
// reference's tf.cast, compression.py:49-66); DIR 1 (unpack): wire source -> f32 destination, exact.
// A lane moves quads: 4 elements = 16 B of f32 and 8 B of the wire type, so every access of a
// wave is one contiguous run (1 KiB of f32, 512 B of wire). (Round 6's first form moved 8 elements
// per lane as one 16-B wire vector and two 16-B f32 accesses 32 B apart: each f32 instruction then
// touched every other 16 B of a 2 KiB span, and config 5's round trip ran at 0.44 of HBM, the
// unpack at 0.37; profiles/r06/cast_probe_*.)

template <int WT>
__device__ __forceinline__ u32x2 narrow4(f32x4 a) {
  if constexpr (WT == kF16) {
    return __builtin_bit_cast(u32x2, __builtin_convertvector(a, f16x4));
  } else {  // bf16: word i = elements 2i (low half) and 2i + 1 (high half)
    const u32x4 x = __builtin_bit_cast(u32x4, a);
    return u32x2{bf16_round_bits(x[0]) | (bf16_round_bits(x[1]) << 16), bf16_round_bits(x[2]) | (bf16_round_bits(x[3]) << 16)};
  }
}

template <int WT>
__device__ __forceinline__ f32x4 widen4(u32x2 v) {
  if constexpr (WT == kF16) return __builtin_convertvector(__builtin_bit_cast(f16x4, v), f32x4);
  else return __builtin_bit_cast(f32x4, u32x4{v[0] << 16, v[0] & 0xffff0000u, v[1] << 16, v[1] & 0xffff0000u});
}

template <int WT>
__device__ __forceinline__ unsigned short narrow1(float f) {
  if constexpr (WT == kF16) return __builtin_bit_cast(unsigned short, (_Float16)f);
  else return (unsigned short)bf16_round_bits(__builtin_bit_cast(unsigned, f));
}

template <int WT>
__device__ __forceinline__ float widen1(unsigned short h) {
  if constexpr (WT == kF16) return (float)__builtin_bit_cast(_Float16, h);
  else return __builtin_bit_cast(float, (unsigned)h << 16);
}

typedef __attribute__((address_space(1))) f32x4 g_f32x4;
typedef __attribute__((address_space(1))) float g_f32;

// One whole tile of kBlock * 16 * U wire bytes, both sides 16-B aligned, moved 16 B per lane on
// both sides: the quads (16 B of f32 = 8 B of wire) are reordered through LDS, so the wire side is
// read or written as 16-B vectors too (8-B-per-lane wire accesses ran the round trip 10 % slower:
// profiles/r06/cast/). Called by whole workgroups; W holds 2 U quads per lane.
template <int U, int DIR, int WT>
__device__ __forceinline__ void cast_tile_staged(int64_t f32_base, int64_t wire_base, u32x2* W) {
  const int tid = threadIdx.x;
  if constexpr (DIR == 0) {
    f32x4 x[2 * U];
#pragma unroll
    for (int u = 0; u < 2 * U; u++)
      x[u] = __builtin_nontemporal_load(reinterpret_cast<const g_f32x4*>(f32_base + 16 * (int64_t)(u * kBlock + tid)));
#pragma unroll
    for (int u = 0; u < 2 * U; u++) W[u * kBlock + tid] = narrow4<WT>(x[u]);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < U; u++)
      store16_pol<2>(wire_base + 16 * (int64_t)(u * kBlock + tid), reinterpret_cast<const u32x4*>(W)[u * kBlock + tid]);
  } else {
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      x[u] = __builtin_nontemporal_load(reinterpret_cast<const g_u32x4*>(wire_base + 16 * (int64_t)(u * kBlock + tid)));
#pragma unroll
    for (int u = 0; u < U; u++) reinterpret_cast<u32x4*>(W)[u * kBlock + tid] = x[u];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2 * U; u++)
      store16_pol<2>(f32_base + 16 * (int64_t)(u * kBlock + tid), __builtin_bit_cast(u32x4, widen4<WT>(W[u * kBlock + tid])));
  }
}

// VAR (sweeps, TIPS_CAST_VARIANT): bit 0 plain loads instead of nt; bits 1-2 the store policy
// (0 = sc1, the default; 1 = plain; 2 = nt); bit 3 (the default) one-segment tiles staged in LDS
// (cast_tile_staged); the other tiles move quads (staging the two-segment and ragged tiles
// as well was measured no faster on config 4's 1000 tensors: 49.41 vs 49.44 us per round trip)
template <int U, int DIR, int WT, int VAR = 8>
__global__ __launch_bounds__(kBlock) void cast_segs_kernel(const CopySeg* __restrict__ tiles,
                                                          const CopySeg* __restrict__ segs, int tile0, int ntiles) {
  constexpr int64_t kTileBytes = (int64_t)kBlock * 16 * U;  // wire bytes
  constexpr int kMaxSeg = (int)(kTileBytes / 256) + 1;
  constexpr int Q = 2 * U;  // quads per lane
  __shared__ CopySeg L[kMaxSeg];
  const int64_t tt = xcd_tile(blockIdx.x, gridDim.x);
  if (tt >= ntiles) return;  // (whole workgroup: before any barrier)
  const int64_t* tr = reinterpret_cast<const int64_t*>(tiles + 2 * (int64_t)(tile0 + tt));
  const int64_t a_src = tr[0], a_dst = tr[1], a_beg = tr[2], a_end = tr[3];
  const int64_t b_src = tr[4], b_dst = tr[5], b_beg = tr[6], b_end = tr[7];
  const int tid = threadIdx.x;
  const bool multi = a_end < 0, two = b_end > 0;
  const int64_t tb = two ? (b_beg & ~(kTileBytes - 1)) : b_beg;
  if constexpr ((VAR & 8) != 0) {
    // (bit 3, the default) a tile inside one segment with both sides 16-B aligned (workgroup-uniform)
    __shared__ u32x2 W[kBlock * Q];
    if (!multi && !two && a_beg <= tb && a_end >= tb + kTileBytes && ((a_src | a_dst) & 15) == 0) {
      if constexpr (DIR == 0) cast_tile_staged<U, 0, WT>(a_src + 2 * tb, a_dst + tb, W);
      else cast_tile_staged<U, 1, WT>(a_dst + 2 * tb, a_src + tb, W);
      return;
    }
  }
  int cnt = 1;
  if (multi) {  // workgroup-uniform branch
    cnt = min((int)a_dst, kMaxSeg);
    if (cnt <= 0) return;
    if (tid < cnt) L[tid] = segs[(int)a_src + tid];
    __syncthreads();
  }
  int64_t sp[Q], dp[Q];
  int len[Q];  // wire bytes of this quad inside its segment (8 = all four elements)
  bool full[Q];
  u32x2 nv[Q];  // unpack: the loaded wire quad
  f32x4 wa[Q];  // pack: the loaded f32 quad
#pragma unroll
  for (int u = 0; u < Q; u++) {
    const int64_t v = tb + (int64_t)u * (kBlock * 8) + (int64_t)tid * 8;
    int64_t g_src, g_dst, g_beg, g_end;
    if (multi) {
      int lo = 0, hi = cnt - 1;  // the last segment beginning at or before v
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (L[mid].begin <= v) lo = mid;
        else hi = mid - 1;
      }
      g_src = L[lo].src;
      g_dst = L[lo].dst;
      g_beg = L[lo].begin;
      g_end = L[lo].end;
    } else {
      const bool b = two && v >= b_beg;
      g_src = b ? b_src : a_src;
      g_dst = b ? b_dst : a_dst;
      g_beg = b ? b_beg : a_beg;
      g_end = b ? b_end : a_end;
    }
    const int64_t left = g_end - v;
    len[u] = (v >= g_beg && left > 0) ? (int)(left < 8 ? left : 8) : 0;
    sp[u] = g_src + (DIR == 0 ? 2 * v : v);  // the f32 side at base + 2 v
    dp[u] = g_dst + (DIR == 0 ? v : 2 * v);
    const int64_t f32_side = DIR == 0 ? sp[u] : dp[u], wire_side = DIR == 0 ? dp[u] : sp[u];
    full[u] = len[u] == 8 && (f32_side & 15) == 0 && (wire_side & 7) == 0;
    if (full[u]) {
      if constexpr (DIR == 0) wa[u] = (VAR & 1) ? *reinterpret_cast<const g_f32x4*>(sp[u])
                                                : __builtin_nontemporal_load(reinterpret_cast<const g_f32x4*>(sp[u]));
      else nv[u] = (VAR & 1) ? *reinterpret_cast<const g_u32x2*>(sp[u])
                             : __builtin_nontemporal_load(reinterpret_cast<const g_u32x2*>(sp[u]));
    }
  }
  constexpr int kStore = (VAR >> 1) & 3;
#pragma unroll
  for (int u = 0; u < Q; u++) {
    if (full[u]) {
      if constexpr (DIR == 0) {
        const u32x2 w = narrow4<WT>(wa[u]);
        if constexpr (kStore == 0) store8_sc1(dp[u], w);
        else if constexpr (kStore == 1) *reinterpret_cast<g_u32x2*>(dp[u]) = w;
        else __builtin_nontemporal_store(w, reinterpret_cast<g_u32x2*>(dp[u]));
      } else {
        store16_pol<kStore == 0 ? 2 : kStore == 1 ? 0 : 1>(dp[u], __builtin_bit_cast(u32x4, widen4<WT>(nv[u])));
      }
    } else {
      for (int e = 0; 2 * e < len[u]; e++) {  // a tensor's ragged end, or a side not aligned
        if constexpr (DIR == 0)
          *reinterpret_cast<g_u16*>(dp[u] + 2 * e) = narrow1<WT>(*reinterpret_cast<const g_f32*>(sp[u] + 4 * e));
        else
          *reinterpret_cast<g_f32*>(dp[u] + 4 * e) = widen1<WT>(*reinterpret_cast<const g_u16*>(sp[u] + 2 * e));
      }
    }
  }
}

// Cast of one contiguous range (a fused list's tensors of at least the threshold, which travel
// through a scratch buffer of the wire type): DIR 0 f32 -> wire, 1 wire -> f32. With both sides
// 16-B aligned, whole 8 KiB wire tiles go through cast_tile_staged (grid-stride over tiles), the
// rest in quads (16 B of f32, 8 B of wire per lane) and the last n % 4 elements one at a time; a
// misaligned range element by element.
template <int DIR, int WT>
__global__ __launch_bounds__(kBlock) void cast_range_kernel(void* __restrict__ dst, const void* __restrict__ src,
                                                           int64_t n) {
  constexpr int U = 2;
  constexpr int64_t kTileElems = (int64_t)kBlock * 8 * U;
  __shared__ u32x2 W[kBlock * 2 * U];
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t f32_side = (int64_t)(DIR == 0 ? src : dst), wire_side = (int64_t)(DIR == 0 ? dst : src);
  int64_t head = 0;
  if (((f32_side | wire_side) & 15) == 0) {
    const int64_t nt = n / kTileElems;
    for (int64_t t = blockIdx.x; t < nt; t += gridDim.x) {  // (workgroup-uniform trip count)
      cast_tile_staged<U, DIR, WT>(f32_side + 4 * t * kTileElems, wire_side + 2 * t * kTileElems, W);
      __syncthreads();  // (every lane's LDS reads before the next tile's writes)
    }
    head = nt * kTileElems;
  }
  if ((f32_side & 15) == 0 && (wire_side & 7) == 0) {
    const int64_t nq = n / 4;
    for (int64_t q = head / 4 + (int64_t)blockIdx.x * kBlock + threadIdx.x; q < nq; q += stride) {
      if constexpr (DIR == 0)
        store8_sc1(wire_side + 8 * q, narrow4<WT>(__builtin_nontemporal_load(reinterpret_cast<const g_f32x4*>(f32_side + 16 * q))));
      else
        store16_pol<2>(f32_side + 16 * q, __builtin_bit_cast(u32x4, widen4<WT>(
                                              __builtin_nontemporal_load(reinterpret_cast<const g_u32x2*>(wire_side + 8 * q)))));
    }
    head = 4 * nq;
  }
  for (int64_t i = head + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    if constexpr (DIR == 0) static_cast<unsigned short*>(dst)[i] = narrow1<WT>(static_cast<const float*>(src)[i]);
    else static_cast<float*>(dst)[i] = widen1<WT>(static_cast<const unsigned short*>(src)[i]);
  }
}

// Several groups of tiles (a step's fusion buckets) in one launch, each group a contiguous range of
// workgroups in group order, XCD-contiguous inside it: the dispatcher hands out workgroups in
// order, so group 0 is done first and its allreduce can start while the later groups are still
// being packed. The launch pays one ramp and drain instead of one per bucket.
// With done[k] set, the last workgroup of group k (a device counter per group, reset by that
// workgroup for the next launch) stores sig_value[k] into *done[k] with a system-scope release, which
// the bucket stream waits on (hipStreamWaitValue64 on signal memory, fusion.cc).
template <int U, int POL>
__global__ __launch_bounds__(kBlock) void copy_segs_groups_kernel(const CopySeg* __restrict__ tiles,
                                                                 const CopySeg* __restrict__ segs, PackGroups g) {
  __shared__ SegStage<U> st;
  int k = 0;
  while (k + 1 < g.n && blockIdx.x >= g.blk0[k + 1]) k++;
  const unsigned local = blockIdx.x - g.blk0[k], gk = g.blk0[k + 1] - g.blk0[k];
  const int64_t tt = xcd_tile(local, gk);
  if (tt < g.ntiles[k]) copy_seg_tile<U, POL>(tiles, segs, g.tile0[k] + (int)tt, st.L);
  if (g.done[k]) {
    __syncthreads();  // (every wave's copies before the workgroup's count)
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(&g.counters[k], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gk - 1) {
      __hip_atomic_store(&g.counters[k], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(g.done[k], g.sig_value[k], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// ---------------------------------------------------------------------------
// Peer transfer (xGMI peer schedule, peer.cc)

struct XferList {
  XferSeg s[kMaxXferSegs];
};

// Workgroup b copies tile b / nseg of segment b % nseg: consecutive workgroups
// (and so every XCD) cover all segments, i.e. all peers' links, at once. Each
// lane issues its four 16-B loads before any store: a remote access over xGMI
// takes microseconds, so bytes in flight, not instructions, set the rate. The
// descriptors cover exactly the tile's 16-B-multiple prefix; the < 16 bytes
// past it (a ragged last chunk) go bytewise.
__global__ __launch_bounds__(kBlock) void xfer_kernel(XferList L, int nseg) {
  constexpr int U = (int)(kXferTileBytes / (kBlock * 16));
  const int seg = (int)(blockIdx.x % (unsigned)nseg);
  const int64_t off = (int64_t)(blockIdx.x / (unsigned)nseg) * kXferTileBytes;
  const XferSeg sg = L.s[seg];
  if (off >= sg.bytes) return;
  const int64_t len = sg.bytes - off < kXferTileBytes ? sg.bytes - off : kXferTileBytes;
  const char* src = sg.src + off;
  char* dst = sg.dst + off;
  const int tid = threadIdx.x;
  if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0) {
    const int len16 = (int)(len & ~(int64_t)15);
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, len16, 0x00020000);
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)dst, (short)0, len16, 0x00020000);
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (u * kBlock + tid) * 16, 0, 0);
#pragma unroll
    for (int u = 0; u < U; u++) __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, (u * kBlock + tid) * 16, 0, 0);
    if (len16 + tid < len) dst[len16 + tid] = src[len16 + tid];
  } else {
    for (int64_t i = tid; i < len; i += kBlock) dst[i] = src[i];
  }
}

// ---------------------------------------------------------------------------
// Launchers

namespace {

constexpr int kNumCUs = 256;

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

template <int DT, int MODE, int UNROLL, bool NTL, bool NTS, int BLOCK>
hipError_t run_sum2(void* dst, const void* a, const void* b, int64_t n, int blocks, hipStream_t s) {
  const int64_t ve = 16 / (int64_t)dtype_size(DT);
  const int64_t nvec = n / ve;
  const int64_t tiles = (nvec + (int64_t)BLOCK * UNROLL - 1) / ((int64_t)BLOCK * UNROLL);
  int64_t grid = (MODE != 0) ? tiles : (blocks > 0 ? blocks : kNumCUs * 8);
  if (grid > tiles) grid = tiles;
  if (grid < 1) grid = 1;
  if (MODE == 2) grid = (grid + 7) / 8 * 8;  // whole XCD rounds; surplus tiles fall off the bounds checks
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL((sum2_kernel<DT, MODE, UNROLL, NTL, NTS, BLOCK>), dim3((unsigned)grid), dim3(BLOCK), 0, s,
                     (u32x4*)dst, (const u32x4*)a, (const u32x4*)b, nvec, nvec * ve, n);
  return hipGetLastError();
}

// nt: 0 = plain, 1 = non-temporal loads and stores, 2 = nt loads only, 3 = nt stores only
template <int DT>
hipError_t sum2_dispatch(void* dst, const void* a, const void* b, int64_t n, int mode, int unroll, int nt, int blocks,
                         int threads, hipStream_t s) {
  if (!(aligned16(dst) && aligned16(a) && aligned16(b))) {
    int64_t grid = (n + kBlock - 1) / kBlock;
    if (grid > kNumCUs * 16) grid = kNumCUs * 16;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((sum2_scalar_kernel<DT>), dim3((unsigned)grid), dim3(kBlock), 0, s, dst, a, b, n);
    return hipGetLastError();
  }
#ifdef TIPS_DEV  // (tuning sweeps: libtips_hip_dev.so only)
  if (mode == 5) {  // persistent streaming, f32, 256 threads; unroll = workgroups per CU (grid = 256 x unroll)
    if constexpr (DT == kF32) {
      if (threads == 256 && (unroll == 1 || unroll == 2 || unroll == 4 || unroll == 8)) {
        const int64_t nvec = n / 4;
        hipLaunchKernelGGL(sum2_stream_kernel, dim3((unsigned)(kNumCUs * unroll)), dim3(256), 0, s, (u32x4*)dst,
                           (const u32x4*)a, (const u32x4*)b, nvec, nvec * 4, n);
        return hipGetLastError();
      }
    }
    return hipErrorInvalidValue;
  }
  if (mode == 6) {  // other tile maps, f32, 256 threads; unroll = stripe in KiB of one operand (0: address order)
    if constexpr (DT == kF32) {
      const int64_t nvec = n / 4, T = (nvec + 255) / 256;
      const int64_t stripe = (int64_t)unroll * 1024 / 4096;  // tiles of 4 KiB
      if (unroll < 0 || (unroll > 0 && stripe < 1)) return hipErrorInvalidValue;
      const int64_t grid = stripe == 0 ? std::max<int64_t>(1, T) : ((T + stripe - 1) / stripe + 7) / 8 * 8 * stripe;
      hipLaunchKernelGGL(sum2_map_kernel, dim3((unsigned)grid), dim3(256), 0, s, (u32x4*)dst, (const u32x4*)a,
                         (const u32x4*)b, nvec, nvec * 4, n, stripe);
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  if (mode == 4) {  // LDS-staged (direct-to-LDS loads), f32, 256 threads; unroll = 16-B vectors per lane
    if constexpr (DT == kF32) {
      const int64_t nvec = n / 4;
      auto grid_for = [&](int64_t tile) { return (unsigned)std::max<int64_t>(8, ((nvec + tile - 1) / tile + 7) / 8 * 8); };
      if (threads == 256 && unroll == 1) {
        hipLaunchKernelGGL((sum2_lds_kernel<1>), dim3(grid_for(256)), dim3(256), 0, s, (u32x4*)dst, (const u32x4*)a,
                           (const u32x4*)b, nvec, nvec * 4, n);
        return hipGetLastError();
      }
      if (threads == 256 && unroll == 2) {
        hipLaunchKernelGGL((sum2_lds_kernel<2>), dim3(grid_for(512)), dim3(256), 0, s, (u32x4*)dst, (const u32x4*)a,
                           (const u32x4*)b, nvec, nvec * 4, n);
        return hipGetLastError();
      }
      if (threads == 256 && unroll == 4) {
        hipLaunchKernelGGL((sum2_lds_kernel<4>), dim3(grid_for(1024)), dim3(256), 0, s, (u32x4*)dst, (const u32x4*)a,
                           (const u32x4*)b, nvec, nvec * 4, n);
        return hipGetLastError();
      }
    }
    return hipErrorInvalidValue;
  }
#endif  // TIPS_DEV
#define TIPS_SUM2_CASE(M, U, NTV, L, S_, B)                      \
  if (mode == M && unroll == U && nt == NTV && threads == B) \
    return run_sum2<DT, M, U, L, S_, B>(dst, a, b, n, blocks, s);
  if (mode == 3) {  // buffer-op variants: nt = index into (load aux, store aux); unroll x threads = tile
    const int64_t ve = 16 / (int64_t)dtype_size(DT);
    const int64_t nvec = n / ve;
    // blocks > 0: that many bytes of (unused) LDS reserved per workgroup, capping workgroups per CU
    // at 160 KiB / blocks (the occupancy sweep); 0 = no cap
    if (blocks < 0 || blocks > 65536) return hipErrorInvalidValue;
    const unsigned shmem = (unsigned)blocks;
#define TIPS_BUF_CASE(I, L, S_, U, B)                                                                          \
  if (nt == I && unroll == U && threads == B) {                                                            \
    hipLaunchKernelGGL((sum2_buf_kernel<DT, L, S_, U, B>),                                                    \
                       dim3((unsigned)stripe_grid((nvec + U * B - 1) / (U * B), sum_stripe_of(U * B))), dim3(B), shmem, s, \
                       (u32x4*)dst, (const u32x4*)a, (const u32x4*)b, nvec, nvec * ve, n, sum_stripe_of(U * B));      \
    return hipGetLastError();                                                                              \
  }
    TIPS_BUF_CASE(7, 2, 2, 1, 128)   // the product default (round 6): nt loads, nt stores, 1 x 16 B per lane, 128 lanes
    TIPS_BUF_CASE(1, 2, 16, 1, 256)  // rounds 2-5's default: nt loads, sc1 stores, 256 lanes
#ifdef TIPS_DEV  // (tuning sweeps: libtips_hip_dev.so only)
    if constexpr (DT == kF32) {
      TIPS_BUF_CASE(0, 2, 0, 1, 256)
      TIPS_BUF_CASE(2, 2, 17, 1, 256)
      TIPS_BUF_CASE(3, 18, 0, 1, 256)
      TIPS_BUF_CASE(4, 3, 0, 1, 256)
      TIPS_BUF_CASE(5, 16, 0, 1, 256)
      TIPS_BUF_CASE(6, 18, 16, 1, 256)
      TIPS_BUF_CASE(7, 2, 2, 1, 256)
      TIPS_BUF_CASE(8, 0, 16, 1, 256)
      TIPS_BUF_CASE(9, 3, 17, 1, 256)
      TIPS_BUF_CASE(1, 2, 16, 2, 256)
      TIPS_BUF_CASE(1, 2, 16, 4, 256)
      TIPS_BUF_CASE(1, 2, 16, 1, 512)
      TIPS_BUF_CASE(1, 2, 16, 2, 128)
      TIPS_BUF_CASE(1, 2, 16, 1, 1024)
      TIPS_BUF_CASE(1, 2, 16, 1, 128)
      TIPS_BUF_CASE(7, 2, 2, 1, 64)   // (round 6: one wave per workgroup, nt stores)
      TIPS_BUF_CASE(7, 2, 2, 2, 128)  // (round 6: 128 lanes, 2 vectors per lane, nt stores)
      TIPS_BUF_CASE(1, 2, 16, 2, 512)
      TIPS_BUF_CASE(7, 2, 2, 1, 512)  // nt loads + nt stores, other tile shapes (rotating-buffer sweep)
      TIPS_BUF_CASE(7, 2, 2, 1, 1024)
      TIPS_BUF_CASE(7, 2, 2, 2, 256)
      TIPS_BUF_CASE(7, 2, 2, 4, 256)
      TIPS_BUF_CASE(7, 2, 2, 2, 512)
      TIPS_BUF_CASE(10, 2, 18, 1, 256)  // nt loads; stores nt sc1, sc0 nt sc1, sc0, sc0 nt
      TIPS_BUF_CASE(11, 2, 19, 1, 256)
      TIPS_BUF_CASE(12, 2, 1, 1, 256)
      TIPS_BUF_CASE(13, 2, 3, 1, 256)
    }
#endif  // TIPS_DEV
#undef TIPS_BUF_CASE
    return hipErrorInvalidValue;
  }
#ifdef TIPS_DEV  // (tuning sweeps: libtips_hip_dev.so only)
  // global_load/store forms: the tuning sweep's other variants (f32 only)
  if constexpr (DT == kF32) {
    TIPS_SUM2_CASE(2, 1, 2, true, false, 256)
    TIPS_SUM2_CASE(1, 1, 2, true, false, 256)
    TIPS_SUM2_CASE(1, 4, 1, true, true, 256)
    TIPS_SUM2_CASE(1, 2, 2, true, false, 256)
    TIPS_SUM2_CASE(1, 8, 2, true, false, 256)
    TIPS_SUM2_CASE(1, 2, 2, true, false, 512)
    TIPS_SUM2_CASE(1, 2, 2, true, false, 128)
    TIPS_SUM2_CASE(1, 1, 2, true, false, 512)
    TIPS_SUM2_CASE(0, 2, 2, true, false, 256)
    TIPS_SUM2_CASE(0, 4, 2, true, false, 256)
    TIPS_SUM2_CASE(2, 2, 2, true, false, 256)
    TIPS_SUM2_CASE(2, 1, 2, true, false, 512)
    TIPS_SUM2_CASE(2, 4, 1, true, true, 256)
    TIPS_SUM2_CASE(1, 1, 0, false, false, 256)
    TIPS_SUM2_CASE(1, 2, 0, false, false, 256)
    TIPS_SUM2_CASE(1, 4, 0, false, false, 256)
    TIPS_SUM2_CASE(1, 8, 0, false, false, 256)
    TIPS_SUM2_CASE(1, 1, 1, true, true, 256)
    TIPS_SUM2_CASE(1, 2, 1, true, true, 256)
    TIPS_SUM2_CASE(1, 8, 1, true, true, 256)
    TIPS_SUM2_CASE(0, 1, 0, false, false, 256)
    TIPS_SUM2_CASE(0, 2, 0, false, false, 256)
    TIPS_SUM2_CASE(0, 4, 0, false, false, 256)
    TIPS_SUM2_CASE(0, 8, 0, false, false, 256)
    TIPS_SUM2_CASE(0, 1, 1, true, true, 256)
    TIPS_SUM2_CASE(0, 2, 1, true, true, 256)
    TIPS_SUM2_CASE(0, 4, 1, true, true, 256)
    TIPS_SUM2_CASE(0, 8, 1, true, true, 256)
    TIPS_SUM2_CASE(1, 4, 2, true, false, 256)
    TIPS_SUM2_CASE(1, 2, 3, false, true, 256)
    TIPS_SUM2_CASE(1, 4, 3, false, true, 256)
    TIPS_SUM2_CASE(1, 2, 1, true, true, 512)
    TIPS_SUM2_CASE(1, 4, 1, true, true, 512)
    TIPS_SUM2_CASE(1, 8, 1, true, true, 512)
    TIPS_SUM2_CASE(1, 1, 1, true, true, 1024)
    TIPS_SUM2_CASE(1, 2, 1, true, true, 1024)
    TIPS_SUM2_CASE(1, 4, 1, true, true, 1024)
    TIPS_SUM2_CASE(1, 4, 2, true, false, 512)
    TIPS_SUM2_CASE(1, 4, 3, false, true, 512)
    TIPS_SUM2_CASE(1, 16, 1, true, true, 256)
    TIPS_SUM2_CASE(1, 16, 1, true, true, 128)
    TIPS_SUM2_CASE(1, 8, 1, true, true, 128)
    TIPS_SUM2_CASE(1, 4, 1, true, true, 128)
    TIPS_SUM2_CASE(1, 8, 1, true, true, 64)
  }
#endif  // TIPS_DEV
#undef TIPS_SUM2_CASE
  return hipErrorInvalidValue;
}

// Default variant for the product path (chosen from the gfx950 sweeps): buffer ops,
// one 16-B vector per lane, 128-lane workgroups (a 2 KiB tile of each operand), nt loads and nt
// stores. Rounds 2-5 shipped 256 lanes with sc1 stores (nt index 1); under XCD stripes the
// 128-lane nt form is 1-3 % faster (profiles/r06/sum2_focus/).
constexpr int kDefMode = 3, kDefUnroll = 1, kDefNT = 7, kDefThreads = 128;

// Bytes the fold keeps in flight per CU (round 5, profiles/r05/): every wave-source pair has one
// 1 KiB wave-load outstanding, and with 9 streams the DRAM efficiency falls once a CU holds much more
// than the ~64 KiB the 2-input sum keeps in flight. Unused LDS reserved per workgroup caps the
// workgroups per CU (160 KiB / reservation): NSRC >= 6, 128 lanes x 5 workgroups = 10 waves
// (80 KiB for 8 sources: 8 x 32 MiB 48.1-49.2 -> 46.9-47.5 us on the sweep's boxes); NSRC 4-5,
// 128 lanes x 8 = 16 waves. 2-3 sources run uncapped (256 lanes x 8 = 32 waves: capping slowed
// 2 x 128 MiB). The reservation leaves the CU at least one RCCL transfer workgroup's worth (19.5
// KiB) at 5 workgroups; uncapped, the fold's 32 waves fill every wave slot anyway.
constexpr int kFoldLdsCap5 = 27648;  // floor(160 KiB / 27648) = 5, 25 KiB left
constexpr int kFoldLdsCap8 = 20480;  // 8

// The capped fold's store policy (TIPS_FOLD_STORE: sc1, the default, or nt; read once). The
// round-5 sweep under eighths found nt stores slower (0.72-0.74 vs 0.78-0.80); an A/B knob for
// the stripe map.
inline bool fold_store_nt() {
  static const bool v = [] {
    const char* e = getenv("TIPS_FOLD_STORE");
    return e && e[0] == 'n' && e[1] == 't' && e[2] == 0;
  }();
  return v;
}

template <int DT, int NSRC>
hipError_t run_multi(void* dst, const SrcList& sl, int64_t n, hipStream_t s) {
  // buffer loads, non-temporal for every source count. Round 1 kept plain loads beyond 4 sources
  // from a sweep that re-read one buffer set (plain 44.7 vs nt 47.3 us, 8 x 32 MiB, Infinity Cache
  // assisted); with operands from HBM, as the direct schedule's fold mostly reads them, nt wins
  // 48.6 vs 57.8 us (profiles/r02/multi_sum_variants.jsonl).
  constexpr int LAUX = 2;
  const int64_t ve = 16 / (int64_t)dtype_size(DT);
  const int64_t nvec = n / ve;
  const int64_t bytes = nvec * 16;
  // 4 vectors per lane for many sources of 3-12 MiB each (8 x 4 MiB: 7.0 vs 8.3 us, 8 x 8 MiB:
  // 12.6 vs 14.3 us; up to 4 sources, 1 vector wins or ties: profiles/r02/multi_sum_small.jsonl)
  const bool u4 = NSRC > 4 && bytes >= (3 << 20) && bytes <= (12 << 20);
  const bool capped = NSRC >= 4 && !u4 && bytes > (12 << 20);
  constexpr int kCapBlock = 128;
  const int block = capped ? kCapBlock : kBlock;
  const int64_t per = (int64_t)block * (u4 ? 4 : 1);
  const int64_t stripe = stripe_of(per);
  const int64_t grid = stripe_grid((nvec + per - 1) / per, stripe);  // surplus workgroups fall off the bounds check
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  if (capped && fold_store_nt())
    hipLaunchKernelGGL((multi_sum_buf_kernel<DT, NSRC, 1, LAUX, kCapBlock, 2>), dim3((unsigned)grid), dim3(kCapBlock),
                       NSRC >= 6 ? kFoldLdsCap5 : kFoldLdsCap8, s, (u32x4*)dst, sl, nvec, nvec * ve, n, stripe);
  else if (capped)
    hipLaunchKernelGGL((multi_sum_buf_kernel<DT, NSRC, 1, LAUX, kCapBlock>), dim3((unsigned)grid), dim3(kCapBlock),
                       NSRC >= 6 ? kFoldLdsCap5 : kFoldLdsCap8, s, (u32x4*)dst, sl, nvec, nvec * ve, n, stripe);
  else if (u4)
    hipLaunchKernelGGL((multi_sum_buf_kernel<DT, NSRC, 4, LAUX>), dim3((unsigned)grid), dim3(kBlock), 0, s,
                       (u32x4*)dst, sl, nvec, nvec * ve, n, stripe);
  else
    hipLaunchKernelGGL((multi_sum_buf_kernel<DT, NSRC, 1, LAUX>), dim3((unsigned)grid), dim3(kBlock), 0, s,
                       (u32x4*)dst, sl, nvec, nvec * ve, n, stripe);
  return hipGetLastError();
}

#ifdef TIPS_DEV  // (tuning sweeps: libtips_hip_dev.so only)
template <int NSRC, int U, int SAUX, int ORDER, int ITER, int ROT, int BLOCK>
hipError_t launch_multi_x(void* dst, const SrcList& sl, int64_t nvec, int64_t n, unsigned shmem, hipStream_t s) {
  const int64_t per = (int64_t)BLOCK * U * ITER;
  int64_t grid = (nvec + per - 1) / per;
  grid = std::max<int64_t>(8, (grid + 7) / 8 * 8);
  if (ORDER == 2 && (grid >> 3) >= 64) grid = (grid + 63) / 64 * 64;  // every XCD's stretch splits into 8 runs
  hipLaunchKernelGGL((multi_sum_x_kernel<NSRC, U, SAUX, ORDER, ITER, ROT, BLOCK>), dim3((unsigned)grid), dim3(BLOCK),
                     shmem, s, (u32x4*)dst, sl, nvec, nvec * 4, n);
  return hipGetLastError();
}

template <int NSRC, int BLOCK, int PIPE>
hipError_t launch_multi_gs(void* dst, const SrcList& sl, int64_t nvec, int64_t n, int wpc, hipStream_t s) {
  const int64_t tiles = (nvec + BLOCK - 1) / BLOCK;
  const int64_t grid = std::max<int64_t>(8, std::min<int64_t>((int64_t)kNumCUs * wpc, (tiles + 7) / 8 * 8));
  hipLaunchKernelGGL((multi_sum_gs_kernel<NSRC, BLOCK, PIPE>), dim3((unsigned)grid), dim3(BLOCK), 0, s, (u32x4*)dst, sl,
                     nvec, nvec * 4, n);
  return hipGetLastError();
}

// Round-5 variants (f32), all nt loads: 8 = address-order tiles; 9 = nt stores; 10 = plain stores;
// 11 / 12 = 2 / 4 consecutive tiles per workgroup in turn; 13 / 14 = 512 / 128 lanes; 15 = load
// order rotated per workgroup; 16 = XCD stretches cut into 8 interleaved runs; 17 / 18 / 19 =
// 20 / 40 / 27 KiB of unused LDS per workgroup (8 / 4 / 5 workgroups per CU); 20 = address order,
// 4 tiles per workgroup; 21 = the shipped shape through this kernel (control); 22 = address order,
// 2 vectors per lane; 23 / 24 / 25 = 80 / 53 / 32 KiB of LDS (2 / 3 / 5 workgroups per CU);
// 26 / 27 / 30 / 34 = 128 lanes with 40 / 20 / 27 / 13 KiB (4 / 8 / 5 / 12 workgroups per CU);
// 28 / 29 = 2 vectors per lane with 40 / 80 KiB; 31 = address order with 40 KiB; 32 / 33 = 64
// lanes, uncapped / 10 KiB (16 per CU); 35 = 128 lanes, 2 vectors, 20 KiB; 40-49 = the grid-stride
// form (multi_sum_gs_kernel): 128 lanes x 4 / 5 / 6 / 8 / 12 workgroups per CU (40-43, 48), the
// same pipelined x 4 / 5 / 3 (44, 45, 49); 256 lanes x 3 (46), pipelined x 2 (47).
template <int NSRC>
hipError_t run_multi_x(void* dst, const SrcList& sl, int64_t n, int variant, hipStream_t s) {
  const int64_t nvec = n / 4;
  switch (variant) {
    case 8: return launch_multi_x<NSRC, 1, 16, 1, 1, 0, 256>(dst, sl, nvec, n, 0, s);
    case 9: return launch_multi_x<NSRC, 1, 2, 0, 1, 0, 256>(dst, sl, nvec, n, 0, s);
    case 10: return launch_multi_x<NSRC, 1, 0, 0, 1, 0, 256>(dst, sl, nvec, n, 0, s);
    case 11: return launch_multi_x<NSRC, 1, 16, 0, 2, 0, 256>(dst, sl, nvec, n, 0, s);
    case 12: return launch_multi_x<NSRC, 1, 16, 0, 4, 0, 256>(dst, sl, nvec, n, 0, s);
    case 13: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 512>(dst, sl, nvec, n, 0, s);
    case 14: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 128>(dst, sl, nvec, n, 0, s);
    case 15: return launch_multi_x<NSRC, 1, 16, 0, 1, 1, 256>(dst, sl, nvec, n, 0, s);
    case 16: return launch_multi_x<NSRC, 1, 16, 2, 1, 0, 256>(dst, sl, nvec, n, 0, s);
    case 17: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 256>(dst, sl, nvec, n, 20 << 10, s);
    case 18: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 256>(dst, sl, nvec, n, 40 << 10, s);
    case 19: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 256>(dst, sl, nvec, n, 27 << 10, s);
    case 20: return launch_multi_x<NSRC, 1, 16, 1, 4, 0, 256>(dst, sl, nvec, n, 0, s);
    case 21: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 256>(dst, sl, nvec, n, 0, s);
    case 22: return launch_multi_x<NSRC, 2, 16, 1, 1, 0, 256>(dst, sl, nvec, n, 0, s);
    case 23: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 256>(dst, sl, nvec, n, 80 << 10, s);
    case 24: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 256>(dst, sl, nvec, n, 53 << 10, s);
    case 25: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 256>(dst, sl, nvec, n, 32 << 10, s);
    case 26: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 128>(dst, sl, nvec, n, 40 << 10, s);
    case 27: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 128>(dst, sl, nvec, n, 20 << 10, s);
    case 28: return launch_multi_x<NSRC, 2, 16, 0, 1, 0, 256>(dst, sl, nvec, n, 40 << 10, s);
    case 29: return launch_multi_x<NSRC, 2, 16, 0, 1, 0, 256>(dst, sl, nvec, n, 80 << 10, s);
    case 30: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 128>(dst, sl, nvec, n, 27 << 10, s);
    case 31: return launch_multi_x<NSRC, 1, 16, 1, 1, 0, 256>(dst, sl, nvec, n, 40 << 10, s);
    case 32: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 64>(dst, sl, nvec, n, 0, s);
    case 33: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 64>(dst, sl, nvec, n, 10 << 10, s);
    case 34: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 128>(dst, sl, nvec, n, 13 << 10, s);
    case 35: return launch_multi_x<NSRC, 2, 16, 0, 1, 0, 128>(dst, sl, nvec, n, 20 << 10, s);
    case 50: return run_multi<kF32, NSRC>(dst, sl, n, s);  // what tips_multi_sum launches
    case 51: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 64>(dst, sl, nvec, n, 16384, s);   // 64 x 10
    case 52: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 64>(dst, sl, nvec, n, 13312, s);   // 64 x 12
    case 53: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 64>(dst, sl, nvec, n, 20480, s);   // 64 x 8
    case 54: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 128>(dst, sl, nvec, n, 26624, s);  // 128 x 6
    case 55: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 128>(dst, sl, nvec, n, 32768, s);  // 128 x 5 (no room)
    case 56: return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 192>(dst, sl, nvec, n, 32768, s);  // 192 x 5
    case 36:  // the round-4 shipped fold (no cap; 4 vectors per lane for > 4 sources of 3-24 MiB)
      if (NSRC > 4 && nvec * 16 >= (3 << 20) && nvec * 16 <= (24 << 20))
        return launch_multi_x<NSRC, 4, 16, 0, 1, 0, 256>(dst, sl, nvec, n, 0, s);
      return launch_multi_x<NSRC, 1, 16, 0, 1, 0, 256>(dst, sl, nvec, n, 0, s);
    case 40: return launch_multi_gs<NSRC, 128, 0>(dst, sl, nvec, n, 4, s);
    case 41: return launch_multi_gs<NSRC, 128, 0>(dst, sl, nvec, n, 5, s);
    case 42: return launch_multi_gs<NSRC, 128, 0>(dst, sl, nvec, n, 6, s);
    case 43: return launch_multi_gs<NSRC, 128, 0>(dst, sl, nvec, n, 8, s);
    case 44: return launch_multi_gs<NSRC, 128, 1>(dst, sl, nvec, n, 4, s);
    case 45: return launch_multi_gs<NSRC, 128, 1>(dst, sl, nvec, n, 5, s);
    case 46: return launch_multi_gs<NSRC, 256, 0>(dst, sl, nvec, n, 3, s);
    case 47: return launch_multi_gs<NSRC, 256, 1>(dst, sl, nvec, n, 2, s);
    case 48: return launch_multi_gs<NSRC, 128, 0>(dst, sl, nvec, n, 12, s);
    case 49: return launch_multi_gs<NSRC, 128, 1>(dst, sl, nvec, n, 3, s);
    default: return hipErrorInvalidValue;
  }
}

// Sweep entry (f32; nsrc 2, 4, 8): 0 = global nt loads (U 2 for nsrc <= 4, else 1),
// 1 = buffer nt loads U 1, 2 = buffer nt loads U 2, 3 = buffer plain loads U 1, 4 = buffer nt loads U 4.
template <int NSRC>
hipError_t run_multi_variant(void* dst, const SrcList& sl, int64_t n, int variant, hipStream_t s) {
  const int64_t nvec = n / 4;
  auto grid_for = [&](int u) {
    int64_t g = (nvec + (int64_t)kBlock * u - 1) / ((int64_t)kBlock * u);
    return (unsigned)std::max<int64_t>(8, (g + 7) / 8 * 8);
  };
  switch (variant) {
    case 0: {
      constexpr int U = NSRC <= 4 ? 2 : 1;
      hipLaunchKernelGGL((multi_sum_kernel<kF32, NSRC, U>), dim3(grid_for(U)), dim3(kBlock), 0, s, (u32x4*)dst, sl,
                         nvec, nvec * 4, n);
      break;
    }
    case 1:
      hipLaunchKernelGGL((multi_sum_buf_kernel<kF32, NSRC, 1, 2>), dim3(grid_for(1)), dim3(kBlock), 0, s,
                         (u32x4*)dst, sl, nvec, nvec * 4, n, (int64_t)0);
      break;
    case 2:
      hipLaunchKernelGGL((multi_sum_buf_kernel<kF32, NSRC, 2, 2>), dim3(grid_for(2)), dim3(kBlock), 0, s,
                         (u32x4*)dst, sl, nvec, nvec * 4, n, (int64_t)0);
      break;
    case 3:
      hipLaunchKernelGGL((multi_sum_buf_kernel<kF32, NSRC, 1, 0>), dim3(grid_for(1)), dim3(kBlock), 0, s,
                         (u32x4*)dst, sl, nvec, nvec * 4, n, (int64_t)0);
      break;
    case 4:
      hipLaunchKernelGGL((multi_sum_buf_kernel<kF32, NSRC, 4, 2>), dim3(grid_for(4)), dim3(kBlock), 0, s,
                         (u32x4*)dst, sl, nvec, nvec * 4, n, (int64_t)0);
      break;
    case 5:  // sc0 loads
      hipLaunchKernelGGL((multi_sum_buf_kernel<kF32, NSRC, 1, 1>), dim3(grid_for(1)), dim3(kBlock), 0, s,
                         (u32x4*)dst, sl, nvec, nvec * 4, n, (int64_t)0);
      break;
    case 6:  // sc1 loads
      hipLaunchKernelGGL((multi_sum_buf_kernel<kF32, NSRC, 1, 16>), dim3(grid_for(1)), dim3(kBlock), 0, s,
                         (u32x4*)dst, sl, nvec, nvec * 4, n, (int64_t)0);
      break;
    case 7:  // plain loads, 2 vectors per lane
      hipLaunchKernelGGL((multi_sum_buf_kernel<kF32, NSRC, 2, 0>), dim3(grid_for(2)), dim3(kBlock), 0, s,
                         (u32x4*)dst, sl, nvec, nvec * 4, n, (int64_t)0);
      break;
    default:
      return run_multi_x<NSRC>(dst, sl, n, variant, s);
  }
  return hipGetLastError();
}
#endif  // TIPS_DEV

// the pull-fold's launch (launch_multi_sum_remote): 4 vectors per lane, 256 lanes, uncapped
template <int DT, int NSRC>
hipError_t run_multi_remote(void* dst, const SrcList& sl, int64_t n, hipStream_t s) {
  const int64_t ve = 16 / (int64_t)dtype_size(DT);
  const int64_t nvec = n / ve;
  int64_t grid = (nvec + 4 * kBlock - 1) / (4 * kBlock);
  grid = std::max<int64_t>(8, (grid + 7) / 8 * 8);  // (xcd_tile: remote sources, not measured with stripes)
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL((multi_sum_buf_kernel<DT, NSRC, 4, 2>), dim3((unsigned)grid), dim3(kBlock), 0, s, (u32x4*)dst, sl,
                     nvec, nvec * ve, n, (int64_t)0);
  return hipGetLastError();
}

template <int DT>
hipError_t multi_dispatch(void* dst, const void* const* srcs, int nsrc, int64_t n, hipStream_t s, bool remote = false) {
  SrcList sl{};
  bool al = aligned16(dst);
  for (int j = 0; j < nsrc; j++) {
    sl.p[j] = (const u32x4*)srcs[j];
    al = al && aligned16(srcs[j]);
  }
  if (!al) {
    int64_t grid = (n + kBlock - 1) / kBlock;
    if (grid > kNumCUs * 16) grid = kNumCUs * 16;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL((multi_sum_scalar_kernel<DT>), dim3((unsigned)grid), dim3(kBlock), 0, s, dst, sl, nsrc, n);
    return hipGetLastError();
  }
  // Two sources: the fold is one add, i.e. the 2-input sum, whose launch (one 16-B vector per lane
  // per operand, buffer ops) runs 2 x 128 MiB at the sum's rate instead of the fold's 0.75 of HBM
  // (VERDICT r05 item 6). Storage-type arithmetic for these four types: bit-identical to the fold.
  if (!remote && nsrc == 2 && (DT == kF32 || DT == kF64 || DT == kI32 || DT == kI64))
    return sum2_dispatch<DT>(dst, srcs[0], srcs[1], n, kDefMode, kDefUnroll, kDefNT, 0, kDefThreads, s);
  if (remote) {
    switch (nsrc) {
#define TIPS_REMOTE_CASE(K) \
  case K: return run_multi_remote<DT, K>(dst, sl, n, s);
      TIPS_REMOTE_CASE(2) TIPS_REMOTE_CASE(3) TIPS_REMOTE_CASE(4) TIPS_REMOTE_CASE(5) TIPS_REMOTE_CASE(6)
      TIPS_REMOTE_CASE(7) TIPS_REMOTE_CASE(8) TIPS_REMOTE_CASE(9) TIPS_REMOTE_CASE(10) TIPS_REMOTE_CASE(11)
      TIPS_REMOTE_CASE(12) TIPS_REMOTE_CASE(13) TIPS_REMOTE_CASE(14) TIPS_REMOTE_CASE(15) TIPS_REMOTE_CASE(16)
#undef TIPS_REMOTE_CASE
      default: return hipErrorInvalidValue;
    }
  }
  switch (nsrc) {
    case 1: return run_multi<DT, 1>(dst, sl, n, s);
    case 2: return run_multi<DT, 2>(dst, sl, n, s);
    case 3: return run_multi<DT, 3>(dst, sl, n, s);
    case 4: return run_multi<DT, 4>(dst, sl, n, s);
    case 5: return run_multi<DT, 5>(dst, sl, n, s);
    case 6: return run_multi<DT, 6>(dst, sl, n, s);
    case 7: return run_multi<DT, 7>(dst, sl, n, s);
    case 8: return run_multi<DT, 8>(dst, sl, n, s);
    case 9: return run_multi<DT, 9>(dst, sl, n, s);
    case 10: return run_multi<DT, 10>(dst, sl, n, s);
    case 11: return run_multi<DT, 11>(dst, sl, n, s);
    case 12: return run_multi<DT, 12>(dst, sl, n, s);
    case 13: return run_multi<DT, 13>(dst, sl, n, s);
    case 14: return run_multi<DT, 14>(dst, sl, n, s);
    case 15: return run_multi<DT, 15>(dst, sl, n, s);
    case 16: return run_multi<DT, 16>(dst, sl, n, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_sum2_variant(void* dst, const void* a, const void* b, int64_t n, int dtype, int mode, int unroll,
                               int nt, int blocks, int threads, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  switch (dtype) {
    case kF32: return sum2_dispatch<kF32>(dst, a, b, n, mode, unroll, nt, blocks, threads, s);
    case kF64: return sum2_dispatch<kF64>(dst, a, b, n, mode, unroll, nt, blocks, threads, s);
    case kI32: return sum2_dispatch<kI32>(dst, a, b, n, mode, unroll, nt, blocks, threads, s);
    case kI64: return sum2_dispatch<kI64>(dst, a, b, n, mode, unroll, nt, blocks, threads, s);
    case kF16: return sum2_dispatch<kF16>(dst, a, b, n, mode, unroll, nt, blocks, threads, s);
    case kBF16: return sum2_dispatch<kBF16>(dst, a, b, n, mode, unroll, nt, blocks, threads, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_sum2(void* dst, const void* a, const void* b, int64_t n, int dtype, hipStream_t s) {
  return launch_sum2_variant(dst, a, b, n, dtype, kDefMode, kDefUnroll, kDefNT, 0, kDefThreads, s);
}

hipError_t launch_multi_sum(void* dst, const void* const* srcs, int nsrc, int64_t n, int dtype, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (nsrc < 1 || nsrc > kMaxSrcs) return hipErrorInvalidValue;
  if (nsrc == 1) {
    if (dst == srcs[0]) return hipSuccess;
    return hipMemcpyAsync(dst, srcs[0], (size_t)n * dtype_size(dtype), hipMemcpyDeviceToDevice, s);
  }
  switch (dtype) {
    case kF32: return multi_dispatch<kF32>(dst, srcs, nsrc, n, s);
    case kF64: return multi_dispatch<kF64>(dst, srcs, nsrc, n, s);
    case kI32: return multi_dispatch<kI32>(dst, srcs, nsrc, n, s);
    case kI64: return multi_dispatch<kI64>(dst, srcs, nsrc, n, s);
    case kF16: return multi_dispatch<kF16>(dst, srcs, nsrc, n, s);
    case kBF16: return multi_dispatch<kBF16>(dst, srcs, nsrc, n, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_multi_sum_remote(void* dst, const void* const* srcs, int nsrc, int64_t n, int dtype, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (nsrc < 1 || nsrc > kMaxSrcs) return hipErrorInvalidValue;
  if (nsrc == 1) return launch_multi_sum(dst, srcs, nsrc, n, dtype, s);
  switch (dtype) {
    case kF32: return multi_dispatch<kF32>(dst, srcs, nsrc, n, s, true);
    case kF64: return multi_dispatch<kF64>(dst, srcs, nsrc, n, s, true);
    case kI32: return multi_dispatch<kI32>(dst, srcs, nsrc, n, s, true);
    case kI64: return multi_dispatch<kI64>(dst, srcs, nsrc, n, s, true);
    case kF16: return multi_dispatch<kF16>(dst, srcs, nsrc, n, s, true);
    case kBF16: return multi_dispatch<kBF16>(dst, srcs, nsrc, n, s, true);
    default: return hipErrorInvalidValue;
  }
}

#ifdef TIPS_DEV  // (tuning sweeps: libtips_hip_dev.so only)
hipError_t launch_multi_sum_variant(void* dst, const void* const* srcs, int nsrc, int64_t n, int dtype, int variant,
                                   hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (dtype != kF32 || !aligned16(dst)) return hipErrorInvalidValue;
  SrcList sl{};
  for (int j = 0; j < nsrc && j < kMaxSrcs; j++) {
    if (!aligned16(srcs[j])) return hipErrorInvalidValue;
    sl.p[j] = (const u32x4*)srcs[j];
  }
  switch (nsrc) {
    case 2: return run_multi_variant<2>(dst, sl, n, variant, s);
    case 4: return run_multi_variant<4>(dst, sl, n, variant, s);
    case 8: return run_multi_variant<8>(dst, sl, n, variant, s);
    default: return hipErrorInvalidValue;
  }
}
#endif  // TIPS_DEV

#ifdef TIPS_DEV  // (tuning sweeps: libtips_hip_dev.so only)
hipError_t launch_copy_tiles(const CopyTile* tiles_dev, int ntiles, hipStream_t s) {
  if (ntiles <= 0) return hipSuccess;
  const unsigned grid = (unsigned)((ntiles + 7) / 8 * 8);
  hipLaunchKernelGGL(copy_tiles_kernel, dim3(grid), dim3(kBlock), 0, s, tiles_dev, ntiles);
  return hipGetLastError();
}

namespace {

template <int G, int U, int LAUX, int SAUX>
hipError_t run_copy_g(const CopyTile* tiles, int ntiles, hipStream_t s) {
  const int64_t groups = (ntiles + G - 1) / G;
  const unsigned grid = (unsigned)std::max<int64_t>(8, (groups + 7) / 8 * 8);
  hipLaunchKernelGGL((copy_tiles_g_kernel<G, U, LAUX, SAUX>), dim3(grid), dim3(kBlock), 0, s, tiles, ntiles);
  return hipGetLastError();
}

template <int U>
hipError_t copy_variant_u(const CopyTile* tiles, int ntiles, int variant, hipStream_t s) {
  switch (variant) {
    case 1: return run_copy_g<1, U, 2, 16>(tiles, ntiles, s);
    case 2: return run_copy_g<2, U, 2, 16>(tiles, ntiles, s);
    case 3: return run_copy_g<4, U, 2, 16>(tiles, ntiles, s);
    case 4: return run_copy_g<8, U, 2, 16>(tiles, ntiles, s);
    case 5: return run_copy_g<2, U, 0, 16>(tiles, ntiles, s);  // plain loads
    case 6: return run_copy_g<2, U, 2, 2>(tiles, ntiles, s);   // nt stores
    case 7: return run_copy_g<2, U, 2, 0>(tiles, ntiles, s);   // plain stores
    case 8: return run_copy_g<4, U, 0, 0>(tiles, ntiles, s);   // plain both
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_copy_tiles_variant(const CopyTile* tiles_dev, int ntiles, int variant, int64_t max_tile_bytes,
                                     hipStream_t s) {
  if (ntiles <= 0) return hipSuccess;
  if (variant == 0) return launch_copy_tiles(tiles_dev, ntiles, s);
  if (max_tile_bytes <= 4096) return copy_variant_u<1>(tiles_dev, ntiles, variant, s);
  if (max_tile_bytes <= 8192) return copy_variant_u<2>(tiles_dev, ntiles, variant, s);
  if (max_tile_bytes <= 16384) return copy_variant_u<4>(tiles_dev, ntiles, variant, s);
  return hipErrorInvalidValue;  // the grouped kernel holds a tile in registers: at most 16 KiB
}

hipError_t launch_pack_tiles(const CopyTile* tiles_dev, int ntiles, int64_t max_tile_bytes, hipStream_t s) {
  if (max_tile_bytes > 16384) return launch_copy_tiles(tiles_dev, ntiles, s);
  return launch_copy_tiles_variant(tiles_dev, ntiles, 1, max_tile_bytes, s);
}
#endif  // TIPS_DEV

namespace {

template <int U>
hipError_t run_copy_segs_groups(const CopySeg* tiles, const CopySeg* segs, const PackGroups& g, int pol, hipStream_t s) {
  const unsigned grid = g.blk0[g.n];
  switch (pol) {
    case 0: hipLaunchKernelGGL((copy_segs_groups_kernel<U, 0>), dim3(grid), dim3(kBlock), 0, s, tiles, segs, g); break;
    case 1: hipLaunchKernelGGL((copy_segs_groups_kernel<U, 1>), dim3(grid), dim3(kBlock), 0, s, tiles, segs, g); break;
    case 2: hipLaunchKernelGGL((copy_segs_groups_kernel<U, 2>), dim3(grid), dim3(kBlock), 0, s, tiles, segs, g); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int U>
hipError_t run_copy_segs(const CopySeg* tiles, const CopySeg* segs, int tile0, int ntiles, int pol, hipStream_t s) {
  const int64_t C = pack_stripe_vecs() / ((int64_t)kBlock * U);  // tiles per stripe (0: xcd_tile)
  const unsigned grid = (unsigned)stripe_grid(ntiles, C);
  switch (pol) {
    case 0: hipLaunchKernelGGL((copy_segs_kernel<U, 0>), dim3(grid), dim3(kBlock), 0, s, tiles, segs, tile0, ntiles, C); break;
    case 1: hipLaunchKernelGGL((copy_segs_kernel<U, 1>), dim3(grid), dim3(kBlock), 0, s, tiles, segs, tile0, ntiles, C); break;
    case 2: hipLaunchKernelGGL((copy_segs_kernel<U, 2>), dim3(grid), dim3(kBlock), 0, s, tiles, segs, tile0, ntiles, C); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_copy_segs(const CopySeg* tiles, const CopySeg* segs, int tile0, int ntiles, int64_t tile_bytes,
                            int pol, hipStream_t s) {
  if (ntiles <= 0) return hipSuccess;
  switch (tile_bytes) {
    case 4096: return run_copy_segs<1>(tiles, segs, tile0, ntiles, pol, s);
    case 8192: return run_copy_segs<2>(tiles, segs, tile0, ntiles, pol, s);
    case 16384: return run_copy_segs<4>(tiles, segs, tile0, ntiles, pol, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_copy_segs_groups(const CopySeg* tiles, const CopySeg* segs, PackGroups g, int64_t tile_bytes, int pol,
                                   hipStream_t s) {
  if (g.n < 1 || g.n > kMaxPackGroups) return hipErrorInvalidValue;
  for (int k = 0; k < g.n; k++)
    if (g.done[k] && !g.counters) return hipErrorInvalidValue;
  int64_t blk = 0;
  for (int k = 0; k < g.n; k++) {  // each group's workgroups: whole XCD rounds (xcd_tile), at least 8
    if (g.ntiles[k] < 0) return hipErrorInvalidValue;
    g.blk0[k] = (unsigned)blk;
    blk += std::max<int64_t>(8, ((int64_t)g.ntiles[k] + 7) / 8 * 8);
  }
  if (blk > 0x7fffffff) return hipErrorInvalidValue;
  g.blk0[g.n] = (unsigned)blk;
  switch (tile_bytes) {
    case 4096: return run_copy_segs_groups<1>(tiles, segs, g, pol, s);
    case 8192: return run_copy_segs_groups<2>(tiles, segs, g, pol, s);
    case 16384: return run_copy_segs_groups<4>(tiles, segs, g, pol, s);
    default: return hipErrorInvalidValue;
  }
}

namespace {
// dynamic LDS per cast workgroup (an occupancy cap: 160 KiB / bytes workgroups per CU), per
// direction; TIPS_CAST_LDS_PACK / TIPS_CAST_LDS_UNPACK (bytes) for sweeps
int cast_lds_bytes(int dir) {
  static const int v[2] = {(int)std::min<long>(65536, std::max<long>(0, getenv("TIPS_CAST_LDS_PACK") ? atol(getenv("TIPS_CAST_LDS_PACK")) : 0)),
                           (int)std::min<long>(65536, std::max<long>(0, getenv("TIPS_CAST_LDS_UNPACK") ? atol(getenv("TIPS_CAST_LDS_UNPACK")) : 0))};
  return v[dir];
}

template <int U, int DIR>
hipError_t run_cast_segs(const CopySeg* tiles, const CopySeg* segs, int tile0, int ntiles, int wire, hipStream_t s) {
  const unsigned grid = (unsigned)std::max<int64_t>(8, ((int64_t)ntiles + 7) / 8 * 8);
  const int lds = cast_lds_bytes(DIR);
  static const int var = getenv("TIPS_CAST_VARIANT") ? atoi(getenv("TIPS_CAST_VARIANT")) : 8;
  if (U == 2 && wire == kF16 && var != 8) {  // (the load / store policy sweep, f16 wire, 8 KiB tiles)
    switch (var) {
      case 0: hipLaunchKernelGGL((cast_segs_kernel<U, DIR, kF16, 0>), dim3(grid), dim3(kBlock), lds, s, tiles, segs, tile0, ntiles); break;
      case 1: hipLaunchKernelGGL((cast_segs_kernel<U, DIR, kF16, 1>), dim3(grid), dim3(kBlock), lds, s, tiles, segs, tile0, ntiles); break;
      case 2: hipLaunchKernelGGL((cast_segs_kernel<U, DIR, kF16, 2>), dim3(grid), dim3(kBlock), lds, s, tiles, segs, tile0, ntiles); break;
      case 3: hipLaunchKernelGGL((cast_segs_kernel<U, DIR, kF16, 3>), dim3(grid), dim3(kBlock), lds, s, tiles, segs, tile0, ntiles); break;
      case 4: hipLaunchKernelGGL((cast_segs_kernel<U, DIR, kF16, 4>), dim3(grid), dim3(kBlock), lds, s, tiles, segs, tile0, ntiles); break;
      default: hipLaunchKernelGGL((cast_segs_kernel<U, DIR, kF16, 5>), dim3(grid), dim3(kBlock), lds, s, tiles, segs, tile0, ntiles); break;
    }
    return hipGetLastError();
  }
  if (wire == kF16)
    hipLaunchKernelGGL((cast_segs_kernel<U, DIR, kF16>), dim3(grid), dim3(kBlock), lds, s, tiles, segs, tile0, ntiles);
  else if (wire == kBF16)
    hipLaunchKernelGGL((cast_segs_kernel<U, DIR, kBF16>), dim3(grid), dim3(kBlock), lds, s, tiles, segs, tile0, ntiles);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

template <int DIR>
hipError_t run_cast_range(void* dst, const void* src, int64_t n, int wire, hipStream_t s) {
  const int64_t grid = std::max<int64_t>(1, std::min<int64_t>((n + kBlock - 1) / kBlock, (int64_t)kNumCUs * 16));
  if (wire == kF16) hipLaunchKernelGGL((cast_range_kernel<DIR, kF16>), dim3((unsigned)grid), dim3(kBlock), 0, s, dst, src, n);
  else if (wire == kBF16) hipLaunchKernelGGL((cast_range_kernel<DIR, kBF16>), dim3((unsigned)grid), dim3(kBlock), 0, s, dst, src, n);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}
}  // namespace

hipError_t launch_cast_segs(const CopySeg* tiles, const CopySeg* segs, int tile0, int ntiles, int64_t tile_bytes,
                            int dir, int wire, hipStream_t s) {
  if (ntiles <= 0) return hipSuccess;
  if (dir != 0 && dir != 1) return hipErrorInvalidValue;
  switch (tile_bytes) {
    case 4096: return dir ? run_cast_segs<1, 1>(tiles, segs, tile0, ntiles, wire, s) : run_cast_segs<1, 0>(tiles, segs, tile0, ntiles, wire, s);
    case 8192: return dir ? run_cast_segs<2, 1>(tiles, segs, tile0, ntiles, wire, s) : run_cast_segs<2, 0>(tiles, segs, tile0, ntiles, wire, s);
    case 16384: return dir ? run_cast_segs<4, 1>(tiles, segs, tile0, ntiles, wire, s) : run_cast_segs<4, 0>(tiles, segs, tile0, ntiles, wire, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_cast_range(void* dst, const void* src, int64_t n, int dir, int wire, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  return dir ? run_cast_range<1>(dst, src, n, wire, s) : run_cast_range<0>(dst, src, n, wire, s);
}

hipError_t launch_xfer(const XferSeg* segs, int nseg, hipStream_t s) {
  if (nseg < 0 || nseg > kMaxXferSegs) return hipErrorInvalidValue;
  XferList L{};
  int64_t max_tiles = 0;
  int m = 0;
  for (int i = 0; i < nseg; i++) {
    if (segs[i].bytes <= 0) continue;
    L.s[m++] = segs[i];
    max_tiles = std::max<int64_t>(max_tiles, (segs[i].bytes + kXferTileBytes - 1) / kXferTileBytes);
  }
  if (m == 0) return hipSuccess;
  const int64_t grid = max_tiles * m;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(xfer_kernel, dim3((unsigned)grid), dim3(kBlock), 0, s, L, m);
  return hipGetLastError();
}

}  // namespace tips
