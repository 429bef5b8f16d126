/*
 * oracle.c — CPU restatement of the TiPS allreduce-SUM path.
 * TEST INFRASTRUCTURE ONLY (see oracle.h): never linked into the product.
 *
 * Reference anchors:
 *   AllreduceCpu<T>            tips/core/collective/utils.h:52-67
 *   MPI_Allreduce(.., MPI_SUM) tips/core/collective/utils.h:60-65
 *   CollectiveOpKind::SUM      tips/core/collective/utils.h:21-25, utils.cc:8-9
 *   dtype mapping              tips/core/collective/utils.h:29-46,
 *                              tips/core/mpi/tips_mpi.h:13-55 (int64 -> MPI_LONG_LONG)
 * Compile with -O2 -fno-fast-math -ffp-contract=off so every float add is
 * one IEEE binary32 add (x86-64 SSE, FLT_EVAL_METHOD == 0).
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

int oracle_elem_size(int dtype) {
  switch (dtype) {
    case ORACLE_F32: return 4;
    case ORACLE_F64: return 8;
    case ORACLE_I32: return 4;
    case ORACLE_I64: return 8;
    case ORACLE_F16: return 2;
    case ORACLE_BF16: return 2;
    default: return 0;
  }
}

/* ---- 16-bit float formats (round-to-nearest-even) ---------------------- */

float oracle_half_to_float(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1fu;
  uint32_t man = h & 0x3ffu;
  uint32_t bits;
  if (exp == 0) {
    if (man == 0) {
      bits = sign;
    } else { /* subnormal: man * 2^-24, exact in binary32 */
      float v = (float)man * (1.0f / 16777216.0f);
      memcpy(&bits, &v, 4);
      bits |= sign;
    }
  } else if (exp == 0x1f) {
    bits = sign | 0x7f800000u | (man << 13);
  } else {
    bits = sign | ((exp + 112u) << 23) | (man << 13);
  }
  float f;
  memcpy(&f, &bits, 4);
  return f;
}

uint16_t oracle_float_to_half(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  uint16_t sign = (uint16_t)((x >> 16) & 0x8000u);
  uint32_t ax = x & 0x7fffffffu;
  if (ax >= 0x7f800000u) { /* inf / nan (nan made quiet, payload top bits kept) */
    if (ax == 0x7f800000u) return sign | 0x7c00u;
    return sign | 0x7e00u | (uint16_t)((ax >> 13) & 0x3ffu);
  }
  if (ax >= 0x477ff000u) return sign | 0x7c00u; /* >= 65520 rounds to inf */
  if (ax < 0x38800000u) {                          /* below 2^-14: subnormal half */
    float v;
    memcpy(&v, &ax, 4);
    return sign | (uint16_t)rintf(v * 16777216.0f); /* exact scale, RNE */
  }
  uint32_t h = ((((ax >> 23) - 112u) << 10) | ((ax & 0x7fffffu) >> 13));
  uint32_t rem = ax & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
  return sign | (uint16_t)h;
}

float oracle_bf16_to_float(uint16_t h) {
  uint32_t bits = (uint32_t)h << 16;
  float f;
  memcpy(&f, &bits, 4);
  return f;
}

uint16_t oracle_float_to_bf16(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  if ((x & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((x >> 16) | 0x40u); /* quiet nan */
  return (uint16_t)((x + 0x7fffu + ((x >> 16) & 1u)) >> 16);
}

int oracle_cast_to16(int code, uint16_t* out, const float* in, int64_t n) {
  int64_t i;
  if (code != ORACLE_F16 && code != ORACLE_BF16) return -1;
  for (i = 0; i < n; i++) out[i] = code == ORACLE_F16 ? oracle_float_to_half(in[i]) : oracle_float_to_bf16(in[i]);
  return 0;
}

int oracle_cast_from16(int code, float* out, const uint16_t* in, int64_t n) {
  int64_t i;
  if (code != ORACLE_F16 && code != ORACLE_BF16) return -1;
  for (i = 0; i < n; i++) out[i] = code == ORACLE_F16 ? oracle_half_to_float(in[i]) : oracle_bf16_to_float(in[i]);
  return 0;
}

/* ---- one MPI_SUM step: out = a + b ------------------------------------- */

int oracle_sum2(int dtype, void* out, const void* a, const void* b, int64_t n) {
  int64_t i;
  switch (dtype) {
    case ORACLE_F32: {
      float* o = (float*)out;
      const float *x = (const float*)a, *y = (const float*)b;
      for (i = 0; i < n; i++) o[i] = x[i] + y[i];
      return 0;
    }
    case ORACLE_F64: {
      double* o = (double*)out;
      const double *x = (const double*)a, *y = (const double*)b;
      for (i = 0; i < n; i++) o[i] = x[i] + y[i];
      return 0;
    }
    case ORACLE_I32: { /* two's-complement wrap: add as unsigned */
      uint32_t* o = (uint32_t*)out;
      const uint32_t *x = (const uint32_t*)a, *y = (const uint32_t*)b;
      for (i = 0; i < n; i++) o[i] = x[i] + y[i];
      return 0;
    }
    case ORACLE_I64: {
      uint64_t* o = (uint64_t*)out;
      const uint64_t *x = (const uint64_t*)a, *y = (const uint64_t*)b;
      for (i = 0; i < n; i++) o[i] = x[i] + y[i];
      return 0;
    }
    case ORACLE_F16: {
      uint16_t* o = (uint16_t*)out;
      const uint16_t *x = (const uint16_t*)a, *y = (const uint16_t*)b;
      for (i = 0; i < n; i++) o[i] = oracle_float_to_half(oracle_half_to_float(x[i]) + oracle_half_to_float(y[i]));
      return 0;
    }
    case ORACLE_BF16: {
      uint16_t* o = (uint16_t*)out;
      const uint16_t *x = (const uint16_t*)a, *y = (const uint16_t*)b;
      for (i = 0; i < n; i++) o[i] = oracle_float_to_bf16(oracle_bf16_to_float(x[i]) + oracle_bf16_to_float(y[i]));
      return 0;
    }
    default: return -1;
  }
}

/* ---- rank-order fold ----------------------------------------------------- */

int oracle_fold(int dtype, void* out, const void* const* in, int p, int64_t n, int wide_acc) {
  int es = oracle_elem_size(dtype);
  if (es == 0 || p < 1) return -1;
  if (n == 0) return 0;
  if (wide_acc && (dtype == ORACLE_F16 || dtype == ORACLE_BF16)) {
    const int half = dtype == ORACLE_F16;
    uint16_t* o = (uint16_t*)out;
    for (int64_t i = 0; i < n; i++) {
      float acc = 0.0f;
      for (int r = 0; r < p; r++) {
        uint16_t v = ((const uint16_t*)in[r])[i];
        float f = half ? oracle_half_to_float(v) : oracle_bf16_to_float(v);
        acc = (r == 0) ? f : acc + f;
      }
      o[i] = half ? oracle_float_to_half(acc) : oracle_float_to_bf16(acc);
    }
    return 0;
  }
  memcpy(out, in[0], (size_t)(n * es));
  for (int r = 1; r < p; r++) {
    int rc = oracle_sum2(dtype, out, out, in[r], n);
    if (rc) return rc;
  }
  return 0;
}

/* ---- ring schedule --------------------------------------------------------- */

void oracle_chunk_bounds(int64_t n, int p, int64_t align_elems, int c, int64_t* begin, int64_t* end) {
  if (align_elems < 1) align_elems = 1;
  int64_t per = (n + p - 1) / p;
  per = (per + align_elems - 1) / align_elems * align_elems;
  int64_t b = (int64_t)c * per, e = b + per;
  if (b > n) b = n;
  if (e > n) e = n;
  *begin = b;
  *end = e;
}

int oracle_ring(int dtype, void* const* outs, const void* const* ins, int p, int64_t n, int64_t align_elems) {
  int es = oracle_elem_size(dtype);
  if (es == 0 || p < 1) return -1;
  if (n == 0) return 0;
  /* Reduce-scatter. At step s rank r sends chunk (r-s) mod p to r+1; rank
   * r+1 sets out[c] = in[c] + received. First step reads `in`, later steps
   * read the running `out`. */
  int64_t per_bytes;
  {
    int64_t b0, e0;
    oracle_chunk_bounds(n, p, align_elems, 0, &b0, &e0);
    per_bytes = (e0 - b0) * es;
  }
  char* wire = (char*)malloc((size_t)(per_bytes > 0 ? per_bytes : 1));
  if (!wire) return -2;
  for (int s = 0; s < p - 1; s++) {
    for (int r = 0; r < p; r++) { /* every rank's send happens "simultaneously": process receivers */
      int src = (r - 1 + p) % p;
      int c = ((src - s) % p + p) % p;
      int64_t b, e;
      oracle_chunk_bounds(n, p, align_elems, c, &b, &e);
      if (e <= b) continue;
      const char* from = (s == 0) ? (const char*)ins[src] : (const char*)outs[src];
      memcpy(wire, from + b * es, (size_t)((e - b) * es));
      oracle_sum2(dtype, (char*)outs[r] + b * es, (const char*)ins[r] + b * es, wire, e - b);
    }
  }
  /* Allgather: rank r owns chunk (r+1) mod p; at step s it forwards chunk
   * (r+1-s) mod p to r+1. p == 1 degenerates to out = in. */
  if (p == 1) memcpy(outs[0], ins[0], (size_t)(n * es));
  for (int s = 0; s < p - 1; s++) {
    for (int r = 0; r < p; r++) {
      int src = (r - 1 + p) % p;
      int c = ((src + 1 - s) % p + p) % p;
      int64_t b, e;
      oracle_chunk_bounds(n, p, align_elems, c, &b, &e);
      if (e <= b) continue;
      memcpy((char*)outs[r] + b * es, (const char*)outs[src] + b * es, (size_t)((e - b) * es));
    }
  }
  free(wire);
  return 0;
}
