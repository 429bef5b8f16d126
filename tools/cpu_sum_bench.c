/*
 * cpu_sum_bench.c — the host-core counterpart of config 2:
 * c[i] = a[i] + b[i] over two 256 MiB fp32 buckets, on 1 thread and on T
 * threads (OpenMP). This is the loop MPI's local MPI_SUM runs per received
 * chunk (tips/core/collective/utils.h:60-65 reaches it through libmpi), timed
 * without any transport, so it is the best a CPU reduction step can do here.
 *
 * BASELINE INSTRUMENT ONLY: never linked into the product.
 *
 * usage: cpu_sum_bench <elements> <iters> <threads>
 * prints one JSON line: seconds per call, algorithmic GB/s (3 x 4 B per element).
 */
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int main(int argc, char** argv) {
  long long n = argc > 1 ? atoll(argv[1]) : 67108864LL;
  int iters = argc > 2 ? atoi(argv[2]) : 10;
  int threads = argc > 3 ? atoi(argv[3]) : 1;
  if (n <= 0 || iters <= 0 || threads <= 0) {
    fprintf(stderr, "usage: %s elements iters threads\n", argv[0]);
    return 2;
  }
  omp_set_num_threads(threads);
  float* a = (float*)aligned_alloc(64, (size_t)n * 4);
  float* b = (float*)aligned_alloc(64, (size_t)n * 4);
  float* c = (float*)aligned_alloc(64, (size_t)n * 4);
  if (!a || !b || !c) return 3;
  /* first touch on the threads that will stream the data */
#pragma omp parallel for schedule(static)
  for (long long i = 0; i < n; i++) {
    a[i] = (float)((i * 2654435761ull) % 1000) * 1e-3f - 0.5f;
    b[i] = (float)((i * 40503ull) % 1000) * 1e-3f - 0.5f;
    c[i] = 0.f;
  }
#pragma omp parallel for schedule(static)
  for (long long i = 0; i < n; i++) c[i] = a[i] + b[i]; /* warm-up */
  double t0 = omp_get_wtime();
  for (int it = 0; it < iters; it++) {
#pragma omp parallel for schedule(static)
    for (long long i = 0; i < n; i++) c[i] = a[i] + b[i];
  }
  double dt = (omp_get_wtime() - t0) / iters;
  double check = 0;
  for (long long i = 0; i < n; i += 4099) check += c[i] - (a[i] + b[i]);
  printf("{\"threads\": %d, \"elements\": %lld, \"iters\": %d, \"sec_per_call\": %.9g, \"gb_s\": %.4g, "
         "\"check\": %g}\n",
         threads, n, iters, dt, 12.0 * (double)n / dt / 1e9, check);
  free(a);
  free(b);
  free(c);
  return check == 0 ? 0 : 1;
}
