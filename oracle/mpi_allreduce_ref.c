/*
 * mpi_allreduce_ref.c — runs the reference's exact data-path call on host
 * memory, for golden vectors and for the CPU baseline.
 *
 * TEST INFRASTRUCTURE ONLY (never linked into the product). This is not a
 * copy of reference source: it is a ~100-line driver that makes the one call
 * the reference's hot path makes,
 *     MPI_Allreduce(in, out, N, mpi_type_trait<T>::type(), MPI_SUM, MPI_COMM_WORLD)
 * (tips/core/collective/utils.h:60-65; types from tips/core/mpi/tips_mpi.h:13-55),
 * against the MPI found in the image (MPICH 3.3.2 under /opt/conda; the
 * reference's README pins OpenMPI v4.1, which is not present).
 *
 * Modes:
 *   golden <dtype> <n> <dir>    read <dir>/in_<rank>.bin, write <dir>/out_<rank>.bin
 *   bench  <dtype> <n> <iters>  time `iters` calls on U[0.5,1.5) data (seed 1000+rank),
 *                               rank 0 prints one JSON line (mean seconds per call).
 * dtype: 0 f32, 1 f64, 2 i32, 3 i64 (collective_messages.fbs:17-23).
 */
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static MPI_Datatype to_mpi(int dtype, int* es) {
  switch (dtype) {
    case 0: *es = 4; return MPI_FLOAT;
    case 1: *es = 8; return MPI_DOUBLE;
    case 2: *es = 4; return MPI_INT;
    case 3: *es = 8; return MPI_LONG_LONG;
    default: *es = 0; return MPI_DATATYPE_NULL;
  }
}

static int read_file(const char* path, void* buf, size_t bytes) {
  FILE* f = fopen(path, "rb");
  if (!f) return -1;
  size_t got = fread(buf, 1, bytes, f);
  fclose(f);
  return got == bytes ? 0 : -1;
}

static int write_file(const char* path, const void* buf, size_t bytes) {
  FILE* f = fopen(path, "wb");
  if (!f) return -1;
  size_t put = fwrite(buf, 1, bytes, f);
  fclose(f);
  return put == bytes ? 0 : -1;
}

/* xorshift64* for the bench fill; the values only need to be positive and finite. */
static uint64_t rng_next(uint64_t* s) {
  uint64_t x = *s;
  x ^= x >> 12;
  x ^= x << 25;
  x ^= x >> 27;
  *s = x;
  return x * 2685821657736338717ull;
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank = 0, size = 1;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  if (argc < 5) {
    if (rank == 0) fprintf(stderr, "usage: %s golden|bench dtype n dir|iters\n", argv[0]);
    MPI_Finalize();
    return 2;
  }
  int dtype = atoi(argv[2]);
  long long n = atoll(argv[3]);
  int es = 0;
  MPI_Datatype t = to_mpi(dtype, &es);
  if (es == 0 || n < 0 || n > 0x7fffffffLL) { /* the reference passes an int count */
    if (rank == 0) fprintf(stderr, "bad dtype or count\n");
    MPI_Finalize();
    return 2;
  }
  size_t bytes = (size_t)n * (size_t)es;
  char* in = (char*)malloc(bytes ? bytes : 1);
  char* out = (char*)malloc(bytes ? bytes : 1);
  int rc = 0;
  if (strcmp(argv[1], "golden") == 0) {
    char path[4096];
    snprintf(path, sizeof path, "%s/in_%d.bin", argv[4], rank);
    if (read_file(path, in, bytes)) {
      fprintf(stderr, "rank %d: cannot read %s\n", rank, path);
      MPI_Abort(MPI_COMM_WORLD, 3);
    }
    rc = MPI_Allreduce(in, out, (int)n, t, MPI_SUM, MPI_COMM_WORLD);
    snprintf(path, sizeof path, "%s/out_%d.bin", argv[4], rank);
    if (rc == 0 && write_file(path, out, bytes)) rc = 4;
  } else if (strcmp(argv[1], "bench") == 0) {
    int iters = atoi(argv[4]);
    uint64_t s = 0x9E3779B97F4A7C15ull ^ (uint64_t)(1000 + rank);
    for (long long i = 0; i < n; i++) {
      double u = 0.5 + (double)(rng_next(&s) >> 11) * (1.0 / 9007199254740992.0);
      if (dtype == 0) ((float*)in)[i] = (float)u;
      else if (dtype == 1) ((double*)in)[i] = u;
      else if (dtype == 2) ((int32_t*)in)[i] = (int32_t)(u * 1000);
      else ((int64_t*)in)[i] = (int64_t)(u * 1000);
    }
    rc |= MPI_Allreduce(in, out, (int)n, t, MPI_SUM, MPI_COMM_WORLD); /* warm-up */
    MPI_Barrier(MPI_COMM_WORLD);
    double t0 = MPI_Wtime();
    for (int it = 0; it < iters && rc == 0; it++) rc |= MPI_Allreduce(in, out, (int)n, t, MPI_SUM, MPI_COMM_WORLD);
    double dt = MPI_Wtime() - t0, dtmax = 0;
    MPI_Reduce(&dt, &dtmax, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    if (rank == 0)
      printf("{\"np\": %d, \"dtype\": %d, \"count\": %lld, \"iters\": %d, \"sec_per_call\": %.9g}\n", size, dtype, n,
             iters, dtmax / (iters > 0 ? iters : 1));
  } else {
    rc = 2;
  }
  free(in);
  free(out);
  MPI_Finalize();
  return rc ? 1 : 0;
}
