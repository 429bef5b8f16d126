/* op_host.c — config 5 (the ResNet-50 gradient set) as the reference's TF op sees it: 214 named
 * HOST allreduces per step, issued from TF-style executor threads through the C-ABI alone.
 *
 * The reference's MPIAllreduce is an async CPU op (tips/tensorflow/ops.cc:86-118): an executor
 * thread runs ComputeAsync, which allocates the output, enqueues the host tensor under the op's
 * name with a callback (EnqueueTensorCollective, coordinator.cc:223-241) and returns; rank 0's
 * background loop (coordinator.cc:355-513) runs every name in readiness order and the callback
 * calls done(). Here each step, four persistent executor threads (TF's inter-op pool) issue their
 * share of the 214 gradients in a per-rank shuffled order with tips_enqueue_allreduce_shaped (the
 * gradient's TF shape) + tips_on_done, and main waits until the last callback has come (the callbacks
 * count; only the last one wakes main, as TF's executor wakes the step's caller once its last op is
 * done): one step = one training step's gradient allreduce. The
 * library fuses the host requests each negotiation cycle hands it (negotiate.cc execute: one
 * tips_fused_allreduce_host call per run of host allreduces).
 *
 * Two builds of this file (Makefile):
 *   tools/_bin/op_host        bench.py's leg: times OP_HOST_STEPS steps after OP_HOST_WARMUP; at
 *                             one rank checks every output bit-exact against its input (the sum of
 *                             one rank), else reports "not checked". Product library only.
 *   tools/_bin/op_host_check  -DOP_HOST_ORACLE, for tests/test_gpu_op_body.py: also checks every
 *                             output of the last step bit-exact against the oracle's rank-order fold
 *                             (oracle_fold) of all ranks' regenerated inputs (test infrastructure).
 * Env: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT (tips_init); OP_HOST_STEPS (20), OP_HOST_WARMUP (3),
 * OP_HOST_THREADS (4). Prints one JSON line. */
#include <dirent.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#ifdef OP_HOST_ORACLE
#include "oracle.h"
#endif
#include "tips_hip.h"

#define MAX_TENSORS 256
#define MAX_THREADS 16

typedef struct {
  int ndim;
  int64_t dims[4];
  int64_t n;
  float* in;
  float* out;
  char name[80];
  atomic_int status;
} Grad;

static Grad g_g[MAX_TENSORS];
static int g_n, g_rank, g_size, g_threads;
static int g_order[MAX_TENSORS];
static atomic_int g_done;
static atomic_int g_failed;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_cv = PTHREAD_COND_INITIALIZER;
static char g_err[512];

static void add(int ndim, int64_t a, int64_t b, int64_t c, int64_t d, const char* what) {
  Grad* g = &g_g[g_n];
  g->ndim = ndim;
  g->dims[0] = a, g->dims[1] = b, g->dims[2] = c, g->dims[3] = d;
  g->n = 1;
  for (int k = 0; k < ndim; k++) g->n *= g->dims[k];
  snprintf(g->name, sizeof g->name, "resnet50/%03d/%s", g_n, what);
  g_n++;
}

/* Keras ResNet-50's trainable gradients in layer-creation order (bench.py resnet50_grad_sizes,
 * SURVEY §8d): stem conv 7x7x3x64 + bias, BN gamma / beta; stages [3, 4, 6, 3] of bottlenecks of
 * widths 64 / 128 / 256 / 512 (x4 expansion, conv biases, a projection shortcut in each stage's
 * first block); dense 2048 x 1000 + bias. 214 tensors, 25,583,592 parameters. */
static void resnet50(void) {
  add(4, 7, 7, 3, 64, "conv");
  add(1, 64, 0, 0, 0, "bias");
  add(1, 64, 0, 0, 0, "gamma");
  add(1, 64, 0, 0, 0, "beta");
  int64_t cin = 64;
  const int64_t widths[4] = {64, 128, 256, 512}, blocks[4] = {3, 4, 6, 3};
  for (int s = 0; s < 4; s++) {
    const int64_t f = widths[s];
    for (int b = 0; b < blocks[s]; b++) {
      if (b == 0) {
        add(4, 1, 1, cin, 4 * f, "shortcut");
        add(1, 4 * f, 0, 0, 0, "bias");
        add(1, 4 * f, 0, 0, 0, "gamma");
        add(1, 4 * f, 0, 0, 0, "beta");
      }
      add(4, 1, 1, cin, f, "conv1");
      add(1, f, 0, 0, 0, "bias");
      add(1, f, 0, 0, 0, "gamma");
      add(1, f, 0, 0, 0, "beta");
      add(4, 3, 3, f, f, "conv2");
      add(1, f, 0, 0, 0, "bias");
      add(1, f, 0, 0, 0, "gamma");
      add(1, f, 0, 0, 0, "beta");
      add(4, 1, 1, f, 4 * f, "conv3");
      add(1, 4 * f, 0, 0, 0, "bias");
      add(1, 4 * f, 0, 0, 0, "gamma");
      add(1, 4 * f, 0, 0, 0, "beta");
      cin = 4 * f;
    }
  }
  add(2, 2048, 1000, 0, 0, "dense");
  add(1, 1000, 0, 0, 0, "bias");
}

/* rank r's element j of gradient i: U[-1, 1) from a splitmix64 hash of (5000 + r, i, j) */
static float value(int r, int i, int64_t j) {
  uint64_t z = ((uint64_t)(5000 + r) << 40) ^ ((uint64_t)i << 28) ^ (uint64_t)j;
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)((double)(z >> 40) / (double)(1ull << 24) * 2.0 - 1.0);
}

static void fill(float* x, int r, int i, int64_t n) {
  for (int64_t j = 0; j < n; j++) x[j] = value(r, i, j);
}

static double now(void);
static double g_t_first_cb, g_t_enq;  /* OP_HOST_TRACE: the step's first callback, the last enqueue */
static atomic_int g_enq_threads;
static double g_t_start[64], g_t_in_enq[64], g_t_in_reg[64];  /* OP_HOST_TRACE, per executor thread */

static void count_done(void) {
  const int k = atomic_fetch_add(&g_done, 1);
  if (k == 0) g_t_first_cb = now();
  if (k + 1 == g_n) {  /* the step's last callback wakes main */
    pthread_mutex_lock(&g_mu);
    pthread_cond_broadcast(&g_cv);
    pthread_mutex_unlock(&g_mu);
  }
}

static void on_done(void* ctx, int status, const char* message) {
  Grad* g = (Grad*)ctx;
  atomic_store(&g->status, status);
  if (status) {
    pthread_mutex_lock(&g_mu);
    if (!g_err[0]) snprintf(g_err, sizeof g_err, "%s: %s", g->name, message);
    pthread_mutex_unlock(&g_mu);
    atomic_fetch_add(&g_failed, 1);
  }
  count_done();
}

/* the executor threads: persistent, released once per step (a barrier), each enqueues its share */
static pthread_barrier_t g_go;
static int g_one_call = 1; /* OP_HOST_ONE_CALL */
static atomic_int g_quit;

static void* executor(void* arg) {
  const int t = (int)(intptr_t)arg;
  while (1) {
    pthread_barrier_wait(&g_go);
    if (atomic_load(&g_quit)) return NULL;
    double t_enq = 0, t_reg = 0;
    if (t < 64) g_t_start[t] = now();
    for (int k = 0; k < g_n; k++) {
      const int i = g_order[k];
      if (i % g_threads != t) continue;
      Grad* g = &g_g[i];
      const double a = now();
      int64_t h;
      double b;
      int rc = TIPS_OK;
      if (g_one_call) { /* the request and its callback in one call (tips_enqueue_allreduce_cb) */
        h = tips_enqueue_allreduce_cb(g->name, g->in, g->out, g->dims, g->ndim, TIPS_FLOAT32, NULL, on_done, g);
        b = now();
      } else { /* OP_HOST_ONE_CALL=0: enqueue, then register the callback (round 4's op body) */
        h = tips_enqueue_allreduce_shaped(g->name, g->in, g->out, g->dims, g->ndim, TIPS_FLOAT32, NULL);
        b = now();
        rc = h < 0 ? TIPS_OK : tips_on_done(h, on_done, g);
      }
      t_enq += b - a;
      t_reg += now() - b;
      if (h < 0 || rc != TIPS_OK) {
        pthread_mutex_lock(&g_mu);
        if (!g_err[0]) snprintf(g_err, sizeof g_err, "%s: %s", g->name, tips_last_error());
        pthread_mutex_unlock(&g_mu);
        atomic_fetch_add(&g_failed, 1);
        count_done();
      }
    }
    if (t < 64) g_t_in_enq[t] = t_enq, g_t_in_reg[t] = t_reg;
    if (atomic_fetch_add(&g_enq_threads, 1) + 1 == g_threads) g_t_enq = now();
  }
}

/* one step: every gradient enqueued by the executor threads; returns when all 214 are done */
static int g_trace;

static int step(void) {
  atomic_store(&g_done, 0);
  atomic_store(&g_enq_threads, 0);
  const double t0 = now();
  pthread_barrier_wait(&g_go);
  struct timespec dl;
  clock_gettime(CLOCK_REALTIME, &dl);
  dl.tv_sec += 120;
  pthread_mutex_lock(&g_mu);
  while (atomic_load(&g_done) < g_n)
    if (pthread_cond_timedwait(&g_cv, &g_mu, &dl) != 0) break;
  pthread_mutex_unlock(&g_mu);
  if (g_trace) {
    fprintf(stderr, "[op_host] step: enqueued %.0f us, first callback %.0f us, last %.0f us\n", (g_t_enq - t0) * 1e6,
            (g_t_first_cb - t0) * 1e6, (now() - t0) * 1e6);
    for (int t = 0; t < g_threads && t < 64; t++)  /* when each thread started; its time inside the two calls */
      fprintf(stderr, "[op_host]   thread %d: start %.0f us, in enqueue %.0f us, in on_done %.0f us\n", t,
              (g_t_start[t] - t0) * 1e6, g_t_in_enq[t] * 1e6, g_t_in_reg[t] * 1e6);
  }
  return atomic_load(&g_done) == g_n && atomic_load(&g_failed) == 0 ? 0 : -1;
}

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int env_int(const char* k, int d) {
  const char* v = getenv(k);
  return v && *v ? atoi(v) : d;
}

/* where the main thread and the library's named threads (tips-neg, tips-done, tips-host) last ran:
 * "name:cpu/first CPU of its L3/socket ..." (/proc/self/task/ * /stat field 39; sysfs topology) */
static int read_first_int(const char* path) {
  FILE* f = fopen(path, "r");
  int v = -1;
  if (f) {
    if (fscanf(f, "%d", &v) != 1) v = -1;
    fclose(f);
  }
  return v;
}

static void thread_placement(char* out, size_t cap) {
  size_t l = 0;
  out[0] = 0;
  DIR* d = opendir("/proc/self/task");
  if (!d) return;
  struct dirent* e;
  while ((e = readdir(d)) != NULL && l + 64 < cap) {
    const long tid = atol(e->d_name);
    if (tid <= 0) continue;
    char path[128], comm[64] = "", stat[1024];
    snprintf(path, sizeof path, "/proc/self/task/%ld/comm", tid);
    FILE* f = fopen(path, "r");
    if (!f) continue;
    if (!fgets(comm, sizeof comm, f)) comm[0] = 0;
    fclose(f);
    comm[strcspn(comm, "\n")] = 0;
    const int is_main = tid == (long)getpid();
    if (!is_main && strncmp(comm, "tips-", 5) != 0) continue;
    snprintf(path, sizeof path, "/proc/self/task/%ld/stat", tid);
    f = fopen(path, "r");
    if (!f) continue;
    const size_t n = fread(stat, 1, sizeof stat - 1, f);
    fclose(f);
    stat[n] = 0;
    char* q = strrchr(stat, ')');
    int cpu = -1, field = 2;
    for (char* t = q ? strtok(q + 1, " ") : NULL; t; t = strtok(NULL, " "))
      if (++field == 39) {
        cpu = atoi(t);
        break;
      }
    snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", cpu);
    const int l3 = read_first_int(path);
    snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%d/topology/physical_package_id", cpu);
    const int sock = read_first_int(path);
    l += (size_t)snprintf(out + l, cap - l, "%s%s:%d/%d/%d", l ? " " : "", is_main ? "main" : comm, cpu, l3, sock);
  }
  closedir(d);
}

int main(void) {
  const int steps = env_int("OP_HOST_STEPS", 20), warmup = env_int("OP_HOST_WARMUP", 3);
  g_threads = env_int("OP_HOST_THREADS", 4);
  g_trace = env_int("OP_HOST_TRACE", 0);
  g_one_call = env_int("OP_HOST_ONE_CALL", 1);
  if (g_threads < 1 || g_threads > MAX_THREADS || steps < 1) return 2;
  resnet50();
  tips_init();
  if (!tips_is_initialize()) {
    printf("{\"ok\": false, \"error\": \"tips_init: %s\"}\n", tips_last_error());
    return 1;
  }
  g_rank = tips_rank();
  g_size = tips_size();
  int64_t total = 0;
  for (int i = 0; i < g_n; i++) {
    Grad* g = &g_g[i];
    g->in = (float*)malloc((size_t)g->n * 4);  /* pageable, as a TF CPU tensor's buffer */
    g->out = (float*)malloc((size_t)g->n * 4); /* the op's allocate_output, reused step after step */
    fill(g->in, g_rank, i, g->n);
    memset(g->out, 0, (size_t)g->n * 4);
    total += g->n;
  }
  for (int i = 0; i < g_n; i++) g_order[i] = i; /* a seeded shuffle, different on every rank */
  uint64_t x = 0x9E3779B97F4A7C15ull * (uint64_t)(g_rank + 1);
  for (int i = g_n - 1; i > 0; i--) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    const int j = (int)(x % (uint64_t)(i + 1)), tmp = g_order[i];
    g_order[i] = g_order[j];
    g_order[j] = tmp;
  }
  pthread_barrier_init(&g_go, NULL, (unsigned)g_threads + 1);
  pthread_t th[MAX_THREADS];
  for (int t = 0; t < g_threads; t++) pthread_create(&th[t], NULL, executor, (void*)(intptr_t)t);
  int rc = 0;
  for (int s = 0; s < warmup && rc == 0; s++) rc = step();
  double best = 1e30, sum = 0;
  double* per = (double*)calloc((size_t)steps, sizeof(double));
  for (int s = 0; s < steps && rc == 0; s++) {
    const double t0 = now();
    rc = step();
    per[s] = now() - t0;
    sum += per[s];
    if (per[s] < best) best = per[s];
  }
  /* the median step: the box's host side is shared (bench.py host_to_host_fused reports the same) */
  for (int a = 1; a < steps; a++)
    for (int b = a; b > 0 && per[b] < per[b - 1]; b--) {
      const double t = per[b];
      per[b] = per[b - 1], per[b - 1] = t;
    }
  const double med = per[steps / 2];
  atomic_store(&g_quit, 1);  /* (a failed step may leave requests open: the threads are only released) */
  pthread_barrier_wait(&g_go);
  for (int t = 0; t < g_threads; t++) pthread_join(th[t], NULL);
  const char* check = "not checked";
  int bad = 0;
  if (rc == 0 && g_size == 1) {
    for (int i = 0; i < g_n; i++) bad += memcmp(g_g[i].in, g_g[i].out, (size_t)g_g[i].n * 4) != 0;
    check = bad ? "FAIL: an output differs from its input" : "identity at one rank, bit-exact";
  }
#ifdef OP_HOST_ORACLE
  if (rc == 0) {
    float** all = (float**)malloc(sizeof(float*) * g_size);
    for (int i = 0; i < g_n && !bad; i++) {
      const Grad* g = &g_g[i];
      float* exp = (float*)malloc((size_t)g->n * 4);
      for (int r = 0; r < g_size; r++) {
        all[r] = (float*)malloc((size_t)g->n * 4);
        fill(all[r], r, i, g->n);
      }
      oracle_fold(ORACLE_F32, exp, (const void* const*)all, g_size, g->n, 1);
      if (memcmp(exp, g->out, (size_t)g->n * 4) != 0) {
        bad++;
        snprintf(g_err, sizeof g_err, "%s differs from the oracle's rank-order fold", g->name);
      }
      for (int r = 0; r < g_size; r++) free(all[r]);
      free(exp);
    }
    free(all);
    check = bad ? "FAIL vs oracle_fold" : "bit-exact vs oracle_fold of all ranks' inputs";
  }
#endif
  char placement[1024];
  thread_placement(placement, sizeof placement);
  tips_shutdown();
  const int ok = rc == 0 && bad == 0;
  const double bytes = (double)total * 4;
  printf("{\"rank\": %d, \"ok\": %s, \"ranks\": %d, \"tensors\": %d, \"elements\": %lld, \"threads\": %d, \"steps\": %d, "
         "\"warmup\": %d, \"ms_per_step\": %.4f, \"ms_mean\": %.4f, \"ms_best\": %.4f, \"algbw_gib_s\": %.3f, "
         "\"check\": \"%s\", \"placement\": \"%s\", \"error\": \"",
         g_rank, ok ? "true" : "false", g_size, g_n, (long long)total, g_threads, steps, warmup, med * 1e3,
         sum / steps * 1e3, best * 1e3, bytes / med / (double)(1ull << 30), check, placement);
  for (const char* c = g_err; *c; c++) putchar(*c == '"' ? '\'' : *c);
  printf("\"}\n");
  free(per);
  return ok ? 0 : 3;
}
