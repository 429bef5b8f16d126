/* op_body.c — the TF op-body pattern of INTEGRATION.md §2 through the C-ABI alone, one process
 * per rank (tests/test_gpu_op_body.py starts the ranks; each is a real RCCL rank).
 *
 * What the reference's ops do (tips/tensorflow/ops.cc:86-118, coordinator.cc:223-241 / 355-513,
 * pinned by coordinator_test.cc:10-45): a TF executor thread runs ComputeAsync, which enqueues the
 * tensor under the op's name with a callback and returns; the coordinator runs every name in rank
 * 0's readiness order and the callback sets the status and calls done(). TF issues the ops on
 * several threads, in a different order on every rank.
 *
 * Here, per rank: four "executor" threads issue named requests for their share of the tensors, in a
 * per-rank shuffled order - allreduces of device (hipMalloc) f32 and i32 tensors, allreduces of
 * host f32 tensors (the reference's ops are CPU ops), and a broadcast - each completed through a
 * tips_on_done callback; a fifth thread meanwhile issues synchronous tips_allreduce calls on its
 * own device buffer, which the library routes through the same negotiation. main waits for every
 * callback, checks every output bit-exact against the oracle's rank-order fold (oracle_fold) of
 * every rank's regenerated inputs, and prints one JSON line.
 *
 * Build: make tools/_bin/op_body. Env: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT (tips_init), and
 * OP_BODY_TENSORS (default 96). */
#include <dirent.h>
#include <execinfo.h>
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <sys/syscall.h>
#include <signal.h>
#include <stdatomic.h>
#include <unistd.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "oracle.h"
#include "tips_hip.h"

#define THREADS 4
#define SYNC_CALLS 12
#define SYNC_N 40000

enum { KIND_DEV_F32 = 0, KIND_DEV_I32 = 1, KIND_HOST_F32 = 2, KIND_BCAST = 3 };

typedef struct {
  int index, kind;
  int64_t n;
  void* in;   /* device or host */
  void* out;
  atomic_int status;
  atomic_int done;
  char msg[256];
} Tensor;

static int g_rank, g_size, g_ntensors;
/* OP_BODY_NONBLOCKING=1: the threads' streams are created non-blocking and the synchronous caller
 * copies with hipMemcpyAsync + hipStreamSynchronize on its own stream (no legacy null stream) */
static int g_nonblocking;
static hipError_t make_stream(hipStream_t* s) {
  return g_nonblocking ? hipStreamCreateWithFlags(s, hipStreamNonBlocking) : hipStreamCreate(s);
}
static hipError_t copy_sync(void* dst, const void* src, size_t n, hipMemcpyKind k, hipStream_t s) {
  if (!g_nonblocking) return hipMemcpy(dst, src, n, k);
  hipError_t e = hipMemcpyAsync(dst, src, n, k, s);
  return e != hipSuccess ? e : hipStreamSynchronize(s);
}
static Tensor* g_t;
static atomic_int g_callbacks;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_cv = PTHREAD_COND_INITIALIZER;
static char g_err[4096];

static void note(const char* fmt, const char* a, int b) {
  pthread_mutex_lock(&g_mu);
  size_t l = strlen(g_err);
  if (l < sizeof g_err - 200) snprintf(g_err + l, sizeof g_err - l, fmt, a, b);
  pthread_mutex_unlock(&g_mu);
}

/* deterministic inputs: rank r's element j of tensor i */
static float f32_of(int r, int i, int64_t j) { return (float)((r * 7919 + i * 131 + j * 17) % 2003) * 0.125f - 97.0f; }
static int32_t i32_of(int r, int i, int64_t j) { return (int32_t)(r * 1000003 + i * 7777 + j * 2654435761u); }
static int64_t n_of(int i) { return 1 + (int64_t)((i * 2654435761u) % 60000); }
static int kind_of(int i) { return i % 13 == 5 ? KIND_BCAST : i % 3; }

static void fill(void* h, int r, int i, int kind, int64_t n) {
  for (int64_t j = 0; j < n; j++) {
    if (kind == KIND_DEV_I32) ((int32_t*)h)[j] = i32_of(r, i, j);
    else ((float*)h)[j] = f32_of(r, i, j);
  }
}

static void on_done(void* ctx, int status, const char* message) {
  Tensor* t = (Tensor*)ctx;
  atomic_store(&t->status, status);
  if (status) snprintf(t->msg, sizeof t->msg, "%s", message);
  atomic_store(&t->done, 1);
  pthread_mutex_lock(&g_mu);
  atomic_fetch_add(&g_callbacks, 1);
  pthread_cond_broadcast(&g_cv);
  pthread_mutex_unlock(&g_mu);
}

typedef struct {
  int thread;
  int* order; /* this rank's shuffled tensor order */
} Job;

static void* executor(void* arg) {
  const Job* job = (const Job*)arg;
  hipStream_t s;
  if (make_stream(&s) != hipSuccess) {
    note("%sthread %d: hipStreamCreate failed; ", "", job->thread);
    return NULL;
  }
  for (int k = 0; k < g_ntensors; k++) {
    const int i = job->order[k];
    if (i % THREADS != job->thread) continue;
    Tensor* t = &g_t[i];
    char name[64];
    snprintf(name, sizeof name, "model/layer%d/grad", i);
    const int dtype = t->kind == KIND_DEV_I32 ? TIPS_INT32 : TIPS_FLOAT32;
    int64_t h;
    int registered = 0; /* the callback came with the request (tips_enqueue_allreduce_cb) */
    if (t->kind == KIND_BCAST) {
      const int64_t shape[1] = {t->n};
      h = tips_enqueue_broadcast(name, t->in, t->out, shape, 1, dtype, 1 % g_size, s);
    } else {
      const int64_t shape[2] = {t->n / 2 ? 2 : 1, t->n / 2 ? t->n / 2 : t->n};
      if (t->n % 2 == 0 && t->n > 1 && i % 3 == 0) { /* a third of the shaped ones: request + callback in one call */
        h = tips_enqueue_allreduce_cb(name, t->in, t->out, shape, 2, dtype, t->kind == KIND_HOST_F32 ? NULL : s,
                                      on_done, t);
        registered = 1;
      } else if (t->n % 2 == 0 && t->n > 1) {
        h = tips_enqueue_allreduce_shaped(name, t->in, t->out, shape, 2, dtype, t->kind == KIND_HOST_F32 ? NULL : s);
      } else {
        h = tips_enqueue_allreduce(name, t->in, t->out, t->n, dtype, t->kind == KIND_HOST_F32 ? NULL : s);
      }
    }
    if (h < 0 || (!registered && tips_on_done(h, on_done, t) != TIPS_OK)) {
      note("%s (tensor %d); ", tips_last_error(), i);
      atomic_store(&t->status, -1);
      atomic_store(&t->done, 1);
      pthread_mutex_lock(&g_mu);
      atomic_fetch_add(&g_callbacks, 1);
      pthread_cond_broadcast(&g_cv);
      pthread_mutex_unlock(&g_mu);
    }
  }
  return NULL;
}

/* synchronous collectives from yet another thread, while named requests are in flight: routed */
static atomic_int g_sync_bad;
static void* sync_caller(void* arg) {
  (void)arg;
  hipStream_t s;
  float *d = NULL, *o = NULL;
  float* h = (float*)malloc(sizeof(float) * SYNC_N);
  float* exp = (float*)malloc(sizeof(float) * SYNC_N);
  float** all = (float**)malloc(sizeof(float*) * g_size);
  if (make_stream(&s) != hipSuccess || hipMalloc((void**)&d, sizeof(float) * SYNC_N) != hipSuccess ||
      hipMalloc((void**)&o, sizeof(float) * SYNC_N) != hipSuccess) {
    atomic_store(&g_sync_bad, 1);
    return NULL;
  }
  for (int r = 0; r < g_size; r++) all[r] = (float*)malloc(sizeof(float) * SYNC_N);
  for (int c = 0; c < SYNC_CALLS; c++) {
    for (int r = 0; r < g_size; r++)
      for (int64_t j = 0; j < SYNC_N; j++) all[r][j] = f32_of(r, 100000 + c, j);
    if (copy_sync(d, all[g_rank], sizeof(float) * SYNC_N, hipMemcpyHostToDevice, s) != hipSuccess ||
        tips_allreduce(d, o, SYNC_N, TIPS_FLOAT32, TIPS_OP_SUM, s) != TIPS_OK || hipStreamSynchronize(s) != hipSuccess ||
        copy_sync(h, o, sizeof(float) * SYNC_N, hipMemcpyDeviceToHost, s) != hipSuccess) {
      note("sync call: %s (%d); ", tips_last_error(), c);
      atomic_store(&g_sync_bad, 1);
      break;
    }
    oracle_fold(ORACLE_F32, exp, (const void* const*)all, g_size, SYNC_N, 1);
    if (memcmp(exp, h, sizeof(float) * SYNC_N) != 0) {
      note("%ssync call %d differs from the fold; ", "", c);
      atomic_store(&g_sync_bad, 1);
    }
  }
  for (int r = 0; r < g_size; r++) free(all[r]);
  free(all);
  free(h);
  free(exp);
  (void)hipFree(d);
  (void)hipFree(o);
  return NULL;
}

/* a watchdog thread: while the run is not finished it reports at 60 and 120 s what the library's
 * threads are doing (tips_debug_state) and which tensors are still open, and at 200 s ends the
 * process with a JSON line saying how far it got and that report */
static atomic_int g_finished;
static void report(char* b, size_t cap) {
  char st[3072];
  tips_debug_state(st, sizeof st);
  size_t l = (size_t)snprintf(b, cap, "callbacks %d of %d; state: %s; open:", atomic_load(&g_callbacks), g_ntensors, st);
  int shown = 0;
  for (int i = 0; i < g_ntensors && shown < 12 && l < cap - 64; i++)
    if (!atomic_load(&g_t[i].done)) {
      l += (size_t)snprintf(b + l, cap - l, " %d(kind %d)", i, g_t[i].kind);
      shown++;
    }
  for (char* c = b; *c; c++)
    if (*c == '"') *c = '\'';
}

/* every thread's stack on stderr (module+offset frames; tools/symbolize_stacks.py names them):
 * each thread of the process is sent SIGUSR1 in turn and prints its own backtrace */
static void on_usr1(int sig) {
  (void)sig;
  void* fr[48];
  const int n = backtrace(fr, 48);
  char hdr[64];
  const int l = snprintf(hdr, sizeof hdr, "--- thread %ld\n", (long)syscall(SYS_gettid));
  if (write(2, hdr, (size_t)l) < 0) return;
  backtrace_symbols_fd(fr, n, 2);
}

/* a fatal signal: the faulting thread's stack on stderr, then the default action */
static void on_fatal(int sig) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  char hdr[96];
  const int l = snprintf(hdr, sizeof hdr, "--- fatal signal %d in thread %ld\n", sig, (long)syscall(SYS_gettid));
  if (write(2, hdr, (size_t)l) < 0) _exit(128 + sig);
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

static void dump_stacks(void) {
  signal(SIGUSR1, on_usr1);
  const long self = (long)syscall(SYS_gettid);
  DIR* d = opendir("/proc/self/task");
  if (!d) return;
  struct dirent* e;
  while ((e = readdir(d)) != NULL) {
    const long tid = atol(e->d_name);
    if (tid <= 0 || tid == self) continue;
    syscall(SYS_tgkill, (long)getpid(), tid, SIGUSR1);
    usleep(50000);
  }
  closedir(d);
}

static void* watchdog(void* arg) {
  (void)arg;
  static char b[4096];
  for (int t = 1; t <= 200; t++) {
    sleep(1);
    if (atomic_load(&g_finished)) return NULL;
    if (t == 60 || t == 120) {
      report(b, sizeof b);
      fprintf(stderr, "[op_body rank %d] t=%ds %s\n", g_rank, t, b);
      if (t == 60) dump_stacks();
    }
  }
  report(b, sizeof b);
  fprintf(stderr, "[op_body rank %d] t=200s %s\n", g_rank, b);
  printf("{\"rank\": %d, \"ok\": false, \"error\": \"watchdog: %s\"}\n", g_rank, b);
  fflush(stdout);
  _exit(4);
  return NULL;
}

int main(void) {
  const char* nt = getenv("OP_BODY_TENSORS");
  g_nonblocking = getenv("OP_BODY_NONBLOCKING") && atoi(getenv("OP_BODY_NONBLOCKING")) != 0;
  g_ntensors = nt ? atoi(nt) : 96;
  signal(SIGSEGV, on_fatal);
  signal(SIGABRT, on_fatal);
  tips_init();
  if (!tips_is_initialize()) {
    printf("{\"ok\": false, \"error\": \"tips_init: %s\"}\n", tips_last_error());
    return 1;
  }
  g_rank = tips_rank();
  g_size = tips_size();
  g_t = (Tensor*)calloc((size_t)g_ntensors, sizeof(Tensor));
  pthread_t wd;
  pthread_create(&wd, NULL, watchdog, NULL);
  pthread_detach(wd);
  for (int i = 0; i < g_ntensors; i++) {
    Tensor* t = &g_t[i];
    t->index = i;
    t->kind = kind_of(i);
    t->n = n_of(i);
    const size_t bytes = (size_t)t->n * 4;
    void* h = malloc(bytes);
    fill(h, g_rank, i, t->kind, t->n);
    if (t->kind == KIND_HOST_F32) {
      t->in = h;
      t->out = malloc(bytes);
    } else {
      if (hipMalloc(&t->in, bytes) != hipSuccess || hipMalloc(&t->out, bytes) != hipSuccess ||
          hipMemcpy(t->in, h, bytes, hipMemcpyHostToDevice) != hipSuccess) {
        printf("{\"ok\": false, \"error\": \"hipMalloc\"}\n");
        return 1;
      }
      free(h);
    }
  }
  /* this rank's order: a seeded shuffle, different on every rank */
  int* order = (int*)malloc(sizeof(int) * g_ntensors);
  for (int i = 0; i < g_ntensors; i++) order[i] = i;
  uint64_t x = 0x9E3779B97F4A7C15ull * (uint64_t)(g_rank + 1);
  for (int i = g_ntensors - 1; i > 0; i--) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    const int j = (int)(x % (uint64_t)(i + 1));
    const int tmp = order[i];
    order[i] = order[j];
    order[j] = tmp;
  }
  /* the negotiation starts with a first named request on every rank before any thread runs: a
   * synchronous collective issued before it on one rank and after it on another would be direct
   * on one and routed on the other (the join refuses such a start, but the direct call would
   * already be waiting in RCCL for a partner that never comes) */
  {
    float* d = NULL;
    if (hipMalloc((void**)&d, 1024) != hipSuccess) return 1;
    const int64_t h = tips_enqueue_allreduce("op_body/start", d, d, 256, TIPS_FLOAT32, NULL);
    if (h < 0 || tips_wait(h) != TIPS_OK) {
      printf("{\"rank\": %d, \"ok\": false, \"error\": \"start: %s\"}\n", g_rank, tips_last_error());
      return 1;
    }
    (void)hipFree(d);
    fprintf(stderr, "[op_body rank %d] negotiation started\n", g_rank);
  }
  /* OP_BODY_PASSES training steps (default 2) over the same names, each in this rank's order,
   * reversed every other step: from the second step on, the names every rank announces by id
   * (the negotiation's response cache) come back decided without rank 0's table */
  const int passes = getenv("OP_BODY_PASSES") ? atoi(getenv("OP_BODY_PASSES")) : 2;
  int callbacks = 0, bad = 0;
  void** all = (void**)malloc(sizeof(void*) * g_size);
  for (int pass = 0; pass < passes && bad == 0; pass++) {
    if (pass > 0) {
      for (int i = 0; i < g_ntensors; i++) {  /* fresh outputs: a stale one from the last step must not pass */
        Tensor* t = &g_t[i];
        atomic_store(&t->done, 0);
        atomic_store(&t->status, 0);
        if (t->kind == KIND_HOST_F32) memset(t->out, 0xA5, (size_t)t->n * 4);
        else if (hipMemset(t->out, 0xA5, (size_t)t->n * 4) != hipSuccess) note("%shipMemset of tensor %d; ", "", i);
      }
      for (int i = 0; i < g_ntensors / 2; i++) {
        const int tmp = order[i];
        order[i] = order[g_ntensors - 1 - i];
        order[g_ntensors - 1 - i] = tmp;
      }
      atomic_store(&g_callbacks, 0);
    }
    pthread_t th[THREADS + 1];
    Job jobs[THREADS];
    for (int k = 0; k < THREADS; k++) {
      jobs[k].thread = k;
      jobs[k].order = order;
      pthread_create(&th[k], NULL, executor, &jobs[k]);
    }
    pthread_create(&th[THREADS], NULL, sync_caller, NULL);
    for (int k = 0; k <= THREADS; k++) pthread_join(th[k], NULL);
    /* every callback, bounded */
    struct timespec dl;
    clock_gettime(CLOCK_REALTIME, &dl);
    dl.tv_sec += 120;
    pthread_mutex_lock(&g_mu);
    while (atomic_load(&g_callbacks) < g_ntensors)
      if (pthread_cond_timedwait(&g_cv, &g_mu, &dl) != 0) break;
    pthread_mutex_unlock(&g_mu);
    callbacks = atomic_load(&g_callbacks);
    if (callbacks != g_ntensors) break;
    for (int i = 0; i < g_ntensors && callbacks == g_ntensors; i++) {
      Tensor* t = &g_t[i];
      const size_t bytes = (size_t)t->n * 4;
      if (atomic_load(&t->status) != 0) {
        note("tensor failed: %s (%d); ", t->msg, i);
        bad++;
        continue;
      }
      void* got = malloc(bytes);
      void* exp = malloc(bytes);
      if (t->kind == KIND_HOST_F32) memcpy(got, t->out, bytes);
      else if (hipMemcpy(got, t->out, bytes, hipMemcpyDeviceToHost) != hipSuccess) note("%sD2H of tensor %d; ", "", i);
      for (int r = 0; r < g_size; r++) {
        all[r] = malloc(bytes);
        fill(all[r], r, i, t->kind, t->n);
      }
      if (t->kind == KIND_BCAST) memcpy(exp, all[1 % g_size], bytes);
      else oracle_fold(t->kind == KIND_DEV_I32 ? ORACLE_I32 : ORACLE_F32, exp, (const void* const*)all, g_size, t->n, 1);
      if (memcmp(got, exp, bytes) != 0) {
        note("%stensor %d differs from the oracle; ", "", i);
        bad++;
      }
      for (int r = 0; r < g_size; r++) free(all[r]);
      free(got);
      free(exp);
    }
  }
  int64_t captured = 0, replayed = 0, cached = 0;
  (void)tips_graph_stats(&captured, &replayed, &cached);
  tips_shutdown();
  atomic_store(&g_finished, 1);
  const int ok = callbacks == g_ntensors && bad == 0 && !atomic_load(&g_sync_bad);
  printf("{\"rank\": %d, \"ok\": %s, \"callbacks\": %d, \"tensors\": %d, \"passes\": %d, \"sync_calls\": %d, "
         "\"captured\": %lld, \"replayed\": %lld, \"error\": \"", g_rank, ok ? "true" : "false", callbacks, g_ntensors,
         passes, SYNC_CALLS, (long long)captured, (long long)replayed);
  for (const char* c = g_err; *c; c++) putchar(*c == '"' ? '\'' : *c);
  printf("\"}\n");
  return ok ? 0 : 3;
}
