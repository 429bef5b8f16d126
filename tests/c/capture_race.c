/* capture_race.c — a multi-threaded C host that calls tips_allreduce directly (no negotiation) on
 * one thread while three other threads of the process keep making ordinary HIP calls: the case
 * VERDICT r05 asked for after the round-5 op-body crash.
 *
 * Thread A, the caller: P phases; each phase allocates an input and an output buffer and runs
 * three rounds over SIZES bucket sizes (4 KiB .. 4 MiB, every one capture-eligible): round 0 is
 * each plan's first call (eager), round 1 its capture and first replay, round 2 replays. Every
 * result is checked bit-exact against the oracle's rank-order fold (oracle_fold) of every rank's
 * regenerated inputs. The reference issues every collective from one thread
 * (coordinator.cc:355-513); a host that calls the C-ABI directly need not.
 *
 * Threads B-D, the churn (CAPTURE_RACE_CHURN):
 *   none    no churn threads
 *   async   their own non-blocking streams, hipMemcpyAsync + hipStreamSynchronize
 *   streams blocking hipStreamCreate / hipStreamDestroy
 *   free    non-blocking streams, hipMalloc / hipMemcpyAsync / hipFree
 *   legacy  hipMemcpy / hipMemset on the legacy null stream
 *   all     blocking hipStreamCreate / hipMalloc / hipMemcpy / hipMemset / hipFree / hipStreamDestroy
 *           in a loop (tests/c/op_body.c's threads, faster)
 *
 * Replays are opt-in (TIPS_GRAPHS=1): a legacy-null-stream call on another thread invalidates a
 * capture in progress, and RCCL crashes inside it. tests/test_gpu_op_body.py runs
 * the legacy churn with replays at their default (off) and the other churns with replays on.
 * Prints one JSON line with the library's graph counters (tips_graph_stats). Build: make
 * tools/_bin/capture_race. Env: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT (tips_init). */
#include <execinfo.h>
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <signal.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "oracle.h"
#include "tips_hip.h"

#define SIZES 40
#define PHASES 3
#define CHURN_THREADS 3

static int g_rank, g_size;
static const char* g_mode;
static atomic_int g_stop, g_churn_bad;
static atomic_long g_churn_ops;

static float val(int r, int phase, int k, int64_t j) {
  return (float)((r * 7919 + phase * 613 + k * 131 + j * 17) % 2003) * 0.125f - 97.0f;
}
static int64_t size_of(int k) { return 1024 + (int64_t)k * 26189; } /* 4 KiB .. ~4 MiB of f32 */

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

#define CK(x)                                    \
  do {                                           \
    if ((x) != hipSuccess) {                     \
      atomic_store(&g_churn_bad, __LINE__);      \
      return NULL;                               \
    }                                            \
  } while (0)

static void* churn(void* arg) {
  const int id = (int)(intptr_t)arg;
  const size_t n = 1 << 16;
  int* h = (int*)malloc(n * sizeof(int));
  for (size_t j = 0; j < n; j++) h[j] = id;
  int* fixed = NULL;
  hipStream_t own = NULL;
  CK(hipMalloc((void**)&fixed, n * sizeof(int)));
  CK(hipStreamCreateWithFlags(&own, hipStreamNonBlocking));
  while (!atomic_load(&g_stop)) {
    if (!strcmp(g_mode, "async")) {
      CK(hipMemcpyAsync(fixed, h, n * sizeof(int), hipMemcpyHostToDevice, own));
      CK(hipStreamSynchronize(own));
      CK(hipMemcpyAsync(h, fixed, n * sizeof(int), hipMemcpyDeviceToHost, own));
      CK(hipStreamSynchronize(own));
    } else if (!strcmp(g_mode, "streams")) {
      hipStream_t t;
      CK(hipStreamCreate(&t));
      CK(hipStreamDestroy(t));
    } else if (!strcmp(g_mode, "free")) {
      int* d = NULL;
      CK(hipMalloc((void**)&d, n * sizeof(int)));
      CK(hipMemcpyAsync(d, h, n * sizeof(int), hipMemcpyHostToDevice, own));
      CK(hipStreamSynchronize(own));
      CK(hipFree(d));
    } else if (!strcmp(g_mode, "legacy")) {
      CK(hipMemcpy(fixed, h, n * sizeof(int), hipMemcpyHostToDevice));
      CK(hipMemset(fixed, 0, n * sizeof(int)));
      CK(hipMemcpy(h, fixed, n * sizeof(int), hipMemcpyDeviceToHost));
    } else { /* all */
      hipStream_t s;
      int* d = NULL;
      CK(hipStreamCreate(&s));
      CK(hipMalloc((void**)&d, n * sizeof(int)));
      CK(hipMemcpy(d, h, n * sizeof(int), hipMemcpyHostToDevice));
      CK(hipMemset(d, 0, n * sizeof(int)));
      CK(hipMemcpy(h, d, n * sizeof(int), hipMemcpyDeviceToHost));
      CK(hipFree(d));
      CK(hipStreamDestroy(s));
    }
    atomic_fetch_add(&g_churn_ops, 1);
  }
  (void)hipFree(fixed);
  (void)hipStreamDestroy(own);
  free(h);
  return NULL;
}

int main(void) {
  signal(SIGSEGV, on_fatal);
  signal(SIGABRT, on_fatal);
  g_mode = getenv("CAPTURE_RACE_CHURN") ? getenv("CAPTURE_RACE_CHURN") : "all";
  tips_init();
  if (!tips_is_initialize()) {
    printf("{\"ok\": false, \"error\": \"tips_init: %s\"}\n", tips_last_error());
    return 1;
  }
  g_rank = tips_rank();
  g_size = tips_size();
  const int64_t nmax = size_of(SIZES - 1);
  float* h = (float*)malloc(sizeof(float) * nmax);
  float* exp = (float*)malloc(sizeof(float) * nmax);
  float** all = (float**)malloc(sizeof(float*) * g_size);
  for (int r = 0; r < g_size; r++) all[r] = (float*)malloc(sizeof(float) * nmax);
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;

  pthread_t th[CHURN_THREADS];
  int nth = 0;
  if (strcmp(g_mode, "none") != 0)
    for (; nth < CHURN_THREADS; nth++) pthread_create(&th[nth], NULL, churn, (void*)(intptr_t)nth);

  int bad = 0, calls = 0;
  char err[512] = "";
  for (int phase = 0; phase < PHASES && !bad; phase++) {
    float *din = NULL, *dout = NULL;
    if (hipMalloc((void**)&din, sizeof(float) * nmax) != hipSuccess ||
        hipMalloc((void**)&dout, sizeof(float) * nmax) != hipSuccess) {
      snprintf(err, sizeof err, "hipMalloc");
      bad++;
      break;
    }
    for (int round = 0; round < 3 && !bad; round++)
      for (int k = 0; k < SIZES && !bad; k++) {
        const int64_t n = size_of(k);
        for (int r = 0; r < g_size; r++)
          for (int64_t j = 0; j < n; j++) all[r][j] = val(r, phase, k, j) + (float)round;
        if (hipMemcpyAsync(din, all[g_rank], sizeof(float) * n, hipMemcpyHostToDevice, s) != hipSuccess ||
            tips_allreduce(din, dout, n, TIPS_FLOAT32, TIPS_OP_SUM, s) != TIPS_OK ||
            hipMemcpyAsync(h, dout, sizeof(float) * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
          snprintf(err, sizeof err, "phase %d round %d size %d: %s", phase, round, k, tips_last_error());
          bad++;
          break;
        }
        calls++;
        oracle_fold(ORACLE_F32, exp, (const void* const*)all, g_size, n, 1);
        if (memcmp(exp, h, sizeof(float) * n) != 0) {
          snprintf(err, sizeof err, "phase %d round %d size %d differs from the fold", phase, round, k);
          bad++;
        }
      }
    (void)hipFree(din);
    (void)hipFree(dout);
  }
  atomic_store(&g_stop, 1);
  for (int k = 0; k < nth; k++) pthread_join(th[k], NULL);
  int64_t captured = 0, replayed = 0, cached = 0;
  const int gs = tips_graph_stats(&captured, &replayed, &cached);
  tips_shutdown();
  const int ok = !bad && !atomic_load(&g_churn_bad);
  printf("{\"rank\": %d, \"ok\": %s, \"mode\": \"%s\", \"calls\": %d, \"captured\": %lld, \"replayed\": %lld, "
         "\"graph_state\": %d, \"churn_ops\": %ld, \"churn_bad_line\": %d, \"error\": \"%s\"}\n",
         g_rank, ok ? "true" : "false", g_mode, calls, (long long)captured, (long long)replayed, gs,
         atomic_load(&g_churn_ops), atomic_load(&g_churn_bad), err);
  return ok ? 0 : 3;
}
