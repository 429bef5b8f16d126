/* tsan_selftest.c — the library's own multi-threaded host paths under ThreadSanitizer (CPU only).
 *
 * Linked against tools/lib/libtips_hip_tsan.so: the same sources as libtips_hip.so with the HOST
 * code built -fsanitize=thread (device code is unchanged; `make tsan`). tests/test_tsan.py runs:
 *   neg RANK SIZE PORT FILE   one rank of tips_negotiation_selftest with FILE's request script
 *                             (dry-run executor: the negotiation thread, the TCP lockstep cycles,
 *                             the completion thread and several issuing threads with callbacks)
 *   pool THREADS RUNS JOBS    tips_host_pool_selftest (the fused host path's copy pool)
 * Exit status: the selftest's return code, or ThreadSanitizer's (TSAN_OPTIONS exitcode) on a race. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tips_hip_dev.h"

static char* slurp(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  char* s = (char*)malloc((size_t)n + 1);
  if (s && fread(s, 1, (size_t)n, f) != (size_t)n) n = 0;
  if (s) s[n] = 0;
  fclose(f);
  return s;
}

int main(int argc, char** argv) {
  if (argc == 6 && strcmp(argv[1], "neg") == 0) {
    char* req = slurp(argv[5]);
    if (!req) return 2;
    static char out[1 << 16];
    int rc = tips_negotiation_selftest(atoi(argv[2]), atoi(argv[3]), "127.0.0.1", atoi(argv[4]), req, out, sizeof out);
    fputs(out, stdout);
    if (rc) fprintf(stderr, "rc %d: %s\n", rc, tips_last_error());
    free(req);
    return rc ? 1 : 0;
  }
  if (argc == 5 && strcmp(argv[1], "pool") == 0) {
    int rc = tips_host_pool_selftest(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]));
    if (rc) fprintf(stderr, "rc %d: %s\n", rc, tips_last_error());
    return rc ? 1 : 0;
  }
  fprintf(stderr, "usage: %s neg RANK SIZE PORT FILE | pool THREADS RUNS JOBS\n", argv[0]);
  return 2;
}
