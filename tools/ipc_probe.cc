// ipc_probe.cc — hipIpcGetMemHandle across the peer schedule's workspace growth.
//   single:  ./ipc_probe single           one process: alloc/export/free sizes 2..256 MiB, 3 kinds
//   pair:    ./ipc_probe pair RANK DIR KIND MODE
//            two processes (same GPU): each round, both export a workspace, import the
//            other's, then grow. MODE 0: close imports, alloc new, export (the first design);
//            MODE 1: alloc new + export while the imports are still open, then close them;
//            MODE 2: as 0, but on an export failure keep the buffer and allocate another.
//   hipcc --offload-arch=gfx950 -O2 -o tools/ipc_probe tools/ipc_probe.cc
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <vector>

static hipError_t alloc(void** p, size_t bytes, int kind) {
  return kind == 0 ? hipMalloc(p, bytes)
                   : hipExtMallocWithFlags(p, bytes, kind == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached);
}

static void put(const std::string& path, const void* buf, size_t n) {
  std::string tmp = path + ".tmp";
  FILE* f = fopen(tmp.c_str(), "wb");
  fwrite(buf, 1, n, f);
  fclose(f);
  rename(tmp.c_str(), path.c_str());
}

static void get(const std::string& path, void* buf, size_t n) {
  for (;;) {
    FILE* f = fopen(path.c_str(), "rb");
    if (f) {
      size_t r = fread(buf, 1, n, f);
      fclose(f);
      if (r == n) return;
    }
    usleep(1000);
  }
}

int pair(int rank, const char* dir, int kind, int mode) {
  hipSetDevice(0);
  void* ws = nullptr;
  void* remote = nullptr;
  int fails = 0, exports = 0;
  std::vector<void*> parked;
  for (int round = 0; round < 8; round++) {
    size_t bytes = (size_t)(2 << 20) << round;  // 2, 4, ... 256 MiB
    if (mode != 1 && remote) { hipIpcCloseMemHandle(remote); remote = nullptr; }
    void* old = ws;
    hipIpcMemHandle_t h;
    hipError_t e;
    for (int attempt = 0;; attempt++) {
      if (alloc(&ws, bytes, kind) != hipSuccess) { printf("alloc failed\n"); return 1; }
      e = hipIpcGetMemHandle(&h, ws);
      exports++;
      if (e == hipSuccess) break;
      fails++;
      printf("rank %d round %d attempt %d: export of %zu MiB at %p failed: %s\n", rank, round, attempt, bytes >> 20, ws,
             hipGetErrorString(e));
      (void)hipGetLastError();
      if (mode != 2 || attempt >= 4) return 2;
      parked.push_back(ws);
    }
    for (void* q : parked) hipFree(q);
    parked.clear();
    if (mode == 1 && remote) { hipIpcCloseMemHandle(remote); remote = nullptr; }
    char path[512];
    snprintf(path, sizeof path, "%s/h_%d_%d", dir, rank, round);
    put(path, &h, sizeof h);
    snprintf(path, sizeof path, "%s/h_%d_%d", dir, 1 - rank, round);
    hipIpcMemHandle_t ph;
    get(path, &ph, sizeof ph);
    e = hipIpcOpenMemHandle(&remote, ph, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) { printf("rank %d round %d: open failed: %s\n", rank, round, hipGetErrorString(e)); return 3; }
    // both sides have opened before either frees its old buffer
    snprintf(path, sizeof path, "%s/o_%d_%d", dir, rank, round);
    put(path, &round, sizeof round);
    snprintf(path, sizeof path, "%s/o_%d_%d", dir, 1 - rank, round);
    int x;
    get(path, &x, sizeof x);
    if (old) hipFree(old);
  }
  if (remote) hipIpcCloseMemHandle(remote);
  hipFree(ws);
  printf("{\"rank\": %d, \"kind\": %d, \"mode\": %d, \"exports\": %d, \"failures\": %d}\n", rank, kind, mode, exports, fails);
  return 0;
}

int single() {
  const char* kinds[] = {"coarse", "fine", "uncached"};
  for (int kind = 0; kind < 3; kind++) {
    void* old = nullptr;
    int fails = 0, total = 0;
    for (int round = 0; round < 3; round++) {
      for (size_t mb = 2; mb <= 256; mb *= 2) {
        void* p = nullptr;
        if (alloc(&p, mb << 20, kind) != hipSuccess) return 1;
        hipIpcMemHandle_t h;
        hipError_t e = hipIpcGetMemHandle(&h, p);
        total++;
        if (e != hipSuccess) {
          fails++;
          (void)hipGetLastError();
        }
        if (old) (void)hipFree(old);
        old = p;
      }
    }
    if (old) (void)hipFree(old);
    printf("{\"kind\": \"%s\", \"handles\": %d, \"failures\": %d}\n", kinds[kind], total, fails);
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 6 && !strcmp(argv[1], "pair")) return pair(atoi(argv[2]), argv[3], atoi(argv[4]), atoi(argv[5]));
  return single();
}
