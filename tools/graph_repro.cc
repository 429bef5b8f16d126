// graph_repro.cc — replayed plans (TIPS_GRAPHS) through libtips_hip's C-ABI alone, no Python (the
// HIP runtime and RCCL of /opt/rocm, which is what a C / cgo / JNI host of the library loads).
// Usage: graph_repro RANK SIZE ID_FILE  (schedule from TIPS_ALGO; one process per rank; with
// NCCL_HOSTID per process the ranks may share one GPU over RCCL's socket transport)
// Three buffers reduced round after round with new data, alternating between two streams, one
// buffer freed and reallocated after round 3; each result checked against the sum of all ranks'
// inputs (small integers in f32: exact in any order). Prints the capture / replay counts.
// TIPS_REPRO_TIME=N: then times N calls on the smallest buffer (host enqueue and completion).
// Build: make repro (tools/_bin/graph_repro)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include <chrono>
#include <string>
#include <vector>

#include "tips_hip.h"

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: graph_repro RANK SIZE ID_FILE\n");
    return 2;
  }
  const int rank = atoi(argv[1]), size = atoi(argv[2]);
  const char* idf = argv[3];
  std::vector<char> id(tips_unique_id_bytes());
  if (rank == 0) {
    if (tips_get_unique_id(id.data(), (int64_t)id.size()) < 0) return 1;
    const std::string tmp = std::string(idf) + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return 1;
    fwrite(id.data(), 1, id.size(), f);
    fclose(f);
    rename(tmp.c_str(), idf);
  } else {
    FILE* f = nullptr;
    for (int i = 0; i < 600 && !(f = fopen(idf, "rb")); i++) usleep(100000);
    if (!f || fread(id.data(), 1, id.size(), f) != id.size()) return 1;
    fclose(f);
  }
  if (tips_init_rank(rank, size, 0, id.data(), (int64_t)id.size()) != 0) {
    fprintf(stderr, "init: %s\n", tips_last_error());
    return 1;
  }
  const int64_t ns[3] = {300007, 70001, 4099};
  float* in[3];
  float* out[3];
  for (int b = 0; b < 3; b++)
    if (hipMalloc(&in[b], ns[b] * 4) != hipSuccess || hipMalloc(&out[b], ns[b] * 4) != hipSuccess) return 1;
  hipStream_t st[2];
  for (auto& s : st)
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
  int bad = 0;
  for (int rnd = 0; rnd < 6; rnd++) {
    if (rnd == 3) {  // a new allocation for buffer 0 (perhaps at the same address): a new graph key
      if (hipFree(in[0]) != hipSuccess || hipMalloc(&in[0], ns[0] * 4) != hipSuccess) return 1;
    }
    for (int b = 0; b < 3; b++) {
      hipStream_t s = st[(rnd + b) % 2];
      std::vector<float> h(ns[b]);
      for (int64_t i = 0; i < ns[b]; i++) h[i] = (float)((i * 7 + rnd * 3 + b + rank * 11) % 97);
      if (hipMemcpyAsync(in[b], h.data(), ns[b] * 4, hipMemcpyHostToDevice, s) != hipSuccess) return 1;
      const bool inplace = b == 1;
      if (tips_allreduce(in[b], inplace ? in[b] : out[b], ns[b], TIPS_FLOAT32, TIPS_OP_SUM, s) != 0) {
        fprintf(stderr, "rank %d allreduce: %s\n", rank, tips_last_error());
        return 1;
      }
      std::vector<float> g(ns[b]);
      if (hipMemcpyAsync(g.data(), inplace ? in[b] : out[b], ns[b] * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
        return 1;
      for (int64_t i = 0; i < ns[b]; i++) {
        float want = 0;
        for (int r = 0; r < size; r++) want += (float)((i * 7 + rnd * 3 + b + r * 11) % 97);
        if (g[i] != want) {
          bad++;
          fprintf(stderr, "rank %d round %d buf %d: element %lld is %g, want %g\n", rank, rnd, b, (long long)i, g[i], want);
          break;
        }
      }
    }
  }
  const char* tn = getenv("TIPS_REPRO_TIME");
  double enq_us = 0, call_us = 0;
  if (tn && atoi(tn) > 0) {
    const int N = atoi(tn);
    if (hipStreamSynchronize(st[0]) != hipSuccess) return 1;
    const double t0 = now_us();
    double enq = 0;
    for (int i = 0; i < N; i++) {
      const double a = now_us();
      if (tips_allreduce(in[2], out[2], ns[2], TIPS_FLOAT32, TIPS_OP_SUM, st[0]) != 0) return 1;
      enq += now_us() - a;
    }
    if (hipStreamSynchronize(st[0]) != hipSuccess) return 1;
    enq_us = enq / N;
    call_us = (now_us() - t0) / N;
  }
  int64_t cap = 0, rep = 0, cached = 0;
  const int off = tips_graph_stats(&cap, &rep, &cached);
  printf("{\"rank\": %d, \"size\": %d, \"bad\": %d, \"captured\": %lld, \"replayed\": %lld, \"cached\": %lld, "
         "\"graphs_off\": %d, \"enqueue_us\": %.2f, \"call_us\": %.2f}\n",
         rank, size, bad, (long long)cap, (long long)rep, (long long)cached, off, enq_us, call_us);
  fflush(stdout);
  tips_shutdown();
  return bad ? 1 : 0;
}
