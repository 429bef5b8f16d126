// sum_sweep.cc — gfx950 tuning sweep for the 2-input bucket-sum kernel.
//
// Config 2 of BASELINE.json: c = a + b over two 256 MiB fp32 buffers, all
// variants of tips_sum_variant interleaved in ONE process (guide §5.4 rule 24:
// N variants x M rounds, report median and min), plus hipMemcpy D2D as the
// streaming reference on the same device. Random data (rule 25).
// Prints one JSON object per variant.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <string>
#include <vector>

#include "../include/tips_hip_dev.h"

#define CHECK(x)                                                                              \
  do {                                                                                        \
    hipError_t e = (x);                                                                       \
    if (e != hipSuccess) {                                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));        \
      exit(1);                                                                                \
    }                                                                                         \
  } while (0)

struct Variant {
  std::string name;
  int mode, unroll, nt, blocks, threads;  // mode -1 = memcpy reference, -3 = tips_bucket_sum default
  std::vector<double> ms;
};

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : (int64_t)67108864;  // 256 MiB fp32
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  const int iters = argc > 3 ? atoi(argv[3]) : 20;
  const size_t bytes = (size_t)n * 4;
  // SWEEP_PAD="pb,pc": each (a, b, c) triple is carved from ONE allocation, b starting pb bytes
  // after a's end and c pc bytes after b's end (their relative placement modulo the DRAM channel /
  // bank interleave). Unset: three separate hipMallocs (2 MiB-aligned, the placement torch gives).
  const char* pad_env = getenv("SWEEP_PAD");
  int64_t pad_b = 0, pad_c = 0;
  if (pad_env) sscanf(pad_env, "%ld,%ld", &pad_b, &pad_c);
  auto alloc3 = [&](float** x, float** y, float** z) {
    if (!pad_env) {
      CHECK(hipMalloc(x, bytes));
      CHECK(hipMalloc(y, bytes));
      CHECK(hipMalloc(z, bytes));
      return;
    }
    char* base = nullptr;
    CHECK(hipMalloc((void**)&base, 3 * bytes + pad_b + pad_c));
    *x = (float*)base;
    *y = (float*)(base + bytes + pad_b);
    *z = (float*)(base + 2 * bytes + pad_b + pad_c);
  };
  float *a, *b, *c;
  alloc3(&a, &b, &c);
  {
    std::vector<float> h(n);
    std::mt19937 g(1);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    for (auto& x : h) x = u(g);
    CHECK(hipMemcpy(a, h.data(), bytes, hipMemcpyHostToDevice));
    for (auto& x : h) x = u(g);
    CHECK(hipMemcpy(b, h.data(), bytes, hipMemcpyHostToDevice));
  }
  // SWEEP_ROT=R: every timed launch uses the next of R (a, b, c) triples. With R >= 2 at 256 MiB no
  // launch finds its operands in the 256 MiB Infinity Cache from an earlier one, so the rate is
  // HBM's; R = 1 (default) re-reads the same buffers, which the Infinity Cache partly serves.
  const char* rot_env = getenv("SWEEP_ROT");
  const int rot = std::max(1, std::min(8, rot_env ? atoi(rot_env) : 1));
  float *A[8] = {a}, *B[8] = {b}, *C[8] = {c};
  for (int r = 1; r < rot; r++) {
    alloc3(&A[r], &B[r], &C[r]);
    CHECK(hipMemcpy(A[r], a, bytes, hipMemcpyDeviceToDevice));
    CHECK(hipMemcpy(B[r], b, bytes, hipMemcpyDeviceToDevice));
  }
  int next_set = 0;
  auto rotate = [&]() {
    const int r = next_set++ % rot;
    a = A[r];
    b = B[r];
    c = C[r];
  };
  std::vector<Variant> vs;
  vs.push_back({"memcpy_d2d", -1, 0, 0, 0, 0, {}});
  vs.push_back({"default", -3, 0, 0, 0, 0, {}});
  vs.push_back({"multi_sum_8src", -4, 0, 0, 0, 0, {}});  // 8 x (n/8) sources -> n/8 output (direct-algorithm kernel)
  const char* ntn[] = {"", "_nt", "_ntld", "_ntst"};
  // (mode 1 = one tile per workgroup) unroll, nt, threads — the f32 variants kernels.hip instantiates
  const int tiles[][3] = {{1, 0, 256}, {2, 0, 256}, {4, 0, 256}, {8, 0, 256}, {1, 1, 256}, {2, 1, 256}, {4, 1, 256},
                          {8, 1, 256}, {2, 2, 256}, {4, 2, 256}, {2, 3, 256}, {4, 3, 256}, {2, 1, 512}, {4, 1, 512},
                          {8, 1, 512}, {1, 1, 1024}, {2, 1, 1024}, {4, 1, 1024}, {4, 2, 512}, {4, 3, 512},
                          {16, 1, 256}, {16, 1, 128}, {8, 1, 128}, {4, 1, 128}, {8, 1, 64},
                          {1, 2, 256}, {8, 2, 256}, {2, 2, 512}, {2, 2, 128}, {1, 2, 512}};
  for (auto& t : tiles)
    vs.push_back({"tile_u" + std::to_string(t[0]) + ntn[t[1]] + "_t" + std::to_string(t[2]), 1, t[0], t[1], 0, t[2], {}});
  const int xcd[][3] = {{1, 2, 256}, {2, 2, 256}, {1, 2, 512}, {4, 1, 256}};
  const char* cpol[] = {"ld_nt/st_plain",   "ld_nt/st_sc1",    "ld_nt/st_sc0sc1", "ld_ntsc1/st_plain",
                        "ld_sc0nt/st_plain", "ld_sc1/st_plain", "ld_ntsc1/st_sc1", "ld_nt/st_nt",
                        "ld_plain/st_sc1",   "ld_sc0nt/st_sc0sc1"};
  for (int i = 0; i < 10; i++) vs.push_back({std::string("buf_") + cpol[i], 3, 1, i, 0, 256, {}});
  const char* stpol[] = {"ld_nt/st_ntsc1", "ld_nt/st_sc0ntsc1", "ld_nt/st_sc0", "ld_nt/st_sc0nt"};
  for (int i = 0; i < 4; i++) vs.push_back({std::string("buf_") + stpol[i], 3, 1, 10 + i, 0, 256, {}});
  for (int kib : {20, 24, 32, 40, 54, 64})  // the default with k KiB of LDS reserved: 160 / k workgroups per CU
    vs.push_back({"buf_ntsc1_occ_lds" + std::to_string(kib) + "k", 3, 1, 1, kib * 1024, 256, {}});
  const int bufshape[][2] = {{2, 256}, {4, 256}, {1, 512}, {2, 128}, {1, 1024}, {1, 128}, {2, 512}};
  for (auto& t : bufshape)
    vs.push_back({"buf_ntsc1_u" + std::to_string(t[0]) + "_t" + std::to_string(t[1]), 3, t[0], 1, 0, t[1], {}});
  const int ntnt[][2] = {{1, 512}, {1, 1024}, {2, 256}, {4, 256}, {2, 512}};  // buffer nt loads + nt stores
  for (auto& t : ntnt)
    vs.push_back({"buf_ntnt_u" + std::to_string(t[0]) + "_t" + std::to_string(t[1]), 3, t[0], 7, 0, t[1], {}});
  for (int w : {1, 2, 4, 8})  // persistent streaming, w workgroups per CU, 2-deep pipeline (mode 5)
    vs.push_back({"stream_w" + std::to_string(w), 5, w, 0, 0, 256, {}});
  for (int u : {1, 2, 4})  // LDS-staged through direct-to-LDS loads (mode 4)
    vs.push_back({"lds_glds_u" + std::to_string(u) + "_t256", 4, u, 0, 0, 256, {}});
  for (auto& t : xcd)
    vs.push_back({"xcd_u" + std::to_string(t[0]) + ntn[t[1]] + "_t" + std::to_string(t[2]), 2, t[0], t[1], 0, t[2], {}});
  for (int u : {1, 2, 4, 8})
    for (int bpc : {2, 8, 16})
      vs.push_back({"gs_u" + std::to_string(u) + "_b" + std::to_string(bpc) + "_nt", 0, u, 1, 256 * bpc, 256, {}});
  for (int u : {2, 4})
    for (int bpc : {2, 4, 8})
      vs.push_back({"gs_u" + std::to_string(u) + "_b" + std::to_string(bpc) + "_ntld", 0, u, 2, 256 * bpc, 256, {}});
  // multi-input sum variants (tips_multi_sum_variant): unroll field = nsrc, nt field = variant
  // blocks field = extra bytes between consecutive sources (0 = back to back, power-of-2 strides)
  for (int ns : {4, 8})
    for (int var = 0; var <= 7; var++)
      for (int pad : {0, 4096})
        vs.push_back({"multi" + std::to_string(ns) + "_v" + std::to_string(var) + "_pad" + std::to_string(pad), -5, ns,
                      var, pad, 0, {}});
  if (argc > 4) {  // optional name filter: comma-separated substrings (exact name with a leading '='); references stay
    std::vector<std::string> pats;
    for (std::string f = argv[4]; !f.empty();) {
      const size_t k = f.find(',');
      pats.push_back(f.substr(0, k));
      f = (k == std::string::npos) ? "" : f.substr(k + 1);
    }
    std::vector<Variant> keep;
    for (auto& v : vs) {
      bool hit = v.mode == -1 || v.mode == -3;
      for (auto& p : pats)
        hit = hit || (p[0] == '=' ? v.name == p.substr(1) : v.name.find(p) != std::string::npos);
      if (hit) keep.push_back(v);
    }
    vs.swap(keep);
  }
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto run = [&](Variant& v) {
    if (v.mode == -1) {
      CHECK(hipMemcpyAsync(c, a, bytes, hipMemcpyDeviceToDevice, s));
    } else if (v.mode == -4) {
      const void* srcs[8];
      for (int j = 0; j < 8; j++) srcs[j] = (j < 4 ? a : b) + (j % 4) * (n / 8);
      if (tips_multi_sum(c, srcs, 8, n / 8, TIPS_FLOAT32, s) != 0) {
        fprintf(stderr, "multi_sum: %s\n", tips_last_error());
        exit(1);
      }
    } else if (v.mode == -5) {
      const int ns = v.unroll;
      const void* srcs[8];
      for (int j = 0; j < ns; j++)
        srcs[j] = (const char*)((j < ns / 2 ? a : b) + (j % (ns / 2)) * (n / ns)) + (j % (ns / 2)) * (int64_t)v.blocks;
      if (tips_multi_sum_variant(c, srcs, ns, n / ns, TIPS_FLOAT32, v.nt, s) != 0) {
        fprintf(stderr, "multi variant %s: %s\n", v.name.c_str(), tips_last_error());
        exit(1);
      }
    } else if (v.mode == -3) {
      if (tips_bucket_sum(c, a, b, n, TIPS_FLOAT32, s) != 0) {
        fprintf(stderr, "bucket_sum: %s\n", tips_last_error());
        exit(1);
      }
    } else if (tips_sum_variant(c, a, b, n, TIPS_FLOAT32, v.mode, v.unroll, v.nt, v.blocks, v.threads, s) != 0) {
      fprintf(stderr, "variant %s: %s\n", v.name.c_str(), tips_last_error());
      exit(1);
    }
  };
  // correctness spot check of every sum variant
  {
    std::vector<float> ha(n), hb(n), hc(n);
    CHECK(hipMemcpy(ha.data(), a, bytes, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(hb.data(), b, bytes, hipMemcpyDeviceToHost));
    for (auto& v : vs) {
      if (v.mode == -1 || v.mode == -4) continue;
      CHECK(hipMemset(c, 0, bytes));
      run(v);
      CHECK(hipStreamSynchronize(s));
      CHECK(hipMemcpy(hc.data(), c, bytes, hipMemcpyDeviceToHost));
      if (v.mode == -5) {  // rank-order fold of the ns slices
        const int ns = v.unroll;
        const int64_t m = n / ns;
        for (int64_t i = 0; i < m; i++) {
          float acc = ha[i];
          for (int j = 1; j < ns; j++) acc += (j < ns / 2 ? ha : hb)[(j % (ns / 2)) * (m + v.blocks / 4) + i];
          if (hc[i] != acc) {
            fprintf(stderr, "variant %s wrong at %lld\n", v.name.c_str(), (long long)i);
            return 1;
          }
        }
        continue;
      }
      for (int64_t i = 0; i < n; i++)
        if (hc[i] != ha[i] + hb[i]) {
          fprintf(stderr, "variant %s wrong at %lld\n", v.name.c_str(), (long long)i);
          return 1;
        }
    }
  }
  for (int r = 0; r < rounds; r++) {
    for (auto& v : vs) {
      rotate();
      run(v);  // warm
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < iters; i++) {
        rotate();
        run(v);
      }
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / iters);
    }
  }
  // the shipped kernel for every dtype on the same 256 MiB buffers (bytes moved are dtype-independent)
  const char* dnames[] = {"f32", "f64", "i32", "i64", "f16", "bf16"};
  for (int dt = 0; dt < 6; dt++) {
    const int64_t cnt = (int64_t)bytes / (dt == 1 || dt == 3 ? 8 : dt >= 4 ? 2 : 4);
    std::vector<double> ms;
    for (int r = 0; r < rounds; r++) {
      rotate();
      (void)tips_bucket_sum(c, a, b, cnt, dt, s);
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < iters; i++) {
        rotate();
        (void)tips_bucket_sum(c, a, b, cnt, dt, s);
      }
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float t = 0;
      CHECK(hipEventElapsedTime(&t, e0, e1));
      ms.push_back(t / iters);
    }
    std::sort(ms.begin(), ms.end());
    printf("{\"variant\": \"default_%s\", \"median_us\": %.2f, \"min_us\": %.2f, \"GBps_median\": %.1f, \"GBps_best\": %.1f}\n",
           dnames[dt], ms[ms.size() / 2] * 1e3, ms[0] * 1e3, 3.0 * bytes / (ms[ms.size() / 2] * 1e-3) / 1e9,
           3.0 * bytes / (ms[0] * 1e-3) / 1e9);
  }
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    const double moved = (v.mode == -1)   ? 2.0 * bytes
                         : (v.mode == -4) ? 9.0 * bytes / 8
                         : (v.mode == -5) ? (double)bytes * (v.unroll + 1) / v.unroll
                                          : 3.0 * bytes;
    printf("{\"variant\": \"%s\", \"median_us\": %.2f, \"min_us\": %.2f, \"GBps_median\": %.1f, \"GBps_best\": %.1f}\n",
           v.name.c_str(), med * 1e3, mn * 1e3, moved / (med * 1e-3) / 1e9, moved / (mn * 1e-3) / 1e9);
  }
  return 0;
}
