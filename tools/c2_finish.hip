// c2_finish.hip — where C2's single-query step goes outside the int8 scan
// (r06). Replays vs_engine.cpp's one-query int8 path
// (launch_gemv_q8: scan + finish) on a resident 1M x 768 fp32 corpus with its
// int8 copy, cosine, k = 10, and prints: the step, the scan alone, the finish
// alone (re-run on one scan's output), and the finish's per-workgroup stage
// clocks (medians / max over the finishing workgroups, us from the earliest
// start): prep, P (radix floor), survivor lists, rescore, hand-off, and the
// last workgroup's merge; plus survivors rescored per query.
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/c2_finish.hip -o tools/c2_finish \
//     -I<pkg>/csrc -L<pkg>/lib -lvsearch -Wl,-rpath,<pkg>/lib
//   c2_finish [ROWS=1000000] [K=10] [REPS=200]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "vs_common.h"
#include "vs_kernels.h"

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 1000000;
  const uint32_t k = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 10;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 200;
  const uint32_t dim = 768;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  float *X, *meta, *glob, *q;
  int8_t* X8;
  CK(hipMalloc(&X, (size_t)(n + 32) * dim * 4));
  CK(hipMemset(X, 0, (size_t)(n + 32) * dim * 4));
  CK(hipMalloc(&X8, (size_t)(n + 32) * dim));
  CK(hipMemset(X8, 0, (size_t)(n + 32) * dim));
  CK(hipMalloc(&meta, (size_t)((n + 32) / 32 + 1) * 8));
  CK(hipMalloc(&glob, vsk::kQ8GlobBytes));
  CK(hipMemset(glob, 0, vsk::kQ8GlobBytes));
  CK(hipMalloc(&q, 64 * dim * 4));
  CK(vsk::launch_generate(0x5EED, 0, n, dim, false, X, 0, st));
  CK(vsk::launch_generate(0xC0FFEE, 0, 64, dim, false, q, 0, st, 1));
  CK(vsk::launch_q8_absmax(X, true, (uint64_t)n * dim, glob, st));
  CK(vsk::launch_q8_set_scale(glob, st));
  CK(vsk::launch_q8_quantize(X, true, n, dim, nullptr, 0, (n + 31) / 32, X8, meta, glob, st));
  const size_t sb = vsk::gemv_q8_scratch_bytes(n, k);
  void* scratch;
  CK(hipMalloc(&scratch, sb));
  uint32_t *ctr, *stats;
  CK(hipMalloc(&ctr, 16));
  CK(hipMemset(ctr, 0, 16));
  CK(hipMalloc(&stats, 16));
  CK(hipMemset(stats, 0, 16));
  uint64_t *dst, *clk;
  CK(hipMalloc(&dst, k * 8));
  const uint32_t nfin = (vsk::gemv_q8_lists(n) + 3) / 4;
  CK(hipMalloc(&clk, (size_t)nfin * 8 * 8));
  int qi = 0;
  auto run = [&](int part, uint32_t* s, uint64_t* c) {
    CK(vsk::launch_gemv_q8(part, X, false, X8, meta, glob, dim, n, 0, q + (size_t)(qi % 64) * dim,
                           true, nullptr, k, scratch, sb, ctr, dst, st, nullptr, 0, s, c));
  };
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto time_arm = [&](const std::function<void()>& f) {
    for (int w = 0; w < 10; ++w) f();
    std::vector<float> tv;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(a, st));
      for (int j = 0; j < reps; ++j) f();
      CK(hipEventRecord(b, st));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      tv.push_back(ms * 1e3f / reps);
    }
    std::sort(tv.begin(), tv.end());
    return tv[2];
  };
  const float t_step = time_arm([&] { run(3, nullptr, nullptr), ++qi; });
  const float t_scan = time_arm([&] { run(1, nullptr, nullptr), ++qi; });
  run(1, nullptr, nullptr);
  const float t_fin = time_arm([&] { run(2, nullptr, nullptr); });
  // one instrumented step per query of the 64, stage clocks pooled
  std::vector<std::vector<double>> stg(7);
  std::vector<double> surv;
  for (int i = 0; i < 64; ++i) {
    qi = i;
    CK(hipMemset(stats, 0, 16));
    CK(hipMemset(clk, 0, (size_t)nfin * 64));
    run(1, nullptr, nullptr);
    run(2, stats, nullptr);  // survivors (its atomics would distort the clocks)
    run(2, nullptr, clk);    // the same finish again, clocks only
    CK(hipStreamSynchronize(st));
    std::vector<uint64_t> h((size_t)nfin * 8);
    CK(hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost));
    uint32_t hs[4];
    CK(hipMemcpy(hs, stats, 16, hipMemcpyDeviceToHost));
    surv.push_back(hs[0]);
    uint64_t t0 = ~0ull;
    for (uint32_t w = 0; w < nfin; ++w)
      if (h[(size_t)w * 8]) t0 = std::min(t0, h[(size_t)w * 8]);
    for (uint32_t w = 0; w < nfin; ++w)
      for (int s = 1; s < 7; ++s)
        if (h[(size_t)w * 8 + s]) stg[s].push_back((h[(size_t)w * 8 + s] - t0) * 0.01);
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
  };
  auto mx = [](const std::vector<double>& v) {
    return v.empty() ? 0.0 : *std::max_element(v.begin(), v.end());
  };
  std::printf("{\"tool\": \"c2_finish\", \"rows\": %u, \"k\": %u, \"finish_wgs\": %u, \"step_us\": %.2f, "
              "\"scan_us\": %.2f, \"finish_us\": %.2f",
              n, k, nfin, t_step, t_scan, t_fin);
  const char* names[7] = {"start", "prep", "P", "lists", "rescore", "handoff", "merge"};
  for (int s = 1; s < 7; ++s)
    std::printf(", \"%s_us_med\": %.2f, \"%s_us_max\": %.2f", names[s], med(stg[s]), names[s], mx(stg[s]));
  std::printf(", \"rescored_per_query_med\": %.1f}\n", med(surv));
  return 0;
}
