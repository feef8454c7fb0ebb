// Ablation harness for the single-query scan (not part of the product):
// GEMV variants (vs_kernels.hip gemv_topk_kernel VAR) timed interleaved on a
// resident N x 768 bf16 corpus (argv[1], default 10M rows), at k = 10 and
// k = 100 (one- and two-register wave lists).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ablate_gemv.hip -o tools/ablate_gemv
#include "../gorilla-rag---agentic-rag-with-mcp-using-golang-microservices_amd/csrc/vs_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace vsk;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e = (x);                                                                    \
    if (e != hipSuccess) {                                                                 \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                              \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

template <int KPL, int VAR>
static float run(const void* X, uint32_t n, const float* q, uint32_t k, uint64_t* out,
                 hipEvent_t a, hipEvent_t b) {
  using S = GemvShape<768, true>;
  GemvGrid g = gemv_grid(n, S::RB);
  hipEventRecord(a, 0);
  hipLaunchKernelGGL((gemv_topk_kernel<768, true, KPL, false, VAR>), dim3(g.nwg),
                     dim3(kGemvThreads), 0, 0, X, n, 0u, q, (const uint64_t*)nullptr, k,
                     g.rows_per_wave, out, (const uint32_t*)nullptr);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : 10000000u;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  void* X;
  float* q;
  uint64_t* out;
  CK(hipMalloc(&X, ((size_t)n + 32) * 768 * 2));
  CK(hipMalloc(&q, 768 * 4));
  CK(hipMalloc(&out, (size_t)1 << 26));
  device_cu_count();
  CK(launch_generate(0x5EED, 0, n, 768, true, X, 0, 0));
  CK(launch_generate(0xC0FFEE, 0, 1, 768, false, q, 0, 0));
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  struct Arm {
    const char* name;
    uint32_t k;
    float (*fn)(const void*, uint32_t, const float*, uint32_t, uint64_t*, hipEvent_t, hipEvent_t);
    std::vector<float> t;
  };
  std::vector<Arm> arms = {
      {"k10 slices", 10, run<1, 1>, {}},    {"k10 interleaved", 10, run<1, 9>, {}},
      {"k100 slices", 100, run<2, 1>, {}},  {"k100 interleaved", 100, run<2, 9>, {}},
  };
  for (int r = 0; r < reps; ++r)
    for (size_t j = 0; j < arms.size(); ++j) {
      auto& arm = arms[(j + (size_t)r) % arms.size()];
      arm.t.push_back(arm.fn(X, n, q, arm.k, out, a, b));
    }
  const double bytes = (double)n * 768 * 2;
  for (auto& arm : arms) {
    std::sort(arm.t.begin(), arm.t.end());
    const float med = arm.t[arm.t.size() / 2];
    printf("%-18s median %.4f ms  min %.4f  HBM %.0f GB/s (%.1f%% of 8 TB/s)\n", arm.name, med,
           arm.t[0], bytes / med / 1e6, bytes / med / 1e6 / 80.0);
  }
  return 0;
}
