// Ablation harness for the batched MFMA scan (not part of the product).
// Builds the kernel in several modes and times them interleaved in one process
// on the same resident corpus (cdna_hip_programming.md §5.4 rule 24):
//   full+bound  : product main pass, thresholds from the sample pass
//   full        : main pass without the sample bound
//   no-epilogue : MFMA + LDS stream, top-k epilogue removed
//   dma-only    : LDS-DMA stream + barriers only
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ablate_mfma.hip -o tools/ablate_mfma
#include "../gorilla-rag---agentic-rag-with-mcp-using-golang-microservices_amd/csrc/vs_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace vsk;

#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);           \
      return 1;                                                         \
    }                                                                   \
  } while (0)

template <int MODE>
static float run(const uint16_t* X, uint32_t n, const uint16_t* Q, const uint64_t* init,
                 uint64_t* out, uint32_t nwg, uint32_t rpw, uint32_t k, hipEvent_t a,
                 hipEvent_t b) {
  hipEventRecord(a, 0);
  hipLaunchKernelGGL((mfma_topk_kernel<768, MODE>), dim3(nwg), dim3(kMfThreads), 0, 0, X, n, 0u,
                     rpw, 0u, Q, 256u, k, init, k, out);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : 10000000u;
  const int reps = argc > 2 ? atoi(argv[2]) : 8;
  const uint32_t k = 10;
  uint16_t *X, *Q;
  uint64_t *out, *skeys;
  CK(hipMalloc(&X, ((size_t)n + 32) * 768 * 2));
  CK(hipMemset(X, 0, ((size_t)n + 32) * 768 * 2));
  CK(hipMalloc(&Q, 256 * 768 * 2));
  CK(launch_generate(0x5EED, 0, n, 768, true, X, 0, 0));
  CK(launch_generate(0xC0FFEE, 0, 256, 768, true, Q, 0, 0));
  uint32_t nwg, rpw;
  device_cu_count();
  mfma_grid(n, &nwg, &rpw);
  CK(hipMalloc(&out, (size_t)nwg * 256 * k * 8));
  CK(hipMalloc(&skeys, (size_t)256 * k * 8));
  // sample pass -> per-query lower bounds (as the engine does)
  uint32_t L = 0;
  const uint32_t tpw = mfma_tiles_per_wg(n);
  CK(launch_mfma(X, 768, n, 0, Q, 256, k, tpw / 64 ? tpw / 64 : 1, nullptr, 0, out, nwg, &L, 0));
  CK(launch_merge(out, L, (uint64_t)256 * k, k, 256, k, k, skeys, 0));
  CK(hipDeviceSynchronize());
  const uint64_t* init = skeys + (k - 1);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::vector<float> t[6];
  for (int r = 0; r < reps; ++r) {
    t[0].push_back(run<0>(X, n, Q, init, out, nwg, rpw, k, a, b));
    t[1].push_back(run<0>(X, n, Q, nullptr, out, nwg, rpw, k, a, b));
    t[2].push_back(run<1>(X, n, Q, nullptr, out, nwg, rpw, k, a, b));
    t[3].push_back(run<2>(X, n, Q, nullptr, out, nwg, rpw, k, a, b));
    t[4].push_back(run<4>(X, n, Q, nullptr, out, nwg, rpw, k, a, b));
    t[5].push_back(run<5>(X, n, Q, nullptr, out, nwg, rpw, k, a, b));
  }
  CK(hipDeviceSynchronize());
  const char* names[6] = {"full+bound", "full", "no-epilogue", "dma-only", "mfma+bar", "mfma-only"};
  const double bytes = (double)n * 768 * 2, flops = 2.0 * 256 * n * 768;
  for (int m = 0; m < 6; ++m) {
    std::sort(t[m].begin(), t[m].end());
    float med = t[m][t[m].size() / 2];
    printf("%-12s median %.3f ms  min %.3f ms  HBM %.0f GB/s  MFMA %.0f TF/s\n", names[m], med,
           t[m][0], bytes / med / 1e6, flops / med / 1e9);
  }
  printf("grid %u WGs x %u rows, sample tiles/wg %u\n", nwg, rpw, tpw / 64);
  return 0;
}
