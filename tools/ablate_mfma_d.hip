// Ablation harness for the batched MFMA scan at D = 1024 (C5's collections;
// not part of the product): one launch = 128 queries (G = 1), k = 50. Arms
// are timed interleaved in one process on one resident corpus, rotating
// their order each rep, VS_ABL_BURST launches back to back per timing.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ablate_mfma_d.hip -o tools/ablate_mfma_d
#include "../gorilla-rag---agentic-rag-with-mcp-using-golang-microservices_amd/csrc/vs_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace vsk;

#define CK(x)                                                 \
  do {                                                        \
    hipError_t e = (x);                                       \
    if (e != hipSuccess) {                                    \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                               \
    }                                                         \
  } while (0)

constexpr int D = 1024;
constexpr int G = mf_groups(D);
constexpr uint32_t NQ = 16 * 8 * G;  // queries per launch

struct Ctx {
  MfArgs args;
  uint32_t nwg;
  hipEvent_t a, b;
};

template <int MODE, int VAR>
static float run(const Ctx& c, bool bound) {
  MfArgs a = c.args;
  if (!bound) a.init_score = nullptr;
  static const int burst = getenv("VS_ABL_BURST") ? atoi(getenv("VS_ABL_BURST")) : 4;
  (void)hipEventRecord(c.a, 0);
  for (int i = 0; i < burst; ++i)
    hipLaunchKernelGGL((mfma_topk_kernel<D, MODE, VAR, G>), dim3(c.nwg), dim3(64 * mf_waves(G)), 0,
                       0, a);
  (void)hipEventRecord(c.b, 0);
  (void)hipEventSynchronize(c.b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, c.a, c.b);
  return ms / burst;
}

struct Arm {
  const char* name;
  float (*fn)(const Ctx&, bool);
  bool bound;
  std::vector<float> t;
};

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : 5000000u;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const uint32_t k = argc > 3 ? (uint32_t)atoi(argv[3]) : 50;
  uint16_t *X, *Q;
  CK(hipMalloc(&X, ((size_t)n + 32) * D * 2));
  CK(hipMemset(X, 0, ((size_t)n + 32) * D * 2));
  CK(hipMalloc(&Q, (size_t)kMfmaQueries * D * 2));
  CK(hipMemset(Q, 0, (size_t)kMfmaQueries * D * 2));
  CK(launch_generate(0x5EED, 0, n, D, true, X, 0, 0));
  CK(launch_generate(0xC0FFEE, 0, NQ, D, true, Q, 0, 0));
  device_cu_count();
  Ctx c{};
  uint32_t rpw;
  mfma_grid(n, &c.nwg, &rpw);
  const uint32_t st = mfma_sample_tiles(n, D, false);
  const uint32_t cap = std::max(mfma_cand_cap(n, k, st), mfma_cand_cap(n, k, 2));
  uint64_t* cand;
  uint32_t *ctile, *cnt;
  float *tmax, *bnd;
  CK(hipMalloc(&cand, (size_t)c.nwg * kMfmaQueries * cap * 32));
  CK(hipMalloc(&ctile, (size_t)c.nwg * kMfmaQueries * cap * 4));
  CK(hipMalloc(&cnt, (size_t)c.nwg * kMfmaQueries * 16));
  CK(hipMalloc(&tmax, (size_t)c.nwg * kMfmaQueries * st * 4 * 4));
  CK(hipMalloc(&bnd, kMfmaQueries * 4));
  uint32_t L = 0;
  CK(launch_mfma_sample(X, false, D, n, 0, Q, NQ, k, st, tmax, c.nwg, &L, 0));
  CK(launch_sample_bound(tmax, L * st, NQ, k, bnd, 0));
  CK(hipDeviceSynchronize());
  MfArgs& g = c.args;
  g.X = X, g.Q = Q, g.init_score = bnd;
  g.cand = cand, g.cand_tile = ctile, g.cand_cnt = cnt, g.cand_cap = cap;
  g.n_rows = n, g.rows_per_wg = rpw, g.nq_valid = NQ, g.k = k;
  CK(hipEventCreate(&c.a));
  CK(hipEventCreate(&c.b));
  std::vector<Arm> arms = {
      {"main (product)", run<0, 0>, true, {}},
      {"no-epilogue", run<1, 0>, false, {}},
      {"dma-only", run<2, 0>, false, {}},
      {"main ring144", run<0, 256>, true, {}},
      {"main cached-dma", run<0, 1024>, true, {}},
      {"main pd3", run<0, 64>, true, {}},
      {"max-only (6)", run<6, 0>, true, {}},
  };
  if (getenv("VS_ABL_ST")) {
    // sample tiles per workgroup vs main-pass epilogue: time sample+bound and
    // the product main pass for each count (candidate capacity re-sized)
    for (uint32_t sti : {2u, 4u, 6u, 8u, 12u, 16u}) {
      const uint32_t capi = mfma_cand_cap(n, k, sti);
      if (capi > cap || sti > st * 4) continue;
      MfArgs m = g;
      m.cand_cap = capi;
      std::vector<float> ts, tm;
      for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(c.a, 0));
        CK(launch_mfma_sample(X, false, D, n, 0, Q, NQ, k, sti, tmax, c.nwg, &L, 0));
        CK(launch_sample_bound(tmax, L * sti, NQ, k, bnd, 0));
        CK(hipEventRecord(c.b, 0));
        CK(hipEventSynchronize(c.b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, c.a, c.b));
        ts.push_back(ms);
        Ctx cc = c;
        cc.args = m;
        tm.push_back(run<0, 0>(cc, true));
      }
      std::sort(ts.begin(), ts.end());
      std::sort(tm.begin(), tm.end());
      printf("sample tiles %2u cap %3u: sample+bound %.1f us  main %.3f ms  sum %.3f ms\n", sti,
             capi, 1e3 * ts[ts.size() / 2], tm[tm.size() / 2],
             ts[ts.size() / 2] + tm[tm.size() / 2]);
    }
    return 0;
  }
  for (int r = 0; r < reps; ++r)
    for (size_t j = 0; j < arms.size(); ++j) {
      auto& arm = arms[(j + (size_t)r) % arms.size()];
      arm.t.push_back(arm.fn(c, arm.bound));
    }
  CK(hipDeviceSynchronize());
  const double bytes = (double)n * D * 2, flops = 2.0 * NQ * n * D;
  printf("D=%d rows=%u k=%u queries/launch=%u grid=%u x %u rows, cap %u\n", D, n, k, NQ, c.nwg,
         rpw, cap);
  for (auto& arm : arms) {
    std::sort(arm.t.begin(), arm.t.end());
    const float med = arm.t[arm.t.size() / 2];
    printf("%-20s median %.3f ms  min %.3f ms  HBM %.0f GB/s  MFMA %.0f TF/s\n", arm.name, med,
           arm.t[0], bytes / med / 1e6, flops / med / 1e9);
  }
  return 0;
}
