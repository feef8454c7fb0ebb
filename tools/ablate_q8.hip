// ablate_q8.hip — where the int8 prefilter pass's time goes (r05; VERDICT r04
// item 2). Builds the pass in several modes and times them interleaved in
// one process on one resident corpus, each timing a burst of back-to-back
// launches (sustained clocks, the serving regime):
//   prod     mfma_topk_kernel<768, 0, 2304, 2, false, true> (the product)
//   noapp    the same, never appending (timing only: wrong answers)
//   noepi    MODE 1: no epilogue at all (MFMA + LDS reads + stream + barriers)
//   stream   the bf16 kernel at D = 384 (768-B rows: the int8 pass's byte
//            stream and chunk geometry) in MODE 2: the LDS-DMA stream alone
//   mfma     the same in MODE 4: MFMAs (16x16x32 bf16, 16 cycles each: the
//            int8 pass's count and cycles) + LDS reads + barriers, no stream
//   mfma-nb  MODE 5: MODE 4 without barriers
//   pair     VAR 33554432: one barrier per pair of tiles (vs_kernels.hip)
//   epipipe  VAR 67108864: each tile's epilogue deferred into the next tile
//   spread   VAR 16384: a chunk's DMA pieces spread over its steps
//   prea     VAR 32768: a tile's first A-fragment reads before the previous
//            tile's epilogue
//   split    VAR 67108864 + 65536: the deferred epilogue split over the next
//            tile's steps 1 .. G + 1
// (r05 records of the dropped arms -- pd2/pd3: A fragments 2 / 3 steps
// ahead, stag: waves 4-7 half a chunk ahead, pair+epi -- all slower than
// prod: profiles/r05_ablate_q8*.json)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ablate_q8.hip -o tools/ablate_q8
//   ablate_q8 [ROWS=10000000] [REPS=5] [BURST=20] [ARM: that arm alone]
#include "../gorilla-rag---agentic-rag-with-mcp-using-golang-microservices_amd/csrc/vs_kernels.hip"
#include "../gorilla-rag---agentic-rag-with-mcp-using-golang-microservices_amd/csrc/vs_q8.hip"

#include <algorithm>
#include <cstdio>
#include <string>
#include <cstdlib>
#include <vector>

using namespace vsk;

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e = (x);                                              \
    if (e != hipSuccess) {                                           \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);        \
      return 1;                                                      \
    }                                                                \
  } while (0)

struct Ctx {
  MfArgs q8, bf;  // int8 pass arguments; the D = 384 bf16 skeleton's
  uint32_t nwg;
  int burst;
  hipEvent_t a, b;
};

template <int D, int MODE, int VAR, bool I8>
static float run(const Ctx& c) {
  const MfArgs& a = I8 ? c.q8 : c.bf;
  hipEventRecord(c.a, 0);
  for (int i = 0; i < c.burst; ++i)
    hipLaunchKernelGGL((mfma_topk_kernel<D, MODE, VAR, 2, false, I8>), dim3(c.nwg), dim3(512), 0, 0,
                       a);
  hipEventRecord(c.b, 0);
  hipEventSynchronize(c.b);
  float ms = 0;
  hipEventElapsedTime(&ms, c.a, c.b);
  return ms / c.burst;
}

struct Arm {
  const char* name;
  float (*fn)(const Ctx&);
  std::vector<float> t;
};

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : 10000000u;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int burst = argc > 3 ? atoi(argv[3]) : 20;
  const uint32_t k = 10, dim = 768;
  uint16_t *X, *Q;
  int8_t *X8, *Q8;
  float *meta, *glob, *par, *tmax, *bnd, *slabs;
  uint32_t *tiles, *cnt, *cmx;
  CK(hipMalloc(&X, ((size_t)n + 32) * dim * 2));
  CK(hipMemset(X, 0, ((size_t)n + 32) * dim * 2));
  CK(hipMalloc(&X8, ((size_t)n + 32) * dim));
  CK(hipMemset(X8, 0, ((size_t)n + 32) * dim));
  CK(hipMalloc(&Q, 256 * dim * 2));
  CK(hipMalloc(&Q8, 256 * dim));
  CK(hipMalloc(&meta, ((size_t)n / 32 + 2) * 8));
  CK(hipMalloc(&glob, 16));
  CK(hipMalloc(&par, 256 * 16 + 64));
  uint32_t* gate = (uint32_t*)(par + 4 * 256);
  CK(launch_generate(0x5EED, 0, n, dim, true, X, 0, 0));
  CK(launch_generate(0xC0FFEE, 0, 256, dim, true, Q, 0, 0));
  CK(hipMemset(glob, 0, 16));
  CK(launch_q8_absmax(X, false, (uint64_t)n * dim, glob, 0));
  CK(launch_q8_set_scale(glob, 0));
  CK(launch_q8_quantize(X, false, n, dim, nullptr, 0, (n + 31) / 32, X8, meta, glob, 0));
  Ctx c{};
  c.burst = burst;
  device_cu_count();
  uint32_t rpw;
  mfma_grid(n, &c.nwg, &rpw);
  const uint32_t st = mfma_sample_tiles(n), cap = mfma_cand_cap(n, k, st, 8.0);
  CK(hipMalloc(&slabs, (size_t)c.nwg * 256 * cap * 32));
  CK(hipMalloc(&tiles, (size_t)c.nwg * 256 * cap * 4));
  CK(hipMalloc(&cnt, (size_t)c.nwg * 256 * 16));
  CK(hipMalloc(&cmx, (size_t)c.nwg * 256 * 16));
  CK(hipMalloc(&tmax, (size_t)c.nwg * 256 * st * 4));
  CK(hipMalloc(&bnd, 256 * 4));
  uint32_t L = 0;
  CK(launch_mfma_sample(X, false, dim, n, 0, Q, 256, k, st, tmax, c.nwg, &L, 0));
  CK(launch_sample_bound_q8(tmax, L * st, 256, k, bnd, Q, false, 256, dim, glob, Q8, par, gate, 0));
  CK(hipDeviceSynchronize());
  MfArgs& a = c.q8;
  a.X = X8, a.Q = Q8, a.init_score = bnd, a.cand = (uint64_t*)slabs, a.cand_tile = tiles;
  a.cand_cnt = cnt, a.cand_max = cmx, a.n_rows = n, a.row_base = 0, a.rows_per_wg = rpw;
  a.nq_valid = 256, a.k = k, a.cand_cap = cap, a.q8par = par, a.q8glob = glob, a.gate = gate;
  // the bf16 skeleton over the same bytes: 768-B rows read as D = 384 bf16
  MfArgs& f = c.bf;
  f = a;
  f.X = X8, f.Q = Q, f.q8par = nullptr, f.q8glob = nullptr, f.init_score = nullptr;
  hipEventCreate(&c.a);
  hipEventCreate(&c.b);
  std::vector<Arm> arms = {
      {"prod", run<768, 0, 2304, true>, {}},
      {"noapp", run<768, 0, 2304 + 16777216, true>, {}},
      {"noepi", run<768, 1, 2304, true>, {}},
      {"stream", run<384, 2, 2304, false>, {}},
      {"mfma", run<384, 4, 2304, false>, {}},
      {"mfma-nb", run<384, 5, 2304, false>, {}},
      {"pair", run<768, 0, 2304 + 33554432, true>, {}},
      {"epipipe", run<768, 0, 2304 + 67108864, true>, {}},
      {"spread", run<768, 0, 2304 + 16384, true>, {}},
      {"prea", run<768, 0, 2304 + 32768, true>, {}},
      {"split", run<768, 0, 2304 + 67108864 + 65536, true>, {}},
  };
  // an arm's name as the 4th argument: that arm alone (PMC passes), R x B launches
  if (argc > 4) {
    for (auto& arm : arms) {
      if (std::string(argv[4]) != arm.name) continue;
      for (int r = 0; r < reps; ++r) arm.t.push_back(arm.fn(c));
      std::sort(arm.t.begin(), arm.t.end());
      printf("{\"rows\": %u, \"%s_ms\": %.4f}\n", n, arm.name, arm.t[arm.t.size() / 2]);
      return 0;
    }
    printf("no arm %s\n", argv[4]);
    return 1;
  }
  for (auto& arm : arms) arm.fn(c);  // warm every arm once
  for (int r = 0; r < reps; ++r)
    for (size_t i = 0; i < arms.size(); ++i) {
      const size_t j = (i + (size_t)r) % arms.size();  // rotate the order per rep
      arms[j].t.push_back(arms[j].fn(c));
    }
  const double bytes = (double)n * dim + 256.0 * dim + 256.0 * k * 12;
  printf("{\"rows\": %u, \"reps\": %d, \"burst\": %d, \"nwg\": %u", n, reps, burst, c.nwg);
  for (auto& arm : arms) {
    std::sort(arm.t.begin(), arm.t.end());
    const double ms = arm.t[arm.t.size() / 2];
    printf(", \"%s_ms\": %.4f, \"%s_hbm_frac\": %.4f", arm.name, ms, arm.name, bytes / (ms * 1e-3) / 8e12);
  }
  // the sample pass (MODE 3, bf16 rows) at 1, 2, 4, 8 tiles per workgroup
  // (the N = 8 share uses 4), timed in bursts, and one launch with the
  // per-workgroup clocks (VAR 8192: start, prologue done, tiles done, end)
  {
    MfArgs sa{};
    sa.X = X, sa.Q = Q, sa.tmax = tmax, sa.n_rows = n, sa.rows_per_wg = rpw;
    sa.nq_valid = 256, sa.k = k;
    const uint32_t sts[4] = {1, 2, 4, 8};
    for (uint32_t st2 : sts) {
      if (st2 > st && st2 > 4) break;  // tmax holds nwg * st tiles per query
      sa.max_tiles = st2;
      std::vector<float> ts;
      for (int r = 0; r < reps; ++r) {
        hipEventRecord(c.a, 0);
        for (int i = 0; i < burst; ++i)
          hipLaunchKernelGGL((mfma_topk_kernel<768, 3, 2304, 2, false, false>), dim3(c.nwg), dim3(512), 0, 0,
                             sa);
        hipEventRecord(c.b, 0);
        hipEventSynchronize(c.b);
        float ms = 0;
        hipEventElapsedTime(&ms, c.a, c.b);
        ts.push_back(ms / burst);
      }
      std::sort(ts.begin(), ts.end());
      printf(", \"sample_st%u_us\": %.2f", st2, ts[ts.size() / 2] * 1e3);
      // VAR 8388608: the ring's first chunks issued before the query-fragment
      // prologue (its latency then overlaps the ~5.5 us of fragment loads)
      ts.clear();
      for (int r = 0; r < reps; ++r) {
        hipEventRecord(c.a, 0);
        for (int i = 0; i < burst; ++i)
          hipLaunchKernelGGL((mfma_topk_kernel<768, 3, 2304 + 8388608, 2, false, false>), dim3(c.nwg), dim3(512),
                             0, 0, sa);
        hipEventRecord(c.b, 0);
        hipEventSynchronize(c.b);
        float ms = 0;
        hipEventElapsedTime(&ms, c.a, c.b);
        ts.push_back(ms / burst);
      }
      std::sort(ts.begin(), ts.end());
      printf(", \"sample_early_st%u_us\": %.2f", st2, ts[ts.size() / 2] * 1e3);
    }
    uint64_t* clkb;
    CK(hipMalloc(&clkb, (size_t)c.nwg * 4 * 8));
    sa.max_tiles = 4 < st ? 4 : st;
    sa.lists = clkb;
    for (int i = 0; i < 3; ++i)
      hipLaunchKernelGGL((mfma_topk_kernel<768, 3, 2304 + 8192, 2, false, false>), dim3(c.nwg), dim3(512), 0, 0,
                         sa);
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> h((size_t)c.nwg * 4);
    CK(hipMemcpy(h.data(), clkb, h.size() * 8, hipMemcpyDeviceToHost));
    uint64_t t0 = ~0ull;
    for (uint32_t b = 0; b < c.nwg; ++b) t0 = std::min(t0, h[4 * b]);
    const char* nm[4] = {"start", "prologue", "tiles", "end"};
    for (int j = 0; j < 4; ++j) {
      std::vector<double> v;
      for (uint32_t b = 0; b < c.nwg; ++b) v.push_back((h[4 * b + j] - t0) * 0.01);
      std::sort(v.begin(), v.end());
      printf(", \"sample_clk_%s_us_med\": %.2f, \"sample_clk_%s_us_max\": %.2f", nm[j], v[v.size() / 2], nm[j],
             v.back());
    }
  }
  // the product variants must append the same slabs: counts and quarter
  // maxima equal to the product's, element for element
  auto snap = [&](float (*fn)(const Ctx&), std::vector<uint32_t>& h) -> int {
    Ctx one = c;
    one.burst = 1;
    CK(hipMemset(cnt, 0xFF, (size_t)c.nwg * 256 * 16));
    fn(one);
    CK(hipDeviceSynchronize());
    h.resize((size_t)c.nwg * 256 * 8);
    CK(hipMemcpy(h.data(), cnt, (size_t)c.nwg * 256 * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h.data() + (size_t)c.nwg * 256 * 4, cmx, (size_t)c.nwg * 256 * 16, hipMemcpyDeviceToHost));
    return 0;
  };
  std::vector<uint32_t> ref, got;
  if (snap(run<768, 0, 2304, true>, ref)) return 1;
  const char* vnames[4] = {"pair", "epipipe", "spread", "split"};
  float (*vfns[4])(const Ctx&) = {run<768, 0, 2304 + 33554432, true>, run<768, 0, 2304 + 67108864, true>,
                                  run<768, 0, 2304 + 16384, true>, run<768, 0, 2304 + 67108864 + 65536, true>};
  for (int v = 0; v < 4; ++v) {
    if (snap(vfns[v], got)) return 1;
    size_t diff = 0;
    for (size_t i = 0; i < ref.size(); ++i) diff += ref[i] != got[i];
    printf(", \"%s_count_max_mismatches\": %zu", vnames[v], diff);
  }
  printf("}\n");
  return 0;
}
