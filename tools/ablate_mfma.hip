// Ablation harness for the batched MFMA scan (not part of the product).
// Builds the kernel in several modes / scheduling variants and times them
// interleaved in one process on the same resident corpus
// (cdna_hip_programming.md §5.4 rule 24). MODE and VAR: vs_kernels.hip.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ablate_mfma.hip -o tools/ablate_mfma
#include "../gorilla-rag---agentic-rag-with-mcp-using-golang-microservices_amd/csrc/vs_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

struct Ctx {
  MfArgs args;
  uint32_t* wgt;
  uint32_t nwg;
  hipEvent_t a, b;
  float* tmax;  // sample-pass arms
  uint32_t st;
};

template <int MODE, int VAR, int G = 2>
static float run(const Ctx& c, bool bound) {
  MfArgs a = c.args;
  if (!bound) a.init_score = nullptr;
  if (VAR & 65536) a.wg_tile = c.wgt;  // ablation: the weighted split
  // VS_ABL_BURST=B: B launches back to back per timing (sustained clocks, as
  // in a serving loop; the time per launch is returned). Default 1
  // (isolated launches). Isolated launches favoured a dynamic tile pool by
  // 8%; back to back it was 3-5% slower than the static split (r01).
  static const int burst = getenv("VS_ABL_BURST") ? atoi(getenv("VS_ABL_BURST")) : 1;
  hipEventRecord(c.a, 0);
  for (int i = 0; i < burst; ++i)
    hipLaunchKernelGGL((mfma_topk_kernel<768, MODE, VAR, G>), dim3(c.nwg), dim3(64 * mf_waves(G)),
                       0, 0, a);
  hipEventRecord(c.b, 0);
  hipEventSynchronize(c.b);
  float ms = 0;
  hipEventElapsedTime(&ms, c.a, c.b);
  return ms / burst;
}

// run() without the main pass's quarter-maxima writes (cand_max = null)
template <int MODE, int VAR, int G = 2>
static float run_nq(const Ctx& c, bool bound) {
  Ctx c2 = c;
  c2.args.cand_max = nullptr;
  return run<MODE, VAR, G>(c2, bound);
}

// the sample pass (MODE 3) over the first st tiles of every workgroup, same
// burst rule as run(); its arguments are built from the main pass's
template <int VAR>
static float run_sample(const Ctx& c, bool) {
  MfArgs a{};
  a.X = c.args.X, a.Q = c.args.Q, a.tmax = c.tmax;
  a.max_tiles = c.st, a.n_rows = c.args.n_rows, a.rows_per_wg = c.args.rows_per_wg;
  a.nq_valid = 256, a.k = c.args.k;
  static const int burst = getenv("VS_ABL_BURST") ? atoi(getenv("VS_ABL_BURST")) : 1;
  hipEventRecord(c.a, 0);
  for (int i = 0; i < burst; ++i)
    hipLaunchKernelGGL((mfma_topk_kernel<768, 3, VAR, 2>), dim3(c.nwg), dim3(512), 0, 0, a);
  hipEventRecord(c.b, 0);
  hipEventSynchronize(c.b);
  float ms = 0;
  hipEventElapsedTime(&ms, c.a, c.b);
  return ms / burst;
}

struct Arm {
  const char* name;
  float (*fn)(const Ctx&, bool);
  bool bound;
  std::vector<float> t;
};

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atol(argv[1]) : 10000000u;
  const int reps = argc > 2 ? atoi(argv[2]) : 8;
  const uint32_t st_over = argc > 3 ? (uint32_t)atoi(argv[3]) : 0;  // sample tiles override
  const uint32_t k = getenv("VS_ABL_K") ? (uint32_t)atoi(getenv("VS_ABL_K")) : 10u;
  uint16_t *X, *Q;
  uint64_t *out, *cand;
  float *tmax, *bnd;
  uint32_t* cnt;
  CK(hipMalloc(&X, ((size_t)n + 32) * 768 * 2));
  CK(hipMemset(X, 0, ((size_t)n + 32) * 768 * 2));
  CK(hipMalloc(&Q, 256 * 768 * 2));
  CK(launch_generate(0x5EED, 0, n, 768, true, X, 0, 0));
  CK(launch_generate(0xC0FFEE, 0, 256, 768, true, Q, 0, 0));
  Ctx c{};
  device_cu_count();
  uint32_t rpw;
  mfma_grid(n, &c.nwg, &rpw);
  CK(hipMalloc(&out, (size_t)c.nwg * 256 * k * 8));
  const uint32_t st = st_over ? st_over : mfma_sample_tiles(n), cap = mfma_cand_cap(n, k, st);
  CK(hipMalloc(&cand, (size_t)c.nwg * 256 * cap * 32));  // main-pass slabs
  uint32_t* ctile;
  CK(hipMalloc(&ctile, (size_t)c.nwg * 256 * cap * 4));
  CK(hipMalloc(&tmax, (size_t)c.nwg * 256 * st * 4));
  CK(hipMalloc(&cnt, (size_t)c.nwg * 256 * 4 * 4));
  uint32_t* qmx;  // the main pass's quarter maxima (r04 select)
  CK(hipMalloc(&qmx, (size_t)c.nwg * 256 * 4 * 4));
  CK(hipMalloc(&bnd, 256 * 4));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  // sample pass -> per-query lower bounds (as the engine does); timed
  uint32_t L = 0;
  const uint32_t tpw = mfma_tiles_per_wg(n);
  std::vector<float> ts;
  for (int r = 0; r < reps; ++r) {
    hipEventRecord(a, 0);
    CK(launch_mfma_sample(X, false, 768, n, 0, Q, 256, k, st, tmax, c.nwg, &L, 0));
    CK(launch_sample_bound(tmax, L * st, 256, k, bnd, 0));
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ts.push_back(ms);
  }
  CK(hipDeviceSynchronize());
  MfArgs& g = c.args;
  g.X = X, g.Q = Q, g.init_score = bnd, g.lists = out;
  g.cand = cand, g.cand_tile = ctile, g.cand_cnt = cnt, g.cand_cap = cap;
  g.cand_max = getenv("VS_ABL_NOQMAX") ? nullptr : qmx;
  g.n_rows = n, g.rows_per_wg = rpw, g.nq_valid = 256, g.k = k;
  c.a = a;
  c.b = b;
  c.tmax = tmax;
  c.st = st;
  // An unrolled, predicated candidate append was no faster than the ctz loop;
  // 4-16 sample tiles at 1.25M rows cut the candidates 2-8x but the main pass
  // gained what the sample pass lost (argv[3] overrides the sample tiles).
  // 24 / 48 KiB K-chunks (VAR 2048 / 4096, + 256 for the 144 KiB ring) were
  // slower than 16 KiB at 10M rows (3.64-3.67 vs 3.48 ms); kept as arms.
  // G = 4 (4 waves x 64 queries, one wave per SIMD, 512 registers): no
  // epilogue 4.23 ms, 3.74 with a 2-step fragment prefetch, 3.60 with a pinned
  // 3-step one, vs 3.35 for G = 2 (10M rows, r01).
  // weighted split: VS_XCD_W = 8 comma-separated weights for blockIdx % 8
  uint32_t* wgt = nullptr;
  {
    std::vector<double> xw(8, 1.0);
    if (const char* e = getenv("VS_XCD_W")) {
      int x = 0;
      for (const char* p = e; *p && x < 8; ++x) {
        xw[x] = atof(p);
        while (*p && *p != ',') ++p;
        if (*p == ',') ++p;
      }
    }
    const uint32_t T = (n + 31) / 32;
    double tot = 0;
    for (uint32_t b = 0; b < c.nwg; ++b) tot += xw[b % 8];
    std::vector<uint32_t> h(c.nwg + 1);
    double acc = 0;
    for (uint32_t b = 0; b < c.nwg; ++b) {
      h[b] = (uint32_t)(acc / tot * T + 0.5);
      acc += xw[b % 8];
    }
    h[c.nwg] = T;
    CK(hipMalloc(&wgt, h.size() * 4));
    CK(hipMemcpy(wgt, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    printf("weighted split: %u..%u tiles per workgroup\n", h[1] - h[0], h[2] - h[1]);
  }
  c.wgt = wgt;
  std::vector<Arm> arms = {
      {"main (product)", run<0, 2048 + 256, 2>, true, {}},  // 24 KiB chunks, 144 KiB ring
      {"main bf 16k", run<0, 0, 2>, true, {}},              // r02 build before: 16 KiB chunks
      {"main branchy", run<0, 524288, 2>, true, {}},        // r01 conditional stream
      {"bf no-replace", run<0, 2097152, 2>, true, {}},      // full quarter drops (inexact)
      {"main bf stag", run<0, 1048576, 2>, true, {}},       // + waves 4-7 half a chunk ahead
      {"bf ring144", run<0, 256, 2>, true, {}},             // 8 chunks in flight
      {"bf 24k ring144", run<0, 2048 + 256, 2>, true, {}},  // 2 barriers / tile
      {"bf 48k ring144", run<0, 4096 + 256, 2>, true, {}},  // 1 barrier / tile
      {"main cached-dma", run<0, 1024, 2>, true, {}},       // regs, default policy
      {"main lds-cnt", run<0, 131072, 2>, true, {}},        // LDS counters + nt
      {"main v13", run<0, 131072 + 1024, 2>, true, {}},     // LDS counters, default policy
      {"main prio", run<0, 262144, 2>, true, {}},           // default + raised priority appends
  };
  // VS_ABL_SET=lds: what the A-fragment LDS reads cost (no epilogue in the
  // MODE 1 / 7 / 10 arms: all reads, hr 0 only = half the reads, one
  // fragment set reused = almost none)
  if (getenv("VS_ABL_SET") && !strcmp(getenv("VS_ABL_SET"), "g4")) {
    // one wave per SIMD, 64 queries each (half the A-fragment LDS reads), on
    // the product's 24 KiB chunks / 144 KiB ring, against the product layout
    arms = {{"no-epi (product)", run<1, 2048 + 256, 2>, false, {}},
            {"no-epi G4 pd1", run<1, 2048 + 256, 4>, false, {}},
            {"no-epi G4 pd3 pin", run<1, 2048 + 256 + 64 + 128, 4>, false, {}},
            {"no-epi G4 pd2 pin", run<1, 2048 + 256 + 32 + 128, 4>, false, {}}};
  } else if (getenv("VS_ABL_SET") && !strcmp(getenv("VS_ABL_SET"), "g4i")) {
    // r03: the one-wave-per-SIMD 64-query layout with the step's fragment
    // reads interleaved into its MFMAs by sched_group_barrier (VAR 4194304),
    // against the product and the product interleaved the same way
    arms = {{"main (product)", run<0, 2048 + 256, 2>, true, {}},
            {"main ilv", run<0, 2048 + 256 + 4194304, 2>, true, {}},
            {"main G4 ilv", run<0, 2048 + 256 + 4194304, 4>, true, {}},
            {"no-epi (product)", run<1, 2048 + 256, 2>, false, {}},
            {"no-epi ilv", run<1, 2048 + 256 + 4194304, 2>, false, {}},
            {"no-epi G4 pd1", run<1, 2048 + 256, 4>, false, {}},
            {"no-epi G4 ilv", run<1, 2048 + 256 + 4194304, 4>, false, {}},
            {"no-epi G4 pd2 ilv", run<1, 2048 + 256 + 32 + 4194304, 4>, false, {}}};
  } else if (getenv("VS_ABL_SET") && !strcmp(getenv("VS_ABL_SET"), "early")) {
    // r04: the ring's first chunks issued before the query-fragment prologue
    // (VAR 8388608) against the product order, main pass and sample pass
    arms = {{"main (product)", run<0, 2048 + 256, 2>, true, {}},
            {"main early", run<0, 2048 + 256 + 8388608, 2>, true, {}},
            {"sample (product)", run_sample<2048 + 256>, false, {}},
            {"sample early", run_sample<2048 + 256 + 8388608>, false, {}}};
  } else if (getenv("VS_ABL_SET") && !strcmp(getenv("VS_ABL_SET"), "lists")) {
    // r04: the sorted-list pass (MODE 8: per-query top-k lists in LDS, no
    // sample pass, no select: a merge of nwg lists instead) at large shards,
    // unbounded and pinned, against the candidate main pass
    arms = {{"main (product)", run<0, 2048 + 256, 2>, true, {}},
            {"lists", run<8, 0, 2>, false, {}},
            {"lists pinned", run<8, 128, 2>, false, {}},
            {"lists 24k", run<8, 2048, 2>, false, {}},
            {"lists bounded", run<8, 0, 2>, true, {}}};
  } else if (getenv("VS_ABL_SET") && !strcmp(getenv("VS_ABL_SET"), "qmax")) {
    // r04: the main pass writing its quarter maxima (product) or not
    arms = {{"main (product)", run<0, 2048 + 256, 2>, true, {}},
            {"main no-qmax", run_nq<0, 2048 + 256, 2>, true, {}}};
  } else if (getenv("VS_ABL_SET") && !strcmp(getenv("VS_ABL_SET"), "product")) {
    // the product main pass alone (sample-tile sweeps: argv[3])
    arms = {{"main (product)", run<0, 2048 + 256, 2>, true, {}}};
  } else if (getenv("VS_ABL_SET") && !strcmp(getenv("VS_ABL_SET"), "barrier")) {
    // timing only: without the barrier the ring is unsynchronised (wrong
    // results, no hazard to the device: no waits depend on the data)
    arms = {{"main (product)", run<0, 2048 + 256, 2>, true, {}},
            {"no-epi (product)", run<1, 2048 + 256, 2>, false, {}},
            {"no-epi no-barrier", run<1, 2048 + 256 + 134217728, 2>, false, {}},
            {"no-epi 16k", run<1, 0, 2>, false, {}},
            {"no-epi 16k no-barrier", run<1, 134217728, 2>, false, {}}};
  } else if (getenv("VS_ABL_SET") && !strcmp(getenv("VS_ABL_SET"), "chunk")) {
    arms = {{"main bf", run<0, 0, 2>, true, {}},
            {"24k ring144", run<0, 2048 + 256, 2>, true, {}},
            {"48k ring144", run<0, 4096 + 256, 2>, true, {}},
            {"ring144", run<0, 256, 2>, true, {}}};
  } else if (getenv("VS_ABL_SET") && !strcmp(getenv("VS_ABL_SET"), "pd")) {
    arms = {{"main bf", run<0, 0, 2>, true, {}},
            {"PD2", run<0, 32, 2>, true, {}}};  // r02: 3.325 vs 3.340 ms, 0.426 vs 0.427 (noise)
  } else if (getenv("VS_ABL_SET") && !strcmp(getenv("VS_ABL_SET"), "lds")) {
    arms = {{"main bf", run<0, 0, 2>, true, {}},
            {"PD2", run<0, 32, 2>, true, {}},
            {"no-epilogue", run<1, 0, 2>, false, {}},
            {"half A reads (10)", run<10, 0, 2>, false, {}},
            {"half A, all MFMA (13)", run<13, 0, 2>, false, {}},
            {"no A reads (7)", run<7, 0, 2>, false, {}},
            {"dma-only", run<2, 0, 2>, false, {}}};
  } else if (!getenv("VS_ABL_SHORT")) {
    arms.push_back({"main weighted", run<0, 65536, 2>, true, {}});
    arms.push_back({"no-epilogue", run<1, 0, 2>, false, {}});
    arms.push_back({"max-only (6)", run<6, 0, 2>, true, {}});
    arms.push_back({"dma-only", run<2, 0, 2>, false, {}});
    arms.push_back({"qf-only", run<12, 0, 2>, false, {}});
    arms.push_back({"G4 no-epi pd3pin", run<1, 64 + 128, 4>, false, {}});
  }

  // arms rotate their position every rep: a fixed order measured position
  // effects of up to 8% (the arm after the tiny ones ran fastest, r01)
  for (int r = 0; r < reps; ++r)
    for (size_t j = 0; j < arms.size(); ++j) {
      auto& arm = arms[(j + (size_t)r) % arms.size()];
      arm.t.push_back(arm.fn(c, arm.bound));
    }
  CK(hipDeviceSynchronize());
  const double bytes = (double)n * 768 * 2, flops = 2.0 * 256 * n * 768;
  std::sort(ts.begin(), ts.end());
  printf("%-16s median %.3f ms  min %.3f ms\n", "sample+bound", ts[ts.size() / 2], ts[0]);
  for (auto& arm : arms) {
    std::sort(arm.t.begin(), arm.t.end());
    const float med = arm.t[arm.t.size() / 2];
    printf("%-16s median %.3f ms  min %.3f ms  HBM %.0f GB/s  MFMA %.0f TF/s\n", arm.name, med,
           arm.t[0], bytes / med / 1e6, flops / med / 1e9);
  }
  // VS_ABL_OVERLAP=1: what pipelining batches would save -- B iterations of
  // [main pass; sample pass + bound of the next batch] on one stream against
  // the sample pass on a second stream, free to start on the CUs the main
  // pass's workgroups leave early (tmax / bound of its own: no hazard)
  if (getenv("VS_ABL_OVERLAP")) {
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    float* tmax2;
    float* bnd2;
    CK(hipMalloc(&tmax2, (size_t)c.nwg * 256 * st * 4));
    CK(hipMalloc(&bnd2, 256 * 4));
    hipEvent_t e_main;
    CK(hipEventCreateWithFlags(&e_main, hipEventDisableTiming));
    const int B = 16;
    for (int rep = 0; rep < 4; ++rep) {
      for (int mode = 0; mode < 2; ++mode) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < B; ++i) {
          MfArgs m = c.args;
          hipLaunchKernelGGL((mfma_topk_kernel<768, 0, 2048 + 256, 2>), dim3(c.nwg), dim3(512), 0, 0,
                             m);
          hipStream_t ss = mode ? s2 : (hipStream_t)0;
          if (mode) {  // the next batch's sample may not pass this batch's main on s2's side
            CK(hipEventRecord(e_main, 0));
          }
          uint32_t L2 = 0;
          CK(launch_mfma_sample(X, false, 768, n, 0, Q, 256, k, st, tmax2, c.nwg, &L2, ss));
          CK(launch_sample_bound(tmax2, L2 * st, 256, k, bnd2, ss));
          if (mode) {
            hipEvent_t e_s;
            CK(hipEventCreateWithFlags(&e_s, hipEventDisableTiming));
            CK(hipEventRecord(e_s, s2));
            CK(hipStreamWaitEvent(0, e_s, 0));  // the next main pass waits for this bound
            CK(hipEventDestroy(e_s));
          }
        }
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("overlap rep %d %-10s %.3f ms per [main + sample + bound]\n", rep,
               mode ? "2 streams" : "1 stream", ms / B);
      }
    }
    return 0;
  }
  // the main pass once more, then its select (timed) and, on the host, how
  // many slab keys pass the select's first bound per query
  {
    MfArgs m = c.args;
    hipLaunchKernelGGL((mfma_topk_kernel<768, 0, 0, 2>), dim3(c.nwg), dim3(512), 0, 0, m);
    CK(hipDeviceSynchronize());
    std::vector<float> tsel;
    for (int r = 0; r < 3 * reps; ++r) {
      hipEventRecord(a, 0);
      CK(launch_select_slabs((const float*)cand, ctile, cnt, c.nwg, cap, 256, k, out, 0, 0,
                             nullptr, c.args.cand_max));
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      tsel.push_back(ms);
    }
    std::sort(tsel.begin(), tsel.end());
    printf("%-16s median %.1f us  min %.1f us\n", "slab select", 1e3 * tsel[tsel.size() / 2],
           1e3 * tsel[0]);
    const uint32_t* cmx = nullptr;
    auto sv = [&](auto kern, const char* name) {
      std::vector<float> tv;
      for (int r = 0; r < 3 * reps; ++r) {
        hipEventRecord(a, 0);
        hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, (const f32x4_t*)cand,
                           (const uint32_t*)ctile, (const uint32_t*)cnt, cmx, c.nwg, cap, k, out,
                           SlabMask{nullptr, 0}, (const uint32_t*)nullptr);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        tv.push_back(ms);
      }
      std::sort(tv.begin(), tv.end());
      printf("%-16s median %.1f us\n", name, 1e3 * tv[tv.size() / 2]);
    };
    sv(select_slab_kernel<1>, "sel: pass 1");
    sv(select_slab_kernel<2>, "sel: + sort");
    sv(select_slab_kernel<3>, "sel: + append");
    sv(select_slab_kernel<0>, "sel: full");
    if (c.args.cand_max) {  // r04: the main pass's quarter maxima
      cmx = qmx;
      sv(select_slab_kernel<0>, "sel: qmax full");
      cmx = nullptr;
    }
    const uint32_t nl = 4 * c.nwg, sub = cap / 4;
    std::vector<uint32_t> hcnt((size_t)256 * nl), htile((size_t)c.nwg * 256 * cap);
    std::vector<float> hsl((size_t)c.nwg * 256 * cap * 8);
    CK(hipMemcpy(hcnt.data(), cnt, hcnt.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(htile.data(), ctile, htile.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hsl.data(), cand, hsl.size() * 4, hipMemcpyDeviceToHost));
    double pass_sum = 0, slab_sum = 0;
    uint32_t pass_max = 0;
    for (uint32_t q = 0; q < 256; ++q) {
      std::vector<uint64_t> bmax(c.nwg, 0), keys;
      for (uint32_t l = 0; l < nl; ++l) {
        const uint32_t n = std::min(hcnt[((size_t)(l >> 2) * 256 + q) * 4 + (l & 3)], sub);
        slab_sum += n;
        for (uint32_t j = 0; j < n; ++j) {
          const size_t e = ((size_t)(l >> 2) * 256 + q) * cap + (l & 3) * sub + j;
          for (int bb = 0; bb < 8; ++bb) {
            const float sc = hsl[8 * e + bb];
            if (sc == -INFINITY) continue;
            const uint64_t key = vs::make_key(sc, htile[e] + 16 * (bb >> 2) + 4 * (l & 3) + (bb & 3));
            keys.push_back(key);
            bmax[l >> 2] = std::max(bmax[l >> 2], key);
          }
        }
      }
      std::sort(bmax.rbegin(), bmax.rend());
      const uint64_t thr = bmax[k - 1] ? bmax[k - 1] - 1 : 0;
      uint32_t np = 0;
      for (uint64_t x : keys) np += x > thr;
      pass_sum += np;
      pass_max = std::max(pass_max, np);
    }
    printf("slabs/query %.1f; keys past the select's first bound: mean %.1f, max %u\n",
           slab_sum / 256, pass_sum / 256, pass_max);
  }
  // per-workgroup clocks [start, prologue done, tiles done, end] of the
  // sample pass (MODE 3) and the main pass (MODE 0), VAR 8192: where the
  // fixed costs go (dispatch spread, prologue, tiles, write-out)
  auto clocks = [&](const char* name, auto kern, const MfArgs& args, int burst) -> int {
    for (int r = 0; r < 2; ++r) {
      hipEventRecord(a, 0);
      for (int i = 0; i < burst; ++i)
        hipLaunchKernelGGL(kern, dim3(c.nwg), dim3(512), 0, 0, args);
      hipEventRecord(b, 0);
      CK(hipDeviceSynchronize());
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      std::vector<uint64_t> clk((size_t)4 * c.nwg);
      CK(hipMemcpy(clk.data(), out, clk.size() * 8, hipMemcpyDeviceToHost));
      uint64_t s0 = ~0ull, s1 = 0, e1 = 0;
      double ph[3] = {0, 0, 0};
      for (uint32_t i = 0; i < c.nwg; ++i) {
        s0 = std::min(s0, clk[4 * i]), s1 = std::max(s1, clk[4 * i]);
        e1 = std::max(e1, clk[4 * i + 3]);
        for (int p = 0; p < 3; ++p) ph[p] += (double)(clk[4 * i + p + 1] - clk[4 * i + p]);
      }
      printf("%s clocks (burst %d): event %.1f us/launch, start spread %.1f us, mean prologue %.1f / "
             "tiles %.1f / write-out %.1f us, span %.1f us\n",
             name, burst, 1e3 * ms / burst, (s1 - s0) / 100.0, ph[0] / c.nwg / 100.0,
             ph[1] / c.nwg / 100.0, ph[2] / c.nwg / 100.0, (e1 - s0) / 100.0);
    }
    return 0;
  };
  {
    MfArgs sa{};
    sa.X = X, sa.Q = Q, sa.tmax = tmax;
    sa.max_tiles = st, sa.n_rows = n, sa.rows_per_wg = rpw, sa.nq_valid = 256, sa.k = k;
    sa.lists = out;
    MfArgs ma = c.args;
    ma.lists = out;
    for (int burst : {1, 8}) {
      if (clocks("sample", mfma_topk_kernel<768, 3, 8192, 2>, sa, burst)) return 1;
      if (clocks("main", mfma_topk_kernel<768, 0, 8192, 2>, ma, burst)) return 1;
      if (getenv("VS_ABL_SET") && !strcmp(getenv("VS_ABL_SET"), "early")) {
        if (clocks("sample early", mfma_topk_kernel<768, 3, 8192 + 8388608, 2>, sa, burst)) return 1;
        if (clocks("main early", mfma_topk_kernel<768, 0, 8192 + 8388608, 2>, ma, burst)) return 1;
      }
    }
  }
  std::vector<uint32_t> hc((size_t)c.nwg * 256 * 4);
  CK(hipMemcpy(hc.data(), cnt, hc.size() * 4, hipMemcpyDeviceToHost));
  uint64_t tot = 0, mx = 0;
  for (uint32_t v : hc) tot += v, mx = v > mx ? v : mx;
  printf("cap %u; grid %u WGs x %u rows, sample tiles/wg %u, slabs/query %.1f, max per buffer %lu\n",
         cap, c.nwg, rpw, st, (double)tot / 256, (unsigned long)mx);
  return 0;
}
