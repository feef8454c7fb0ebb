// share_pipe.hip — the batched int8 path's per-batch stages at one shard's
// size, timed back to back (r05; VERDICT r04 item 1: the N = 8 share's fixed
// cost). Replays vs_engine.cpp search_mfma's int8 branch with the library's
// launchers on one resident corpus and times R batches per arm (events only
// around the whole loop, so the arms see the serving regime):
//   full      query prep + sample pass + bound/int8 queries + int8 pass +
//             select (the product's sequence since r05)
//   r04gate   full + r04's two gated launches (stand-downs)
//   noselect  without the select (and gates)
//   pass      the int8 pass alone (bound precomputed)
//   front     query prep + sample pass + bound only
// then one batch with select_q8's per-workgroup stage clocks (start, bound,
// survivors, rescore, end; medians over the queries, us).
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/share_pipe.hip -o tools/share_pipe \
//     -I<pkg>/csrc -L<pkg>/lib -lvsearch -Wl,-rpath,<pkg>/lib
//   share_pipe [ROWS=1250000] [K=10] [REPS=200] [DIM=768] [NQ=256 / 128 above 768-d]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
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
  const uint32_t n = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 1250000;
  const uint32_t k = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 10;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 200;
  const uint32_t dim = argc > 4 ? (uint32_t)std::atoi(argv[4]) : 768;
  // queries per batch: one int8 launch's worth (256 up to 768-d, 128 above)
  const uint32_t nq = argc > 5 ? (uint32_t)std::atoi(argv[5]) : (dim <= 768 ? 256u : 128u), PS = 256;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint16_t *X, *qb;
  int8_t *X8, *q8q;
  float *meta, *glob, *qf, *qp, *q8par, *tmax, *bound, *slabs;
  CK(hipMalloc(&X, (size_t)(n + 32) * dim * 2));
  CK(hipMemset(X, 0, (size_t)(n + 32) * dim * 2));
  CK(hipMalloc(&X8, (size_t)(n + 32) * dim));
  CK(hipMemset(X8, 0, (size_t)(n + 32) * dim));
  CK(hipMalloc(&meta, (size_t)((n + 32) / 32 + 1) * 8));
  CK(hipMalloc(&glob, vsk::kQ8GlobBytes));
  CK(hipMemset(glob, 0, vsk::kQ8GlobBytes));
  CK(hipMalloc(&qf, (size_t)PS * dim * 4));
  CK(hipMalloc(&qp, (size_t)PS * dim * 4));
  CK(hipMalloc(&qb, (size_t)PS * dim * 2));
  CK(hipMalloc(&q8q, (size_t)PS * dim));
  CK(hipMalloc(&q8par, PS * 16 + 64));
  uint32_t* gate = (uint32_t*)(q8par + 4 * PS);
  CK(vsk::launch_generate(0x5EED, 0, n, dim, true, X, 0, st));
  CK(vsk::launch_generate(0xC0FFEE, 0, nq, dim, false, qf, 0, st, 1));
  CK(hipMemsetAsync(glob, 0, 16, st));
  CK(vsk::launch_q8_absmax(X, false, (uint64_t)n * dim, glob, st));
  CK(vsk::launch_q8_set_scale(glob, st));
  CK(vsk::launch_q8_quantize(X, false, n, dim, nullptr, 0, (n + 31) / 32, X8, meta, glob, st));
  const uint32_t maxl = vsk::mfma_max_lists(n);
  const uint32_t st0 = vsk::mfma_sample_tiles(n, dim, false);
  const uint32_t tpw = vsk::mfma_tiles_per_wg(n);
  const char* fe = std::getenv("VS_Q8_SAMPLE");  // as vs_engine.cpp: the sample factor override
  const double f = fe && std::atof(fe) > 0 ? std::atof(fe) : (k <= 16 ? 1.0 : k <= 64 ? 2.0 : 4.0);
  const uint32_t stl = (uint32_t)std::max(1.0, std::min({(double)vsk::kMfmaMaxSampleTiles, (double)tpw,
                                                          st0 * f}));
  const uint32_t cap = vsk::mfma_cand_cap(n, k, stl);
  const uint32_t cap8 = vsk::mfma_cand_cap(n, k, st0, 8.0);
  const uint32_t capx = std::max(cap, cap8);
  const size_t slots = (size_t)maxl * PS * capx;
  CK(hipMalloc(&slabs, slots * 36));
  uint32_t* slab_tile = (uint32_t*)((char*)slabs + slots * 32);
  uint32_t* cnt;
  CK(hipMalloc(&cnt, (size_t)maxl * PS * 4 * 4 * 2));
  uint32_t* qmax = cnt + (size_t)maxl * PS * 4;
  CK(hipMalloc(&tmax, (size_t)maxl * stl * PS * 4));
  CK(hipMalloc(&bound, PS * 4));
  uint64_t *out, *clk;
  CK(hipMalloc(&out, (size_t)nq * k * 8));
  CK(hipMalloc(&clk, (size_t)nq * 16 * 8));
  CK(hipMemset(clk, 0, (size_t)nq * 16 * 8));

  uint32_t L = 0;
  auto prep = [&]() { CK(vsk::launch_query_prep(qf, nq, dim, false, true, nullptr, qb, st)); };
  auto sample = [&]() {
    CK(vsk::launch_mfma_sample(X, false, dim, n, 0, qb, nq, k, stl, tmax, maxl, &L, st, nullptr));
  };
  auto boundq8 = [&]() {
    CK(vsk::launch_sample_bound_q8(tmax, L * stl, nq, k, bound, qb, false, nq, dim, glob, q8q, q8par,
                                   gate, st));
  };
  auto pass = [&]() {
    CK(vsk::launch_mfma_cand_q8(X8, dim, n, 0, q8q, nq, k, bound, q8par, glob, slabs, slab_tile, cap8,
                                cnt, qmax, maxl, &L, gate, st, nullptr));
  };
  auto select = [&](uint64_t* c) {
    CK(vsk::launch_select_q8(slabs, slab_tile, cnt, qmax, L, cap8, nq, k, out, 0, X, qb, false, dim,
                             q8par, glob, meta, bound, X8, q8q, nullptr, n, st, nullptr, c));
  };
  // r04's two gated launches (the bf16 pass + select behind every int8
  // batch, standing down unless *gate): kept as an arm to price them
  auto gated = [&]() {
    CK(vsk::launch_mfma_cand(X, false, dim, n, 0, qb, nq, k, bound, slabs, slab_tile, cap, cnt, maxl, &L,
                             st, nullptr, qmax, gate));
    CK(vsk::launch_select_slabs(slabs, slab_tile, cnt, L, cap, nq, k, out, st, 0, nullptr, qmax, gate));
  };
  // one full batch first: bounds and int8 queries for the "pass" arm
  prep(), sample(), boundq8(), pass(), select(nullptr);
  CK(hipStreamSynchronize(st));
  uint32_t hg = 0;
  CK(hipMemcpy(&hg, gate, 4, hipMemcpyDeviceToHost));

  struct Arm {
    const char* name;
    std::function<void()> f;
  };
  // (r05) a speculative bound's best case: every query's bound set just under
  // its exact k-th score (from the full batch above), then the int8 pass and
  // the select alone -- no query prep, sample or bound launch. The select's
  // k-th must reach the bound (checked below): the exactness test a
  // speculative bound would rely on.
  std::vector<uint64_t> hk((size_t)nq * k);
  CK(hipMemcpy(hk.data(), out, hk.size() * 8, hipMemcpyDeviceToHost));
  std::vector<float> hb(nq), hb0(nq);
  CK(hipMemcpy(hb0.data(), bound, nq * 4, hipMemcpyDeviceToHost));
  for (uint32_t q = 0; q < nq; ++q) {
    const float sk = vs::key_score(hk[(size_t)q * k + k - 1]);
    hb[q] = sk - 1e-4f * std::max(1.f, std::fabs(sk));
  }
  float* sbound;
  CK(hipMalloc(&sbound, nq * 4));
  CK(hipMemcpy(sbound, hb.data(), nq * 4, hipMemcpyHostToDevice));
  auto pass_s = [&]() {
    CK(vsk::launch_mfma_cand_q8(X8, dim, n, 0, q8q, nq, k, sbound, q8par, glob, slabs, slab_tile, cap8,
                                cnt, qmax, maxl, &L, gate, st, nullptr));
  };
  auto select_s = [&]() {
    CK(vsk::launch_select_q8(slabs, slab_tile, cnt, qmax, L, cap8, nq, k, out, 0, X, qb, false, dim,
                             q8par, glob, meta, sbound, X8, q8q, nullptr, n, st, nullptr, nullptr));
  };
  // (r06) the product's speculative sequence (vs_engine.cpp search_mfma),
  // priced launch by launch: the collection's ratio for k set from the batch
  // above (0.97 x its smallest k-th per |q|), then query prep + int8 queries
  // with the bound and the go / verdict words, the pass and the select gated
  // on go, the check, and behind it the five fallback launches that stand
  // down when the batch verified
  vsk::Q8SpecK* sk = vsk::q8_spec_k(glob);
  vsk::Q8SpecStat* sstat = vsk::q8_spec_stat(glob);
  {
    std::vector<float> hq((size_t)nq * dim);
    CK(hipMemcpy(hq.data(), qf, hq.size() * 4, hipMemcpyDeviceToHost));
    double rmin = 1e30;
    for (uint32_t q = 0; q < nq; ++q) {
      double a2 = 0;
      for (uint32_t d = 0; d < dim; ++d) a2 += (double)hq[(size_t)q * dim + d] * hq[(size_t)q * dim + d];
      rmin = std::min(rmin, (double)vs::key_score(hk[(size_t)q * k + k - 1]) / std::sqrt(a2));
    }
    const float r = (float)(0.97 * rmin);
    CK(hipMemcpy(&sk[k].ratio, &r, 4, hipMemcpyHostToDevice));
  }
  const uint32_t* go = gate + vsk::kGateGo;
  auto q8q_spec = [&]() {
    CK(vsk::launch_q8_query(qb, false, nq, dim, glob, q8q, q8par, gate, st, &sk[k].ratio, bound,
                            &sk[k], sstat, true));
  };
  auto pass_g = [&]() {
    CK(vsk::launch_mfma_cand_q8(X8, dim, n, 0, q8q, nq, k, bound, q8par, glob, slabs, slab_tile, cap8,
                                cnt, qmax, maxl, &L, gate, st, nullptr, go));
  };
  auto select_g = [&]() {
    CK(vsk::launch_select_q8(slabs, slab_tile, cnt, qmax, L, cap8, nq, k, out, 0, X, qb, false, dim,
                             q8par, glob, meta, bound, X8, q8q, nullptr, n, st, nullptr, nullptr, go));
  };
  auto verify = [&]() {
    CK(vsk::launch_q8_verify_record(out, nq, k, dim, bound, q8par, glob, true, gate, &sk[k], sstat,
                                    nullptr, st, go));
  };
  const uint32_t* fb = gate + vsk::kGateVerdict;
  auto fallback = [&]() {
    CK(vsk::launch_mfma_sample(X, false, dim, n, 0, qb, nq, k, stl, tmax, maxl, &L, st, nullptr, fb));
    CK(vsk::launch_sample_bound_q8(tmax, L * stl, nq, k, bound, qb, false, nq, dim, glob, q8q, q8par,
                                   nullptr, st, fb));
    CK(vsk::launch_mfma_cand_q8(X8, dim, n, 0, q8q, nq, k, bound, q8par, glob, slabs, slab_tile, cap8,
                                cnt, qmax, maxl, &L, gate, st, nullptr, fb));
    CK(vsk::launch_select_q8(slabs, slab_tile, cnt, qmax, L, cap8, nq, k, out, 0, X, qb, false, dim,
                             q8par, glob, meta, bound, X8, q8q, nullptr, n, st, nullptr, nullptr, fb));
    CK(vsk::launch_q8_verify_record(out, nq, k, dim, bound, q8par, glob, false, nullptr, &sk[k], sstat,
                                    nullptr, st, fb));
  };
  std::vector<Arm> arms = {
      {"specseq_fb", [&] { prep(), q8q_spec(), pass_g(), select_g(), verify(), fallback(); }},
      {"specseq", [&] { prep(), q8q_spec(), pass_g(), select_g(), verify(); }},
      {"specseq_nover", [&] { prep(), q8q_spec(), pass_g(), select_g(); }},
      {"specseq_noprep", [&] { q8q_spec(), pass_g(), select_g(), verify(); }},
      {"specseq_pass", [&] { q8q_spec(), pass_g(); }},
      {"spec", [&] { pass_s(), select_s(); }},
      {"full", [&] { prep(), sample(), boundq8(), pass(), select(nullptr); }},
      {"r04gate", [&] { prep(), sample(), boundq8(), pass(), select(nullptr), gated(); }},
      {"noselect", [&] { prep(), sample(), boundq8(), pass(); }},
      {"pass", [&] { pass(); }},
      {"front", [&] { prep(), sample(), boundq8(); }},
  };
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::printf("{\"rows\": %u, \"k\": %u, \"dim\": %u, \"nq\": %u, \"reps\": %d, \"sample_tiles\": %u, "
              "\"cap8\": %u, \"gate\": %u", n, k, dim, nq, reps, stl, cap8, hg);
  // arms interleaved over rounds (clock drift spreads evenly); medians
  const int rounds = 5;
  std::vector<std::vector<float>> t(arms.size());
  for (int r = 0; r < rounds; ++r)
    for (size_t i = 0; i < arms.size(); ++i) {
      for (int w = 0; w < 5; ++w) arms[i].f();
      CK(hipEventRecord(a, st));
      for (int j = 0; j < reps; ++j) arms[i].f();
      CK(hipEventRecord(b, st));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      t[i].push_back(ms * 1e3f / reps);
    }
  for (size_t i = 0; i < arms.size(); ++i) {
    std::sort(t[i].begin(), t[i].end());
    std::printf(", \"%s_us\": %.2f", arms[i].name, t[i][rounds / 2]);
  }
  // select stage clocks (wall_clock64: 100 MHz) and counts (slabs read,
  // survivors, slow-path queries, queries whose quarter bound beat the sample's)
  uint32_t* stats;
  CK(hipMalloc(&stats, 16));
  CK(hipMemset(stats, 0, 16));
  prep(), sample(), boundq8(), pass();
  CK(vsk::launch_select_q8(slabs, slab_tile, cnt, qmax, L, cap8, nq, k, out, 0, X, qb, false, dim, q8par,
                           glob, meta, bound, X8, q8q, nullptr, n, st, stats, clk));
  CK(hipStreamSynchronize(st));
  std::vector<uint64_t> h((size_t)nq * 16);
  CK(hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost));
  uint64_t t0 = ~0ull;
  for (uint32_t q = 0; q < nq; ++q) t0 = std::min(t0, h[(size_t)q * 16]);
  const char* names[12] = {"start", "bound",  "survivors", "rescore", "end",    "p1",
                           "round1", "p2", "s_lossy",  "s_owner", "s_issue", "s_tested"};
  for (int s = 0; s < 12; ++s) {
    std::vector<double> v;
    for (uint32_t q = 0; q < nq; ++q)
      if (h[(size_t)q * 16 + s]) v.push_back((h[(size_t)q * 16 + s] - t0) * 0.01);
    std::sort(v.begin(), v.end());
    if (!v.empty())
      std::printf(", \"sel_%s_us_med\": %.2f, \"sel_%s_us_max\": %.2f", names[s], v[v.size() / 2], names[s],
                  v.back());
  }
  // the speculative arm's answers: equal to the full pipeline's, and every
  // query's k-th at or above its bound
  pass_s(), select_s();
  CK(hipStreamSynchronize(st));
  std::vector<uint64_t> hk2((size_t)nq * k);
  CK(hipMemcpy(hk2.data(), out, hk2.size() * 8, hipMemcpyDeviceToHost));
  uint32_t spec_diff = 0, spec_below = 0;
  for (size_t i = 0; i < hk.size(); ++i) spec_diff += hk[i] != hk2[i];
  for (uint32_t q = 0; q < nq; ++q) spec_below += vs::key_score(hk2[(size_t)q * k + k - 1]) < hb[q];
  double gap = 0;
  for (uint32_t q = 0; q < nq; ++q) gap += hb[q] - hb0[q];
  std::printf(", \"spec_keys_differ\": %u, \"spec_kth_below_bound\": %u, \"spec_bound_gain_mean\": %.5f",
              spec_diff, spec_below, gap / nq);
  // (r05) a speculative bound from another batch's statistics: r = 0.97 x the
  // smallest k-th score per unit |q| over batch A (the one above), applied to
  // a fresh batch B (the next nq queries of the stream) as b(q) = r |q|;
  // B's keys through the full pipeline and through pass + select under that
  // bound, compared, and B's queries whose k-th fell under their bound (the
  // ones a gated fallback would redo) counted
  {
    auto norms = [&](std::vector<float>& nv) {
      std::vector<float> hq((size_t)nq * dim);
      CK(hipMemcpy(hq.data(), qf, hq.size() * 4, hipMemcpyDeviceToHost));
      nv.assign(nq, 0.f);
      for (uint32_t q = 0; q < nq; ++q) {
        double a2 = 0;
        for (uint32_t d = 0; d < dim; ++d) a2 += (double)hq[(size_t)q * dim + d] * hq[(size_t)q * dim + d];
        nv[q] = (float)std::sqrt(a2);
      }
    };
    std::vector<float> na, nb;
    norms(na);
    double rmin = 1e30;
    for (uint32_t q = 0; q < nq; ++q)
      if (na[q] > 0) rmin = std::min(rmin, (double)vs::key_score(hk[(size_t)q * k + k - 1]) / na[q]);
    const float r = (float)(rmin > 0 ? rmin * 0.97 : 0.0);
    CK(vsk::launch_generate(0xC0FFEE, nq, nq, dim, false, qf, 0, st, 1));
    CK(hipStreamSynchronize(st));
    norms(nb);
    prep(), sample(), boundq8(), pass(), select(nullptr);
    CK(hipStreamSynchronize(st));
    std::vector<uint64_t> kb((size_t)nq * k), kb2((size_t)nq * k);
    CK(hipMemcpy(kb.data(), out, kb.size() * 8, hipMemcpyDeviceToHost));
    std::vector<float> bb(nq);
    for (uint32_t q = 0; q < nq; ++q) bb[q] = r * nb[q];
    CK(hipMemcpy(sbound, bb.data(), nq * 4, hipMemcpyHostToDevice));
    pass_s(), select_s();
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(kb2.data(), out, kb2.size() * 8, hipMemcpyDeviceToHost));
    uint32_t diff = 0, below = 0;
    for (size_t i = 0; i < kb.size(); ++i) diff += kb[i] != kb2[i];
    for (uint32_t q = 0; q < nq; ++q) below += vs::key_score(kb[(size_t)q * k + k - 1]) < bb[q];
    auto time_arm = [&](const std::function<void()>& f) {
      for (int w = 0; w < 5; ++w) f();
      std::vector<float> tv;
      for (int rr = 0; rr < 3; ++rr) {
        CK(hipEventRecord(a, st));
        for (int j = 0; j < reps; ++j) f();
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        tv.push_back(ms * 1e3f / reps);
      }
      std::sort(tv.begin(), tv.end());
      return tv[1];
    };
    const float tf = time_arm([&] { prep(), sample(), boundq8(), pass(), select(nullptr); });
    const float ts = time_arm([&] { pass_s(), select_s(); });
    std::printf(", \"fresh_ratio\": %.5f, \"fresh_full_us\": %.2f, \"fresh_spec_us\": %.2f, "
                "\"fresh_keys_differ_where_kth_reaches_bound\": %u, \"fresh_kth_below_bound\": %u",
                r, tf, ts, below ? 0u : diff, below);
    if (below) {  // keys of queries whose k-th reached their bound must still agree
      uint32_t d2 = 0;
      for (uint32_t q = 0; q < nq; ++q)
        if (vs::key_score(kb[(size_t)q * k + k - 1]) >= bb[q])
          for (uint32_t j = 0; j < k; ++j) d2 += kb[(size_t)q * k + j] != kb2[(size_t)q * k + j];
      std::printf(", \"fresh_keys_differ_verified_queries\": %u", d2);
    }
  }
  uint32_t hs[4];
  CK(hipMemcpy(hs, stats, 16, hipMemcpyDeviceToHost));
  std::printf(", \"sel_slabs_per_query\": %.1f, \"sel_survivors_per_query\": %.1f, \"sel_slow_queries\": %u, "
              "\"sel_quarter_bound_won\": %u", (double)hs[0] / nq, (double)hs[1] / nq, hs[2], hs[3]);
  std::printf("}\n");
  return 0;
}
