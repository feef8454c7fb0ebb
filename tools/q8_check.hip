// q8_check.hip — checks the int8 prefilter's pieces on the device against a
// host computation (r04): quantisation (x8, tile bounds), int8 queries and
// their bounds, the int8 MFMA pass's dots (every slab admitted: no bound),
// and that each row's fp32 score lies inside [L, U].
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/q8_check.hip -o tools/q8_check \
//     -I<pkg>/csrc -L<pkg>/lib -lvsearch -Wl,-rpath,<pkg>/lib
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "vs_common.h"
#include "vs_kernels.h"

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

// Stats mode: q8_check N [NQ [DIM [K]]] (N > 65536): device-generated rows and
// queries, the pipeline once, slabs / survivors per query; no host check.
int stats_mode(uint32_t n, uint32_t nq, uint32_t dim, uint32_t k) {
  uint16_t *dX, *dQ;
  int8_t *dX8, *dQ8;
  float *meta, *glob, *par, *tmax, *bound;
  CK(hipMalloc(&dX, (size_t)(n + 32) * dim * 2));
  CK(hipMalloc(&dQ, (size_t)256 * dim * 2));
  CK(hipMalloc(&dX8, (size_t)(n + 32) * dim));
  CK(hipMalloc(&dQ8, (size_t)256 * dim));
  CK(hipMalloc(&meta, (size_t)(n / 32 + 2) * 8));
  CK(hipMalloc(&glob, 16));
  CK(hipMalloc(&par, 256 * 16 + 64));
  CK(hipMemset(dX, 0, (size_t)(n + 32) * dim * 2));
  CK(vsk::launch_generate(0x5EED, 0, n, dim, true, dX, 0, 0));
  CK(vsk::launch_generate(0xC0FFEE, 0, nq, dim, true, dQ, 0, 0));
  CK(hipMemset(glob, 0, 16));
  CK(vsk::launch_q8_absmax(dX, false, (uint64_t)n * dim, glob, 0));
  CK(vsk::launch_q8_set_scale(glob, 0));
  CK(vsk::launch_q8_quantize(dX, false, n, dim, nullptr, 0, (n + 31) / 32, dX8, meta, glob, 0));
  uint32_t* gate = (uint32_t*)(par + 4 * 256);
  CK(vsk::launch_q8_query(dQ, false, nq, dim, glob, dQ8, par, gate, 0));
  const uint32_t nwg = vsk::mfma_max_lists(n), st = vsk::mfma_sample_tiles(n, dim, false);
  const uint32_t cap = vsk::mfma_cand_cap(n, k, st, 8.0);  // as search_mfma
  float* slabs;
  uint32_t *tiles, *cnt, *cmx, *stats;
  const size_t slots = (size_t)nwg * 256 * cap;
  CK(hipMalloc(&slabs, slots * 32));
  CK(hipMalloc(&tiles, slots * 4));
  CK(hipMalloc(&cnt, (size_t)nwg * 256 * 16));
  CK(hipMalloc(&cmx, (size_t)nwg * 256 * 16));
  CK(hipMalloc(&stats, 16));
  CK(hipMemset(stats, 0, 16));
  CK(hipMalloc(&tmax, (size_t)256 * nwg * st * 4));
  CK(hipMalloc(&bound, 256 * 4));
  uint64_t* out;
  CK(hipMalloc(&out, 256 * k * 8));
  uint32_t L = 0;
  CK(vsk::launch_mfma_sample(dX, false, dim, n, 0, dQ, nq, k, st, tmax, nwg, &L, 0));
  CK(vsk::launch_sample_bound(tmax, L * st, nq, k, bound, 0));
  CK(vsk::launch_mfma_cand_q8(dX8, dim, n, 0, dQ8, nq, k, bound, par, glob, slabs, tiles, cap, cnt,
                              cmx, nwg, &L, gate, 0));
  CK(vsk::launch_select_q8(slabs, tiles, cnt, cmx, nwg, cap, nq, k, out, 0, dX, dQ, false, dim, par, glob,
                           meta, bound, dX8, dQ8, nullptr, n, 0, stats));
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> hc((size_t)nwg * 256 * 4);
  CK(hipMemcpy(hc.data(), cnt, hc.size() * 4, hipMemcpyDeviceToHost));
  uint32_t hs[2], hgate;
  CK(hipMemcpy(hs, stats, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&hgate, gate, 4, hipMemcpyDeviceToHost));
  uint64_t tot = 0, qmax = 0;
  for (uint32_t w = 0; w < nwg; ++w)
    for (uint32_t q = 0; q < nq; ++q)
      for (uint32_t kq = 0; kq < 4; ++kq) {
        const uint32_t c = hc[((size_t)w * 256 + q) * 4 + kq];
        tot += c;
        qmax = std::max<uint64_t>(qmax, c);
      }
  std::printf("{\"rows\": %u, \"dim\": %u, \"k\": %u, \"queries\": %u, \"cap\": %u, \"gate\": %u, "
              "\"slabs_per_query\": %.1f, \"fullest_quarter\": %llu, "
              "\"slabs_read_per_query\": %.1f, \"survivors_per_query\": %.1f}\n",
              n, dim, k, nq, cap, hgate, (double)tot / nq, (unsigned long long)qmax, (double)hs[0] / nq,
              (double)hs[1] / nq);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::atoi(argv[1]) > 65536)
    return stats_mode((uint32_t)std::atoi(argv[1]), argc > 2 ? (uint32_t)std::atoi(argv[2]) : 256,
                      argc > 3 ? (uint32_t)std::atoi(argv[3]) : 768,
                      argc > 4 ? (uint32_t)std::atoi(argv[4]) : 10);
  const uint32_t dim = 768, n = 65536, nq = 4, k = 10;
  std::mt19937 rng(7);
  std::normal_distribution<float> nd;
  std::vector<uint16_t> X((size_t)(n + 32) * dim, 0), Q((size_t)256 * dim, 0);
  for (uint32_t r = 0; r < n; ++r) {
    double s = 0;
    std::vector<float> v(dim);
    for (auto& x : v) x = nd(rng), s += (double)x * x;
    for (uint32_t d = 0; d < dim; ++d) X[(size_t)r * dim + d] = vs::f32_to_bf16((float)(v[d] / std::sqrt(s)));
  }
  for (uint32_t q = 0; q < nq; ++q) {
    double s = 0;
    std::vector<float> v(dim);
    for (auto& x : v) x = nd(rng), s += (double)x * x;
    for (uint32_t d = 0; d < dim; ++d) Q[(size_t)q * dim + d] = vs::f32_to_bf16((float)(v[d] / std::sqrt(s)));
  }
  uint16_t *dX, *dQ;
  int8_t *dX8, *dQ8;
  float *meta, *glob, *par;
  CK(hipMalloc(&dX, X.size() * 2));
  CK(hipMalloc(&dQ, Q.size() * 2));
  CK(hipMalloc(&dX8, (size_t)(n + 32) * dim));
  CK(hipMalloc(&dQ8, (size_t)256 * dim));
  CK(hipMalloc(&meta, (size_t)(n / 32 + 2) * 8));
  CK(hipMalloc(&glob, 16));
  CK(hipMalloc(&par, 256 * 16 + 64));
  CK(hipMemcpy(dX, X.data(), X.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dQ, Q.data(), Q.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemset(dX8, 0, (size_t)(n + 32) * dim));
  CK(hipMemset(glob, 0, 16));
  CK(vsk::launch_q8_absmax(dX, false, (uint64_t)n * dim, glob, 0));
  CK(vsk::launch_q8_set_scale(glob, 0));
  CK(vsk::launch_q8_quantize(dX, false, n, dim, nullptr, 0, n / 32, dX8, meta, glob, 0));
  uint32_t* gate = (uint32_t*)(par + 4 * 256);
  CK(vsk::launch_q8_query(dQ, false, nq, dim, glob, dQ8, par, gate, 0));
  uint32_t nwg = vsk::mfma_max_lists(n), tpw = vsk::mfma_tiles_per_wg(n);
  const uint32_t cap = 4 * tpw < 64 ? 64 : 4 * tpw;
  std::printf("nwg %u tiles/wg %u cap %u\n", nwg, tpw, cap);
  float* slabs;
  uint32_t *tiles, *cnt;
  const size_t slots = (size_t)nwg * 256 * cap;
  CK(hipMalloc(&slabs, slots * 32));
  CK(hipMalloc(&tiles, slots * 4));
  CK(hipMalloc(&cnt, (size_t)nwg * 256 * 4 * 4));
  uint32_t* cmx;
  CK(hipMalloc(&cmx, (size_t)nwg * 256 * 4 * 4));
  uint32_t L = 0;
  CK(vsk::launch_mfma_cand_q8(dX8, dim, n, 0, dQ8, nq, k, nullptr, par, glob, slabs, tiles, cap,
                              cnt, cmx, nwg, &L, gate, 0));
  CK(hipDeviceSynchronize());
  std::vector<int8_t> X8((size_t)n * dim), Q8((size_t)nq * dim);
  std::vector<float> hm((size_t)(n / 32) * 2), hg(4), hp(4 * nq);
  CK(hipMemcpy(X8.data(), dX8, X8.size(), hipMemcpyDeviceToHost));
  CK(hipMemcpy(Q8.data(), dQ8, Q8.size(), hipMemcpyDeviceToHost));
  CK(hipMemcpy(hm.data(), meta, hm.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hg.data(), glob, 16, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hp.data(), par, hp.size() * 4, hipMemcpyDeviceToHost));
  uint32_t hgate = 0;
  CK(hipMemcpy(&hgate, gate, 4, hipMemcpyDeviceToHost));
  std::printf("glob absmax %g dmax %g nmax %g S %g gate %u\n", hg[0], hg[1], hg[2], hg[3], hgate);
  int bad_q = 0;
  const float S = hg[3];
  for (uint32_t r = 0; r < n; ++r)
    for (uint32_t d = 0; d < dim; ++d) {
      const float x = vs::bf16_to_f32(X[(size_t)r * dim + d]);
      float y = std::nearbyint(x / S);
      y = std::fmin(std::fmax(y, -127.f), 127.f);
      if ((int)y != X8[(size_t)r * dim + d] && bad_q++ < 5)
        std::printf("x8 mismatch r %u d %u: %d vs %d\n", r, d, (int)y, X8[(size_t)r * dim + d]);
    }
  std::printf("x8 mismatches: %d\n", bad_q);
  std::vector<uint32_t> hc((size_t)nwg * 256 * 4);
  CK(hipMemcpy(hc.data(), cnt, hc.size() * 4, hipMemcpyDeviceToHost));
  std::vector<int32_t> hs(slots * 8);
  std::vector<uint32_t> ht(slots);
  CK(hipMemcpy(hs.data(), slabs, slots * 32, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ht.data(), tiles, slots * 4, hipMemcpyDeviceToHost));
  long checked = 0, bad_dot = 0, bad_bound = 0;
  for (uint32_t q = 0; q < nq; ++q) {
    for (uint32_t w = 0; w < nwg; ++w)
      for (uint32_t kq = 0; kq < 4; ++kq) {
        const uint32_t c = hc[((size_t)w * 256 + q) * 4 + kq];
        for (uint32_t j = 0; j < c; ++j) {
          const size_t e = ((size_t)w * 256 + q) * cap + kq * (cap / 4) + j;
          for (int b = 0; b < 8; ++b) {
            const uint32_t row = ht[e] + 16 * (b >> 2) + 4 * kq + (b & 3);
            const int got = hs[e * 8 + b];
            if (row >= n) continue;
            int want = 0;
            double ex = 0;
            for (uint32_t d = 0; d < dim; ++d) {
              want += (int)X8[(size_t)row * dim + d] * (int)Q8[(size_t)q * dim + d];
              ex += (double)vs::bf16_to_f32(X[(size_t)row * dim + d]) *
                    (double)vs::bf16_to_f32(Q[(size_t)q * dim + d]);
            }
            ++checked;
            if (got != want && bad_dot++ < 5)
              std::printf("dot mismatch q %u row %u: %d vs %d\n", q, row, got, want);
            const float dt = hm[2 * (row / 32)], nt = hm[2 * (row / 32) + 1];
            const float m = hp[4 * q + 1] * dt + (hp[4 * q + 2] + hp[4 * q + 3]) * nt;
            const float Lb = (float)want * hp[4 * q] - m, Ub = (float)want * hp[4 * q] + m;
            if ((ex < Lb || ex > Ub) && bad_bound++ < 5)
              std::printf("bound miss q %u row %u: %g not in [%g, %g]\n", q, row, ex, Lb, Ub);
          }
        }
      }
    std::printf("q %u par sqS %g a %g c %g sigma %g\n", q, hp[4 * q], hp[4 * q + 1], hp[4 * q + 2],
                hp[4 * q + 3]);
  }
  std::printf("checked %ld dots: %ld wrong, %ld outside bounds\n", checked, bad_dot, bad_bound);
  // the whole pipeline: sample pass + bound (bf16), int8 pass with the bound,
  // select_q8 -> top k against the host's exact top k
  const uint32_t st = vsk::mfma_sample_tiles(n, dim, false);
  float *tmax, *bound;
  uint64_t* out;
  CK(hipMalloc(&tmax, (size_t)256 * nwg * st * 4));
  CK(hipMalloc(&bound, 256 * 4));
  CK(hipMalloc(&out, 256 * k * 8));
  CK(hipMemset(out, 0, 256 * k * 8));
  CK(vsk::launch_mfma_sample(dX, false, dim, n, 0, dQ, nq, k, st, tmax, nwg, &L, 0));
  CK(vsk::launch_sample_bound(tmax, L * st, nq, k, bound, 0));
  CK(vsk::launch_q8_query(dQ, false, nq, dim, glob, dQ8, par, gate, 0));
  CK(vsk::launch_mfma_cand_q8(dX8, dim, n, 0, dQ8, nq, k, bound, par, glob, slabs, tiles, cap,
                              cnt, cmx, nwg, &L, gate, 0));
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(hc.data(), cnt, hc.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&hgate, gate, 4, hipMemcpyDeviceToHost));
  std::vector<float> hb(nq);
  CK(hipMemcpy(hb.data(), bound, nq * 4, hipMemcpyDeviceToHost));
  for (uint32_t q = 0; q < nq; ++q) {
    uint64_t tot = 0;
    for (uint32_t w = 0; w < nwg; ++w)
      for (uint32_t kq = 0; kq < 4; ++kq) tot += hc[((size_t)w * 256 + q) * 4 + kq];
    std::printf("q %u sample bound %g slabs %llu\n", q, hb[q], (unsigned long long)tot);
  }
  std::printf("gate after int8 pass %u\n", hgate);
  CK(hipMemcpy(hs.data(), slabs, slots * 32, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ht.data(), tiles, slots * 4, hipMemcpyDeviceToHost));
  for (uint32_t q = 0; q < nq; ++q) {
    int mn = INT_MAX, mxall = INT_MIN;
    for (uint32_t w = 0; w < nwg; ++w)
      for (uint32_t kq = 0; kq < 4; ++kq) {
        const uint32_t c = hc[((size_t)w * 256 + q) * 4 + kq];
        for (uint32_t j = 0; j < c; ++j) {
          const size_t e = ((size_t)w * 256 + q) * cap + kq * (cap / 4) + j;
          int m = INT_MIN;
          for (int b = 0; b < 8; ++b) m = std::max(m, hs[e * 8 + b]);
          mn = std::min(mn, m);
          mxall = std::max(mxall, m);
        }
      }
    const double th = (hb[q] - hp[4 * q + 1] * hg[1] - (hp[4 * q + 2] + 2 * hp[4 * q + 3]) * hg[2]) /
                      hp[4 * q] - 1;
    int best = INT_MIN;
    for (uint32_t r = 0; r < n; ++r) {
      int dd = 0;
      for (uint32_t d = 0; d < dim; ++d) dd += (int)X8[(size_t)r * dim + d] * (int)Q8[(size_t)q * dim + d];
      best = std::max(best, dd);
    }
    std::printf("q %u host threshold %.1f; admitted slab maxima in [%d, %d]; best dot %d\n", q, th,
                mn, mxall, best);
  }
  CK(vsk::launch_select_q8(slabs, tiles, cnt, cmx, nwg, cap, nq, k, out, 0, dX, dQ, false, dim, par, glob, meta,
                           bound, dX8, dQ8, nullptr, n, 0));
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(&hgate, gate, 4, hipMemcpyDeviceToHost));
  std::vector<uint64_t> ho(nq * k);
  CK(hipMemcpy(ho.data(), out, nq * k * 8, hipMemcpyDeviceToHost));
  std::printf("gate after select %u\n", hgate);
  int bad_top = 0;
  for (uint32_t q = 0; q < nq; ++q) {
    std::vector<std::pair<double, uint32_t>> sc(n);
    for (uint32_t r = 0; r < n; ++r) {
      double ex = 0;
      for (uint32_t d = 0; d < dim; ++d)
        ex += (double)vs::bf16_to_f32(X[(size_t)r * dim + d]) * (double)vs::bf16_to_f32(Q[(size_t)q * dim + d]);
      sc[r] = {ex, r};
    }
    std::partial_sort(sc.begin(), sc.begin() + k, sc.end(),
                      [](const auto& a, const auto& b) { return a.first > b.first; });
    for (uint32_t j = 0; j < k; ++j) {
      const uint64_t key = ho[q * k + j];
      const uint32_t row = vs::key_row(key);
      const float s = vs::key_score(key);
      const bool ok = key && (row == sc[j].second || std::fabs(sc[j].first - s) < 1e-5 * std::fabs(s));
      if (!ok && bad_top++ < 10)
        std::printf("q %u rank %u: got row %u score %g, want row %u score %g\n", q, j, row, s,
                    sc[j].second, sc[j].first);
    }
  }
  std::printf("top-k mismatches: %d\n", bad_top);
  return (bad_q || bad_dot || bad_bound || checked == 0 || bad_top) ? 1 : 0;
}
