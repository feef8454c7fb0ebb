// vs_q8.hip — store and query side of the int8 prefilter (r04; DESIGN.md §5
// "int8 prefilter", launchers declared in vs_kernels.h).
//
// A bf16 collection keeps an int8 copy x8 = clamp(rint(x / S), -127, 127)
// with one scale S per collection, and per 32-row tile two bounds rounded
// up: dt = max_r |x_r - S x8_r| and nt = max_r |x_r|. A query q (bf16) gets
// its own scale sq and the same pair |sq q8|, |q - sq q8|. Then, exactly,
//   q . x = sq S (q8 . x8) + sq q8 . (x - S x8) + (q - sq q8) . x,
// and Cauchy-Schwarz bounds the two error terms by |sq q8| dt + |q - sq q8| nt,
// so an exact int32 dot on v_mfma_i32_16x16x64_i8 brackets the fp32 score.
// Every norm is summed in fp64 and rounded up, so the brackets hold for the
// values the device stores, not just in exact arithmetic.
#include <climits>
#include <hip/hip_runtime.h>
#include <math.h>

#include "vs_bound_dev.h"
#include "vs_common.h"
#include "vs_kernels.h"
#include "vs_qprep_dev.h"
#include "vs_spec_dev.h"

namespace vsk {
namespace {

__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = v + __shfl_xor(v, m, 64);
  return v;
}
__device__ __forceinline__ float norm_up(double s) { return q8_norm_up(s); }  // vs_bound_dev.h
__device__ __forceinline__ void atomic_max_pos(float* p, float v) {
  // non-negative floats order as their bit patterns
  atomicMax((unsigned int*)p, __float_as_uint(v));
}

// max |x| over n bf16 values, 16 B per lane per step
__global__ __launch_bounds__(256) void q8_absmax_kernel(const uint4* __restrict__ X, uint64_t n16,
                                                        float* __restrict__ glob) {
  uint32_t m = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const uint4 v = X[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t lo = w[j] & 0x7FFFu, hi = (w[j] >> 16) & 0x7FFFu;
      m = lo > m ? lo : m;
      m = hi > m ? hi : m;
    }
  }
  // bf16 magnitude bits order as the values (NaN never stored: preprocess
  // output of finite input)
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) {
    const uint32_t o = __shfl_xor(m, s, 64);
    m = o > m ? o : m;
  }
  if ((threadIdx.x & 63) == 0 && m) atomic_max_pos(glob, vs::bf16_to_f32((uint16_t)m));
}

// max |x| over n fp32 values (fp32 collections, r04)
__global__ __launch_bounds__(256) void q8_absmax_f32_kernel(const uint4* __restrict__ X, uint64_t n4,
                                                            float* __restrict__ glob) {
  uint32_t m = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const uint4 v = X[i];
    const uint32_t w[4] = {v.x & 0x7FFFFFFFu, v.y & 0x7FFFFFFFu, v.z & 0x7FFFFFFFu, v.w & 0x7FFFFFFFu};
#pragma unroll
    for (int j = 0; j < 4; ++j) m = w[j] > m ? w[j] : m;
  }
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) {
    const uint32_t o = __shfl_xor(m, s, 64);
    m = o > m ? o : m;
  }
  if ((threadIdx.x & 63) == 0 && m) atomic_max_pos(glob, __uint_as_float(m));
}

// two consecutive elements of a bf16 (32-bit word) or fp32 (64-bit) row
template <bool F32>
__device__ __forceinline__ void load2(const void* X, uint64_t e, bool live, float& x0, float& x1) {
  if constexpr (F32) {
    const float2 v = live ? *(const float2*)((const float*)X + e) : float2{0.f, 0.f};
    x0 = v.x, x1 = v.y;
  } else {
    const uint32_t xv = live ? *(const uint32_t*)((const uint16_t*)X + e) : 0u;
    x0 = __uint_as_float(xv << 16), x1 = __uint_as_float(xv & 0xFFFF0000u);
  }
}

__global__ void q8_set_scale_kernel(float* glob) {
  const float a = glob[0];
  glob[3] = a > 0.f ? a / 127.f : 1.f;
}

// One wave per 32-row tile; lane l holds elements 2l, 2l + 1 (+128 j) of a row.
template <bool F32>
__global__ __launch_bounds__(256) void q8_quantize_kernel(
    const void* __restrict__ X, uint32_t n_rows, uint32_t dim,
    const uint32_t* __restrict__ tiles, uint32_t t0, uint32_t ntiles, int8_t* __restrict__ X8,
    float* __restrict__ meta, float* __restrict__ glob) {
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= ntiles) return;
  const int lane = threadIdx.x & 63;
  const uint32_t tile = tiles ? tiles[i] : t0 + i;
  const float S = glob[3];
  float dt = 0.f, nt = 0.f;
  for (uint32_t rr = 0; rr < 32; ++rr) {
    const uint64_t r = (uint64_t)tile * 32 + rr;
    const bool live = r < n_rows;
    double dd = 0.0, xx = 0.0;
    for (uint32_t d = 2 * lane; d < dim; d += 128) {
      float x0, x1;
      load2<F32>(X, r * dim + d, live, x0, x1);
      const float y0 = fminf(fmaxf(rintf(x0 / S), -127.f), 127.f);
      const float y1 = fminf(fmaxf(rintf(x1 / S), -127.f), 127.f);
      // S * y is exact in fp64 (24 x 7 bits), and so is x - S y (x: 24 bits)
      const double e0 = (double)x0 - (double)S * (double)y0;
      const double e1 = (double)x1 - (double)S * (double)y1;
      dd = dd + e0 * e0 + e1 * e1;
      xx = xx + (double)x0 * (double)x0 + (double)x1 * (double)x1;
      const uint16_t pk = (uint16_t)(uint8_t)(int8_t)(int)y0 | ((uint16_t)(uint8_t)(int8_t)(int)y1 << 8);
      *(uint16_t*)(X8 + r * dim + d) = pk;
    }
    if (!live) continue;
    dd = wave_sum_d(dd);
    xx = wave_sum_d(xx);
    dt = fmaxf(dt, norm_up(dd));
    nt = fmaxf(nt, norm_up(xx));
  }
  if (lane == 0) {
    meta[2 * (size_t)tile] = dt;
    meta[2 * (size_t)tile + 1] = nt;
    atomic_max_pos(glob + 1, dt);
    atomic_max_pos(glob + 2, nt);
  }
}

// A ratio a speculative batch may start from: set (> 0) and finite.
__device__ __forceinline__ bool ratio_set(float r) { return r > 0.f && r < 1e38f; }

// (r06) The speculative try's go / verdict words (vs_kernels.h Q8SpecK): one
// thread, before any launch of the batch reads them.
__device__ __forceinline__ void spec_decide(const float* __restrict__ ratio, Q8SpecK* __restrict__ sk,
                                            Q8SpecStat* __restrict__ stat, uint32_t* __restrict__ gate,
                                            bool force) {
  bool go = ratio_set(*ratio);
  if (go && !force) {
    // (the host reads the same verdict from its advice words and normally
    // enqueues no try at all while loose)
    go = __hip_atomic_load(&sk->loose, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
    // every kQ8SpecProbe-th try runs the sample path, which re-judges `loose`
    if (go) go = (atomicAdd(&sk->since, 1u) + 1u) % kQ8SpecProbe != 0u;
  }
  gate[kGateVerdict] = go ? 0u : 1u;
  gate[kGateGo] = go ? 1u : 0u;
  atomicAdd(go ? &stat->tries : &stat->skipped, 1ull);
}

// One wave per query (bf16 queries of a bf16 collection, or the fp32
// preprocessed queries of an fp32 one; with `src`, this wave's query read
// from there -- its LDS copy -- instead of from qb).
// (r05) With `ratio` (a collection's learned k-th score per unit |q|, DESIGN.md
// §5 "Speculative bound"), also bound[i] = ratio x |q| (-inf while the ratio
// is unset: the batch then stands down, spec_decide).
template <bool F32>
__device__ __forceinline__ void q8_query_block(uint32_t blk, const void* __restrict__ qb,
                                               uint32_t nq, uint32_t dim,
                                               const float* __restrict__ glob,
                                               int8_t* __restrict__ q8, float* __restrict__ q8par,
                                               uint32_t* __restrict__ gate,
                                               const float* __restrict__ ratio = nullptr,
                                               float* __restrict__ bound = nullptr,
                                               Q8SpecK* __restrict__ sk = nullptr,
                                               Q8SpecStat* __restrict__ stat = nullptr,
                                               bool force = false, const void* src = nullptr) {
  if (gate && blk == 0 && threadIdx.x == 0) {
    if (sk)
      spec_decide(ratio, sk, stat, gate, force);
    else
      gate[kGateVerdict] = 0u;
  }
  const uint32_t i = blk * 4 + (threadIdx.x >> 6);
  if (i >= nq) return;
  const int lane = threadIdx.x & 63;
  const uint64_t x = (uint64_t)i * dim;
  const void* qv = src ? src : qb;
  const uint64_t x_in = src ? 0 : x;
  float amax = 0.f;
  for (uint32_t d = 2 * lane; d < dim; d += 128) {
    float x0, x1;
    load2<F32>(qv, x_in + d, true, x0, x1);
    amax = fmaxf(amax, fmaxf(fabsf(x0), fabsf(x1)));
  }
  amax = wave_max_f(amax);
  const float sq = amax > 0.f ? amax / 127.f : 0.f;
  double aa = 0.0, cc = 0.0, nn = 0.0;
  for (uint32_t d = 2 * lane; d < dim; d += 128) {
    float x0, x1;
    load2<F32>(qv, x_in + d, true, x0, x1);
    const float y0 = sq > 0.f ? fminf(fmaxf(rintf(x0 / sq), -127.f), 127.f) : 0.f;
    const float y1 = sq > 0.f ? fminf(fmaxf(rintf(x1 / sq), -127.f), 127.f) : 0.f;
    const double s0 = (double)sq * (double)y0, s1 = (double)sq * (double)y1;
    const double e0 = (double)x0 - s0, e1 = (double)x1 - s1;
    aa = aa + s0 * s0 + s1 * s1;
    cc = cc + e0 * e0 + e1 * e1;
    nn = nn + (double)x0 * (double)x0 + (double)x1 * (double)x1;
    const uint16_t pk = (uint16_t)(uint8_t)(int8_t)(int)y0 | ((uint16_t)(uint8_t)(int8_t)(int)y1 << 8);
    *(uint16_t*)(q8 + (size_t)i * dim + d) = pk;
  }
  aa = wave_sum_d(aa);
  cc = wave_sum_d(cc);
  nn = wave_sum_d(nn);
  if (lane == 0) {
    // sigma covers, per unit of |x|: the fp32 evaluation error of an MFMA or
    // rescore score (<= 2 dim u |q| |x| each, u = 2^-24) on both sides of a
    // bound, and the float rounding of sqS * dot, m and the comparisons
    const float sigma = q8_sigma(dim, norm_up(nn));
    float* p = q8par + 4 * (size_t)i;
    p[0] = sq * glob[3];
    p[1] = norm_up(aa);
    p[2] = norm_up(cc);
    p[3] = sigma;
    if (bound) {
      const float r = *ratio;
      bound[i] = ratio_set(r) ? r * (float)sqrt(nn) : -INFINITY;
    }
  }
}

template <bool F32>
__global__ __launch_bounds__(256) void q8_query_kernel(const void* __restrict__ qb, uint32_t nq,
                                                       uint32_t dim, const float* __restrict__ glob,
                                                       int8_t* __restrict__ q8,
                                                       float* __restrict__ q8par,
                                                       uint32_t* __restrict__ gate,
                                                       const float* __restrict__ ratio,
                                                       float* __restrict__ bound,
                                                       Q8SpecK* __restrict__ sk,
                                                       Q8SpecStat* __restrict__ stat, uint32_t force) {
  q8_query_block<F32>(blockIdx.x, qb, nq, dim, glob, q8, q8par, gate, ratio, bound, sk, stat,
                      force != 0u);
}

// (r06) The speculative path's first launch: the queries' preprocessing
// (query_prep_kernel's, vs_qprep_dev.h, bit for bit) fused with their int8
// images and the speculative bound (q8_query_kernel's, reading each query
// from the wave's LDS copy instead of from global memory): one launch and one
// kernel boundary instead of two.
static_assert(64u * kQPrepMax == kQueryPrepFusedMaxDim, "the fused launch's dim limit");
template <bool F32>
__global__ __launch_bounds__(256) void q8_prep_query_kernel(
    const float* __restrict__ in, uint32_t nq, uint32_t dim, int cosine, int round_qp,
    float* __restrict__ qp, uint16_t* __restrict__ qbf, const float* __restrict__ glob,
    int8_t* __restrict__ q8, float* __restrict__ q8par, uint32_t* __restrict__ gate,
    const float* __restrict__ ratio, float* __restrict__ bound, Q8SpecK* __restrict__ sk,
    Q8SpecStat* __restrict__ stat, uint32_t force) {
  // a wave's query as the int8 image reads it: fp32 (F32) or bf16 values
  __shared__ __attribute__((aligned(16))) uint32_t lq[4][(F32 ? 64 : 32) * kQPrepMax];
  const int lane = threadIdx.x & 63;
  const uint32_t w = threadIdx.x >> 6, i = blockIdx.x * 4 + w;
  if (i < nq)
    query_prep_one(in, i, dim, cosine, round_qp, qp, qbf, lane, F32 ? (float*)lq[w] : nullptr,
                   F32 ? nullptr : (uint16_t*)lq[w]);
  __syncthreads();
  q8_query_block<F32>(blockIdx.x, F32 ? (const void*)qp : (const void*)qbf, nq, dim, glob, q8, q8par,
                      gate, ratio, bound, sk, stat, force != 0u, lq[w]);
}

// After a batch's select (one workgroup, thread q = query q): its k-th key's
// exact score s against the bound b it ran with. A speculative batch is exact
// iff s reaches b - sigma nmax for every query (every row the pass left out
// has U below that, so below s; rows the select left out are beaten by the
// quarter bound's k rows): otherwise the verdict word is raised and the batch
// re-runs on the sample path, gated on it (r05).
// (r06) What the batch teaches the next one: r05 lowered
// one running minimum with every verified query, so a single off-topic query
// pinned the bound of every later batch near zero until the next write. Now a
// verified (or sample-path) batch REPLACES the ratio with 0.97 x the
// (1 + n/64)-th smallest of its queries' s / |q| (s > 0): up to n/64 outliers
// a batch are ignored, and whatever a batch teaches lasts one batch. A failed
// check counts itself and starts a cool-down (back-off doubling to 64 batches
// over consecutive failures), so traffic whose every batch holds an outlier
// settles on the sample path instead of paying for two passes a batch.
// run_if: stand down unless *run_if.
__global__ __launch_bounds__(kMfmaQueries) void q8_verify_record_kernel(
    const uint64_t* __restrict__ keys, uint32_t nq, uint32_t k, SpecVerifyArgs a,
    const uint32_t* __restrict__ run_if) {
  if (run_if && *run_if == 0u) return;
  __shared__ float rq[kMfmaQueries];
  __shared__ float pick;
  const uint32_t q = threadIdx.x;
  float r = INFINITY, qn = 0.f, b = -INFINITY;
  bool ok = true;
  if (q < nq) {
    b = a.bound[q];
    spec_query_vals(keys[(size_t)q * k + k - 1], a.q8par[4 * (size_t)q + 3], b, a.glob[2], a.dim,
                    a.check != 0u, r, qn, ok);
  }
  spec_verify_core(q < nq, r, qn, b, ok, a, rq, &pick);  // vs_spec_dev.h
}

// Workgroups [0, nq_bound): the sample bound of query blockIdx.x; the rest:
// four queries' int8 image each (the two never share data).
template <bool F32>
__global__ __launch_bounds__(kBoundThreads) void sample_bound_q8_kernel(
    const float* __restrict__ tmax, uint32_t m, uint32_t k, float* __restrict__ bound, int passes,
    uint32_t nq_bound, const void* __restrict__ qb, uint32_t nq, uint32_t dim,
    const float* __restrict__ glob, int8_t* __restrict__ q8, float* __restrict__ q8par,
    uint32_t* __restrict__ gate, const uint32_t* __restrict__ run_if) {
  if (run_if && *run_if == 0u) return;  // (r05) the fallback behind a verified speculative batch
  if (blockIdx.x < nq_bound)
    sample_bound_block(tmax, m, k, bound, passes, blockIdx.x);
  else
    q8_query_block<F32>(blockIdx.x - nq_bound, qb, nq, dim, glob, q8, q8par, gate);
}

}  // namespace

hipError_t launch_q8_absmax(const void* X, bool f32, uint64_t n, float* glob, hipStream_t st) {
  if (n % 8) return hipErrorInvalidValue;  // whole rows of dim % 128 == 0
  const uint64_t n16 = f32 ? n / 4 : n / 8;  // 16-B loads
  uint64_t blocks = (n16 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks == 0) return hipSuccess;
  if (f32)
    hipLaunchKernelGGL(q8_absmax_f32_kernel, dim3((uint32_t)blocks), dim3(256), 0, st,
                       (const uint4*)X, n16, glob);
  else
    hipLaunchKernelGGL(q8_absmax_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, (const uint4*)X,
                       n16, glob);
  return hipGetLastError();
}

hipError_t launch_q8_set_scale(float* glob, hipStream_t st) {
  hipLaunchKernelGGL(q8_set_scale_kernel, dim3(1), dim3(1), 0, st, glob);
  return hipGetLastError();
}

hipError_t launch_q8_quantize(const void* X, bool f32, uint32_t n_rows, uint32_t dim,
                              const uint32_t* tiles, uint32_t t0, uint32_t ntiles, int8_t* X8,
                              float* meta, float* glob, hipStream_t st) {
  if (dim % 128 || dim == 0) return hipErrorInvalidValue;
  if (ntiles == 0) return hipSuccess;
  if (f32)
    hipLaunchKernelGGL(q8_quantize_kernel<true>, dim3((ntiles + 3) / 4), dim3(256), 0, st, X,
                       n_rows, dim, tiles, t0, ntiles, X8, meta, glob);
  else
    hipLaunchKernelGGL(q8_quantize_kernel<false>, dim3((ntiles + 3) / 4), dim3(256), 0, st, X,
                       n_rows, dim, tiles, t0, ntiles, X8, meta, glob);
  return hipGetLastError();
}

hipError_t launch_q8_query(const void* q, bool f32, uint32_t nq, uint32_t dim, const float* glob,
                           int8_t* q8, float* q8par, uint32_t* gate, hipStream_t st,
                           const float* ratio, float* bound, Q8SpecK* spec_k, Q8SpecStat* stat,
                           bool force) {
  if (dim % 128 || dim == 0 || (bound && !ratio) || (spec_k && (!ratio || !stat || !gate)))
    return hipErrorInvalidValue;
  if (nq == 0) return hipSuccess;
  if (f32)
    hipLaunchKernelGGL(q8_query_kernel<true>, dim3((nq + 3) / 4), dim3(256), 0, st, q, nq, dim,
                       glob, q8, q8par, gate, ratio, bound, spec_k, stat, force ? 1u : 0u);
  else
    hipLaunchKernelGGL(q8_query_kernel<false>, dim3((nq + 3) / 4), dim3(256), 0, st, q, nq, dim,
                       glob, q8, q8par, gate, ratio, bound, spec_k, stat, force ? 1u : 0u);
  return hipGetLastError();
}

hipError_t launch_q8_prep_query(const float* in, bool cosine, bool round_qp, float* qp,
                                uint16_t* qbf, bool f32, uint32_t nq, uint32_t dim,
                                const float* glob, int8_t* q8, float* q8par, uint32_t* gate,
                                hipStream_t st, const float* ratio, float* bound, Q8SpecK* spec_k,
                                Q8SpecStat* stat, bool force) {
  if (dim % 128 || dim == 0 || dim > 64u * kQPrepMax || !ratio || !bound || !spec_k || !stat ||
      !gate || (f32 ? !qp : !qbf))
    return hipErrorInvalidValue;
  if (nq == 0) return hipSuccess;
  if (f32)
    hipLaunchKernelGGL(q8_prep_query_kernel<true>, dim3((nq + 3) / 4), dim3(256), 0, st, in, nq, dim,
                       (int)cosine, (int)round_qp, qp, qbf, glob, q8, q8par, gate, ratio, bound,
                       spec_k, stat, force ? 1u : 0u);
  else
    hipLaunchKernelGGL(q8_prep_query_kernel<false>, dim3((nq + 3) / 4), dim3(256), 0, st, in, nq,
                       dim, (int)cosine, (int)round_qp, qp, qbf, glob, q8, q8par, gate, ratio,
                       bound, spec_k, stat, force ? 1u : 0u);
  return hipGetLastError();
}

hipError_t launch_q8_verify_record(const uint64_t* keys, uint32_t nq, uint32_t k, uint32_t dim,
                                   const float* bound, const float* q8par, const float* glob,
                                   bool check, uint32_t* gate, Q8SpecK* spec_k, Q8SpecStat* stat,
                                   uint32_t* advice, hipStream_t st, const uint32_t* run_if) {
  if (nq == 0 || nq > kMfmaQueries || k == 0 || !spec_k || !stat || (check && !gate))
    return hipErrorInvalidValue;
  const SpecVerifyArgs a{check ? 1u : 0u, dim, bound, q8par, glob, gate, spec_k, stat, advice,
                         nullptr, nullptr};
  hipLaunchKernelGGL(q8_verify_record_kernel, dim3(1), dim3(kMfmaQueries), 0, st, keys, nq, k, a,
                     run_if);
  return hipGetLastError();
}

hipError_t launch_sample_bound_q8(const float* tmax, uint32_t m, uint32_t nq_bound, uint32_t k,
                                  float* bound, const void* q, bool f32, uint32_t nq,
                                  uint32_t dim, const float* glob, int8_t* q8, float* q8par,
                                  uint32_t* gate, hipStream_t st, const uint32_t* run_if) {
  static_assert(kBoundThreads == 256, "four query waves per workgroup");
  if (dim % 128 || dim == 0 || nq == 0 || nq_bound == 0 || nq_bound > kMfmaQueries || k == 0 ||
      k > kMfmaMaxK)
    return hipErrorInvalidValue;
  const dim3 grid(nq_bound + (nq + 3) / 4);
  const int passes = sample_bound_passes();
  if (f32)
    hipLaunchKernelGGL(sample_bound_q8_kernel<true>, grid, dim3(kBoundThreads), 0, st, tmax, m, k,
                       bound, passes, nq_bound, q, nq, dim, glob, q8, q8par, gate, run_if);
  else
    hipLaunchKernelGGL(sample_bound_q8_kernel<false>, grid, dim3(kBoundThreads), 0, st, tmax, m, k,
                       bound, passes, nq_bound, q, nq, dim, glob, q8, q8par, gate, run_if);
  return hipGetLastError();
}

}  // namespace vsk
