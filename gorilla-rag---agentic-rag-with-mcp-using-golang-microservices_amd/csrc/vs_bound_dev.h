// vs_bound_dev.h — the sample bound's per-query body (device side), shared by
// sample_bound_kernel (vs_kernels.hip) and the int8 path's fused bound +
// query-quantisation launch (vs_q8.hip, r04). Algorithm: see the comment
// above sample_bound_kernel in vs_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace vsk {

constexpr int kBoundThreads = 256;

__device__ __forceinline__ uint32_t ord_f32(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_f32(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

// int8 prefilter bounds (vs_q8.hip; r05 also the single-query scan on the
// int8 copy, vs_kernels.hip): sqrt of a non-negative fp64 sum, rounded up to
// float with a relative margin for the sum's own fp64 rounding (dim <= 2^11
// terms: far below 2^-30)
__device__ __forceinline__ float q8_norm_up(double s) {
  return __double2float_ru(sqrt(s) * (1.0 + 0x1p-30));
}
// sigma per unit of |x|: the fp32 evaluation error of any score of the scans
// or of a rescore (<= 2 dim u |q| |x| each, u = 2^-24) on both sides of a
// bound, and the float rounding of sqS * dot, m and the comparisons
__device__ __forceinline__ float q8_sigma(uint32_t dim, float q_norm_up) {
  return (float)((4.0 * dim + 64.0) * 0x1p-24 * (double)q_norm_up * (1.0 + 0x1p-20));
}

// One workgroup of kBoundThreads: bound[q] = the radix-select lower bound on
// the k-th largest of the m values at tmax + q * m (`passes` 8-bit digits).
__device__ __forceinline__ void sample_bound_block(const float* __restrict__ tmax, uint32_t m,
                                                   uint32_t k, float* __restrict__ bound,
                                                   int passes, uint32_t q) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t wsum[kBoundThreads / 64];
  __shared__ uint32_t pick, above;
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (m < k) {
    if (tid == 0) bound[q] = -INFINITY;
    return;
  }
  const float* v = tmax + (size_t)q * m;
  uint32_t prefix = 0, kk = k;  // the kk-th largest of the values matching prefix
#pragma unroll 1
  for (int pass = 0; pass < passes; ++pass) {
    const int shift = 24 - 8 * pass;
    const uint32_t hmask = pass == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
    hist[tid] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < m; i += kBoundThreads) {
      const uint32_t u = ord_f32(v[i]);
      if ((u & hmask) == prefix) atomicAdd(&hist[(u >> shift) & 255u], 1u);
    }
    __syncthreads();
    // inclusive scan over the digits in descending order (thread t: digit 255 - t)
    const uint32_t c = hist[255 - tid];
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    for (uint32_t j = 0; j < w; ++j) x += wsum[j];
    // exactly one digit has (count above) < kk <= (count above + its own)
    if (x >= kk && x - c < kk) pick = tid, above = x - c;
    __syncthreads();
    prefix |= (uint32_t)(255 - pick) << shift;
    kk -= above;
    __syncthreads();  // pick / above / wsum / hist are rewritten by the next pass
  }
  // the bucket of -inf starts below ord(-inf), in the negative-NaN codes
  if (tid == 0) bound[q] = prefix <= ord_f32(-INFINITY) ? -INFINITY : unord_f32(prefix);
}

}  // namespace vsk
