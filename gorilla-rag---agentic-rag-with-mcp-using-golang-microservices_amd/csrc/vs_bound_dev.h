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

// One 8-bit radix digit (r06): the digit of a complete 256-bin histogram
// (LDS, 16-B aligned) holding the kk-th largest value, and the count of
// values above that digit, worked out by every wave on its own -- lane l
// takes digits 255 - 4l .. 252 - 4l (descending), a wave prefix sum, a ballot
// -- so the pick needs no LDS round trip and no barrier after it (the form it
// replaced split the scan over 4 waves and shared the pick: 4 more barriers a
// pass). false: the histogram holds fewer than kk values.
__device__ __forceinline__ bool wave_digit_pick(const uint32_t* hist, uint32_t kk, uint32_t lane,
                                                uint32_t& dig, uint32_t& above) {
  const uint4 o = *(const uint4*)(hist + 252 - 4 * lane);
  const uint32_t s4 = o.x + o.y + o.z + o.w;
  uint32_t x = s4;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  const uint64_t bal = __ballot(x >= kk);
  if (bal == 0) return false;
  const int L = __builtin_ctzll(bal);
  const uint32_t ow = __builtin_amdgcn_readlane(o.w, L), oz = __builtin_amdgcn_readlane(o.z, L),
                 oy = __builtin_amdgcn_readlane(o.y, L);
  uint32_t a = __builtin_amdgcn_readlane(x - s4, L), g = 255u - 4u * (uint32_t)L;
  if (a + ow < kk) {
    a += ow, --g;
    if (a + oz < kk) {
      a += oz, --g;
      if (a + oy < kk) a += oy, --g;
    }
  }
  dig = g, above = a;
  return true;
}

constexpr int kBoundMaxPasses = 4;

// One workgroup of kBoundThreads: bound[q] = the radix-select lower bound on
// the k-th largest of the m values at tmax + q * m (`passes` <= 4 8-bit
// digits). One histogram a pass, zeroed up front: one barrier a pass (r06;
// five before).
__device__ __forceinline__ void sample_bound_block(const float* __restrict__ tmax, uint32_t m,
                                                   uint32_t k, float* __restrict__ bound,
                                                   int passes, uint32_t q) {
  __shared__ __attribute__((aligned(16))) uint32_t hist[kBoundMaxPasses][256];
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  if (m < k) {
    if (tid == 0) bound[q] = -INFINITY;
    return;
  }
  const float* v = tmax + (size_t)q * m;
  for (uint32_t i = tid; i < (uint32_t)(kBoundMaxPasses * 256); i += kBoundThreads)
    (&hist[0][0])[i] = 0;
  __syncthreads();
  uint32_t prefix = 0, kk = k;  // the kk-th largest of the values matching prefix
#pragma unroll 1
  for (int pass = 0; pass < passes; ++pass) {
    const int shift = 24 - 8 * pass;
    const uint32_t hmask = pass == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
    for (uint32_t i = tid; i < m; i += kBoundThreads) {
      const uint32_t u = ord_f32(v[i]);
      if ((u & hmask) == prefix) atomicAdd(&hist[pass][(u >> shift) & 255u], 1u);
    }
    __syncthreads();
    // m >= k values: some digit holds the kk-th (the prefix's bucket holds kk
    // or more by construction)
    uint32_t dig = 0, above = 0;
    wave_digit_pick(hist[pass], kk, lane, dig, above);
    prefix |= dig << shift;
    kk -= above;
  }
  // the bucket of -inf starts below ord(-inf), in the negative-NaN codes
  if (tid == 0) bound[q] = prefix <= ord_f32(-INFINITY) ? -INFINITY : unord_f32(prefix);
}

}  // namespace vsk
