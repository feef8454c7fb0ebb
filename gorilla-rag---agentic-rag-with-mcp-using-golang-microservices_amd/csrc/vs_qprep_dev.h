// vs_qprep_dev.h — one query's preprocessing on one wave (device side), shared
// by query_prep_kernel (vs_kernels.hip) and the speculative path's fused
// preprocessing + int8-image launch (vs_q8.hip q8_prep_query_kernel, r06), so
// the two write the same bits.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "vs_common.h"

namespace vsk {

constexpr int kQPrepMax = 24;  // dim <= 64 * kQPrepMax = 1536

// Query i of `in` (fp32, dim <= 64 * kQPrepMax) on the calling wave. All of a
// lane's elements are loaded at once (one memory latency instead of dim/64
// dependent ones: 9 -> ~4 us per batch), the squared norm is summed in the
// store side's order (lane l: elements l, l+64, ... in sequence, then the same
// butterfly) and only for cosine, and each output is optional: qp = fp32
// (rounded to bf16 values when round_qp: what a bf16 scan multiplies), qb =
// bf16 copy; lf / lb: the same values as qp / qb, element d at [d] (the
// wave's own LDS copy).
__device__ __forceinline__ void query_prep_one(const float* __restrict__ in, uint32_t i,
                                               uint32_t dim, int cosine, int round_qp,
                                               float* __restrict__ qp, uint16_t* __restrict__ qb,
                                               int lane, float* lf = nullptr,
                                               uint16_t* lb = nullptr) {
  const float* x = in + (size_t)i * dim;
  float v[kQPrepMax];
#pragma unroll
  for (int j = 0; j < kQPrepMax; ++j) {
    const uint32_t d = (uint32_t)lane + 64u * (uint32_t)j;
    v[j] = d < dim ? x[d] : 0.f;
  }
  bool keep = true;
  double nrm = 1.0;
  if (cosine) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < kQPrepMax; ++j) {
      const double t = (double)v[j];
      s = s + t * t;  // zero padding adds exact zeros: same sum as the store side
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s = s + __shfl_xor(s, m, 64);
    keep = vs::cosine_keep(s);
    nrm = sqrt(s);
  }
#pragma unroll
  for (int j = 0; j < kQPrepMax; ++j) {
    const uint32_t d = (uint32_t)lane + 64u * (uint32_t)j;
    if (d >= dim) break;
    const float y = keep ? v[j] : (float)((double)v[j] / nrm);
    const uint16_t h = vs::f32_to_bf16(y);
    const float yp = round_qp ? vs::bf16_to_f32(h) : y;
    if (qp) qp[(size_t)i * dim + d] = yp;
    if (qb) qb[(size_t)i * dim + d] = h;
    if (lf) lf[d] = yp;
    if (lb) lb[d] = h;
  }
}

}  // namespace vsk
