// vs_spec_dev.h — the speculative bound's per-batch check and record (device
// side; DESIGN.md §5 "The speculative bound made robust"), shared by
// q8_verify_record_kernel (vs_q8.hip, its own launch) and the int8 select's
// last workgroup (vs_kernels.hip select_q8_kernel, r06: the same code at the
// end of the select, one launch fewer a batch).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "vs_common.h"
#include "vs_kernels.h"

namespace vsk {

// One query's part: its k-th key's exact score s against the bound b it ran
// with (check: s must reach b - sigma nmax), and its ratio r = s / |q| (+inf:
// none -- no k-th, s <= 0 or a zero query). |q| from sigma = (4 dim + 64)
// 2^-24 |q| (1 + 2^-20) (vs_bound_dev.h q8_sigma).
__device__ __forceinline__ void spec_query_vals(uint64_t key, float sig, float b, float nmax,
                                                uint32_t dim, bool check, float& r, float& qn,
                                                bool& ok) {
  const float s = key ? vs::key_score(key) : -INFINITY;
  ok = !check || (key != 0 && s >= b - sig * nmax);
  qn = (float)((double)sig / ((4.0 * dim + 64.0) * 0x1p-24 * (1.0 + 0x1p-20)));
  r = key != 0 && s > 0.f && qn > 0.f ? s / qn : INFINITY;
}

// The batch's verdict and what it teaches (every thread of the block calls
// it; thread t < nq holds query t's values, the others has = false). rq: LDS,
// kMfmaQueries floats; pick: LDS, one float.
// Check (a speculative batch): any failed query raises the verdict word (the
// sample path re-answers the batch, gated on it), counts a failure and starts
// a cool-down (back-off doubling to kQ8SpecMaxBackoff over consecutive
// failures, the length handed to the host's advice word); a verified batch
// clears the back-off. A verified or sample-path batch REPLACES the ratio with
// 0.97 x the (1 + n/64)-th smallest of its queries' ratios (up to n/64
// outliers ignored). Record (the sample path) also judges the bound loose when
// over a quarter of the queries' sample bounds sit above R |q|.
__device__ __forceinline__ void spec_verify_core(bool has, float r, float qn, float b, bool ok,
                                                 const SpecVerifyArgs& a, float* rq, float* pick) {
  const uint32_t t = threadIdx.x;
  if (!has) r = INFINITY, ok = true;
  if (t < kMfmaQueries) rq[t] = r;
  if (t == 0) *pick = INFINITY;
  const int nbad = __syncthreads_count(!ok);
  const int nvalid = __syncthreads_count(r < INFINITY);
  // the m-th smallest ratio (ties by query index), m = 1 + nvalid / 64
  if (t < kMfmaQueries && r < INFINITY) {
    const int m = 1 + nvalid / 64;
    int rank = 0;
    for (uint32_t j = 0; j < kMfmaQueries; ++j) {
      const float o = rq[j];
      rank += (o < r) || (o == r && j < t);
    }
    if (rank == m - 1) *pick = r;
  }
  __syncthreads();
  const float pk = *pick;
  const float R = 0.97f * pk;  // the ratio this batch teaches (+inf: none)
  // (sample path) queries whose sample bound the speculative bound R |q|
  // would fall under: each would admit more rows than its sample pass does
  const int nloose = __syncthreads_count(!a.check && r < INFINITY && R * qn < b);
  if (t != 0) return;
  Q8SpecK* sk = a.sk;
  if (a.check) {
    if (nbad) {
      a.gate[kGateVerdict] = 1u;
      atomicAdd(&a.stat->fails, 1ull);
      // the cool-down: the host runs the next `bo` batches of this k on the
      // sample path alone, counting them off its advice word
      const uint32_t bo = sk->backoff;
      sk->backoff = bo ? (2 * bo < kQ8SpecMaxBackoff ? 2 * bo : kQ8SpecMaxBackoff) : 1u;
      if (a.advice && bo)
        __hip_atomic_store(a.advice + kQ8SpecK, bo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;  // the sample path's record replaces the ratio
    }
    sk->backoff = 0u;
  }
  if (pk < INFINITY) sk->ratio = R;
  if (!a.check) {
    const uint32_t loose = pk < INFINITY && 4 * nloose > nvalid ? 1u : 0u;
    sk->loose = loose;
    sk->since = 0u;
    if (a.advice) __hip_atomic_store(a.advice, loose, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace vsk
