// vs_kernels.hip — CDNA4 (gfx950) kernels of the exact top-k search engine.
//
// The reference's hot loop is Qdrant's exact scan behind Points.Search
// (rag/vector-service/main.go:249-254): score every stored row against the
// preprocessed query and keep the best `limit`. Here that loop is:
//   * gemv_topk_kernel  — one query, HBM-bound stream of the resident matrix
//                         (16-B coalesced loads, wave reduction, per-wave
//                         register top-k list), fp32 or bf16 rows;
//   * mfma_topk_kernel  — up to 256 queries per launch, bf16 / fp32 rows
//                         streamed once through an LDS ring by LDS-DMA,
//                         scores on v_mfma_f32_16x16x32_bf16 (fp32:
//                         16x16x4_f32) with the query block resident in
//                         registers; a sample pass bounds each query's k-th
//                         score and the main pass keeps only 8-row slabs
//                         that reach it (select_slab_kernel picks the top k);
//   * merge_keys_kernel — global top-k over per-workgroup / per-shard lists.
// Store side (upsert, Qdrant cosine preprocess) and the synthetic generator
// are here too. Numerics contract: include/vsearch.h and DESIGN.md.
#include <climits>
#include <cstdlib>
#include <cstring>
#include <hip/hip_runtime.h>
#include <math.h>

#include "vs_common.h"
#include "vs_bound_dev.h"
#include "vs_kernels.h"
#include "vs_qprep_dev.h"
#include "vs_spec_dev.h"

namespace vsk {

using vs::make_key;
using vs::key_score;

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(3))) volatile uint64_t lds_vu64_t;

// ---------------------------------------------------------------------------
// wave helpers (wave64)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}
// Wave sum on the VALU (no LDS-path shuffles): DPP xor-1 / xor-2 / half-row
// and row mirrors leave every lane of 16-lane row r holding the row sum S_r
// (symmetric pairs: bit-identical in all lanes), then (S_0 + S_1) + (S_2 +
// S_3) from four readlanes -- wave-uniform by construction. (The gfx950
// permlane16/32_swap builtins were miscompiled by this hipcc: the second
// result aliased the first; tools/test_dpp.hip.)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  const int b = __builtin_bit_cast(int, v);
  const float s0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0));
  const float s1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16));
  const float s2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32));
  const float s3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48));
  return (s0 + s1) + (s2 + s3);
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = v + __shfl_xor(v, m, 64);
  return v;
}
__device__ __forceinline__ long long wave_sum_i64(long long v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int ln) {
  uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, ln);
  uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), ln);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_up64(uint64_t v) {
  uint32_t lo = __shfl_up((unsigned)(uint32_t)v, 1, 64);
  uint32_t hi = __shfl_up((unsigned)(uint32_t)(v >> 32), 1, 64);
  return ((uint64_t)hi << 32) | lo;
}

// Sorted (descending) key list of up to 64*KPL entries distributed over the
// lanes of one wave: entry i*64 + lane lives in e[i] of that lane. All lanes
// call insert() with the same key (wave-uniform), so the list stays uniform.
template <int KPL>
struct WaveList {
  uint64_t e[KPL];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int i = 0; i < KPL; ++i) e[i] = 0;
  }
  __device__ __forceinline__ uint64_t kth(uint32_t k) const {
    const uint32_t idx = k - 1, blk = idx >> 6;
    uint64_t v = 0;
#pragma unroll
    for (int i = 0; i < KPL; ++i)
      if ((uint32_t)i == blk) v = e[i];
    return readlane64(v, (int)(idx & 63));
  }
  __device__ __forceinline__ void insert(uint64_t x, uint32_t k, int lane) {
    uint32_t pos = 0;
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      const bool gt = ((uint32_t)(i * 64 + lane) < k) && (e[i] > x);
      pos += (uint32_t)__popcll(__ballot(gt));
    }
    uint64_t carry = 0;
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      uint64_t up = shfl_up64(e[i]);
      const uint64_t last = readlane64(e[i], 63);
      if (lane == 0) up = carry;
      carry = last;
      const uint32_t idx = (uint32_t)(i * 64 + lane);
      const uint64_t nv = idx < pos ? e[i] : (idx == pos ? x : up);
      e[i] = idx < k ? nv : 0;
    }
  }
};

// ---------------------------------------------------------------------------
// store side: Qdrant cosine preprocess + dtype conversion
// ---------------------------------------------------------------------------
// One wave per vector. The squared norm is accumulated in fp64 in a fixed
// order (lane l sums elements l, l+64, ... sequentially; then an xor
// butterfly), so the result is bit-reproducible and the oracle restates it.
template <bool BF16>
__global__ __launch_bounds__(256) void preprocess_kernel(
    const float* __restrict__ in, uint32_t n, uint32_t dim, int cosine,
    void* __restrict__ dst, const uint64_t* __restrict__ dst_rows, uint64_t dst0,
    uint16_t* __restrict__ also_bf16) {
  const int lane = threadIdx.x & 63;
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const float* x = in + (size_t)i * dim;
  double s = 0.0;
  for (uint32_t d = lane; d < dim; d += 64) {
    const double v = (double)x[d];
    s = s + v * v;
  }
  s = wave_sum_f64(s);
  const bool keep = !cosine || vs::cosine_keep(s);
  const double nrm = sqrt(s);
  const uint64_t row = dst_rows ? dst_rows[i] : dst0 + i;
  for (uint32_t d = lane; d < dim; d += 64) {
    const float v = x[d];
    const float y = keep ? v : (float)((double)v / nrm);
    if (BF16)
      ((uint16_t*)dst)[row * dim + d] = vs::f32_to_bf16(y);
    else
      ((float*)dst)[row * dim + d] = y;
    if (also_bf16) also_bf16[row * dim + d] = vs::f32_to_bf16(y);
  }
}

// Query side (search): one wave per query, dim <= 64 * kQPrepMax
// (vs_qprep_dev.h query_prep_one).
__global__ __launch_bounds__(256) void query_prep_kernel(const float* __restrict__ in, uint32_t n,
                                                         uint32_t dim, int cosine, int round_qp,
                                                         float* __restrict__ qp,
                                                         uint16_t* __restrict__ qb) {
  const int lane = threadIdx.x & 63;
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  query_prep_one(in, i, dim, cosine, round_qp, qp, qb, lane);
}

hipError_t launch_query_prep(const float* in, uint32_t n, uint32_t dim, bool cosine,
                             bool round_qp, float* qp, uint16_t* qb, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (dim > 64u * kQPrepMax) {  // wide vectors: the store side's loop kernel
    hipError_t e = launch_preprocess(in, n, dim, cosine, false, qp, nullptr, 0, st, qb);
    if (e != hipSuccess || !round_qp || !qp) return e;
    return launch_round_bf16(qp, (uint64_t)n * dim, qp, st);
  }
  hipLaunchKernelGGL(query_prep_kernel, dim3((n + 3) / 4), dim3(256), 0, st, in, n, dim,
                     (int)cosine, (int)round_qp, qp, qb);
  return hipGetLastError();
}

hipError_t launch_preprocess(const float* in, uint32_t n, uint32_t dim,
                             bool cosine, bool bf16, void* dst,
                             const uint64_t* dst_rows, uint64_t dst0,
                             hipStream_t st, uint16_t* also_bf16) {
  if (n == 0) return hipSuccess;
  dim3 grid((n + 3) / 4), block(256);
  if (bf16)
    hipLaunchKernelGGL(preprocess_kernel<true>, grid, block, 0, st, in, n, dim,
                       (int)cosine, dst, dst_rows, dst0, also_bf16);
  else
    hipLaunchKernelGGL(preprocess_kernel<false>, grid, block, 0, st, in, n, dim,
                       (int)cosine, dst, dst_rows, dst0, also_bf16);
  return hipGetLastError();
}

// Snapshot checksum: HBM-bound streaming reduction, 16-B loads, one 64-bit
// atomic per wave. Algorithmic bytes = nbytes.
typedef unsigned u32x4_ck __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void checksum_kernel(const u32x4_ck* __restrict__ p,
                                                       uint64_t npairs, uint64_t nbytes,
                                                       uint64_t* __restrict__ out) {
  uint64_t s = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < npairs; j += stride) {
    const u32x4_ck v = __builtin_nontemporal_load(p + j);
    s += vs::snap_word(((uint64_t)v.y << 32) | v.x, 2 * j);
    s += vs::snap_word(((uint64_t)v.w << 32) | v.z, 2 * j + 1);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // tail: < 16 bytes, words zero-padded
    const unsigned char* b = (const unsigned char*)p;
    for (uint64_t w = 2 * npairs; w * 8 < nbytes; ++w) {
      uint64_t x = 0;
      for (int i = 0; i < 8 && w * 8 + i < nbytes; ++i) x |= (uint64_t)b[w * 8 + i] << (8 * i);
      s += vs::snap_word(x, w);
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if ((threadIdx.x & 63) == 0 && s) atomicAdd((unsigned long long*)out, (unsigned long long)s);
}

// The same sum over the rows of one shard of a row-striped collection
// (global row = local * stride + offset; row_bytes % 8 == 0, so a row is a
// whole number of words): word w of local row l carries the global word
// index (l * stride + offset) * row_bytes / 8 + w. Summing the shards' sums
// gives the checksum of the collection in global row order.
__global__ __launch_bounds__(256) void checksum_rows_kernel(const uint64_t* __restrict__ p,
                                                            uint64_t nwords, uint32_t wpr,
                                                            uint64_t stride, uint64_t offset,
                                                            uint64_t* __restrict__ out) {
  uint64_t s = 0;
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nwords; j += step) {
    const uint64_t l = j / wpr, w = j - l * wpr;
    s += vs::snap_word(__builtin_nontemporal_load(p + j), (l * stride + offset) * wpr + w);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if ((threadIdx.x & 63) == 0 && s) atomicAdd((unsigned long long*)out, (unsigned long long)s);
}

hipError_t launch_checksum_rows(const void* p, uint64_t rows, uint32_t row_bytes, uint64_t stride,
                                uint64_t offset, uint64_t* d_out, hipStream_t st) {
  hipError_t e = hipMemsetAsync(d_out, 0, 8, st);
  if (e != hipSuccess || rows == 0) return e;
  if ((uintptr_t)p % 8 || row_bytes % 8) return hipErrorInvalidValue;
  const uint64_t nwords = rows * (row_bytes / 8);
  uint64_t blocks = (nwords + 255) / 256;
  const uint64_t cap = (uint64_t)device_cu_count() * 16;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(checksum_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     (const uint64_t*)p, nwords, row_bytes / 8, stride, offset, d_out);
  return hipGetLastError();
}

// Shard keys (local rows) -> global rows of a row-striped collection:
// global = base + local * stride + offset. Order-preserving within a shard
// (local row order = global row order), so a shard's sorted list stays
// sorted and ties keep the row-ascending rule. 0 (empty) stays 0.
__global__ void remap_keys_kernel(uint64_t* __restrict__ keys, uint64_t n, uint32_t stride,
                                  uint32_t offset, uint32_t base) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t key = keys[i];
  if (key == 0) return;
  const uint32_t local = vs::key_row(key);
  keys[i] = (key & 0xFFFFFFFF00000000ull) | (uint32_t)(0xFFFFFFFFu - (base + local * stride + offset));
}

hipError_t launch_remap_keys(uint64_t* keys, uint64_t n, uint32_t stride, uint32_t offset,
                             uint32_t base, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(remap_keys_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, keys,
                     n, stride, offset, base);
  return hipGetLastError();
}

hipError_t launch_checksum(const void* p, uint64_t nbytes, uint64_t* d_out, hipStream_t st) {
  hipError_t e = hipMemsetAsync(d_out, 0, 8, st);
  if (e != hipSuccess || nbytes == 0) return e;
  if ((uintptr_t)p % 16) return hipErrorInvalidValue;
  const uint64_t npairs = nbytes / 16;
  uint64_t blocks = (npairs + 255) / 256;
  const uint64_t cap = (uint64_t)device_cu_count() * 16;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(checksum_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const u32x4_ck*)p,
                     npairs, nbytes, d_out);
  return hipGetLastError();
}

// Synthetic unit rows: x_d = m_d / sqrt(sum m^2) with m_d the Irwin-Hall
// integers of vs::gen_int; the integer sum is exact and order-free, the
// division and sqrt are correctly rounded fp64 ops, so host and device agree.
template <bool BF16>
__global__ __launch_bounds__(256) void generate_kernel(uint64_t seed, uint64_t grow0,
                                                       uint64_t gstride, uint64_t n, uint32_t dim,
                                                       void* __restrict__ dst,
                                                       uint64_t dst0) {
  const int lane = threadIdx.x & 63;
  const uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const uint64_t rk = vs::gen_row_key(seed, grow0 + i * gstride);
  long long s = 0;
  for (uint32_t d = lane; d < dim; d += 64) {
    const long long m = vs::gen_int(rk, d);
    s += m * m;
  }
  s = wave_sum_i64(s);
  const double nrm = sqrt((double)s);
  const uint64_t row = dst0 + i;
  for (uint32_t d = lane; d < dim; d += 64) {
    const int32_t m = vs::gen_int(rk, d);
    const float y = s > 0 ? (float)((double)m / nrm) : 0.0f;
    if (BF16)
      ((uint16_t*)dst)[row * dim + d] = vs::f32_to_bf16(y);
    else
      ((float*)dst)[row * dim + d] = y;
  }
}

hipError_t launch_generate(uint64_t seed, uint64_t grow0, uint64_t n,
                           uint32_t dim, bool bf16, void* dst, uint64_t dst0,
                           hipStream_t st, uint64_t gstride) {
  if (n == 0) return hipSuccess;
  const uint64_t kChunk = 1ull << 24;  // keep gridDim.x well below 2^31
  for (uint64_t o = 0; o < n; o += kChunk) {
    const uint64_t m = (n - o < kChunk) ? n - o : kChunk;
    dim3 grid((unsigned)((m + 3) / 4)), block(256);
    if (bf16)
      hipLaunchKernelGGL(generate_kernel<true>, grid, block, 0, st, seed, grow0 + o * gstride,
                         gstride, m, dim, dst, dst0 + o);
    else
      hipLaunchKernelGGL(generate_kernel<false>, grid, block, 0, st, seed, grow0 + o * gstride,
                         gstride, m, dim, dst, dst0 + o);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

__global__ void to_bf16_kernel(const float* __restrict__ in, uint64_t n,
                               uint16_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = vs::f32_to_bf16(in[i]);
}
__global__ void round_bf16_kernel(const float* __restrict__ in, uint64_t n,
                                  float* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = vs::bf16_to_f32(vs::f32_to_bf16(in[i]));
}
hipError_t launch_to_bf16(const float* in, uint64_t n, uint16_t* out, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(to_bf16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     in, n, out);
  return hipGetLastError();
}
hipError_t launch_round_bf16(const float* in, uint64_t n, float* out, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(round_bf16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     st, in, n, out);
  return hipGetLastError();
}

// merge of sorted key lists (merge_query, defined with merge_keys_kernel
// below; the one-launch GEMV's last workgroup runs it too)
constexpr int kMergeThreads = 512;
constexpr int kMergeCap = 4096;
constexpr int kMergeHeld = 16;  // fast path: keys per thread held in registers
__device__ __forceinline__ void merge_query(const uint64_t* __restrict__ lists, uint32_t L,
                                            uint64_t lstride, uint64_t qstride, uint32_t kin,
                                            uint32_t k, uint32_t q, uint64_t* __restrict__ out,
                                            uint64_t* buf, uint64_t* red, uint32_t& cnt,
                                            bool tourney);

// ---------------------------------------------------------------------------
// single-query scan (GEMV) + per-wave top-k
// ---------------------------------------------------------------------------
constexpr int kGemvThreads = 512;
constexpr int kGemvWaves = kGemvThreads / 64;
static_assert(kGemvThreads == kMergeThreads, "the one-launch GEMV merges in its last workgroup");

// Wave 0's query preprocessing into LDS, as query_prep_kernel does it (the
// same fp64 norm in the same order, so the same bits): prep bit 0 = cosine
// normalise, bit 1 = round to bf16 values. The caller syncs.
template <int D>
__device__ __forceinline__ void prep_query_wave(const float* __restrict__ q, int prep, float* qs,
                                                int lane) {
  constexpr int PJ = D / 64;
  float v[PJ];
#pragma unroll
  for (int j = 0; j < PJ; ++j) v[j] = q[lane + 64 * j];
  bool keep = true;
  double nrm = 1.0;
  if (prep & 1) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < PJ; ++j) {
      const double t = (double)v[j];
      s = s + t * t;
    }
    s = wave_sum_f64(s);
    keep = vs::cosine_keep(s);
    nrm = sqrt(s);
  }
#pragma unroll
  for (int j = 0; j < PJ; ++j) {
    const float y = keep ? v[j] : (float)((double)v[j] / nrm);
    qs[lane + 64 * j] = (prep & 2) ? vs::bf16_to_f32(vs::f32_to_bf16(y)) : y;
  }
}

constexpr int cgcd(int a, int b) { return b == 0 ? a : cgcd(b, a % b); }
// non-temporal loads: 75.5% -> 81-86% of 8 TB/s on 10M x 768 bf16 and
// 1M x 768 fp32 (tools/ablate_gemv.hip). VAR 2 (DPP wave
// sum) measured within noise of the shuffle sum.
constexpr int kGemvVar = 1 | 8;  // non-temporal loads, interleaved wave steps
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

// Payload filter pre-mask: bit r of allow[] (local row r)
// admits the row; a null bitmap admits every row. `r` is wave-uniform, so the
// word comes through the scalar cache (one 64-row word serves 64 rows).
__device__ __forceinline__ bool row_allowed(const uint64_t* __restrict__ allow, uint32_t r) {
  return !allow || ((allow[r >> 6] >> (r & 63)) & 1u);
}

// Rows of D elements are cut into 16-byte chunks; one wave covers RB whole
// rows per step with J chunks per lane (RB*CPR == 64*J), so every load is a
// fully coalesced 1 KiB wave-instruction and each lane's query slice is
// loop-invariant (kept in registers).
template <int D, bool BF16>
struct GemvShape {
  static constexpr int EPC = BF16 ? 8 : 4;  // elements per 16-B chunk
  static constexpr int CPR = D / EPC;       // chunks per row
  static constexpr int RB = 64 / cgcd(CPR, 64);
  static constexpr int J = RB * CPR / 64;
  static constexpr size_t RBYTES = (size_t)D * (BF16 ? 2 : 4);
  static_assert(D % EPC == 0, "row must be a whole number of 16-B chunks");
};

template <bool BF16>
__device__ __forceinline__ float chunk_dot(const uint4& c, const float* qv) {
  if constexpr (BF16) {
    const uint32_t w[4] = {c.x, c.y, c.z, c.w};
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc = fmaf(__builtin_bit_cast(float, w[t] << 16), qv[2 * t], acc);
      acc = fmaf(__builtin_bit_cast(float, w[t] & 0xFFFF0000u), qv[2 * t + 1], acc);
    }
    return acc;
  } else {
    float acc = __builtin_bit_cast(float, c.x) * qv[0];
    acc = fmaf(__builtin_bit_cast(float, c.y), qv[1], acc);
    acc = fmaf(__builtin_bit_cast(float, c.z), qv[2], acc);
    acc = fmaf(__builtin_bit_cast(float, c.w), qv[3], acc);
    return acc;
  }
}

// After the scan each wave holds its list; KPL <= 2 lists (k <= 128) are
// merged across the workgroup in LDS (one list per workgroup), larger ones
// are written per wave. r02: at k = 100 the per-wave lists (8 per workgroup,
// 6144 per scan) made the merge kernel's work 8x larger than the scan's own
// merge here: 0.9 ms of a 3.2 ms single-query step at 10M rows.
template <int KPL>
__device__ __forceinline__ void gemv_emit(WaveList<KPL>& L, uint64_t theta, uint32_t k,
                                          int lane, int w, uint64_t* __restrict__ out) {
  (void)theta;
  if constexpr (KPL <= 2) {
    // r03: by rank, not by serial inserts. Each wave list is sorted, distinct
    // (distinct rows) and 0 past its keys, so a key's place in the
    // workgroup's list is its index in its own list plus, for each other
    // wave, the number of that wave's keys above it (a binary search over
    // sm[ow][0, k)); every lane places its keys at once. The serial form had
    // wave 0 insert the other 7 lists one key at a time: at k = 100 over 33
    // rows per wave, 231 dependent inserts at the end of every workgroup.
    __shared__ uint64_t sm[kGemvWaves][64 * KPL];
    __shared__ uint32_t nzw[kGemvWaves];
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      sm[w][i * 64 + lane] = L.e[i];
      nz += (uint32_t)__popcll(__ballot(L.e[i] != 0));
    }
    if (lane == 0) nzw[w] = nz;
    __syncthreads();
    uint32_t tot = 0;
#pragma unroll
    for (int ow = 0; ow < kGemvWaves; ++ow) tot += nzw[ow];
    uint32_t top = 1;  // highest power of two <= k
    while (top * 2 <= k) top *= 2;
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      const uint32_t e = (uint32_t)(i * 64 + lane);
      const uint64_t x = L.e[i];
      if (e < k && x != 0) {
        uint32_t r = e;
#pragma unroll
        for (int ow = 0; ow < kGemvWaves; ++ow) {
          if (ow == w) continue;
          uint32_t pos = 0;  // entries of sm[ow][0, k) above x
          for (uint32_t st = top; st > 0; st >>= 1)
            if (pos + st <= k && sm[ow][pos + st - 1] > x) pos += st;
          r += pos;
        }
        if (r < k) out[(size_t)blockIdx.x * k + r] = x;
      }
    }
    for (uint32_t r = tot + threadIdx.x; r < k; r += kGemvThreads) out[(size_t)blockIdx.x * k + r] = 0;
  } else {
    const size_t li = (size_t)blockIdx.x * kGemvWaves + w;
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      const uint32_t idx = (uint32_t)(i * 64 + lane);
      if (idx < k) out[li * k + idx] = L.e[i];
    }
  }
}

// VAR (ablation knobs, tools/ablate_gemv.hip): 1 = non-temporal loads,
// 2 = DPP/permlane wave sum, 4 = loads two steps ahead instead of one.
// GATHER: the scan walks positions [0, n_rows) of the compacted row list
// rows[] (a selective filter, compact_rows_kernel) instead of the rows
// themselves; each gathered row is still one contiguous, coalesced read, and
// the list entries are fetched one step ahead of the row data.
// KPL == 0 (large k, vs_kernels.h launch_gemv_scores): no list; every row's
// score leaves as its order-preserving 32-bit image (the key's high word, 0
// for a masked row) in sc[row], and the top 11 bits of each unmasked image
// are counted into hist[2048] (the first digit of the radix select).
// After a workgroup's stores to mapped host memory: every storing wave drains
// them, the workgroup meets, one lane releases at system scope and stores
// `seq` to *flag (the host spins on it, then reads the stores).
__device__ __forceinline__ void publish_host(uint64_t* flag, uint64_t seq) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ONE (r03, one query, KPL <= 2, no gather): `q` is the RAW query, which
// wave 0 of every workgroup preprocesses into LDS (prep bits as
// query_prep_kernel), `out` receives the per-workgroup lists, and the last
// workgroup to finish (an agent-scope counter) merges them with merge_query
// into `dst` -- then, with `flag`, publishes `seq` there for the host. One
// launch instead of query prep + scan + merge.
template <int KPL>
__device__ __forceinline__ void gemv_one_finish(const uint64_t* lists, uint32_t k,
                                                uint32_t* counter, uint64_t* dst,
                                                uint64_t* flag, uint64_t seq) {
  __shared__ uint64_t buf[kMergeCap];
  __shared__ uint64_t red[kMergeThreads / 64];
  __shared__ uint32_t cnt;
  __shared__ int last;
  // hand-off (MI355X_MICROARCH.md, valid producer / consumer forms): every
  // storing wave drains its list stores, the workgroup meets, ONE lane
  // releases at agent scope and adds to the counter; the last adder acquires
  // once, then the whole workgroup reads with plain loads. (A __threadfence()
  // per thread -- an L2 write-back and an L1 invalidate per wave in every
  // workgroup -- made a 20k-row search 3x slower.)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t prev =
        __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == gridDim.x - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  // the sample-bound path only (a constant: the tournament's registers would
  // raise the scan's VGPR count)
  merge_query(lists, gridDim.x, k, 0, k, k, 0, dst, buf, red, cnt, false);
  if (threadIdx.x == 0) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (flag) publish_host(flag, seq);
}

template <int D, bool BF16, int KPL, bool GATHER, int VAR, bool ONE>
__device__ __forceinline__ void gemv_topk_body(
    const void* __restrict__ Xv, uint32_t n_rows, uint32_t row_base,
    const float* __restrict__ q, const uint64_t* __restrict__ allow, uint32_t k,
    uint32_t rows_per_wave, uint64_t* __restrict__ out, const uint32_t* __restrict__ rows,
    uint32_t* __restrict__ hist, int prep, uint32_t* counter, uint64_t* dst, uint64_t* flag,
    uint64_t seq) {
  static_assert(!ONE || (KPL >= 1 && KPL <= 2 && !GATHER), "one-launch: list scans, no gather");
  using S = GemvShape<D, BF16>;
  constexpr bool kScores = KPL == 0;
  __shared__ uint32_t lhist[kScores ? kRselBins : 1];
  if constexpr (kScores) {
    for (int i = threadIdx.x; i < kRselBins; i += kGemvThreads) lhist[i] = 0;
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t gw = (uint64_t)blockIdx.x * kGemvWaves + w;
  // VAR 8: waves interleave their RB-row steps over the whole range (wave gw
  // reads steps gw, gw + waves, ...) instead of each streaming a contiguous
  // slice: all waves then work inside a few MB of the corpus at a time, so
  // the address translations they need stay cached (6144 slices of a 154 GB
  // corpus ran at 79% of HBM peak against 84% for 15 GB).
  constexpr bool kIlv = (VAR & 8) != 0;
  const uint32_t nw = gridDim.x * kGemvWaves;
  const uint32_t stride = kIlv ? nw * S::RB : S::RB;
  const uint64_t lo64 = kIlv ? gw * S::RB : gw * rows_per_wave;
  const uint32_t lo = lo64 < n_rows ? (uint32_t)lo64 : n_rows;
  const uint32_t hi = kIlv ? n_rows
                           : ((uint64_t)lo + rows_per_wave < n_rows ? lo + rows_per_wave : n_rows);

  int rowsel[S::J];
  int coff[S::J];  // chunk index within its row
#pragma unroll
  for (int j = 0; j < S::J; ++j) {
    const int c = lane + 64 * j;
    rowsel[j] = (S::RB == 1) ? 0 : c / S::CPR;
    coff[j] = c % S::CPR;
  }

  WaveList<kScores ? 1 : KPL> L;
  L.init();
  uint64_t theta = 0;
  const char* X = (const char*)Xv;
  // score mode: lane i of (obuf, rbuf) holds the i-th buffered row's image
  // and row number; nbuf rows are buffered (wave-uniform)
  uint32_t obuf = 0, rbuf = 0;
  int nbuf = 0;
  auto flush_scores = [&]() {
    if (lane < nbuf) {
      ((uint32_t*)out)[rbuf] = obuf;
      if (obuf) atomicAdd(&lhist[obuf >> (32 - kRselBits0)], 1u);
    }
    nbuf = 0;
  };
  (void)flush_scores;

  constexpr bool kNT = (VAR & 1) != 0, kDpp = (VAR & 2) != 0;
  constexpr int DEPTH = (VAR & 4) ? 2 : 1;
  uint4 buf[DEPTH + 1][S::J];
  uint32_t ixn[S::J];  // GATHER: rows of the next position to load
  auto fetch_ix = [&](uint32_t r0) {
#pragma unroll
    for (int j = 0; j < S::J; ++j) {
      const uint32_t pos = r0 + rowsel[j];
      ixn[j] = rows[pos < hi ? pos : hi - 1];
    }
  };
  auto load = [&](uint4* dst, uint32_t r0) {
#pragma unroll
    for (int j = 0; j < S::J; ++j) {
      uint32_t row;
      if constexpr (GATHER) {
        row = ixn[j];
      } else {
        row = r0 + rowsel[j];
        row = row < hi ? row : hi - 1;
      }
      const char* p = X + (size_t)row * S::RBYTES + (size_t)coff[j] * 16;
      if constexpr (kNT) {
        const u32x4_t v = __builtin_nontemporal_load((const u32x4_t*)p);
        dst[j] = uint4{v[0], v[1], v[2], v[3]};
      } else {
        dst[j] = *(const uint4*)p;
      }
    }
  };
  // the first rows' loads go out before the query is read (r03: in the
  // one-launch form, before wave 0's query preprocessing and its barrier),
  // except where holding them across the preprocessing would take the
  // one-launch kernel past 80 VGPRs (3 workgroups per CU): 4 chunks per lane
  auto prologue = [&]() {
    if (lo < hi) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        const uint32_t r0 = lo + d * stride;
        if constexpr (GATHER) fetch_ix(r0 < hi ? r0 : lo);
        load(buf[d], r0 < hi ? r0 : lo);
      }
      if constexpr (GATHER) fetch_ix(lo + DEPTH * stride);
    }
  };
  constexpr bool kEarly = !ONE || S::J <= 3;
  if constexpr (kEarly) prologue();
  float qv[S::J][S::EPC];
  const float* qsrc = q;
  if constexpr (ONE) {
    __shared__ float qs[D];
    if (w == 0) prep_query_wave<D>(q, prep, qs, lane);
    __syncthreads();
    qsrc = qs;
  }
#pragma unroll
  for (int j = 0; j < S::J; ++j)
#pragma unroll
    for (int e = 0; e < S::EPC; ++e) qv[j][e] = qsrc[coff[j] * S::EPC + e];
  if constexpr (!kEarly) prologue();
  if (lo < hi) {
    for (uint32_t r = lo; r < hi; r += stride) {
      const uint32_t rn = r + DEPTH * stride;
      load(buf[DEPTH], rn < hi ? rn : r);
      if constexpr (GATHER) fetch_ix(rn + stride);
      float p[S::RB];
#pragma unroll
      for (int b = 0; b < S::RB; ++b) p[b] = 0.f;
#pragma unroll
      for (int j = 0; j < S::J; ++j) {
        const float d = chunk_dot<BF16>(buf[0][j], qv[j]);
        if constexpr (S::RB == 1) {
          p[0] += d;
        } else {
#pragma unroll
          for (int b = 0; b < S::RB; ++b) p[b] += (rowsel[j] == b) ? d : 0.f;
        }
      }
#pragma unroll
      for (int b = 0; b < S::RB; ++b) {
        const float s = kDpp ? wave_sum_dpp(p[b]) : wave_sum(p[b]);
        const uint32_t row = r + b;
        if constexpr (kScores) {
          // every lane holds every sum: the wave-uniform image goes into lane
          // `nbuf` of a 64-row buffer, written out (one store and one LDS
          // histogram add per 64 rows) when full
          if (row < hi) {
            const uint32_t o = row_allowed(allow, row) ? (uint32_t)(make_key(s, 0) >> 32) : 0u;
            obuf = lane == nbuf ? o : obuf;
            rbuf = lane == nbuf ? row : rbuf;
            ++nbuf;
          }
        } else if (row < hi && (GATHER || row_allowed(allow, row))) {
          const uint64_t key = make_key(s, row_base + (GATHER ? rows[row] : row));
          if (key > theta) {
            L.insert(key, k, lane);
            theta = L.kth(k);
          }
        }
      }
      if constexpr (kScores) {
        if (nbuf > 64 - S::RB) flush_scores();
      }
#pragma unroll
      for (int d = 0; d < DEPTH; ++d)
#pragma unroll
        for (int j = 0; j < S::J; ++j) buf[d][j] = buf[d + 1][j];
    }
  }
  if constexpr (kScores) {
    flush_scores();
    __syncthreads();
    for (int i = threadIdx.x; i < kRselBins; i += kGemvThreads)
      if (lhist[i]) atomicAdd(&hist[i], lhist[i]);
  } else {
    gemv_emit<KPL>(L, theta, k, lane, w, out);
    if constexpr (ONE) {
      if (counter) gemv_one_finish<KPL>(out, k, counter, dst, flag, seq);
    }
  }
}

template <int D, bool BF16, int KPL, bool GATHER = false, int VAR = kGemvVar, bool ONE = false>
__global__ __launch_bounds__(kGemvThreads) void gemv_topk_kernel(
    const void* __restrict__ Xv, uint32_t n_rows, uint32_t row_base,
    const float* __restrict__ q, const uint64_t* __restrict__ allow, uint32_t k,
    uint32_t rows_per_wave, uint64_t* __restrict__ out,
    const uint32_t* __restrict__ rows = nullptr, uint32_t* __restrict__ hist = nullptr,
    int prep = 0, uint32_t* counter = nullptr, uint64_t* dst = nullptr, uint64_t* flag = nullptr,
    uint64_t seq = 0) {
  gemv_topk_body<D, BF16, KPL, GATHER, VAR, ONE>(Xv, n_rows, row_base, q, allow, k,
                                                 rows_per_wave, out, rows, hist, prep, counter,
                                                 dst, flag, seq);
}

// The raw query travels in the kernel's argument segment (r03): QueryArg is
// the first argument, so the query starts at the segment pointer; no H2D.
template <int D>
struct QueryArg {
  float v[D];
};
template <int D, bool BF16, int KPL>
__global__ __launch_bounds__(kGemvThreads) void gemv_one_arg_kernel(
    QueryArg<D> qa, const void* __restrict__ Xv, uint32_t n_rows, uint32_t row_base,
    const uint64_t* __restrict__ allow, uint32_t k, uint32_t rows_per_wave,
    uint64_t* __restrict__ out, int prep) {
  const float* q = (const float*)(const __attribute__((address_space(4))) float*)
      __builtin_amdgcn_kernarg_segment_ptr();
  gemv_topk_body<D, BF16, KPL, false, kGemvVar, true>(Xv, n_rows, row_base, q, allow, k,
                                                       rows_per_wave, out, nullptr, nullptr, prep,
                                                       nullptr, nullptr, nullptr, 0);
}

// Any dimension: one row per wave step, lane-strided scalar loads.
template <bool BF16, int KPL, bool GATHER = false>
__global__ __launch_bounds__(kGemvThreads) void gemv_topk_generic_kernel(
    const void* __restrict__ Xv, uint32_t dim, uint32_t n_rows, uint32_t row_base,
    const float* __restrict__ q, const uint64_t* __restrict__ allow, uint32_t k,
    uint32_t rows_per_wave, uint64_t* __restrict__ out,
    const uint32_t* __restrict__ rows = nullptr, uint32_t* __restrict__ hist = nullptr) {
  constexpr bool kScores = KPL == 0;  // as in gemv_topk_kernel
  __shared__ uint32_t lhist[kScores ? kRselBins : 1];
  if constexpr (kScores) {
    for (int i = threadIdx.x; i < kRselBins; i += kGemvThreads) lhist[i] = 0;
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t gw = (uint64_t)blockIdx.x * kGemvWaves + w;
  const uint64_t lo64 = gw * rows_per_wave;
  const uint32_t lo = lo64 < n_rows ? (uint32_t)lo64 : n_rows;
  const uint32_t hi = (uint64_t)lo + rows_per_wave < n_rows ? lo + rows_per_wave : n_rows;
  WaveList<kScores ? 1 : KPL> L;
  L.init();
  uint64_t theta = 0;
  for (uint32_t pos = lo; pos < hi; ++pos) {
    const uint32_t r = GATHER ? rows[pos] : pos;
    float p = 0.f;
    for (uint32_t d = lane; d < dim; d += 64) {
      const float x =
          BF16 ? vs::bf16_to_f32(__builtin_nontemporal_load((const uint16_t*)Xv + (size_t)r * dim + d))
               : __builtin_nontemporal_load((const float*)Xv + (size_t)r * dim + d);
      p = fmaf(x, q[d], p);
    }
    const float s = wave_sum(p);
    if constexpr (kScores) {
      if (lane == 0) {
        const uint32_t o = row_allowed(allow, r) ? (uint32_t)(make_key(s, 0) >> 32) : 0u;
        ((uint32_t*)out)[r] = o;
        if (o) atomicAdd(&lhist[o >> (32 - kRselBits0)], 1u);
      }
      continue;
    }
    const uint64_t key = make_key(s, row_base + r);
    if (key > theta && (GATHER || row_allowed(allow, r))) {
      L.insert(key, k, lane);
      theta = L.kth(k);
    }
  }
  if constexpr (kScores) {
    __syncthreads();
    for (int i = threadIdx.x; i < kRselBins; i += kGemvThreads)
      if (lhist[i]) atomicAdd(&hist[i], lhist[i]);
  } else {
    gemv_emit<KPL>(L, theta, k, lane, w, out);
  }
}

static int g_cu_count = 0;
int device_cu_count() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  g_cu_count = cus;
  return cus;
}

static int gemv_kpl(uint32_t k) { return k <= 64 ? 1 : (k <= 128 ? 2 : 16); }

// Rows-per-wave floor of small scans: 2 since r02 (was 16). Swept over
// 221 .. 200k rows x 768 fp32, k 5 and 100 (tools/tiny_sweep.py,
// profiles/r02c_tiny_sweep.jsonl): fewer rows per wave shortens the serial
// list inserts of a high-k scan (221 rows, k = 100: 73.6 -> 43.3 us; 20k rows:
// 140 -> 112 us) and costs nothing at k = 5. VS_GEMV_MIN_RPW overrides it
// (read once) for that sweep.
static uint32_t gemv_min_rpw() {
  static const uint32_t v = [] {
    const char* e = getenv("VS_GEMV_MIN_RPW");
    const int x = e ? atoi(e) : 2;
    return (uint32_t)(x > 0 ? x : 2);
  }();
  return v;
}
#define kGemvMinRowsPerWave gemv_min_rpw()

struct GemvGrid {
  uint32_t nwg, rows_per_wave;
};
static GemvGrid gemv_grid(uint32_t n_rows, int rb) {
  const int cus = g_cu_count ? g_cu_count : device_cu_count();
  uint64_t want = (uint64_t)cus * 3;  // 3 x 8 waves per CU
  // small scans (small collections, gathered selective filters) are latency
  // bound: spread them down to kGemvMinRowsPerWave rows per wave
  const uint64_t by_rows =
      ((uint64_t)n_rows + kGemvWaves * kGemvMinRowsPerWave - 1) / (kGemvWaves * kGemvMinRowsPerWave);
  if (want > by_rows) want = by_rows;
  if (want < 1) want = 1;
  const uint64_t waves = want * kGemvWaves;
  uint64_t rpw = ((uint64_t)n_rows + waves - 1) / waves;
  rpw = (rpw + rb - 1) / rb * rb;
  if (rpw == 0) rpw = rb;
  const uint64_t nwg = (((uint64_t)n_rows + rpw - 1) / rpw + kGemvWaves - 1) / kGemvWaves;
  return GemvGrid{(uint32_t)(nwg ? nwg : 1), (uint32_t)rpw};
}

uint32_t gemv_max_lists(uint32_t dim, bool bf16, uint32_t n_rows, uint32_t k) {
  (void)dim;
  (void)bf16;
  GemvGrid g = gemv_grid(n_rows, 1);
  // rb > 1 only lowers the workgroup count; rb == 1 is the upper bound.
  const uint32_t per = gemv_kpl(k) <= 2 ? 1 : kGemvWaves;
  return g.nwg * per;
}

template <int D, bool BF16, bool GATHER>
static void gemv_launch_kpl(int kpl, dim3 grid, dim3 block, hipStream_t st, const void* X,
                            uint32_t n_rows, uint32_t row_base, const float* q,
                            const uint64_t* allow, uint32_t k, uint32_t rpw, uint64_t* out,
                            const uint32_t* rows) {
  if (kpl == 1)
    hipLaunchKernelGGL((gemv_topk_kernel<D, BF16, 1, GATHER>), grid, block, 0, st, X, n_rows,
                       row_base, q, allow, k, rpw, out, rows);
  else if (kpl == 2)
    hipLaunchKernelGGL((gemv_topk_kernel<D, BF16, 2, GATHER>), grid, block, 0, st, X, n_rows,
                       row_base, q, allow, k, rpw, out, rows);
  else
    hipLaunchKernelGGL((gemv_topk_kernel<D, BF16, 16, GATHER>), grid, block, 0, st, X, n_rows,
                       row_base, q, allow, k, rpw, out, rows);
}

template <int D, bool BF16>
static hipError_t gemv_dispatch_kpl(const void* X, uint32_t n_rows, uint32_t row_base,
                                    const float* q, const uint64_t* allow, uint32_t k,
                                    uint64_t* out, uint32_t max_lists, uint32_t* nlists,
                                    hipStream_t st, const uint32_t* rows) {
  using S = GemvShape<D, BF16>;
  GemvGrid g = gemv_grid(n_rows, S::RB);
  const int kpl = gemv_kpl(k);
  const uint32_t lists = g.nwg * (kpl <= 2 ? 1 : kGemvWaves);
  if (lists > max_lists) return hipErrorInvalidValue;
  *nlists = lists;
  dim3 grid(g.nwg), block(kGemvThreads);
  if (rows)
    gemv_launch_kpl<D, BF16, true>(kpl, grid, block, st, X, n_rows, row_base, q, nullptr, k,
                                   g.rows_per_wave, out, rows);
  else
    gemv_launch_kpl<D, BF16, false>(kpl, grid, block, st, X, n_rows, row_base, q, allow, k,
                                    g.rows_per_wave, out, nullptr);
  return hipGetLastError();
}

template <int D, bool BF16>
static hipError_t gemv_one_d(const void* X, uint32_t n_rows, uint32_t row_base, const float* q_raw,
                             int prep, const uint64_t* allow, uint32_t k, uint64_t* lists,
                             uint32_t max_lists, uint32_t* counter, uint64_t* dst, uint64_t* flag,
                             uint64_t seq, hipStream_t st, uint32_t* nlists, const float* q_host) {
  using S = GemvShape<D, BF16>;
  const GemvGrid g = gemv_grid(n_rows, S::RB);
  if (g.nwg > max_lists) return hipErrorInvalidValue;
  if (nlists) *nlists = g.nwg;
  if constexpr (D <= (int)kGemvSmallArgDim) {
    if (q_host) {  // no merge in the kernel (counter unused): the lists, then launch_merge
      QueryArg<D> qa;
      std::memcpy(qa.v, q_host, sizeof(qa.v));
      if (gemv_kpl(k) == 1)
        hipLaunchKernelGGL((gemv_one_arg_kernel<D, BF16, 1>), dim3(g.nwg), dim3(kGemvThreads), 0,
                           st, qa, X, n_rows, row_base, allow, k, g.rows_per_wave, lists, prep);
      else
        hipLaunchKernelGGL((gemv_one_arg_kernel<D, BF16, 2>), dim3(g.nwg), dim3(kGemvThreads), 0,
                           st, qa, X, n_rows, row_base, allow, k, g.rows_per_wave, lists, prep);
      return hipGetLastError();
    }
  }
  if (gemv_kpl(k) == 1)
    hipLaunchKernelGGL((gemv_topk_kernel<D, BF16, 1, false, kGemvVar, true>), dim3(g.nwg),
                       dim3(kGemvThreads), 0, st, X, n_rows, row_base, q_raw, allow, k,
                       g.rows_per_wave, lists, nullptr, nullptr, prep, counter, dst, flag, seq);
  else
    hipLaunchKernelGGL((gemv_topk_kernel<D, BF16, 2, false, kGemvVar, true>), dim3(g.nwg),
                       dim3(kGemvThreads), 0, st, X, n_rows, row_base, q_raw, allow, k,
                       g.rows_per_wave, lists, nullptr, nullptr, prep, counter, dst, flag, seq);
  return hipGetLastError();
}

bool gemv_one_ok(uint32_t dim, uint32_t k) {
  if (k == 0 || k > 128) return false;
  // not 1536: the wave-0 preprocessing of 24 values per lane takes that scan
  // to 88-106 VGPRs (63-85 without it), below 3 workgroups per CU
  switch (dim) {
    case 128: case 256: case 384: case 512: case 768: case 1024: return true;
    default: return false;
  }
}

hipError_t launch_gemv_one(const void* X, bool bf16, uint32_t dim, uint32_t n_rows,
                           uint32_t row_base, const float* q_raw, bool cosine,
                           const uint64_t* allow, uint32_t k, uint64_t* lists, uint32_t max_lists,
                           uint32_t* counter, uint64_t* dst, hipStream_t st, uint64_t* flag,
                           uint64_t seq, uint32_t* nlists, const float* q_host) {
  if (!gemv_one_ok(dim, k) || n_rows == 0 || (counter && !dst)) return hipErrorInvalidValue;
  if (q_host && (counter || dim > kGemvSmallArgDim)) return hipErrorInvalidValue;
  const int prep = (cosine ? 1 : 0) | (bf16 ? 2 : 0);
#define VS_ONE_CASE(DD)                                                                      \
  case DD:                                                                                   \
    return bf16 ? gemv_one_d<DD, true>(X, n_rows, row_base, q_raw, prep, allow, k, lists,    \
                                       max_lists, counter, dst, flag, seq, st, nlists,       \
                                       q_host)                                               \
                : gemv_one_d<DD, false>(X, n_rows, row_base, q_raw, prep, allow, k, lists,   \
                                        max_lists, counter, dst, flag, seq, st, nlists,      \
                                        q_host);
  switch (dim) {
    VS_ONE_CASE(128)
    VS_ONE_CASE(256)
    VS_ONE_CASE(384)
    VS_ONE_CASE(512)
    VS_ONE_CASE(768)
    VS_ONE_CASE(1024)
    default:
      return hipErrorInvalidValue;
  }
#undef VS_ONE_CASE
}

template <bool BF16, bool GATHER>
static void gemv_generic_kpl(int kpl, dim3 grid, dim3 block, hipStream_t st, const void* X,
                             uint32_t dim, uint32_t n_rows, uint32_t row_base, const float* q,
                             const uint64_t* allow, uint32_t k, uint32_t rpw, uint64_t* out,
                             const uint32_t* rows) {
  if (kpl == 1)
    hipLaunchKernelGGL((gemv_topk_generic_kernel<BF16, 1, GATHER>), grid, block, 0, st, X, dim,
                       n_rows, row_base, q, allow, k, rpw, out, rows);
  else if (kpl == 2)
    hipLaunchKernelGGL((gemv_topk_generic_kernel<BF16, 2, GATHER>), grid, block, 0, st, X, dim,
                       n_rows, row_base, q, allow, k, rpw, out, rows);
  else
    hipLaunchKernelGGL((gemv_topk_generic_kernel<BF16, 16, GATHER>), grid, block, 0, st, X, dim,
                       n_rows, row_base, q, allow, k, rpw, out, rows);
}

template <bool BF16>
static hipError_t gemv_generic(const void* X, uint32_t dim, uint32_t n_rows,
                               uint32_t row_base, const float* q, const uint64_t* allow,
                               uint32_t k, uint64_t* out, uint32_t max_lists, uint32_t* nlists,
                               hipStream_t st, const uint32_t* rows) {
  GemvGrid g = gemv_grid(n_rows, 1);
  const int kpl = gemv_kpl(k);
  const uint32_t lists = g.nwg * (kpl <= 2 ? 1 : kGemvWaves);
  if (lists > max_lists) return hipErrorInvalidValue;
  *nlists = lists;
  dim3 grid(g.nwg), block(kGemvThreads);
  if (rows)
    gemv_generic_kpl<BF16, true>(kpl, grid, block, st, X, dim, n_rows, row_base, q, nullptr, k,
                                 g.rows_per_wave, out, rows);
  else
    gemv_generic_kpl<BF16, false>(kpl, grid, block, st, X, dim, n_rows, row_base, q, allow, k,
                                  g.rows_per_wave, out, nullptr);
  return hipGetLastError();
}

hipError_t launch_gemv(const void* X, bool bf16, uint32_t dim, uint32_t n_rows,
                       uint32_t row_base, const float* q, uint32_t k, uint64_t* out,
                       uint32_t max_lists, uint32_t* nlists, hipStream_t st,
                       const uint64_t* allow, const uint32_t* rows) {
  if (k == 0 || k > kMaxK || n_rows == 0) return hipErrorInvalidValue;
#define VS_GEMV_CASE(DD)                                                              \
  case DD:                                                                            \
    return bf16 ? gemv_dispatch_kpl<DD, true>(X, n_rows, row_base, q, allow, k, out,  \
                                              max_lists, nlists, st, rows)            \
                : gemv_dispatch_kpl<DD, false>(X, n_rows, row_base, q, allow, k, out, \
                                               max_lists, nlists, st, rows);
  switch (dim) {
    VS_GEMV_CASE(128)
    VS_GEMV_CASE(256)
    VS_GEMV_CASE(384)
    VS_GEMV_CASE(512)
    VS_GEMV_CASE(768)
    VS_GEMV_CASE(1024)
    VS_GEMV_CASE(1536)
    VS_GEMV_CASE(2048)
    VS_GEMV_CASE(3072)
    VS_GEMV_CASE(4096)
    default:
      return bf16 ? gemv_generic<true>(X, dim, n_rows, row_base, q, allow, k, out,
                                       max_lists, nlists, st, rows)
                  : gemv_generic<false>(X, dim, n_rows, row_base, q, allow, k, out,
                                        max_lists, nlists, st, rows);
  }
#undef VS_GEMV_CASE
}

template <int D, bool BF16>
static hipError_t gemv_scores_d(const void* X, uint32_t n_rows, const float* q,
                                const uint64_t* allow, uint32_t* sc, uint32_t* hist,
                                hipStream_t st) {
  using S = GemvShape<D, BF16>;
  const GemvGrid g = gemv_grid(n_rows, S::RB);
  // contiguous row slices per wave (no step interleave): a wave's 64
  // buffered images are 64 consecutive rows, one coalesced 256-B store (the
  // interleaved order scattered them over 32 lines shared with other waves:
  // 2.62 ms against 2.29 for the list scan at 10M x 768 bf16)
  hipLaunchKernelGGL((gemv_topk_kernel<D, BF16, 0, false, (kGemvVar & ~8)>), dim3(g.nwg),
                     dim3(kGemvThreads), 0, st, X, n_rows, 0u, q, allow, 0u, g.rows_per_wave,
                     (uint64_t*)sc, nullptr, hist);
  return hipGetLastError();
}

hipError_t launch_gemv_scores(const void* X, bool bf16, uint32_t dim, uint32_t n_rows,
                              const float* q, const uint64_t* allow, uint32_t* sc, uint32_t* hist,
                              hipStream_t st) {
  if (n_rows == 0) return hipErrorInvalidValue;
#define VS_SCORES_CASE(DD) \
  case DD:                 \
    return bf16 ? gemv_scores_d<DD, true>(X, n_rows, q, allow, sc, hist, st) \
                : gemv_scores_d<DD, false>(X, n_rows, q, allow, sc, hist, st);
  switch (dim) {
    VS_SCORES_CASE(128)
    VS_SCORES_CASE(256)
    VS_SCORES_CASE(384)
    VS_SCORES_CASE(512)
    VS_SCORES_CASE(768)
    VS_SCORES_CASE(1024)
    VS_SCORES_CASE(1536)
    VS_SCORES_CASE(2048)
    VS_SCORES_CASE(3072)
    VS_SCORES_CASE(4096)
    default: {
      const GemvGrid g = gemv_grid(n_rows, 1);
      if (bf16)
        hipLaunchKernelGGL((gemv_topk_generic_kernel<true, 0, false>), dim3(g.nwg),
                           dim3(kGemvThreads), 0, st, X, dim, n_rows, 0u, q, allow, 0u,
                           g.rows_per_wave, (uint64_t*)sc, nullptr, hist);
      else
        hipLaunchKernelGGL((gemv_topk_generic_kernel<false, 0, false>), dim3(g.nwg),
                           dim3(kGemvThreads), 0, st, X, dim, n_rows, 0u, q, allow, 0u,
                           g.rows_per_wave, (uint64_t*)sc, nullptr, hist);
      return hipGetLastError();
    }
  }
#undef VS_SCORES_CASE
}

// The wave's earlier stores (every lane's) reach host-visible memory before
// lane 0 publishes `seq`: a host that reads the word then reads the keys.
__device__ __forceinline__ void signal_host(uint64_t* flag, uint64_t seq, int lane) {
  __threadfence_system();
  if (lane == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Small collections, one query, k <= 16, no filter: query preprocessing,
// scan and the workgroup merge in one launch of one workgroup, which writes
// the final k keys (what query prep + gemv + merge produce, bit for bit: the
// same per-row sums, the same exact top k). Saves two dependent launches of a
// search that is all launch latency (221 rows).
// The one workgroup's 8 waves each walk ~n_rows / 8 rows, so the scan is a
// chain of dependent row steps (load, FMAs, a 6-step shuffle reduction, the
// list insert): 17 us at 221 rows with one row step at a time, whatever the
// load depth. Here each wave takes U row groups per step -- all their loads
// issued first, their U reductions independent -- so the chains overlap
// (221 rows: 17.1 us -> 12.6 with U = 4).
// Each row's sum is formed exactly as in gemv_topk_kernel (the same lane /
// chunk layout, the same accumulation and the same xor tree), so its scores
// are the same bits. Wave 0 first preprocesses the raw query into LDS as
// query_prep_kernel does (prep bit 0: cosine, bit 1: round to bf16 values).
//
// Several workgroups (r03): one workgroup reads the whole collection through
// one CU (221 rows x 3 KB at C1: the CU's bandwidth and the row steps were
// most of the 12.7 us), so the rows are spread over gridDim.x workgroups,
// each preparing the query itself. Each writes its k keys to part[wg][k]
// with agent-scope (sc1) stores, waits for them (vmcnt), and adds 1 to
// *counter (agent-scope atomic); the workgroup whose add returns
// gridDim.x - 1 reads every part with sc1 loads after a workgroup barrier
// and writes the merged top k, then resets the counter (MI355X_MICROARCH.md
// cross-CU hand-off, first row: one signaling lane per storing workgroup,
// the last adder consumes). One launch of one workgroup when gridDim.x == 1.
//
// Host completion word (r03): with `flag`, `out` is mapped pinned host memory
// and the writing wave, after its key stores, fences at system scope and
// stores `seq` to *flag (host memory too); the host spins on that word instead
// of a D2H copy and the stream's completion event, which cost ~6 us of a
// ~18 us round trip (tools/rt_floor.hip, profiles/r03_rt_floor_graph_flag.json).
template <int D, bool BF16, int U>
__device__ __forceinline__ void gemv_small_body(
    const void* __restrict__ Xv, uint32_t n_rows, uint32_t row_base, const float* __restrict__ q,
    uint32_t k, int prep, uint64_t* __restrict__ out, uint64_t* __restrict__ part,
    uint32_t* __restrict__ counter, uint64_t* flag, uint64_t seq) {
  using S = GemvShape<D, BF16>;
  static_assert(D % 64 == 0 && D <= 64 * kQPrepMax, "query_prep_kernel's shapes only");
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // the first row step's loads go out before the query prep (they do not
  // depend on it), so their HBM latency hides under wave 0's fp64 prep
  int rowsel[S::J];
  int coff[S::J];
#pragma unroll
  for (int j = 0; j < S::J; ++j) {
    const int c = lane + 64 * j;
    rowsel[j] = (S::RB == 1) ? 0 : c / S::CPR;
    coff[j] = c % S::CPR;
  }
  const char* X = (const char*)Xv;
  const uint32_t n_groups = (n_rows + S::RB - 1) / S::RB;
  const uint32_t nw = gridDim.x * kGemvWaves;  // waves of the launch
  const uint32_t gfirst = blockIdx.x * kGemvWaves + (uint32_t)w;
  uint4 buf[U][S::J];
  auto load_step = [&](uint32_t g0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int j = 0; j < S::J; ++j) {
        // rows past the end read the last row again (never keyed)
        uint32_t row = (g0 + (uint32_t)u * nw) * S::RB + rowsel[j];
        row = row < n_rows ? row : n_rows - 1;
        buf[u][j] = *(const uint4*)(X + (size_t)row * S::RBYTES + (size_t)coff[j] * 16);
      }
    }
  };
  if (gfirst < n_groups) load_step(gfirst);
  __shared__ float qs[D];
  if (w == 0) prep_query_wave<D>(q, prep, qs, lane);
  __syncthreads();
  float qv[S::J][S::EPC];
#pragma unroll
  for (int j = 0; j < S::J; ++j)
#pragma unroll
    for (int e = 0; e < S::EPC; ++e) qv[j][e] = qs[coff[j] * S::EPC + e];
  WaveList<1> L;
  L.init();
  uint64_t theta = 0;
  for (uint32_t g0 = gfirst; g0 < n_groups; g0 += nw * U) {
    if (g0 != gfirst) load_step(g0);
    float sc[U][S::RB];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float p[S::RB];
#pragma unroll
      for (int b = 0; b < S::RB; ++b) p[b] = 0.f;
#pragma unroll
      for (int j = 0; j < S::J; ++j) {
        const float d = chunk_dot<BF16>(buf[u][j], qv[j]);
        if constexpr (S::RB == 1) {
          p[0] += d;
        } else {
#pragma unroll
          for (int b = 0; b < S::RB; ++b) p[b] += (rowsel[j] == b) ? d : 0.f;
        }
      }
#pragma unroll
      for (int b = 0; b < S::RB; ++b) sc[u][b] = wave_sum(p[b]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int b = 0; b < S::RB; ++b) {
        const uint32_t row = (g0 + (uint32_t)u * nw) * S::RB + b;
        if (row < n_rows) {
          const uint64_t key = make_key(sc[u][b], row_base + row);
          if (key > theta) {
            L.insert(key, k, lane);
            theta = L.kth(k);
          }
        }
      }
    }
  }
  // Workgroup merge by rank, not by serial inserts (35 dependent inserts in
  // wave 0 at k = 5): the first k keys of the 8 wave lists go to LDS; a key's
  // place in the output is the number of larger keys among them (keys are
  // unique: distinct rows), so every lane places its own keys at once. The
  // output is the same sorted top k, zero-filled past the nonzero keys.
  __shared__ uint64_t sm[kGemvWaves][64];
  __shared__ int last_wg;
  sm[w][lane] = L.e[0];
  __syncthreads();
  const bool multi = gridDim.x > 1;
  if (w == 0) {
    const uint32_t tot = kGemvWaves * k;  // <= 128
    const uint32_t c0 = (uint32_t)lane, c1 = (uint32_t)lane + 64;
    const uint64_t x0 = c0 < tot ? sm[c0 / k][c0 % k] : 0;
    const uint64_t x1 = c1 < tot ? sm[c1 / k][c1 % k] : 0;
    uint32_t r0 = 0, r1 = 0, nz = 0;
    for (int ow = 0; ow < kGemvWaves; ++ow)
      for (uint32_t j = 0; j < k; ++j) {
        const uint64_t y = sm[ow][j];  // uniform LDS broadcast
        r0 += y > x0 ? 1u : 0u;
        r1 += y > x1 ? 1u : 0u;
        nz += y != 0 ? 1u : 0u;
      }
    if (!multi) {
      if (x0 && r0 < k) out[r0] = x0;
      if (x1 && r1 < k) out[r1] = x1;
      if ((uint32_t)lane >= nz && (uint32_t)lane < k) out[lane] = 0;
      if (flag) signal_host(flag, seq, lane);
    } else {
      // this workgroup's k keys (0-padded) -> part, agent-scope stores
      uint64_t* dst = part + (size_t)blockIdx.x * k;
      if (x0 && r0 < k) __hip_atomic_store(dst + r0, x0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (x1 && r1 < k) __hip_atomic_store(dst + r1, x1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((uint32_t)lane >= nz && (uint32_t)lane < k)
        __hip_atomic_store(dst + lane, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the stores landed before the add
      int l = 0;
      if (lane == 0)
        l = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            gridDim.x - 1;
      l = __shfl(l, 0, 64);
      if (lane == 0) last_wg = l;
    }
  }
  if (!multi) return;
  __syncthreads();  // last_wg published; the adding wave's add has returned
  if (!last_wg) return;
  // the last workgroup: every part (sc1 loads, after the barrier above), ranked
  __shared__ uint64_t pk[kGemvSmallMaxParts * kGemvSmallMaxK];
  const uint32_t tot = gridDim.x * k;
  for (uint32_t i = threadIdx.x; i < tot; i += kGemvThreads)
    pk[i] = __hip_atomic_load(part + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (w == 0) {
    uint32_t nz = 0;
    uint32_t r[kGemvSmallMaxParts * kGemvSmallMaxK / 64];
    uint64_t x[kGemvSmallMaxParts * kGemvSmallMaxK / 64];
#pragma unroll
    for (int i = 0; i < kGemvSmallMaxParts * kGemvSmallMaxK / 64; ++i) {
      const uint32_t c = (uint32_t)lane + 64u * i;
      x[i] = c < tot ? pk[c] : 0;
      r[i] = 0;
    }
    for (uint32_t j = 0; j < tot; ++j) {
      const uint64_t y = pk[j];  // uniform LDS broadcast
      nz += y != 0 ? 1u : 0u;
#pragma unroll
      for (int i = 0; i < kGemvSmallMaxParts * kGemvSmallMaxK / 64; ++i) r[i] += y > x[i] ? 1u : 0u;
    }
#pragma unroll
    for (int i = 0; i < kGemvSmallMaxParts * kGemvSmallMaxK / 64; ++i)
      if (x[i] && r[i] < k) out[r[i]] = x[i];
    if ((uint32_t)lane >= nz && (uint32_t)lane < k) out[lane] = 0;
    if (lane == 0) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (flag) signal_host(flag, seq, lane);
  }
}

template <int D, bool BF16, int U>
__global__ __launch_bounds__(kGemvThreads) void gemv_small_kernel(
    const void* __restrict__ Xv, uint32_t n_rows, uint32_t row_base, const float* __restrict__ q,
    uint32_t k, int prep, uint64_t* __restrict__ out, uint64_t* __restrict__ part,
    uint32_t* __restrict__ counter, uint64_t* flag, uint64_t seq) {
  gemv_small_body<D, BF16, U>(Xv, n_rows, row_base, q, k, prep, out, part, counter, flag, seq);
}

// The same search with the raw query in the kernel's argument segment (r03):
// the dispatch carries it, so the call needs no H2D copy. QueryArg is the
// first argument, so the query starts at the segment pointer.
template <int D, bool BF16, int U>
__global__ __launch_bounds__(kGemvThreads) void gemv_small_arg_kernel(
    QueryArg<D> qa, const void* __restrict__ Xv, uint32_t n_rows, uint32_t row_base, uint32_t k,
    int prep, uint64_t* __restrict__ out, uint64_t* __restrict__ part,
    uint32_t* __restrict__ counter, uint64_t* flag, uint64_t seq) {
  const float* q = (const float*)(const __attribute__((address_space(4))) float*)
      __builtin_amdgcn_kernarg_segment_ptr();
  gemv_small_body<D, BF16, U>(Xv, n_rows, row_base, q, k, prep, out, part, counter, flag, seq);
}

uint32_t gemv_small_parts(uint32_t dim, bool bf16, uint32_t n_rows) {
  // one row-group step per wave: 8 waves x U groups x RB rows per workgroup
  const uint32_t epc = bf16 ? 8 : 4, cpr = dim / epc;
  uint32_t g = 64, c = cpr;  // RB = 64 / gcd(CPR, 64)
  while (c) {
    const uint32_t t = g % c;
    g = c;
    c = t;
  }
  const uint32_t rb = 64 / g, j = rb * cpr / 64;
  const uint32_t u = j <= 3 ? 4 : (12 / j > 0 ? 12 / j : 1);
  const uint32_t per_wg = (uint32_t)kGemvWaves * u * rb;
  const uint32_t w = (n_rows + per_wg - 1) / per_wg;
  // VS_SMALL_PARTS caps the workgroups (read once; ablation)
  static const uint32_t cap = [] {
    const char* e = getenv("VS_SMALL_PARTS");
    const int x = e ? atoi(e) : (int)kGemvSmallMaxParts;
    return (uint32_t)std::min(std::max(x, 1), (int)kGemvSmallMaxParts);
  }();
  return std::min<uint32_t>(std::max<uint32_t>(w, 1), cap);
}

template <int D, bool BF16>
static void gemv_small_launch(const void* X, uint32_t n_rows, uint32_t row_base,
                              const float* q_raw, int prep, uint32_t k, uint64_t* out,
                              uint64_t* part, uint32_t* counter, uint64_t* flag, uint64_t seq,
                              const float* q_host, hipStream_t st) {
  // row groups per step: 4 (8 with the next step's loads issued ahead was
  // slower: 14.9 us against 12.6 at 221 rows), fewer past 3 chunks per lane
  constexpr int J = GemvShape<D, BF16>::J;
  constexpr int U = J <= 3 ? 4 : (12 / J > 0 ? 12 / J : 1);
  const uint32_t nwg = part ? gemv_small_parts(D, BF16, n_rows) : 1;
  if constexpr (D <= (int)kGemvSmallArgDim) {
    if (q_host) {
      QueryArg<D> qa;
      std::memcpy(qa.v, q_host, sizeof(qa.v));
      hipLaunchKernelGGL((gemv_small_arg_kernel<D, BF16, U>), dim3(nwg), dim3(kGemvThreads), 0,
                         st, qa, X, n_rows, row_base, k, prep, out, part, counter, flag, seq);
      return;
    }
  }
  hipLaunchKernelGGL((gemv_small_kernel<D, BF16, U>), dim3(nwg), dim3(kGemvThreads), 0, st, X,
                     n_rows, row_base, q_raw, k, prep, out, part, counter, flag, seq);
}

bool gemv_small_ok(uint32_t dim, uint32_t n_rows, uint32_t k) {
  if (n_rows == 0 || n_rows > kGemvSmallMaxRows || k == 0 || k > kGemvSmallMaxK) return false;
  switch (dim) {
    case 128: case 256: case 384: case 512: case 768: case 1024: case 1536: return true;
    default: return false;
  }
}

hipError_t launch_gemv_small(const void* X, bool bf16, uint32_t dim, uint32_t n_rows,
                             uint32_t row_base, const float* q_raw, bool cosine, uint32_t k,
                             uint64_t* out, hipStream_t st, uint64_t* part, uint32_t* counter,
                             uint64_t* flag, uint64_t seq, const float* q_host) {
  if (!gemv_small_ok(dim, n_rows, k)) return hipErrorInvalidValue;
  if (q_host && dim > kGemvSmallArgDim) return hipErrorInvalidValue;
  if (!counter) part = nullptr;
  const int prep = (cosine ? 1 : 0) | (bf16 ? 2 : 0);
#define VS_SMALL_CASE(DD)                                                                   \
  case DD:                                                                                  \
    if (bf16)                                                                               \
      gemv_small_launch<DD, true>(X, n_rows, row_base, q_raw, prep, k, out, part, counter,  \
                                  flag, seq, q_host, st);                                   \
    else                                                                                    \
      gemv_small_launch<DD, false>(X, n_rows, row_base, q_raw, prep, k, out, part, counter, \
                                   flag, seq, q_host, st);                                  \
    break;
  switch (dim) {
    VS_SMALL_CASE(128)
    VS_SMALL_CASE(256)
    VS_SMALL_CASE(384)
    VS_SMALL_CASE(512)
    VS_SMALL_CASE(768)
    VS_SMALL_CASE(1024)
    VS_SMALL_CASE(1536)
    default:
      return hipErrorInvalidValue;
  }
#undef VS_SMALL_CASE
  return hipGetLastError();
}

// Filter bitmap -> compacted list of the allowed local rows, ascending, for
// the GATHER scans. Ascending order makes the list (and so every gathered
// score: a row's position in its wave step decides its summation order) a
// function of the bitmap alone, whichever way it was built. Three launches:
// per-block popcounts of 256 words (16384 rows), an in-place exclusive scan
// of those counts in one workgroup, then each block places its rows.
constexpr int kCompactThreads = 256;

__device__ __forceinline__ uint64_t compact_word(const uint64_t* __restrict__ allow,
                                                 uint32_t n_rows, uint32_t wi) {
  const uint32_t nwords = (n_rows + 63) / 64;
  uint64_t w = wi < nwords ? allow[wi] : 0;
  if (wi == nwords - 1 && (n_rows & 63)) w &= (1ull << (n_rows & 63)) - 1;
  return w;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t t = __shfl_up(v, off);
    if (lane >= off) v += t;
  }
  return v;
}

__global__ __launch_bounds__(kCompactThreads) void compact_count_kernel(
    const uint64_t* __restrict__ allow, uint32_t n_rows, uint32_t* __restrict__ block_cnt) {
  __shared__ uint32_t part[kCompactThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t c = (uint32_t)__popcll(compact_word(allow, n_rows, blockIdx.x * kCompactThreads + threadIdx.x));
  const uint32_t t = wave_incl_scan(c, lane);
  if (lane == 63) part[w] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t sum = 0;
    for (int v = 0; v < kCompactThreads / 64; ++v) sum += part[v];
    block_cnt[blockIdx.x] = sum;
  }
}

// One workgroup: exclusive scan of block_cnt[0, n) in place, 256 at a time.
__global__ __launch_bounds__(kCompactThreads) void compact_scan_kernel(uint32_t* __restrict__ block_cnt,
                                                                       uint32_t n) {
  __shared__ uint32_t part[kCompactThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < n; b0 += kCompactThreads) {
    const uint32_t i = b0 + threadIdx.x;
    const uint32_t c = i < n ? block_cnt[i] : 0;
    const uint32_t inc = wave_incl_scan(c, lane);
    if (lane == 63) part[w] = inc;
    __syncthreads();
    uint32_t base = carry, tot = 0;
    for (int v = 0; v < kCompactThreads / 64; ++v) {
      if (v < w) base += part[v];
      tot += part[v];
    }
    if (i < n) block_cnt[i] = base + inc - c;
    carry += tot;
    __syncthreads();  // part[] is rewritten by the next chunk
  }
}

__global__ __launch_bounds__(kCompactThreads) void compact_rows_kernel(
    const uint64_t* __restrict__ allow, uint32_t n_rows, const uint32_t* __restrict__ block_base,
    uint32_t* __restrict__ rows) {
  __shared__ uint32_t part[kCompactThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t wi = blockIdx.x * kCompactThreads + threadIdx.x;
  uint64_t word = compact_word(allow, n_rows, wi);
  const uint32_t c = (uint32_t)__popcll(word);
  const uint32_t inc = wave_incl_scan(c, lane);
  if (lane == 63) part[w] = inc;
  __syncthreads();
  uint32_t o = block_base[blockIdx.x] + inc - c;
  for (int v = 0; v < w; ++v) o += part[v];
  while (word) {
    rows[o++] = wi * 64u + (uint32_t)(__ffsll((unsigned long long)word) - 1);
    word &= word - 1;
  }
}

uint32_t compact_scratch_words(uint32_t n_rows) {
  return ((n_rows + 63) / 64 + kCompactThreads - 1) / kCompactThreads;
}

hipError_t launch_compact_rows(const uint64_t* allow, uint32_t n_rows, uint32_t* rows,
                               uint32_t* scratch, hipStream_t st) {
  if (n_rows == 0) return hipErrorInvalidValue;
  const uint32_t nb = compact_scratch_words(n_rows);
  hipLaunchKernelGGL(compact_count_kernel, dim3(nb), dim3(kCompactThreads), 0, st, allow,
                     n_rows, scratch);
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(kCompactThreads), 0, st, scratch, nb);
  hipLaunchKernelGGL(compact_rows_kernel, dim3(nb), dim3(kCompactThreads), 0, st, allow, n_rows,
                     scratch, rows);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// batched bf16 scan on MFMA + fused top-k
// ---------------------------------------------------------------------------
// Workgroup = 8 waves, two per SIMD (waves w and w+4 share one); wave w owns
// queries [32w, 32w+32) as two 16-query column groups of
// v_mfma_f32_16x16x32_bf16 and keeps their B-operand fragments for the whole
// row (2 x D/32 k-steps x 4 VGPRs = 192 at D = 768) resident in registers, so
// the query block is read once per CU and only the corpus streams. The
// workgroup streams its contiguous row range HBM -> LDS once, by LDS-DMA
// (global_load_lds_dwordx4; 1 KiB pieces = 8 rows x 128 B), through a ring of
// K-chunks (32 rows x 256 k = 16 KiB); AHEAD chunks stay in flight across the
// raw s_barrier that publishes each chunk (counted vmcnt, never a drain
// inside the loop). Per 32-k step a wave reads two A fragments (rows 0-15 and
// 16-31 of the tile, ds_read_b128) and each feeds both query groups: 4 MFMAs
// per 2 LDS reads. Scores never reach HBM.
//
// Top-k, main pass (MODE 0). Every query starts from a lower bound on its
// global k-th score (init_score, the sample pass below). The tile epilogue
// tests each lane's 8 scores per group against it (one v_max3 chain); a lane
// whose maximum reaches it appends its 8-score slab, unsorted, to its own
// quarter of the query's candidate buffer in global memory (count and slot
// in registers, fire-and-forget stores), and select_slab_kernel picks the
// top k of all workgroups' slabs. No wave ever waits on a list in the loop,
// so no stall reaches the other seven waves through the per-chunk barrier.
// A full buffer quarter (many near-equal rows) keeps its best slabs in place
// (mf_replace_min): exact, so no batch is ever re-run and the host never
// waits on the device.
//
// Sample pass (MODE 3): the same scan over the first 1/128 of every
// workgroup's tiles, writing per (query, tile) only the TILE MAXIMUM;
// sample_bound_kernel takes the k-th largest of them (k distinct rows reach
// it), a lower bound on the global k-th score: rows under it can never enter
// the result. MODE 8 (sorted per-query lists in LDS, mf_insert) serves
// small collections (fewer than 8 tiles per workgroup, k <= 16).
// Query groups (16 queries each) per wave: G = 2 -> 8 waves of 32 queries
// (two per SIMD, 256 queries per launch; D <= 768); G = 1 -> 8 waves of 16
// queries (128 per launch: the B fragments of D = 1024 / 1536 then fit the
// 256-register budget); G = 4 (ablation) -> 4 waves of 64 queries (one per
// SIMD, 512-register budget), which halves the LDS reads per MFMA.
constexpr int kMfG = 2;
constexpr int mf_waves(int g) { return g == 4 ? 4 : 8; }
// query groups per wave from the row bytes: the B fragments of a wave's
// queries take G * rby / 16 VGPRs, <= 192 (bf16 D <= 768 and fp32 D <= 384:
// G = 2; bf16 D = 1024 / 1536 and fp32 D = 512 / 768: G = 1)
constexpr int mf_groups_b(int rby) { return rby <= 1536 ? 2 : 1; }
constexpr int mf_groups(int d) { return mf_groups_b(2 * d); }
constexpr int kMfListLen = (int)kMfmaListMaxK;                  // entries per query list
constexpr int kMfListBytes = (int)kMfmaQueries * kMfListLen * 8;  // 32 KiB
constexpr int kMfRingBytes = 112 * 1024;
static_assert(kMfmaListMaxK == 16, "list insert assumes 4 lanes x 4 entries per query");

typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef int i32x4_t __attribute__((ext_vector_type(4)));

// Kernel arguments (one struct, passed by value in the kernarg segment).
struct MfArgs {
  const void* X;            // corpus rows (bf16 or fp32), row-major, 32 rows of padding
  const void* Q;            // kMfmaQueries x D, the collection's dtype (zero-padded)
  const float* init_score;  // nullable: per-query lower bound on the k-th score (MODE 0 / 8)
  uint64_t* lists;          // MODE 8: [nwg][kMfmaQueries][k] sorted keys
  float* tmax;              // MODE 3: [kMfmaQueries][nwg * max_tiles] tile maxima
  uint64_t* cand;           // MODE 0: [nwg][kMfmaQueries][cand_cap] slabs of 8 f32 scores
                            // (32 B); quarter kq of a query's buffer belongs to its lane kq
  uint32_t* cand_tile;      // MODE 0: first global row of each slab's tile
  uint32_t* cand_cnt;       // MODE 0: [nwg][kMfmaQueries][4] slabs per quarter
  uint32_t* cand_max;       // MODE 0, nullable: [nwg][kMfmaQueries][4] each quarter's largest
                            // admitted score as vs::score_ord (0: no slab), for the select
  const uint64_t* allow;    // nullable: filter pre-mask, bit r admits local row r
  uint32_t n_rows, row_base, rows_per_wg, max_tiles, nq_valid, k, cand_cap;
  const uint32_t* wg_tile;  // nullable: workgroup b scans tiles [wg_tile[b], wg_tile[b+1])
  // int8 prefilter pass (I8, r04; DESIGN.md §5 "int8 prefilter"): per query
  // {sqS, a, c, sigma} (q8par, float4) and the collection's {-, dmax, nmax, S}
  // (q8glob) turn the sample bound into an integer dot threshold. A full
  // quarter keeps counting past its capacity (lossy: the select recomputes
  // it, r05); the pass raises no word of its own.
  const float* q8par;
  const float* q8glob;
  uint32_t* gate;  // (unused since r05; the batch's control words, vs_kernels.h kGate*)
  // nullable: the launch does nothing unless *run_if != 0 (the passes of a
  // speculative try, gated on its go word, and the sample path behind it,
  // gated on its verdict: vs_engine.cpp search_mfma)
  const uint32_t* run_if;
};

// XOR swizzle of the 16-B chunk inside a 128-B row piece: spreads the
// ds_read_b128 lane groups of the 16x16x32 A fragment over all 64 banks
// (conflict-free, measured SQ_LDS_BANK_CONFLICT = 0).
__device__ __forceinline__ int mf_swz(int ri, int rg) {
  return ((ri >> 1) & 3) | ((rg & 1) << 2);
}

// max of three scores; hipcc forms one v_max3_f32 (checked in the .s). It
// must stay compiler-visible, not inline asm: the hazard recognizer then
// inserts the wait states an MFMA result needs before a VALU read (s_nop 5-7
// on gfx950) -- an asm v_max3 read stale accumulators once the schedule
// placed it right after the tile's last MFMA (r01).
__device__ __forceinline__ float fmax3(float a, float b, float c) {
  return __builtin_fmaxf(__builtin_fmaxf(a, b), c);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 16-B-per-lane LDS-DMA (global_load_lds_dwordx4) to the wave-uniform LDS
// byte address `lds` (+ lane*16). Issued from inline asm so hipcc's waitcnt
// pass does not see an LDS store and cannot drain vmcnt before every
// ds_read of the ring; completion is counted by wait_vmcnt<N>() by hand.
// M0 is written and restored inside the statement (§5.7: M0 is reserved).
// Address = wave-uniform 64-bit base (SGPRs) + per-lane 32-bit byte offset.
template <bool NT = false>
__device__ __forceinline__ void glds16(const void* sbase, uint32_t voff, uint32_t lds) {
  unsigned keep;
  if constexpr (NT)
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(sbase), "s"(lds)
        : "memory");
  else
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(sbase), "s"(lds)
        : "memory");
}

// Ablation only (MODE 11): the same LDS-DMA instruction moving 4 B per lane.
__device__ __forceinline__ void glds4(const void* sbase, uint32_t voff, uint32_t lds) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dword %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds)
      : "memory");
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  const uint32_t lo = __shfl((unsigned)(uint32_t)v, src, 64);
  const uint32_t hi = __shfl((unsigned)(uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}

// Inserts survivors into the per-query LDS lists of one 16-query group.
// Lane (col, kq) holds candidate bits `m` (bit b -> key_of(b)) for query
// column col; all 64 lanes must be active (wave-uniform call site). Each
// round takes one candidate per query (lowest kq lane, lowest bit); the
// query's four lanes then insert it together: lane kq holds entries
// 4kq .. 4kq+3 of the list `lst` (this query's 16 entries, q-major).
// Entries at positions >= k stay 0; a candidate ranking at position >= k
// changes nothing, so the list is always the top-min(k, n) of what was
// offered. Once the list is full, th_s rises to the score of its k-th key.
// `volatile` keeps every LDS access in program order across rounds (a wave's
// DS instructions execute in order); the pointer stays in LDS address space.
template <typename KeyOf>
__device__ __forceinline__ void mf_insert(uint32_t m, KeyOf key_of, lds_vu64_t* lst,
                                          uint32_t k, int lane, int col, int kq, float& th_s) {
  while (__any(m != 0)) {
    const uint64_t bal = __ballot(m != 0);
    const uint32_t qb = (uint32_t)((bal >> col) & 1) | (uint32_t)((bal >> (col + 15)) & 2) |
                        (uint32_t)((bal >> (col + 30)) & 4) | (uint32_t)((bal >> (col + 45)) & 8);
    const int sel = __builtin_ctz(qb | 16u);  // 4: no candidate for this query
    const uint64_t x = shfl64(key_of(__builtin_ctz(m | 256u)), col + 16 * (sel & 3));
    if (kq == sel) m &= m - 1;
    if (sel != 4) {  // uniform over the query's four lanes
      const uint32_t j0 = (uint32_t)(4 * kq);
      const uint64_t e0 = lst[j0], e1 = lst[j0 + 1], e2 = lst[j0 + 2], e3 = lst[j0 + 3];
      uint32_t gt = (uint32_t)(e0 > x) + (uint32_t)(e1 > x) + (uint32_t)(e2 > x) +
                    (uint32_t)(e3 > x);
      gt += __shfl_xor(gt, 16, 64);
      gt += __shfl_xor(gt, 32, 64);
      const uint64_t prev = shfl64(e3, lane >= 16 ? lane - 16 : lane);
      auto nv = [&](uint32_t j, uint64_t cur, uint64_t below) -> uint64_t {
        const uint64_t v = j < gt ? cur : (j == gt ? x : below);
        return j < k ? v : 0;
      };
      const uint64_t n0 = nv(j0, e0, prev), n1 = nv(j0 + 1, e1, e0), n2 = nv(j0 + 2, e2, e1),
                     n3 = nv(j0 + 3, e3, e2);
      if (gt < k) {
        lst[j0] = n0;
        lst[j0 + 1] = n1;
        lst[j0 + 2] = n2;
        lst[j0 + 3] = n3;
      }
      const int ks = (int)((k - 1) & 3);
      const uint64_t mk = ks == 0 ? n0 : (ks == 1 ? n1 : (ks == 2 ? n2 : n3));
      const uint64_t kth = shfl64(mk, col + 16 * (int)((k - 1) >> 2));
      if (kth) {
        const float ks_ = key_score(kth);
        th_s = ks_ > th_s ? ks_ : th_s;
      }
    }
  }
}

__device__ __forceinline__ int imax3(int a, int b, int c) {
  return __builtin_elementwise_max(__builtin_elementwise_max(a, b), c);
}

// I8 main pass: the integer dot threshold of query q. Rows whose upper bound
// U = sqS * dot + a * dmax + (c + sigma) * nmax is below b - sigma * nmax
// (b: the sample bound, a lower bound on the k-th score as computed by an
// fp32 pass) cannot be in the top k ("int8 prefilter"), so
// dot >= (b - a dmax - (c + 2 sigma) nmax) / sqS admits every row that can;
// one unit lower absorbs the float rounding of this expression.
template <typename Args>
__device__ __forceinline__ int q8_dot_threshold(const Args& a, uint32_t q, bool valid, float b) {
  if (!valid) return INT_MAX;
  if (b == -INFINITY) return INT_MIN + 2;  // no bound: every row
  const f32x4_t p = ((const f32x4_t*)a.q8par)[q];  // sqS, a, c, sigma
  const float dmax = a.q8glob[1], nmax = a.q8glob[2];
  if (!(p[0] > 0.f)) return INT_MIN + 2;  // a zero query: every dot is 0
  const float t = (b - p[1] * dmax - (p[2] + 2.f * p[3]) * nmax) / p[0] - 1.f;
  if (t <= -1073741824.f) return INT_MIN + 2;
  if (t >= 1073741824.f) return 1073741824;
  return (int)floorf(t);
}

// Raises this lane's running quarter maximum (LDS word `base` + tid of the
// main pass's counter area) to the slab maximum mx: a no-return ds_max_u32 on
// the order-preserving image (-0 ranked as +0, as vs::make_key does). Rare
// path; the thread id is taken opaque so no address is hoisted into the tile
// loop, and nothing waits on the atomic (the write-out's LDS read is ordered
// after it: one wave's LDS operations complete in order).
template <typename P>
__device__ __forceinline__ void mf_quarter_max(P cntl, uint32_t base, float mx) {
  uint32_t tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
  lds_u32_t* w = (lds_u32_t*)(cntl + base + tid);
  __hip_atomic_fetch_max(w, vs::score_ord(mx == 0.0f ? 0.0f : mx), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_WORKGROUP);
}

// A full quarter of a main-pass candidate buffer (slots [base, base + sub)):
// the new slab (scores v0, v1 of global tile row tile, masked maximum mx)
// replaces the slot whose masked maximum is smallest -- among equal maxima
// the latest tile (highest rows) -- if mx is larger. Exact for k <= sub:
// every slab dropped this way (or never stored) is beaten by sub >= k keys of
// distinct rows, one per slot kept (a larger score, or an equal score of an
// earlier, lower-row tile of this workgroup's ascending scan). Rare path: the
// slots' maxima are recomputed from the stored slabs (8 scores, the filter
// bits of their rows applied), so the append path stores no maximum.
template <typename Args>
__device__ __forceinline__ void mf_replace_min(const Args& a, uint32_t base, uint32_t sub,
                                               f32x4_t v0, f32x4_t v1, uint32_t tile, float mx) {
  // opaque: no address built from it is hoisted out of this rare path into
  // the tile loop (whose registers are all taken)
  asm volatile("" : "+v"(base));
  uint32_t tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const uint32_t kq = (tid & 63u) >> 4;  // this lane's rows 4kq+i and 16+4kq+i of a tile
  float msel = INFINITY;
  uint32_t tsel = 0, jsel = 0;
  for (uint32_t j = 0; j < sub; ++j) {
    const f32x4_t* sl = (const f32x4_t*)a.cand + 2 * (size_t)(base + j);
    const f32x4_t s0 = sl[0], s1 = sl[1];
    const uint32_t t = a.cand_tile[base + j];
    uint32_t am = 0xFFu;
    if (a.allow) {
      const uint32_t lr = t - a.row_base;  // local first row of the slot's tile
      const uint32_t tw = (uint32_t)(a.allow[lr >> 6] >> (lr & 32)) >> (4 * kq);
      am = (tw & 0xFu) | ((tw >> 12) & 0xF0u);
    }
    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      m = ((am >> i) & 1u) && s0[i] > m ? s0[i] : m;
      m = ((am >> (4 + i)) & 1u) && s1[i] > m ? s1[i] : m;
    }
    // selects, not branches: every load is consumed on every path
    const bool lt = m < msel || (m == msel && t > tsel);
    msel = lt ? m : msel;
    tsel = lt ? t : tsel;
    jsel = lt ? j : jsel;
  }
  if (mx > msel) {
    const size_t e = base + jsel;
    f32x4_t* sl = (f32x4_t*)a.cand + 2 * e;
    sl[0] = v0;
    sl[1] = v1;
    a.cand_tile[e] = tile;
  }
  // Leave no load of this path outstanding: the compiler's wait analysis
  // merges this path into the tile loop, and a pending load here became an
  // unconditional vmcnt(0) in the loop, draining the DMA ring every chunk
  // (+17% main pass, r02). vmcnt(0), expcnt / lgkmcnt untouched.
  __builtin_amdgcn_s_waitcnt(0x0F70);
}

template <bool B>
struct MfFull {
  static constexpr bool value = B;
};
template <int V>
struct MfSet {
  static constexpr int value = V;
};

// Byte geometry of the streamed rows (EB = element bytes: 2 bf16, 4 fp32).
// A step is 64 bytes of a row: 32 k of bf16 (one 16x16x32 MFMA per row half
// and query group) or 16 k of fp32 (four 16x16x4 MFMAs).
template <int D, int RING = kMfRingBytes, int TAIL = kMfListBytes, int WAVES = 8, int CSX = 0,
          int EB = 2>
struct MfShape {
  static constexpr int RBY = D * EB;                      // bytes per row
  static constexpr int T = RBY / 64;                      // 64-B MFMA steps per row
  // 128-B pieces per row per chunk (CSX overrides: ablation of chunk sizes)
  static constexpr int CS4 = CSX ? CSX : ((RBY % 512 == 0) ? 4 : 2);
  static constexpr int CT = CS4 * 2;                      // steps per chunk
  static constexpr int CPT = RBY / (128 * CS4);           // chunks per 32-row tile
  static constexpr int PIECES = CS4 * 4;                  // 1 KiB LDS-DMA pieces per chunk
  static constexpr int PPW = PIECES / WAVES;              // pieces per wave per chunk
  static constexpr int CHUNK_BYTES = PIECES * 1024;       // 32 rows x CS4*128 B
  static constexpr int NSLOT = RING / CHUNK_BYTES;
  static constexpr int AHEAD = NSLOT - 1;                 // chunks in flight
  static constexpr int LDS_BYTES = NSLOT * CHUNK_BYTES + TAIL;  // ring + lists / counters
  static_assert(RBY % 256 == 0, "MFMA scan needs whole 256-B row segments");
  static_assert(RBY % (128 * CS4) == 0, "whole chunks per tile");
  static_assert(AHEAD >= 2, "at least two chunks in the ring ahead");
  static_assert(PPW >= 1 && PPW * WAVES == PIECES, "pieces split evenly over waves");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

// MODE: 0 = main pass (candidate buffers), 3 = sample pass (tile maxima), 8 =
// main pass with sorted lists (overflow fallback). Ablation builds only
// (tools/ablate_mfma.hip): 1 = no top-k epilogue, 2 = LDS-DMA stream only,
// 4 = MFMA + LDS reads + barriers with no DMA, 5 = 4 without barriers, 6 =
// threshold filter only (never keeps a row), 7 = 1 with one A-fragment read
// per chunk, 10 = 1 reading only half the A fragments (the compiler then
// merges the two row halves' MFMA chains: invalid as a timing), 11 = 1 with
// 4-B LDS-DMA (a quarter of the bytes, same instructions), 13 = 1 with half
// the A-fragment reads and every MFMA kept (r02: -5.5% against 1; a K-split
// of query pairs that would halve the reads in the product needed 32
// accumulator VGPRs and spilled, and its spill-free form needs a shorter
// ring, which cost +2.4%: not kept). VAR 32 / 64: A fragments read 2 / 3 steps ahead instead of 1;
// VAR 128: each step's reads and MFMAs pinned in program order; VAR 512:
// the chunk's LDS-DMA pieces spread over its steps instead of at its head;
// VAR 1024: flips the corpus stream's load policy (MODE 0 default: non-temporal
// LDS-DMA; other modes: default policy). VAR 131072 (MODE 0): append counters
// in LDS instead of registers (the r01-v13 form).
// F32: fp32 rows and queries on v_mfma_f32_16x16x4_f32 (exact f32 products,
// fp32 accumulation; 1/16 of the bf16 rate, so the pass is MFMA-bound): same
// stream, layout and epilogue, a step's 16-B fragment holding 4 k of each
// lane's k-quarter, consumed by four MFMAs.
template <int D, int MODE = 0, int VAR = 0, int G = mf_groups(D), bool F32 = false, bool I8 = false>
__global__ __launch_bounds__(64 * mf_waves(G), mf_waves(G) == 4 ? 1 : 8 / mf_waves(G)) void mfma_topk_kernel(
    const MfArgs a) {
  constexpr int WAVES = mf_waves(G), THREADS = 64 * WAVES, QPW = 16 * G;
  constexpr int EB = F32 ? 4 : (I8 ? 1 : 2);
  static_assert(!I8 || (!F32 && (MODE == 0 || MODE == 1 || MODE == 6)), "int8: the main pass only");
  if (a.run_if && *a.run_if == 0u) return;  // uniform: the whole launch stands down
  constexpr int RBY = D * EB;
  static_assert(WAVES * QPW <= (int)kMfmaQueries, "one launch covers <= kMfmaQueries");
  static_assert(G * (RBY / 64) * 4 <= (mf_waves(G) == 4 ? 400 : 192),
                "B fragments must fit the register budget");
  // VAR 256: a 144 KiB ring (more chunks in flight); LDS lists only in MODE 8
  constexpr bool kBigRing = (VAR & 256) != 0 && MODE != 8;
  // VAR 2048 / 4096: 24 / 48 KiB K-chunks (384 / 768 k of 32 rows) at D = 768
  constexpr int kCsx = (VAR & 4096) ? 12 : ((VAR & 2048) ? 6 : 0);
  // candidate passes keep each lane's per-group append counters in LDS (a
  // register each would push the kernel past 256 VGPRs, and the compiler
  // then drops the A-fragment prefetch of the streaming loop: r01)
  // VAR 131072 (ablation): counters in LDS, and each lane's running quarter
  // maximum beside them (a second set), so cand_max is written in that form too
  constexpr bool kLdsCnt = MODE == 0 && (VAR & 131072) != 0;
  constexpr int kCntBytes = MODE == 0 ? 64 * WAVES * G * 4 * (kLdsCnt ? 2 : 1) : 0;
  using S = MfShape<D, kBigRing ? 144 * 1024 : kMfRingBytes,
                    MODE == 8 ? kMfListBytes : 16 + kCntBytes, WAVES, kCsx, EB>;
  constexpr bool kDma = MODE != 4 && MODE != 5;  // ablation modes without the stream
  constexpr bool kLists = MODE == 8;
  constexpr int PPW = S::PPW;
  constexpr int kPD0 = (VAR & 64) ? 3 : ((VAR & 32) ? 2 : 1);
  constexpr int kPD = ((S::CPT * S::CT) % (kPD0 + 1) == 0) ? kPD0 : 1;
  // each step's fragment reads + MFMAs kept in program order, so the one-step
  // prefetch survives scheduling (3.38 vs 3.63 ms at 10M rows); the sorted-list
  // pass would spill with it
  constexpr bool kPin = (VAR & 128) != 0 || MODE != 8;
  // VAR 4194304 (ablation, r03): instead of pinning a step's fragment reads
  // ahead of its MFMAs, ask the scheduler to interleave them: after every G
  // MFMAs one ds_read_b128 of a later step (sched_group_barrier), so the LDS
  // reads issue in the MFMA gaps rather than in one burst
  constexpr bool kIlvSched = (VAR & 4194304) != 0;
  // VAR 8192 (ablation): per-workgroup start / end wall clock into a.lists
  constexpr bool kClock = (VAR & 8192) != 0;
  uint64_t tclk0 = 0;
  if constexpr (kClock) tclk0 = wall_clock64();
  // ONE shared array: a second __shared__ object makes hipcc drain vmcnt
  // before LDS reads (cdna_hip_programming.md §5, trap 4(a)).
  __shared__ __attribute__((aligned(16))) unsigned char smem[S::LDS_BYTES];
  lds_vu64_t* lists = (lds_vu64_t*)(lds_ptr_t)(smem + S::NSLOT * S::CHUNK_BYTES);
  typedef __attribute__((address_space(3))) volatile uint32_t lds_vu32_t;
  lds_vu32_t* cntl = (lds_vu32_t*)(lds_ptr_t)(smem + S::NSLOT * S::CHUNK_BYTES + 16);

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 15;  // MFMA column (query in group) / A-fragment row
  const int kq = lane >> 4;   // 8-element k slice; C rows 4kq .. 4kq+3
  const uint32_t k = a.k;
  uint32_t wr0 = blockIdx.x * a.rows_per_wg;
  uint32_t wr1 = (uint64_t)wr0 + a.rows_per_wg < a.n_rows ? wr0 + a.rows_per_wg : a.n_rows;
  if (a.wg_tile) {  // a weighted split (per-XCD speeds)
    wr0 = a.wg_tile[blockIdx.x] * 32u;
    const uint64_t e = (uint64_t)a.wg_tile[blockIdx.x + 1] * 32u;
    wr1 = e < a.n_rows ? (uint32_t)e : a.n_rows;
  }
  uint32_t ntiles = (wr1 - wr0 + 31) / 32;
  if (a.max_tiles && ntiles > a.max_tiles) ntiles = a.max_tiles;
  const uint32_t nchunks = ntiles * S::CPT;
  const uint32_t tstride = gridDim.x * a.max_tiles;  // MODE 3: tile maxima per query

  if constexpr (kLists)
    for (int i = threadIdx.x; i < (int)kMfmaQueries * kMfListLen; i += THREADS) lists[i] = 0;

  // LDS-DMA source mapping: piece (s4l, rg) of a chunk holds rows rg*8 ..
  // rg*8+7, bytes [128*s4, 128*s4+128) of each; lane -> (row lane>>3,
  // 16-B position lane&7 holding chunk (lane&7) ^ swz). The per-lane part of
  // each piece's address is a loop-invariant 32-bit offset; the per-chunk part
  // is a scalar base advanced chunk by chunk (the chunk issued at step c is
  // c + AHEAD). Tiles past the last row read the collection's 32 rows of
  // allocation padding (vs_engine.cpp grow()) and are masked in the epilogue.
  constexpr bool kNtDma = (MODE == 0) != ((VAR & 1024) != 0);
  const uint32_t lds_base = (uint32_t)(uintptr_t)(lds_ptr_t)smem;
  uint32_t loff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int b = w + WAVES * i;
    const int s4l = b >> 2, rg = b & 3;
    const int g_ri = lane >> 3, c16 = (lane & 7) ^ mf_swz(g_ri, rg);
    loff[i] = (uint32_t)((rg * 8 + g_ri) * RBY + s4l * 128 + c16 * 16);
  }
  constexpr bool kSpread = (VAR & 512) != 0;  // pieces spread over the chunk's steps
  const unsigned char* xnext = (const unsigned char*)a.X + (size_t)wr0 * RBY;  // next chunk to issue
  uint32_t unext = 0;     // its chunk index within the tile
  uint32_t snext = 0;     // its ring slot byte offset
  auto issue_piece = [&](int i) {
    const int b = w + WAVES * i;
    const int s4l = b >> 2, rg = b & 3;
    if constexpr (MODE == 11)
      glds4(xnext, loff[i], lds_base + snext + (uint32_t)((s4l * 4 + rg) * 1024));
    else
      glds16<kNtDma>(xnext, loff[i], lds_base + snext + (uint32_t)((s4l * 4 + rg) * 1024));
  };
  auto advance = [&]() {
    const bool last = unext == S::CPT - 1;
    xnext += last ? (size_t)(32 * RBY - (S::CPT - 1) * S::CS4 * 128) : (size_t)S::CS4 * 128;
    unext = last ? 0 : unext + 1;
    snext = snext + S::CHUNK_BYTES == (uint32_t)(S::NSLOT * S::CHUNK_BYTES) ? 0
                                                                           : snext + S::CHUNK_BYTES;
  };
  auto issue_next = [&]() {
#pragma unroll
    for (int i = 0; i < PPW; ++i) issue_piece(i);
    advance();
  };
  // Branch-free stream (default of the product passes, MODE 0 / 3 / 8; VAR
  // 524288 flips it: back to the conditional stream, or on for ablation
  // modes; r02: main pass -2.5 to -3.2% at 10M / 1.25M rows, back to back).
  // Every chunk step issues its pieces: past
  // the last chunk they re-read the workgroup's first chunk (valid memory, an
  // L2 hit) into the slot being refilled, which is never read again; so the
  // vmcnt waits are the same every step (no branches in the chunk loop, which
  // let hipcc's waitcnt pass keep the fragment reads' order: lgkmcnt(2), not
  // lgkmcnt(0), before a chunk's first MFMAs). Drained before the exit.
  constexpr bool kBF = (((VAR & 524288) != 0) != (MODE == 0 || MODE == 3 || MODE == 8)) && !kSpread;
  // The dummy pieces past the last chunk all read the pass's FIRST chunk (the
  // same bytes for every workgroup: L2 hits after one miss per XCD). r05: each
  // workgroup re-read its own first chunk, which the stream had long evicted:
  // AHEAD x 24 KiB x 256 workgroups of HBM re-reads, +2.2% of the traffic at
  // the N = 8 share (profiles/pmc_traffic.json c3_i8@1250000, build 67398432).
  const unsigned char* const xsafe = (const unsigned char*)a.X;
  auto bf_src = [&](bool real) -> const unsigned char* {
    // wave-uniform by construction; readfirstlane keeps it in SGPRs for the
    // asm's "s" operand whatever the divergence analysis concludes
    const uint64_t sp = (uint64_t)(uintptr_t)(real ? xnext : xsafe);
    return (const unsigned char*)(uintptr_t)(
        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(sp >> 32)) << 32) |
        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sp));
  };
  auto bf_piece = [&](const unsigned char* src, int i) {
    const int b = w + WAVES * i;
    const int s4l = b >> 2, rg = b & 3;
    glds16<kNtDma>(src, loff[i],
                   (uint32_t)__builtin_amdgcn_readfirstlane(
                       (int)(lds_base + snext + (uint32_t)((s4l * 4 + rg) * 1024))));
  };
  auto issue_next_bf = [&](bool real) {
    const unsigned char* src = bf_src(real);
#pragma unroll
    for (int i = 0; i < PPW; ++i) bf_piece(src, i);
    advance();
  };
  // VAR 8388608 (r04): the ring's first AHEAD chunks are issued before the
  // query-fragment prologue instead of after it, so the corpus fill (~5 us at
  // ~25 GB/s per CU) overlaps the ~6 us of B-fragment loads from L2 that every
  // launch starts with; the prologue's vmcnt(0) drain then covers both.
  constexpr bool kEarlyFill = (VAR & 8388608) != 0;
  // VAR 33554432 (r05, int8 pass): one barrier per PAIR of chunks (tiles: a
  // 24 KiB chunk is one 32-row tile of 768-B int8 rows) instead of one per
  // chunk, and the two freed slots refilled at once. With 6 slots: before the
  // barrier of the pair (c, c + 1) chunks up to c + 2 have landed (c + 3 may
  // pend), the barrier frees the previous pair's slots, and chunks c + 4,
  // c + 5 are issued into them (4 chunks ahead instead of 5). The per-tile
  // fixed cost (wait, barrier, DMA issue) is half the int8 pass's 48 MFMAs
  // per wave and tile where the bf16 pass had 96.
  constexpr bool kPair = (VAR & 33554432) != 0 && kBF && S::CPT == 1 && S::NSLOT == 6 &&
                         (VAR & 1048576) == 0 && kDma;
  constexpr uint32_t kFill = kPair ? (uint32_t)S::AHEAD - 1 : (uint32_t)S::AHEAD;
  // VAR 16384 (r05, ablation): the branch-free stream's pieces of a chunk
  // spread over its steps -- piece 0 after the barrier, piece i after step
  // i * CT / PPW -- instead of all PPW back to back after the barrier, where
  // both waves of a SIMD issue theirs while the matrix pipe waits. Same
  // slots and waits: every piece of chunk c + AHEAD is issued before the
  // next chunk's vmcnt wait counts them.
  constexpr bool kBFSpread = (VAR & 16384) != 0 && kBF && !kPair && (VAR & 1048576) == 0 && kDma &&
                             PPW > 1 && S::CT >= PPW;
  const unsigned char* bf_cur = xsafe;  // (kBFSpread) the chunk being issued
  if constexpr (kDma && kBF && kEarlyFill) {
#pragma unroll
    for (uint32_t c = 0; c < kFill; ++c) issue_next_bf(c < nchunks);
  }
  // B operand of group g: Q[query 32w+16g+col][32t + 8kq + j], j = 0..7.
  bf16x8_t qf[G][S::T];
  uint32_t ql[G];
  bool qvalid[G];
  float th_s[G];     // admit rows whose score reaches th_s
  int th_i[G];       // I8: admit rows whose int8 dot reaches th_i
  // cntl[g * THREADS + tid]: keys this lane appended to its quarter of the
  // query's buffer (candidate passes). The main pass keeps the counts and
  // each lane's first slot in registers instead (no LDS round trip and no
  // address rebuild in the append path; 256 VGPRs, no spill), and streams the
  // corpus non-temporally: back to back, -2.0% at 1.25M rows and -1.2% at 10M
  // against LDS counters and default-policy DMA (r01, 2 x 40 / 16 reps).
  constexpr bool kRegCnt = MODE == 0 && (VAR & 131072) == 0;
  uint32_t cnt_r[G], slot0[G];
  int qmx_r[G];  // I8: the largest dot this lane appended (INT_MIN: none)
#pragma unroll
  for (int g = 0; g < G; ++g) {
    qmx_r[g] = INT_MIN;
    // (the register-count main pass keeps each lane's running quarter maximum
    // here instead: score_ord of the largest admitted score, 0 = none)
    if constexpr (kCntBytes > 0) cntl[g * THREADS + threadIdx.x] = 0u;
    if constexpr (kLdsCnt) cntl[(G + g) * THREADS + threadIdx.x] = 0u;
    if constexpr (kRegCnt) {
      cnt_r[g] = 0u;
      slot0[g] = (uint32_t)(((size_t)blockIdx.x * kMfmaQueries +
                             (uint32_t)(w * QPW + g * 16 + col)) * a.cand_cap +
                            (uint32_t)kq * (a.cand_cap >> 2));
    }
    ql[g] = (uint32_t)(w * QPW + g * 16 + col);
    qvalid[g] = ql[g] < a.nq_valid;
    const uint4* qrow = (const uint4*)((const unsigned char*)a.Q + (size_t)ql[g] * RBY);
#pragma unroll
    for (int t = 0; t < S::T; ++t) qf[g][t] = __builtin_bit_cast(bf16x8_t, qrow[4 * t + kq]);
    th_s[g] = (a.init_score && qvalid[g]) ? a.init_score[ql[g]] : -INFINITY;
    if constexpr (I8) th_i[g] = q8_dot_threshold(a, ql[g], qvalid[g], th_s[g]);
  }

  // VAR 8192: the prologue's loads drained and timed (ablation only)
  uint64_t tclk1 = 0, tclk2 = 0;
  if constexpr (kClock) {
    __builtin_amdgcn_s_waitcnt(0);
    tclk1 = wall_clock64();
  }

  // A operand read offsets: half hr (tile rows 16hr..16hr+15), lane reads row
  // 16hr + col, 16-B chunk 4*(t&1) + kq of piece t>>1.
  int off[2][2];
#pragma unroll
  for (int hr = 0; hr < 2; ++hr) {
    const int rr = 16 * hr + col, rg = rr >> 3, ri = rr & 7, sw = mf_swz(ri, rg);
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) off[hr][tt] = rg * 1024 + ri * 128 + (((4 * tt + kq) ^ sw) << 4);
  }
  auto lds_a = [&](const unsigned char* sb, int s, int hr) -> bf16x8_t {
    return __builtin_bit_cast(bf16x8_t, *(const uint4*)(sb + (s >> 1) * 4096 + off[hr][s & 1]));
  };

  // The query fragments and bounds are loads the compiler's waitcnt pass
  // tracks; drain them here with the builtin (which the pass sees), so it
  // does not place vmcnt waits for them inside the loop, where the hardware
  // counter also holds the ring's LDS-DMA pieces (invisible to the pass).
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), expcnt/lgkmcnt untouched
  if constexpr (MODE == 12) {  // ablation: the prologue's query-fragment loads only
#pragma unroll
    for (int g = 0; g < G; ++g) asm volatile("" ::"v"(qf[g][0]), "v"(qf[g][S::T - 1]));
    return;
  }
  __syncthreads();  // lists / counts initialised
  if constexpr (kDma && kBF) {
    if constexpr (!kEarlyFill) {
#pragma unroll
      for (uint32_t c = 0; c < kFill; ++c) issue_next_bf(c < nchunks);
    }
    wait_vmcnt<PPW * (kFill - 1)>();
  } else {
    if constexpr (kDma)
      for (uint32_t c = 0; c < (uint32_t)S::AHEAD; ++c)
        if (c < nchunks) issue_next();
    // publish chunk 0
    if ((uint32_t)S::AHEAD <= nchunks)
      wait_vmcnt<PPW * (S::AHEAD - 1)>();
    else
      wait_vmcnt<0>();
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  // A fragments are read PD 32-k steps ahead of their MFMAs, across chunk
  // boundaries inside a tile: chunk c+1 is published by the barrier at the
  // head of chunk c, so the reads for the first PD steps of chunk c+1 are
  // issued during the last steps of chunk c. A tile's first PD steps are
  // read after the previous tile's epilogue, before the first barrier (its
  // chunk was published one barrier earlier), so no fragment is live across
  // the epilogue. NB = PD + 1 register sets rotate with the step index,
  // which repeats every tile because NB divides the steps per tile.
  constexpr int STEPS = S::CPT * S::CT;
  constexpr int NB = kPD + 1;
  static_assert(STEPS % NB == 0, "A-fragment ring must divide the steps per tile");
  uint32_t scur = 0;  // ring slot byte offset of chunk c
  // Candidate passes instantiate a tile's body twice: full 32-row tiles get a
  // straight-line epilogue; the (at most one) partial last tile masks rows.
  // The sorted-list pass keeps one body with a runtime test (its register
  // allocation with the peeled form spilled; r01).
  constexpr bool kPeel = MODE != 8;
  // VAR 1048576 (with the branch-free stream): waves 4-7 run half a chunk
  // ahead of their SIMD partners 0-3. Their per-chunk wait + barrier + DMA
  // issue sits between steps CT/2 - 1 and CT/2 of the chunk instead of before
  // step 0 (same barrier count, same slots: a wave only reads chunks the
  // barrier before its steps published, and the slot refilled at barrier c,
  // chunk c - 1's, is done for every wave), so the two waves of a SIMD reach
  // their LDS-read bursts and barriers half a chunk apart instead of in
  // lockstep (MI355X_MICROARCH.md, two waves per SIMD, item 9).
  constexpr bool kStag = (VAR & 1048576) != 0 && kBF && WAVES == 8;
  // int8 pass epilogue of one tile (accumulators ac, first row trow0): a lane
  // whose largest dot of the tile reaches the query's integer threshold
  // appends its 8 dots (int32 bits) -- the select bounds and rescores them.
  // Padding and filtered-out rows (the pre-mask) are INT_MIN in the slab:
  // never a maximum, never a survivor.
  // (r05) split in two halves, so the deferred form below can place them in
  // different MFMA steps: q8_epi_mx masks query group g's dots of the tile
  // (padding / filtered rows -> INT_MIN, in ac) and returns their maximum;
  // q8_epi_app appends them when that reaches the group's threshold.
  auto q8_epi_am = [&](uint32_t trow0) -> uint32_t {
    uint32_t am = 0xFFu;
    if (a.allow) {
      const uint32_t tw = (uint32_t)(a.allow[trow0 >> 6] >> (trow0 & 32)) >> (4 * kq);
      am = (tw & 0xFu) | ((tw >> 12) & 0xF0u);
    }
    return am;
  };
  // (may_filter false: the caller knows a.allow is null -- the split form)
  auto q8_epi_mx = [&](f32x4_t (&ac)[2][G], int g, uint32_t trow0, bool full, uint32_t am,
                       bool may_filter = true) -> int {
    // whole-vector bit casts: this hipcc miscompiles __builtin_bit_cast of
    // one ext_vector element (it reads element 0; tools/q8_check.hip found it)
    const i32x4_t a0 = __builtin_bit_cast(i32x4_t, ac[0][g]);
    const i32x4_t a1 = __builtin_bit_cast(i32x4_t, ac[1][g]);
    int v[8];
#pragma unroll
    for (int b = 0; b < 4; ++b) v[b] = a0[b], v[4 + b] = a1[b];
    if (!full || (may_filter && a.allow)) {  // uniform: unfiltered full tiles skip it
      // the row base and mask bits are taken opaque inside the branch: the
      // compiler otherwise hoists their 16 adds/ands into every unfiltered
      // full tile (r05 ISA: 17 of the epilogue's 38 VALU per tile)
      uint32_t rb = trow0 + 4 * kq, amv = am;
      asm volatile("" : "+v"(rb), "+v"(amv));
#pragma unroll
      for (int b = 0; b < 8; ++b)
        if (rb + 16 * (b >> 2) + (b & 3) >= wr1 || !((amv >> b) & 1u)) v[b] = INT_MIN;
      ac[0][g] = __builtin_bit_cast(f32x4_t, i32x4_t{v[0], v[1], v[2], v[3]});
      ac[1][g] = __builtin_bit_cast(f32x4_t, i32x4_t{v[4], v[5], v[6], v[7]});
    }
    return imax3(imax3(v[0], v[1], v[2]), imax3(v[3], v[4], v[5]), imax3(v[6], v[7], INT_MIN));
  };
  auto q8_epi_app = [&](f32x4_t (&ac)[2][G], int g, uint32_t trow0, int mx) {
    // VAR 16777216 (timing ablation only, wrong answers): never append
    if ((VAR & 16777216) != 0) {
      asm volatile("" ::"v"(mx >= th_i[g]));
      return;
    }
    if (mx >= th_i[g]) {  // th_i > INT_MIN: padding never passes; invalid queries: INT_MAX
      const uint32_t sub = a.cand_cap >> 2;
      const uint32_t cg = cnt_r[g];
      // r05: a full quarter keeps counting (a count past its capacity
      // marks it lossy: select_q8 recomputes its rows from the int8
      // copy) and its largest dot stays exact; no hand-back
      if (cg < sub) {
        const size_t slot = (size_t)slot0[g] + cg;
        f32x4_t* sp = (f32x4_t*)a.cand + 2 * slot;
        sp[0] = ac[0][g];
        sp[1] = ac[1][g];
        a.cand_tile[slot] = a.row_base + trow0;
      }
      cnt_r[g] = cg + 1;
      qmx_r[g] = mx > qmx_r[g] ? mx : qmx_r[g];
    }
  };
  auto q8_epi = [&](f32x4_t (&ac)[2][G], uint32_t trow0, bool full) {
    const uint32_t am = q8_epi_am(trow0);
#pragma unroll
    for (int g = 0; g < G; ++g) q8_epi_app(ac, g, trow0, q8_epi_mx(ac, g, trow0, full, am));
  };
  // VAR 67108864 (r05, int8 pass): the epilogue of tile t runs after the first
  // step's MFMAs of tile t + 1, on the other of two accumulator sets, so its
  // VALU work and its wait for the tile's last MFMA results overlap the
  // matrix pipe instead of stalling it at every tile's end
  constexpr bool kEpiPipe = I8 && MODE == 0 && (VAR & 67108864) != 0;
  f32x4_t accq[kEpiPipe ? 2 : 1][2][G];
  uint32_t prow0 = 0;
  bool pfull = true, have_prev = false;
  // VAR 65536 (r05, with 67108864): the deferred epilogue split over the next
  // tile's steps -- group g's maximum after step 1 + g, the appends after
  // step G + 1 -- so its compares sit in the MFMA steps' issue gaps instead
  // of one block. Only full tiles are deferred (a partial last tile runs its
  // own at once); the first tile's "previous" set starts as INT_MIN dots,
  // which never pass, so no step tests whether a previous tile exists.
  constexpr bool kEpiSplit = kEpiPipe && (VAR & 65536) != 0;
  // (the launcher runs this form only without a filter: a.allow is null)
  int mxp[G];
  if constexpr (kEpiSplit) {
#pragma unroll
    for (int hr = 0; hr < 2; ++hr)
#pragma unroll
      for (int g = 0; g < G; ++g) {
        accq[1][hr][g] = __builtin_bit_cast(f32x4_t, i32x4_t{INT_MIN, INT_MIN, INT_MIN, INT_MIN});
        mxp[g] = INT_MIN;
      }
    prow0 = wr0;
  }
  // VAR 32768 (r05, ablation): a tile's first PD A-fragment reads are issued
  // at the end of the previous tile, before its epilogue (the next tile's
  // first chunk was published by the barrier at the head of this tile's last
  // chunk), so their LDS latency overlaps the epilogue instead of opening
  // the next tile after its barrier
  constexpr bool kPreA = (VAR & 32768) != 0 && MODE != 2 && MODE != 7 && !kStag;
  constexpr int kAH = MODE == 10 || MODE == 13 ? 1 : 2;
  bf16x8_t afr_k[NB][2];
  auto read_first = [&]() {
#pragma unroll
    for (int p = 0; p < kPD; ++p)
#pragma unroll
      for (int hr = 0; hr < kAH; ++hr) afr_k[p][hr] = lds_a(smem + scur, p, hr);
  };
  auto tile = [&](uint32_t t, auto full_tag, auto stag_tag, auto set_tag) {
    constexpr bool STAG = decltype(stag_tag)::value;
    constexpr int SET = decltype(set_tag)::value;
    constexpr int SYNC_STEP = STAG ? S::CT / 2 : 0;
    f32x4_t (&acc)[2][G] = accq[kEpiPipe ? SET : 0];  // [row half][query group]
#pragma unroll
    for (int hr = 0; hr < 2; ++hr)
#pragma unroll
      for (int g = 0; g < G; ++g) acc[hr][g] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    bf16x8_t afr_l[NB][2];
    bf16x8_t(&afr)[NB][2] = *(kPreA ? &afr_k : &afr_l);
#pragma unroll
    for (int u = 0; u < S::CPT; ++u) {
      const uint32_t c = t * S::CPT + u;
      const uint32_t snxt =
          scur + S::CHUNK_BYTES == (uint32_t)(S::NSLOT * S::CHUNK_BYTES) ? 0 : scur + S::CHUNK_BYTES;
      const unsigned char* sb = smem + scur;
      const unsigned char* sbn = smem + snxt;
      if (MODE != 2 && u == 0 && !kPreA) {
#pragma unroll
        for (int p = 0; p < kPD; ++p)
#pragma unroll
          for (int hr = 0; hr < (MODE == 10 || MODE == 13 ? 1 : 2); ++hr) afr[p][hr] = lds_a(sb, p, hr);
      }
      const bool refill = kDma && c + S::AHEAD < nchunks;
      auto sync_chunk = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        // chunk c+1 landed for this wave: chunks c+2 .. c+AHEAD-1 may pend
        // (pairs: chunks up to c+2 landed, c+3 may pend)
        if constexpr (kPair) {
          wait_vmcnt<PPW>();
        } else if constexpr (kDma && kBF) {
          wait_vmcnt<PPW * (S::AHEAD - 2)>();
        } else if constexpr (kDma) {
          if (c + S::AHEAD <= nchunks)
            wait_vmcnt<PPW * (S::AHEAD - 2)>();
          else
            wait_vmcnt<0>();
        }
        // VAR 134217728 (timing ablation only: the ring is then unsynchronised
        // and the results garbage): no barrier at all
        if constexpr (MODE != 5 && (VAR & 134217728) == 0)
          __builtin_amdgcn_s_barrier();  // chunk c+1 visible; slot c-1 free
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (kPair) {
          issue_next_bf(c + 4 < nchunks);
          issue_next_bf(c + 5 < nchunks);
        } else if constexpr (kBFSpread) {
          bf_cur = bf_src(refill);
          bf_piece(bf_cur, 0);
        } else if constexpr (kDma && kBF) {
          issue_next_bf(refill);
        } else if (!kSpread && refill) {
          issue_next();
        }
      };
      if constexpr (kPair) {
        if ((c & 1u) == 0) sync_chunk();  // uniform
      } else if constexpr (!STAG || MODE == 2) {
        sync_chunk();
      }
      if constexpr (MODE != 2) {
#pragma unroll
        for (int s = 0; s < S::CT; ++s) {
          if constexpr (STAG) {
            if (s == SYNC_STEP) sync_chunk();
          }
          const int sig = u * S::CT + s;
          // prefetch step sig + PD (this chunk or the next one)
          if (MODE != 7 && sig + kPD < STEPS) {
            const int sp = s + kPD;
#pragma unroll
            for (int hr = 0; hr < (MODE == 10 || MODE == 13 ? 1 : 2); ++hr)
              afr[(sig + kPD) % NB][hr] =
                  sp < S::CT ? lds_a(sb, sp, hr) : lds_a(sbn, sp - S::CT, hr);
          }
          if constexpr (kPin && !kIlvSched) __builtin_amdgcn_sched_barrier(0);
          if constexpr (F32) {
            // lane (col, kq) holds k = 16 step + 4 kq + j in element j of both
            // fragments: MFMA j sums those k over the four lane quarters
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
              for (int hr = 0; hr < 2; ++hr) {
                const f32x4_t av = __builtin_bit_cast(f32x4_t, afr[sig % NB][hr]);
#pragma unroll
                for (int g = 0; g < G; ++g) {
                  const f32x4_t bv = __builtin_bit_cast(f32x4_t, qf[g][u * S::CT + s]);
                  acc[hr][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], bv[j], acc[hr][g], 0, 0,
                                                                    0);
                }
              }
          } else {
#pragma unroll
            for (int hr = 0; hr < 2; ++hr) {
              const bf16x8_t av = afr[MODE == 7 ? 0 : sig % NB][MODE == 10 || MODE == 13 ? 0 : hr];
#pragma unroll
              for (int g = 0; g < G; ++g) {
                // MODE 13 (ablation): half the A reads with every MFMA kept --
                // row half 1 reuses half 0's fragment against the next step's
                // query fragment (a distinct chain, so nothing merges)
                const int qs = MODE == 13 && hr == 1 ? (sig + 1) % S::T : sig;
                if constexpr (I8)  // 64 int8 k per step; exact int32 sums (bits kept in acc)
                  acc[hr][g] = __builtin_bit_cast(
                      f32x4_t, __builtin_amdgcn_mfma_i32_16x16x64_i8(
                                   __builtin_bit_cast(i32x4_t, av),
                                   __builtin_bit_cast(i32x4_t, qf[g][qs]),
                                   __builtin_bit_cast(i32x4_t, acc[hr][g]), 0, 0, 0));
                else
                  acc[hr][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, qf[g][qs], acc[hr][g], 0,
                                                                       0, 0);
              }
            }
          }
          if constexpr (kIlvSched) {
#pragma unroll
            for (int hr = 0; hr < 2; ++hr) {
              __builtin_amdgcn_sched_group_barrier(0x008, G, 0);  // G MFMAs
              __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one DS read
            }
          }
          if constexpr (kPin) __builtin_amdgcn_sched_barrier(0);
          if constexpr (kEpiSplit) {
            if (u == 0) {  // compile-time: u, s unrolled
              if (s >= 1 && s <= G)
                mxp[s - 1] = q8_epi_mx(accq[1 - SET], s - 1, prow0, true, 0xFFu, false);
              if (s == G + 1) {
#pragma unroll
                for (int g = 0; g < G; ++g) q8_epi_app(accq[1 - SET], g, prow0, mxp[g]);
              }
            }
          } else if constexpr (kEpiPipe) {
            if (u == 0 && s == 0 && have_prev) {
              q8_epi(accq[1 - SET], prow0, pfull);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
          if constexpr (kBFSpread) {
#pragma unroll
            for (int i = 1; i < PPW; ++i)
              if (s == (i * S::CT) / PPW) {
                bf_piece(bf_cur, i);
                if (i == PPW - 1) advance();
              }
          }
          if constexpr (kSpread) {
            // piece i after step i * CT / PPW (the last one also advances)
#pragma unroll
            for (int i = 0; i < PPW; ++i)
              if (s == (i * S::CT) / PPW && refill) {
                issue_piece(i);
                if (i == PPW - 1) advance();
              }
          }
        }
      }
      scur = snxt;
    }
    if constexpr (kPreA) read_first();  // the next tile's (past the last: unused)
    if constexpr (MODE == 1 || MODE == 2 || MODE == 4 || MODE == 5 || MODE == 7 || MODE == 10 ||
                  MODE == 11 || MODE == 13) {
#pragma unroll
      for (int hr = 0; hr < 2; ++hr)
#pragma unroll
        for (int g = 0; g < G; ++g) asm volatile("" ::"v"(acc[hr][g][hr * 2 + (g & 1)]));
      return;
    }
    // epilogue: acc[hr][g][i] = score(row trow0 + 16hr + 4kq + i, query ql[g])
    const uint32_t trow0 = wr0 + t * 32;
    const bool full = kPeel ? decltype(full_tag)::value : trow0 + 32 <= wr1;
    // filter pre-mask: the tile's 32 rows are one half of a 64-row word
    // (trow0 % 32 == 0); a lane's rows 4kq+i and 16+4kq+i are bits i and 4+i
    // of am. Masked rows score -inf and never pass.
    uint32_t am = 0xFFu;
    if (a.allow && !(I8 && MODE == 0)) {
      const uint32_t tw = (uint32_t)(a.allow[trow0 >> 6] >> (trow0 & 32)) >> (4 * kq);
      am = (tw & 0xFu) | ((tw >> 12) & 0xF0u);
      // the main pass leaves its accumulators as they are (the slab's masked
      // rows are dropped by the select, which reads the same mask): a
      // conditional rewrite here costs a copy of all 16 every tile
      if constexpr (MODE != 0) {
#pragma unroll
        for (int hr = 0; hr < 2; ++hr)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int g = 0; g < G; ++g)
              acc[hr][g][i] = ((am >> (hr * 4 + i)) & 1u) ? acc[hr][g][i] : -INFINITY;
      }
    }
    if constexpr (I8 && MODE == 0) {
      if constexpr (kEpiSplit) {  // full tiles: in the next tile's steps (or at the end)
        if (full)
          prow0 = trow0;
        else
          q8_epi(acc, trow0, false);
      } else if constexpr (kEpiPipe) {  // run after the next tile's first step (or at the end)
        prow0 = trow0, pfull = full, have_prev = true;
      } else {
        q8_epi(acc, trow0, full);
      }
      return;
    } else if constexpr (I8) {
#pragma unroll
      for (int g = 0; g < G; ++g) asm volatile("" ::"v"(acc[0][g][0]), "v"(acc[1][g][3]));
      return;
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float mx = -INFINITY;
      if (MODE == 0 && full && a.allow) {
        // the mask bits are taken opaque inside the branch, so their tests
        // are not hoisted into every unfiltered tile
        uint32_t amv = am;
        asm volatile("" : "+v"(amv));
        float v[8];
#pragma unroll
        for (int b = 0; b < 8; ++b)
          v[b] = ((amv >> b) & 1u) ? acc[b >> 2][g][b & 3] : -INFINITY;
        mx = fmax3(fmax3(v[0], v[1], v[2]), fmax3(v[3], v[4], v[5]), fmax3(v[6], v[7], -INFINITY));
      } else if (full) {
        mx = fmax3(fmax3(acc[0][g][0], acc[0][g][1], acc[0][g][2]),
                   fmax3(acc[0][g][3], acc[1][g][0], acc[1][g][1]),
                   fmax3(acc[1][g][2], acc[1][g][3], -INFINITY));
      } else {
#pragma unroll
        for (int hr = 0; hr < 2; ++hr)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t row = trow0 + 16 * hr + 4 * kq + i;
            if constexpr (MODE == 0) {  // padding / masked rows leave the slab as -inf
              if (row >= wr1 || !((am >> (hr * 4 + i)) & 1u)) acc[hr][g][i] = -INFINITY;
            }
            if (row < wr1 && acc[hr][g][i] > mx) mx = acc[hr][g][i];
          }
      }
      if constexpr (MODE == 0) {
        // Main pass: a lane whose max reaches the bound appends its whole
        // 8-score slab (the two accumulators as they are) and the tile's first
        // row to its quarter of the query's buffer; select_cand_kernel expands
        // slabs into keys. No per-row mask, key packing or loop here: the rare
        // path is a few instructions, and any wave in it holds up the other
        // seven at the next chunk barrier (r01: -0.12 ms at 1.25M rows).
        if (qvalid[g] && mx >= th_s[g] && mx != -INFINITY) {
          const uint32_t sub = a.cand_cap >> 2;
          const uint32_t cg = kRegCnt ? cnt_r[g] : cntl[g * THREADS + threadIdx.x];
          if (cg >= sub) {
            // VAR 131072 (LDS counters, ablation only) drops the slab: inexact
            // The quarter is full (many near-equal rows): keep the sub slabs
            // with the largest maximum keys. A slab this evicts (or never
            // stores) has a maximum key below those of all sub slabs kept,
            // i.e. below sub >= k keys of distinct rows, so none of its rows
            // can be in the top k (mfma_cand_cap gives sub >= k): exact, with
            // no re-run. Rare path: the slabs are read back from memory.
            // VAR 2097152 (ablation): drops the slab, inexact
            if constexpr (kRegCnt && (VAR & 2097152) == 0) {
              mf_replace_min(a, slot0[g], sub, acc[0][g], acc[1][g], a.row_base + trow0, mx);
              // the quarter's maximum never leaves it (a replacement evicts the
              // smallest), so the running maximum stays exact
              mf_quarter_max(cntl, g * THREADS, mx);
            }
          } else if constexpr (kRegCnt) {
            // VAR 262144 (ablation): the appending wave runs at raised
            // priority, so it reaches the next chunk barrier sooner
            if constexpr ((VAR & 262144) != 0) __builtin_amdgcn_s_setprio(3);
            const size_t slot = (size_t)slot0[g] + cg;
            f32x4_t* sp = (f32x4_t*)a.cand + 2 * slot;
            sp[0] = acc[0][g];
            sp[1] = acc[1][g];
            a.cand_tile[slot] = a.row_base + trow0;
            cnt_r[g] = cg + 1;
            mf_quarter_max(cntl, g * THREADS, mx);
            if constexpr ((VAR & 262144) != 0) __builtin_amdgcn_s_setprio(0);
          } else {
            // the address is rebuilt here from an opaque thread id, so none
            // of it is hoisted out of the tile loop (its register budget)
            uint32_t tid = threadIdx.x;
            asm volatile("" : "+v"(tid));
            // layout [wg][query][cap], a quarter = sub slots: a workgroup's
            // stores stay in its own region (a query-major layout spread each
            // wave's stores over 16 regions 0.5 MiB apart: +4% main pass, r01)
            const uint32_t qo = (tid >> 6) * QPW + g * 16 + (tid & 15);
            const size_t slot = ((size_t)blockIdx.x * kMfmaQueries + qo) * a.cand_cap +
                                ((tid & 63) >> 4) * sub + cg;
            f32x4_t* sp = (f32x4_t*)a.cand + 2 * slot;
            sp[0] = acc[0][g];
            sp[1] = acc[1][g];
            a.cand_tile[slot] = a.row_base + trow0;
            cntl[g * THREADS + threadIdx.x] = cg + 1;
            mf_quarter_max(cntl, (G + g) * THREADS, mx);
          }
        }
        continue;
      }
      // sample pass: the tile maximum per query (the 4 lane quarters'
      // maxima), one float per (query, tile): no keys, ballots or counters
      if constexpr (MODE == 3) {
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        if (kq == 0 && qvalid[g])
          a.tmax[(size_t)ql[g] * tstride + (size_t)blockIdx.x * a.max_tiles + t] = mx;
        continue;
      }
      if constexpr (MODE == 6) {
        asm volatile("" ::"v"(mx));
        continue;
      }
      const float lvl = th_s[g];
      if (__any(qvalid[g] && mx >= lvl)) {
        uint32_t m = 0;
#pragma unroll
        for (int hr = 0; hr < 2; ++hr)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t row = trow0 + 16 * hr + 4 * kq + i;
            const bool p = qvalid[g] && (full || row < wr1) && ((am >> (hr * 4 + i)) & 1u) &&
                           acc[hr][g][i] >= lvl;
            m |= (uint32_t)p << (hr * 4 + i);
          }
        auto key_of = [&](int b) -> uint64_t {
          float sc = acc[0][g][0];
#pragma unroll
          for (int bb = 1; bb < 8; ++bb) sc = b == bb ? acc[bb >> 2][g][bb & 3] : sc;
          const uint32_t row = trow0 + 16 * (b >> 2) + 4 * kq + (b & 3);
          return make_key(sc, a.row_base + row);
        };
        mf_insert(m, key_of, lists + (size_t)ql[g] * kMfListLen, k, lane, col, kq, th_s[g]);
      }
    }
  };
  if constexpr (kPreA) read_first();  // tile 0's (chunk 0 published above)
  uint32_t nfull = (wr1 - wr0) / 32;
  if (nfull > ntiles) nfull = ntiles;
  // (kEpiPipe) tiles alternate between the two accumulator sets
  auto tile_p = [&](uint32_t t, auto full_tag, auto stag_tag) {
    if constexpr (kEpiPipe) {
      if (t & 1u)
        tile(t, full_tag, stag_tag, MfSet<1>{});
      else
        tile(t, full_tag, stag_tag, MfSet<0>{});
    } else {
      tile(t, full_tag, stag_tag, MfSet<0>{});
    }
  };
  auto run_tiles = [&](auto stag_tag) {
    if constexpr (kPeel) {
      for (uint32_t t = 0; t < nfull; ++t) tile_p(t, MfFull<true>{}, stag_tag);
      for (uint32_t t = nfull; t < ntiles; ++t) tile_p(t, MfFull<false>{}, stag_tag);
    } else {
      for (uint32_t t = 0; t < ntiles; ++t) tile_p(t, MfFull<false>{}, stag_tag);
    }
    if constexpr (kEpiSplit) {  // the last tile's, when it is a deferred full one
      if (ntiles == nfull && nfull > 0) {
        if ((nfull - 1) & 1u)
          q8_epi(accq[1], prow0, true);
        else
          q8_epi(accq[0], prow0, true);
      }
    } else if constexpr (kEpiPipe) {  // the last tile's epilogue
      if (have_prev) {
        if ((ntiles - 1) & 1u)
          q8_epi(accq[1], prow0, pfull);
        else
          q8_epi(accq[0], prow0, pfull);
      }
    }
  };
  if constexpr (kStag) {
    if (w >= 4)
      run_tiles(MfFull<true>{});
    else
      run_tiles(MfFull<false>{});
  } else {
    run_tiles(MfFull<false>{});
  }
  if constexpr (kDma && kBF) wait_vmcnt<0>();  // no LDS-DMA outlives the workgroup
  if constexpr (kClock) tclk2 = wall_clock64();
  // each wave owns its queries' lists / counters: no barrier before the write-out
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if constexpr (MODE == 0) {
      // the int8 pass writes its counts and maxima query-major ([query][wg][4],
      // r05: select_q8 reads a query's 4 nwg quarters in one coalesced load)
      const size_t ci = I8 ? ((size_t)ql[g] * gridDim.x + blockIdx.x) * 4 + kq
                           : ((size_t)blockIdx.x * kMfmaQueries + ql[g]) * 4 + kq;
      a.cand_cnt[ci] = kRegCnt ? cnt_r[g] : cntl[g * THREADS + threadIdx.x];
      if (a.cand_max)
        a.cand_max[ci] =
            kRegCnt ? (I8 ? (uint32_t)qmx_r[g] : cntl[g * THREADS + threadIdx.x])
                    : cntl[(G + g) * THREADS + threadIdx.x];
    } else if constexpr (MODE == 3) {
      // a workgroup with fewer tiles than max_tiles: the rest are empty
      for (uint32_t t = ntiles + kq; t < a.max_tiles; t += 4)
        if (qvalid[g]) a.tmax[(size_t)ql[g] * tstride + (size_t)blockIdx.x * a.max_tiles + t] =
            -INFINITY;
    } else if constexpr (kLists) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t j = (uint32_t)(4 * kq + t);
        if (j < k)
          a.lists[((size_t)blockIdx.x * kMfmaQueries + ql[g]) * k + j] =
              lists[(size_t)ql[g] * kMfListLen + j];
      }
    }
  }
  if constexpr (kClock)
    if (threadIdx.x == 0) {  // [start, prologue done, tiles done, end] per workgroup
      a.lists[4 * blockIdx.x] = tclk0;
      a.lists[4 * blockIdx.x + 1] = tclk1;
      a.lists[4 * blockIdx.x + 2] = tclk2;
      a.lists[4 * blockIdx.x + 3] = wall_clock64();
    }
}

bool mfma_supported(uint32_t dim, bool f32) {
  if (f32) return dim == 768 || dim == 512 || dim == 384 || dim == 256 || dim == 128;
  return dim == 768 || dim == 512 || dim == 384 || dim == 256 || dim == 128 || dim == 1024 ||
         dim == 1536;
}

uint32_t mfma_queries(uint32_t dim, bool f32) {
  const int g = mf_groups_b((int)dim * (f32 ? 4 : 2));
  return (uint32_t)(mf_waves(g) * 16 * g);
}

void mfma_grid(uint32_t n_rows, uint32_t* nwg, uint32_t* rows_per_wg) {
  const int cus = g_cu_count ? g_cu_count : device_cu_count();
  uint64_t want = (uint64_t)cus < kMfmaMaxLists ? (uint64_t)cus : kMfmaMaxLists;
  const uint64_t tiles = ((uint64_t)n_rows + 31) / 32;
  if (want > tiles) want = tiles;
  if (want < 1) want = 1;
  uint64_t rpw = (((uint64_t)n_rows + want - 1) / want + 31) / 32 * 32;
  if (rpw == 0) rpw = 32;
  *rows_per_wg = (uint32_t)rpw;
  *nwg = (uint32_t)(((uint64_t)n_rows + rpw - 1) / rpw);
  if (*nwg == 0) *nwg = 1;
}

uint32_t mfma_max_lists(uint32_t n_rows) {
  uint32_t nwg, rpw;
  mfma_grid(n_rows, &nwg, &rpw);
  return nwg;
}

uint32_t mfma_tiles_per_wg(uint32_t n_rows) {
  uint32_t nwg, rpw;
  mfma_grid(n_rows, &nwg, &rpw);
  return (rpw + 31) / 32;
}

// bf16 rows of D = 768 stream in 24 KiB K-chunks (two per 32-row tile, so
// two barriers per tile instead of three) through a 144 KiB ring (5 chunks in
// flight): -0.75% / -1.7% main pass at 10M / 1.25M rows back to back
// (profiles/r02_ablation_chunk_*.txt; VAR 2048 + 256 in the ablation set).
template <int MODE, int D, bool F32>
constexpr int mf_product_var() {
  return (!F32 && D == 768 && (MODE == 0 || MODE == 3)) ? 2048 + 256 : 0;
}

template <int MODE, int D, bool F32>
static void mfma_launch_d(uint32_t nwg, const MfArgs& a, hipStream_t st) {
  constexpr int G = mf_groups_b(D * (F32 ? 4 : 2));
  hipLaunchKernelGGL((mfma_topk_kernel<D, MODE, mf_product_var<MODE, D, F32>(), G, F32>),
                     dim3(nwg), dim3(64 * mf_waves(G)), 0, st, a);
}

template <int MODE>
static hipError_t mfma_launch_mode(uint32_t dim, bool f32, uint32_t nwg, const MfArgs& a,
                                   hipStream_t st) {
  if (f32) {
    switch (dim) {
      case 768: mfma_launch_d<MODE, 768, true>(nwg, a, st); break;
      case 512: mfma_launch_d<MODE, 512, true>(nwg, a, st); break;
      case 384: mfma_launch_d<MODE, 384, true>(nwg, a, st); break;
      case 256: mfma_launch_d<MODE, 256, true>(nwg, a, st); break;
      case 128: mfma_launch_d<MODE, 128, true>(nwg, a, st); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  switch (dim) {
    case 768: mfma_launch_d<MODE, 768, false>(nwg, a, st); break;
    case 512: mfma_launch_d<MODE, 512, false>(nwg, a, st); break;
    case 384: mfma_launch_d<MODE, 384, false>(nwg, a, st); break;
    case 256: mfma_launch_d<MODE, 256, false>(nwg, a, st); break;
    case 128: mfma_launch_d<MODE, 128, false>(nwg, a, st); break;
    case 1024: mfma_launch_d<MODE, 1024, false>(nwg, a, st); break;
    case 1536: mfma_launch_d<MODE, 1536, false>(nwg, a, st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

static bool mfma_args_ok(uint32_t dim, bool f32, uint32_t n_rows, uint32_t nq_valid, uint32_t k) {
  return mfma_supported(dim, f32) && k >= 1 && k <= kMfmaMaxK && n_rows > 0 && nq_valid >= 1 &&
         nq_valid <= mfma_queries(dim, f32);
}

hipError_t launch_mfma_sample(const void* X, bool f32, uint32_t dim, uint32_t n_rows,
                              uint32_t row_base, const void* Q, uint32_t nq_valid,
                              uint32_t k, uint32_t max_tiles, float* tmax, uint32_t max_lists,
                              uint32_t* nlists, hipStream_t st, const uint64_t* allow,
                              const uint32_t* run_if) {
  if (!mfma_args_ok(dim, f32, n_rows, nq_valid, k) || max_tiles == 0) return hipErrorInvalidValue;
  MfArgs a{};
  mfma_grid(n_rows, nlists, &a.rows_per_wg);
  if (*nlists > max_lists) return hipErrorInvalidValue;
  a.X = X, a.Q = Q, a.tmax = tmax;
  a.n_rows = n_rows, a.row_base = row_base, a.max_tiles = max_tiles, a.nq_valid = nq_valid;
  a.k = k, a.allow = allow, a.run_if = run_if;
  return mfma_launch_mode<3>(dim, f32, *nlists, a, st);
}

hipError_t launch_mfma_lists(const void* X, bool f32, uint32_t dim, uint32_t n_rows,
                             uint32_t row_base, const void* Q, uint32_t nq_valid,
                             uint32_t k, const float* init_score, uint64_t* lists,
                             uint32_t max_lists,
                             uint32_t* nlists, hipStream_t st, const uint64_t* allow) {
  if (!mfma_args_ok(dim, f32, n_rows, nq_valid, k) || k > kMfmaListMaxK)
    return hipErrorInvalidValue;
  MfArgs a{};
  mfma_grid(n_rows, nlists, &a.rows_per_wg);
  if (*nlists > max_lists) return hipErrorInvalidValue;
  a.X = X, a.Q = Q, a.init_score = init_score, a.lists = lists;
  a.n_rows = n_rows, a.row_base = row_base, a.nq_valid = nq_valid, a.k = k;
  a.allow = allow;
  return mfma_launch_mode<8>(dim, f32, *nlists, a, st);
}

hipError_t launch_mfma_cand(const void* X, bool f32, uint32_t dim, uint32_t n_rows,
                            uint32_t row_base, const void* Q, uint32_t nq_valid, uint32_t k,
                            const float* init_score, float* slabs,
                            uint32_t* slab_tile, uint32_t cand_cap,
                            uint32_t* cand_cnt, uint32_t max_lists, uint32_t* nlists,
                            hipStream_t st, const uint64_t* allow, uint32_t* cand_max,
                            const uint32_t* run_if) {
  if (!mfma_args_ok(dim, f32, n_rows, nq_valid, k) || cand_cap < 4 * k || cand_cap % 4 ||
      cand_cap > kMfmaMaxCandCap)
    return hipErrorInvalidValue;
  MfArgs a{};
  mfma_grid(n_rows, nlists, &a.rows_per_wg);
  if (*nlists > max_lists) return hipErrorInvalidValue;
  a.X = X, a.Q = Q, a.init_score = init_score, a.cand = (uint64_t*)slabs;
  a.cand_tile = slab_tile, a.cand_cnt = cand_cnt, a.cand_max = cand_max;
  a.n_rows = n_rows, a.row_base = row_base;
  a.nq_valid = nq_valid, a.k = k, a.cand_cap = cand_cap, a.allow = allow;
  a.run_if = run_if;
  return mfma_launch_mode<0>(dim, f32, *nlists, a, st);
}

// int8 prefilter pass (r04): D = 768 rows of int8 (768 B, whole-row 24 KiB
// K-chunks through the 144 KiB ring), 256 queries; D = 1024 (C5's rows):
// 16 KiB chunks (32 rows x 512 B) through the 144 KiB ring, 128 queries per
// launch as the bf16 pass and sample pass there. No filter.
bool q8_supported(uint32_t dim, bool f32) {
  return f32 ? dim == 768 : (dim == 768 || dim == 1024);
}

template <int VAR>
static hipError_t launch_q8_var(uint32_t nwg, const MfArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((mfma_topk_kernel<768, 0, VAR, 2, false, true>), dim3(nwg), dim3(512), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_mfma_cand_q8(const void* X8, uint32_t dim, uint32_t n_rows, uint32_t row_base,
                               const void* Q8, uint32_t nq_valid, uint32_t k,
                               const float* init_score, const float* q8par, const float* q8glob,
                               float* slabs, uint32_t* slab_tile, uint32_t cand_cap,
                               uint32_t* cand_cnt, uint32_t* cand_max, uint32_t max_lists,
                               uint32_t* nlists, uint32_t* gate, hipStream_t st,
                               const uint64_t* allow, const uint32_t* run_if) {
  if (!q8_supported(dim, false) || !mfma_args_ok(dim, false, n_rows, nq_valid, k) || cand_cap < 4 ||
      cand_cap % 4 || cand_cap > kMfmaMaxCandCap || !q8par || !q8glob || !gate || !cand_max)
    return hipErrorInvalidValue;
  MfArgs a{};
  mfma_grid(n_rows, nlists, &a.rows_per_wg);
  if (*nlists > max_lists) return hipErrorInvalidValue;
  a.X = X8, a.Q = Q8, a.init_score = init_score, a.cand = (uint64_t*)slabs;
  a.cand_tile = slab_tile, a.cand_cnt = cand_cnt, a.cand_max = cand_max;
  a.n_rows = n_rows, a.row_base = row_base;
  a.nq_valid = nq_valid, a.k = k, a.cand_cap = cand_cap;
  a.q8par = q8par, a.q8glob = q8glob, a.gate = gate, a.allow = allow, a.run_if = run_if;
  if (dim == 1024) {
    hipLaunchKernelGGL((mfma_topk_kernel<1024, 0, 256, 1, false, true>), dim3(*nlists), dim3(512), 0,
                       st, a);
    return hipGetLastError();
  }
  static const int var = [] {
    const char* e = getenv("VS_Q8_VAR");
    return e ? atoi(e) : 2048 + 256;
  }();
  switch (var) {  // VS_Q8_VAR: ablation arms (read once)
    case 0: return launch_q8_var<0>(*nlists, a, st);
    case 256: return launch_q8_var<256>(*nlists, a, st);
    case 2048 + 256 + 16777216: return launch_q8_var<2048 + 256 + 16777216>(*nlists, a, st);
    default: return launch_q8_var<2048 + 256>(*nlists, a, st);
  }
}

uint32_t mfma_cand_cap(uint32_t n_rows, uint32_t k, uint32_t sample_tiles, double scale) {
  uint32_t nwg, rpw;
  mfma_grid(n_rows, &nwg, &rpw);
  const double tpw = (rpw + 31) / 32;
  // expected survivors of the sample bound per (workgroup, query): the bound
  // is the k-th of ~k / f rows (f = sampled fraction), spread over nwg
  const double e = scale * (double)k * tpw / (double)(sample_tiles ? sample_tiles : 1) / nwg;
  const double want = 3.0 * e + 32.0;
  uint32_t cap = 64;
  while (cap < want && cap < kMfmaMaxCandCap) cap <<= 1;
  // a lane's quarter holds sub = cap / 4 slabs; a full quarter keeps the
  // sub best (mf_replace_min), exact while sub >= k
  while (cap < 4 * k) cap <<= 1;
  return cap;
}

uint32_t mfma_sample_tiles(uint32_t n_rows, uint32_t dim, bool f32) {
  // 1/128 of every workgroup's tiles, at least 4 when it has 64 or more: with
  // the slab select, whose cost grows with the survivors, 4 instead of 2
  // tiles at 1.25M rows (the N = 8 share) saved 2-3 us per batch (r01). With
  // tile maxima stored as floats (r02) the sample pass costs ~5 us per tile
  // and the select ~1.4 us per 100 survivors per query: at 10M rows 1/128
  // (9 tiles: 61 + 24 us) beats 1/64 (19 tiles: 110 + 16 us;
  // profiles/r02_sample_tiles_10m.txt). bf16 rows of 1024 / 1536 (128-query
  // launches, HBM-bound): 1/64, since there every candidate append slows the
  // stream (5M x 1024: sample + main 1.776 -> 1.735 ms at k = 50 and 1.631
  // -> 1.603 at k = 10 for 4 -> 8 tiles; profiles/r02_sample_tiles_d1024_*).
  const uint32_t tpw = mfma_tiles_per_wg(n_rows);
  const bool hbm_bound = !f32 && mf_groups_b((int)dim * 2) == 1;
  uint32_t st = tpw / (hbm_bound ? 64 : 128);
  if (tpw >= 64 && st < 4) st = 4;
  if (st < 1) st = 1;
  if (st > kMfmaMaxSampleTiles) st = kMfmaMaxSampleTiles;
  return st;
}

// ---------------------------------------------------------------------------
// select: top-k of per-workgroup candidate buffers
// ---------------------------------------------------------------------------
// One workgroup per query; thread t owns lane quarters t and t + 512 of the
// 4 * nwg quarter lists. First bound: the k-th largest of the per-buffer
// maxima (k keys of k distinct rows) -- no key below it can be in the top k,
// which leaves a few dozen of the usual hundreds of candidates. Fast path:
// every thread re-reads its own quarters and appends the keys above the bound
// to an LDS buffer, which is sorted once. Only if more than kMfmaSelBuf keys
// pass (adversarial ties) does the workgroup fall back to streaming all
// candidates in chunks through the buffer (prefix sum of the counts; the
// running top-k is re-sorted whenever a chunk added something). Any total is
// handled.
constexpr int kSelThreads = 512;

__device__ __forceinline__ void bitonic_sort_desc_n(uint64_t* buf, int n_pow2, int nthreads) {
  for (int size = 2; size <= n_pow2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < n_pow2 / 2; i += nthreads) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool desc = ((lo & size) == 0);
        const uint64_t x = buf[lo], y = buf[hi];
        if ((x < y) == desc) {
          buf[lo] = y;
          buf[hi] = x;
        }
      }
      __syncthreads();
    }
  }
}

// Bitonic sort of one u64 per lane across a wave, descending (lane 0 gets
// the largest): 21 shuffle stages, no LDS, no barrier.
__device__ __forceinline__ uint64_t wave_sort_desc(uint64_t x, int lane) {
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const uint32_t lo = __shfl_xor((unsigned)(uint32_t)x, stride, 64);
      const uint32_t hi = __shfl_xor((unsigned)(uint32_t)(x >> 32), stride, 64);
      const uint64_t y = ((uint64_t)hi << 32) | lo;
      const bool keep_max = ((lane & stride) == 0) == ((lane & size) == 0);
      x = keep_max ? (x > y ? x : y) : (x < y ? x : y);
    }
  return x;
}

// First bound of a select, for k <= 64: the k-th largest of the 64 maxima of
// 4 consecutive per-buffer maxima lmax[0, 256) (k keys of k distinct rows
// reach it, so it is <= the k-th largest of all 256 and of the result).
// Wave 0 computes it; the caller publishes it with a barrier.
__device__ __forceinline__ uint64_t sel_bound_wave(const uint64_t* lmax, uint32_t k, int lane) {
  const uint64_t* g4 = lmax + 4 * lane;
  const uint64_t a = g4[0] > g4[1] ? g4[0] : g4[1], b = g4[2] > g4[3] ? g4[2] : g4[3];
  const uint64_t g = wave_sort_desc(a > b ? a : b, lane);
  return shfl64(g, (int)k - 1);
}

// Final top k of c <= 64 keys in buf by wave 0 alone: sorted in registers and
// written out (0-padded to k <= kMfmaMaxK).
__device__ __forceinline__ void sel_finish_wave(const uint64_t* buf, uint32_t c, uint32_t k,
                                                int lane, uint64_t* out) {
  const uint64_t x = wave_sort_desc((uint32_t)lane < c ? buf[lane] : 0ull, lane);
  for (uint32_t j = (uint32_t)lane; j < k; j += 64) out[j] = j < 64 ? x : 0ull;
}


// Top 64 of two descending wave lists (one key per lane): the element-wise
// maximum of one list and the other reversed is a bitonic sequence holding
// the 64 largest keys; a half-cleaner cascade sorts it descending.
__device__ __forceinline__ uint64_t wave_merge_top(uint64_t a, uint64_t b_desc, int lane) {
  const uint64_t br = shfl64(b_desc, 63 - lane);
  uint64_t y = a > br ? a : br;
#pragma unroll
  for (int stride = 32; stride > 0; stride >>= 1) {
    const uint32_t lo = __shfl_xor((unsigned)(uint32_t)y, stride, 64);
    const uint32_t hi = __shfl_xor((unsigned)(uint32_t)(y >> 32), stride, 64);
    const uint64_t o = ((uint64_t)hi << 32) | lo;
    y = (lane & stride) == 0 ? (y > o ? y : o) : (y < o ? y : o);
  }
  return y;
}

// Main-pass slabs: slab j of quarter list l holds the scores of rows
// tile + 16 (b / 4) + 4 kq + b % 4, b = 0..7 (the MFMA accumulator layout; kq
// = l & 3). A score of -inf is a padding row; with a filter pre-mask `allow`
// (bit r = local row r = global - row_base; nullable) the main pass leaves
// masked rows in the slab and the select drops them here.
struct SlabMask {
  const uint64_t* allow;
  uint32_t row_base;
};
// the 8 mask bits of a slab (tile % 32 == 0 locally: one half of a word)
__device__ __forceinline__ uint32_t slab_bits(SlabMask fm, uint32_t tile, uint32_t kq) {
  if (!fm.allow) return 0xFFu;
  const uint32_t r = tile - fm.row_base;
  const uint32_t tw = (uint32_t)(fm.allow[r >> 6] >> (r & 32)) >> (4 * kq);
  return (tw & 0xFu) | ((tw >> 12) & 0xF0u);
}

// Slab select, compacted (the main pass's buffers; one workgroup per query).
// A query's slabs are few (~600-800 at k = 10) but spread over 4 * nwg lists
// of 0-8 each, so per-list rounds of loads would cost as many dependent
// memory round trips as the longest list in a wave. Instead: one round for
// the 1024 counts, a block prefix sum, an LDS owner table (flat slab index ->
// list), then every thread loads up to kSelHeld slabs of the flat range in
// ONE round and keeps them in registers for both passes. Pass 1: per
// buffer (workgroup) the maximum admitted score, LDS atomicMax; the k-th
// largest is a score bound (k distinct rows reach it). Pass 2: keys of the
// held scores that reach it -> buf, sorted once. More slabs than the
// workgroup holds (large k, adversarial ties) go through the same passes in
// chunks, re-loading; more than kMfmaSelBuf keys past the bound take the
// streaming path of select_cand_kernel.
constexpr int kSelHeld = 4;                      // slabs per thread per chunk
constexpr uint32_t kSelChunk = kSelHeld * kSelThreads;  // 2048 slabs

template <int SV = 0>
__global__ __launch_bounds__(kSelThreads) void select_slab_kernel(
    const f32x4_t* __restrict__ slabs, const uint32_t* __restrict__ tiles,
    const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ cmax, uint32_t nwg,
    uint32_t cap, uint32_t k, uint64_t* __restrict__ out, SlabMask fm,
    const uint32_t* __restrict__ run_if) {
  if (run_if && *run_if == 0u) return;  // the int8 pass answered this batch
  __shared__ uint64_t buf[kMfmaSelBuf];
  __shared__ uint64_t lmax[kMfmaMaxLists];
  __shared__ uint32_t pre[4 * kMfmaMaxLists + 1];
  __shared__ uint16_t owner[kSelChunk];
  __shared__ uint32_t wtot[kSelThreads / 64];
  __shared__ uint32_t fill, spill;
  __shared__ uint64_t thr_sh;
  static_assert(4 * kMfmaMaxLists == 2 * kSelThreads, "two lists per thread");
  const uint32_t q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t sub = cap >> 2, nl = 4 * nwg;
  // lists 2 tid, 2 tid + 1: counts and, with cmax, maxima (all loads in
  // flight at once; past nl: 0)
  const uint32_t l0 = 2 * tid;
  uint32_t c0 = 0, c1 = 0, x0 = 0, x1 = 0;
  {
    const uint32_t a0 = l0 < nl ? l0 : 0u, a1 = l0 + 1 < nl ? l0 + 1 : 0u;
    const size_t i0 = ((size_t)(a0 >> 2) * kMfmaQueries + q) * 4 + (a0 & 3);
    const size_t i1 = ((size_t)(a1 >> 2) * kMfmaQueries + q) * 4 + (a1 & 3);
    const uint32_t r0 = cnt[i0], r1 = cnt[i1];
    if (cmax) x0 = cmax[i0], x1 = cmax[i1];
    c0 = l0 < nl ? (r0 < sub ? r0 : sub) : 0u;
    c1 = l0 + 1 < nl ? (r1 < sub ? r1 : sub) : 0u;
    x0 = c0 ? x0 : 0u;
    x1 = c1 ? x1 : 0u;
  }
  if (tid < kMfmaMaxLists) lmax[tid] = 0;
  if (tid == 0) fill = 0, spill = 0;
  // the bound from lmax (per-buffer maxima as keys, row word 0): the k-th
  // largest has k keys of k distinct rows at or above it. Admit keys > thr.
  auto bound_from_lmax = [&]() -> uint64_t {
    if (k <= 64) {
      if (w == 0) {
        const uint64_t b = sel_bound_wave(lmax, k, (int)lane);
        if (lane == 0) thr_sh = b ? b - 1 : 0;
      }
      __syncthreads();
      return thr_sh;
    }
    bitonic_sort_desc_n(lmax, (int)kMfmaMaxLists, kSelThreads);
    return (k <= kMfmaMaxLists && lmax[k - 1] != 0) ? lmax[k - 1] - 1 : 0;
  };
  uint64_t thr = 0;
  if (cmax) {
    // r04: the main pass recorded each quarter's largest admitted score, so
    // the per-buffer maxima (and the bound) come without reading a slab, and
    // only quarters whose maximum passes the bound -- ~k of 4 nwg -- are read
    // below (any key above the bound lies in one of them)
    __syncthreads();  // lmax zeroed
    if (x0) atomicMax((unsigned long long*)&lmax[l0 >> 2], (unsigned long long)x0 << 32);
    if (x1) atomicMax((unsigned long long*)&lmax[(l0 + 1) >> 2], (unsigned long long)x1 << 32);
    __syncthreads();
    thr = bound_from_lmax();
    if (((uint64_t)x0 << 32) <= thr) c0 = 0;
    if (((uint64_t)x1 << 32) <= thr) c1 = 0;
  }
  // block exclusive prefix sum of the counts (with cmax: of the passing quarters)
  uint32_t incl = c0 + c1;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if ((int)lane >= d) incl += y;
  }
  if (lane == 63) wtot[w] = incl;
  __syncthreads();
  uint32_t woff = 0, total = 0;
#pragma unroll
  for (int i = 0; i < kSelThreads / 64; ++i) {
    const uint32_t x = wtot[i];
    woff += (uint32_t)i < w ? x : 0u;
    total += x;
  }
  const uint32_t ex = woff + incl - (c0 + c1);
  pre[l0] = ex;
  pre[l0 + 1] = ex + c0;
  if (tid == 0) pre[2 * kSelThreads] = total;
  for (uint32_t j = 0; j < c0; ++j)
    if (ex + j < kSelChunk) owner[ex + j] = (uint16_t)l0;
  for (uint32_t j = 0; j < c1; ++j)
    if (ex + c0 + j < kSelChunk) owner[ex + c0 + j] = (uint16_t)(l0 + 1);
  __syncthreads();
  const uint32_t T = total;
  // slot j of quarter list l (layout [wg][query][cap], a quarter = sub slots)
  auto slab_at = [&](uint32_t l, uint32_t j) -> size_t {
    return ((size_t)(l >> 2) * kMfmaQueries + q) * cap + (l & 3) * sub + j;
  };
  // flat slab i -> its list (owner table inside the first chunk, else a
  // binary search of pre), its entry and kq
  auto list_of = [&](uint32_t i) -> uint32_t {
    if (i < kSelChunk) return owner[i];
    uint32_t lo = 0, hi = 2 * kSelThreads;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (pre[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
  };
  f32x4_t v[kSelHeld][2];
  uint32_t tl[kSelHeld], ls[kSelHeld], bits[kSelHeld];
  auto load_chunk = [&](uint32_t base) {
#pragma unroll
    for (int u = 0; u < kSelHeld; ++u) {
      const uint32_t i = base + tid + (uint32_t)u * kSelThreads;
      const bool ok = i < T;
      const uint32_t l = ok ? list_of(i) : 0u;
      const size_t e = slab_at(l, ok ? i - pre[l] : 0u);
      ls[u] = l;
      v[u][0] = slabs[2 * e];
      v[u][1] = slabs[2 * e + 1];
      tl[u] = tiles[e];
      bits[u] = ok ? 0xFFu : 0u;
    }
#pragma unroll
    for (int u = 0; u < kSelHeld; ++u)
      if (bits[u]) bits[u] = slab_bits(fm, tl[u], ls[u] & 3);
  };
  if (!cmax) {
    // pass 1: per buffer (workgroup) maximum admitted score
    for (uint32_t base = 0; base < T; base += kSelChunk) {
      load_chunk(base);
#pragma unroll
      for (int u = 0; u < kSelHeld; ++u) {
        float sv[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) sv[b] = ((bits[u] >> b) & 1u) ? v[u][b >> 2][b & 3] : -INFINITY;
        const float m = fmax3(fmax3(sv[0], sv[1], sv[2]), fmax3(sv[3], sv[4], sv[5]),
                              fmax3(sv[6], sv[7], -INFINITY));
        if (m != -INFINITY)
          atomicMax((unsigned long long*)&lmax[ls[u] >> 2],
                    (unsigned long long)make_key(m, 0xFFFFFFFFu));
      }
    }
    __syncthreads();
    if constexpr (SV == 1) return;
    thr = bound_from_lmax();
  }
  // the bound is a score with the smallest row key, so thr + 1 is its key
  const float thr_s = thr ? key_score(thr + 1) : -INFINITY;
  if constexpr (SV == 2) return;
  // pass 2: keys reaching the bound -> buf (held slabs when one chunk did it)
  for (uint32_t base = 0; base < T; base += kSelChunk) {
    if (T > kSelChunk || cmax) load_chunk(base);  // else pass 1's registers hold them
#pragma unroll
    for (int u = 0; u < kSelHeld; ++u)
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const float sc = v[u][b >> 2][b & 3];
        if (((bits[u] >> b) & 1u) && sc >= thr_s) {
          const uint64_t x = make_key(
              sc, tl[u] + 16u * (uint32_t)(b >> 2) + 4u * (ls[u] & 3) + (uint32_t)(b & 3));
          if (x > thr) {
            const uint32_t pos = atomicAdd(&fill, 1u);
            if (pos < (uint32_t)kMfmaSelBuf) buf[pos] = x; else spill = 1u;
          }
        }
      }
  }
  __syncthreads();
  if constexpr (SV == 3) return;
  uint32_t nR = 0;  // running top-k in buf[0, nR)
  if (!spill && fill <= 64) {
    if (w == 0) sel_finish_wave(buf, fill, k, (int)lane, out + (size_t)q * k);
    return;
  }
  if (!spill) {
    const uint32_t c = fill;
    if (c) {
      int p2 = 1;
      while ((uint32_t)p2 < c) p2 <<= 1;
      for (uint32_t i = c + tid; i < (uint32_t)p2; i += kSelThreads) buf[i] = 0;
      __syncthreads();
      bitonic_sort_desc_n(buf, p2, kSelThreads);
      nR = c < k ? c : k;
    }
  } else {
    // more than kMfmaSelBuf keys reach the bound: stream the slabs in chunks
    // of (kMfmaSelBuf - k) / 8 through buf, keeping a running top k
    const uint32_t chunk = (kMfmaSelBuf - k) / 8;
    for (uint32_t base = 0; base < T; base += chunk) {
      if (tid == 0) fill = nR;
      __syncthreads();
      const uint32_t end = base + chunk < T ? base + chunk : T;
      for (uint32_t i = base + tid; i < end; i += kSelThreads) {
        const uint32_t l = list_of(i);
        const size_t e = slab_at(l, i - pre[l]);
        const f32x4_t v0 = slabs[2 * e], v1 = slabs[2 * e + 1];
        const uint32_t t = tiles[e];
        const uint32_t bb8 = slab_bits(fm, t, l & 3);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          const float sc = b < 4 ? v0[b] : v1[b - 4];
          const uint32_t row = t + 16u * (uint32_t)(b >> 2) + 4u * (l & 3) + (uint32_t)(b & 3);
          const uint64_t x = (((bb8 >> b) & 1u) && sc != -INFINITY) ? make_key(sc, row) : 0ull;
          if (x > thr) buf[atomicAdd(&fill, 1u)] = x;
        }
      }
      __syncthreads();
      const uint32_t c = fill;
      if (c > nR) {
        int p2 = 1;
        while ((uint32_t)p2 < c) p2 <<= 1;
        for (uint32_t i = c + tid; i < (uint32_t)p2; i += kSelThreads) buf[i] = 0;
        __syncthreads();
        bitonic_sort_desc_n(buf, p2, kSelThreads);
        nR = c < k ? c : k;
        if (nR == k && buf[k - 1] > thr) thr = buf[k - 1];
      }
      __syncthreads();
    }
  }
  for (uint32_t j = tid; j < k; j += kSelThreads) out[(size_t)q * k + j] = j < nR ? buf[j] : 0;
}

// ---------------------------------------------------------------------------
// sample bound: per query, a lower bound on the k-th largest of m tile maxima
// (k maxima of k distinct tiles: k distinct rows score at least that much, so
// it bounds the query's global k-th score from below). Radix select on the
// order-preserving 32-bit image of the scores, 8 bits per pass, LDS histogram
// + one block scan per pass; one workgroup per query. Two passes: the bound is
// the lowest value of the 16-bit bucket holding the k-th largest (at least k
// maxima reach it; it sits below the exact k-th by under 2^-7 relative, which
// admits a few more rows than the exact value would, for half the passes;
// r04: four passes, the exact k-th maximum, cut the candidates by 5% at 10M
// rows and did not make the main pass faster, so two stay the default).
// Fewer than k maxima give -inf: every row is then admitted.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBoundThreads) void sample_bound_kernel(
    const float* __restrict__ tmax, uint32_t m, uint32_t k, float* __restrict__ bound,
    int passes, const uint32_t* __restrict__ run_if) {
  if (run_if && *run_if == 0u) return;  // (r05) the fallback behind a verified speculative batch
  sample_bound_block(tmax, m, k, bound, passes, blockIdx.x);  // vs_bound_dev.h
}

// Radix passes of the sample bound (VS_BOUND_PASSES, read once; 2 = the
// 16-bit bucket floor, up to 2^-7 relative under the k-th maximum; 4 = the
// k-th maximum exactly, a tighter bound: fewer main-pass candidates)
int sample_bound_passes() {
  static const int v = [] {
    const char* e = getenv("VS_BOUND_PASSES");
    const int x = e ? atoi(e) : 2;
    return x < 2 ? 2 : (x > 4 ? 4 : x);
  }();
  return v;
}

hipError_t launch_sample_bound(const float* tmax, uint32_t m, uint32_t nq, uint32_t k,
                               float* bound, hipStream_t st, const uint32_t* run_if) {
  if (nq == 0 || nq > kMfmaQueries || k == 0 || k > kMfmaMaxK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sample_bound_kernel, dim3(nq), dim3(kBoundThreads), 0, st, tmax, m, k, bound,
                     sample_bound_passes(), run_if);
  return hipGetLastError();
}

static bool select_args_ok(uint32_t nwg, uint32_t cap, uint32_t nq, uint32_t k) {
  return nwg != 0 && nwg <= kMfmaMaxLists && cap >= 4 && cap % 4 == 0 && k != 0 &&
         k <= kMfmaMaxK && nq != 0 && nq <= kMfmaQueries;
}


hipError_t launch_select_slabs(const float* slabs, const uint32_t* slab_tile,
                               const uint32_t* cand_cnt, uint32_t nwg, uint32_t cap, uint32_t nq,
                               uint32_t k, uint64_t* out, hipStream_t st, uint32_t row_base,
                               const uint64_t* allow, const uint32_t* cand_max,
                               const uint32_t* run_if) {
  if (!select_args_ok(nwg, cap, nq, k)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(select_slab_kernel<0>, dim3(nq), dim3(kSelThreads), 0, st,
                     (const f32x4_t*)slabs, slab_tile, cand_cnt, cand_max, nwg, cap, k, out,
                     SlabMask{allow, row_base}, run_if);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// select of the int8 prefilter pass (r04): bound, rescore, top k
// ---------------------------------------------------------------------------
// One workgroup per query over the I8 main pass's slabs (8 int32 dots of one
// lane's rows of a tile). With the query's {sqS, a, c, sigma} and the tile's
// {dt, nt} (largest quantisation-error norm and row norm of its 32 rows),
// every slab row has L = sqS dot - m - sigma nt <= its fp32 score <= U =
// sqS dot + m + sigma nt, m = a dt + c nt. From the quarters'
// largest dots: each quarter's largest L (global m); the k-th largest of
// those is a lower bound on the k-th score (the quarters hold disjoint rows),
// and so is b - sigma nmax (the sample bound). Rows whose U reaches the larger of the
// two (read from the quarters whose largest U does) are the only ones that
// can be in the top k; they are rescored from the bf16 rows on the bf16
// pass's own MFMA chain -- the same score bits -- and the top k of those keys
// is the bf16 pass's answer. A lossy quarter that can reach the cutoff is
// recomputed from the int8 copy, and more survivors than the LDS buffer holds
// stream through a running top k (r05); nothing is handed to another pass.

// SV (timing ablation, VS_Q8_SEL_SV): return after stage SV. F32: fp32 rows
// and queries, survivors rescored on the f32 pass's v_mfma_f32_16x16x4_f32
// chain (four MFMAs per 16-B fragment, as that pass), so again its bits.
// The int8 copy's rows, the queries' int8 images and what the select's slow
// path needs to recompute a lossy quarter (r05): its workgroup's rows
// [wg * rows_per_wg, ...) of the static split (mfma_grid), the pre-mask.
struct Q8Rows {
  const int8_t* x8;
  const int8_t* q8;        // [query][dim] int8 images (vs_q8.hip)
  const uint64_t* allow;   // nullable: bit r admits local row r
  uint32_t n_rows, rows_per_wg, row_base;
};

// A zero query: every score is exactly 0 (products of 0, -0 ranked as +0), so
// the top k are the k lowest allowed rows. Wave-level; k <= kMfmaMaxK.
__device__ __forceinline__ void q8_zero_query(const Q8Rows& r8, uint32_t k, uint32_t lane,
                                              uint64_t* __restrict__ out) {
  uint32_t found = 0;
  for (uint32_t w0 = 0; found < k && (uint64_t)w0 * 64 < r8.n_rows; w0 += 64) {
    const uint32_t wi = w0 + lane;  // this lane's 64-row word
    uint64_t bits = 0;
    if ((uint64_t)wi * 64 < r8.n_rows) {
      bits = r8.allow ? r8.allow[wi] : ~0ull;
      const uint32_t left = r8.n_rows - wi * 64;
      if (left < 64) bits &= (1ull << left) - 1ull;
    }
    const uint32_t pc = (uint32_t)__popcll(bits);
    uint32_t incl = pc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, 64);
      if (lane >= (uint32_t)o) incl += y;
    }
    uint32_t pos = found + incl - pc;
    while (bits && pos < k) {
      const uint32_t b = (uint32_t)__builtin_ctzll(bits);
      out[pos++] = make_key(0.0f, r8.row_base + wi * 64 + b);
      bits &= bits - 1;
    }
    found += (uint32_t)__shfl((int)incl, 63, 64);
  }
  for (uint32_t j = found + lane; j < k; j += 64) out[j] = 0;
}

// The exact int32 dot of an int8 row with an int8 query image in LDS (D bytes).
template <int D>
__device__ __forceinline__ int q8_row_dot(const int8_t* __restrict__ xr, const int8_t* qs) {
  int d = 0;
#pragma unroll 4
  for (int c = 0; c < D / 16; ++c) {
    const uint4 x = *(const uint4*)(xr + 16 * c);
    const int4 y = *(const int4*)(qs + 16 * c);
    d = __builtin_amdgcn_sdot4((int)x.x, y.x, d, false);
    d = __builtin_amdgcn_sdot4((int)x.y, y.y, d, false);
    d = __builtin_amdgcn_sdot4((int)x.z, y.z, d, false);
    d = __builtin_amdgcn_sdot4((int)x.w, y.w, d, false);
  }
  return d;
}

template <int D, int SV, bool F32>
__device__ __forceinline__ void select_q8_body(
    const f32x4_t* __restrict__ slabs, const uint32_t* __restrict__ tiles,
    const uint32_t* __restrict__ cnt, const int* __restrict__ cmax, uint32_t nwg, uint32_t cap,
    uint32_t k, uint64_t* __restrict__ out, uint32_t row_base, const void* __restrict__ X,
    const void* __restrict__ qb, uint32_t dim, const f32x4_t* __restrict__ q8par,
    const float* __restrict__ q8glob, const float* __restrict__ meta,
    const float* __restrict__ bound, const Q8Rows r8, uint32_t two_from, uint32_t opts,
    uint32_t* __restrict__ stats, uint64_t* __restrict__ clk) {
  __shared__ uint64_t buf[kMfmaSelBuf];
  __shared__ uint64_t res[kMfmaSelBuf];  // rescored keys
  __shared__ uint32_t pre[4 * kMfmaMaxLists + 1];
  __shared__ uint16_t owner[2 * kSelChunk];  // (r05) the first 4096 slabs' lists
  __shared__ uint32_t wtot[kSelThreads / 64];
  __shared__ uint32_t wscr[kSelThreads / 64][16];  // a wave's group of 16 rows
  __shared__ uint32_t fill, spill, rfill;
  __shared__ __attribute__((aligned(16))) uint32_t hist[3][256];  // kth_floor's histograms
  // (tools/share_pipe.hip) per-workgroup wall clock at the stage boundaries:
  // 0 start, 1 bound, 2 survivors, 3 rescore, 4 end; two rounds: 5 first
  // floor, 6 first round, 7 second floor; inside the survivor stage (thread
  // 0's view): 8 lossy test, 9 owners written, 10 first round's loads
  // issued, 11 its rows tested ([nq][16])
  auto tick = [&](int i) {
    if (clk && threadIdx.x == 0) clk[(size_t)blockIdx.x * 16 + i] = wall_clock64();
  };
  tick(0);
  const uint32_t q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t sub = cap >> 2, nl = 4 * nwg;
  const f32x4_t par = q8par[q];  // sqS, a, c, sigma
  const float sqS = par[0], pa = par[1], pc = par[2], sig = par[3];
  const float dmax = q8glob[1], nmax = q8glob[2];
  const float mg = pa * dmax + (pc + sig) * nmax;  // m + sigma n of any row
  const float b = bound[q];
  // quarter lists 2 tid, 2 tid + 1 (l = 4 wg + kq): counts and largest
  // appended dots, query-major ([query][wg][4], r05: one coalesced load each)
  const uint32_t l0 = 2 * tid;
  uint32_t c0 = 0, c1 = 0;
  int x0 = INT_MIN, x1 = INT_MIN;
  bool lossy0 = false, lossy1 = false;  // the pass dropped slabs of the quarter
  if (l0 < nl) {  // nl is even: l0 + 1 < nl too
    const uint2 cc = *(const uint2*)(cnt + (size_t)q * nl + l0);
    const int2 mm = *(const int2*)(cmax + (size_t)q * nl + l0);
    c0 = cc.x < sub ? cc.x : sub;
    c1 = cc.y < sub ? cc.y : sub;
    lossy0 = cc.x > sub;
    lossy1 = cc.y > sub;
    x0 = c0 ? mm.x : INT_MIN;
    x1 = c1 ? mm.y : INT_MIN;
  }
  if (tid == 0) fill = 0, spill = 0, rfill = 0;
  // a zero query (a = |sq q8| = 0 and c = |q - sq q8| = 0): every score is
  // exactly 0, so the answer is the k lowest allowed rows (the tie rule)
  if (pa == 0.0f && pc == 0.0f) {
    if (w == 0) q8_zero_query(r8, k, lane, out + (size_t)q * k);
    tick(4);
    return;
  }
  // The floor P of the 24-bit bucket holding the kk-th largest high word (an
  // order-preserving score image) of v[0, n), n >= kk: at least kk entries
  // have a high word >= P. Three 8-bit radix passes as the sample bound
  // (vs_bound_dev.h), over LDS. (r05: every k; the register sorts and wave
  // merges it replaced cost ~4 us per use in the select's latency chain.)
  // (r06) a histogram a pass, zeroed up front, and wave_digit_pick: 5
  // barriers a call instead of 15. 0 (no floor) if n < kk.
  auto kth_floor = [&](const uint64_t* v, uint32_t n, uint32_t kk) -> uint32_t {
    __syncthreads();  // the previous call's waves are done with hist
    for (uint32_t i = tid; i < 3 * 256; i += kSelThreads) (&hist[0][0])[i] = 0;
    __syncthreads();
    uint32_t prefix = 0;
#pragma unroll
    for (int pass = 0; pass < 3; ++pass) {
      const int shift = 24 - 8 * pass;
      const uint32_t hmask = pass == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
      for (uint32_t i = tid; i < n; i += kSelThreads) {
        const uint32_t u = (uint32_t)(v[i] >> 32);
        if ((u & hmask) == prefix) atomicAdd(&hist[pass][(u >> shift) & 255u], 1u);
      }
      __syncthreads();
      uint32_t dig, above;
      if (!wave_digit_pick(hist[pass], kk, lane, dig, above)) return 0u;  // uniform
      prefix |= dig << shift;
      kk -= above;
    }
    return prefix;
  };
  // Each quarter's largest dot gives its lower bound sqS dot - mg; the
  // quarters hold disjoint rows, so k rows reach the k-th largest of those,
  // which bounds the k-th score from below (its radix floor, P0, as well).
  // (The k-th of per-workgroup maxima, the first form, sat far under the
  // k-th score once k neared the 256 workgroups: at k = 50, 4578 survivors
  // per query against 2821.)
  auto lo_img = [&](int x) -> uint32_t {
    if (x == INT_MIN) return 0u;
    const float L = (float)x * sqS - mg;
    return vs::score_ord(L == 0.0f ? 0.0f : L);
  };
  const uint32_t y0 = lo_img(x0), y1 = lo_img(x1);
  buf[l0] = (uint64_t)y0 << 32;
  buf[l0 + 1] = (uint64_t)y1 << 32;
  const uint32_t nzq = (uint32_t)__syncthreads_count(y0 != 0) + (uint32_t)__syncthreads_count(y1 != 0);
  // opts bit 0 (VS_Q8_SEL_P0=0, ablation): no quarter bound, the sample's alone
  const uint32_t P0 = nzq >= k && !(opts & 1u) ? kth_floor(buf, 2 * kSelThreads, k) : 0u;
  const float tl_b = b == -INFINITY ? -INFINITY : b - sig * nmax;
  const float tl_l = P0 ? vs::ord_score(P0) : -INFINITY;
  const float Tcut = tl_b > tl_l ? tl_b : tl_l;
  if (stats && tid == 0 && tl_l > tl_b) atomicAdd(stats + 3, 1u);  // (tools) the quarter bound won
  tick(1);
  if constexpr (SV == 1) return;
  // only quarters whose largest dot can reach Tcut hold survivors
  if (c0 && (float)x0 * sqS + mg < Tcut) c0 = 0, lossy0 = false;
  if (c1 && (float)x1 * sqS + mg < Tcut) c1 = 0, lossy1 = false;
  // a lossy quarter that can reach Tcut: its rows are recomputed (slow path)
  const bool slow = __syncthreads_or(lossy0 || lossy1) != 0;
  tick(8);
  if (lossy0) c0 = 0;
  if (lossy1) c1 = 0;
  uint32_t incl = c0 + c1;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if ((int)lane >= d) incl += y;
  }
  if (lane == 63) wtot[w] = incl;
  __syncthreads();
  uint32_t woff = 0, total = 0;
#pragma unroll
  for (int i = 0; i < kSelThreads / 64; ++i) {
    const uint32_t x = wtot[i];
    woff += (uint32_t)i < w ? x : 0u;
    total += x;
  }
  const uint32_t ex = woff + incl - (c0 + c1);
  pre[l0] = ex;
  pre[l0 + 1] = ex + c0;
  if (tid == 0) pre[2 * kSelThreads] = total;
  for (uint32_t j = 0; j < c0; ++j)
    if (ex + j < 2 * kSelChunk) owner[ex + j] = (uint16_t)l0;
  for (uint32_t j = 0; j < c1; ++j)
    if (ex + c0 + j < 2 * kSelChunk) owner[ex + c0 + j] = (uint16_t)(l0 + 1);
  __syncthreads();
  tick(9);
  const uint32_t T = total;
  auto slab_at = [&](uint32_t l, uint32_t j) -> size_t {
    return ((size_t)(l >> 2) * kMfmaQueries + q) * cap + (l & 3) * sub + j;
  };
  auto list_of = [&](uint32_t i) -> uint32_t {
    if (i < 2 * kSelChunk) return owner[i];
    uint32_t lo = 0, hi = 2 * kSelThreads;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (pre[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
  };
  // the passing quarters' slabs: rows whose upper bound (the tile's m) reaches Tcut
  // (r05: 8 slabs held per thread, so a query's ~3.5k (10M, k = 10) to ~17k
  // (C5, k = 50) slabs take half the dependent slab -> meta round trips)
  constexpr int kQ8Held = 2 * kSelHeld;
  for (uint32_t base = 0; base < (slow ? 0u : T); base += kQ8Held * kSelThreads) {
    i32x4_t v[kQ8Held][2];
    uint32_t tl[kQ8Held], ls[kQ8Held];
    bool ok[kQ8Held];
#pragma unroll
    for (int u = 0; u < kQ8Held; ++u) {
      const uint32_t i = base + tid + (uint32_t)u * kSelThreads;
      ok[u] = i < T;
      const uint32_t l = ok[u] ? list_of(i) : 0u;
      const size_t e = slab_at(l, ok[u] ? i - pre[l] : 0u);
      ls[u] = l;
      v[u][0] = __builtin_bit_cast(i32x4_t, slabs[2 * e]);
      v[u][1] = __builtin_bit_cast(i32x4_t, slabs[2 * e + 1]);
      tl[u] = ok[u] ? tiles[e] : row_base;
    }
    if (base == 0) tick(10);
#pragma unroll
    for (int u = 0; u < kQ8Held; ++u) {
      const uint32_t lt = (tl[u] - row_base) >> 5;
      const float dt = meta[2 * (size_t)lt], nt = meta[2 * (size_t)lt + 1];
      const float mt = pa * dt + (pc + sig) * nt;
      if (!ok[u]) continue;
#pragma unroll
      for (int bb = 0; bb < 8; ++bb) {
        const int dv = v[u][bb >> 2][bb & 3];
        if (dv == INT_MIN) continue;
        const float U = (float)dv * sqS + mt;
        if (U >= Tcut) {
          const uint32_t row = tl[u] - row_base + 16u * (uint32_t)(bb >> 2) + 4u * (ls[u] & 3) +
                               (uint32_t)(bb & 3);
          const uint32_t pos = atomicAdd(&fill, 1u);
          // survivor entry: the upper bound's order-preserving image, the row
          // (-0 as +0, as make_key ranks it: images compare across the two)
          if (pos < (uint32_t)kMfmaSelBuf)
            buf[pos] = ((uint64_t)vs::score_ord(U == 0.0f ? 0.0f : U) << 32) | row;
          else spill = 1u;
        }
      }
    }
    if (base == 0) tick(11);
  }
  __syncthreads();
  tick(2);
  if constexpr (SV == 2) return;
  const uint32_t ns = fill;
  if (stats && tid == 0) {  // (tools/q8_check.hip) slabs read, survivors
    atomicAdd(stats, T);
    atomicAdd(stats + 1, ns);
  }
  // rescore on the bf16 pass's own arithmetic: 16 survivors per group as the
  // A rows of v_mfma_f32_16x16x32_bf16, the query as every B column, the
  // row's 64-B steps in the pass's order from a zero accumulator -- each
  // score is the bf16 pass's, bit for bit (an MFMA output element depends
  // on its own row, column and accumulator only). Lane (col, kq) loads bytes
  // 64 s + 16 kq of row col of the group and of the query, as the pass does.
  constexpr int RBY = D * (F32 ? 4 : 2);  // row bytes
  constexpr int TS = RBY / 64;            // 64-B steps per row
  // rows past 24 steps (bf16 D = 1024, fp32): the query's fragments come from
  // LDS, and rows are read in rounds of 16 / 24 steps
  constexpr bool kQL = TS > 24;
  constexpr int HS = TS % 24 == 0 ? 24 : (TS % 16 == 0 ? 16 : TS);  // steps held per round
  static_assert(TS % HS == 0, "whole rounds of steps");
  __shared__ uint4 qsh[kQL ? RBY / 16 : 1];
  const int col = (int)(lane & 15), kq = (int)(lane >> 4);
  uint4 qf[kQL ? 1 : TS];
  {
    const uint4* qrow = (const uint4*)((const unsigned char*)qb + (size_t)q * RBY);
    if constexpr (kQL) {
      for (uint32_t i = tid; i < (uint32_t)RBY / 16; i += kSelThreads) qsh[i] = qrow[i];
      __syncthreads();
    } else {
#pragma unroll
      for (int t = 0; t < TS; ++t) qf[t] = qrow[4 * t + kq];
    }
  }
  // the score of row r (lane col's) by the pass's chain; C[4 kq + i][col] =
  // the score of the group's row 4 kq + i (every column alike)
  auto score16 = [&](uint32_t r) -> f32x4_t {
    const uint4* xrow = (const uint4*)((const unsigned char*)X + (size_t)r * RBY);
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int h = 0; h < TS / HS; ++h) {
      uint4 af[HS];
#pragma unroll
      for (int t = 0; t < HS; ++t) af[t] = xrow[4 * (h * HS + t) + kq];
#pragma unroll
      for (int t = 0; t < HS; ++t) {
        const int ts = h * HS + t;
        const uint4 bq = kQL ? qsh[4 * ts + kq] : qf[kQL ? 0 : ts];
        if constexpr (F32) {
          const f32x4_t av = __builtin_bit_cast(f32x4_t, af[t]), bv = __builtin_bit_cast(f32x4_t, bq);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], bv[j], acc, 0, 0, 0);
        } else {
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[t]),
                                                        __builtin_bit_cast(bf16x8_t, bq), acc, 0, 0, 0);
        }
      }
    }
    return acc;
  };
  // Rescore the survivors buf[0, ns) whose entry passes `pred` into res: each
  // wave takes 64 entries at a time and runs the passing ones in groups of
  // 16 (ballot ranks place them in its wscr row), one slot reservation per
  // group.
  // (r05) A wave packs its passing entries across its 64-entry slices into
  // full groups of 16 (wscr[w][0, pend) carries a partial group from slice
  // to slice): a sparse pass (round 1 picks ~k of thousands) runs a group per
  // wave instead of a near-empty group per slice.
  auto run_group = [&](uint32_t cnt16) {
    const uint32_t r = wscr[w][(uint32_t)col < cnt16 ? col : 0];
    const f32x4_t acc = score16(r);
    uint32_t slot = 0;
    if (lane == 0) slot = atomicAdd(&rfill, cnt16);
    slot = (uint32_t)__shfl((int)slot, 0, 64);
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const uint32_t j = 4 * (uint32_t)kq + (uint32_t)ii;
      const uint32_t rj = (uint32_t)__shfl((int)r, (int)j, 64);  // lane j (kq = 0) has row j
      if (col == 0 && j < cnt16) res[slot + j] = make_key(acc[ii], row_base + rj);
    }
    __builtin_amdgcn_wave_barrier();
  };
  auto rescore_n = [&](uint32_t nb, auto pred) {
    uint32_t pend = 0;  // rows waiting in wscr[w][0, pend) (wave-uniform)
    for (uint32_t base = w * 64; base < nb; base += kSelThreads) {
      const uint32_t i = base + lane;
      const uint64_t e = i < nb ? buf[i] : 0ull;
      const bool pass = i < nb && pred(e);
      const uint64_t bal = __ballot(pass);
      const uint32_t rank = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
      const uint32_t total = (uint32_t)__popcll(bal);
      for (uint32_t done = 0; done < total;) {
        const uint32_t take = 16 - pend < total - done ? 16 - pend : total - done;
        if (pass && rank >= done && rank < done + take) wscr[w][pend + rank - done] = (uint32_t)e;
        __builtin_amdgcn_wave_barrier();
        pend += take;
        done += take;
        if (pend == 16) {
          run_group(16);
          pend = 0;
        }
      }
    }
    if (pend) run_group(pend);
  };
  auto rescore_where = [&](auto pred) { rescore_n(ns, pred); };
  // (r05) Slow path -- a passing lossy quarter (the pass dropped slabs: its
  // rows are recomputed from the int8 copy) or more survivors than the
  // buffer: an exact streaming top k over the same candidates. Rounds of at
  // most 4096 rows whose U image reaches the cutoff (the passing quarters'
  // slabs, one per thread; then the lossy quarters' rows, a tile's 8 rows of
  // the quarter per thread) are rescored on the pass's chain; the running
  // top k stays in res[0, rfill) and the cutoff rises to its k-th exact score
  // (no row under it can enter). Replaces r04's hand-back of the whole batch
  // to a gated bf16 pass, whose two launches every batch paid ~5-8 us for.
  if (slow || spill) {  // uniform
    __shared__ uint32_t cut_sh, nlq;
    __shared__ uint16_t lq[4 * kMfmaMaxLists];
    __shared__ __attribute__((aligned(16))) int8_t q8s[D];
    for (uint32_t i = tid; i < D / 16; i += kSelThreads)
      ((uint4*)q8s)[i] = ((const uint4*)(r8.q8 + (size_t)q * D))[i];
    if (tid == 0) {
      cut_sh = Tcut == -INFINITY ? 0u : vs::score_ord(Tcut == 0.0f ? 0.0f : Tcut);
      rfill = 0, nlq = 0, fill = 0;
    }
    __syncthreads();
    if (lossy0) lq[atomicAdd(&nlq, 1u)] = (uint16_t)l0;
    if (lossy1) lq[atomicAdd(&nlq, 1u)] = (uint16_t)(l0 + 1);
    auto push = [&](float U, uint32_t row) {  // row: local
      const uint32_t img = vs::score_ord(U == 0.0f ? 0.0f : U);
      if (img >= cut_sh) buf[atomicAdd(&fill, 1u)] = ((uint64_t)img << 32) | row;
    };
    auto round_end = [&]() {
      __syncthreads();
      const uint32_t nb = fill;
      if (nb == 0) return;  // uniform
      rescore_n(nb, [](uint64_t) { return true; });
      __syncthreads();
      const uint32_t nr = rfill;
      if (nr > k) {
        // keep the top k: the keys in or above the k-th's bucket, sorted
        const uint32_t P = kth_floor(res, nr, k);
        if (tid == 0) fill = 0;
        __syncthreads();
        for (uint32_t i = tid; i < nr; i += kSelThreads)
          if ((uint32_t)(res[i] >> 32) >= P) buf[atomicAdd(&fill, 1u)] = res[i];
        __syncthreads();
        const uint32_t nf = fill;
        int p2 = 1;
        while ((uint32_t)p2 < nf) p2 <<= 1;
        for (uint32_t i = nf + tid; i < (uint32_t)p2; i += kSelThreads) buf[i] = 0;
        __syncthreads();
        bitonic_sort_desc_n(buf, p2, kSelThreads);
        for (uint32_t j = tid; j < k; j += kSelThreads) res[j] = buf[j];
        __syncthreads();
        if (tid == 0) {
          rfill = k;
          const uint32_t sk = (uint32_t)(res[k - 1] >> 32);  // the k-th exact score's image
          cut_sh = sk > cut_sh ? sk : cut_sh;
        }
      }
      if (tid == 0) fill = 0;
      __syncthreads();
    };
    for (uint32_t base = 0; base < T; base += kSelThreads) {
      const uint32_t i = base + tid;
      if (i < T) {
        const uint32_t l = list_of(i);
        const size_t e = slab_at(l, i - pre[l]);
        const i32x4_t v0 = __builtin_bit_cast(i32x4_t, slabs[2 * e]);
        const i32x4_t v1 = __builtin_bit_cast(i32x4_t, slabs[2 * e + 1]);
        const uint32_t lr0 = tiles[e] - row_base, lt = lr0 >> 5;
        const float mt = pa * meta[2 * (size_t)lt] + (pc + sig) * meta[2 * (size_t)lt + 1];
#pragma unroll
        for (int bb = 0; bb < 8; ++bb) {
          const int dv = bb < 4 ? v0[bb] : v1[bb - 4];
          if (dv != INT_MIN)
            push((float)dv * sqS + mt,
                 lr0 + 16u * (uint32_t)(bb >> 2) + 4u * (l & 3) + (uint32_t)(bb & 3));
        }
      }
      round_end();
    }
    const uint32_t nlossy = nlq;
    for (uint32_t j = 0; j < nlossy; ++j) {
      const uint32_t l = lq[j], wg = l >> 2, kql = l & 3;
      const uint32_t wr0 = wg * r8.rows_per_wg;
      const uint32_t wr1 = (uint64_t)wr0 + r8.rows_per_wg < r8.n_rows ? wr0 + r8.rows_per_wg : r8.n_rows;
      const uint32_t t0 = wr0 / 32, t1 = (wr1 + 31) / 32;
      for (uint32_t base = t0; base < t1; base += kSelThreads) {
        const uint32_t tt = base + tid;
        if (tt < t1) {
          const float mt = pa * meta[2 * (size_t)tt] + (pc + sig) * meta[2 * (size_t)tt + 1];
#pragma unroll 1
          for (int bb = 0; bb < 8; ++bb) {
            const uint32_t row = tt * 32 + 16u * (uint32_t)(bb >> 2) + 4u * kql + (uint32_t)(bb & 3);
            if (row < wr1 && row_allowed(r8.allow, row))
              push((float)q8_row_dot<D>(r8.x8 + (size_t)row * D, q8s) * sqS + mt, row);
          }
        }
        round_end();
      }
    }
    // the running top k (sorted once a round compacted it)
    const uint32_t nr = rfill;
    if (nr <= 64) {
      if (w == 0) sel_finish_wave(res, nr, k, (int)lane, out + (size_t)q * k);
    } else {
      int p2 = 1;
      while ((uint32_t)p2 < nr) p2 <<= 1;
      for (uint32_t i = nr + tid; i < (uint32_t)p2; i += kSelThreads) res[i] = 0;
      __syncthreads();
      bitonic_sort_desc_n(res, p2, kSelThreads);
      for (uint32_t j = tid; j < k; j += kSelThreads) out[(size_t)q * k + j] = j < nr ? res[j] : 0;
    }
    if (stats && tid == 0) atomicAdd(stats + 2, 1u);  // (tools) slow-path queries
    tick(4);
    return;
  }
  if (ns > k + 64 && ns >= two_from) {
    // Two rounds (r04; r05: radix floors for every k): the survivors whose U
    // image reaches P1 (the floor of the bucket of the k-th largest U: at
    // least k of them) first; P2, the floor of the k-th best exact score
    // among those, is at most the k-th score, so only survivors under P1
    // whose U reaches P2 can still enter -- the window shrinks from ~2m to ~m.
    const uint32_t P1 = kth_floor(buf, ns, k);
    tick(5);
    rescore_where([&](uint64_t e) { return (uint32_t)(e >> 32) >= P1; });
    __syncthreads();
    tick(6);
    const uint32_t P2 = kth_floor(res, rfill, k);
    tick(7);
    rescore_where([&](uint64_t e) {
      const uint32_t u = (uint32_t)(e >> 32);
      return u < P1 && u >= P2;
    });
  } else {
    rescore_where([&](uint64_t) { return true; });
  }
  if constexpr (SV == 3) return;
  __syncthreads();
  tick(3);
  // the final top k: the keys whose score image reaches the floor of the
  // k-th (at least k, a few more in its bucket), sorted
  const uint32_t nr = rfill;
  const uint64_t* fin = res;
  uint32_t nf = nr;
  if (nr > 64) {
    const uint32_t P3 = kth_floor(res, nr, k);
    if (tid == 0) fill = 0;
    __syncthreads();
    for (uint32_t i = tid; i < nr; i += kSelThreads) {
      const uint64_t e = res[i];
      if ((uint32_t)(e >> 32) >= P3) buf[atomicAdd(&fill, 1u)] = e;
    }
    __syncthreads();
    fin = buf;
    nf = fill;
  }
  if (nf <= 64) {
    if (w == 0) sel_finish_wave(fin, nf, k, (int)lane, out + (size_t)q * k);
    tick(4);
    return;
  }
  uint64_t* srt = const_cast<uint64_t*>(fin);
  int p2 = 1;
  while ((uint32_t)p2 < nf) p2 <<= 1;
  for (uint32_t i = nf + tid; i < (uint32_t)p2; i += kSelThreads) srt[i] = 0;
  __syncthreads();
  bitonic_sort_desc_n(srt, p2, kSelThreads);
  for (uint32_t j = tid; j < k; j += kSelThreads) out[(size_t)q * k + j] = j < nf ? srt[j] : 0;
  tick(4);
}

// The select kernel: the body above, then -- with SpecVerifyArgs (r06
// ablation, VS_Q8_SEL_VERIFY=1; measured no faster than the launch it saves)
// -- the batch's check (a speculative batch) or record (a sample-path one) by
// the last workgroup to finish, the work q8_verify_record_kernel does in a
// launch of its own (vs_spec_dev.h): each workgroup hands its query's values
// over (vq) and takes a ticket (agent-scope release / acquire, as
// gemv_one_finish); the last runs spec_verify_core over all of them and
// leaves the ticket zero. run_if: stand down unless *run_if.
template <int D, int SV = 0, bool F32 = false>
__global__ __launch_bounds__(kSelThreads) void select_q8_kernel(
    const f32x4_t* __restrict__ slabs, const uint32_t* __restrict__ tiles,
    const uint32_t* __restrict__ cnt, const int* __restrict__ cmax, uint32_t nwg, uint32_t cap,
    uint32_t k, uint64_t* __restrict__ out, uint32_t row_base, const void* __restrict__ X,
    const void* __restrict__ qb, uint32_t dim, const f32x4_t* __restrict__ q8par,
    const float* __restrict__ q8glob, const float* __restrict__ meta,
    const float* __restrict__ bound, const Q8Rows r8, uint32_t two_from, uint32_t opts,
    uint32_t* __restrict__ stats, uint64_t* __restrict__ clk, const uint32_t* __restrict__ run_if,
    const SpecVerifyArgs va) {
  if (run_if && *run_if == 0u) return;  // (r05) the fallback behind a verified speculative batch
  select_q8_body<D, SV, F32>(slabs, tiles, cnt, cmax, nwg, cap, k, out, row_base, X, qb, dim, q8par,
                             q8glob, meta, bound, r8, two_from, opts, stats, clk);
  if (!va.vq) return;
  __shared__ float vrq[kMfmaQueries];
  __shared__ float vpick;
  __shared__ int vlast;
  __syncthreads();  // every path of the body has written this query's k keys
  const uint32_t q = blockIdx.x, nq = gridDim.x, t = threadIdx.x;
  if (t == 0) {
    float r, qn;
    bool ok;
    const float b = va.bound[q];
    spec_query_vals(out[(size_t)q * k + k - 1], va.q8par[4 * (size_t)q + 3], b, va.glob[2], va.dim,
                    va.check != 0u, r, qn, ok);
    va.vq[q] = float4{r, qn, b, ok ? 1.f : 0.f};
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const uint32_t prev =
        __hip_atomic_fetch_add(va.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    vlast = prev == nq - 1;
    if (vlast) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  if (!vlast) return;
  float4 v{INFINITY, 0.f, -INFINITY, 1.f};
  if (t < nq) v = va.vq[t];
  spec_verify_core(t < nq, v.x, v.y, v.z, v.w != 0.f, va, vrq, &vpick);
  if (t == 0) __hip_atomic_store(va.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

hipError_t launch_select_q8(const float* slabs, const uint32_t* slab_tile, const uint32_t* cand_cnt,
                            const uint32_t* cand_max, uint32_t nwg, uint32_t cap, uint32_t nq,
                            uint32_t k, uint64_t* out,
                            uint32_t row_base, const void* X, const void* qb, bool f32, uint32_t dim,
                            const float* q8par, const float* q8glob, const float* meta,
                            const float* bound, const void* X8, const void* Q8,
                            const uint64_t* allow, uint32_t n_rows, hipStream_t st, uint32_t* stats,
                            uint64_t* clk, const uint32_t* run_if, const SpecVerifyArgs* verify) {
  if (!select_args_ok(nwg, cap, nq, k) || !cand_max || !X8 || !Q8) return hipErrorInvalidValue;
  if (verify && (!verify->vq || !verify->ticket || !verify->sk || !verify->stat || !verify->bound ||
                 (verify->check && !verify->gate) || nq > kMfmaQueries))
    return hipErrorInvalidValue;
  const SpecVerifyArgs va = verify ? *verify : SpecVerifyArgs{};
  uint32_t gwg = 0, rpw = 0;
  mfma_grid(n_rows, &gwg, &rpw);
  if (gwg != nwg) return hipErrorInvalidValue;  // the pass's static split
  const Q8Rows r8{(const int8_t*)X8, (const int8_t*)Q8, allow, n_rows, rpw, row_base};
  // VS_Q8_TWO_ROUND_FROM (read once): the survivor count from which the
  // select rescores in two rounds (the top k by U first, then only survivors
  // whose U reaches their k-th exact score); below it, one round
  static const uint32_t two_from = [] {
    const char* e = getenv("VS_Q8_TWO_ROUND_FROM");
    return e ? (uint32_t)atoi(e) : 0u;
  }();
  static const int sv = [] {
    const char* e = getenv("VS_Q8_SEL_SV");
    return e ? atoi(e) : 0;
  }();
  static const uint32_t opts = [] {
    const char* e = getenv("VS_Q8_SEL_P0");
    return e && atoi(e) == 0 ? 1u : 0u;
  }();
  decltype(&select_q8_kernel<768, 0, false>) kern;
  if (f32 && dim == 768)
    kern = select_q8_kernel<768, 0, true>;
  else if (!f32 && dim == 1024)
    kern = select_q8_kernel<1024, 0, false>;
  else if (!f32 && dim == 768)
    kern = sv == 1 ? select_q8_kernel<768, 1> : sv == 2 ? select_q8_kernel<768, 2>
         : sv == 3 ? select_q8_kernel<768, 3> : select_q8_kernel<768, 0>;
  else
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(kern, dim3(nq), dim3(kSelThreads), 0, st, (const f32x4_t*)slabs, slab_tile,
                     cand_cnt, (const int*)cand_max, nwg, cap, k, out, row_base, X, qb, dim,
                     (const f32x4_t*)q8par, q8glob, meta, bound, r8, two_from, opts, stats, clk,
                     run_if, va);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// merge: global top-k over L sorted lists per query
// ---------------------------------------------------------------------------
// One workgroup per query. Lower bound: the k-th entry of any full list is
// <= the global k-th key, so only keys >= max_l list_l[k-1] can enter. The
// candidates are streamed in chunks; survivors are appended to an LDS buffer
// that also holds the running top-k, which is re-sorted (bitonic) only when a
// chunk added something. Correct for any input; fast when the bound is good.
__device__ __forceinline__ void bitonic_sort_desc(uint64_t* buf, int n_pow2) {
  for (int size = 2; size <= n_pow2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < n_pow2 / 2; i += kMergeThreads) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool desc = ((lo & size) == 0);
        const uint64_t a = buf[lo], b = buf[hi];
        if ((a < b) == desc) {
          buf[lo] = b;
          buf[hi] = a;
        }
      }
      __syncthreads();
    }
  }
}

// buf[0, c) sorted descending -> its distinct non-zero keys moved to the
// front, in order (wave 0, 64 keys per round, in place: a key is written at
// or before the slot it was read from, after its whole round was read).
// Returns the number of distinct keys to every thread (through cnt_sh).
__device__ __forceinline__ uint32_t dedupe_sorted(uint64_t* buf, uint32_t c, uint32_t& cnt_sh) {
  if (threadIdx.x < 64) {
    const int lane = (int)threadIdx.x;
    uint32_t w = 0;
    uint64_t prev = 0;  // the (original) key before this round; keys are non-zero
    for (uint32_t b = 0; b < c; b += 64) {
      const uint32_t i = b + (uint32_t)lane;
      const uint64_t x = i < c ? buf[i] : 0ull;
      uint64_t p = shfl_up64(x);
      if (lane == 0) p = prev;
      prev = readlane64(x, 63);
      const bool keep = x != 0 && x != p;
      const uint64_t bal = __ballot(keep);
      if (keep) buf[w + (uint32_t)__popcll(bal & ((1ull << lane) - 1))] = x;
      w += (uint32_t)__popcll(bal);
    }
    if (lane == 0) cnt_sh = w;
  }
  __syncthreads();
  return cnt_sh;
}

// A key of buf[0, ns) with at least k sampled keys at or above it: for
// ns <= 256 the smallest with at most k - 1 above it (by rank), through nz the
// non-zero sampled keys; past 256 the k-th distinct key after a sort, nz the
// distinct ones. ~0 if none. ns <= kMergeThreads, red holds kMergeThreads / 64
// words. Ends with buf free for reuse.
__device__ __forceinline__ uint64_t sample_kth(uint64_t* buf, uint32_t ns, uint32_t k,
                                               uint64_t* red, uint32_t& nz) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (ns > 256) {
    // ranking every key against all ns is LDS-bandwidth bound past a few
    // hundred keys (each broadcast read still returns a KiB per wave): sort
    // instead, then the k-th distinct key (exactly k distinct keys >= it)
    int p2 = 1;
    while ((uint32_t)p2 < ns) p2 <<= 1;
    for (uint32_t i = ns + threadIdx.x; i < (uint32_t)p2; i += kMergeThreads) buf[i] = 0;
    __syncthreads();
    bitonic_sort_desc(buf, p2);
    __shared__ uint32_t u_sh;
    const uint32_t u = dedupe_sorted(buf, ns, u_sh);
    nz = u;
    const uint64_t sb = u >= k ? buf[k - 1] : ~0ull;
    __syncthreads();  // buf reads done
    return sb;
  }
  const uint64_t x = threadIdx.x < ns ? buf[threadIdx.x] : 0ull;
  uint64_t cand = ~0ull;
  uint32_t nzc = x != 0 ? 1u : 0u;
  if (x != 0) {
    uint32_t r = 0;
    for (uint32_t j = 0; j < ns; ++j) r += buf[j] > x ? 1u : 0u;
    if (r < k) cand = x;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t y = __shfl_xor(cand, o, 64);
    cand = y < cand ? y : cand;
    nzc += __shfl_xor(nzc, o, 64);
  }
  __syncthreads();  // buf reads done
  if (lane == 0) {
    red[w] = cand;
    buf[w] = nzc;
  }
  __syncthreads();
  uint64_t sb = ~0ull;
  nz = 0;
  for (int i = 0; i < kMergeThreads / 64; ++i) {
    sb = red[i] < sb ? red[i] : sb;
    nz += (uint32_t)buf[i];
  }
  __syncthreads();  // red / buf reads done
  return sb;
}

// The c survivors buf[0, c) (every key at or above a sample bound) -> the
// top k of their distinct keys in out[0, k): by rank when c <= 512 (a
// repeated key counts at its first position only), else bitonic sort +
// dedupe. False (nothing written) when they hold fewer than k distinct keys
// or c > kMergeCap. cnt_sh: shared scratch.
__device__ __forceinline__ bool place_survivors(uint64_t* buf, uint32_t c, uint32_t k,
                                                uint64_t* __restrict__ out, uint32_t& cnt_sh) {
  if (c <= 64) {  // rank is O(c^2) LDS broadcast reads: a sort past a few dozen
    const uint32_t t = threadIdx.x;
    const uint64_t x = t < c ? buf[t] : 0ull;
    bool first = x != 0;
    for (uint32_t i = 0; first && i < t; ++i) first = buf[i] != x;
    buf[kMergeThreads + t] = first ? x : 0ull;
    const uint32_t u2 = (uint32_t)__syncthreads_count(first);
    if (u2 < k) return false;
    if (first) {
      uint32_t rank = 0;
      for (uint32_t i = 0; i < c; ++i) rank += buf[kMergeThreads + i] > x ? 1u : 0u;
      if (rank < k) out[rank] = x;
    }
    return true;
  }
  if (c > (uint32_t)kMergeCap) return false;
  int p3 = 1;
  while ((uint32_t)p3 < c) p3 <<= 1;
  for (uint32_t i = c + threadIdx.x; i < (uint32_t)p3; i += kMergeThreads) buf[i] = 0;
  __syncthreads();
  bitonic_sort_desc(buf, p3);
  const uint32_t u2 = dedupe_sorted(buf, c, cnt_sh);
  if (u2 < k) return false;
  for (uint32_t j = threadIdx.x; j < k; j += kMergeThreads) out[j] = buf[j];
  return true;
}

// Top-k of query q over L lists (merge_keys_kernel; also select_slab_kernel's
// overflow fallback). buf holds >= kMergeCap keys; red / cnt are the
// caller's shared scratch. One workgroup of kMergeThreads threads.
__device__ __forceinline__ void merge_query(const uint64_t* __restrict__ lists, uint32_t L,
                                            uint64_t lstride, uint64_t qstride, uint32_t kin,
                                            uint32_t k, uint32_t q, uint64_t* __restrict__ out,
                                            uint64_t* buf, uint64_t* red, uint32_t& cnt,
                                            bool tourney) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;

  // Fast path (single-query GEMV merges and shard merges at k <= 32): all
  // L * kin keys fit kMergeHeld per thread, so they are read in ONE memory
  // round trip, and the top k is taken by tournament: each wave extracts its
  // k largest (wave max by xor-shuffles, k rounds; 0 = empty; every copy of
  // an extracted key is dropped, so a key listed twice comes out once), then
  // wave 0 extracts the k largest of the 8 waves' winners. The
  // general path below filters against max_l list_l[k-1], which admitted
  // hundreds of keys here (a weak bound over many short lists) and paid a
  // block-wide bitonic sort for them.
  const uint64_t total0 = (uint64_t)L * kin;
  // Few keys (cross-shard merges: P x k; small collections): one key per
  // thread, and each key's output slot is its rank, the number of keys above
  // it among the distinct keys (a loop of LDS broadcast reads; 0 = empty). No
  // shuffle rounds: P = 8, k = 10 was 10 + 10 dependent wave-max rounds.
  // (r03: up to 128 keys -- the rank loops are O(keys^2) LDS broadcast reads,
  // 448 keys took ~10 us more than the sample-bound path below)
  if (total0 <= 128) {
    const uint32_t t = threadIdx.x, tot = (uint32_t)total0;
    uint64_t x = 0;
    if (t < tot) {
      const uint32_t l = t / kin, j = t - l * kin;
      x = lists[l * lstride + q * qstride + j];
    }
    buf[t] = x;
    __syncthreads();
    // a key listed more than once (overlapping or replicated lists) is kept
    // at its first position only, so ranks are distinct and every slot below
    // the number of distinct keys is written
    bool first = x != 0;
    for (uint32_t i = 0; first && i < t; ++i) first = buf[i] != x;
    buf[kMergeThreads + t] = first ? x : 0ull;
    __syncthreads();
    if (first) {
      uint32_t rank = 0;
      for (uint32_t i = 0; i < tot; ++i) rank += buf[kMergeThreads + i] > x ? 1u : 0u;
      if (rank < k) out[(size_t)q * k + rank] = x;
    }
    const uint32_t nz = (uint32_t)__syncthreads_count(first);  // also: buf reads done
    for (uint32_t r = nz + t; r < k; r += kMergeThreads) out[(size_t)q * k + r] = 0;
    return;
  }
  // (r03: off unless VS_MERGE_TOURNEY=1 -- the sample-bound path below is
  // faster; profiles/r03_merge_tourney_ab.jsonl, r03_merge_lat.jsonl)
  if (tourney && L >= 256 && k <= 10 && total0 <= (uint64_t)kMergeThreads * kMergeHeld) {
    uint64_t x[kMergeHeld];
    // every load issued unconditionally (clamped index), all in flight at
    // once; a conditional load per key compiled to one round trip each
#pragma unroll
    for (int u = 0; u < kMergeHeld; ++u) {
      const uint32_t i0 = threadIdx.x + (uint32_t)u * kMergeThreads;
      const uint32_t i = i0 < total0 ? i0 : 0u;
      const uint32_t l = i / kin, j = i - l * kin;
      x[u] = lists[l * lstride + q * qstride + j];
    }
#pragma unroll
    for (int u = 0; u < kMergeHeld; ++u)
      if (threadIdx.x + (uint32_t)u * kMergeThreads >= total0) x[u] = 0;
    auto lane_max = [&]() {
      uint64_t m = 0;
#pragma unroll
      for (int u = 0; u < kMergeHeld; ++u) m = x[u] > m ? x[u] : m;
      return m;
    };
    auto wave_max = [&](uint64_t v) {
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) {
        const uint64_t o = __shfl_xor(v, m, 64);
        v = o > v ? o : v;
      }
      return v;
    };
    uint64_t lm = lane_max();
    for (uint32_t r = 0; r < k; ++r) {
      const uint64_t wm = wave_max(lm);
      if (lane == 0) buf[w * 32 + r] = wm;
      if (wm != 0 && lm == wm) {  // every lane holding it drops all its copies
#pragma unroll
        for (int u = 0; u < kMergeHeld; ++u) x[u] = x[u] == wm ? 0ull : x[u];
        lm = lane_max();
      }
    }
    __syncthreads();
    if (w == 0) {
      // 8 waves x k winners: lane l holds winners l, l + 64, l + 128, l + 192
      uint64_t y[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t e = (uint32_t)lane + 64u * (uint32_t)u, ww = e / 32, rr = e % 32;
        y[u] = rr < k ? buf[ww * 32 + rr] : 0ull;
      }
      uint64_t m2 = 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) m2 = y[u] > m2 ? y[u] : m2;
      for (uint32_t r = 0; r < k; ++r) {
        const uint64_t wm = wave_max(m2);
        if (lane == 0) out[(size_t)q * k + r] = wm;
        if (wm != 0 && m2 == wm) {
#pragma unroll
          for (int u = 0; u < 4; ++u) y[u] = y[u] == wm ? 0ull : y[u];
          m2 = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u) m2 = y[u] > m2 ? y[u] : m2;
        }
      }
    }
    return;
  }

  // Sample bound + list walk (r03). The lists are sorted descending without
  // repeats, so the k-th largest key among the first m entries of every list
  // (a subset of the keys) has at least k keys at or above it -- k DISTINCT
  // keys unless lists share keys (replicated shards), which the walk's result
  // reveals (fewer than k distinct survivors: the filter below runs instead).
  // That key bounds the k-th largest key overall from below, so each list is
  // read only down to it: for a single-query GEMV merge a step or two per
  // list instead of all L x kin keys (the filter below read every key and
  // bitonic-sorted whatever passed max_l list_l[k-1], a weak bound: 175 us for
  // 758 lists of 100 at 200k rows). The sample (<= 512 keys: one per thread,
  // so a weaker bound for many lists) is ranked, not sorted, and so are the
  // survivors when they are <= 512: no sort on the common path.
  // Lists held in registers (the common single-query merge: one list per
  // scan workgroup, L >= 2k / 4): each thread loads the first 4 entries of
  // lists t and t + 512 at once, so the sample and the walk's first step are
  // one memory round trip; only a list whose 4th key still passes the bound
  // is read further.
  if (L <= 2u * kMergeThreads && 4ull * L >= 2ull * k) {
    const uint32_t m0 = (2 * k + L - 1) / L;
    const uint32_t m = m0 < 1 ? 1 : (m0 > kin ? kin : (m0 > 4 ? 4 : m0));
    uint64_t h[2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const uint32_t l = threadIdx.x + (uint32_t)a * kMergeThreads;
      const uint64_t* lp = lists + (size_t)(l < L ? l : 0) * lstride + q * qstride;
#pragma unroll
      for (int v = 0; v < 4; ++v) h[a][v] = (l < L && (uint32_t)v < kin) ? lp[v] : 0ull;
    }
    const uint32_t cap = k * 8 < 128 ? 128 : (k * 8 > (uint32_t)kMergeThreads ? kMergeThreads : k * 8);
    const uint32_t ns = L * m < cap ? L * m : cap;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const uint32_t l = threadIdx.x + (uint32_t)a * kMergeThreads;
#pragma unroll
      for (int v = 0; v < 4; ++v)
        if ((uint32_t)v < m && l * m + (uint32_t)v < ns) buf[l * m + v] = h[a][v];
    }
    __syncthreads();
    uint32_t nz;
    const uint64_t sb = sample_kth(buf, ns, k, red, nz);
    if (nz >= k && sb != ~0ull) {
      const uint64_t thr = sb - 1;
      if (threadIdx.x == 0) cnt = 0;
      __syncthreads();
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const uint32_t l = threadIdx.x + (uint32_t)a * kMergeThreads;
#pragma unroll
        for (int v = 0; v < 4; ++v)
          if (h[a][v] > thr) {
            const uint32_t at = atomicAdd(&cnt, 1u);
            if (at < (uint32_t)kMergeCap) buf[at] = h[a][v];
          }
        if (l < L && h[a][3] > thr) {  // the rest of this list, one thread
          const uint64_t* lp = lists + (size_t)l * lstride + q * qstride;
          for (uint32_t j = 4; j < kin; ++j) {
            const uint64_t x = lp[j];
            if (x <= thr) break;
            const uint32_t at = atomicAdd(&cnt, 1u);
            if (at < (uint32_t)kMergeCap) buf[at] = x;
          }
        }
      }
      __syncthreads();
      if (place_survivors(buf, cnt, k, out + (size_t)q * k, cnt)) return;
    }
  } else {
    // Sample bound + list walk over global memory (few lists, or very many)
    constexpr uint32_t kSample = kMergeThreads;  // one sampled key per thread
    const uint32_t m0 = (2 * k + L - 1) / L;
    const uint32_t m = m0 < 1 ? 1 : (m0 > kin ? kin : m0);
    const uint64_t ns64 = (uint64_t)L * m;
    const uint32_t ns = ns64 < (uint64_t)kSample ? (uint32_t)ns64 : kSample;
    (void)ns64;
    if (threadIdx.x < ns) {
      const uint32_t l = threadIdx.x / m, j = threadIdx.x - l * m;
      buf[threadIdx.x] = lists[l * lstride + q * qstride + j];
    }
    __syncthreads();
    uint32_t nz;
    const uint64_t sb = sample_kth(buf, ns, k, red, nz);
    if (nz >= k && sb != ~0ull) {
      const uint64_t sthr = sb - 1;  // survivors: keys >= sb
      if (threadIdx.x == 0) cnt = 0;
      __syncthreads();
      // tpl threads per list (a power of two <= 64: lanes of one wave), each
      // step reading 4 consecutive keys per thread; a list's walk ends at the
      // first step whose last key is under the bound
      uint32_t tpl = 1;
      while (tpl < 64 && (uint64_t)L * tpl * 2 <= (uint64_t)kMergeThreads) tpl <<= 1;
      const uint32_t gpb = kMergeThreads / tpl;
      const uint32_t g = threadIdx.x / tpl, sl = threadIdx.x % tpl;
      const int src = (lane & ~(int)(tpl - 1)) + (int)tpl - 1;
      for (uint32_t l = g; l < L; l += gpb) {
        const uint64_t* lp = lists + l * lstride + q * qstride;
        for (uint32_t j0 = 0; j0 < kin; j0 += tpl * 4) {
          uint64_t x[4];
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const uint32_t j = j0 + sl * 4 + (uint32_t)v;
            x[v] = j < kin ? lp[j] : 0ull;
          }
#pragma unroll
          for (int v = 0; v < 4; ++v)
            if (x[v] > sthr) {
              const uint32_t at = atomicAdd(&cnt, 1u);
              if (at < (uint32_t)kMergeCap) buf[at] = x[v];
            }
          if (__shfl(x[3], src, 64) <= sthr) break;  // the group's last key
        }
      }
      __syncthreads();
      if (place_survivors(buf, cnt, k, out + (size_t)q * k, cnt)) return;
    }
  }
  // fewer than k distinct survivors (lists sharing keys inflated the sample's
  // ranks), or more survivors than the buffer holds (whose distinct count is
  // unknown): the filter below, without the sample bound
  __syncthreads();

  // initial bound (strict filter "key > thr")
  uint64_t b = 0;
  if (kin >= k)
    for (uint32_t l = threadIdx.x; l < L; l += kMergeThreads) {
      const uint64_t x = lists[l * lstride + q * qstride + (k - 1)];
      b = x > b ? x : b;
    }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    const uint64_t o = __shfl_xor(b, m, 64);
    b = o > b ? o : b;
  }
  if (lane == 0) red[w] = b;
  __syncthreads();
  uint64_t bound = 0;
  for (int i = 0; i < kMergeThreads / 64; ++i) bound = red[i] > bound ? red[i] : bound;
  uint64_t thr = bound ? bound - 1 : 0;  // admit the bound itself

  const uint64_t total = (uint64_t)L * kin;
  const uint32_t chunk = kMergeCap - k;
  uint32_t nR = 0;  // running top-k size in buf[0, nR)
  for (uint64_t base = 0; base < total; base += chunk) {
    if (threadIdx.x == 0) cnt = nR;
    __syncthreads();
    const uint64_t end = base + chunk < total ? base + chunk : total;
    // 8 independent loads in flight per thread, then the (rare) appends
    for (uint64_t i0 = base + threadIdx.x; i0 < end; i0 += 8 * kMergeThreads) {
      uint64_t x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint64_t i = i0 + (uint64_t)u * kMergeThreads;
        x[u] = 0;
        if (i < end) {
          const uint32_t l = (uint32_t)(i / kin), j = (uint32_t)(i - (uint64_t)l * kin);
          x[u] = lists[l * lstride + q * qstride + j];
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (x[u] > thr) buf[atomicAdd(&cnt, 1u)] = x[u];
    }
    __syncthreads();
    const uint32_t c = cnt;
    if (c > nR) {
      int p2 = 1;
      while ((uint32_t)p2 < c) p2 <<= 1;
      for (int i = (int)c + threadIdx.x; i < p2; i += kMergeThreads) buf[i] = 0;
      __syncthreads();
      bitonic_sort_desc(buf, p2);
      const uint32_t u = dedupe_sorted(buf, c, cnt);
      nR = u < k ? u : k;
      if (nR == k) {
        const uint64_t kth = buf[k - 1];
        thr = kth > thr ? kth : thr;
      }
    }
    __syncthreads();
  }
  for (uint32_t j = threadIdx.x; j < k; j += kMergeThreads)
    out[(size_t)q * k + j] = j < nR ? buf[j] : 0;
}

__global__ __launch_bounds__(kMergeThreads) void merge_keys_kernel(
    const uint64_t* __restrict__ lists, uint32_t L, uint64_t lstride, uint64_t qstride,
    uint32_t kin, uint32_t k, uint64_t* __restrict__ out, int tourney, uint64_t* flag,
    uint64_t seq) {
  __shared__ uint64_t buf[kMergeCap];
  __shared__ uint64_t red[kMergeThreads / 64];
  __shared__ uint32_t cnt;
  merge_query(lists, L, lstride, qstride, kin, k, blockIdx.x, out, buf, red, cnt, tourney != 0);
  if (flag) publish_host(flag, seq);  // merge_query returns on block-uniform paths
}

// VS_MERGE_TOURNEY=1 (read once; ablation) gives back the register
// tournament for k <= 10 over >= 256 lists. Off by default since r03: the
// sample-bound path with register-held list prefixes is faster at every shape
// measured (one query, 768 lists x 10: 10.2 against 14.2 us;
// profiles/r03_merge_lat.jsonl)
static int merge_tourney() {
  static const int v = [] {
    const char* e = getenv("VS_MERGE_TOURNEY");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  return v;
}

hipError_t launch_merge(const uint64_t* lists, uint32_t L, uint64_t lstride,
                        uint64_t qstride, uint32_t nq, uint32_t kin, uint32_t k, uint64_t* out,
                        hipStream_t st, uint64_t* flag, uint64_t seq) {
  if (k == 0 || k > kMaxK || nq == 0 || L == 0 || kin == 0) return hipErrorInvalidValue;
  if (flag && nq != 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(merge_keys_kernel, dim3(nq), dim3(kMergeThreads), 0, st, lists, L,
                     lstride, qstride, kin, k, out, merge_tourney(), flag, seq);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// single query on the int8 copy (r05; DESIGN.md §5 "Single query on the int8
// copy")
// ---------------------------------------------------------------------------
// A one-query search streams D * e bytes per row through the GEMV; the
// collection's int8 copy (the batched path's prefilter, vs_q8.hip) holds the
// same rows in D bytes (1/2 of bf16, 1/4 of fp32). The bracket is the batched
// int8 path's (select_q8_kernel): with the query's int8 image {sqS, a, c,
// sigma} and the row's tile {dt, nt}, L = sqS dot - mt <= s <= U = sqS dot +
// mt, mt = a dt + (c + sigma) nt, where dot = q8 . x8 is an exact int32 and s
// is the row's fp32 GEMV score (sigma covers any fp32 summation order).
//  1. gemv_q8_scan_kernel: every row's dot on v_dot4_i32_i8 (16 B of a row
//     per lane, 4 rows per wave step, waves interleaved over the rows as the
//     GEMV's), its U and L; per wave the KP = 64 KPL largest U keys (a
//     register list, merged per workgroup by rank: gemv_emit) and, per
//     workgroup (r06; per wave before), the largest L key's score image.
//  2. gemv_q8_finish_kernel: P = the floor of the 24-bit bucket holding the
//     k-th largest of the workgroups' L images (k distinct rows reach it, so
//     it is at most the k-th GEMV score); each workgroup list's entries whose
//     U reaches P are rescored on the GEMV's own per-row arithmetic
//     (gemv_row_score: the same loads, chunk_dot, order and wave_sum, hence
//     the same bits); a list that dropped a key whose U reaches P is replaced
//     by every row of its scan workgroup. Each finishing workgroup appends
//     the keys of its waves' top k whose score reaches P (nothing under P can
//     be in the top k) with one agent-scope add, and the last one
//     (agent-scope hand-off, as gemv_one_finish) sorts that short array.
// Every row of the GEMV's top k has U >= s >= k-th score >= P, so it is
// rescored and its key is the GEMV's: the answer equals the GEMV's bit for bit.
#ifndef VS_Q8G_LISTS
#define VS_Q8G_LISTS 8
#endif
#ifndef VS_Q8G_PASSES
#define VS_Q8G_PASSES 2
#endif
constexpr int kQ8gLists = VS_Q8G_LISTS;  // scan-workgroup lists per finishing workgroup
// the finish's P: 8-bit radix passes over the top 8 x kQ8gPasses bits of the
// workgroup L images (the floor of that bucket), from registers
constexpr int kQ8gPasses = VS_Q8G_PASSES;
constexpr int kQ8gHeld = 2;  // values per thread: up to 1024 scan workgroups

template <int D>
struct Q8GemvShape {
  static constexpr int CPR = D / 16;          // 16-B chunks per int8 row
  static constexpr int RB = 4;                // rows per wave step: one tile (4 | 32)
  static constexpr int J = RB * CPR / 64;     // chunks per lane per step
  static_assert((RB * CPR) % 64 == 0, "whole chunks per lane");
};

template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
}
// exact int32 wave sum (any order), as wave_sum_dpp: rows of 16 lanes by DPP,
// then four readlanes
__device__ __forceinline__ int wave_isum(int v) {
  v += dpp_i<0xB1>(v);
  v += dpp_i<0x4E>(v);
  v += dpp_i<0x141>(v);
  v += dpp_i<0x140>(v);
  return (__builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16)) +
         (__builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48));
}

// 16 int8 products of a chunk on v_dot4_i32_i8 (exact)
__device__ __forceinline__ int chunk_dot8(const uint4& x, const int4& q) {
  int d = __builtin_amdgcn_sdot4((int)x.x, q.x, 0, false);
  d = __builtin_amdgcn_sdot4((int)x.y, q.y, d, false);
  d = __builtin_amdgcn_sdot4((int)x.z, q.z, d, false);
  return __builtin_amdgcn_sdot4((int)x.w, q.w, d, false);
}

// Wave 0: the prepped query qs (LDS, fp32) -> its int8 image q8s and {sqS, a,
// c, sigma} in par (the formulas of vs_q8.hip q8_query_block; S = the
// collection's scale). Each lane reads only the qs entries it wrote.
template <int D>
__device__ __forceinline__ void q8_query_wave(const float* qs, int8_t* q8s, float* par, float S,
                                              int lane) {
  constexpr int PJ = D / 64;
  float v[PJ];
  float amax = 0.f;
#pragma unroll
  for (int j = 0; j < PJ; ++j) {
    v[j] = qs[lane + 64 * j];
    amax = fmaxf(amax, fabsf(v[j]));
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) amax = fmaxf(amax, __shfl_xor(amax, m, 64));
  const float sq = amax > 0.f ? amax / 127.f : 0.f;
  double aa = 0.0, cc = 0.0, nn = 0.0;
#pragma unroll
  for (int j = 0; j < PJ; ++j) {
    const float y = sq > 0.f ? fminf(fmaxf(rintf(v[j] / sq), -127.f), 127.f) : 0.f;
    const double sy = (double)sq * (double)y, e = (double)v[j] - sy;
    aa = aa + sy * sy;
    cc = cc + e * e;
    nn = nn + (double)v[j] * (double)v[j];
    q8s[lane + 64 * j] = (int8_t)(int)y;
  }
  aa = wave_sum_f64(aa);
  cc = wave_sum_f64(cc);
  nn = wave_sum_f64(nn);
  if (lane == 0) {
    par[0] = sq * S;
    par[1] = q8_norm_up(aa);
    par[2] = q8_norm_up(cc);
    par[3] = q8_sigma(D, q8_norm_up(nn));
  }
}

template <int D, int KPL>
__global__ __launch_bounds__(kGemvThreads) void gemv_q8_scan_kernel(
    const int8_t* __restrict__ X8, uint32_t n_rows, uint32_t row_base,
    const float* __restrict__ q_raw, int prep, const float* __restrict__ meta,
    const float* __restrict__ glob, const uint64_t* __restrict__ allow,
    uint64_t* __restrict__ ulist, uint32_t* __restrict__ lbest) {
  using S = Q8GemvShape<D>;
  constexpr int KP = 64 * KPL;
  __shared__ float qs[D];
  __shared__ __attribute__((aligned(16))) int8_t q8s[D];
  __shared__ float par[4];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t gw = blockIdx.x * kGemvWaves + w, nw = gridDim.x * kGemvWaves;
  const uint32_t stride = nw * S::RB;
  int rowsel[S::J], coff[S::J];
#pragma unroll
  for (int j = 0; j < S::J; ++j) {
    const int c = lane + 64 * j;
    rowsel[j] = c / S::CPR;
    coff[j] = c % S::CPR;
  }
#ifndef VS_Q8G_DEPTH
#define VS_Q8G_DEPTH 2
#endif
  // Steps in flight: DEPTH - 1 ahead of the one being summed; each step's
  // tile {dt, nt} is loaded with its rows (r06), not after its dots. (Two or
  // three steps ahead measured slower at C2 -- 129.4 / 131.8 against 125.0 us
  // per scan, the registers cost occupancy: profiles/r06_c2_scan_depth_*.)
  constexpr int DEPTH = VS_Q8G_DEPTH;
  uint4 buf[DEPTH][S::J];
  float2 tmb[DEPTH];
  auto load = [&](int slot, uint32_t r0) {
#pragma unroll
    for (int j = 0; j < S::J; ++j) {
      uint32_t row = r0 + rowsel[j];
      row = row < n_rows ? row : n_rows - 1;
      const u32x4_t v = __builtin_nontemporal_load(
          (const u32x4_t*)(X8 + (size_t)row * D + (size_t)coff[j] * 16));
      buf[slot][j] = uint4{v[0], v[1], v[2], v[3]};
    }
    tmb[slot] = ((const float2*)meta)[r0 >> 5];  // the step's rows share one tile (r0 % 4 == 0)
  };
  const uint32_t lo = gw * S::RB;
#pragma unroll
  for (int d = 0; d < DEPTH - 1; ++d) {
    const uint32_t r0 = lo + (uint32_t)d * stride;
    if (r0 < n_rows) load(d, r0);
  }
  if (w == 0) {
    prep_query_wave<D>(q_raw, prep, qs, lane);  // the GEMV's query, bit for bit
    q8_query_wave<D>(qs, q8s, par, glob[3], lane);
  }
  __syncthreads();
  int4 qv[S::J];
#pragma unroll
  for (int j = 0; j < S::J; ++j) qv[j] = *(const int4*)(q8s + coff[j] * 16);
  const float sqS = par[0], pa = par[1], pc = par[2] + par[3];
  WaveList<KPL> Lst;
  Lst.init();
  uint64_t theta = 0, lmax = 0;
  for (uint32_t r = lo; r < n_rows; r += stride) {
    const uint32_t rn = r + (uint32_t)(DEPTH - 1) * stride;
    load(DEPTH - 1, rn < n_rows ? rn : r);
    int p[S::RB];
#pragma unroll
    for (int b = 0; b < S::RB; ++b) p[b] = 0;
#pragma unroll
    for (int j = 0; j < S::J; ++j) {
      const int d = chunk_dot8(buf[0][j], qv[j]);
#pragma unroll
      for (int b = 0; b < S::RB; ++b) p[b] += rowsel[j] == b ? d : 0;
    }
    // the step's tile {dt, nt}
    const float2 tm = tmb[0];
    const float mt = pa * tm.x + pc * tm.y;
#pragma unroll
    for (int b = 0; b < S::RB; ++b) {
      const int dot = wave_isum(p[b]);
      const uint32_t row = r + b;
      if (row < n_rows && row_allowed(allow, row)) {
        const float xs = (float)dot * sqS;  // |dot| < 2^24: exact in fp32
        const uint64_t ku = make_key(xs + mt, row_base + row);
        if (ku > theta) {
          Lst.insert(ku, KP, lane);
          theta = Lst.kth(KP);
        }
        const uint64_t kl = make_key(xs - mt, row_base + row);
        lmax = kl > lmax ? kl : lmax;
      }
    }
#pragma unroll
    for (int d = 0; d < DEPTH - 1; ++d) {
#pragma unroll
      for (int j = 0; j < S::J; ++j) buf[d][j] = buf[d + 1][j];
      tmb[d] = tmb[d + 1];
    }
  }
  gemv_emit<KPL>(Lst, theta, KP, lane, w, ulist);
  // (r06) the workgroup's largest L image: the finish takes the k-th largest
  // over workgroups (each reached by a distinct row), 8x fewer values than
  // one per wave, and as tight whenever the top k rows sit in distinct
  // workgroups (k <= 128 of ~768)
  __shared__ uint32_t lb;
  if (threadIdx.x == 0) lb = 0;
  __syncthreads();
  if (lane == 0) atomicMax(&lb, (uint32_t)(lmax >> 32));
  __syncthreads();
  if (threadIdx.x == 0) lbest[blockIdx.x] = lb;
}

// The score of local row `row` exactly as the GEMV scan computes it (its
// step's lane layout: the row is row % RB of a step starting at a multiple of
// RB; the lane's chunks of that row in j order, wave_sum): the same bits.
// Lanes without a chunk of the row add nothing (p stays +0, as the scan's
// zero addends leave it). qs: the prepped query (LDS).
template <int D, bool BF16>
__device__ __forceinline__ float gemv_row_score(const void* __restrict__ Xv, uint32_t row,
                                                const float* qs, int lane) {
  using S = GemvShape<D, BF16>;
  const uint32_t b = S::RB == 1 ? 0u : row % (uint32_t)S::RB, r0 = row - b;
  const char* X = (const char*)Xv;
  uint4 c[S::J];
  bool mine[S::J];
  int co[S::J];
#pragma unroll
  for (int j = 0; j < S::J; ++j) {
    const int cc = lane + 64 * j;
    const uint32_t rs = S::RB == 1 ? 0u : (uint32_t)(cc / S::CPR);
    co[j] = cc % S::CPR;
    mine[j] = rs == b;
    c[j] = mine[j] ? *(const uint4*)(X + (size_t)(r0 + rs) * S::RBYTES + (size_t)co[j] * 16)
                   : uint4{0u, 0u, 0u, 0u};
  }
  float p = 0.f;
#pragma unroll
  for (int j = 0; j < S::J; ++j)
    if (mine[j]) {
      float qv[S::EPC];
#pragma unroll
      for (int e = 0; e < S::EPC; ++e) qv[e] = qs[co[j] * S::EPC + e];
      p += chunk_dot<BF16>(c[j], qv);
    }
  return wave_sum(p);
}

template <int D, bool BF16, int KPL>
__global__ __launch_bounds__(kGemvThreads) void gemv_q8_finish_kernel(
    const void* __restrict__ X, uint32_t n_rows, uint32_t row_base,
    const float* __restrict__ q_raw, int prep, const uint64_t* __restrict__ allow, uint32_t k,
    const uint64_t* __restrict__ ulist, const uint32_t* __restrict__ lbest, uint32_t nscan,
    uint64_t* __restrict__ cand, uint32_t* __restrict__ ctr, uint64_t* __restrict__ dst,
    uint64_t* flag, uint64_t seq, uint32_t* __restrict__ stats, uint64_t* __restrict__ clk) {
  using SQ = Q8GemvShape<D>;
  constexpr int KP = 64 * KPL;
  __shared__ float qs[D];
  __shared__ __attribute__((aligned(16))) uint32_t hist[kQ8gPasses][256];
  __shared__ uint64_t surv[kQ8gLists * KP];
  __shared__ uint32_t ns_sh, fb_sh;
  const int lane = threadIdx.x & 63;
  const uint32_t tid = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane((int)(tid >> 6));
  // (tools) stage wall clocks of this workgroup: clk[block][0..7]
  auto stamp = [&](int s) {
    if (clk && tid == 0) clk[(size_t)blockIdx.x * 8 + s] = wall_clock64();
  };
  stamp(0);
  // (r06) the scan's outputs this workgroup reads -- the L images for P and
  // its lists' entries -- are loaded before the query's prep, so their
  // latency runs under it
  const uint32_t m = nscan;
  uint32_t lv[kQ8gHeld];
#pragma unroll
  for (int j = 0; j < kQ8gHeld; ++j) {
    const uint32_t i = tid + (uint32_t)j * kGemvThreads;
    lv[j] = i < m ? lbest[i] : 0u;
  }
  constexpr int kHeldE = (kQ8gLists * KP + kGemvThreads - 1) / kGemvThreads;
  const uint32_t l0 = blockIdx.x * kQ8gLists;
  uint64_t ev[kHeldE];
#pragma unroll
  for (int t = 0; t < kHeldE; ++t) {
    const uint32_t i = tid + (uint32_t)t * kGemvThreads, l = l0 + i / KP;
    ev[t] = i < (uint32_t)(kQ8gLists * KP) && l < nscan ? ulist[(size_t)l * KP + i % KP] : 0ull;
  }
  if (w == 0) prep_query_wave<D>(q_raw, prep, qs, lane);
  if (tid == 0) ns_sh = 0, fb_sh = 0;
  for (uint32_t i = tid; i < (uint32_t)(kQ8gPasses * 256); i += kGemvThreads) (&hist[0][0])[i] = 0;
  __syncthreads();
  stamp(1);
  // 1. P: the radix floor of the k-th largest workgroup L image (0 = a
  // workgroup without rows; one per scan workgroup since r06), 0 when fewer
  // than k are nonzero. (A per-wave bit-by-bit select over the 768 values,
  // no barriers, and an exact rank count of every value against all m in LDS
  // (36 us against 5.5) both measured slower: tools/c2_finish,
  // profiles/r06_c2_finish_*.)
  // The values are held in registers (up to kQ8gHeld per thread: every grid
  // of gfx950's 256 CUs), read from global memory once, not once a pass.
  // (r06) One barrier a pass: every pass has its own histogram (zeroed before
  // the prep's barrier) and every wave picks the digit itself
  // (wave_digit_pick, vs_bound_dev.h; before: 5 barriers a pass).
  uint32_t P = 0;
  {
    uint32_t prefix = 0, kk = k;
    bool some = true;
#pragma unroll
    for (int pass = 0; pass < kQ8gPasses; ++pass) {
      const int shift = 24 - 8 * pass;
      const uint32_t hmask = pass == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
#pragma unroll
      for (int j = 0; j < kQ8gHeld; ++j) {
        const uint32_t u = lv[j];
        if (u && (u & hmask) == prefix) atomicAdd(&hist[pass][(u >> shift) & 255u], 1u);
      }
      __syncthreads();
      // fewer than kk values under the prefix: only when fewer than k are
      // nonzero (pass 0); P = 0 then
      uint32_t dig, above;
      if (!wave_digit_pick(hist[pass], kk, (uint32_t)lane, dig, above)) {
        some = false;
        break;
      }
      prefix |= dig << shift;
      kk -= above;
    }
    P = some ? prefix : 0u;
  }
  stamp(2);
  // 2. the lists' entries whose U reaches P; a list whose dropped keys may
  // reach P (its last entry does) is replaced by all of its workgroup's rows
#pragma unroll
  for (int t = 0; t < kHeldE; ++t) {
    const uint32_t i = tid + (uint32_t)t * kGemvThreads, l = l0 + i / KP, j = i % KP;
    const uint64_t e = ev[t];  // 0 past the lists
    if (j == KP - 1 && e != 0 && (uint32_t)(e >> 32) >= P) atomicOr(&fb_sh, 1u << (l - l0));
    if (e != 0 && (uint32_t)(e >> 32) >= P) surv[atomicAdd(&ns_sh, 1u)] = e;
  }
  __syncthreads();
  stamp(3);
  // 3. rescore: wave w takes survivors w, w + 8, ... (those of fallback lists
  // are rescored below with every row of their workgroup)
  const uint32_t fb = fb_sh, ns = ns_sh;
  WaveList<KPL> R;
  R.init();
  uint64_t theta = 0;
  auto offer = [&](uint32_t row) {  // local row
    const float s = gemv_row_score<D, BF16>(X, row, qs, lane);
    const uint64_t key = make_key(s, row_base + row);
    if (key > theta) {
      R.insert(key, k, lane);
      theta = R.kth(k);
    }
  };
  uint32_t rescored = 0;
  for (uint32_t i = (uint32_t)w; i < ns; i += kGemvWaves) {
    const uint64_t e = surv[i];
    const uint32_t row = vs::key_row(e) - row_base;
    // the scan workgroup this row belongs to (interleaved 4-row steps)
    const uint32_t l = ((row / SQ::RB) % (nscan * kGemvWaves)) / kGemvWaves;
    if ((fb >> (l - l0)) & 1u) continue;
    offer(row);
    ++rescored;
  }
  if (fb) {
    // every row of each fallback list's workgroup: wave w takes its scan wave w
    const uint32_t stride = nscan * kGemvWaves * SQ::RB;
    for (int li = 0; li < kQ8gLists; ++li) {
      if (!((fb >> li) & 1u)) continue;
      const uint32_t gw = (l0 + li) * kGemvWaves + w;
      for (uint32_t r = gw * SQ::RB; r < n_rows; r += stride)
        for (uint32_t b = 0; b < (uint32_t)SQ::RB; ++b) {
          const uint32_t row = r + b;
          if (row < n_rows && row_allowed(allow, row)) {
            offer(row);
            ++rescored;
          }
        }
    }
  }
  if (stats && lane == 0) {
    atomicAdd(&stats[0], rescored);
    if (w == 0) atomicAdd(&stats[1], (uint32_t)__popc(fb));
  }
  // 4. the keys that can still be in the top k -> one compact array. P is at
  // most the k-th score (k distinct rows have L >= P), so a key whose exact
  // score image is under P cannot be; every key at or above it was rescored
  // (its U >= its score >= P). One agent-scope add per workgroup reserves its
  // place (r06: r05 appended every wave's top k through that counter, ~300
  // adds, and the last workgroup sorted the pile; before this form each
  // workgroup wrote its merged top k and the last merged 96 lists).
  __shared__ uint32_t wcnt[kGemvWaves], wbase;
  uint32_t mine = 0;
#pragma unroll
  for (int i = 0; i < KPL; ++i)
    mine += (uint32_t)__popcll(__ballot(R.e[i] != 0 && (uint32_t)(R.e[i] >> 32) >= P));
  if (lane == 0) wcnt[w] = mine;
  __syncthreads();
  if (tid == 0) {
    uint32_t tot = 0;
    for (int j = 0; j < kGemvWaves; ++j) tot += wcnt[j];
    wbase = tot ? __hip_atomic_fetch_add(&ctr[1], tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                : 0u;
  }
  __syncthreads();
  {
    uint32_t at = wbase;
    for (int j = 0; j < w; ++j) at += wcnt[j];
#pragma unroll
    for (int i = 0; i < KPL; ++i) {
      const bool keep = R.e[i] != 0 && (uint32_t)(R.e[i] >> 32) >= P;
      const uint64_t bal = __ballot(keep);
      const uint32_t rank = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
      if (keep) cand[at + rank] = R.e[i];
      at += (uint32_t)__popcll(bal);
    }
  }
  // 5. hand-off: the last workgroup takes the top k of the array
  __shared__ uint64_t mbuf[kMergeCap];
  __shared__ uint64_t red[kMergeThreads / 64];
  __shared__ uint32_t mcnt;
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  stamp(4);
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t prev =
        __hip_atomic_fetch_add(&ctr[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == gridDim.x - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      mcnt = __hip_atomic_load(&ctr[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  stamp(5);
  if (!last) return;
  const uint32_t N = mcnt;
  __syncthreads();
  if (N <= 64) {  // the usual case: a few keys past P; one wave sorts them
    if (w == 0) {
      const uint64_t x = wave_sort_desc((uint32_t)lane < N ? cand[lane] : 0ull, lane);
      for (uint32_t j = (uint32_t)lane; j < k; j += 64) dst[j] = j < 64 ? x : 0ull;
    }
  } else if (N <= (uint32_t)kMergeCap) {  // sorted in LDS
    int p2 = 64;
    while ((uint32_t)p2 < N) p2 <<= 1;
    for (uint32_t i = tid; i < (uint32_t)p2; i += kGemvThreads) mbuf[i] = i < N ? cand[i] : 0ull;
    __syncthreads();
    bitonic_sort_desc_n(mbuf, p2, kGemvThreads);
    for (uint32_t j = tid; j < k; j += kGemvThreads) dst[j] = j < N ? mbuf[j] : 0ull;
  } else {  // (P = 0: fewer than k scanned rows' bounds) every key, N lists of one
    merge_query(cand, N, 1, 0, 1, k, 0, dst, mbuf, red, mcnt, false);
  }
  if (tid == 0) {
    __hip_atomic_store(&ctr[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&ctr[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  stamp(6);
  if (flag) publish_host(flag, seq);
}

bool gemv_q8_ok(uint32_t dim, uint32_t k) { return (dim == 768 || dim == 1024) && k >= 1 && k <= 128; }

uint32_t gemv_q8_lists(uint32_t n_rows) { return gemv_grid(n_rows, 4).nwg; }

size_t gemv_q8_scratch_bytes(uint32_t n_rows, uint32_t k) {
  const uint64_t nscan = gemv_q8_lists(n_rows);
  const uint64_t kp = k <= 64 ? 64 : 128;
  const uint64_t nfin = (nscan + kQ8gLists - 1) / kQ8gLists;
  return (size_t)(nscan * kp * 8 + (nscan * kGemvWaves * 4 + 7) / 8 * 8 + nfin * kGemvWaves * k * 8);
}

template <int D, bool BF16, int KPL>
static void gemv_q8_launch(int part, const void* X, const int8_t* X8, const float* meta,
                           const float* glob, uint32_t n_rows, uint32_t row_base,
                           const float* q_raw, int prep, const uint64_t* allow, uint32_t k,
                           uint32_t nscan, uint64_t* ulist, uint32_t* lbest, uint64_t* cand,
                           uint32_t* ctr, uint64_t* dst, uint64_t* flag, uint64_t seq,
                           uint32_t* stats, uint64_t* clk, hipStream_t st) {
  if (part & 1)
    hipLaunchKernelGGL((gemv_q8_scan_kernel<D, KPL>), dim3(nscan), dim3(kGemvThreads), 0, st, X8,
                       n_rows, row_base, q_raw, prep, meta, glob, allow, ulist, lbest);
  if (part & 2)
    hipLaunchKernelGGL((gemv_q8_finish_kernel<D, BF16, KPL>),
                     dim3((nscan + kQ8gLists - 1) / kQ8gLists), dim3(kGemvThreads), 0, st, X,
                     n_rows, row_base, q_raw, prep, allow, k, ulist, lbest, nscan, cand, ctr, dst,
                     flag, seq, stats, clk);
}

hipError_t launch_gemv_q8(int part, const void* X, bool bf16, const int8_t* X8, const float* meta,
                          const float* glob, uint32_t dim, uint32_t n_rows, uint32_t row_base,
                          const float* q_raw, bool cosine, const uint64_t* allow, uint32_t k,
                          void* scratch, size_t scratch_bytes, uint32_t* ctr, uint64_t* dst,
                          hipStream_t st, uint64_t* flag, uint64_t seq, uint32_t* stats,
                          uint64_t* clk) {
  if (!gemv_q8_ok(dim, k) || n_rows == 0 || !X || !X8 || !meta || !glob || !q_raw || !ctr ||
      !dst || scratch_bytes < gemv_q8_scratch_bytes(n_rows, k))
    return hipErrorInvalidValue;
  const uint32_t nscan = gemv_q8_lists(n_rows);
  if (nscan > (uint32_t)(kQ8gHeld * kGemvThreads)) return hipErrorInvalidValue;  // > 341 CUs
  const uint32_t kp = k <= 64 ? 64 : 128;
  uint64_t* ulist = (uint64_t*)scratch;
  uint32_t* lbest = (uint32_t*)(ulist + (size_t)nscan * kp);
  uint64_t* cand =
      (uint64_t*)((char*)lbest + ((size_t)nscan * kGemvWaves * 4 + 7) / 8 * 8);
  const int prep = (cosine ? 1 : 0) | (bf16 ? 2 : 0);
#define VS_Q8G(DD, BB, KK)                                                                    \
  gemv_q8_launch<DD, BB, KK>(part, X, X8, meta, glob, n_rows, row_base, q_raw, prep, allow, k,  \
                             nscan, ulist, lbest, cand, ctr, dst, flag, seq, stats, clk, st)
  if (dim == 768) {
    if (bf16) { if (kp == 64) VS_Q8G(768, true, 1); else VS_Q8G(768, true, 2); }
    else { if (kp == 64) VS_Q8G(768, false, 1); else VS_Q8G(768, false, 2); }
  } else {
    if (bf16) { if (kp == 64) VS_Q8G(1024, true, 1); else VS_Q8G(1024, true, 2); }
    else { if (kp == 64) VS_Q8G(1024, false, 1); else VS_Q8G(1024, false, 2); }
  }
#undef VS_Q8G
  return hipGetLastError();
}

}  // namespace vsk
