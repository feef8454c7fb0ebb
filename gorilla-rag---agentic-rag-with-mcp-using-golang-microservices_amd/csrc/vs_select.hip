// vs_select.hip — large-k selection (k > kMaxK) for gfx950.
//
// Qdrant answers any `limit` (rag/vector-service/main.go:252 passes
// uint64(req.TopK) through), so the engine has a path past the register
// lists of the scans (kMaxK keys). For one query over n rows:
//
//   launch_gemv_scores  (vs_kernels.hip) every row's score image o(r) = the
//                       result key's high word (order-preserving, 0 = masked)
//                       -> sc[n], and the counts of its top 11 bits;
//   launch_rsel         the k-th largest 64-bit key K = o << 32 | ~(row_base
//                       + r) by radix select on the device: six digits (11,
//                       11, 10 bits of o, then 11, 11, 10 of the row word),
//                       each a histogram pass over sc (only keys inside the
//                       bucket chosen so far count) and a one-workgroup pick.
//                       Keys are distinct, so exactly k are >= K. A digit
//                       whose bucket holds exactly the keys still needed ends
//                       the search: the later passes return at once (the row
//                       word is only walked when scores tie at K's high word);
//                       then every key >= K is appended to `sel`;
//   launch_sort_keys_desc the k keys, descending (rocPRIM radix sort).
//
// sc is 4 bytes per row against the 2-4 KB row the score pass reads, so the
// path costs one HBM scan of the collection plus ~3 passes over sc.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "vs_kernels.h"

namespace vsk {

namespace {

constexpr int kHistThreads = 256;
constexpr int kPickThreads = 256;

// digit p: (shift, bits) of the 64-bit key
__host__ __device__ constexpr int digit_shift(int p) {
  return p == 0 ? 53 : p == 1 ? 42 : p == 2 ? 32 : p == 3 ? 21 : p == 4 ? 10 : 0;
}
__host__ __device__ constexpr int digit_bits(int p) { return (p == 2 || p == 5) ? 10 : 11; }

__device__ __forceinline__ uint64_t key_of(uint32_t o, uint32_t row_base, uint32_t r) {
  return ((uint64_t)o << 32) | (uint32_t)(0xFFFFFFFFu - (row_base + r));
}

// Counts digit p of the keys inside the bucket fixed so far (digits < p).
__global__ __launch_bounds__(kHistThreads) void rsel_hist_kernel(
    const uint32_t* __restrict__ sc, uint32_t n, uint32_t row_base,
    const RselState* __restrict__ st, int p, uint32_t* __restrict__ hist) {
  if (st->done) return;  // wave-uniform: every thread reads the same word
  __shared__ uint32_t lh[kRselBins];
  const int shift = digit_shift(p), bits = digit_bits(p);
  const uint32_t mask = (1u << bits) - 1;
  for (int i = threadIdx.x; i < (1 << bits); i += kHistThreads) lh[i] = 0;
  __syncthreads();
  const uint32_t plen = st->plen;
  const uint64_t pre = st->prefix >> (64 - plen);
  const uint32_t stride = gridDim.x * kHistThreads * 4;
  for (uint32_t b = (blockIdx.x * kHistThreads + threadIdx.x) * 4; b < n; b += stride) {
    uint32_t o[4];
    if (b + 4 <= n) {
      const uint4 v = *(const uint4*)(sc + b);  // sc is 16-B aligned (a device allocation)
      o[0] = v.x, o[1] = v.y, o[2] = v.z, o[3] = v.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = b + j < n ? sc[b + j] : 0u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!o[j]) continue;
      const uint64_t key = key_of(o[j], row_base, b + j);
      if ((key >> (64 - plen)) == pre) atomicAdd(&lh[(uint32_t)(key >> shift) & mask], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < (1 << bits); i += kHistThreads)
    if (lh[i]) atomicAdd(&hist[i], lh[i]);
}

// One workgroup: picks digit p's bucket holding the krem-th largest key of
// the current bucket, updates the state, and zeroes the histogram for the
// next pass. Pass 0 also initialises the state (krem = keff).
__global__ __launch_bounds__(kPickThreads) void rsel_pick_kernel(uint32_t* __restrict__ hist,
                                                                RselState* __restrict__ st,
                                                                int p, uint32_t keff) {
  __shared__ uint32_t h[kRselBins];
  __shared__ uint32_t tot[kPickThreads];
  __shared__ uint32_t pick_bin, pick_above;
  const int t = threadIdx.x;
  const int bits = digit_bits(p), nb = 1 << bits, per = nb / kPickThreads;
  if (p == 0 && t == 0) {
    st->prefix = 0;
    st->thr = 0;
    st->plen = 0;
    st->krem = keff;
    st->done = 0;
    st->count = 0;
  }
  __syncthreads();
  const bool done = p > 0 && st->done;  // uniform
  if (done) return;
  uint32_t mine = 0;
  for (int i = 0; i < per; ++i) {
    const uint32_t v = hist[t * per + i];
    h[t * per + i] = v;
    mine += v;
  }
  tot[t] = mine;
  __syncthreads();
  const uint32_t krem = p == 0 ? keff : st->krem;
  if (t == 0) {
    // walk the per-thread totals from the top bucket down to the one that
    // crosses krem, then that thread's buckets
    uint32_t above = 0;
    int tt = kPickThreads - 1;
    for (; tt > 0 && above + tot[tt] < krem; --tt) above += tot[tt];
    int b = tt * per + per - 1;
    for (; b > tt * per && above + h[b] < krem; --b) above += h[b];
    pick_bin = (uint32_t)b;
    pick_above = above;
  }
  __syncthreads();
  for (int i = 0; i < per; ++i) hist[t * per + i] = 0;  // clean for the next pass / query
  if (t == 0) {
    const int shift = digit_shift(p);
    const uint32_t b = pick_bin;
    const uint32_t need = krem - pick_above;
    const uint64_t prefix = st->prefix | ((uint64_t)b << shift);
    st->prefix = prefix;
    st->plen = 64 - shift;
    st->krem = need;
    if (h[b] == need || shift == 0) {  // the bucket is taken whole: every key >= prefix
      st->thr = prefix;
      st->done = 1;
    }
  }
}

// Appends every key >= thr (exactly keff of them) to sel, one atomic per wave.
__global__ __launch_bounds__(kHistThreads) void rsel_compact_kernel(
    const uint32_t* __restrict__ sc, uint32_t n, uint32_t row_base, RselState* __restrict__ st,
    uint64_t* __restrict__ sel) {
  const uint64_t thr = st->thr;
  const int lane = threadIdx.x & 63;
  const uint32_t stride = gridDim.x * kHistThreads;
  for (uint32_t b = blockIdx.x * kHistThreads; b < n; b += stride) {
    const uint32_t r = b + threadIdx.x;
    const uint32_t o = r < n ? sc[r] : 0u;
    const uint64_t key = o ? key_of(o, row_base, r) : 0;
    const bool take = o && key >= thr;
    const uint64_t m = __ballot(take);
    if (!m) continue;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&st->count, (uint32_t)__popcll(m));
    base = __shfl(base, 0, 64);
    if (take) sel[base + __popcll(m & ((1ull << lane) - 1))] = key;
  }
}

// ---- three-launch selection (r03) ---------------------------------------------
// Two grid passes over sc and one workgroup after the score pass, instead of
// 12 launches:
//  f1: every workgroup picks the first digit's bucket b0 from the score
//      pass's histogram (the same walk everywhere), appends every key above
//      b0 (exactly `above0` of them) to sel, and counts the second digit
//      (key bits 52..42) of the keys in b0 into hist1;
//  f2: every workgroup picks b1 from hist1 the same way, appends the keys of
//      b0 whose second digit is above b1 to sel, and the keys of (b0, b1) to
//      cand;
//  f3: one workgroup selects the keys still needed from cand -- all of them,
//      or by radix passes over the rest of the key (in LDS up to 4096 keys)
//      -- and leaves hist, hist1 and the counters zeroed.
// Keys are distinct, so the counts are exact at every step.
constexpr int kFusedThreads = 256;
constexpr int kFusedSortCap = 4096;

// thread 0: the bucket of h[0, nb) (descending) holding the krem-th largest
// key and the keys in the buckets above it; tot = per-thread sums of nb /
// kFusedThreads consecutive buckets.
__device__ void fused_pick(const uint32_t* h, const uint32_t* tot, int nb, uint32_t krem,
                           uint32_t* bin, uint32_t* above) {
  const int per = nb / kFusedThreads;
  uint32_t a = 0;
  int tt = kFusedThreads - 1;
  for (; tt > 0 && a + tot[tt] < krem; --tt) a += tot[tt];
  int b = tt * per + per - 1;
  for (; b > tt * per && a + h[b] < krem; --b) a += h[b];
  *bin = (uint32_t)b;
  *above = a;
}

// the whole workgroup: h <- g[0, 2048), then thread 0 picks; returns the
// bucket, *above the keys above it, *cnt its keys
__device__ uint32_t load_pick(const uint32_t* __restrict__ g, uint32_t krem, uint32_t* h,
                              uint32_t* tot, uint32_t* s_bin, uint32_t* s_above,
                              uint32_t* above, uint32_t* cnt) {
  constexpr int per = kRselBins / kFusedThreads;
  const int t = threadIdx.x;
  uint32_t mine = 0;
  for (int i = 0; i < per; ++i) {
    const uint32_t v = g[t * per + i];
    h[t * per + i] = v;
    mine += v;
  }
  tot[t] = mine;
  __syncthreads();
  if (t == 0) fused_pick(h, tot, kRselBins, krem, s_bin, s_above);
  __syncthreads();
  *above = *s_above;
  *cnt = h[*s_bin];
  return *s_bin;
}

__device__ __forceinline__ uint64_t sc_key(uint32_t o, uint32_t row_base, uint32_t r) {
  return ((uint64_t)o << 32) | (uint32_t)(0xFFFFFFFFu - (row_base + r));
}

// sc[b, b + 4) (0 past n): one 16-B load when whole (sc is a device
// allocation, 16-B aligned, and b is a multiple of 4)
__device__ __forceinline__ void load4(const uint32_t* __restrict__ sc, uint32_t n, uint32_t b,
                                      uint32_t* o) {
  if (b + 4 <= n) {
    const uint4 v = *(const uint4*)(sc + b);
    o[0] = v.x, o[1] = v.y, o[2] = v.z, o[3] = v.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = b + j < n ? sc[b + j] : 0u;
  }
}

// the lanes' take[0..3] keys appended at *cursor with ONE atomic per wave for
// all four (an append's atomic is a round trip the stores wait on)
__device__ __forceinline__ void wave_append4(const bool* take, const uint64_t* key,
                                             uint32_t* cursor, uint64_t* dst) {
  const int lane = threadIdx.x & 63;
  uint64_t m[4];
  uint32_t off[4], total = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    m[j] = __ballot(take[j]);
    off[j] = total;
    total += (uint32_t)__popcll(m[j]);
  }
  if (!total) return;
  uint32_t base = 0;
  if (lane == 0) base = atomicAdd(cursor, total);
  base = __shfl(base, 0, 64);
  const uint64_t below = (1ull << lane) - 1;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (take[j]) dst[base + off[j] + (uint32_t)__popcll(m[j] & below)] = key[j];
}

// appends the lanes' `take` keys at *cursor (one atomic per wave)
__device__ __forceinline__ void wave_append(bool take, uint64_t key, uint32_t* cursor,
                                            uint64_t* dst) {
  const int lane = threadIdx.x & 63;
  const uint64_t m = __ballot(take);
  if (!m) return;
  uint32_t base = 0;
  if (lane == 0) base = atomicAdd(cursor, (uint32_t)__popcll(m));
  base = __shfl(base, 0, 64);
  if (take) dst[base + __popcll(m & ((1ull << lane) - 1))] = key;
}

__global__ __launch_bounds__(kFusedThreads) void rsel_f1_kernel(
    const uint32_t* __restrict__ sc, uint32_t n, uint32_t row_base, uint32_t keff,
    const uint32_t* __restrict__ hist, uint32_t* __restrict__ hist1, uint32_t* __restrict__ ctr,
    uint64_t* __restrict__ sel) {
  __shared__ uint32_t h[kRselBins];
  __shared__ uint32_t tot[kFusedThreads];
  __shared__ uint32_t s_bin, s_above;
  uint32_t above0, h0;
  const uint32_t b0 = load_pick(hist, keff, h, tot, &s_bin, &s_above, &above0, &h0);
  (void)above0;
  (void)h0;
  for (int i = threadIdx.x; i < kRselBins; i += kFusedThreads) h[i] = 0;  // -> 2nd digit
  __syncthreads();
  const uint32_t stride = gridDim.x * kFusedThreads * 4;
  for (uint32_t b4 = (blockIdx.x * kFusedThreads + threadIdx.x) * 4; b4 - threadIdx.x * 4 < n;
       b4 += stride) {
    uint32_t o4[4];
    load4(sc, n, b4, o4);
    bool tk[4];
    uint64_t ky[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t o = o4[j], r = b4 + (uint32_t)j;
      const uint32_t bin = o >> (32 - kRselBits0);
      ky[j] = sc_key(o, row_base, r);
      tk[j] = o && bin > b0;
      if (o && bin == b0) atomicAdd(&h[(uint32_t)(ky[j] >> 42) & (kRselBins - 1)], 1u);
    }
    wave_append4(tk, ky, &ctr[0], sel);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kRselBins; i += kFusedThreads)
    if (h[i]) atomicAdd(&hist1[i], h[i]);
}

__global__ __launch_bounds__(kFusedThreads) void rsel_f2_kernel(
    const uint32_t* __restrict__ sc, uint32_t n, uint32_t row_base, uint32_t keff,
    const uint32_t* __restrict__ hist, const uint32_t* __restrict__ hist1,
    uint32_t* __restrict__ ctr, uint64_t* __restrict__ sel, uint64_t* __restrict__ cand) {
  __shared__ uint32_t h[kRselBins];
  __shared__ uint32_t tot[kFusedThreads];
  __shared__ uint32_t s_bin, s_above;
  const int t = threadIdx.x;
  uint32_t above0, h0, above1, h1;
  const uint32_t b0 = load_pick(hist, keff, h, tot, &s_bin, &s_above, &above0, &h0);
  __syncthreads();
  const uint32_t b1 = load_pick(hist1, keff - above0, h, tot, &s_bin, &s_above, &above1, &h1);
  (void)h0;
  (void)h1;
  const uint32_t stride = gridDim.x * kFusedThreads * 4;
  for (uint32_t b4 = (blockIdx.x * kFusedThreads + (uint32_t)t) * 4; b4 - (uint32_t)t * 4 < n;
       b4 += stride) {
    uint32_t o4[4];
    load4(sc, n, b4, o4);
    bool tk[4], tc[4];
    uint64_t ky[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t o = o4[j], r = b4 + (uint32_t)j;
      ky[j] = sc_key(o, row_base, r);
      const bool in0 = o && (o >> (32 - kRselBits0)) == b0;
      const uint32_t d1 = (uint32_t)(ky[j] >> 42) & (kRselBins - 1);
      tk[j] = in0 && d1 > b1;
      tc[j] = in0 && d1 == b1;
    }
    wave_append4(tk, ky, &ctr[0], sel);
    wave_append4(tc, ky, &ctr[1], cand);
  }
}

// One workgroup: the keys still needed, from cand[0, h1) -> sel[above0 +
// above1, keff); then hist, hist1 and the counters are zeroed for the next
// query. (As the last workgroup of rsel_f2 this needed an agent-scope release
// in every workgroup -- an L2 write-back each, 1024 of them at 10M rows, and
// f2 took 63 us; a launch boundary orders it for free.)
__global__ __launch_bounds__(kFusedThreads) void rsel_f3_kernel(
    uint32_t keff, uint32_t* __restrict__ hist, uint32_t* __restrict__ hist1,
    uint32_t* __restrict__ ctr, uint64_t* __restrict__ sel, const uint64_t* __restrict__ cand) {
  __shared__ uint32_t h[kRselBins];
  __shared__ uint32_t tot[kFusedThreads];
  __shared__ uint32_t s_bin, s_above, s_done;
  __shared__ unsigned long long s_prefix;
  __shared__ uint64_t sk[kFusedSortCap];
  const int t = threadIdx.x;
  uint32_t above0, h0, above1, h1;
  const uint32_t b0 = load_pick(hist, keff, h, tot, &s_bin, &s_above, &above0, &h0);
  __syncthreads();
  const uint32_t krem1 = keff - above0;
  const uint32_t b1 = load_pick(hist1, krem1, h, tot, &s_bin, &s_above, &above1, &h1);
  (void)h0;
  __syncthreads();
  const uint32_t need = krem1 - above1;
  uint64_t* dst = sel + above0 + above1;
  if (need == h1) {
    for (uint32_t i = t; i < h1; i += kFusedThreads) dst[i] = cand[i];
  } else {
    // radix passes over the rest of the key (11, 11, 10, 10 bits) -- over an
    // LDS copy when cand fits 4096 keys (a bitonic sort of 4096 was slower:
    // 78 barrier stages), else over cand in global memory (ties, huge k)
    const uint64_t* src = cand;
    if (h1 <= (uint32_t)kFusedSortCap) {
      for (uint32_t i = t; i < h1; i += kFusedThreads) sk[i] = cand[i];
      src = sk;
    }
    if (t == 0) {
      s_prefix = ((unsigned long long)b0 << 53) | ((unsigned long long)b1 << 42);
      s_done = 0;
    }
    uint32_t krem = need;
    for (int p = 0; p < 4; ++p) {
      const int shift = p == 0 ? 31 : p == 1 ? 20 : p == 2 ? 10 : 0;
      const int bits = p <= 1 ? 11 : 10, nb = 1 << bits;
      __syncthreads();
      if (s_done) break;
      for (int i = t; i < kRselBins; i += kFusedThreads) h[i] = 0;
      __syncthreads();
      const uint64_t pre = s_prefix >> (shift + bits);
      for (uint32_t i0 = t; i0 < h1; i0 += 4 * kFusedThreads) {
        uint64_t kk[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t i = i0 + (uint32_t)u * kFusedThreads;
          kk[u] = i < h1 ? src[i] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (i0 + (uint32_t)u * kFusedThreads < h1 && (kk[u] >> (shift + bits)) == pre)
            atomicAdd(&h[(uint32_t)(kk[u] >> shift) & (uint32_t)(nb - 1)], 1u);
      }
      __syncthreads();
      const int per = nb / kFusedThreads;
      uint32_t m = 0;
      for (int i = 0; i < per; ++i) m += h[t * per + i];
      tot[t] = m;
      __syncthreads();
      if (t == 0) {
        uint32_t b, a;
        fused_pick(h, tot, nb, krem, &b, &a);
        s_prefix |= (unsigned long long)b << shift;
        s_above = a;
        if (h[b] == krem - a || shift == 0) s_done = 1;  // the bucket is taken whole
      }
      __syncthreads();
      krem -= s_above;
    }
    __syncthreads();
    const uint64_t thr = s_prefix;  // exactly `need` keys of cand are >= thr
    if (t == 0) s_above = 0;
    __syncthreads();
    for (uint32_t base = 0; base < h1; base += kFusedThreads) {
      const uint32_t i = base + (uint32_t)t;
      const uint64_t key = i < h1 ? src[i] : 0ull;
      wave_append(i < h1 && key >= thr, key, &s_above, dst);
    }
  }
  // clean for the next query
  for (int i = t; i < kRselBins; i += kFusedThreads) {
    hist[i] = 0;
    hist1[i] = 0;
  }
  if (t == 0) {
    ctr[0] = 0;
    ctr[1] = 0;
    ctr[2] = 0;
  }
}

uint32_t grid_for(uint32_t n, int threads, int per_thread) {
  const int cus = device_cu_count();
  const uint64_t want = ((uint64_t)n + (uint64_t)threads * per_thread - 1) /
                        ((uint64_t)threads * per_thread);
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)cus * 4));
}

}  // namespace

hipError_t launch_rsel(const uint32_t* sc, uint32_t n_rows, uint32_t row_base, uint32_t keff,
                       uint32_t* hist, RselState* state, uint64_t* sel, hipStream_t st) {
  if (n_rows == 0 || keff == 0 || keff > n_rows) return hipErrorInvalidValue;
  const uint32_t gh = grid_for(n_rows, kHistThreads, 4);
  hipLaunchKernelGGL(rsel_pick_kernel, dim3(1), dim3(kPickThreads), 0, st, hist, state, 0, keff);
  for (int p = 1; p < 6; ++p) {
    hipLaunchKernelGGL(rsel_hist_kernel, dim3(gh), dim3(kHistThreads), 0, st, sc, n_rows, row_base,
                       state, p, hist);
    hipLaunchKernelGGL(rsel_pick_kernel, dim3(1), dim3(kPickThreads), 0, st, hist, state, p, keff);
  }
  hipLaunchKernelGGL(rsel_compact_kernel, dim3(grid_for(n_rows, kHistThreads, 1)),
                     dim3(kHistThreads), 0, st, sc, n_rows, row_base, state, sel);
  return hipGetLastError();
}

hipError_t launch_rsel_fused(const uint32_t* sc, uint32_t n_rows, uint32_t row_base,
                             uint32_t keff, uint32_t* hist, uint32_t* hist1, uint32_t* ctr,
                             uint64_t* sel, uint64_t* cand, hipStream_t st) {
  if (n_rows == 0 || keff == 0 || keff > n_rows) return hipErrorInvalidValue;
  const dim3 g(grid_for(n_rows, kFusedThreads, 4)), b(kFusedThreads);
  hipLaunchKernelGGL(rsel_f1_kernel, g, b, 0, st, sc, n_rows, row_base, keff, hist, hist1, ctr,
                     sel);
  hipLaunchKernelGGL(rsel_f2_kernel, g, b, 0, st, sc, n_rows, row_base, keff, hist, hist1, ctr,
                     sel, cand);
  hipLaunchKernelGGL(rsel_f3_kernel, dim3(1), b, 0, st, keff, hist, hist1, ctr, sel, cand);
  return hipGetLastError();
}

size_t sort_keys_temp_bytes(uint64_t n) {
  size_t bytes = 0;
  if (rocprim::radix_sort_keys_desc(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                    (size_t)n) != hipSuccess)
    return 0;
  return bytes;
}

hipError_t launch_sort_keys_desc(const uint64_t* in, uint64_t* out, uint64_t n, void* temp,
                                 size_t temp_bytes, hipStream_t st) {
  if (n == 0) return hipSuccess;
  size_t bytes = temp_bytes;
  return rocprim::radix_sort_keys_desc(temp, bytes, in, out, (size_t)n, 0, 64, st);
}

// ---- merge of L lists for any k ---------------------------------------------
namespace {

constexpr int kGatherThreads = 256;
constexpr int kUniqThreads = 256;

// tmp[q][l * kin + j] = lists[l * lstride + q * qstride + j]
__global__ __launch_bounds__(kGatherThreads) void merge_gather_kernel(
    const uint64_t* __restrict__ lists, uint32_t L, uint64_t lstride, uint64_t qstride,
    uint32_t nq, uint32_t kin, uint64_t* __restrict__ tmp, uint32_t* __restrict__ offs) {
  const uint64_t per = (uint64_t)L * kin, total = per * nq;
  for (uint64_t i = (uint64_t)blockIdx.x * kGatherThreads + threadIdx.x; i < total;
       i += (uint64_t)gridDim.x * kGatherThreads) {
    const uint64_t q = i / per, r = i % per, l = r / kin, j = r % kin;
    tmp[i] = lists[l * lstride + q * qstride + j];
  }
  if (blockIdx.x == 0)
    for (uint32_t q = threadIdx.x; q <= nq; q += kGatherThreads) offs[q] = (uint32_t)(q * per);
}

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t off = 0, all = 0;
  for (int i = 0; i < kUniqThreads / 64; ++i) {
    if (i < w) off += wsum[i];
    all += wsum[i];
  }
  __syncthreads();  // wsum is reused by the next call
  *total = all;
  return off + x - v;
}

// One workgroup per query: the sorted segment's distinct non-zero keys, the
// first k of them, 0-padded.
__global__ __launch_bounds__(kUniqThreads) void merge_unique_kernel(
    const uint64_t* __restrict__ sorted, uint64_t per, uint32_t k, uint64_t* __restrict__ out) {
  __shared__ uint32_t wsum[kUniqThreads / 64];
  const uint32_t q = blockIdx.x;
  const uint64_t* seg = sorted + (uint64_t)q * per;
  uint64_t* o = out + (uint64_t)q * k;
  uint32_t base = 0;
  for (uint64_t t0 = 0; t0 < per && base < k; t0 += kUniqThreads) {
    const uint64_t i = t0 + threadIdx.x;
    const uint64_t key = i < per ? seg[i] : 0;
    const bool keep = key != 0 && (i == 0 || seg[i - 1] != key);
    uint32_t total;
    const uint32_t pos = base + block_excl_scan(keep ? 1u : 0u, wsum, &total);
    if (keep && pos < k) o[pos] = key;
    base += total;
    if (total == 0) break;  // zeros sort last: the rest is empty
  }
  for (uint32_t j = base + threadIdx.x; j < k; j += kUniqThreads) o[j] = 0;
}

struct MergeScratch {
  uint64_t* tmp;
  uint64_t* sorted;
  uint32_t* offs;
  void* temp;
  size_t temp_bytes;
};

size_t seg_sort_temp(uint64_t total, uint32_t nq) {
  size_t bytes = 0;
  if (rocprim::segmented_radix_sort_keys_desc(nullptr, bytes, (uint64_t*)nullptr,
                                              (uint64_t*)nullptr, (unsigned int)total, nq,
                                              (uint32_t*)nullptr, (uint32_t*)nullptr) != hipSuccess)
    return 0;
  return bytes;
}

size_t align256(size_t x) { return (x + 255) / 256 * 256; }

MergeScratch carve(void* base, uint32_t L, uint32_t nq, uint32_t kin) {
  const uint64_t total = (uint64_t)L * kin * nq;
  char* p = (char*)base;
  MergeScratch m;
  m.tmp = (uint64_t*)p;
  p += align256(total * 8);
  m.sorted = (uint64_t*)p;
  p += align256(total * 8);
  m.offs = (uint32_t*)p;
  p += align256((size_t)(nq + 1) * 4);
  m.temp = p;
  m.temp_bytes = seg_sort_temp(total, nq);
  return m;
}

}  // namespace

size_t merge_large_scratch(uint32_t L, uint32_t nq, uint32_t kin) {
  const uint64_t total = (uint64_t)L * kin * nq;
  return align256(total * 8) * 2 + align256((size_t)(nq + 1) * 4) + align256(seg_sort_temp(total, nq));
}

hipError_t launch_merge_large(const uint64_t* lists, uint32_t L, uint64_t lstride,
                              uint64_t qstride, uint32_t nq, uint32_t kin, uint32_t k,
                              uint64_t* out, void* scratch, size_t scratch_bytes, hipStream_t st) {
  if (L == 0 || nq == 0 || kin == 0 || k == 0) return hipErrorInvalidValue;
  const uint64_t per = (uint64_t)L * kin, total = per * nq;
  if (total >= 0xFFFFFFFFull || scratch_bytes < merge_large_scratch(L, nq, kin))
    return hipErrorInvalidValue;
  MergeScratch m = carve(scratch, L, nq, kin);
  hipLaunchKernelGGL(merge_gather_kernel,
                     dim3((uint32_t)std::min<uint64_t>((total + kGatherThreads - 1) / kGatherThreads,
                                                       4096)),
                     dim3(kGatherThreads), 0, st, lists, L, lstride, qstride, nq, kin, m.tmp, m.offs);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t tb = m.temp_bytes;
  e = rocprim::segmented_radix_sort_keys_desc(m.temp, tb, m.tmp, m.sorted, (unsigned int)total, nq,
                                              m.offs, m.offs + 1, 0, 64, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(merge_unique_kernel, dim3(nq), dim3(kUniqThreads), 0, st, m.sorted, per, k, out);
  return hipGetLastError();
}

}  // namespace vsk
