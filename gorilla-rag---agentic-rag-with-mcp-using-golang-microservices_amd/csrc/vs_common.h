// vs_common.h — definitions shared by the HIP kernels and the host engine.
//
// Everything here is bit-exact between host and device: integer hashing,
// bf16 round-to-nearest-even, and the order-preserving result key. The
// oracle (oracle/vsearch_oracle.c) restates the same definitions
// independently; tests/ check that both agree bit for bit.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define VS_HD __host__ __device__ __forceinline__
#else
#define VS_HD static inline
#endif

namespace vs {

// ---- counter-based synthetic generator -----------------------
// splitmix64 finaliser (Steele, Lea & Flood 2014).
VS_HD uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
VS_HD uint64_t gen_row_key(uint64_t seed, uint64_t row) {
  return splitmix64(seed ^ (row * 0xD1B54A32D192ED03ull));
}
// Irwin-Hall(4) integer sample in [-131070, 131070]: four 16-bit uniforms
// summed and centred. Exact in int32 and in fp32.
VS_HD int32_t gen_int(uint64_t row_key, uint32_t col) {
  uint64_t h = splitmix64(row_key + (uint64_t)col);
  return (int32_t)((h & 0xFFFFu) + ((h >> 16) & 0xFFFFu) + ((h >> 32) & 0xFFFFu) +
                   (h >> 48)) - 131070;
}

// ---- snapshot checksum --------------------------------
// H = sum over the little-endian 64-bit words w_i of a byte range (the last
// one zero-padded) of splitmix64(w_i ^ (i * phi)), mod 2^64: position
// dependent, order-free to sum, so a device reduction and a sequential host
// loop agree bit for bit.
VS_HD uint64_t snap_word(uint64_t w, uint64_t i) {
  return splitmix64(w ^ (i * 0x9E3779B97F4A7C15ull));
}

// ---- bf16 ------------------------------------------------------------------
VS_HD uint16_t f32_to_bf16(float f) {
  uint32_t u = __builtin_bit_cast(uint32_t, f);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu))  // NaN stays NaN
    return (uint16_t)((u >> 16) | 0x0040u);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
VS_HD float bf16_to_f32(uint16_t h) {
  return __builtin_bit_cast(float, (uint32_t)h << 16);
}

// ---- result keys (include/vsearch.h "Result key layout") --------------------
VS_HD uint32_t score_ord(float s) {
  uint32_t u = __builtin_bit_cast(uint32_t, s);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
VS_HD float ord_score(uint32_t o) {
  uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
  return __builtin_bit_cast(float, u);
}
VS_HD uint64_t make_key(float s, uint32_t row) {
  if (s == 0.0f) s = 0.0f;  // -0.0 ranks as +0.0
  return ((uint64_t)score_ord(s) << 32) | (uint32_t)(0xFFFFFFFFu - row);
}
VS_HD float key_score(uint64_t k) { return ord_score((uint32_t)(k >> 32)); }
VS_HD uint32_t key_row(uint64_t k) { return 0xFFFFFFFFu - (uint32_t)k; }

// Cosine preprocess skip rule (upstream Qdrant is_length_zero_or_normalized):
// squared length below FLT_EPSILON, or within 1e-6 of 1 -> leave unchanged.
VS_HD bool cosine_keep(double sq) {
  const double eps = 1.1920928955078125e-07;  // FLT_EPSILON
  double d = sq - 1.0;
  if (d < 0) d = -d;
  return sq < eps || d <= 1.0e-6;
}

}  // namespace vs
