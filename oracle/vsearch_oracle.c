/*
 * vsearch_oracle.c — CPU restatement of the reference search path.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product links, loads or calls this
 * file; it is used by tests/, __graft_entry__.smoke() (as the checker) and by
 * bench.py's cpu_baseline leg (timed beside the GPU, never as the product).
 *
 * What it restates (reference: ThiruEigen7/GoRilla-Rag, snapshot 2026-02-20):
 *  - rag/vector-service/main.go:249-254: Points.Search with Limit = top_k,
 *    WithPayload, no filter / offset / score_threshold / exact flag, against
 *    collections created with Distance_Cosine and the default f32 datatype
 *    (main.go:102-112). The arithmetic runs inside the un-vendored Qdrant
 *    server (docker-compose.yml:5, image qdrant/qdrant:latest, UNPINNED; wire
 *    API pinned by github.com/qdrant/go-client v1.7.0, go.mod:6). Restated
 *    from Qdrant's published exact-search algorithm:
 *      lib/segment/src/spaces/simple.rs  CosineMetric::preprocess: squared
 *        length; unchanged if < f32::EPSILON or |len2 - 1| <= 1e-6; else
 *        x / sqrt(len2).
 *      similarity = dot product of the preprocessed vectors (Cosine and Dot).
 *      top-`limit` by score descending (fixed-length priority queue).
 *    Tie order is unspecified upstream; here: score desc, then row asc.
 *  - This restatement accumulates the squared norm in fp64 in a fixed order
 *    (lane-strided partial sums over 64 lanes, then an xor butterfly) so it is
 *    bit-exact against the device preprocess; the oracle's search scores are
 *    computed in fp64 from the stored fp32 values and rounded once.
 *
 * Parity pinning: the reference repository holds no tests, fixtures or stored
 * embeddings for this path — "parity unpinned" by
 * reference data. The oracle is pinned instead by analytic known-answer tests
 * (tests/test_oracle.py) and by agreement with an independent numpy
 * restatement (oracle/oracle.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* ---- counter-based generator ---- */
static uint64_t o_splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
static int32_t o_gen_int(uint64_t seed, uint64_t row, uint32_t col) {
  uint64_t rk = o_splitmix64(seed ^ (row * 0xD1B54A32D192ED03ull));
  uint64_t h = o_splitmix64(rk + (uint64_t)col);
  return (int32_t)((h & 0xFFFFu) + ((h >> 16) & 0xFFFFu) + ((h >> 32) & 0xFFFFu) + (h >> 48)) -
         131070;
}

uint16_t oracle_f32_to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static float o_bf16_round(float f) {
  uint32_t u = (uint32_t)oracle_f32_to_bf16(f) << 16;
  float r;
  memcpy(&r, &u, 4);
  return r;
}

/* n rows (global numbers grow0 ..) of unit vectors; bf16 != 0 -> values
 * rounded to bf16 (returned widened to f32). */
void oracle_generate(uint64_t seed, uint64_t grow0, uint64_t n, uint32_t dim, int bf16,
                     float* out) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    int64_t s = 0;
    for (uint32_t d = 0; d < dim; ++d) {
      int64_t m = o_gen_int(seed, grow0 + (uint64_t)i, d);
      s += m * m;
    }
    double nrm = sqrt((double)s);
    float* o = out + (size_t)i * dim;
    for (uint32_t d = 0; d < dim; ++d) {
      int32_t m = o_gen_int(seed, grow0 + (uint64_t)i, d);
      float y = s > 0 ? (float)((double)m / nrm) : 0.0f;
      o[d] = bf16 ? o_bf16_round(y) : y;
    }
  }
}

/* Same rows, raw storage: bf16 bit patterns (bf16 != 0) or fp32. */
void oracle_generate_raw(uint64_t seed, uint64_t grow0, uint64_t n, uint32_t dim, int bf16,
                         void* out) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    int64_t s = 0;
    for (uint32_t d = 0; d < dim; ++d) {
      int64_t m = o_gen_int(seed, grow0 + (uint64_t)i, d);
      s += m * m;
    }
    double nrm = sqrt((double)s);
    for (uint32_t d = 0; d < dim; ++d) {
      int32_t m = o_gen_int(seed, grow0 + (uint64_t)i, d);
      float y = s > 0 ? (float)((double)m / nrm) : 0.0f;
      if (bf16)
        ((uint16_t*)out)[(size_t)i * dim + d] = oracle_f32_to_bf16(y);
      else
        ((float*)out)[(size_t)i * dim + d] = y;
    }
  }
}

/* Qdrant cosine preprocess with the fixed-order fp64 squared norm. */
static double o_sqnorm(const float* x, uint32_t dim) {
  double lane[64];
  for (int l = 0; l < 64; ++l) {
    double s = 0.0;
    for (uint32_t d = (uint32_t)l; d < dim; d += 64) {
      double v = (double)x[d];
      s = s + v * v;
    }
    lane[l] = s;
  }
  for (int m = 32; m >= 1; m >>= 1) {
    double t[64];
    for (int l = 0; l < 64; ++l) t[l] = lane[l] + lane[l ^ m];
    memcpy(lane, t, sizeof(t));
  }
  return lane[0];
}

void oracle_preprocess(const float* in, uint64_t n, uint32_t dim, int cosine, int bf16,
                       float* out) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    const float* x = in + (size_t)i * dim;
    float* o = out + (size_t)i * dim;
    double s = o_sqnorm(x, dim);
    double d1 = fabs(s - 1.0);
    int keep = !cosine || s < 1.1920928955078125e-07 || d1 <= 1.0e-6;
    double nrm = sqrt(s);
    for (uint32_t d = 0; d < dim; ++d) {
      float y = keep ? x[d] : (float)((double)x[d] / nrm);
      o[d] = bf16 ? o_bf16_round(y) : y;
    }
  }
}

/* ---- exact top-k ---- */
typedef struct {
  double s;
  uint64_t row;
} o_hit;

/* a better than b: score desc, row asc */
static int o_better(const o_hit* a, const o_hit* b) {
  return a->s > b->s || (a->s == b->s && a->row < b->row);
}

/* insert into a sorted (best first) array of size *n <= k */
static void o_push(o_hit* h, uint32_t* n, uint32_t k, o_hit x) {
  if (*n == k && !o_better(&x, &h[k - 1])) return;
  uint32_t j = (*n < k) ? (*n)++ : k - 1;
  while (j > 0 && o_better(&x, &h[j - 1])) {
    h[j] = h[j - 1];
    --j;
  }
  h[j] = x;
}

/* X: n x dim stored (already preprocessed) values; Q: nq x dim preprocessed
 * queries. Scores are fp64 dot products; out_scores gets them rounded to f32.
 * out_scores64 (optional) gets the fp64 values. */
void oracle_search(const float* X, uint64_t n, uint32_t dim, const float* Q, uint32_t nq,
                   uint32_t k, uint64_t row_base, float* out_scores, double* out_scores64,
                   uint64_t* out_rows, uint32_t* out_count) {
  int nth = 1;
#ifdef _OPENMP
  nth = omp_get_max_threads();
#endif
  o_hit* heaps = (o_hit*)malloc(sizeof(o_hit) * (size_t)nth * k);
  uint32_t* cnts = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)nth);
  for (uint32_t qi = 0; qi < nq; ++qi) {
    const float* q = Q + (size_t)qi * dim;
    memset(cnts, 0, sizeof(uint32_t) * (size_t)nth);
#pragma omp parallel
    {
      int t = 0;
#ifdef _OPENMP
      t = omp_get_thread_num();
#endif
      o_hit* h = heaps + (size_t)t * k;
#pragma omp for schedule(static)
      for (int64_t r = 0; r < (int64_t)n; ++r) {
        const float* x = X + (size_t)r * dim;
        double s = 0.0;
        for (uint32_t d = 0; d < dim; ++d) s += (double)x[d] * (double)q[d];
        o_hit hit = {s, row_base + (uint64_t)r};
        o_push(h, &cnts[t], k, hit);
      }
    }
    o_hit* best = (o_hit*)malloc(sizeof(o_hit) * k);
    uint32_t nb = 0;
    for (int t = 0; t < nth; ++t)
      for (uint32_t j = 0; j < cnts[t]; ++j) o_push(best, &nb, k, heaps[(size_t)t * k + j]);
    for (uint32_t j = 0; j < k; ++j) {
      size_t o = (size_t)qi * k + j;
      if (j < nb) {
        if (out_scores) out_scores[o] = (float)best[j].s;
        if (out_scores64) out_scores64[o] = best[j].s;
        if (out_rows) out_rows[o] = best[j].row;
      } else {
        if (out_scores) out_scores[o] = 0.f;
        if (out_scores64) out_scores64[o] = 0.0;
        if (out_rows) out_rows[o] = 0;
      }
    }
    if (out_count) out_count[qi] = nb;
    free(best);
  }
  free(heaps);
  free(cnts);
}

/* Exact fp64 scores of given (query, row) pairs — used to re-score the rows a
 * device returned. X is indexed by local row (row - row_base). */
void oracle_rescore(const float* X, uint32_t dim, const float* Q, uint32_t nq, uint32_t k,
                    const uint64_t* rows, const uint32_t* count, uint64_t row_base,
                    double* out) {
  for (uint32_t qi = 0; qi < nq; ++qi)
    for (uint32_t j = 0; j < k; ++j) {
      size_t o = (size_t)qi * k + j;
      if (j >= count[qi]) {
        out[o] = 0.0;
        continue;
      }
      const float* x = X + (size_t)(rows[o] - row_base) * dim;
      const float* q = Q + (size_t)qi * dim;
      double s = 0.0;
      for (uint32_t d = 0; d < dim; ++d) s += (double)x[d] * (double)q[d];
      out[o] = s;
    }
}

/* ---- streaming oracle over a generated corpus ----
 * Exact top-k of preprocessed queries Q (nq x dim, fp32) against the rows a
 * collection filled by vs_generate holds: global rows grow0 .. grow0+n-1 of
 * `seed`, bf16-rounded when bf16 != 0. Rows are regenerated
 * block by block inside each thread, so no n x dim host array exists: this is
 * what lets the tests check C3 (10M rows) and C4 (100M rows) at their full
 * size. Scores are fp64 dot products of the stored values (same rule as
 * oracle_search); ties by row ascending. Each row's score is computed by one
 * thread in a fixed order, so the result does not depend on the thread count. */
static void o_gen_row(uint64_t seed, uint64_t row, uint32_t dim, int bf16, int32_t* m,
                      double* out) {
  const uint64_t rk = o_splitmix64(seed ^ (row * 0xD1B54A32D192ED03ull));
  int64_t s = 0;
  for (uint32_t d = 0; d < dim; ++d) {
    const uint64_t h = o_splitmix64(rk + (uint64_t)d);
    m[d] = (int32_t)((h & 0xFFFFu) + ((h >> 16) & 0xFFFFu) + ((h >> 32) & 0xFFFFu) + (h >> 48)) -
           131070;
    s += (int64_t)m[d] * m[d];
  }
  const double nrm = sqrt((double)s);
  for (uint32_t d = 0; d < dim; ++d) {
    float y = s > 0 ? (float)((double)m[d] / nrm) : 0.0f;
    if (bf16) y = o_bf16_round(y);
    out[d] = (double)y;
  }
}

static double o_dot64(const double* x, const double* q, uint32_t dim) {
  double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  uint32_t d = 0;
  for (; d + 4 <= dim; d += 4) {
    a0 += x[d] * q[d];
    a1 += x[d + 1] * q[d + 1];
    a2 += x[d + 2] * q[d + 2];
    a3 += x[d + 3] * q[d + 3];
  }
  for (; d < dim; ++d) a0 += x[d] * q[d];
  return (a0 + a1) + (a2 + a3);
}

void oracle_search_generated(uint64_t seed, uint64_t grow0, uint64_t n, uint32_t dim, int bf16,
                             const float* Q, uint32_t nq, uint32_t k, int threads,
                             double* out_scores64, uint64_t* out_rows, uint32_t* out_count) {
  int nth = threads > 0 ? threads : 1;
#ifdef _OPENMP
  if (threads <= 0) nth = omp_get_max_threads();
#else
  nth = 1;
#endif
  double* q64 = (double*)malloc(sizeof(double) * (size_t)nq * dim);
  for (size_t i = 0; i < (size_t)nq * dim; ++i) q64[i] = (double)Q[i];
  o_hit* heaps = (o_hit*)malloc(sizeof(o_hit) * (size_t)nth * nq * k);
  uint32_t* cnts = (uint32_t*)calloc((size_t)nth * nq, sizeof(uint32_t));
#pragma omp parallel num_threads(nth)
  {
    int t = 0;
#ifdef _OPENMP
    t = omp_get_thread_num();
#endif
    int32_t* m = (int32_t*)malloc(sizeof(int32_t) * dim);
    double* x = (double*)malloc(sizeof(double) * dim);
    o_hit* h = heaps + (size_t)t * nq * k;
    uint32_t* c = cnts + (size_t)t * nq;
#pragma omp for schedule(dynamic, 4096)
    for (int64_t r = 0; r < (int64_t)n; ++r) {
      const uint64_t row = grow0 + (uint64_t)r;
      o_gen_row(seed, row, dim, bf16, m, x);
      for (uint32_t qi = 0; qi < nq; ++qi) {
        const double sc = o_dot64(x, q64 + (size_t)qi * dim, dim);
        o_hit* hq = h + (size_t)qi * k;
        if (c[qi] == k && !(sc > hq[k - 1].s || (sc == hq[k - 1].s && row < hq[k - 1].row)))
          continue;
        o_hit hit = {sc, row};
        o_push(hq, &c[qi], k, hit);
      }
    }
    free(m);
    free(x);
  }
  o_hit* best = (o_hit*)malloc(sizeof(o_hit) * k);
  for (uint32_t qi = 0; qi < nq; ++qi) {
    uint32_t nb = 0;
    for (int t = 0; t < nth; ++t)
      for (uint32_t j = 0; j < cnts[(size_t)t * nq + qi]; ++j)
        o_push(best, &nb, k, heaps[((size_t)t * nq + qi) * k + j]);
    for (uint32_t j = 0; j < k; ++j) {
      const size_t o = (size_t)qi * k + j;
      if (out_scores64) out_scores64[o] = j < nb ? best[j].s : 0.0;
      if (out_rows) out_rows[o] = j < nb ? best[j].row : 0;
    }
    if (out_count) out_count[qi] = nb;
  }
  free(best);
  free(q64);
  free(heaps);
  free(cnts);
}

/* Exact fp64 scores of (query, global row) pairs of a generated corpus. */
void oracle_rescore_generated(uint64_t seed, uint32_t dim, int bf16, const float* Q, uint32_t nq,
                              uint32_t k, const uint64_t* rows, const uint32_t* count,
                              double* out) {
#pragma omp parallel
  {
    int32_t* m = (int32_t*)malloc(sizeof(int32_t) * dim);
    double* x = (double*)malloc(sizeof(double) * dim);
    double* q = (double*)malloc(sizeof(double) * dim);
#pragma omp for schedule(static)
    for (int64_t qi = 0; qi < (int64_t)nq; ++qi) {
      for (uint32_t d = 0; d < dim; ++d) q[d] = (double)Q[(size_t)qi * dim + d];
      for (uint32_t j = 0; j < k; ++j) {
        const size_t o = (size_t)qi * k + j;
        if (j >= count[qi]) {
          out[o] = 0.0;
          continue;
        }
        o_gen_row(seed, rows[o], dim, bf16, m, x);
        out[o] = o_dot64(x, q, dim);
      }
    }
    free(m);
    free(x);
    free(q);
  }
}

/* ---- CPU baseline: restatement of Qdrant's plain exact scan ----
 * fp32 dot with O_LANES independent accumulators (one SIMD register's worth
 * of lanes: 8 under AVX2 -- Qdrant's AVX path -- and 16 in the AVX-512
 * build, liboracle_avx512.so), OpenMP over row blocks, per-thread
 * fixed-length top-k, then a merge. Values are read as stored (fp32, or
 * bf16 widened). Returns the number of threads used. */
#ifdef __AVX512F__
#define O_LANES 16
#else
#define O_LANES 8
#endif
static float o_hsum(float* acc) { /* pairwise tree: lanes j and j + w */
  for (int w = O_LANES / 2; w >= 1; w /= 2)
    for (int j = 0; j < w; ++j) acc[j] += acc[j + w];
  return acc[0];
}
static float o_dot_f32(const float* x, const float* q, uint32_t dim) {
  float acc[O_LANES] = {0};
  uint32_t d = 0;
  for (; d + O_LANES <= dim; d += O_LANES)
    for (int j = 0; j < O_LANES; ++j) acc[j] += x[d + j] * q[d + j];
  float s = o_hsum(acc);
  for (; d < dim; ++d) s += x[d] * q[d];
  return s;
}
static float o_dot_bf16(const uint16_t* x, const float* q, uint32_t dim) {
  float acc[O_LANES] = {0};
  uint32_t d = 0;
  for (; d + O_LANES <= dim; d += O_LANES)
    for (int j = 0; j < O_LANES; ++j) {
      uint32_t u = (uint32_t)x[d + j] << 16;
      float v;
      memcpy(&v, &u, 4);
      acc[j] += v * q[d + j];
    }
  float s = o_hsum(acc);
  for (; d < dim; ++d) {
    uint32_t u = (uint32_t)x[d] << 16;
    float v;
    memcpy(&v, &u, 4);
    s += v * q[d];
  }
  return s;
}

/* SIMD width the CPU baseline was built for (8 = AVX2, 16 = AVX-512). */
int oracle_cpu_scan_lanes(void) { return O_LANES; }

int oracle_cpu_scan(const void* X, int bf16, uint64_t n, uint32_t dim, const float* Q,
                    uint32_t nq, uint32_t k, int threads, float* out_scores,
                    uint64_t* out_rows) {
  int nth = threads > 0 ? threads : 1;
#ifdef _OPENMP
  if (threads <= 0) nth = omp_get_max_threads();
#else
  nth = 1;
#endif
  o_hit* heaps = (o_hit*)malloc(sizeof(o_hit) * (size_t)nth * k);
  uint32_t* cnts = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)nth);
  for (uint32_t qi = 0; qi < nq; ++qi) {
    const float* q = Q + (size_t)qi * dim;
    memset(cnts, 0, sizeof(uint32_t) * (size_t)nth);
#pragma omp parallel num_threads(nth)
    {
      int t = 0;
#ifdef _OPENMP
      t = omp_get_thread_num();
#endif
      o_hit* h = heaps + (size_t)t * k;
      uint32_t c = 0;
#pragma omp for schedule(static)
      for (int64_t r = 0; r < (int64_t)n; ++r) {
        float s = bf16 ? o_dot_bf16((const uint16_t*)X + (size_t)r * dim, q, dim)
                       : o_dot_f32((const float*)X + (size_t)r * dim, q, dim);
        if (c == k && !((double)s > h[k - 1].s)) continue;
        o_hit hit = {(double)s, (uint64_t)r};
        o_push(h, &c, k, hit);
      }
      cnts[t] = c;
    }
    o_hit best[1024];
    uint32_t nb = 0, kk = k > 1024 ? 1024 : k;
    for (int t = 0; t < nth; ++t)
      for (uint32_t j = 0; j < cnts[t]; ++j) o_push(best, &nb, kk, heaps[(size_t)t * k + j]);
    for (uint32_t j = 0; j < kk; ++j) {
      if (out_scores) out_scores[(size_t)qi * k + j] = j < nb ? (float)best[j].s : 0.f;
      if (out_rows) out_rows[(size_t)qi * k + j] = j < nb ? best[j].row : 0;
    }
  }
  free(heaps);
  free(cnts);
  return nth;
}

/* ---- snapshot checksum (include/vsearch.h vs_checksum) ----
 * Not part of the reference (Qdrant's on-disk format is its own); restated
 * from this repository's file-format definition: the sum mod 2^64 over the
 * little-endian 64-bit words w_i of the byte range (last word zero-padded)
 * of splitmix64(w_i ^ i * 0x9E3779B97F4A7C15). Sequential loop, one word at
 * a time. */
uint64_t oracle_checksum(const void* p, uint64_t nbytes) {
  const unsigned char* b = (const unsigned char*)p;
  uint64_t s = 0;
  for (uint64_t w = 0; w * 8 < nbytes; ++w) {
    uint64_t x = 0;
    for (int i = 0; i < 8 && w * 8 + i < nbytes; ++i) x |= (uint64_t)b[w * 8 + i] << (8 * i);
    s += o_splitmix64(x ^ (w * 0x9E3779B97F4A7C15ull));
  }
  return s;
}
