// TEST DOUBLE for the ThreadSanitizer build of the service layer
// (tests/test_tsan_service.py). Never linked into the product: the product's
// libvsearch.so is the HIP engine and has no CPU path. This file implements
// just the include/vsearch.h calls csrc/service/ makes, with a brute-force CPU
// scan under one reader/writer lock, so the service's own locking (collection
// map, per-collection state, filter cache, batcher queues) can run under TSAN
// on a machine without a GPU. Results follow the C-ABI contract (score desc,
// row asc; cosine rows and queries normalised) but nothing here is a parity
// reference: the oracle is oracle/.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/vsearch.h"

namespace {

thread_local std::string t_err;

int fail(int rc, const std::string& m) {
  t_err = m;
  return rc;
}

struct Coll {
  uint32_t dim = 0;
  int metric = VS_METRIC_COSINE, dtype = VS_DTYPE_F32;
  std::vector<float> rows;  // preprocessed
  uint64_t n() const { return dim ? rows.size() / dim : 0; }
};

struct Filter {
  std::string coll;
  uint64_t rows = 0;
  std::vector<uint64_t> bits;
};

void normalise(float* v, uint32_t dim) {
  double s = 0;
  for (uint32_t d = 0; d < dim; ++d) s += (double)v[d] * v[d];
  if (s > 0) {
    const float inv = (float)(1.0 / std::sqrt(s));
    for (uint32_t d = 0; d < dim; ++d) v[d] *= inv;
  }
}

}  // namespace

struct vs_engine {
  std::shared_mutex mu;
  std::map<std::string, std::shared_ptr<Coll>> colls;
  std::map<uint64_t, Filter> filters;
  uint64_t next_filter = 1;
};

extern "C" {

int vs_open(const vs_config*, vs_engine** out) {
  if (!out) return fail(VS_ERR_INVALID_ARG, "null out");
  *out = new vs_engine();
  return VS_OK;
}

void vs_close(vs_engine* e) { delete e; }

// Two pretend devices: a collection's "device" is a hash of its name, so the
// service's per-device batcher lanes run under TSAN too.
int vs_collection_placement(vs_engine* e, const char* name, int32_t* device) {
  std::shared_lock<std::shared_mutex> g(e->mu);
  if (!e->colls.count(name)) return fail(VS_ERR_NOT_FOUND, "not found");
  *device = (int32_t)(std::hash<std::string>()(name) % 2);
  return VS_OK;
}

const char* vs_last_error(void) { return t_err.c_str(); }

int vs_collection_create(vs_engine* e, const char* name, uint32_t dim, int metric, int dtype,
                         uint64_t, uint64_t) {
  std::unique_lock<std::shared_mutex> g(e->mu);
  if (e->colls.count(name)) return fail(VS_ERR_EXISTS, "exists");
  auto c = std::make_shared<Coll>();
  c->dim = dim, c->metric = metric, c->dtype = dtype;
  e->colls[name] = c;
  return VS_OK;
}

int vs_collection_info(vs_engine* e, const char* name, uint32_t* dim, uint64_t* rows,
                       int* metric, int* dtype) {
  std::shared_lock<std::shared_mutex> g(e->mu);
  auto it = e->colls.find(name);
  if (it == e->colls.end()) return fail(VS_ERR_NOT_FOUND, "not found");
  if (dim) *dim = it->second->dim;
  if (rows) *rows = it->second->n();
  if (metric) *metric = it->second->metric;
  if (dtype) *dtype = it->second->dtype;
  return VS_OK;
}

int vs_collection_drop(vs_engine* e, const char* name) {
  std::unique_lock<std::shared_mutex> g(e->mu);
  if (!e->colls.erase(name)) return fail(VS_ERR_NOT_FOUND, "not found");
  for (auto it = e->filters.begin(); it != e->filters.end();)
    it = it->second.coll == name ? e->filters.erase(it) : std::next(it);
  return VS_OK;
}

int vs_upsert(vs_engine* e, const char* coll, uint64_t n, uint32_t dim, const uint64_t* rows,
              const float* vecs) {
  std::unique_lock<std::shared_mutex> g(e->mu);
  auto it = e->colls.find(coll);
  if (it == e->colls.end()) return fail(VS_ERR_NOT_FOUND, "not found");
  Coll& c = *it->second;
  if (dim != c.dim) return fail(VS_ERR_DIM_MISMATCH, "dim");
  uint64_t top = c.n();
  for (uint64_t i = 0; i < n; ++i) top = std::max(top, rows[i] + 1);
  c.rows.resize(top * dim, 0.f);
  for (uint64_t i = 0; i < n; ++i) {
    float* dst = c.rows.data() + rows[i] * dim;
    std::memcpy(dst, vecs + i * dim, dim * sizeof(float));
    if (c.metric == VS_METRIC_COSINE) normalise(dst, dim);
  }
  return VS_OK;
}

int vs_generate(vs_engine* e, const char* coll, uint64_t n, uint64_t seed) {
  std::unique_lock<std::shared_mutex> g(e->mu);
  auto it = e->colls.find(coll);
  if (it == e->colls.end()) return fail(VS_ERR_NOT_FOUND, "not found");
  Coll& c = *it->second;
  const uint64_t base = c.n();
  c.rows.resize((base + n) * c.dim);
  uint64_t s = seed * 0x9E3779B97F4A7C15ull + 1;
  for (uint64_t i = base * c.dim; i < c.rows.size(); ++i) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    c.rows[i] = (float)((double)(s >> 11) / 9007199254740992.0 - 0.5);
  }
  for (uint64_t r = base; r < base + n; ++r) normalise(c.rows.data() + r * c.dim, c.dim);
  return VS_OK;
}

// Qdrant-style f32 dot: 8-lane vector accumulators, then a fixed-order sum
// (so the CPU backend of tools/c1_http.py is a fair SIMD scan, not a scalar
// loop).
static float dot(const float* x, const float* q, uint32_t dim) {
  typedef float v8 __attribute__((vector_size(32)));
  v8 a0 = {0, 0, 0, 0, 0, 0, 0, 0}, a1 = a0;
  uint32_t d = 0;
  for (; d + 16 <= dim; d += 16) {
    v8 x0, x1, q0, q1;
    std::memcpy(&x0, x + d, 32);
    std::memcpy(&x1, x + d + 8, 32);
    std::memcpy(&q0, q + d, 32);
    std::memcpy(&q1, q + d + 8, 32);
    a0 += x0 * q0;
    a1 += x1 * q1;
  }
  a0 += a1;
  float s = 0;
  for (int j = 0; j < 8; ++j) s += a0[j];
  for (; d < dim; ++d) s += x[d] * q[d];
  return s;
}

static int search_impl(vs_engine* e, const char* coll, const float* q, uint32_t nq, uint32_t dim,
                       uint32_t k, const uint64_t* allow, float* os, uint64_t* orow,
                       uint32_t* ocnt) {
  std::shared_lock<std::shared_mutex> g(e->mu);
  auto it = e->colls.find(coll);
  if (it == e->colls.end()) return fail(VS_ERR_NOT_FOUND, "not found");
  const Coll& c = *it->second;
  if (dim != c.dim) return fail(VS_ERR_DIM_MISMATCH, "dim");
  if (k == 0 || k > 1024) return fail(VS_ERR_INVALID_ARG, "k");
  std::vector<float> qq(dim);
  for (uint32_t i = 0; i < nq; ++i) {
    std::memcpy(qq.data(), q + (size_t)i * dim, dim * sizeof(float));
    if (c.metric == VS_METRIC_COSINE) normalise(qq.data(), dim);
    std::vector<std::pair<float, uint64_t>> hits;
    for (uint64_t r = 0; r < c.n(); ++r) {
      if (allow && !((allow[r / 64] >> (r % 64)) & 1)) continue;
      hits.push_back({dot(c.rows.data() + r * dim, qq.data(), dim), r});
    }
    const size_t m = std::min<size_t>(k, hits.size());
    std::partial_sort(hits.begin(), hits.begin() + m, hits.end(), [](auto& a, auto& b) {
      return a.first != b.first ? a.first > b.first : a.second < b.second;
    });
    ocnt[i] = (uint32_t)m;
    for (uint32_t j = 0; j < k; ++j) {
      os[(size_t)i * k + j] = j < m ? hits[j].first : 0.f;
      orow[(size_t)i * k + j] = j < m ? hits[j].second : 0;
    }
  }
  return VS_OK;
}

int vs_search(vs_engine* e, const char* coll, const float* q, uint32_t nq, uint32_t dim,
              uint32_t k, float* os, uint64_t* orow, uint32_t* ocnt) {
  return search_impl(e, coll, q, nq, dim, k, nullptr, os, orow, ocnt);
}

int vs_search_filtered(vs_engine* e, const char* coll, const float* q, uint32_t nq, uint32_t dim,
                       uint32_t k, const uint64_t* allow, uint64_t, float* os, uint64_t* orow,
                       uint32_t* ocnt) {
  return search_impl(e, coll, q, nq, dim, k, allow, os, orow, ocnt);
}

int vs_filter_create(vs_engine* e, const char* coll, const uint64_t* allow, uint64_t words,
                     uint64_t* id) {
  std::unique_lock<std::shared_mutex> g(e->mu);
  auto it = e->colls.find(coll);
  if (it == e->colls.end()) return fail(VS_ERR_NOT_FOUND, "not found");
  Filter f{coll, it->second->n(), std::vector<uint64_t>(allow, allow + words)};
  *id = e->next_filter++;
  e->filters[*id] = std::move(f);
  return VS_OK;
}

int vs_filter_drop(vs_engine* e, uint64_t id) {
  std::unique_lock<std::shared_mutex> g(e->mu);
  return e->filters.erase(id) ? VS_OK : fail(VS_ERR_NOT_FOUND, "no filter");
}

int vs_search_filter_id(vs_engine* e, const char* coll, const float* q, uint32_t nq,
                        uint32_t dim, uint32_t k, uint64_t id, float* os, uint64_t* orow,
                        uint32_t* ocnt) {
  std::vector<uint64_t> bits;
  {
    std::shared_lock<std::shared_mutex> g(e->mu);
    auto f = e->filters.find(id);
    auto c = e->colls.find(coll);
    if (f == e->filters.end() || c == e->colls.end() || f->second.coll != coll ||
        f->second.rows != c->second->n())
      return fail(VS_ERR_INVALID_ARG, "stale filter");
    bits = f->second.bits;
  }
  return search_impl(e, coll, q, nq, dim, k, bits.data(), os, orow, ocnt);
}

// snapshot: header (dim, metric, dtype, rows) + fp32 rows
int vs_snapshot(vs_engine* e, const char* coll, const char* path) {
  std::shared_lock<std::shared_mutex> g(e->mu);
  auto it = e->colls.find(coll);
  if (it == e->colls.end()) return fail(VS_ERR_NOT_FOUND, "not found");
  const Coll& c = *it->second;
  FILE* f = std::fopen(path, "wb");
  if (!f) return fail(VS_ERR_IO, "open");
  const uint64_t hdr[4] = {c.dim, (uint64_t)c.metric, (uint64_t)c.dtype, c.n()};
  bool ok = std::fwrite(hdr, sizeof(hdr), 1, f) == 1 &&
            (c.rows.empty() || std::fwrite(c.rows.data(), 4, c.rows.size(), f) == c.rows.size());
  ok = std::fclose(f) == 0 && ok;
  return ok ? VS_OK : fail(VS_ERR_IO, "write");
}

int vs_restore(vs_engine* e, const char* coll, const char* path) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return fail(VS_ERR_IO, "open");
  uint64_t hdr[4];
  auto c = std::make_shared<Coll>();
  bool ok = std::fread(hdr, sizeof(hdr), 1, f) == 1;
  if (ok) {
    c->dim = (uint32_t)hdr[0], c->metric = (int)hdr[1], c->dtype = (int)hdr[2];
    c->rows.resize(hdr[3] * hdr[0]);
    ok = c->rows.empty() || std::fread(c->rows.data(), 4, c->rows.size(), f) == c->rows.size();
  }
  std::fclose(f);
  if (!ok) return fail(VS_ERR_IO, "read");
  std::unique_lock<std::shared_mutex> g(e->mu);
  if (e->colls.count(coll)) return fail(VS_ERR_EXISTS, "exists");
  e->colls[coll] = c;
  return VS_OK;
}

int vs_health(vs_engine* e, char* buf, size_t len) {
  std::shared_lock<std::shared_mutex> g(e->mu);
  const int n = std::snprintf(buf, len,
                              "{\"status\":\"healthy\",\"engine\":\"tsan-test-double\","
                              "\"collections\":%zu}",
                              e->colls.size());
  return n > 0 && (size_t)n < len ? VS_OK : fail(VS_ERR_INVALID_ARG, "buffer");
}

}  // extern "C"
