// vs_engine.cpp — host side of the engine: the C-ABI of include/vsearch.h.
//
// One vs_engine owns one HIP device, one stream and a set of resident
// collections (row-major fp32/bf16 matrices in HBM). It replaces the Qdrant
// server and the gRPC client globals of rag/vector-service/main.go:44-65.
// All device work of an engine is serialised on its stream; collections are
// guarded by reader/writer locks (search = reader, upsert = writer), which is
// what net/http's goroutine-per-request handlers (main.go:77) need.
#include <hip/hip_runtime.h>
#include <link.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/vsearch.h"
#include "vs_common.h"
#include "vs_dev.h"
#include "vs_kernels.h"

namespace vsd {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
int fail_hip(hipError_t e, const char* what) {
  return fail(e == hipErrorOutOfMemory ? VS_ERR_OOM : VS_ERR_DEVICE,
              std::string(what) + ": " + hipGetErrorString(e));
}



std::atomic<uint64_t> g_coll_gen{1};

std::shared_ptr<Collection> find_coll(DevEngine* eng, const char* name) {
  DevStore& st = *eng->store;
  std::lock_guard<std::mutex> g(st.map_mu);
  auto it = st.colls.find(name ? name : "");
  return it == st.colls.end() ? nullptr : it->second;
}

std::shared_ptr<DevFilter> find_filter(DevEngine* eng, uint64_t filter_id) {
  DevStore& st = *eng->store;
  std::lock_guard<std::mutex> g(st.filt_mu);
  auto it = st.filters.find(filter_id);
  return it == st.filters.end() ? nullptr : it->second;
}

DevEngine* pick_context(DevEngine* eng, std::unique_lock<std::mutex>* lk, bool heavy) {
  const std::vector<DevEngine*>& cx = eng->store->ctx;
  if (heavy) {  // batched scans of large collections queue on the primary's stream
    *lk = std::unique_lock<std::mutex>(cx[0]->work_mu);
    return cx[0];
  }
  // an idle context first (no host search in flight on it), then any free lock
  for (int pass = 0; pass < 2; ++pass)
    for (DevEngine* c : cx) {
      if (pass == 0 && c->inflight.load(std::memory_order_relaxed) != 0) continue;
      std::unique_lock<std::mutex> g(c->work_mu, std::try_to_lock);
      if (g.owns_lock()) {
        *lk = std::move(g);
        return c;
      }
    }
  DevEngine* best = cx[0];
  for (DevEngine* c : cx)
    if (c->inflight.load(std::memory_order_relaxed) < best->inflight.load(std::memory_order_relaxed))
      best = c;
  *lk = std::unique_lock<std::mutex>(best->work_mu);
  return best;
}

hipError_t set_dev(DevEngine* eng) { return hipSetDevice(eng->device); }

// Makes `s` the engine's current stream (work_mu held). Work enqueued on s
// is ordered after everything enqueued so far on the previous stream, so the
// scratch buffers are never used by two streams at once; a caller that keeps
// using one stream (a serving loop on torch's current stream) pays nothing.
hipError_t use_stream(DevEngine* eng, hipStream_t s) {
  if (s == eng->stream) return hipSuccess;
  hipError_t e = hipEventRecord(eng->xev, eng->stream);
  if (e == hipSuccess) e = hipStreamWaitEvent(s, eng->xev, 0);
  if (e == hipSuccess) eng->stream = s;
  return e;
}

bool timing_on(DevEngine* eng) { return (eng->flags & VS_FLAG_TIMING) != 0; }

bool timing_wanted(DevEngine* eng, const std::vector<EventPair>& v) {
  return timing_on(eng) && (&v == &eng->scan_ev || (eng->flags & VS_FLAG_TIMING_MERGE));
}

hipError_t ev_begin(DevEngine* eng, std::vector<EventPair>& v) {
  if (!timing_wanted(eng, v)) return hipSuccess;
  if (&v == &eng->scan_ev && (eng->flags & VS_FLAG_TIMING_SAMPLE)) {
    // bracket one scan in scan_period (search_core: 4 for batches, 16 for one
    // query), the period-th first: not the first scan after a synchronize
    const uint32_t p = eng->scan_period;
    eng->scan_skip = eng->scan_tick++ % p != p - 1;
    if (eng->scan_skip) return hipSuccess;
  }
  EventPair p{};
  for (hipEvent_t* ev : {&p.a, &p.b}) {
    if (!eng->ev_pool.empty()) {
      *ev = eng->ev_pool.back();
      eng->ev_pool.pop_back();
    } else {
      hipError_t e = hipEventCreate(ev);
      if (e != hipSuccess) return e;
    }
  }
  v.push_back(p);
  return hipEventRecord(p.a, eng->stream);
}
hipError_t ev_end(DevEngine* eng, std::vector<EventPair>& v) {
  if (!timing_wanted(eng, v) || v.empty()) return hipSuccess;
  if (&v == &eng->scan_ev && (eng->flags & VS_FLAG_TIMING_SAMPLE) && eng->scan_skip)
    return hipSuccess;
  return hipEventRecord(v.back().b, eng->stream);
}

// Rows allocated past the capacity: the MFMA scan streams whole 32-row tiles
// and reads (then masks) up to 31 rows beyond the last one.
constexpr uint64_t kPadRows = 32;
// q8_glob: {absmax, dmax, nmax, S}, then (r06) the speculative bound's
// counters and per-k state (vs_kernels.h Q8SpecStat / Q8SpecK)
using vsk::kQ8GlobBytes;
using vsk::kQ8SpecK;
// Filtered single-query searches gather the allowed rows when at most
// 1 / kGatherDensityDen of the collection is allowed: below
// that density the scattered 1.5-3 KB row reads stay near the streaming rate,
// and the compaction launch is paid back many times over.
constexpr uint64_t kGatherDensityDen = 8;
// Per-query launch overhead of a gathered scan (scan + merge launches,
// ~10 us) in bytes of HBM streaming, for the batch decision in search_core.
constexpr uint64_t kGatherCallBytes = 64ull << 20;
static_assert(kSpecK == vsk::kQ8SpecK, "vs_spec_host.h sizes the host bookkeeping by k");
// Collection bytes from which a batched host search is "heavy" (heavy_search).
constexpr uint64_t kHeavyBytes = 256ull << 20;
// Smallest batch of an fp32 collection that takes the MFMA pass.
constexpr uint32_t kF32MfmaMinQueries = 4;

// Grows a collection to hold `need` rows (writer lock held by the caller).
int grow(DevEngine* eng, Collection& c, uint64_t need) {
  if (need <= c.cap) return VS_OK;
  // The int8 copy is rebuilt at the new capacity anyway (q8_after_write:
  // q8_cap < cap), so free it first: the peak of a grow stays old + new rows,
  // not old + new + the old copy. No pass may still read it.
  if (c.q8) {
    VS_HIP(hipStreamSynchronize(eng->stream), "sync");
    c.q8_free();
  }
  uint64_t ncap = std::max<uint64_t>({need, c.cap + c.cap / 2, 1024});
  void* nd = nullptr;
  hipError_t e = hipMalloc(&nd, (ncap + kPadRows) * c.row_bytes());
  if (e != hipSuccess) {
    // exact fit as a last resort
    ncap = need;
    e = hipMalloc(&nd, (ncap + kPadRows) * c.row_bytes());
    if (e != hipSuccess) return fail_hip(e, "collection grow");
  }
  // zero the padding so masked tail rows are finite
  VS_HIP(hipMemsetAsync((char*)nd + ncap * c.row_bytes(), 0, kPadRows * c.row_bytes(),
                        eng->stream),
         "pad rows");
  if (c.data && c.rows) {
    VS_HIP(hipMemcpyAsync(nd, c.data, c.rows * c.row_bytes(), hipMemcpyDeviceToDevice,
                          eng->stream),
           "collection grow copy");
    VS_HIP(hipStreamSynchronize(eng->stream), "collection grow sync");
  }
  if (c.data) (void)hipFree(c.data);
  c.data = nd;
  c.cap = ncap;
  return VS_OK;
}

// ---- int8 prefilter copy (vs_kernels.h "int8 prefilter") ------
// On by default; VS_Q8=0 (read once) makes no copy, and batched searches then
// read the bf16 rows only.
bool q8_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("VS_Q8");
    return !(e && e[0] == '0');
  }();
  return v;
}

// A collection keeps an int8 copy once its batched searches take the
// candidate pass (8 or more tiles per workgroup) -- q8_supported dims (bf16
// 768 / 1024, fp32 768).
bool q8_wanted(const DevEngine* eng, const Collection& c) {
  return q8_enabled() && !(eng->flags & VS_FLAG_NO_PREFILTER) &&
         vsk::q8_supported(c.dim, c.dtype == VS_DTYPE_F32) &&
         c.rows < 0xFFFFFFFFull && vsk::mfma_tiles_per_wg((uint32_t)c.rows) >= 8;
}

uint64_t q8_reserve_bytes(int flags, uint32_t dim, int dtype, uint64_t rows) {
  if (!q8_enabled() || (flags & VS_FLAG_NO_PREFILTER) || rows >= 0xFFFFFFFFull ||
      !vsk::q8_supported(dim, dtype == VS_DTYPE_F32) || vsk::mfma_tiles_per_wg((uint32_t)rows) < 8)
    return 0;
  return (rows + kPadRows) * dim + ((rows + kPadRows) / 32 + 1) * 8;
}

// Brings the int8 copy up to date after a store-side write of rows [r0, r1)
// (or, with d_tiles, of the nt tiles listed there), on eng->stream, the
// writer lock and work_mu held, c.rows already counting the new rows. The
// whole copy is rebuilt -- a new scale S from max |x| -- when it is first made,
// when the collection's buffer grew, and whenever the rows have doubled since
// S was chosen (rows quantised with an older S stay exact: their error
// bounds are measured, not assumed). No memory for the copy: none is kept,
// and batched searches read the bf16 rows.
int q8_after_write_impl(DevEngine* eng, Collection& c, uint64_t r0, uint64_t r1,
                        const uint32_t* d_tiles, uint32_t nt);

// Any failure after the rows were written leaves the copy behind the rows, and
// its bounds would no longer cover them: drop it (batched searches then take
// the bf16 / f32 pass until the next full rebuild).
// VS_Q8_FAIL_AFTER_WRITE=1 (tests only, read once) injects such a failure.
bool q8_fail_injected() {
  static const bool v = [] {
    const char* e = std::getenv("VS_Q8_FAIL_AFTER_WRITE");
    return e && e[0] == '1';
  }();
  return v;
}

int q8_after_write(DevEngine* eng, Collection& c, uint64_t r0, uint64_t r1,
                   const uint32_t* d_tiles = nullptr, uint32_t nt = 0) {
  int rc = q8_fail_injected() && c.q8
               ? fail(VS_ERR_DEVICE, "int8 copy: injected failure (VS_Q8_FAIL_AFTER_WRITE)")
               : q8_after_write_impl(eng, c, r0, r1, d_tiles, nt);
  if (rc != VS_OK && c.q8) {
    (void)hipStreamSynchronize(eng->stream);
    c.q8_free();
  }
  return rc;
}

// The speculative bound's per-k state back to unset (zero: no ratio, no
// cool-down; its counters stay), and a new generation, so no context uses a
// ratio learned on the rows before this write (r05).
hipError_t q8_spec_reset(DevEngine* eng, Collection& c) {
  static std::atomic<uint64_t> next_gen{1};
  c.q8_gen = next_gen.fetch_add(1);
  spec_advice_reset(c.q8_advice);
  return hipMemsetAsync(vsk::q8_spec_k(c.q8_glob), 0, (size_t)kQ8SpecK * sizeof(vsk::Q8SpecK),
                        eng->stream);
}

int q8_after_write_impl(DevEngine* eng, Collection& c, uint64_t r0, uint64_t r1,
                        const uint32_t* d_tiles, uint32_t nt) {
  if (!q8_wanted(eng, c)) return VS_OK;
  const uint32_t dim = c.dim;
  const uint32_t rows = (uint32_t)c.rows;
  const bool full = !c.q8 || c.q8_cap < c.cap || c.rows >= 2 * c.q8_scaled_at;
  if (full) {
    if (c.q8_cap < c.cap) {
      VS_HIP(hipStreamSynchronize(eng->stream), "sync");  // no pass reads the old copy
      c.q8_free();
      const uint64_t tiles = (c.cap + kPadRows) / 32 + 1;
      hipError_t e = hipMalloc(&c.q8, (c.cap + kPadRows) * dim);
      if (e == hipSuccess) e = hipMalloc((void**)&c.q8_meta, tiles * 8);
      if (e == hipSuccess) e = hipMalloc((void**)&c.q8_glob, kQ8GlobBytes);
      if (e == hipSuccess)
        e = hipHostMalloc((void**)&c.q8_advice, 2 * kQ8SpecK * 4,
                          hipHostMallocCoherent | hipHostMallocMapped);
      if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&c.q8_advice_dev, c.q8_advice, 0);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        c.q8_free();
        return VS_OK;
      }
      c.q8_cap = c.cap;
      VS_HIP(hipMemsetAsync(c.q8, 0, (c.cap + kPadRows) * dim, eng->stream), "zero int8 copy");
      VS_HIP(hipMemsetAsync(vsk::q8_spec_stat(c.q8_glob), 0, sizeof(vsk::Q8SpecStat), eng->stream),
             "zero speculative-bound counters");
    }
    VS_HIP(hipMemsetAsync(c.q8_glob, 0, 16, eng->stream), "zero int8 bounds");
    VS_HIP(q8_spec_reset(eng, c), "reset speculative-bound ratios");
    VS_HIP(vsk::launch_q8_absmax(c.data, c.dtype == VS_DTYPE_F32, (uint64_t)rows * dim, c.q8_glob,
                                 eng->stream),
           "int8 scale");
    VS_HIP(vsk::launch_q8_set_scale(c.q8_glob, eng->stream), "int8 scale");
    VS_HIP(vsk::launch_q8_quantize(c.data, c.dtype == VS_DTYPE_F32, rows, dim, nullptr, 0,
                                   (rows + 31) / 32, (int8_t*)c.q8, c.q8_meta, c.q8_glob,
                                   eng->stream),
           "int8 copy");
    c.q8_scaled_at = c.rows;
    return VS_OK;
  }
  VS_HIP(q8_spec_reset(eng, c), "reset speculative-bound ratios");
  if (d_tiles) {
    VS_HIP(vsk::launch_q8_quantize(c.data, c.dtype == VS_DTYPE_F32, rows, dim, d_tiles, 0, nt,
                                   (int8_t*)c.q8, c.q8_meta, c.q8_glob, eng->stream),
           "int8 copy");
  } else if (r1 > r0) {
    const uint32_t t0 = (uint32_t)(r0 / 32), t1 = (uint32_t)((r1 - 1) / 32) + 1;
    VS_HIP(vsk::launch_q8_quantize(c.data, c.dtype == VS_DTYPE_F32, rows, dim, nullptr, t0, t1 - t0,
                                   (int8_t*)c.q8, c.q8_meta, c.q8_glob, eng->stream),
           "int8 copy");
  }
  return VS_OK;
}

// ---- snapshot file format (include/vsearch.h vs_snapshot) -------------------
struct SnapHeader {
  char magic[8];  // "VSNAP01\0"
  uint32_t version, header_bytes;
  uint32_t dim;
  int32_t metric, dtype;
  uint32_t elem_bytes;
  uint64_t rows, row_base, data_bytes;
  uint64_t data_checksum;
  uint64_t header_checksum;  // vs::snap_word sum over the 64 bytes above
  uint8_t reserved[56];      // zero
};
static_assert(sizeof(SnapHeader) == 128, "snapshot header is 128 bytes");
constexpr char kSnapMagic[8] = {'V', 'S', 'N', 'A', 'P', '0', '1', '\0'};
constexpr size_t kSnapChunk = 64ull << 20;  // D2H / H2D staging per chunk

uint64_t header_sum(const SnapHeader& h) {
  uint64_t w[8], s = 0;
  std::memcpy(w, &h, 64);
  for (int i = 0; i < 8; ++i) s += vs::snap_word(w[i], (uint64_t)i);
  return s;
}

struct PinnedPair {  // two staging buffers: one in flight, one on disk I/O
  void* p[2] = {nullptr, nullptr};
  ~PinnedPair() {
    for (void* q : p)
      if (q) (void)hipHostFree(q);
  }
  hipError_t alloc(size_t n) {
    for (void*& q : p) {
      hipError_t e = hipHostMalloc(&q, n, hipHostMallocDefault);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
};

// A snapshot's own stream and checksum word (vs_snapshot runs outside work_mu).
struct SnapStream {
  hipStream_t st = nullptr;
  uint64_t* sum = nullptr;
  hipError_t open() {
    hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&sum, 8);
    return e;
  }
  ~SnapStream() {
    if (st) (void)hipStreamSynchronize(st);
    if (sum) (void)hipFree(sum);
    if (st) (void)hipStreamDestroy(st);
  }
};

struct FileCloser {
  FILE* f = nullptr;
  ~FileCloser() {
    if (f) std::fclose(f);
  }
};

int device_checksum(DevEngine* eng, const Collection& c, uint64_t* out) {
  VS_HIP(eng->scratch8.ensure(8), "alloc checksum");
  VS_HIP(vsk::launch_checksum(c.data, c.rows * c.row_bytes(), eng->scratch8.as<uint64_t>(),
                              eng->stream),
         "checksum");
  VS_HIP(hipMemcpyAsync(out, eng->scratch8.p, 8, hipMemcpyDeviceToHost, eng->stream),
         "checksum D2H");
  VS_HIP(hipStreamSynchronize(eng->stream), "checksum sync");
  return VS_OK;
}

// Single-query scans (GEMV path) of preprocessed fp32 queries qp[q0 .. q0+n)
// -> keys d_keys[i * k], one scan + merge per query. For bf16 collections qp
// already holds bf16-rounded values (search_core's query prep). With `gather`
// (n_gather device row indices) only those rows are scanned.
// Workgroups of the first stage of a two-stage merge of L lists of k keys
// (1 = one stage). The one-workgroup merge's fast paths cover up to 8192
// keys at k <= 32; past that (large k over many lists) a first stage of G
// workgroups, each over L / G lists, runs the merge in parallel. G divides
// L and leaves >= 8 lists per group.
uint32_t merge_groups(uint32_t L, uint32_t k) {
  // r03: off unless VS_MERGE_TWO_STAGE=1 (read once). With the sample-bound
  // merge one workgroup is as fast or faster at every size measured (bf16,
  // one query: 2k rows k = 100 89.7 -> 47.6 us, 20k 71.3 -> 63.5, 12.5M
  // 2962 -> 2953; profiles/r03_merge_two_stage_ab.jsonl)
  static const bool two = [] {
    const char* e = std::getenv("VS_MERGE_TWO_STAGE");
    return e && e[0] == '1';
  }();
  if (!two || k <= 32 || (uint64_t)L * k <= 8192) return 1;
  for (uint32_t g = 64; g >= 4; --g)
    if (L % g == 0 && L / g >= 8) return g;
  return 1;
}

int search_gemv(DevEngine* eng, Collection& c, float* qp, uint32_t q0, uint32_t n, uint32_t k,
                uint64_t* d_keys, const uint64_t* allow = nullptr,
                const uint32_t* gather = nullptr, uint32_t n_gather = 0,
                HostDirect* direct = nullptr) {
  const uint32_t dim = c.dim;
  const bool bf16 = c.dtype == VS_DTYPE_BF16;
  const uint32_t n_rows = gather ? n_gather : (uint32_t)c.rows;
  const uint32_t row_base = (uint32_t)c.row_base;
  const uint32_t maxl = vsk::gemv_max_lists(dim, bf16, n_rows, k);
  const size_t lbytes = (size_t)maxl * k * 8;
  const size_t mbytes = (size_t)64 * k * 8;  // two-stage merge: <= 64 groups
  if (eng->lists.bytes < lbytes || eng->merge_tmp.bytes < mbytes) {
    VS_HIP(hipStreamSynchronize(eng->stream), "sync");
    VS_HIP(eng->lists.ensure(lbytes), "alloc list scratch");
    VS_HIP(eng->merge_tmp.ensure(mbytes), "alloc merge scratch");
  }
  for (uint32_t i = q0; i < q0 + n; ++i) {
    uint32_t L = 0;
    VS_HIP(ev_begin(eng, eng->scan_ev), "event");
    VS_HIP(vsk::launch_gemv(c.data, bf16, dim, n_rows, row_base, qp + (size_t)i * dim, k,
                            eng->lists.as<uint64_t>(), maxl, &L, eng->stream, allow, gather),
           "gemv scan");
    VS_HIP(ev_end(eng, eng->scan_ev), "event");
    VS_HIP(ev_begin(eng, eng->merge_ev), "event");
    const uint32_t G = merge_groups(L, k);
    if (G > 1) {
      // two stages: G workgroups each take the top k of L / G lists, then
      // one merges the G lists (exact: the global top k is among the groups'
      // top k). One workgroup over 768 x 100 keys took 195 us (12.5M rows,
      // k = 100: 6% of the step).
      VS_HIP(vsk::launch_merge(eng->lists.as<uint64_t>(), L / G, k, (uint64_t)(L / G) * k, G, k,
                               k, eng->merge_tmp.as<uint64_t>(), eng->stream),
             "merge (groups)");
      VS_HIP(vsk::launch_merge(eng->merge_tmp.as<uint64_t>(), G, k, 0, 1, k, k,
                               d_keys + (size_t)(i - q0) * k, eng->stream),
             "merge");
    } else if (direct && n == 1) {  // the keys and the completion word to the host
      VS_HIP(vsk::launch_merge(eng->lists.as<uint64_t>(), L, k, 0, 1, k, k, direct->keys,
                               eng->stream, direct->flag, direct->seq),
             "merge");
      direct->used = true;
    } else {
      VS_HIP(vsk::launch_merge(eng->lists.as<uint64_t>(), L, k, 0, 1, k, k,
                               d_keys + (size_t)(i - q0) * k, eng->stream),
             "merge");
    }
    VS_HIP(ev_end(eng, eng->merge_ev), "event");
  }
  return VS_OK;
}

// Large k (k > vsk::kMaxK: Qdrant serves any limit, rag/vector-service/
// main.go:252): per query one score pass over the collection (the GEMV
// stream writing every row's score image instead of keeping a list), radix
// select of the k-th key on the device, compaction of the k keys, rocPRIM
// sort (vs_select.hip). keff = min(k, unmasked rows) keys per query; the
// rest of each [k] row of d_keys is 0. Exact, no host round trip.
// Smallest k of the large-k path for a streamed scan (VS_LARGE_K_FROM
// overrides, read once; never above kMaxK + 1, the list scans' limit). The
// GEMV list path keeps k <= 128 in 1-2 registers per lane; past that (16 per
// lane) its inserts cost more than the select: at 10M x 768 bf16 one query
// took 3.30 / 4.15 / 8.12 ms at k = 129 / 256 / 1024 on the list path
// against 2.63-2.66 ms for any k on the large-k path (2.34-2.49 ms for the
// list path at k <= 128; profiles/r03_large_k_threshold.jsonl).
// The large-k selection in two launches (on unless VS_RSEL_FUSED=0; read
// once): rsel_f1/f2 instead of the 12-launch digit chain.
bool rsel_fused() {
  static const bool v = [] {
    const char* e = std::getenv("VS_RSEL_FUSED");
    return !(e && e[0] == '0');
  }();
  return v;
}

uint32_t large_k_from() {
  static const uint32_t v = [] {
    const char* e = std::getenv("VS_LARGE_K_FROM");
    const long x = e ? std::atol(e) : (long)vsk::kMfmaMaxK + 1;
    return (uint32_t)std::min<long>(std::max<long>(x, 1), (long)vsk::kMaxK + 1);
  }();
  return v;
}

int search_large_k(DevEngine* eng, Collection& c, const float* qp, uint32_t nq, uint32_t k,
                   uint64_t* d_keys, const uint64_t* allow, uint64_t avail) {
  const uint32_t n_rows = (uint32_t)c.rows;
  const uint32_t keff = (uint32_t)std::min<uint64_t>(k, avail);
  if (keff < k)
    VS_HIP(hipMemsetAsync(d_keys, 0, (size_t)nq * k * 8, eng->stream), "clear keys");
  if (keff == 0) return VS_OK;
  const size_t sort_bytes = vsk::sort_keys_temp_bytes(keff);
  if (!sort_bytes) return fail(VS_ERR_INTERNAL, "sort scratch size");
  if (eng->lk_sc.bytes < (size_t)n_rows * 4 || eng->lk_hist.bytes < vsk::kRselBins * 4 ||
      eng->lk_state.bytes < sizeof(vsk::RselState) || eng->lk_sel.bytes < (size_t)keff * 8 ||
      eng->lk_sort.bytes < sort_bytes) {
    VS_HIP(hipStreamSynchronize(eng->stream), "sync");
    VS_HIP(eng->lk_sc.ensure((size_t)n_rows * 4), "alloc score images");
    const bool fresh = eng->lk_hist.bytes < vsk::kRselBins * 4;
    VS_HIP(eng->lk_hist.ensure(vsk::kRselBins * 4), "alloc digit histogram");
    if (fresh) VS_HIP(hipMemsetAsync(eng->lk_hist.p, 0, eng->lk_hist.bytes, eng->stream), "zero");
    VS_HIP(eng->lk_state.ensure(sizeof(vsk::RselState)), "alloc select state");
    VS_HIP(eng->lk_sel.ensure((size_t)keff * 8), "alloc selected keys");
    VS_HIP(eng->lk_sort.ensure(sort_bytes), "alloc sort scratch");
  }
  const bool fused = rsel_fused();
  constexpr size_t kCtrBytes = 16 + vsk::kRselBins * 4;  // 3 counters (+pad), hist1
  if (fused && (eng->lk_cand.bytes < (size_t)n_rows * 8 || eng->lk_ctr.bytes < kCtrBytes)) {
    VS_HIP(hipStreamSynchronize(eng->stream), "sync");
    VS_HIP(eng->lk_cand.ensure((size_t)n_rows * 8), "alloc boundary-bucket keys");
    const bool fresh = eng->lk_ctr.bytes < kCtrBytes;
    VS_HIP(eng->lk_ctr.ensure(kCtrBytes), "alloc select counters");
    if (fresh) VS_HIP(hipMemsetAsync(eng->lk_ctr.p, 0, kCtrBytes, eng->stream), "zero");
  }
  uint32_t* sc = eng->lk_sc.as<uint32_t>();
  uint32_t* hist = eng->lk_hist.as<uint32_t>();
  for (uint32_t i = 0; i < nq; ++i) {
    VS_HIP(ev_begin(eng, eng->scan_ev), "event");
    VS_HIP(vsk::launch_gemv_scores(c.data, c.dtype == VS_DTYPE_BF16, c.dim, n_rows,
                                   qp + (size_t)i * c.dim, allow, sc, hist, eng->stream),
           "score pass");
    VS_HIP(ev_end(eng, eng->scan_ev), "event");
    VS_HIP(ev_begin(eng, eng->merge_ev), "event");
    if (fused)
      VS_HIP(vsk::launch_rsel_fused(sc, n_rows, (uint32_t)c.row_base, keff, hist,
                                    (uint32_t*)((char*)eng->lk_ctr.p + 16),
                                    eng->lk_ctr.as<uint32_t>(), eng->lk_sel.as<uint64_t>(),
                                    eng->lk_cand.as<uint64_t>(), eng->stream),
             "radix select (two launches)");
    else
      VS_HIP(vsk::launch_rsel(sc, n_rows, (uint32_t)c.row_base, keff, hist,
                              eng->lk_state.as<vsk::RselState>(), eng->lk_sel.as<uint64_t>(),
                              eng->stream),
             "radix select");
    VS_HIP(vsk::launch_sort_keys_desc(eng->lk_sel.as<uint64_t>(), d_keys + (size_t)i * k, keff,
                                      eng->lk_sort.p, eng->lk_sort.bytes, eng->stream),
           "sort selected keys");
    VS_HIP(ev_end(eng, eng->merge_ev), "event");
  }
  return VS_OK;
}

int merge_any(DevEngine* eng, const uint64_t* lists, uint32_t L, uint64_t lstride,
              uint64_t qstride, uint32_t nq, uint32_t kin, uint32_t k, uint64_t* out) {
  if (k <= vsk::kMaxK && kin <= vsk::kMaxK) {
    VS_HIP(vsk::launch_merge(lists, L, lstride, qstride, nq, kin, k, out, eng->stream), "merge");
    return VS_OK;
  }
  const size_t need = vsk::merge_large_scratch(L, nq, kin);
  if (eng->merge_big.bytes < need) {
    VS_HIP(hipStreamSynchronize(eng->stream), "sync");
    VS_HIP(eng->merge_big.ensure(need), "alloc merge scratch");
  }
  VS_HIP(vsk::launch_merge_large(lists, L, lstride, qstride, nq, kin, k, out, eng->merge_big.p,
                                 eng->merge_big.bytes, eng->stream),
         "merge (large k)");
  return VS_OK;
}

// The main pass records each candidate quarter's largest score and the
// select reads only the quarters that can hold a top-k key (r04; default on,
// VS_SELECT_QMAX=0 gives back the select that re-reads every slab; read once).
bool select_qmax() {
  static const bool v = [] {
    const char* e = std::getenv("VS_SELECT_QMAX");
    return !(e && e[0] == '0');
  }();
  return v;
}

// VS_Q8_SAMPLE=<factor>: overrides the int8 path's sample-tile factor (read
// once; ablation only; 0 = the k-dependent default in search_mfma)
// VS_Q8_SPEC (read once; default 1): batched int8 searches of bf16
// collections run on a speculative bound once the context has learned the
// collection's ratio for a k' >= k (r05); 0 = the sample path always
bool q8_spec_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("VS_Q8_SPEC");
    return !(e && e[0] == '0');
  }();
  return v;
}
// VS_Q8_SPEC_FORCE_FAIL=1 (tests only, read once): speculative batches run on
// a ratio of 12.08 (0x41 bytes), far above any unit-vector score, so every
// one fails its check and the gated sample path must answer it
bool q8_spec_force_fail() {
  static const bool v = [] {
    const char* e = std::getenv("VS_Q8_SPEC_FORCE_FAIL");
    return e && e[0] == '1';
  }();
  return v;
}

double q8_sample_scale() {
  static const double v = [] {
    const char* e = std::getenv("VS_Q8_SAMPLE");
    return e ? std::atof(e) : 0.0;
  }();
  return v;
}

// VS_Q8_PREP_APART=1: the int8 queries in their own launch (the r04 form
// before the fused bound + query launch; ablation only, read once)
// VS_Q8_SEL_VERIFY=1 (ablation): the batch's check / record by the int8
// select's last workgroup instead of a launch of its own after the select.
// One launch fewer, and no faster: 0.2768 / 0.2776 against 0.2763 / 0.2759 ms
// at the N = 8 share, C3 level (profiles/r06_sel_verify_ab.json) -- the last
// workgroup's hand-off costs what the launch did.
bool q8_sel_verify() {
  static const bool v = [] {
    const char* e = std::getenv("VS_Q8_SEL_VERIFY");
    return e && e[0] == '1';
  }();
  return v;
}

bool q8_prep_apart() {
  static const bool v = [] {
    const char* e = std::getenv("VS_Q8_PREP_APART");
    return e && e[0] == '1';
  }();
  return v;
}

// VS_SAMPLE_SCALE=<factor>: the same for the bf16 / f32 pass (ablation only)
double plain_sample_scale() {
  static const double v = [] {
    const char* e = std::getenv("VS_SAMPLE_SCALE");
    return e ? std::atof(e) : 0.0;
  }();
  return v;
}

// Batched scan on MFMA: bf16 rows on 16x16x32 bf16 MFMA (256
// queries per pass at dim <= 768), fp32 rows on 16x16x4 f32 MFMA (128):
//  1. sample pass over 1/128 of every workgroup's tiles -> tile maxima ->
//     sample_bound_kernel: per-query lower bound on the global k-th score;
//  2. main pass: rows reaching the bound -> candidate buffers -> select. A
//     full buffer quarter keeps its best slabs (exact, vs_kernels.h), so no
//     pass is ever re-run and nothing here waits on the device.
// Small collections (fewer than 8 tiles per workgroup) take the sorted-list
// pass (k <= 16) or the GEMV path.
// The query preprocessing search_core leaves to search_mfma (r06): enqueued
// first on every path, except that a speculative int8 batch fuses it into its
// first launch (launch_q8_prep_query).
struct QPrep {
  const float* in;
  bool cosine, round_qp;
  float* qp;     // fp32 copy (or null)
  uint16_t* qb;  // bf16 copy (or null)
};

int search_mfma(DevEngine* eng, Collection& c, float* qp, uint32_t nq, uint32_t k,
                uint64_t* d_keys, const uint64_t* allow, const QPrep& prep) {
  const uint32_t dim = c.dim;
  const uint32_t n_rows = (uint32_t)c.rows;
  const uint32_t row_base = (uint32_t)c.row_base;
  const bool f32 = c.dtype == VS_DTYPE_F32;
  const uint32_t P = vsk::mfma_queries(dim, f32);  // queries per pass
  const uint32_t PS = vsk::kMfmaQueries;      // query stride of the pass buffers
  const uint32_t npass = (nq + P - 1) / P;
  const uint32_t maxl = vsk::mfma_max_lists(n_rows);
  const uint32_t tpw = vsk::mfma_tiles_per_wg(n_rows);
  const bool fast = tpw >= 8;
  auto prep_now = [&]() -> int {
    VS_HIP(vsk::launch_query_prep(prep.in, nq, dim, prep.cosine, prep.round_qp, prep.qp, prep.qb,
                                  eng->stream),
           "query preprocess");
    return VS_OK;
  };
  if (!fast && k > vsk::kMfmaListMaxK) {
    const int rc = prep_now();
    if (rc != VS_OK) return rc;
    return search_gemv(eng, c, qp, 0, nq, k, d_keys, allow);
  }
  // int8 prefilter (batches of a collection with an int8 copy; a pre-mask
  // rides along as in the bf16 pass)
  const bool q8 = fast && c.q8 && c.q8_cap >= c.rows && q8_enabled();
  // The int8 path's sample grows with k: its admission window (2m) is wider
  // than the bf16 pass's, so a tighter k-th bound pays for more sample tiles
  // sooner (r04 sweep, profiles/r04_q8_sample_sweep.jsonl: x2 for k in 17..64,
  // x4 above; k = 50 at 10M +6%, k = 100 +7%; k <= 16 flat)
  const uint32_t st0 = vsk::mfma_sample_tiles(n_rows, dim, f32);
  uint32_t st = st0;
  if (q8 || plain_sample_scale() > 0) {
    const double f = !q8 ? plain_sample_scale()
                         : q8_sample_scale() > 0 ? q8_sample_scale()
                                                 : (k <= 16 ? 1.0 : k <= 64 ? 2.0 : 4.0);
    st = (uint32_t)std::max(1.0, std::min({(double)vsk::kMfmaMaxSampleTiles, (double)tpw, st * f}));
  }
  const uint32_t cap = vsk::mfma_cand_cap(n_rows, k, st);
  // the int8 pass admits ~5x the bf16 pass's rows (7.6k slabs per query at
  // 10M rows, k = 10; fullest quarter 29 -- tools/q8_check.hip stats mode):
  // sized at 8x so a full quarter (and the bf16 hand-back) stays rare
  // (at the unscaled sample size: a tighter bound shrinks the bf16-like part
  // of the admissions, not the window's)
  const uint32_t cap8 = q8 ? vsk::mfma_cand_cap(n_rows, k, st0, 8.0) : 0;
  const uint32_t capx = q8 ? cap8 : cap;  // (r05: no bf16 pass behind the int8 one)
  const size_t lbytes = fast ? 0 : (size_t)maxl * PS * k * 8;
  const size_t sbytes = (size_t)PS * 4;  // per-query sample bounds
  // main pass slabs: 32 B of scores + a 4-B tile row per slot
  const size_t slots = (size_t)maxl * PS * capx;
  const size_t cbytes = slots * 36;
  const size_t scbytes = (size_t)maxl * st * PS * 4;  // tile maxima, [query][wg * st]
  // counts [maxl][PS][4], then (select_qmax) the quarters' maxima, same shape
  const size_t nbytes = (size_t)maxl * PS * 4 * 4 * 2;
  const size_t q8qb = q8 ? (size_t)PS * dim : 0, q8pb = q8 ? vsk::kQ8ParBytes : 0;
  if (eng->lists.bytes < lbytes || eng->sample_bound.bytes < sbytes || eng->cand.bytes < cbytes ||
      eng->scand.bytes < scbytes || eng->cand_cnt.bytes < nbytes || eng->q8_q.bytes < q8qb ||
      eng->q8_par.bytes < q8pb) {
    VS_HIP(hipStreamSynchronize(eng->stream), "sync");
    VS_HIP(eng->lists.ensure(lbytes), "alloc list scratch");
    VS_HIP(eng->sample_bound.ensure(sbytes), "alloc sample bounds");
    VS_HIP(eng->cand.ensure(cbytes), "alloc candidate scratch");
    VS_HIP(eng->scand.ensure(scbytes), "alloc sample tile maxima");
    VS_HIP(eng->cand_cnt.ensure(nbytes), "alloc candidate counts");
    VS_HIP(eng->q8_q.ensure(q8qb), "alloc int8 queries");
    VS_HIP(eng->q8_par.ensure(q8pb), "alloc int8 query bounds");
    // the select's verify ticket (vsk::kQ8ParBytes) starts at zero
    if (q8pb) VS_HIP(hipMemsetAsync(eng->q8_par.p, 0, eng->q8_par.bytes, eng->stream), "zero");
  }
  const void* X = c.data;
  uint64_t* lists = eng->lists.as<uint64_t>();
  float* slabs = eng->cand.as<float>();
  uint32_t* slab_tile = (uint32_t*)((char*)eng->cand.p + slots * 32);
  float* bound = eng->sample_bound.as<float>();
  float* tmax = eng->scand.as<float>();
  uint32_t* cnt = eng->cand_cnt.as<uint32_t>();
  // the quarters' maxima (bf16 / f32 pass: largest admitted score, int8 pass:
  // largest appended dot) beside the counts
  uint32_t* qmax = cnt + (size_t)maxl * PS * 4;
  uint32_t* qmax_sel = select_qmax() ? qmax : nullptr;
  // queries q .. in the collection's dtype: the bf16 copy, or the preprocessed
  // fp32 queries themselves (zero-padded past nq)
  auto qptr = [&](uint32_t q) -> const void* {
    return f32 ? (const void*)(qp + (size_t)q * dim)
               : (const void*)(eng->q_bf16.as<uint16_t>() + (size_t)q * dim);
  };
  if (q8) {
    // int8 pass: up to 256 queries per launch (128 at 1024-d); the sample and
    // bf16 / f32 passes run P queries a launch (fp32 768-d: 128, so two each)
    const uint32_t P8 = vsk::mfma_queries(dim, false);
    int8_t* q8q = eng->q8_q.as<int8_t>();
    float* q8par = eng->q8_par.as<float>();
    uint32_t* gate = (uint32_t*)(q8par + 4 * PS);
    float4* vq = (float4*)((char*)gate + 64);  // the select's verify hand-over
    uint32_t* ticket = (uint32_t*)(vq + PS);
    // Speculative bound (r05): unfiltered batches whose k (or a
    // larger k') this context has seen answered in this generation of the
    // copy start from bound = ratio x |q| instead of a sample pass. The
    // select's answer is exact iff every query's k-th exact score reaches its
    // bound - sigma nmax (q8_verify_record); otherwise the sample path re-runs
    // the whole batch, every launch gated on the verdict word. The ratio's
    // device state decides on the device whether the try runs at all (r06:
    // unset ratio or a cool-down after failed checks -> go = 0, the
    // speculative launches stand down and the sample path answers).
    const bool spec_rec =
        q8_spec_enabled() && !(eng->flags & VS_FLAG_NO_SPECULATIVE) && !allow && k < kQ8SpecK;
    SpecPlan plan;  // spec_k -1: the sample path (vs_spec_host.h)
    plan.record = spec_rec;
    if (spec_rec)
      plan = spec_plan(eng->spec_seen, c.gen, c.q8_gen, k, c.q8_advice, q8_spec_force_fail(),
                       c.spec_host_skips);
    const int spec_k = plan.spec_k;
    const bool record = plan.record;
    // (r06) one speculative launch (the whole batch in one int8 launch) makes
    // the preprocessed queries too; every other batch preprocesses first
    const bool fused_prep = spec_k >= 0 && nq <= P8 && dim <= vsk::kQueryPrepFusedMaxDim;
    if (!fused_prep) {
      const int rc = prep_now();
      if (rc != VS_OK) return rc;
    }
    vsk::Q8SpecK* sk = vsk::q8_spec_k(c.q8_glob);
    vsk::Q8SpecStat* sstat = vsk::q8_spec_stat(c.q8_glob);
    const uint32_t* verdict = gate + vsk::kGateVerdict;
    const uint32_t* go = gate + vsk::kGateGo;
    for (uint32_t q0 = 0; q0 < nq; q0 += P8) {
      const uint32_t nv = std::min(P8, nq - q0);
      uint64_t* out = d_keys + (size_t)q0 * k;
      uint32_t L = 0;
      const uint32_t* run_if = nullptr;  // the sample path below: gated after a speculative try
      if (spec_k >= 0) {
        const float* r_use = &sk[spec_k].ratio;
        const bool force = q8_spec_force_fail();
        if (force) {  // (tests) 0x41414141 = 12.08f, far above any unit-vector score
          VS_HIP(hipMemsetAsync(gate + vsk::kGateForced, 0x41, 4, eng->stream), "forced ratio");
          r_use = (const float*)(gate + vsk::kGateForced);
        }
        if (fused_prep)
          VS_HIP(vsk::launch_q8_prep_query(prep.in, prep.cosine, prep.round_qp, prep.qp, prep.qb, f32,
                                           nv, dim, c.q8_glob, q8q, q8par, gate, eng->stream, r_use,
                                           bound, &sk[k], sstat, force),
                 "query preprocess + int8 queries + speculative bound");
        else
          VS_HIP(vsk::launch_q8_query(qptr(q0), f32, nv, dim, c.q8_glob, q8q, q8par, gate,
                                      eng->stream, r_use, bound, &sk[k], sstat, force),
                 "int8 queries + speculative bound");
        VS_HIP(ev_begin(eng, eng->scan_ev), "event");
        VS_HIP(vsk::launch_mfma_cand_q8(c.q8, dim, n_rows, row_base, q8q, nv, k, bound, q8par,
                                        c.q8_glob, slabs, slab_tile, cap8, cnt, qmax, maxl, &L, gate,
                                        eng->stream, allow, go),
               "int8 scan");
        VS_HIP(ev_end(eng, eng->scan_ev), "event");
        // the check: its own launch (or the select's last workgroup: ablation)
        const vsk::SpecVerifyArgs vchk{1u,    dim,   bound, q8par, c.q8_glob, gate,
                                       &sk[k], sstat, c.q8_advice_dev + k, vq, ticket};
        VS_HIP(ev_begin(eng, eng->merge_ev), "event");
        VS_HIP(vsk::launch_select_q8(slabs, slab_tile, cnt, qmax, L, cap8, nv, k, out, row_base, X,
                                     qptr(q0), f32, dim, q8par, c.q8_glob, c.q8_meta, bound, c.q8,
                                     q8q, allow, n_rows, eng->stream, nullptr, nullptr, go,
                                     q8_sel_verify() ? &vchk : nullptr),
               "int8 select");
        VS_HIP(ev_end(eng, eng->merge_ev), "event");
        if (!q8_sel_verify())
          VS_HIP(vsk::launch_q8_verify_record(out, nv, k, dim, bound, q8par, c.q8_glob, true, gate,
                                              &sk[k], sstat, c.q8_advice_dev + k, eng->stream, go),
                 "speculative bound check");
        run_if = verdict;
      }
      // 1. sample pass(es) -> per-query lower bounds on the k-th score; the
      // first bound launch also makes the batch's int8 queries and zeroes the
      // verdict word (not behind a speculative try: the word is then its verdict)
      for (uint32_t s0 = 0; s0 < nv; s0 += P) {
        const uint32_t ns = std::min(P, nv - s0);
        VS_HIP(vsk::launch_mfma_sample(X, f32, dim, n_rows, row_base, qptr(q0 + s0), ns, k, st,
                                       tmax, maxl, &L, eng->stream, allow, run_if),
               "mfma sample scan");
        if (s0 == 0 && (!q8_prep_apart() || run_if)) {
          VS_HIP(vsk::launch_sample_bound_q8(tmax, L * st, ns, k, bound, qptr(q0), f32, nv, dim,
                                             c.q8_glob, q8q, q8par, run_if ? nullptr : gate,
                                             eng->stream, run_if),
                 "sample bound + int8 queries");
        } else {
          if (s0 == 0)
            VS_HIP(vsk::launch_q8_query(qptr(q0), f32, nv, dim, c.q8_glob, q8q, q8par, gate,
                                        eng->stream),
                   "int8 queries");
          VS_HIP(vsk::launch_sample_bound(tmax, L * st, ns, k, bound + s0, eng->stream, run_if),
                 "sample bound");
        }
      }
      // 2. int8 pass -> bounded candidates -> rescored top k (r05: the select
      // recomputes a quarter the pass overflowed and streams a survivor spill
      // itself; no gated bf16 launches behind it)
      if (!run_if) VS_HIP(ev_begin(eng, eng->scan_ev), "event");
      VS_HIP(vsk::launch_mfma_cand_q8(c.q8, dim, n_rows, row_base, q8q, nv, k, bound, q8par,
                                      c.q8_glob, slabs, slab_tile, cap8, cnt, qmax, maxl, &L, gate,
                                      eng->stream, allow, run_if),
             "int8 scan");
      if (!run_if) VS_HIP(ev_end(eng, eng->scan_ev), "event");
      // the sample path's answer is exact: with `record` it replaces the
      // ratio (its own launch, or the select's last workgroup: ablation)
      const vsk::SpecVerifyArgs vrec{0u,    dim,   bound, q8par, c.q8_glob, nullptr,
                                     &sk[k], sstat, c.q8_advice_dev + k, vq, ticket};
      const bool rec_in_sel = record && q8_sel_verify();
      if (!run_if) VS_HIP(ev_begin(eng, eng->merge_ev), "event");
      VS_HIP(vsk::launch_select_q8(slabs, slab_tile, cnt, qmax, L, cap8, nv, k, out, row_base, X,
                                   qptr(q0), f32, dim, q8par, c.q8_glob, c.q8_meta, bound, c.q8,
                                   q8q, allow, n_rows, eng->stream, nullptr, nullptr, run_if,
                                   rec_in_sel ? &vrec : nullptr),
             "int8 select");
      if (!run_if) VS_HIP(ev_end(eng, eng->merge_ev), "event");
      if (record && !rec_in_sel)
        VS_HIP(vsk::launch_q8_verify_record(out, nv, k, dim, bound, q8par, c.q8_glob, false, nullptr,
                                            &sk[k], sstat, c.q8_advice_dev + k, eng->stream,
                                            run_if),
               "speculative bound record");
    }
    if (spec_rec) spec_seen_mark(plan, k);
    return VS_OK;
  }
  {
    const int rc = prep_now();
    if (rc != VS_OK) return rc;
  }
  for (uint32_t p = 0; p < npass; ++p) {
    const uint32_t q0 = p * P;
    const uint32_t nv = std::min(P, nq - q0);
    uint64_t* out = d_keys + (size_t)q0 * k;
    const void* qb = qptr(q0);
    uint32_t L = 0;
    if (!fast) {
      VS_HIP(ev_begin(eng, eng->scan_ev), "event");
      VS_HIP(vsk::launch_mfma_lists(X, f32, dim, n_rows, row_base, qb, nv, k, nullptr, lists,
                                    maxl, &L, eng->stream, allow),
             "mfma scan (lists)");
      VS_HIP(ev_end(eng, eng->scan_ev), "event");
      VS_HIP(ev_begin(eng, eng->merge_ev), "event");
      VS_HIP(vsk::launch_merge(lists, L, (uint64_t)PS * k, k, nv, k, k, out, eng->stream),
             "merge");
      VS_HIP(ev_end(eng, eng->merge_ev), "event");
      continue;
    }
    // 1. sample pass -> tile maxima -> per-query bound (k-th largest maximum)
    VS_HIP(vsk::launch_mfma_sample(X, f32, dim, n_rows, row_base, qb, nv, k, st, tmax, maxl, &L,
                                   eng->stream, allow),
           "mfma sample scan");
    VS_HIP(vsk::launch_sample_bound(tmax, L * st, nv, k, bound, eng->stream), "sample bound");
    // 2. main pass -> candidates -> select
    VS_HIP(ev_begin(eng, eng->scan_ev), "event");
    VS_HIP(vsk::launch_mfma_cand(X, f32, dim, n_rows, row_base, qb, nv, k, bound, slabs,
                                 slab_tile, cap, cnt, maxl, &L, eng->stream, allow, qmax_sel),
           "mfma scan");
    VS_HIP(ev_end(eng, eng->scan_ev), "event");
    VS_HIP(ev_begin(eng, eng->merge_ev), "event");
    VS_HIP(vsk::launch_select_slabs(slabs, slab_tile, cnt, L, cap, nv, k, out, eng->stream,
                                    row_base, allow, qmax_sel),
           "select");
    VS_HIP(ev_end(eng, eng->merge_ev), "event");
  }
  return VS_OK;
}

int gemv_one();
uint32_t large_k_from();

// One query on the int8 copy (r05; on unless VS_Q8_GEMV=0, read
// once): a collection with an int8 copy streams it instead of its rows, and
// the bracketed survivors are rescored on the GEMV's own arithmetic.
bool q8_gemv_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("VS_Q8_GEMV");
    return !(e && e[0] == '0');
  }();
  return v;
}
bool q8_gemv_path(const Collection& c, uint32_t nq, uint32_t k) {
  return nq == 1 && q8_gemv_enabled() && q8_enabled() && c.q8 && c.q8_cap >= c.rows &&
         c.rows > 0 && c.row_base + c.rows < 0xFFFFFFFFull && vsk::gemv_q8_ok(c.dim, k) &&
         k < large_k_from();
}

bool small_path(const Collection& c, uint32_t nq, uint32_t k, bool filtered) {
  return nq == 1 && !filtered && c.rows > 0 && c.row_base + c.rows < 0xFFFFFFFFull &&
         vsk::gemv_small_ok(c.dim, (uint32_t)c.rows, k);
}

// search_core's one-launch GEMV form takes this unfiltered search (and the
// small path does not): its query may then travel in the kernel arguments
bool gemv_one_path(const Collection& c, uint32_t nq, uint32_t k) {
  return nq == 1 && c.rows > 0 && c.row_base + c.rows < 0xFFFFFFFFull &&
         !small_path(c, nq, k, false) && k < large_k_from() && gemv_one() == 2 &&
         vsk::gemv_one_ok(c.dim, k) && !q8_gemv_path(c, nq, k);
}

// Core search on device data. d_q: nq x dim fp32 on this device, ordered on
// eng->stream. Writes nq x k keys to d_keys. work_mu and the collection's
// reader lock are held by the caller.
int search_core(DevEngine* eng, Collection& c, const float* d_q, uint32_t nq, uint32_t k,
                uint64_t* d_keys, const uint64_t* allow, uint64_t allowed,
                const uint32_t* allow_list, HostDirect* direct) {
  const uint32_t dim = c.dim;
  const bool bf16 = c.dtype == VS_DTYPE_BF16;
  const bool cosine = c.metric == VS_METRIC_COSINE;
  // (r06) VS_FLAG_TIMING_SAMPLE's period: a one-query step (~0.15 ms at C2)
  // pays ~2% for every 4th step's event pair, a batch (~1.8 ms at C3) ~0.2%
  eng->scan_period = nq == 1 ? 16u : 4u;
  if (c.rows == 0) {
    VS_HIP(hipMemsetAsync(d_keys, 0, (size_t)nq * k * 8, eng->stream), "clear keys");
    return VS_OK;
  }
  if (c.rows >= 0xFFFFFFFFull || c.row_base + c.rows >= 0xFFFFFFFFull)
    return fail(VS_ERR_INVALID_ARG, "collection exceeds 2^32-1 rows");
  // one query over a small collection (config C1): prep, scan and merge in
  // one launch (the same keys as the three launches below, bit for bit)
  constexpr size_t kPartBytes = (size_t)vsk::kGemvSmallMaxParts * vsk::kGemvSmallMaxK * 8;
  // the small path's parts + counter, and the one-launch GEMV's counter (the
  // word after it): zeroed once, left zero by the kernels
  auto ensure_counters = [&]() -> int {
    if (eng->small_part.bytes < kPartBytes + 64) {
      VS_HIP(hipStreamSynchronize(eng->stream), "sync");
      VS_HIP(eng->small_part.ensure(kPartBytes + 64), "alloc small-scan parts");
      VS_HIP(hipMemsetAsync(eng->small_part.p, 0, eng->small_part.bytes, eng->stream), "zero");
    }
    return VS_OK;
  };
  if (small_path(c, nq, k, allow != nullptr)) {
    const int rc0 = ensure_counters();
    if (rc0 != VS_OK) return rc0;
    VS_HIP(ev_begin(eng, eng->scan_ev), "event");
    VS_HIP(vsk::launch_gemv_small(c.data, bf16, dim, (uint32_t)c.rows, (uint32_t)c.row_base, d_q,
                                  cosine, k, direct ? direct->keys : d_keys, eng->stream,
                                  eng->small_part.as<uint64_t>(),
                                  (uint32_t*)((char*)eng->small_part.p + kPartBytes),
                                  direct ? direct->flag : nullptr, direct ? direct->seq : 0,
                                  direct ? direct->host_q : nullptr),
           "small scan");
    VS_HIP(ev_end(eng, eng->scan_ev), "event");
    if (direct) direct->used = true;
    return VS_OK;
  }

  // 1. query preprocessing (cosine normalise) -> q_pre (fp32). The fp32
  // MFMA path reads q_pre directly, whole passes of kMfmaQueries rows: rows
  // past nq are padding (zeroed at allocation; later only ever finite
  // queries of earlier calls), masked by the kernels.
  const size_t qbytes = (size_t)((nq + vsk::kMfmaQueries - 1) / vsk::kMfmaQueries) *
                        vsk::kMfmaQueries * dim * 4;
  if (eng->q_pre.bytes < qbytes) {
    VS_HIP(hipStreamSynchronize(eng->stream), "sync");
    VS_HIP(eng->q_pre.ensure(qbytes), "alloc query scratch");
    VS_HIP(hipMemsetAsync(eng->q_pre.p, 0, eng->q_pre.bytes, eng->stream), "zero query scratch");
  }
  float* qp = eng->q_pre.as<float>();
  // batched path: bf16 collections from 2 queries, fp32 ones from 4 (the fp32
  // pass is MFMA-bound at 1/16 of the bf16 rate: ~3 single-query HBM scans)
  bool use_mfma = nq >= (bf16 ? 2u : kF32MfmaMinQueries) && k <= vsk::kMfmaMaxK &&
                  vsk::mfma_supported(dim, !bf16);
  // selective filter: scan only the allowed rows, gathered through a
  // compacted row list (cost ~ allowed rows instead of all rows), one GEMV
  // per query. A batch leaves the MFMA pass for it only while nq gathers
  // (each charged kGatherCallBytes of launch overhead) read less than the
  // one streamed pass.
  const uint64_t rbytes = (uint64_t)dim * (bf16 ? 2 : 4);
  const bool gather = allow && allowed * kGatherDensityDen <= c.rows &&
                      (!use_mfma || (double)nq * (double)(allowed * rbytes + kGatherCallBytes) <=
                                        (double)c.rows * (double)rbytes);
  if (gather) use_mfma = false;
  // one query on the int8 copy (r05): scan + finishing launch, the GEMV's keys
  if (!use_mfma && !gather && q8_gemv_path(c, nq, k)) {
    const int rc0 = ensure_counters();
    if (rc0 != VS_OK) return rc0;
    const size_t sb = vsk::gemv_q8_scratch_bytes((uint32_t)c.rows, k);
    if (eng->q8g.bytes < sb) {
      VS_HIP(hipStreamSynchronize(eng->stream), "sync");
      VS_HIP(eng->q8g.ensure(sb), "alloc int8 single-query scratch");
    }
    uint32_t* ctr = (uint32_t*)((char*)eng->small_part.p + kPartBytes + 8);
    for (int part = 1; part <= 2; ++part) {
      auto& ev = part == 1 ? eng->scan_ev : eng->merge_ev;
      VS_HIP(ev_begin(eng, ev), "event");
      VS_HIP(vsk::launch_gemv_q8(part, c.data, bf16, (const int8_t*)c.q8, c.q8_meta, c.q8_glob,
                                 dim, (uint32_t)c.rows, (uint32_t)c.row_base, d_q, cosine, allow,
                                 k, eng->q8g.p, eng->q8g.bytes, ctr,
                                 direct ? direct->keys : d_keys, eng->stream,
                                 direct ? direct->flag : nullptr, direct ? direct->seq : 0),
             part == 1 ? "int8 single-query scan" : "int8 single-query rescore");
      VS_HIP(ev_end(eng, ev), "event");
    }
    if (direct) direct->used = true;
    return VS_OK;
  }
  // one query on the GEMV list path: query prep, scan and merge in one launch
  // (the last workgroup merges), the answer straight to the host with `direct`
  if (nq == 1 && !use_mfma && !gather && k < large_k_from() && gemv_one() != 0 &&
      vsk::gemv_one_ok(dim, k)) {
    const int rc0 = ensure_counters();
    if (rc0 != VS_OK) return rc0;
    const uint32_t maxl = vsk::gemv_max_lists(dim, bf16, (uint32_t)c.rows, k);
    if (eng->lists.bytes < (size_t)maxl * k * 8) {
      VS_HIP(hipStreamSynchronize(eng->stream), "sync");
      VS_HIP(eng->lists.ensure((size_t)maxl * k * 8), "alloc list scratch");
    }
    const bool fused_merge = gemv_one() == 1;
    uint32_t L = 0;
    VS_HIP(ev_begin(eng, eng->scan_ev), "event");
    VS_HIP(vsk::launch_gemv_one(
               c.data, bf16, dim, (uint32_t)c.rows, (uint32_t)c.row_base, d_q, cosine, allow, k,
               eng->lists.as<uint64_t>(), maxl,
               fused_merge ? (uint32_t*)((char*)eng->small_part.p + kPartBytes + 4) : nullptr,
               direct ? direct->keys : d_keys, eng->stream,
               fused_merge && direct ? direct->flag : nullptr, direct ? direct->seq : 0, &L,
               !fused_merge && direct ? direct->host_q : nullptr),
           "gemv scan (one launch)");
    VS_HIP(ev_end(eng, eng->scan_ev), "event");
    if (!fused_merge) {  // the workgroup lists -> launch_merge (two launches)
      VS_HIP(ev_begin(eng, eng->merge_ev), "event");
      VS_HIP(vsk::launch_merge(eng->lists.as<uint64_t>(), L, k, 0, 1, k, k,
                               direct ? direct->keys : d_keys, eng->stream,
                               direct ? direct->flag : nullptr, direct ? direct->seq : 0),
             "merge");
      VS_HIP(ev_end(eng, eng->merge_ev), "event");
    }
    if (direct) direct->used = true;
    return VS_OK;
  }
  // the bf16 MFMA path reads a bf16 copy, 256 queries per pass (rows past nq
  // are padding: finite, and masked by the kernels)
  uint16_t* qb = nullptr;
  if (use_mfma && bf16) {
    const uint32_t P = vsk::kMfmaQueries;
    const size_t bbytes = (size_t)((nq + P - 1) / P) * P * dim * 2;
    if (eng->q_bf16.bytes < bbytes) {
      VS_HIP(hipStreamSynchronize(eng->stream), "sync");
      VS_HIP(eng->q_bf16.ensure(bbytes), "alloc bf16 query scratch");
      VS_HIP(hipMemsetAsync(eng->q_bf16.p, 0, bbytes, eng->stream), "zero bf16 queries");
    }
    qb = eng->q_bf16.as<uint16_t>();
  }
  // the fp32 copy feeds the GEMV path and the fp32 MFMA path; the bf16 MFMA
  // path needs it only where small collections send k > 16 to the GEMV path
  const bool need_qp = !use_mfma || !bf16 ||
                       (k > vsk::kMfmaListMaxK && vsk::mfma_tiles_per_wg((uint32_t)c.rows) < 8);
  if (use_mfma)  // (r06) it enqueues the preprocessing itself (QPrep)
    return search_mfma(eng, c, qp, nq, k, d_keys, allow,
                       QPrep{d_q, cosine, bf16, need_qp ? qp : nullptr, qb});
  VS_HIP(vsk::launch_query_prep(d_q, nq, dim, cosine, bf16, need_qp ? qp : nullptr, qb,
                                eng->stream),
         "query preprocess");
  // k past the list scans, or past the list path's break-even on a streamed
  // scan (a selective filter's gather reads only its rows: lists up to 1024)
  if (k > vsk::kMaxK || (k >= large_k_from() && !gather))
    return search_large_k(eng, c, qp, nq, k, d_keys, allow, allow ? allowed : c.rows);
  if (gather) {
    if (allowed == 0) {
      VS_HIP(hipMemsetAsync(d_keys, 0, (size_t)nq * k * 8, eng->stream), "clear keys");
      return VS_OK;
    }
    if (!allow_list) {  // not precompacted (vs_filter_create): compact now
      const size_t sc = (size_t)vsk::compact_scratch_words((uint32_t)c.rows) * 4;
      if (eng->gather_rows.bytes < allowed * 4 || eng->gather_cnt.bytes < sc) {
        VS_HIP(hipStreamSynchronize(eng->stream), "sync");
        VS_HIP(eng->gather_rows.ensure(allowed * 4), "alloc gather list");
        VS_HIP(eng->gather_cnt.ensure(sc), "alloc compaction scratch");
      }
      VS_HIP(vsk::launch_compact_rows(allow, (uint32_t)c.rows, eng->gather_rows.as<uint32_t>(),
                                      eng->gather_cnt.as<uint32_t>(), eng->stream),
             "compact filter rows");
      allow_list = eng->gather_rows.as<uint32_t>();
    }
    return search_gemv(eng, c, qp, 0, nq, k, d_keys, nullptr, allow_list, (uint32_t)allowed);
  }
  return search_gemv(eng, c, qp, 0, nq, k, d_keys, allow, nullptr, 0, direct);
}

void decode_host(const uint64_t* keys, uint32_t nq, uint32_t k, float* scores,
                 uint64_t* rows, uint32_t* count, uint32_t ko) {
  if (ko < k) ko = k;
  for (uint32_t i = 0; i < nq; ++i) {
    uint32_t c = 0;
    for (uint32_t j = 0; j < ko; ++j) {
      const uint64_t key = j < k ? keys[(size_t)i * k + j] : 0ull;
      if (key == 0) {
        if (scores) scores[(size_t)i * ko + j] = 0.f;
        if (rows) rows[(size_t)i * ko + j] = 0;
        continue;
      }
      ++c;
      if (scores) scores[(size_t)i * ko + j] = vs::key_score(key);
      if (rows) rows[(size_t)i * ko + j] = vs::key_row(key);
    }
    if (count) count[i] = c;
  }
}


const char* last_error() { return g_last_error.c_str(); }

// Search contexts per device (VS_CONTEXTS, read once; default 2, at most 8).
int contexts_per_device() {
  static const int v = [] {
    const char* e = std::getenv("VS_CONTEXTS");
    const int x = e ? std::atoi(e) : 2;
    return x < 1 ? 1 : (x > 8 ? 8 : x);
  }();
  return v;
}

void close_context(DevEngine* eng) {
  (void)hipStreamSynchronize(eng->stream);
  for (auto& p : eng->scan_ev) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  for (auto& p : eng->merge_ev) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  for (hipEvent_t ev : eng->ev_pool) (void)hipEventDestroy(ev);
  eng->host_slots.clear();
  eng->up.reset();
  (void)hipStreamSynchronize(eng->own);
  if (eng->xev) (void)hipEventDestroy(eng->xev);
  if (eng->own) (void)hipStreamDestroy(eng->own);
  delete eng;
}

int open(int dev, uint32_t flags, DevEngine** out) {
  if (!out) return fail(VS_ERR_INVALID_ARG, "out is NULL");
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0)
    return fail(VS_ERR_DEVICE, "no HIP device available (the engine has no CPU fallback)");
  if (dev < 0) VS_HIP(hipGetDevice(&dev), "hipGetDevice");
  if (dev >= n) return fail(VS_ERR_INVALID_ARG, "device ordinal out of range");
  VS_HIP(hipSetDevice(dev), "hipSetDevice");
  std::string name;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) == hipSuccess)
    name = std::string(prop.name) + " " + prop.gcnArchName;
  auto store = std::make_shared<DevStore>();
  const int nctx = contexts_per_device();
  for (int i = 0; i < nctx; ++i) {
    auto eng = std::make_unique<DevEngine>();
    eng->device = dev;
    eng->flags = flags;
    eng->device_name = name;
    eng->store = store;
    hipError_t he = hipStreamCreateWithFlags(&eng->own, hipStreamNonBlocking);
    if (he == hipSuccess) he = hipEventCreateWithFlags(&eng->xev, hipEventDisableTiming);
    if (he != hipSuccess) {
      const int rc = fail_hip(he, "context stream");
      if (eng->own) (void)hipStreamDestroy(eng->own);
      for (DevEngine* c : store->ctx) close_context(c);
      return rc;
    }
    eng->stream = eng->own;
    store->ctx.push_back(eng.release());
  }
  vsk::device_cu_count();
  *out = store->ctx[0];
  return VS_OK;
}

void close(DevEngine* eng) {
  if (!eng) return;
  (void)hipSetDevice(eng->device);
  std::shared_ptr<DevStore> st = eng->store;
  for (DevEngine* c : st->ctx) (void)hipStreamSynchronize(c->stream);
  {
    std::lock_guard<std::mutex> g(st->filt_mu);
    st->filters.clear();
  }
  {
    std::lock_guard<std::mutex> g(st->map_mu);
    st->colls.clear();
  }
  for (DevEngine* c : st->ctx) close_context(c);
  st->ctx.clear();
}

int collection_create(DevEngine* eng, const char* name, uint32_t dim, int metric, int dtype,
                         uint64_t capacity_hint, uint64_t row_base) {
  if (!eng || !name || !*name) return fail(VS_ERR_INVALID_ARG, "collection name required");
  if (dim == 0 || dim > 65536) return fail(VS_ERR_INVALID_ARG, "dim must be in [1, 65536]");
  if (metric != VS_METRIC_COSINE && metric != VS_METRIC_DOT)
    return fail(VS_ERR_INVALID_ARG, "unknown metric");
  if (dtype != VS_DTYPE_F32 && dtype != VS_DTYPE_BF16)
    return fail(VS_ERR_INVALID_ARG, "unknown dtype");
  VS_HIP(set_dev(eng), "hipSetDevice");
  auto c = std::make_shared<Collection>();
  c->name = name;
  c->gen = g_coll_gen.fetch_add(1);
  c->dim = dim;
  c->metric = metric;
  c->dtype = dtype;
  c->row_base = row_base;
  DevStore& st = *eng->store;
  {
    std::lock_guard<std::mutex> g(st.map_mu);
    if (st.colls.count(name))
      return fail(VS_ERR_EXISTS, std::string("collection ") + name + " already exists");
    st.colls[name] = c;
  }
  if (capacity_hint) {
    std::unique_lock<std::shared_mutex> wl(c->mu);
    std::lock_guard<std::mutex> g(eng->work_mu);
    VS_HIP(use_stream(eng, eng->own), "stream order");
    int rc = grow(eng, *c, capacity_hint);
    if (rc != VS_OK) {
      std::lock_guard<std::mutex> g2(st.map_mu);
      st.colls.erase(name);
      return rc;
    }
  }
  return VS_OK;
}

int collection_info(DevEngine* eng, const char* name, uint32_t* dim, uint64_t* rows,
                       int* metric, int* dtype) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  auto c = find_coll(eng, name);
  if (!c) return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (name ? name : "") +
                                            " not found");
  std::shared_lock<std::shared_mutex> rl(c->mu);
  if (dim) *dim = c->dim;
  if (rows) *rows = c->rows;
  if (metric) *metric = c->metric;
  if (dtype) *dtype = c->dtype;
  return VS_OK;
}

int prefilter_bytes(DevEngine* eng, const char* name, uint64_t* bytes) {
  if (!eng || !bytes) return fail(VS_ERR_INVALID_ARG, "engine and bytes are required");
  auto c = find_coll(eng, name);
  if (!c) return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (name ? name : "") +
                                            " not found");
  std::shared_lock<std::shared_mutex> rl(c->mu);
  *bytes = c->q8 ? (c->q8_cap + kPadRows) * c->dim : 0;
  return VS_OK;
}

// (r06) The speculative bound's counters of a collection (vs_kernels.h
// Q8SpecStat), after every search enqueued so far on this device finished.
int spec_stats(DevEngine* eng, const char* name, uint64_t out[4]) {
  if (!eng || !out) return fail(VS_ERR_INVALID_ARG, "engine and out are required");
  auto c = find_coll(eng, name);
  if (!c) return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (name ? name : "") +
                                            " not found");
  std::shared_lock<std::shared_mutex> rl(c->mu);
  std::memset(out, 0, 4 * sizeof(uint64_t));
  if (!c->q8_glob) return VS_OK;
  VS_HIP(set_dev(eng), "set device");
  VS_HIP(hipDeviceSynchronize(), "sync");
  vsk::Q8SpecStat h{};
  VS_HIP(hipMemcpy(&h, vsk::q8_spec_stat(c->q8_glob), sizeof(h), hipMemcpyDeviceToHost),
         "read speculative-bound counters");
  out[0] = h.tries, out[1] = h.fails;
  out[2] = h.skipped + c->spec_host_skips.load(std::memory_order_relaxed);
  return VS_OK;
}

int collection_drop(DevEngine* eng, const char* name) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  std::shared_ptr<Collection> c;
  DevStore& st = *eng->store;
  {
    std::lock_guard<std::mutex> g(st.map_mu);
    auto it = st.colls.find(name ? name : "");
    if (it == st.colls.end())
      return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (name ? name : "") +
                                        " not found");
    c = it->second;
    st.colls.erase(it);
  }
  std::unique_lock<std::shared_mutex> wl(c->mu);
  std::lock_guard<std::mutex> g(eng->work_mu);
  (void)set_dev(eng);
  VS_HIP(use_stream(eng, eng->own), "stream order");
  (void)hipStreamSynchronize(eng->stream);
  // the collection's resident filters go with it (their HBM, and no later
  // collection of the same name and row count can pick them up)
  std::lock_guard<std::mutex> gf(st.filt_mu);
  for (auto it = st.filters.begin(); it != st.filters.end();)
    it = it->second->coll_gen == c->gen ? st.filters.erase(it) : std::next(it);
  return VS_OK;  // memory released with the last reference
}

// staging chunk: VS_UPSERT_CHUNK_MB (1..64, default 16; 4 / 8 / 32 measured slower) — an ablation knob
size_t upsert_chunk_bytes() {
  static const size_t v = [] {
    const char* e = std::getenv("VS_UPSERT_CHUNK_MB");
    const long mb = e ? std::strtol(e, nullptr, 10) : 16;
    return (size_t)std::min(64L, std::max(1L, mb)) << 20;
  }();
  return v;
}

// memcpy of a large block by up to 4 threads (into pinned staging: one
// core's copy rate, ~10 GB/s, is below what PCIe takes)
void copy_parallel(void* dst, const void* src, size_t bytes) {
  constexpr size_t kSerial = 2ull << 20;
  if (bytes <= kSerial) {
    std::memcpy(dst, src, bytes);
    return;
  }
  const size_t parts = std::min<size_t>(4, bytes / kSerial + 1);
  const size_t step = (bytes / parts + 63) & ~(size_t)63;
  std::vector<std::thread> th;
  for (size_t p = 1; p < parts; ++p) {
    const size_t a = p * step, b = std::min(bytes, a + step);
    if (a < b) th.emplace_back([=] { std::memcpy((char*)dst + a, (const char*)src + a, b - a); });
  }
  std::memcpy(dst, src, std::min(bytes, step));
  for (auto& t : th) t.join();
}

int upsert(DevEngine* eng, const char* coll, uint64_t n, uint32_t dim_in,
              const uint64_t* rows, const float* vecs) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (n == 0) return VS_OK;
  if (!rows || !vecs) return fail(VS_ERR_INVALID_ARG, "rows and vecs are required");
  auto c = find_coll(eng, coll);
  if (!c) return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (coll ? coll : "") +
                                            " not found");
  if (dim_in != c->dim)
    return fail(VS_ERR_DIM_MISMATCH, "Vector dimension error: expected dim: " +
                                         std::to_string(c->dim) + ", got " + std::to_string(dim_in));
  std::unique_lock<std::shared_mutex> wl(c->mu);
  // Rows in strictly ascending order (an ingest appending its points, a bulk
  // load) are taken as they are; otherwise the last occurrence of each row
  // wins, in row order.
  bool ascending = true;
  for (uint64_t i = 1; i < n && ascending; ++i) ascending = rows[i - 1] < rows[i];
  std::vector<std::pair<uint64_t, uint64_t>> order;  // (row, index), sorted
  std::vector<uint64_t> keep_idx;
  if (!ascending) {
    order.resize(n);
    for (uint64_t i = 0; i < n; ++i) order[i] = {rows[i], i};
    std::stable_sort(order.begin(), order.end(),
                     [](const auto& a, const auto& b) { return a.first < b.first; });
    keep_idx.reserve(n);
    for (uint64_t i = 0; i < n; ++i)
      if (i + 1 == n || order[i + 1].first != order[i].first) keep_idx.push_back(i);
  }
  const uint64_t m = ascending ? n : keep_idx.size();
  auto row_of = [&](uint64_t t) { return ascending ? rows[t] : order[keep_idx[t]].first; };
  auto src_of = [&](uint64_t t) { return ascending ? t : order[keep_idx[t]].second; };
  // appended rows must be exactly [rows, rows + m')
  uint64_t expect = c->rows;
  for (uint64_t t = 0; t < m; ++t) {
    const uint64_t r = row_of(t);
    if (r >= c->rows) {
      if (r != expect)
        return fail(VS_ERR_INVALID_ARG, "upsert would leave a hole: appended rows must be "
                                        "contiguous from the current row count");
      ++expect;
    }
  }
  if (expect >= 0xFFFFFFFFull) return fail(VS_ERR_INVALID_ARG, "too many rows");
  std::lock_guard<std::mutex> g(eng->work_mu);
  VS_HIP(set_dev(eng), "hipSetDevice");
  VS_HIP(use_stream(eng, eng->own), "stream order");
  int rc = grow(eng, *c, expect);
  if (rc != VS_OK) return rc;
  const uint32_t dim = c->dim;
  const size_t rb = (size_t)dim * 4;
  // chunks of <= 16 MiB of fp32 vectors + rows, double-buffered through pinned
  // memory: the host fills chunk i+1 while chunk i crosses PCIe and the
  // device normalises it (vsk::launch_preprocess, HBM-bound)
  const uint64_t per =
      std::min<uint64_t>(m, std::max<uint64_t>(1, upsert_chunk_bytes() / (rb + 8)));
  if (!eng->up) eng->up = std::make_unique<UpsertStage>();
  UpsertStage& stg = *eng->up;
  VS_HIP(stg.ensure(per * rb + per * 8), "alloc pinned upsert staging");
  for (int j = 0; j < 2; ++j) {
    VS_HIP(stg.vecs[j].ensure(per * rb), "alloc upsert scratch");
    VS_HIP(stg.rows[j].ensure(per * 8), "alloc upsert scratch");
  }
  int j = 0;
  for (uint64_t o = 0; o < m; o += per, j ^= 1) {
    const uint64_t cnt = std::min(per, m - o);
    if (stg.armed[j]) VS_HIP(hipEventSynchronize(stg.done[j]), "upsert staging");
    float* hv = (float*)stg.pin[j];
    uint64_t* hr = (uint64_t*)((char*)stg.pin[j] + per * rb);
    if (ascending) {
      copy_parallel(hv, vecs + o * dim, cnt * rb);
      std::memcpy(hr, rows + o, cnt * 8);
    } else {
      for (uint64_t t = 0; t < cnt; ++t) {
        hr[t] = row_of(o + t);
        std::memcpy(&hv[t * dim], vecs + src_of(o + t) * dim, rb);
      }
    }
    VS_HIP(hipMemcpyAsync(stg.vecs[j].p, hv, cnt * rb, hipMemcpyHostToDevice, eng->stream),
           "upsert H2D");
    VS_HIP(hipMemcpyAsync(stg.rows[j].p, hr, cnt * 8, hipMemcpyHostToDevice, eng->stream),
           "upsert H2D");
    VS_HIP(hipEventRecord(stg.done[j], eng->stream), "upsert staging");
    stg.armed[j] = true;
    VS_HIP(vsk::launch_preprocess(stg.vecs[j].as<float>(), (uint32_t)cnt, dim,
                                  c->metric == VS_METRIC_COSINE, c->dtype == VS_DTYPE_BF16,
                                  c->data, stg.rows[j].as<uint64_t>(), 0, eng->stream),
           "upsert preprocess");
  }
  c->rows = expect;
  // the tile list outlives the final synchronize: its H2D copy reads pageable
  // memory, which HIP may still be consuming after hipMemcpyAsync returns
  std::vector<uint32_t> tl;
  if (q8_wanted(eng, *c)) {
    // the tiles this call wrote: one range for dense ascending rows (an
    // append), else the distinct tiles of the (row-sorted) kept rows
    const uint64_t span = ascending ? rows[n - 1] / 32 - rows[0] / 32 + 1 : 0;
    if (ascending && span <= n / 16 + 64) {
      rc = q8_after_write(eng, *c, rows[0], rows[n - 1] + 1);
    } else {
      for (uint64_t t = 0; t < m; ++t) {
        const uint32_t ti = (uint32_t)(row_of(t) / 32);
        if (tl.empty() || tl.back() != ti) tl.push_back(ti);
      }
      hipError_t e = hipStreamSynchronize(eng->stream);  // q8_tiles is free
      if (e == hipSuccess) e = eng->q8_tiles.ensure(tl.size() * 4);
      if (e == hipSuccess)
        e = hipMemcpyAsync(eng->q8_tiles.p, tl.data(), tl.size() * 4, hipMemcpyHostToDevice,
                           eng->stream);
      rc = e != hipSuccess ? fail_hip(e, "int8 copy: tile list")
                           : q8_after_write(eng, *c, 0, 0, eng->q8_tiles.as<uint32_t>(),
                                            (uint32_t)tl.size());
      if (rc != VS_OK && c->q8) {  // the rows are written; the copy is now stale
        (void)hipStreamSynchronize(eng->stream);
        c->q8_free();
      }
    }
    if (rc != VS_OK) return rc;
  }
  VS_HIP(hipStreamSynchronize(eng->stream), "upsert sync");
  return VS_OK;
}

int generate(DevEngine* eng, const char* coll, uint64_t n, uint64_t seed, uint64_t g0,
             uint64_t stride) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  auto c = find_coll(eng, coll);
  if (!c) return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (coll ? coll : "") +
                                            " not found");
  if (n == 0) return VS_OK;
  std::unique_lock<std::shared_mutex> wl(c->mu);
  if (c->rows + n >= 0xFFFFFFFFull) return fail(VS_ERR_INVALID_ARG, "too many rows");
  std::lock_guard<std::mutex> g(eng->work_mu);
  VS_HIP(set_dev(eng), "hipSetDevice");
  VS_HIP(use_stream(eng, eng->own), "stream order");
  int rc = grow(eng, *c, c->rows + n);
  if (rc != VS_OK) return rc;
  // g0 == UINT64_MAX: the collection's own next global rows (row_base + rows)
  if (g0 == UINT64_MAX) g0 = c->row_base + c->rows, stride = 1;
  VS_HIP(vsk::launch_generate(seed, g0, n, c->dim, c->dtype == VS_DTYPE_BF16, c->data, c->rows,
                              eng->stream, stride),
         "generate");
  c->rows += n;
  rc = q8_after_write(eng, *c, c->rows - n, c->rows);
  if (rc != VS_OK) return rc;
  VS_HIP(hipStreamSynchronize(eng->stream), "generate sync");
  return VS_OK;
}

int generate_vectors(DevEngine* eng, uint64_t seed, uint64_t row0, uint64_t n, uint32_t dim,
                        float* d_out, void* stream) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (n == 0) return VS_OK;
  if (!d_out || dim == 0) return fail(VS_ERR_INVALID_ARG, "bad output buffer");
  VS_HIP(set_dev(eng), "hipSetDevice");
  VS_HIP(vsk::launch_generate(seed, row0, n, dim, false, d_out, 0, (hipStream_t)stream),
         "generate vectors");
  return VS_OK;
}

int read_rows(DevEngine* eng, const char* coll, uint64_t first, uint64_t n, float* out) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  auto c = find_coll(eng, coll);
  if (!c) return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (coll ? coll : "") +
                                            " not found");
  std::shared_lock<std::shared_mutex> rl(c->mu);
  if (first + n > c->rows || first + n < first)
    return fail(VS_ERR_INVALID_ARG, "row range out of bounds");
  if (n == 0) return VS_OK;
  if (!out) return fail(VS_ERR_INVALID_ARG, "out is NULL");
  std::lock_guard<std::mutex> g(eng->work_mu);
  VS_HIP(set_dev(eng), "hipSetDevice");
  VS_HIP(use_stream(eng, eng->own), "stream order");
  const size_t count = (size_t)n * c->dim;
  if (c->dtype == VS_DTYPE_F32) {
    VS_HIP(hipMemcpyAsync(out, (const char*)c->data + first * c->row_bytes(), count * 4,
                          hipMemcpyDeviceToHost, eng->stream),
           "read D2H");
    VS_HIP(hipStreamSynchronize(eng->stream), "read sync");
  } else {
    std::vector<uint16_t> tmp(count);
    VS_HIP(hipMemcpyAsync(tmp.data(), (const char*)c->data + first * c->row_bytes(), count * 2,
                          hipMemcpyDeviceToHost, eng->stream),
           "read D2H");
    VS_HIP(hipStreamSynchronize(eng->stream), "read sync");
    for (size_t i = 0; i < count; ++i) out[i] = vs::bf16_to_f32(tmp[i]);
  }
  return VS_OK;
}

// Stored rows [first, first + n) as stored (bf16 / fp32 bytes) -> host.
int read_raw(DevEngine* eng, const char* coll, uint64_t first, uint64_t n, void* out) {
  auto c = find_coll(eng, coll);
  if (!c) return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (coll ? coll : "") +
                                            " not found");
  std::shared_lock<std::shared_mutex> rl(c->mu);
  if (first + n > c->rows || first + n < first)
    return fail(VS_ERR_INVALID_ARG, "row range out of bounds");
  if (n == 0) return VS_OK;
  std::lock_guard<std::mutex> g(eng->work_mu);
  VS_HIP(set_dev(eng), "hipSetDevice");
  VS_HIP(use_stream(eng, eng->own), "stream order");
  VS_HIP(hipMemcpyAsync(out, (const char*)c->data + first * c->row_bytes(), n * c->row_bytes(),
                        hipMemcpyDeviceToHost, eng->stream),
         "read D2H");
  VS_HIP(hipStreamSynchronize(eng->stream), "read sync");
  return VS_OK;
}

// Appends n rows given exactly as stored (no preprocessing): restore path.
int append_raw(DevEngine* eng, const char* coll, uint64_t n, const void* rows) {
  auto c = find_coll(eng, coll);
  if (!c) return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (coll ? coll : "") +
                                            " not found");
  if (n == 0) return VS_OK;
  std::unique_lock<std::shared_mutex> wl(c->mu);
  if (c->rows + n >= 0xFFFFFFFFull) return fail(VS_ERR_INVALID_ARG, "too many rows");
  std::lock_guard<std::mutex> g(eng->work_mu);
  VS_HIP(set_dev(eng), "hipSetDevice");
  VS_HIP(use_stream(eng, eng->own), "stream order");
  int rc = grow(eng, *c, c->rows + n);
  if (rc != VS_OK) return rc;
  VS_HIP(hipMemcpyAsync((char*)c->data + c->rows * c->row_bytes(), rows, n * c->row_bytes(),
                        hipMemcpyHostToDevice, eng->stream),
         "restore H2D");
  c->rows += n;
  rc = q8_after_write(eng, *c, c->rows - n, c->rows);
  if (rc != VS_OK) return rc;
  VS_HIP(hipStreamSynchronize(eng->stream), "restore sync");
  return VS_OK;
}

// Checksum contribution of one shard of a row-striped collection
// (vsk::launch_checksum_rows); the collection's checksum is the sum.
int checksum_shard(DevEngine* eng, const char* coll, uint64_t stride, uint64_t offset,
                   uint64_t* out) {
  auto c = find_coll(eng, coll);
  if (!c) return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (coll ? coll : "") +
                                            " not found");
  std::shared_lock<std::shared_mutex> rl(c->mu);
  if (c->row_bytes() % 8)
    return fail(VS_ERR_INVALID_ARG, "a sharded collection's checksum needs rows of whole "
                                    "8-byte words (bf16: dim % 4 == 0, fp32: dim % 2 == 0)");
  std::lock_guard<std::mutex> g(eng->work_mu);
  VS_HIP(set_dev(eng), "hipSetDevice");
  VS_HIP(use_stream(eng, eng->own), "stream order");
  VS_HIP(eng->scratch8.ensure(8), "alloc checksum");
  VS_HIP(vsk::launch_checksum_rows(c->data, c->rows, (uint32_t)c->row_bytes(), stride, offset,
                                   eng->scratch8.as<uint64_t>(), eng->stream),
         "checksum");
  VS_HIP(hipMemcpyAsync(out, eng->scratch8.p, 8, hipMemcpyDeviceToHost, eng->stream),
         "checksum D2H");
  VS_HIP(hipStreamSynchronize(eng->stream), "checksum sync");
  return VS_OK;
}

// vs_search / vs_search_filtered: host queries in, host results out.
// Popcount of the bitmap over the collection's rows (on the host, which holds
// the bitmap: 156k words at 10M rows). The build targets baseline x86-64, where
// __builtin_popcountll is a bit-trick sequence; the POPCNT instruction is
// used when the CPU has it.
static uint64_t popcount_words_sw(const uint64_t* allow, uint64_t nw) {
  uint64_t allowed = 0;
  for (uint64_t i = 0; i < nw; ++i) allowed += (uint64_t)__builtin_popcountll(allow[i]);
  return allowed;
}
__attribute__((target("popcnt"))) static uint64_t popcount_words_hw(const uint64_t* allow,
                                                                     uint64_t nw) {
  uint64_t allowed = 0;
  for (uint64_t i = 0; i < nw; ++i) allowed += (uint64_t)__builtin_popcountll(allow[i]);
  return allowed;
}

uint64_t popcount_rows(const uint64_t* allow, uint64_t rows) {
  const uint64_t nw = (rows + 63) / 64;
  if (nw == 0) return 0;
  static const bool hw = __builtin_cpu_supports("popcnt");
  const uint64_t allowed = hw ? popcount_words_hw(allow, nw - 1) : popcount_words_sw(allow, nw - 1);
  uint64_t w = allow[nw - 1];
  if (rows & 63) w &= (1ull << (rows & 63)) - 1;
  return allowed + (uint64_t)__builtin_popcountll(w);
}

// Waits for a search's completion event: polled for up to kSpinUs (a small
// collection's search completes within tens of microseconds, and a blocking
// wait adds the thread's wake-up to its latency), then a blocking wait (a
// long scan does not keep a host core busy).
// VS_SPIN_US overrides the 60 us (read once; 0 = block at once).
int64_t spin_us() {
  static const int64_t v = [] {
    const char* e = std::getenv("VS_SPIN_US");
    return e ? (int64_t)std::atoll(e) : (int64_t)60;
  }();
  return v;
}
hipError_t wait_event(hipEvent_t ev) {
  const int64_t lim = spin_us();
  const auto t0 = std::chrono::steady_clock::now();
  while (lim > 0) {
    const hipError_t q = hipEventQuery(ev);
    if (q != hipErrorNotReady) return q;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(lim)) break;
  }
  return hipEventSynchronize(ev);
}

// One HIP runtime per process (r04). torch's ROCm wheel ships its own
// libamdhip64.so and links it by file name, while this library links
// libamdhip64.so.7 by soname: when this library is loaded first, importing
// torch later maps a SECOND runtime (and HSA runtime) into the process. The
// two have separate null streams and queues with no ordering between them, so
// a device-pointer search on "torch's stream" is not ordered with torch's own
// work at all: the round-3 driver run read a query's keys before the select
// kernel had written them (tests/test_placement_gpu.py). Device-pointer entry
// points refuse to run in such a process instead of racing. The scan is a
// dl_iterate_phdr walk, repeated only when the loader's add/remove counters
// moved since the last one.
namespace {
struct RtScan {
  unsigned long long adds = 0, subs = 0;
  bool probe = true;  // the first callback only reads the loader's counters
  std::vector<std::string> paths;
};
int rt_visit(struct dl_phdr_info* info, size_t, void* p) {
  RtScan& s = *(RtScan*)p;
  if (s.probe) {
    s.adds = info->dlpi_adds;
    s.subs = info->dlpi_subs;
    return 1;
  }
  const char* n = info->dlpi_name ? info->dlpi_name : "";
  const char* b = std::strrchr(n, '/');
  b = b ? b + 1 : n;
  if (std::strncmp(b, "libamdhip64.so", 14) == 0) s.paths.emplace_back(n);
  return 0;
}
}  // namespace

int one_hip_runtime() {
  static std::mutex mu;
  static unsigned long long seen_adds = ~0ull, seen_subs = ~0ull;
  static std::string problem;
  RtScan s;
  dl_iterate_phdr(rt_visit, &s);
  std::lock_guard<std::mutex> g(mu);
  if (s.adds != seen_adds || s.subs != seen_subs) {
    RtScan full;
    full.probe = false;
    dl_iterate_phdr(rt_visit, &full);
    problem.clear();
    if (full.paths.size() > 1)
      problem = "two HIP runtimes are loaded in this process (" + full.paths[0] + " and " +
                full.paths[1] +
                "): device pointers and streams of one are not ordered with the other's work; "
                "load one runtime (import torch before libvsearch, engine.load_library does)";
    seen_adds = s.adds;
    seen_subs = s.subs;
  }
  return problem.empty() ? VS_OK : fail(VS_ERR_DEVICE, problem);
}

// Spins on a completion word in mapped host memory for up to spin_us(): true
// once it holds seq.
bool wait_word(const uint64_t* w, uint64_t seq) {
  const int64_t lim = spin_us();
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 0;; ++i) {
    if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == seq) return true;
    if ((i & 63) == 63 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(lim))
      return false;
  }
}

// The small path's host completion word (on unless VS_DIRECT_COMPLETION=0;
// read once): the D2H copy + event it replaces cost ~6 us of C1's round trip.
bool direct_completion() {
  static const bool v = [] {
    const char* e = std::getenv("VS_DIRECT_COMPLETION");
    return !(e && e[0] == '0');
  }();
  return v;
}

// One-query GEMV searches with the query prep fused into the scan
// (VS_GEMV_ONE, read once): 2 (default) = prep + scan in one launch, then
// the merge; 1 = the merge too, by the last workgroup; 0 = prep, scan and
// merge as three launches.
int gemv_one() {
  static const int v = [] {
    const char* e = std::getenv("VS_GEMV_ONE");
    return e ? std::atoi(e) : 2;
  }();
  return v;
}

// The small path's query in the kernel arguments (on unless VS_QUERY_ARGS=0;
// read once): no H2D copy for one-query calls on small collections.
bool query_args() {
  static const bool v = [] {
    const char* e = std::getenv("VS_QUERY_ARGS");
    return !(e && e[0] == '0');
  }();
  return v;
}

// The same for the one-launch GEMV form (on unless VS_QUERY_ARGS_GEMV=0;
// read once): one query at 2k / 20k / 200k rows 31.0 / 41.0 / 127.5 ->
// 27.9 / 37.0 / 123.8 us (profiles/r03_query_args_gemv_ab.jsonl).
bool query_args_gemv() {
  static const bool v = [] {
    const char* e = std::getenv("VS_QUERY_ARGS_GEMV");
    return !(e && e[0] == '0');
  }();
  return v;
}

// A batched search of a large collection (the MFMA passes fill every CU for
// milliseconds): such calls queue behind each other on the primary context,
// so two of them never split the device and the batcher's pipelining (the
// next batch formed as the running one ends) keeps its batches whole. C5,
// 3 x 5M x 1024: two batched calls on two streams cut the mean batch at 64
// clients from 21 to 16 and QPS by 20% (profiles/r03_c5_contexts_*.jsonl).
bool heavy_search(const Collection& c, uint32_t nq) {
  return nq >= 2 && c.rows * c.row_bytes() >= kHeavyBytes;
}

int search_host(DevEngine* eng, const char* coll, const float* queries, uint32_t nq,
                uint32_t dim, uint32_t k, const uint64_t* allow, uint64_t allow_words,
                float* out_scores, uint64_t* out_rows, uint32_t* out_count,
                uint64_t filter_id) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (k == 0) return fail(VS_ERR_INVALID_ARG, "k must be at least 1");
  if (nq == 0) return VS_OK;
  if (!queries) return fail(VS_ERR_INVALID_ARG, "queries is NULL");
  auto c = find_coll(eng, coll);
  if (!c) return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (coll ? coll : "") +
                                            " not found");
  if (dim != c->dim)
    return fail(VS_ERR_DIM_MISMATCH, "Vector dimension error: expected dim: " +
                                         std::to_string(c->dim) + ", got " + std::to_string(dim));
  std::shared_lock<std::shared_mutex> rl(c->mu);
  if (allow && allow_words < (c->rows + 63) / 64)
    return fail(VS_ERR_INVALID_ARG, "filter bitmap has " + std::to_string(allow_words) +
                                        " words, the collection needs " +
                                        std::to_string((c->rows + 63) / 64));
  // a limit past the collection returns every row, as Qdrant does: search
  // (and size the keys, staging and sort scratch) for min(k, rows); the
  // caller's outputs keep their stride k, zero past the rows
  const uint32_t ko = k;
  k = (uint32_t)std::min<uint64_t>(k, std::max<uint64_t>(c->rows, 1));
  // the filter stays referenced until the device is done with it (a
  // concurrent vs_filter_drop only unlinks it)
  std::shared_ptr<DevFilter> df;
  if (filter_id) {
    df = find_filter(eng, filter_id);
    if (!df) return fail(VS_ERR_NOT_FOUND, "filter " + std::to_string(filter_id) + " not found");
    if (df->coll_gen != c->gen || df->rows != c->rows)
      return fail(VS_ERR_INVALID_ARG, "filter " + std::to_string(filter_id) +
                                          " was built for another collection state");
  }
  // a search context of the device: an idle one if any, so concurrent host
  // searches run on separate streams (and overlap on the device)
  std::unique_lock<std::mutex> g;
  DevEngine* cx = pick_context(eng, &g, heavy_search(*c, nq));
  cx->inflight.fetch_add(1, std::memory_order_relaxed);
  struct Leave {
    DevEngine* cx;
    ~Leave() { cx->inflight.fetch_sub(1, std::memory_order_relaxed); }
  } leave{cx};
  VS_HIP(set_dev(cx), "hipSetDevice");
  VS_HIP(use_stream(cx, cx->own), "stream order");
  const size_t qbytes = (size_t)nq * c->dim * 4;
  const size_t kbytes = (size_t)nq * k * 8;
  const size_t abytes = allow ? (size_t)((c->rows + 63) / 64) * 8 : 0;
  if (cx->q_in.bytes < qbytes || cx->keys.bytes < kbytes || cx->allow.bytes < abytes) {
    VS_HIP(hipStreamSynchronize(cx->stream), "sync");
    VS_HIP(cx->q_in.ensure(qbytes), "alloc query input");
    VS_HIP(cx->keys.ensure(kbytes), "alloc keys");
    VS_HIP(cx->allow.ensure(abytes), "alloc filter bitmap");
  }
  // an idle pinned staging slot (one per call in flight on this context)
  HostSlot* hs = nullptr;
  for (auto& x : cx->host_slots)
    if (!x->busy) {
      hs = x.get();
      break;
    }
  if (!hs) {
    cx->host_slots.push_back(std::make_unique<HostSlot>());
    hs = cx->host_slots.back().get();
  }
  VS_HIP(hs->ensure(qbytes, kbytes), "alloc pinned staging");
  // a call the one-launch small path takes writes its keys and a completion
  // word straight to the slot's mapped buffer; its query travels in the
  // kernel arguments (dim <= kGemvSmallArgDim: no H2D at all)
  const bool direct = nq == 1 && !abytes && !df && k <= vsk::kMaxK && direct_completion();
  const bool qarg = direct &&
                    (small_path(*c, nq, k, false) || (query_args_gemv() && gemv_one_path(*c, nq, k))) &&
                    c->dim <= vsk::kGemvSmallArgDim && query_args();
  if (!qarg) std::memcpy(hs->in, queries, qbytes);
  // busy from the first enqueue that reads the slot: a failure after it
  // drains the stream before the slot is released (a queued H2D may still
  // read hs->in, a queued D2H write hs->out)
  hs->busy = true;
  auto abandon = [&](int rc) {
    (void)hipStreamSynchronize(cx->stream);
    hs->busy = false;
    return rc;
  };
  hipError_t e = hipSuccess;
  if (!qarg) e = hipMemcpyAsync(cx->q_in.p, hs->in, qbytes, hipMemcpyHostToDevice, cx->stream);
  if (e != hipSuccess) return abandon(fail_hip(e, "query H2D"));
  if (abytes) {  // pageable: HIP stages it (a shipped-bitmap call, not the batcher's path)
    e = hipMemcpyAsync(cx->allow.p, allow, abytes, hipMemcpyHostToDevice, cx->stream);
    if (e != hipSuccess) return abandon(fail_hip(e, "filter bitmap H2D"));
  }
  HostDirect hd;
  HostDirect* hdp = nullptr;
  if (direct) {
    e = hs->ensure_mapped(vsk::kMaxK + 1);
    if (e != hipSuccess) return abandon(fail_hip(e, "alloc mapped completion"));
    hd.keys = hs->mapped_dev;
    hd.flag = hs->mapped_dev + vsk::kMaxK;
    hd.seq = ++hs->seq;
    hd.host_q = qarg ? queries : nullptr;
    hdp = &hd;
  }
  int rc;
  if (df)
    rc = search_core(cx, *c, cx->q_in.as<float>(), nq, k, cx->keys.as<uint64_t>(),
                     df->bits.as<uint64_t>(), df->allowed,
                     df->list.p ? df->list.as<uint32_t>() : nullptr);
  else
    rc = search_core(cx, *c, cx->q_in.as<float>(), nq, k, cx->keys.as<uint64_t>(),
                     abytes ? cx->allow.as<uint64_t>() : nullptr,
                     abytes ? popcount_rows(allow, c->rows) : 0, nullptr, hdp);
  if (rc != VS_OK) return abandon(rc);
  if (qarg && !hd.used) return abandon(fail(VS_ERR_INTERNAL, "small path not taken"));
  if (!hd.used) e = hipMemcpyAsync(hs->out, cx->keys.p, kbytes, hipMemcpyDeviceToHost, cx->stream);
  if (e == hipSuccess) e = hipEventRecord(hs->done, cx->stream);
  if (e != hipSuccess) return abandon(fail_hip(e, "keys D2H"));
  // wait for the device outside work_mu: the next call on this context (its
  // q_in, keys and scratch are ordered on its stream) enqueues behind this one
  g.unlock();
  hipError_t we = hipSuccess;
  if (hd.used) {
    // the kernel's completion word: its keys are in place once it reads seq
    // (the H2D that read hs->in ran before the kernel; nothing after the
    // kernel touches the slot). Past the spin limit, the stream's event.
    const uint64_t* word = hs->mapped + vsk::kMaxK;
    if (!wait_word(word, hd.seq)) {
      we = hipEventSynchronize(hs->done);
      if (we == hipSuccess && __atomic_load_n(word, __ATOMIC_ACQUIRE) != hd.seq)
        we = hipErrorLaunchFailure;  // the stream completed without the word
    }
    if (we == hipSuccess) decode_host(hs->mapped, nq, k, out_scores, out_rows, out_count, ko);
  } else {
    we = wait_event(hs->done);
    if (we == hipSuccess) decode_host((const uint64_t*)hs->out, nq, k, out_scores, out_rows, out_count, ko);
  }
  g.lock();
  hs->busy = false;
  VS_HIP(we, "search sync");
  return VS_OK;
}

int filter_create(DevEngine* eng, const char* coll, const uint64_t* allow,
                     uint64_t allow_words, uint64_t* filter_id) {
  if (!eng || !allow || !filter_id) return fail(VS_ERR_INVALID_ARG, "NULL argument");
  auto c = find_coll(eng, coll);
  if (!c) return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (coll ? coll : "") +
                                            " not found");
  std::shared_lock<std::shared_mutex> rl(c->mu);
  const uint64_t nw = (c->rows + 63) / 64;
  if (allow_words < nw)
    return fail(VS_ERR_INVALID_ARG, "filter bitmap has " + std::to_string(allow_words) +
                                        " words, the collection needs " + std::to_string(nw));
  if (c->rows >= 0xFFFFFFFFull) return fail(VS_ERR_INVALID_ARG, "collection exceeds 2^32-1 rows");
  std::lock_guard<std::mutex> g(eng->work_mu);
  VS_HIP(set_dev(eng), "hipSetDevice");
  VS_HIP(use_stream(eng, eng->own), "stream order");
  auto f = std::make_shared<DevFilter>();
  f->coll = coll;
  f->coll_gen = c->gen;
  f->rows = c->rows;
  f->allowed = popcount_rows(allow, c->rows);
  VS_HIP(f->bits.ensure(std::max<uint64_t>(nw, 1) * 8), "alloc filter bitmap");
  if (nw)
    VS_HIP(hipMemcpyAsync(f->bits.p, allow, nw * 8, hipMemcpyHostToDevice, eng->stream),
           "filter bitmap H2D");
  // selective: keep the compacted row list too (search_core's gather path)
  if (f->allowed && f->allowed * kGatherDensityDen <= c->rows) {
    VS_HIP(f->list.ensure(f->allowed * 4), "alloc filter row list");
    const size_t sc = (size_t)vsk::compact_scratch_words((uint32_t)c->rows) * 4;
    if (eng->gather_cnt.bytes < sc) {
      VS_HIP(hipStreamSynchronize(eng->stream), "sync");
      VS_HIP(eng->gather_cnt.ensure(sc), "alloc compaction scratch");
    }
    VS_HIP(vsk::launch_compact_rows(f->bits.as<uint64_t>(), (uint32_t)c->rows,
                                    f->list.as<uint32_t>(), eng->gather_cnt.as<uint32_t>(),
                                    eng->stream),
           "compact filter rows");
  }
  VS_HIP(hipStreamSynchronize(eng->stream), "filter sync");  // ready for every context
  DevStore& st = *eng->store;
  std::lock_guard<std::mutex> gf(st.filt_mu);
  *filter_id = st.next_filter++;
  st.filters.emplace(*filter_id, std::move(f));
  return VS_OK;
}

int filter_drop(DevEngine* eng, uint64_t filter_id) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  std::shared_ptr<DevFilter> f;  // freed here unless a search still holds it
  {
    DevStore& st = *eng->store;
    std::lock_guard<std::mutex> gf(st.filt_mu);
    auto it = st.filters.find(filter_id);
    if (it == st.filters.end())
      return fail(VS_ERR_NOT_FOUND, "filter " + std::to_string(filter_id) + " not found");
    f = std::move(it->second);
    st.filters.erase(it);
  }
  if (f.use_count() == 1) {  // the primary's device-pointer searches may still read it
    std::lock_guard<std::mutex> g(eng->work_mu);
    VS_HIP(set_dev(eng), "hipSetDevice");
    VS_HIP(hipStreamSynchronize(eng->stream), "sync");
  }
  return VS_OK;
}

int search_keys(DevEngine* eng, const char* coll, const float* d_queries, uint32_t nq,
                   uint32_t dim, uint32_t k, uint64_t* d_keys, void* stream) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (k == 0) return fail(VS_ERR_INVALID_ARG, "k must be at least 1");
  if (nq == 0) return VS_OK;
  if (!d_queries || !d_keys) return fail(VS_ERR_INVALID_ARG, "NULL device pointer");
  auto c = find_coll(eng, coll);
  if (!c) return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (coll ? coll : "") +
                                            " not found");
  if (dim != c->dim)
    return fail(VS_ERR_DIM_MISMATCH, "Vector dimension error: expected dim: " +
                                         std::to_string(c->dim) + ", got " + std::to_string(dim));
  std::shared_lock<std::shared_mutex> rl(c->mu);
  std::lock_guard<std::mutex> g(eng->work_mu);
  VS_HIP(set_dev(eng), "hipSetDevice");
  // enqueue on the caller's stream (ordered after the engine's previous work)
  VS_HIP(use_stream(eng, (hipStream_t)stream), "stream order");
  return search_core(eng, *c, d_queries, nq, k, d_keys);
}

int merge_keys(DevEngine* eng, const uint64_t* d_lists, uint32_t n_lists, uint32_t nq,
                  uint32_t k_in, uint32_t k, uint64_t* d_out_keys, void* stream) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (k == 0 || k_in == 0 || n_lists == 0) return fail(VS_ERR_INVALID_ARG, "bad merge shape");
  if (nq == 0) return VS_OK;
  if (!d_lists || !d_out_keys) return fail(VS_ERR_INVALID_ARG, "NULL device pointer");
  std::lock_guard<std::mutex> g(eng->work_mu);
  VS_HIP(set_dev(eng), "hipSetDevice");
  hipStream_t cs = (hipStream_t)stream;
  if (k <= vsk::kMaxK && k_in <= vsk::kMaxK) {
    // the list merge has no scratch of its own: it runs directly on the caller's stream
    hipError_t e = vsk::launch_merge(d_lists, n_lists, (uint64_t)nq * k_in, k_in, nq, k_in, k,
                                     d_out_keys, cs);
    if (e != hipSuccess) return fail_hip(e, "merge");
    return VS_OK;
  }
  // the sort merge uses the engine's scratch: ordered after its last user
  VS_HIP(use_stream(eng, cs), "stream order");
  return merge_any(eng, d_lists, n_lists, (uint64_t)nq * k_in, k_in, nq, k_in, k, d_out_keys);
}

int decode_keys(DevEngine* eng, const uint64_t* d_keys, uint32_t nq, uint32_t k,
                   float* out_scores, uint64_t* out_rows, uint32_t* out_count, void* stream) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  if (nq == 0 || k == 0) return VS_OK;
  VS_HIP(set_dev(eng), "hipSetDevice");
  std::vector<uint64_t> h((size_t)nq * k);
  hipStream_t cs = (hipStream_t)stream;
  VS_HIP(hipMemcpyAsync(h.data(), d_keys, h.size() * 8, hipMemcpyDeviceToHost, cs),
         "keys D2H");
  VS_HIP(hipStreamSynchronize(cs), "decode sync");
  decode_host(h.data(), nq, k, out_scores, out_rows, out_count);
  return VS_OK;
}

int checksum(DevEngine* eng, const char* coll, uint64_t* out) {
  if (!eng || !out) return fail(VS_ERR_INVALID_ARG, "engine and out are required");
  auto c = find_coll(eng, coll);
  if (!c) return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (coll ? coll : "") +
                                            " not found");
  std::shared_lock<std::shared_mutex> rl(c->mu);
  std::lock_guard<std::mutex> g(eng->work_mu);
  VS_HIP(set_dev(eng), "hipSetDevice");
  VS_HIP(use_stream(eng, eng->own), "stream order");
  return device_checksum(eng, *c, out);
}

int snapshot(DevEngine* eng, const char* coll, const char* path) {
  if (!eng || !path) return fail(VS_ERR_INVALID_ARG, "engine and path are required");
  auto c = find_coll(eng, coll);
  if (!c) return fail(VS_ERR_NOT_FOUND, std::string("collection ") + (coll ? coll : "") +
                                            " not found");
  // Upserts wait (reader lock: the rows and their buffer stay put); searches
  // and every other engine call proceed. The snapshot touches none of the
  // engine's scratch or its stream: it runs on a stream and an 8-byte
  // checksum buffer of its own, so it never takes work_mu, and a multi-GB
  // disk write does not hold up /search or /health.
  std::shared_lock<std::shared_mutex> rl(c->mu);
  VS_HIP(set_dev(eng), "hipSetDevice");
  SnapStream ss;
  VS_HIP(ss.open(), "snapshot stream");
  SnapHeader h{};
  std::memcpy(h.magic, kSnapMagic, 8);
  h.version = 1;
  h.header_bytes = sizeof(SnapHeader);
  h.dim = c->dim;
  h.metric = c->metric;
  h.dtype = c->dtype;
  h.elem_bytes = (uint32_t)c->elem();
  h.rows = c->rows;
  h.row_base = c->row_base;
  h.data_bytes = c->rows * c->row_bytes();
  VS_HIP(vsk::launch_checksum(c->data, h.data_bytes, ss.sum, ss.st), "checksum");
  VS_HIP(hipMemcpyAsync(&h.data_checksum, ss.sum, 8, hipMemcpyDeviceToHost, ss.st),
         "checksum D2H");
  VS_HIP(hipStreamSynchronize(ss.st), "checksum sync");
  h.header_checksum = header_sum(h);
  const std::string tmp = std::string(path) + ".tmp";
  FileCloser fc;
  fc.f = std::fopen(tmp.c_str(), "wb");
  if (!fc.f) return fail(VS_ERR_IO, "cannot open " + tmp + " for writing");
  if (std::fwrite(&h, sizeof(h), 1, fc.f) != 1) return fail(VS_ERR_IO, "write failed: " + tmp);
  PinnedPair pin;
  const size_t chunk = std::min<size_t>(kSnapChunk, std::max<size_t>(h.data_bytes, 1));
  VS_HIP(pin.alloc(chunk), "pinned staging");
  // chunk i+1 is copied D2H while chunk i is written
  const char* src = (const char*)c->data;
  uint64_t nchunks = (h.data_bytes + chunk - 1) / chunk;
  if (nchunks)
    VS_HIP(hipMemcpyAsync(pin.p[0], src, std::min<uint64_t>(chunk, h.data_bytes),
                          hipMemcpyDeviceToHost, ss.st),
           "snapshot D2H");
  for (uint64_t i = 0; i < nchunks; ++i) {
    const uint64_t off = i * chunk, n = std::min<uint64_t>(chunk, h.data_bytes - off);
    VS_HIP(hipStreamSynchronize(ss.st), "snapshot sync");
    if (i + 1 < nchunks)
      VS_HIP(hipMemcpyAsync(pin.p[(i + 1) & 1], src + off + n,
                            std::min<uint64_t>(chunk, h.data_bytes - off - n),
                            hipMemcpyDeviceToHost, ss.st),
             "snapshot D2H");
    if (std::fwrite(pin.p[i & 1], 1, n, fc.f) != n) {
      (void)hipStreamSynchronize(ss.st);
      return fail(VS_ERR_IO, "write failed: " + tmp);
    }
  }
  const bool ok = std::fflush(fc.f) == 0 && std::fclose(fc.f) == 0;
  fc.f = nullptr;
  if (!ok || std::rename(tmp.c_str(), path) != 0)
    return fail(VS_ERR_IO, std::string("cannot finish ") + path);
  return VS_OK;
}

int restore(DevEngine* eng, const char* coll, const char* path) {
  if (!eng || !path || !coll || !*coll)
    return fail(VS_ERR_INVALID_ARG, "engine, collection and path are required");
  FileCloser fc;
  fc.f = std::fopen(path, "rb");
  if (!fc.f) return fail(VS_ERR_IO, std::string("cannot open ") + path);
  SnapHeader h{};
  if (std::fread(&h, sizeof(h), 1, fc.f) != 1 || std::memcmp(h.magic, kSnapMagic, 8) != 0 ||
      h.version != 1 || h.header_bytes != sizeof(SnapHeader) || header_sum(h) != h.header_checksum)
    return fail(VS_ERR_IO, std::string("not a vsearch snapshot (bad header): ") + path);
  const uint32_t elem = h.dtype == VS_DTYPE_BF16 ? 2 : 4;
  if (h.elem_bytes != elem || h.data_bytes != h.rows * h.dim * (uint64_t)elem)
    return fail(VS_ERR_IO, std::string("inconsistent snapshot header: ") + path);
  int rc = collection_create(eng, coll, h.dim, h.metric, h.dtype, h.rows, h.row_base);
  if (rc != VS_OK) return rc;
  auto c = find_coll(eng, coll);
  if (!c) return fail(VS_ERR_INTERNAL, "restored collection vanished");
  std::unique_lock<std::shared_mutex> wl(c->mu);
  uint64_t sum = 0;
  int err = VS_OK;  // failures are undone after work_mu is released
  std::string msg;
  {
    std::lock_guard<std::mutex> g(eng->work_mu);
    hipError_t e = set_dev(eng);
    if (e == hipSuccess) e = use_stream(eng, eng->own);
    PinnedPair pin;
    const size_t chunk = std::min<size_t>(kSnapChunk, std::max<size_t>(h.data_bytes, 1));
    if (e == hipSuccess) e = pin.alloc(chunk);
    // chunk i is read from disk while chunk i-1 is copied H2D
    char* dst = (char*)c->data;
    const uint64_t nchunks = (h.data_bytes + chunk - 1) / chunk;
    for (uint64_t i = 0; i < nchunks && e == hipSuccess && err == VS_OK; ++i) {
      const uint64_t off = i * chunk, n = std::min<uint64_t>(chunk, h.data_bytes - off);
      if (i >= 2) e = hipStreamSynchronize(eng->stream);  // buffer i&1 free again
      if (e != hipSuccess) break;
      if (std::fread(pin.p[i & 1], 1, n, fc.f) != n) {
        err = VS_ERR_IO;
        msg = std::string("truncated snapshot: ") + path;
        break;
      }
      e = hipMemcpyAsync(dst + off, pin.p[i & 1], n, hipMemcpyHostToDevice, eng->stream);
    }
    const hipError_t es = hipStreamSynchronize(eng->stream);  // staging is freed below
    if (e == hipSuccess) e = es;
    if (err == VS_OK && e != hipSuccess) {
      err = VS_ERR_DEVICE;
      msg = std::string("restore upload: ") + hipGetErrorString(e);
    }
    if (err == VS_OK) {
      c->rows = h.rows;
      err = q8_after_write(eng, *c, 0, c->rows);
      if (err == VS_OK) err = device_checksum(eng, *c, &sum);
      if (err != VS_OK) msg = last_error();
      else if (sum != h.data_checksum) {
        err = VS_ERR_IO;
        msg = std::string("snapshot checksum mismatch: ") + path;
      }
    }
  }
  wl.unlock();
  if (err != VS_OK) {
    (void)collection_drop(eng, coll);
    return fail(err, msg);
  }
  return VS_OK;
}

int health(DevEngine* eng, char* buf, size_t len) {
  if (!eng || !buf || len == 0) return fail(VS_ERR_INVALID_ARG, "bad health buffer");
  size_t freeb = 0, totalb = 0;
  std::string status = "healthy", err;
  hipError_t e = hipSetDevice(eng->device);
  if (e == hipSuccess) e = hipMemGetInfo(&freeb, &totalb);
  if (e != hipSuccess) {
    status = "degraded";
    err = hipGetErrorString(e);
  }
  size_t ncoll;
  {
    std::lock_guard<std::mutex> g(eng->store->map_mu);
    ncoll = eng->store->colls.size();
  }
  int n = std::snprintf(buf, len,
                        "{\"status\":\"%s\",\"engine\":\"vsearch-hip\",\"device\":%d,"
                        "\"device_name\":\"%s\",\"hbm_free_bytes\":%zu,\"hbm_total_bytes\":%zu,"
                        "\"collections\":%zu%s%s%s}",
                        status.c_str(), eng->device, eng->device_name.c_str(), freeb, totalb,
                        ncoll, err.empty() ? "" : ",\"error\":\"", err.c_str(),
                        err.empty() ? "" : "\"");
  if (n < 0 || (size_t)n >= len) return fail(VS_ERR_INVALID_ARG, "health buffer too small");
  return e == hipSuccess ? VS_OK : fail(VS_ERR_DEVICE, err);
}

int timing(DevEngine* eng, double* scan_ms_sum, uint64_t* scan_count, double* merge_ms_sum,
           uint64_t* merge_count, int reset) {
  if (!eng) return fail(VS_ERR_INVALID_ARG, "engine is NULL");
  VS_HIP(set_dev(eng), "hipSetDevice");
  VS_HIP(hipDeviceSynchronize(), "timing sync");
  double sm = 0, mm = 0;
  uint64_t sn = 0, mn = 0;
  for (DevEngine* cx : eng->store->ctx) {  // every search context of the device
    std::lock_guard<std::mutex> g(cx->work_mu);
    auto drain = [cx](std::vector<EventPair>& v, double& acc, uint64_t& n) {
      for (auto& p : v) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
          acc += ms;
          ++n;
        }
        cx->ev_pool.push_back(p.a);
        cx->ev_pool.push_back(p.b);
      }
      v.clear();
    };
    drain(cx->scan_ev, cx->scan_ms, cx->scan_n);
    drain(cx->merge_ev, cx->merge_ms, cx->merge_n);
    sm += cx->scan_ms, sn += cx->scan_n, mm += cx->merge_ms, mn += cx->merge_n;
    if (reset) {
      cx->scan_ms = cx->merge_ms = 0;
      cx->scan_n = cx->merge_n = 0;
      cx->scan_tick = 0;  // the sampling restarts (VS_FLAG_TIMING_SAMPLE)
    }
  }
  if (scan_ms_sum) *scan_ms_sum = sm;
  if (scan_count) *scan_count = sn;
  if (merge_ms_sum) *merge_ms_sum = mm;
  if (merge_count) *merge_count = mn;
  return VS_OK;
}

}  // namespace vsd
