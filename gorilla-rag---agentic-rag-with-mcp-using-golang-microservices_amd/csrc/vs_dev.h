// vs_dev.h — one device's engine (internal; the public boundary is
// include/vsearch.h). A DevEngine owns one HIP device, its stream, its
// scratch and the collections (or collection shards) resident on it;
// vs_api.cpp builds the C-ABI's vs_engine from one DevEngine (a single-GPU
// engine) or several (a row-sharded multi-GPU engine).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <bitset>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/vsearch.h"
#include "vs_kernels.h"
#include "vs_spec_host.h"

namespace vsd {

int fail(int code, const std::string& msg);
int fail_hip(hipError_t e, const char* what);
#define VS_HIP(call, what)                           \
  do {                                               \
    hipError_t e_ = (call);                          \
    if (e_ != hipSuccess) return ::vsd::fail_hip(e_, what); \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) {
    o.p = nullptr;
    o.bytes = 0;
  }
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  // Grows the buffer; the caller has drained the stream that used it.
  hipError_t ensure(size_t want) {
    if (want <= bytes) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    size_t b = std::max(want, (size_t)4096);
    hipError_t e = hipMalloc(&p, b);
    if (e == hipSuccess) bytes = b;
    return e;
  }
  template <typename T>
  T* as() const {
    return (T*)p;
  }
};

struct Collection {
  std::string name;
  uint64_t gen = 0;  // unique per created collection (never reused in a process)
  uint32_t dim = 0;
  int metric = VS_METRIC_COSINE;
  int dtype = VS_DTYPE_F32;
  uint64_t row_base = 0;
  void* data = nullptr;  // cap x dim elements
  uint64_t rows = 0, cap = 0;
  std::shared_mutex mu;
  // int8 prefilter copy (r04, vs_kernels.h "int8 prefilter"): bf16
  // collections of q8_supported dims once they take the batched pass; kept
  // in step with `data` by every store-side call (q8_after_write)
  void* q8 = nullptr;         // (q8_cap + kPadRows) x dim int8
  float* q8_meta = nullptr;   // {dt, nt} per 32-row tile
  float* q8_glob = nullptr;   // {absmax, dmax, nmax, S}, then the speculative
                              // bound's counters and per-k state (vs_kernels.h)
  // (r06) the speculative bound's advice to the host, coherent mapped pinned
  // memory the device writes (vs_kernels.h Q8SpecK): [k] 1 = the bound is
  // loose for k (enqueue the sample path alone), [kQ8SpecK + k] batches of k
  // left in a cool-down after a failed check (counted off by the host)
  uint32_t* q8_advice = nullptr;
  uint32_t* q8_advice_dev = nullptr;
  std::atomic<uint64_t> spec_host_skips{0};  // batches the advice kept off a try
  uint64_t q8_cap = 0;        // rows the int8 buffers hold
  // (r05) bumped by every store-side write (the ratios are reset with it):
  // unique in the process, so a context's record of the ratios it learned
  // is valid only for the generation it learned them in
  uint64_t q8_gen = 0;
  uint64_t q8_scaled_at = 0;  // rows when S was last chosen (rescaled at 2x)
  size_t elem() const { return dtype == VS_DTYPE_BF16 ? 2 : 4; }
  size_t row_bytes() const { return elem() * dim; }
  void q8_free() {
    if (q8) (void)hipFree(q8);
    if (q8_meta) (void)hipFree(q8_meta);
    if (q8_glob) (void)hipFree(q8_glob);
    if (q8_advice) (void)hipHostFree(q8_advice);
    q8 = nullptr, q8_meta = nullptr, q8_glob = nullptr, q8_cap = 0, q8_scaled_at = 0;
    q8_advice = q8_advice_dev = nullptr;
  }
  ~Collection() {
    if (data) (void)hipFree(data);
    q8_free();
  }
};

struct EventPair {
  hipEvent_t a, b;
};

// Pinned staging of one host search call (search_host): the queries go H2D
// and the keys D2H asynchronously through it, so a call holds work_mu only
// while it enqueues and waits for the device outside it; a call arriving
// meanwhile (another batcher worker, another collection) enqueues behind it
// on the same stream, and the device runs the two back to back.
struct HostSlot {
  void* in = nullptr;
  void* out = nullptr;
  size_t in_bytes = 0, out_bytes = 0;
  hipEvent_t done = nullptr;
  bool busy = false;  // between its enqueue and the end of its decode
  // one-query completion (r03): up to kMaxK keys + the sequence word, in
  // coherent mapped pinned memory the last kernel writes directly (HostDirect)
  uint64_t* mapped = nullptr;
  uint64_t* mapped_dev = nullptr;  // the same memory as the device sees it
  uint64_t seq = 0;
  HostSlot() = default;
  HostSlot(const HostSlot&) = delete;
  HostSlot& operator=(const HostSlot&) = delete;
  ~HostSlot() {
    if (in) (void)hipHostFree(in);
    if (out) (void)hipHostFree(out);
    if (done) (void)hipEventDestroy(done);
    if (mapped) (void)hipHostFree(mapped);
  }
  size_t mapped_words = 0;
  // grows the mapped completion buffer (the slot is idle); zero-filled, so a
  // fresh word never equals a sequence number (they start at 1)
  hipError_t ensure_mapped(size_t words) {
    if (mapped && words <= mapped_words) return hipSuccess;
    if (mapped) {
      (void)hipHostFree(mapped);
      mapped = mapped_dev = nullptr;
      mapped_words = 0;
    }
    void* p = nullptr;
    const hipError_t e = hipHostMalloc(&p, words * 8, hipHostMallocCoherent | hipHostMallocMapped);
    if (e != hipSuccess) return e;
    std::memset(p, 0, words * 8);
    void* d = nullptr;
    const hipError_t e2 = hipHostGetDevicePointer(&d, p, 0);
    if (e2 != hipSuccess) {
      (void)hipHostFree(p);
      return e2;
    }
    mapped = (uint64_t*)p;
    mapped_dev = (uint64_t*)d;
    mapped_words = words;
    return hipSuccess;
  }
  // grows the pinned buffers (the slot is idle: nothing in flight uses them)
  hipError_t ensure(size_t in_b, size_t out_b) {
    hipError_t e = hipSuccess;
    if (!done) e = hipEventCreateWithFlags(&done, hipEventDisableTiming);
    if (e == hipSuccess && in_b > in_bytes) {
      if (in) (void)hipHostFree(in);
      in = nullptr;
      in_bytes = 0;
      e = hipHostMalloc(&in, in_b, hipHostMallocDefault);
      if (e == hipSuccess) in_bytes = in_b;
    }
    if (e == hipSuccess && out_b > out_bytes) {
      if (out) (void)hipHostFree(out);
      out = nullptr;
      out_bytes = 0;
      e = hipHostMalloc(&out, out_b, hipHostMallocDefault);
      if (e == hipSuccess) out_bytes = out_b;
    }
    return e;
  }
};


// Upsert staging (r04): two pinned host buffers (vectors + row numbers of one
// chunk each) and two device buffers, so the host gathers chunk i+1 while
// chunk i crosses PCIe and is preprocessed; done[j] marks the H2D out of
// pin[j] complete. Guarded by the owning context's work_mu.
struct UpsertStage {
  void* pin[2] = {nullptr, nullptr};
  size_t pin_bytes = 0;
  hipEvent_t done[2] = {nullptr, nullptr};
  bool armed[2] = {false, false};
  DevBuf vecs[2], rows[2];
  UpsertStage() = default;
  UpsertStage(const UpsertStage&) = delete;
  UpsertStage& operator=(const UpsertStage&) = delete;
  ~UpsertStage() {
    for (int j = 0; j < 2; ++j) {
      if (done[j]) (void)hipEventSynchronize(done[j]);
      if (pin[j]) (void)hipHostFree(pin[j]);
      if (done[j]) (void)hipEventDestroy(done[j]);
    }
  }
  // pinned buffers of at least b bytes each (the stage is idle: no H2D pending)
  hipError_t ensure(size_t b) {
    for (int j = 0; j < 2; ++j)
      if (!done[j]) {
        const hipError_t e = hipEventCreateWithFlags(&done[j], hipEventDisableTiming);
        if (e != hipSuccess) return e;
      }
    if (b <= pin_bytes) return hipSuccess;
    size_t r = 1ull << 20;  // powers of two from 1 MiB: few re-allocations
    while (r < b) r <<= 1;
    b = r;
    for (int j = 0; j < 2; ++j) {
      if (armed[j]) (void)hipEventSynchronize(done[j]);  // an earlier call that failed
      if (pin[j]) (void)hipHostFree(pin[j]);
      pin[j] = nullptr;
      armed[j] = false;
    }
    pin_bytes = 0;
    for (int j = 0; j < 2; ++j) {
      const hipError_t e = hipHostMalloc(&pin[j], b, hipHostMallocDefault);
      if (e != hipSuccess) return e;
    }
    pin_bytes = b;
    return hipSuccess;
  }
};

// A device-resident filter (vs_filter_create): bitmap, popcount and, when
// selective, the compacted row list. Shared: a search holds its reference
// until the device has finished with it, so a concurrent drop is safe.
struct DevFilter {
  std::string coll;
  uint64_t coll_gen = 0;           // Collection::gen it was built for
  uint64_t rows = 0, allowed = 0;  // collection rows it was built over
  DevBuf bits, list;               // bitmap; compacted rows when selective
};

struct DevEngine;

// What the search contexts of one device share: the resident collections and
// filters. ctx[0] is the primary context (stores, filters, device-pointer
// searches, snapshots); host searches take any idle context.
struct DevStore {
  std::mutex map_mu;
  std::unordered_map<std::string, std::shared_ptr<Collection>> colls;
  std::mutex filt_mu;
  std::unordered_map<uint64_t, std::shared_ptr<DevFilter>> filters;
  uint64_t next_filter = 1;
  std::vector<DevEngine*> ctx;
};

// One search context of a device: its stream, its scratch and its staging.
// Contexts of a device run concurrently (separate streams): two host
// searches on different contexts overlap on the device, not only on the host.
struct DevEngine {
  int device = 0;
  uint32_t flags = 0;
  hipStream_t own = nullptr;     // the context's stream
  hipStream_t stream = nullptr;  // the stream device work is enqueued on now (own or a caller's)
  hipEvent_t xev = nullptr;      // orders a newly used stream after the previous one
  std::string device_name;
  std::shared_ptr<DevStore> store;
  std::atomic<int> inflight{0};  // host searches on this context not yet returned
  std::mutex work_mu;  // scratch buffers + stream
  DevBuf q_in, q_pre, q_bf16, lists, keys, sample_bound;
  std::unique_ptr<UpsertStage> up;  // upsert staging, made at the first upsert
  DevBuf q8_q, q8_par, q8_tiles;    // int8 prefilter: int8 queries, {sqS, a, c, sigma} + gate,
                                    // tiles an upsert touched
  DevBuf cand, cand_cnt;            // MFMA main pass candidates (vs_kernels.h)
  DevBuf merge_tmp;                 // first stage of a two-stage GEMV merge
  DevBuf scand;                     // MFMA sample pass tile maxima
  DevBuf scratch8;                  // u64 result of the snapshot checksum
  DevBuf allow;                     // filter pre-mask of the current vs_search_filtered
  DevBuf gather_rows, gather_cnt;   // its compacted row list (selective filters) + scan scratch
  // large-k path (k > vsk::kMaxK): score images, digit histogram (kept
  // zeroed between uses), select state, the selected keys, sort scratch;
  // large merges (vs_merge_keys / shard merges at k > kMaxK)
  DevBuf lk_sc, lk_hist, lk_state, lk_sel, lk_sort, merge_big;
  DevBuf lk_cand, lk_ctr;  // fused selection: boundary-bucket keys, 3 counters
  // small-collection search spread over workgroups: their keys + the
  // completion counter (zeroed at allocation; each launch leaves it zero)
  DevBuf small_part;
  DevBuf q8g;  // one query on the int8 copy: workgroup lists, wave bounds, candidates
  // (r05) per collection (Collection::gen): what this context has answered
  // on its stream, for the speculative bound (vs_spec_host.h spec_plan)
  SpecSeenMap spec_seen;
  std::vector<uint64_t> h_keys;
  std::vector<std::unique_ptr<HostSlot>> host_slots;  // search_host staging, guarded by work_mu
  // timing
  std::vector<EventPair> scan_ev, merge_ev;
  std::vector<hipEvent_t> ev_pool;  // recycled timing events (none created on the hot path)
  double scan_ms = 0, merge_ms = 0;
  uint64_t scan_n = 0, merge_n = 0;
  uint64_t scan_tick = 0;   // scan launches seen (VS_FLAG_TIMING_SAMPLE)
  bool scan_skip = false;   // the current scan launch is not bracketed
  uint32_t scan_period = 4; // VS_FLAG_TIMING_SAMPLE brackets one scan in this many
};

// ---- per-device operations (vs_engine.cpp); same contracts as the C-ABI
// functions of the same name, for one device and its local rows. `eng` is a
// device's primary context unless said otherwise ----
// Opens the primary context and VS_CONTEXTS - 1 more (default 2 in all).
int open(int device, uint32_t flags, DevEngine** out);
void close(DevEngine* eng);  // the primary: closes every context of the device
// A filter of the device's store (nullptr: none); the reference keeps it alive.
std::shared_ptr<DevFilter> find_filter(DevEngine* eng, uint64_t filter_id);
// The context a host search should use (locked on return: `lk` owns its
// work_mu): the primary for a heavy search (vs_engine.cpp heavy_search),
// else an idle one if any, else the least busy one (waited for).
DevEngine* pick_context(DevEngine* eng, std::unique_lock<std::mutex>* lk, bool heavy = false);
bool heavy_search(const Collection& c, uint32_t nq);
std::shared_ptr<Collection> find_coll(DevEngine* eng, const char* name);
hipError_t set_dev(DevEngine* eng);
hipError_t use_stream(DevEngine* eng, hipStream_t s);
int collection_create(DevEngine* eng, const char* name, uint32_t dim, int metric, int dtype,
                      uint64_t capacity_hint, uint64_t row_base);
int collection_info(DevEngine* eng, const char* name, uint32_t* dim, uint64_t* rows, int* metric,
                    int* dtype);
int collection_drop(DevEngine* eng, const char* name);
int prefilter_bytes(DevEngine* eng, const char* name, uint64_t* bytes);
int spec_stats(DevEngine* eng, const char* name, uint64_t out[4]);
int upsert(DevEngine* eng, const char* coll, uint64_t n, uint32_t dim, const uint64_t* rows,
           const float* vecs);
// appends n generator rows whose global numbers are g0, g0 + stride, ...
int generate(DevEngine* eng, const char* coll, uint64_t n, uint64_t seed, uint64_t g0,
             uint64_t stride);
int generate_vectors(DevEngine* eng, uint64_t seed, uint64_t row0, uint64_t n, uint32_t dim,
                     float* d_out, void* stream);
int read_rows(DevEngine* eng, const char* coll, uint64_t first, uint64_t n, float* out);
int read_raw(DevEngine* eng, const char* coll, uint64_t first, uint64_t n, void* out);
int append_raw(DevEngine* eng, const char* coll, uint64_t n, const void* rows);
int checksum_shard(DevEngine* eng, const char* coll, uint64_t stride, uint64_t offset,
                   uint64_t* out);
const char* last_error();
int search_host(DevEngine* eng, const char* coll, const float* queries, uint32_t nq,
                uint32_t dim, uint32_t k, const uint64_t* allow, uint64_t allow_words,
                float* out_scores, uint64_t* out_rows, uint32_t* out_count,
                uint64_t filter_id = 0);
int filter_create(DevEngine* eng, const char* coll, const uint64_t* allow, uint64_t allow_words,
                  uint64_t* filter_id);
int filter_drop(DevEngine* eng, uint64_t filter_id);
int search_keys(DevEngine* eng, const char* coll, const float* d_queries, uint32_t nq,
                uint32_t dim, uint32_t k, uint64_t* d_keys, void* stream);
int merge_keys(DevEngine* eng, const uint64_t* d_lists, uint32_t n_lists, uint32_t nq,
               uint32_t k_in, uint32_t k, uint64_t* d_out_keys, void* stream);
// launch_merge for any k on eng->stream (k or k_in > vsk::kMaxK: the sort
// merge, scratch grown here); work_mu held by the caller.
int merge_any(DevEngine* eng, const uint64_t* lists, uint32_t L, uint64_t lstride,
              uint64_t qstride, uint32_t nq, uint32_t kin, uint32_t k, uint64_t* out);
int decode_keys(DevEngine* eng, const uint64_t* d_keys, uint32_t nq, uint32_t k,
                float* out_scores, uint64_t* out_rows, uint32_t* out_count, void* stream);
// keys [nq][k] -> outputs of row stride ko >= k (slots k .. ko-1 zeroed: a
// search clamped to the collection's rows answers into the caller's stride)
void decode_host(const uint64_t* keys, uint32_t nq, uint32_t k, float* scores, uint64_t* rows,
                 uint32_t* count, uint32_t ko = 0);
int checksum(DevEngine* eng, const char* coll, uint64_t* out);
int snapshot(DevEngine* eng, const char* coll, const char* path);
int restore(DevEngine* eng, const char* coll, const char* path);
int health(DevEngine* eng, char* buf, size_t len);
int timing(DevEngine* eng, double* scan_ms_sum, uint64_t* scan_count, double* merge_ms_sum,
           uint64_t* merge_count, int reset);
uint64_t popcount_rows(const uint64_t* allow, uint64_t rows);
// Waits for ev: a short spin on hipEventQuery, then hipEventSynchronize.
hipError_t wait_event(hipEvent_t ev);
// VS_OK when this process maps one HIP runtime; else VS_ERR_DEVICE with both
// paths in the message. Entry points that take the caller's device pointers
// and stream call it first ("one HIP runtime per process").
int one_hip_runtime();

// Search of device queries d_q (nq x dim fp32 on this device, ordered on
// eng->stream) -> keys d_keys [nq][k] in local rows + row_base; work_mu and
// the collection's reader lock held by the caller. Asynchronous: nothing
// waits on the device unless a scratch buffer has to grow.
// With `direct` (one query), a search whose last kernel can publish to the
// host -- the one-launch small path, or the GEMV list path's merge -- writes
// its keys to direct->keys (mapped pinned host memory) and then direct->seq
// to *direct->flag, and sets direct->used; d_keys is then not written. Other
// paths leave direct->used false and write d_keys.
struct HostDirect {
  uint64_t* keys = nullptr;  // device views of the mapped buffer
  uint64_t* flag = nullptr;
  uint64_t seq = 0;
  const float* host_q = nullptr;  // raw query in host memory: sent in the kernel arguments
  bool used = false;
};
// search_core's one-launch small path takes this search (one query, no
// filter, a small collection, k <= kGemvSmallMaxK)
bool small_path(const Collection& c, uint32_t nq, uint32_t k, bool filtered);
int search_core(DevEngine* eng, Collection& c, const float* d_q, uint32_t nq, uint32_t k,
                uint64_t* d_keys, const uint64_t* allow = nullptr, uint64_t allowed = 0,
                const uint32_t* allow_list = nullptr, HostDirect* direct = nullptr);
// Bytes of the int8 copy a collection of `rows` rows would keep on an engine
// opened with `flags` (0 when it keeps none): placement reserves them beside
// the rows.
uint64_t q8_reserve_bytes(int flags, uint32_t dim, int dtype, uint64_t rows);

}  // namespace vsd
